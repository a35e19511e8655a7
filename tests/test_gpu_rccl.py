"""C3's collective path on a real MI355X at world size 1 (BASELINE.json configs[2]).

bench.py --gpus 1 --dist starts `torch.distributed.run --nproc-per-node 1` as a CHILD process (the
test process never execs), and the rank takes the same branch an 8-GPU rank takes:
init_process_group("nccl", device_id=...) (RCCL on ROCm), the solve plus
mpcqp.distributed.allgather_forces inside the timed loop, the all-gather's HIP-event span
(extras.allgather_ms, max over ranks) and the gathered-u0 check, then oracle parity on the sample.
This is no scaling measurement: one rank, one GPU; no 1/2/4/8 curve is measured here (8-GPU runs belong
to the driver).  The second test compares the world-1 RCCL rate with the non-distributed rate on C3's
8192-robot shard (the rank's stream layout must not cost the solve more than 5 %).  A rank
that runs RCCL solves its shard as one part — the caller's stream and RCCL's: the batch split's two
internal streams would exceed the process's four hardware queues (measured: three parts under RCCL
2.86M QP/s against 2.91-3.00M for one part)."""
import json
import math
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=300):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    argv = [sys.executable, os.path.join(REPO, "bench.py"), *args]
    out = subprocess.run(argv, capture_output=True, text=True, timeout=timeout, cwd=REPO, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-3000:]
    return json.loads(lines[0])


def test_bench_rccl_world1_gathers_and_matches_oracle():
    rec = _bench("--gpus", "1", "--dist", "--steps", "4", "--warmup", "1", "--batch", "2048")
    print(json.dumps({k: rec[k] for k in ("value", "ms_per_step", "extras", "parity")}))
    assert rec["n_gpus"] == 1 and rec["config"]["ranks_seen"] == 1
    assert rec["config"]["collective"].startswith("RCCL")
    ex = rec["extras"]
    assert ex["backend"] == "nccl"
    assert math.isfinite(ex["allgather_ms"]) and ex["allgather_ms"] >= 0.0
    assert math.isfinite(ex["solve_kernel_ms_max_over_ranks"]) and ex["solve_kernel_ms_max_over_ranks"] > 0.0
    par = rec["parity"]
    assert par["gathered_u0_equals_rank_results"]
    assert par["instances"] == 2048
    assert par["status_equal"] and par["iters_equal"]
    assert par["max_rel_err_u0"] <= 1e-4
    assert par["max_rel_err_u0"] <= 1e-8  # regression sentinel at the achieved accuracy (~1e-10)


def test_rccl_world1_rate_within_5_percent_of_plain():
    """C3's per-rank workload (8192 robots) with and without the process group and per-step RCCL
    all-gather: the distributed rate is at least 95 % of the plain one."""
    common = ["--gpus", "1", "--steps", "20", "--warmup", "3", "--batch", "8192", "--no-cpu", "--no-extras"]
    plain = _bench(*common)
    dist = _bench(*common, "--dist")
    from gpu_helpers import note
    note("rccl world 1 vs plain (8192 robots)", plain_qps=plain["value"], dist_qps=dist["value"],
         ratio=dist["value"] / plain["value"], allgather_ms=dist["extras"]["allgather_ms"])
    assert dist["roofline"]["parts"] == 1
    assert dist["value"] >= 0.95 * plain["value"], (dist["value"], plain["value"])

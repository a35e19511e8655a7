"""Multi-rank path on CPU: world_size-2 gloo, contiguous robot shards + all-gather of forces.

The per-rank solve here is the CPU oracle standing in for the device solve (tests only); the code
under test is mpcqp.distributed (shard_range / allgather_forces), used by bench.py on RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import mpcqp
from mpcqp.distributed import allgather_forces, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, total, out_dir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "oracle")]
    import pyoracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    st = mpcqp.synthetic_go1(total, seed=123, gait="trot")
    recs = mpcqp.assemble_compute_grf(st, 10)
    b, e = shard_range(total, world, rank)
    res = pyoracle.solve_batch(pyoracle.default_params(10), recs[b:e], nthreads=1)
    local = torch.from_numpy(np.ascontiguousarray(res["u0"]))
    full = allgather_forces(local, total)
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), full.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("total", [8, 7])
def test_sharded_allgather_matches_single_rank(oracle, tmp_path, total):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), total, str(tmp_path)), nprocs=world, join=True)
    st = mpcqp.synthetic_go1(total, seed=123, gait="trot")
    ref = oracle.solve_batch(oracle.default_params(10), mpcqp.assemble_compute_grf(st, 10), nthreads=2)
    for r in range(world):
        got = np.load(tmp_path / f"rank{r}.npy")
        np.testing.assert_array_equal(got, ref["u0"])


def test_shard_range_partitions():
    for total in (0, 1, 7, 8, 65536, 65537):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [e - b for b, e in spans]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("world,batch", [(1, 32), (2, 48), (3, 16), (8, None)])
def test_bench_launcher_shards_and_gathers(world, batch):
    """bench.py --gpus N as the driver runs it: the parent starts torch.distributed.run as a child
    (no GPU touched), N ranks take contiguous shards of ONE seeded global batch, run the production
    per-step call path (solve -> mpcqp.distributed.allgather_forces, here over gloo with a CPU stub
    in place of the device solve) and rank 0 checks the world size and the gathered forces."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    argv = [sys.executable, os.path.join(repo, "bench.py"), "--gpus", str(world), "--cpu-stub",
            "--steps", "2", "--warmup", "1"]
    if world == 1:  # the distributed branch at world 1 (what tests/test_gpu_rccl.py runs over RCCL)
        argv.append("--dist")
    if batch is not None:
        argv += ["--batch", str(batch)]
    else:  # the driver's 8-GPU line: no --batch, so the default must be C3 (8192 robots per GPU)
        batch = 8192
    out = subprocess.run(argv, capture_output=True, text=True, timeout=600, cwd=repo)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == world and rec["config"]["ranks_seen"] == world
    assert rec["config"]["global_batch"] == world * batch
    assert rec["parity"]["gather_exact"] and rec["parity"]["instances"] == world * batch
    assert rec["value"] > 0 and rec["scaling"] == "weak"
    assert rec["extras"]["allgather_ms"] >= 0.0
    if world == 8:
        assert rec["config"]["global_batch"] == 65536 and rec["config"]["workload"].startswith("C3:")


def test_bench_default_batch_is_c2_at_one_gpu_and_c3_shard_above():
    import bench
    assert bench.parse_args([]).batch == 4096
    assert bench.parse_args(["--gpus", "8"]).batch == 8192
    assert bench.parse_args(["--gpus", "2", "--batch", "100"]).batch == 100
    assert bench.config_name(10, 4096, 1, "trot", False) == "C2"
    assert bench.config_name(10, 8192, 8, "trot", False) == "C3"
    assert bench.config_name(20, 4096, 1, "trot", False) == "C4"


def _fg_worker(rank, world, port, total, steps, out_dir):
    from mpcqp.distributed import ForceGather
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, e = shard_range(total, world, rank)
    fg = ForceGather(total, 12)
    res = torch.zeros((e - b, 30), dtype=torch.float64)
    hs = []
    for t in range(steps):
        # step t's "results": rows of 30 doubles whose first 12 identify (tick, robot, column)
        res.copy_(torch.arange(b, e, dtype=torch.float64)[:, None] * 100.0 + torch.arange(30.0)[None, :] + 1e5 * t)
        hs.append(fg.gather(res))
        if t >= 1:  # the previous tick's forces are complete although this tick's gather is in flight
            np.save(os.path.join(out_dir, f"r{rank}_t{t - 1}.npy"), fg.result(hs[t - 1]).numpy())
    np.save(os.path.join(out_dir, f"r{rank}_t{steps - 1}.npy"), fg.result(hs[-1]).numpy())
    fg.drain()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("total", [10, 9])
def test_force_gather_double_buffered(tmp_path, total):
    """mpcqp.distributed.ForceGather (bench.py's per-tick exchange): every tick's gathered forces are
    that tick's u0 of every rank, with the buffers reused every second tick and unequal shards."""
    world, steps = 2, 5
    mp.spawn(_fg_worker, args=(world, _free_port(), total, steps, str(tmp_path)), nprocs=world, join=True)
    for t in range(steps):
        exp = (np.arange(total, dtype=np.float64)[:, None] * 100.0 + np.arange(12.0)[None, :] + 1e5 * t)
        for r in range(world):
            np.testing.assert_array_equal(np.load(tmp_path / f"r{r}_t{t}.npy"), exp)

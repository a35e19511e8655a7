#!/usr/bin/env python3
"""Benchmark: batched Go1 convex-MPC QP solves/sec on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch of synthetic robot states resident in HBM:
scale_kernel (OSQP scale_data on the condensed Hessian's closed-form columns) + wave_kernel
(OSQP-0.6 ADMM with the KKT solve in the impulse-space Schur form at N <= 10 -- the Riccati form, in
the same wave, for robots with rank-deficient feet or an ill-conditioned Schur core (none at C2) --
and the Riccati form with its factorization on MFMA above; extraction), and for N > 1 ranks the RCCL
all-gather of the solved forces over xGMI (north_star, config C3).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--horizon 10]

--gpus N > 1 without a torch.distributed environment: this process starts
`python -m torch.distributed.run --nproc-per-node N bench.py ...` as a child (it never touches the
GPU itself) and exits with the child's code.  Every rank takes the contiguous shard
shard_range(N*B, N, rank) of ONE seeded global batch of N*B robots (weak scaling: B robots per GPU,
8192 by default when N > 1, so --gpus 8 is C3's 65536 robots), solves it and all-gathers u0 with mpcqp.distributed.allgather_forces.
Rank 0 checks the world size, checks the gathered forces against the CPU oracle on a 4096-robot
sample spread over every shard, and prints ONE JSON line.

At N = 1 the line also carries the CPU baseline (the oracle on the host cores) and extra keys,
each with its own parity sample: e2e (host buffers in and out through mpcqp_solve_batch_host),
assemble_e2e (raw robot-state rows -> on-device assembly -> solve), c4 (horizon 20), c5 (mixed
gait, random mu, 8192 robots), c3_shard (one GPU's 8192-robot share of C3), batch_scaling (4096 to
65536 robots on one GPU), two_streams (independent C2 batches alternating over two handles and
streams: one batch's dispatch tail overlaps the next), warm_tick (closed-loop warm-started ticks).  At N > 1 the line carries
extras.allgather_ms (max over ranks of the per-step all-gather span).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "go1-qp-mpc-controller_amd"))

METRIC = "MPC QP solves/sec (horizon=10, 12 GRF vars) at 1/2/4/8 MI355X vs CPU OSQP"
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector (= FP64 matrix) peak, spec
PARITY_SAMPLE = 4096
C2_BATCH = 4096           # BASELINE configs[1]: 4096 robots on one MI355X
C3_BATCH_PER_GPU = 8192   # BASELINE configs[2]: 65536 robots sharded over 8 MI355X
C3_GPUS = 8


def algorithmic_flops(N, iters, rho_updates):
    """SURVEY §8(d) structure-exploiting FLOP count per QP, with actual k (iters) and r."""
    S, n, m = 13, 12 * N, 20 * N
    nnzA = 36 * N
    F_cond = (N - 1) * 2 * S ** 3 + (N * (N - 1) // 2) * 2 * S ** 2 * 12
    F_H = (N * (N + 1) * (N + 2) // 6) * (2 * 12 * 12 * S) + n
    F_g = 2 * S ** 2 * N + 12 * S * N * (N + 1)
    F_scale = 10 * (3 * n ** 2 + 3 * nnzA)
    F_chol = n ** 3 / 3.0
    F_iter = 2 * n ** 2 + 4 * nnzA + 10 * m + 6 * n
    F_check = 2 * n ** 2 + 4 * nnzA
    k = np.asarray(iters, dtype=np.float64)
    r = np.asarray(rho_updates, dtype=np.float64)
    return float(np.sum(F_cond + F_H + F_g + F_scale + F_chol * (1 + r) + F_iter * k
                        + F_check * np.ceil(k / 25.0)))


def load_traffic(config_key, kernel):
    """Per-launch HBM bytes of `kernel` measured by a separate rocprofv3 --pmc pass (profiles/),
    or None when no pass of that kernel on this configuration is on file."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            e = json.load(f).get(config_key, {})
    except (OSError, ValueError):
        return None
    for part in kernel.split(" + "):  # every kernel of the solve must be in the measured set
        short = part.split("::")[-1].split("<")[0]  # e.g. wave_kernel
        tmpl = part[part.find("<"):part.find(">") + 1] if "<" in part else ""
        if (short + tmpl).replace(" ", "") not in e.get("kernel", "").replace(" ", ""):
            return None
    return e.get("hbm_bytes_per_launch")


def load_executed(config_key, kernel):
    """Executed binary64 FLOPs per solve of `kernel` from a separate rocprofv3 --pmc pass
    (profiles/pmc_flops.json, tools/pmc_flops.py: SQ_INSTS_VALU_{FMA,ADD,MUL}_F64 x 64 lanes, FMA = 2,
    plus SQ_INSTS_VALU_MFMA_MOPS_F64 x 512), or None when no pass of that kernel is on file.  An upper
    bound on useful FLOPs: masked and padding lanes are counted."""
    path = os.path.join(REPO, "profiles", "pmc_flops.json")
    try:
        with open(path) as f:
            e = json.load(f).get(config_key, {})
    except (OSError, ValueError):
        return None
    names = " + ".join(k.get("kernel", "") for k in e.get("kernels", [])).replace(" ", "")
    for part in kernel.split(" + "):
        short = part.split("::")[-1].split("<")[0]
        tmpl = part[part.find("<"):part.find(">") + 1] if "<" in part else ""
        if (short + tmpl).replace(" ", "") not in names:
            return None
    return e.get("executed_f64_flop_per_solve")


def executed_fields(config_key, kernel, ms):
    ex = load_executed(config_key, kernel)
    if ex is None:
        return {"executed_flop_per_launch": None, "executed_tflops": None, "executed_frac": None}
    tf = ex / (ms * 1e-3) / 1e12
    return {"executed_flop_per_launch": ex, "executed_tflops": tf, "executed_frac": tf / FP64_PEAK_TFLOPS}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None,
                    help="robots per GPU; default 4096 at --gpus 1 (C2, BASELINE configs[1]) and 8192 for "
                         "--gpus N > 1 (C3, configs[2]: 65536 robots over 8 GPUs)")
    ap.add_argument("--horizon", type=int, default=10)
    ap.add_argument("--gait", default="trot", choices=["trot", "stance", "mixed"])
    ap.add_argument("--mixed-mu", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=4096,
                    help="instances timed on the CPU oracle (4096 x ~2.3 ms = ~10 s of CPU work)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: min(16, usable cpus)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the e2e / c4 / c5 / warm_tick keys")
    ap.add_argument("--dist", action="store_true",
                    help="take the distributed branch (process group, per-step all-gather, allgather_ms, "
                         "gathered parity) at any world size, --gpus 1 included: a world-1 RCCL run on one "
                         "GPU exercises the C3 collective path's code before an 8-GPU node does")
    ap.add_argument("--cpu-stub", action="store_true",
                    help="TEST ONLY: gloo backend on the CPU, a deterministic stub in place of the device "
                         "solve (exercises the launcher, sharding and all-gather without a GPU)")
    args = ap.parse_args(argv)
    if args.batch is None:
        args.batch = C2_BATCH if args.gpus == 1 else C3_BATCH_PER_GPU
    return args


def oracle_module():
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle  # checker / CPU-baseline leg only (test infrastructure)
    pyoracle.build()
    return pyoracle


def parity_of(got, ref):
    """u0 relative error (SURVEY §8(c) gate 1e-4), status and iteration equality."""
    err = np.max(np.abs(got["u0"] - ref["u0"]), axis=1) / np.maximum(np.max(np.abs(ref["u0"]), axis=1), 1.0)
    return {"max_rel_err_u0": float(np.max(err)) if err.size else 0.0, "instances": int(len(ref)),
            "status_equal": bool(np.all(got["status"] == ref["status"])),
            "iters_equal": bool(np.all(got["iters"] == ref["iters"])),
            "iters_equal_frac": float(np.mean(got["iters"] == ref["iters"])) if len(ref) else 1.0}


def config_name(N, batch_per_gpu, world, gait, mixed_mu):
    """BASELINE.json config id of a bench line (None when the line is none of them)."""
    if N == 10 and gait == "trot" and not mixed_mu:
        if world == 1 and batch_per_gpu == C2_BATCH:
            return "C2"
        if batch_per_gpu == C3_BATCH_PER_GPU:
            return "C3" if world == C3_GPUS else f"C3 shard size ({world} GPU{'s' if world > 1 else ''})"
    if N == 20 and gait == "trot" and world == 1 and batch_per_gpu == C2_BATCH:
        return "C4"
    if N == 10 and gait == "mixed" and mixed_mu and batch_per_gpu == 8192 and world == 1:
        return "C5"
    return None


def workload(N, total, gait, mixed_mu):
    """One seeded synthetic global batch; every rank builds the same one."""
    import mpcqp
    config_id = 1 if (gait == "trot" and not mixed_mu) else 4
    states = mpcqp.synthetic_go1(total, seed=config_id * 1000, gait=gait, mixed_mu=mixed_mu)
    return states, mpcqp.assemble_compute_grf(states, N)


def stub_results(recs):
    """--cpu-stub: a deterministic per-robot stand-in for the solve (u0 from the record bytes)."""
    import mpcqp
    res = np.zeros(recs.shape[0], dtype=mpcqp.RESULT_DTYPE)
    res["u0"] = recs[:, :12] * 3.0 + recs[:, 44:56]
    res["status"] = 1
    res["iters"] = 25
    return res


def as_rows(res):
    """mpcqp_result structured array -> [B, 30] float64 rows (bit copy) and back."""
    return np.frombuffer(res.tobytes(), dtype=np.float64).reshape(len(res), -1)


def run_rank(args):
    import torch
    import torch.distributed as dist
    import mpcqp
    from mpcqp.distributed import ForceGather, allgather_forces, env_rank, shard_range

    world, rank, local_rank = env_rank()
    dist_on = world > 1 or args.dist  # the process group and the per-step all-gather (C3 path)
    if args.cpu_stub:
        dev = torch.device("cpu")
        if dist_on:
            dist.init_process_group("gloo")
    else:
        dev = torch.device("cuda", local_rank)
        torch.cuda.set_device(dev)
        if dist_on:
            dist.init_process_group("nccl", device_id=dev)
    ranks_seen = dist.get_world_size() if dist_on else 1
    if ranks_seen != args.gpus:
        raise SystemExit(f"bench: {ranks_seen} ranks but --gpus {args.gpus}")

    N, B = args.horizon, args.batch
    total = B * world
    states, recs_global = workload(N, total, args.gait, args.mixed_mu)
    b0, b1 = shard_range(total, world, rank)
    recs_np = np.ascontiguousarray(recs_global[b0:b1])
    Bl = b1 - b0
    RD = mpcqp._lib.RESULT_DOUBLES

    params = None
    solver = None
    if args.cpu_stub:
        stub = torch.from_numpy(as_rows(stub_results(recs_np)).copy())
        d_res = torch.zeros((Bl, RD), dtype=torch.float64)

        def solve():
            d_res.copy_(stub)
        sync = (lambda: None)
        events = None
        gevents = None
    else:
        params = mpcqp.default_params(N)
        solver = mpcqp.MpcQpSolver(params, device=local_rank)
        if dist_on and "MPCQP_SPLIT" not in os.environ:
            # a rank that runs RCCL solves its shard as one part: the caller's stream, RCCL's and the
            # split's two internal streams would exceed the process's four hardware queues
            # (GPU_MAX_HW_QUEUES); measured at C3's 8192-robot shard with the all-gather every step:
            # one part 3.00M QP/s, three parts 2.86M, no all-gather 3.02M (profiles/r06/rccl)
            solver.set_split(1)
        solver.reserve(Bl)
        d_rec = torch.from_numpy(recs_np).to(dev)
        d_res = torch.zeros((Bl, RD), dtype=torch.float64, device=dev)
        stream = torch.cuda.current_stream(dev)

        def solve():
            solver.solve_device(d_rec.data_ptr(), Bl, d_res.data_ptr(), 0, stream.cuda_stream)

        def sync():
            torch.cuda.synchronize(dev)
        events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.steps)]
        # the all-gather's own span (measured after the timed loop, one blocking gather per solve:
        # RCCL then makes the solve stream wait for it; for the gloo stub the host clock)
        gevents = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(min(args.steps, 10))] if dist_on else None
    gather_host_s = []
    # the production exchange, u0 of every robot on every rank after every solve: double-buffered
    # asynchronous all-gathers (mpcqp.distributed.ForceGather), each on RCCL's stream beside the next
    # solve; the timed region ends after the last one completed
    fg = ForceGather(total, 12, device=dev) if dist_on else None

    def step(k=None):
        if events is not None and k is not None:
            events[k][0].record(stream)
        solve()
        if events is not None and k is not None:
            events[k][1].record(stream)
        if dist_on:
            return fg.gather(d_res)
        return None

    for _ in range(args.warmup):
        step()
    if dist_on:
        fg.drain()
    sync()
    if dist_on:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(args.steps):
        full = step(k)
    if dist_on:
        full = fg.result(full)  # the last step's forces (waits for its all-gather)
        fg.drain()
    sync()
    if dist_on:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in events])) if events else None
    gather_ms = None
    if dist_on:
        # the all-gather's span alone (outside the timed region): solve, then one blocking gather
        # (solve end -> gather end; max over ranks below)
        for k in range(len(gevents) if gevents is not None else min(args.steps, 10)):
            solve()
            if gevents is not None:
                gevents[k][0].record(stream)
                allgather_forces(d_res[:, :12].contiguous(), total)
                gevents[k][1].record(stream)
            else:
                tg = time.perf_counter()
                allgather_forces(d_res[:, :12].contiguous(), total)
                gather_host_s.append(time.perf_counter() - tg)
        sync()
        if gevents is not None:
            gather_ms = float(np.mean([a.elapsed_time(b) for a, b in gevents]))
        else:
            gather_ms = float(np.mean(gather_host_s)) * 1e3
        gm = torch.tensor([gather_ms, kern_ms if kern_ms is not None else 0.0], dtype=torch.float64, device=dev)
        dist.all_reduce(gm, op=dist.ReduceOp.MAX)
        gather_ms = float(gm[0].item())
        kern_max_ms = float(gm[1].item())

    # whole results of every rank (outside the timed region) for the parity sample
    if dist_on:
        all_rows = allgather_forces(d_res, total).cpu().numpy()
        u0_full = full.cpu().numpy()
    else:
        all_rows = d_res.cpu().numpy()
        u0_full = all_rows[:, :12]
    res_all = np.frombuffer(np.ascontiguousarray(all_rows).tobytes(), dtype=mpcqp.RESULT_DTYPE).copy()
    local_res = res_all[b0:b1]
    value = total * args.steps / elapsed

    out = None
    if rank == 0:
        out = {"metric": METRIC, "value": value, "unit": "QP/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "f64",
               "data": "synthetic (seeded Go1 states per SURVEY §8(d); no dataset needed)"}
        cname = config_name(N, B, world, args.gait, args.mixed_mu)
        workload_s = (f"{cname + ': ' if cname else ''}"
                      f"Go1 convex-MPC GRF QP, horizon {N} (n={12 * N}, m={20 * N}), {B} robots/GPU, "
                      f"{args.gait} gait{', mu~U(0.3,0.9)' if args.mixed_mu else ''}; "
                      f"cold-start OSQP-0.6 settings, adaptive-rho interval 25")
        out["config"] = {"workload": workload_s, "batch_per_gpu": B, "global_batch": total, "horizon": N,
                         "gait": args.gait, "parallelism": f"dp{world}", "ranks_seen": ranks_seen,
                         "sharding": "contiguous shard_range of one seeded global batch per rank",
                         "collective": "RCCL all_gather of u0 per step (mpcqp.distributed.allgather_forces)"
                         if dist_on else "none"}
        gather_ok = bool(np.array_equal(u0_full, res_all["u0"])) if dist_on else True
        if dist_on:
            out["extras"] = {"allgather_ms": gather_ms, "solve_kernel_ms_max_over_ranks": kern_max_ms,
                             "allgather_what": ("the all-gather of u0 alone, measured after the timed loop: "
                                                "end of a solve -> end of one blocking all-gather (HIP "
                                                "events on the solve stream; gloo stub: host clock), mean "
                                                "over 10 solves, max over ranks.  Inside the timed loop the "
                                                "gathers are double-buffered and asynchronous (ForceGather): "
                                                "each runs on RCCL's stream beside the next solve"),
                             "allgather_bytes_per_rank": int(Bl * 12 * 8),
                             "backend": dist.get_backend()}
        if args.cpu_stub:
            exp = stub_results(recs_global)
            out["parity"] = {"gather_exact": bool(np.array_equal(u0_full, exp["u0"]) and gather_ok),
                             "instances": int(total)}
            out["roofline"] = None
            out["cpu_baseline"] = None
        else:
            ks = 1 if N <= 10 else 0  # KKT form of the launch: Schur (N <= 10, default weights) / Riccati
            eff_name = f"mpcqp::wv::scale_kernel<{N}> + mpcqp::wv::wave_kernel<{N}, {ks}>"
            flops = algorithmic_flops(N, local_res["iters"], local_res["rho_updates"])  # rank 0's launch
            achieved = flops / (kern_ms * 1e-3) / 1e12
            key = f"N{N}_B{B}_{args.gait}{'_mu' if args.mixed_mu else ''}"
            out["roofline"] = {
                "bound": "valu_fp64", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": achieved / FP64_PEAK_TFLOPS, "traffic": load_traffic(key, eff_name),
                "kernel": eff_name, "kernel_ms": kern_ms, "algorithmic_flop_per_launch": flops,
                # the FLOPs the kernels actually issue (PMC pass, profiles/pmc_flops.json) over the same
                # span: the Schur form executes fewer than SURVEY §8(d)'s dense count
                **executed_fields(key, eff_name, kern_ms),
                "parts": solver.split_parts(Bl),
                "kernel_ms_what": ("span of one solve call on the caller's stream (HIP events): the batch's "
                                   "scale_kernel + wave_kernel pairs, split into `parts` concurrent parts on the "
                                   "handle's internal streams; a rocprofv3 kernel trace gives the same span as "
                                   "the first launch's start to the last launch's end of each step "
                                   "(tools/trace_span.py)"),
                "note": ("binary64 on the VALU (v_fmac_f64 DPP) and the matrix cores (v_mfma_f64_16x16x4f64): "
                         + ("impulse-space Schur-form KKT solve (one dense 6N x 6N mat-vec per ADMM "
                            "iteration, blocked Gauss-Jordan per rho on the matrix cores)" if N <= 10 else
                            "Riccati-form KKT solve (chains of 12x12 mat-vecs per iteration, factorization "
                            "on v_mfma_f64_16x16x4f64)")
                         + "; FLOPs = SURVEY §8(d)'s structure-exploiting count per robot with its actual "
                           "iterations and rho updates; peak = FP64 vector spec (= FP64 MFMA peak on gfx950)")}
            pyoracle = None
            if not args.no_cpu:
                pyoracle = oracle_module()
                op = pyoracle.default_params(N, q=list(params.q_weights), r=list(params.r_weights))
                S = min(PARITY_SAMPLE, total)
                idx = np.unique(np.linspace(0, total - 1, S).astype(np.int64))  # every shard represented
                ref = pyoracle.solve_batch(op, recs_global[idx], nthreads=min(16, os.cpu_count() or 1))
                out["parity"] = parity_of(res_all[idx], ref)
                out["parity"]["sample"] = f"{len(idx)} robots evenly spaced over the global batch"
                out["parity"]["gathered_u0_equals_rank_results"] = gather_ok
                if not dist_on:
                    out["cpu_baseline"] = cpu_baseline(pyoracle, op, recs_np, args)
            else:
                out["parity"] = None
            out["cpu_baseline"] = out.get("cpu_baseline")
            out["stats"] = {"mean_iters": float(res_all["iters"].mean()), "max_iters": int(res_all["iters"].max()),
                            "mean_rho_updates": float(res_all["rho_updates"].mean()),
                            "solved_frac": float(np.mean(res_all["status"] == 1)),
                            "handoff_count": list(solver.handoff_counts()) if N <= 10 else None}
            if not dist_on and not args.no_extras:
                out["extras"] = extras(args, solver, params, recs_np, states, local_res, pyoracle, dev)
    if solver is not None:
        solver.close()
    if dist_on:
        dist.destroy_process_group()
    return out


def host_cpu():
    """(model name, nproc, CPUs this process may run on) of the host."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = os.cpu_count() or 1
    return model, os.cpu_count() or 1, usable


def cpu_baseline(pyoracle, op, recs_np, args):
    S = min(args.cpu_sample, recs_np.shape[0])
    model, nproc, usable = host_cpu()
    # The GPU box allots 16 CPUs per GPU (its harness rule for worker pools; nproc there shows the
    # whole machine): the timed run uses that share, and the line also gives the all-cores figure
    # extrapolated from the single-thread rate (robots are independent: linear at best).
    nthr = args.cpu_threads or min(16, usable)
    pyoracle.solve_batch(op, recs_np[:min(S, 64)], nthreads=nthr)  # warm
    tc = time.perf_counter()
    pyoracle.solve_batch(op, recs_np[:S], nthreads=nthr)
    tcpu = time.perf_counter() - tc
    t1 = time.perf_counter()
    n1 = min(S, 128)
    pyoracle.solve_batch(op, recs_np[:n1], nthreads=1)
    t1 = (time.perf_counter() - t1) / n1
    return {"value": S / tcpu, "unit": "QP/s", "cores": nthr, "kind": "port",
            "sample": f"first {S} instances of this workload (same seed) on oracle/mpc_oracle.c "
                      f"(binary64 ConvexMpc + OSQP-0.6 restatement), {nthr} host threads; "
                      f"single-thread {t1 * 1e6:.0f} us/QP",
            "single_thread_us_per_qp": t1 * 1e6, "cpu_model": model, "nproc": nproc,
            "cpus_usable": usable, "threads_used": nthr,
            "all_cores_extrapolated_value": nproc / t1,
            "all_cores_note": "nproc x the single-thread rate (perfect scaling assumed; an upper bound "
                              "on the whole host, not measured: the box allots 16 CPUs per GPU)"}


def _timed(fn, steps, stream):
    """mean ms per call of fn() between HIP events on `stream` (one warm call first)."""
    import torch
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(stream)
    for _ in range(steps):
        fn()
    ev[1].record(stream)
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / steps


def extras(args, solver, params, recs_np, states, base_res, pyoracle, dev):
    """N = 1 extra keys (SURVEY §8(d) end-to-end figures, configs C4 / C5, warm ticks)."""
    import torch
    import mpcqp
    from mpcqp.records import synthetic_go1_ticks

    N, B = args.horizon, recs_np.shape[0]
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    RD = mpcqp._lib.RESULT_DOUBLES
    steps = max(3, args.steps // 2)
    nthr = min(16, os.cpu_count() or 1)
    ex = {}

    def res_of(t):
        return np.frombuffer(t.cpu().numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE).copy()

    # -- e2e: host records in, host results out, through the C ABI's host wrapper -------------
    h_rec = torch.from_numpy(recs_np).pin_memory()
    h_res = torch.zeros((B, RD), dtype=torch.float64).pin_memory()
    solver.solve_host_ptr(h_rec.data_ptr(), B, h_res.data_ptr())
    t0 = time.perf_counter()
    for _ in range(steps):
        solver.solve_host_ptr(h_rec.data_ptr(), B, h_res.data_ptr())
    ms_pin = (time.perf_counter() - t0) / steps * 1e3
    got_pin = np.frombuffer(h_res.numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE)
    res_pg = solver.solve_host(recs_np)
    t0 = time.perf_counter()
    for _ in range(steps):
        res_pg = solver.solve_host(recs_np)
    ms_pg = (time.perf_counter() - t0) / steps * 1e3
    ex["e2e"] = {"value": B / (ms_pin * 1e-3), "unit": "QP/s", "ms_per_call": ms_pin,
                 "what": "mpcqp_solve_batch_host: pinned host records -> H2D -> solve -> D2H of the "
                         "results, synchronous (wall clock per call)",
                 "pageable_value": B / (ms_pg * 1e-3), "pageable_ms_per_call": ms_pg,
                 "bytes_h2d": int(recs_np.nbytes), "bytes_d2h": int(B * mpcqp.RESULT_DTYPE.itemsize),
                 "parity": {"bitwise_equal_device_path": bool(
                     np.array_equal(as_rows(got_pin), as_rows(base_res)) and
                     np.array_equal(as_rows(res_pg), as_rows(base_res)))}}

    # -- assemble_e2e: raw *CtrlStates rows resident in HBM -> assembly kernel -> solve ---------
    d_st = torch.from_numpy(mpcqp.pack_states(states)[:B]).to(dev)
    d_rec2 = torch.zeros((B, mpcqp.rec_size(N)), dtype=torch.float64, device=dev)
    d_res2 = torch.zeros((B, RD), dtype=torch.float64, device=dev)

    def asm_solve():
        mpcqp.assemble_records_device(N, d_st.data_ptr(), B, d_rec2.data_ptr(), sp)
        solver.solve_device(d_rec2.data_ptr(), B, d_res2.data_ptr(), 0, sp)
    ms = _timed(asm_solve, steps, stream)
    ex["assemble_e2e"] = {"value": B / (ms * 1e-3), "unit": "QP/s", "ms_per_step": ms,
                          "what": "mpcqp_assemble_records_device + mpcqp_solve_batch_device (HIP events)",
                          "parity": {"records_bitwise_equal_host_assembly": bool(
                              np.array_equal(d_rec2.cpu().numpy(), recs_np)),
                              "u0_bitwise_equal_device_path": bool(
                              np.array_equal(res_of(d_res2)["u0"], base_res["u0"]))}}

    # -- two_streams: consecutive independent C2 batches alternating over two handles / streams, so
    # that one batch's dispatch tail overlaps the next batch's start (the caller-side remedy for the
    # tail; not the headline: there one batch is solved at a time) -------------------------------
    sA, sB = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    with mpcqp.MpcQpSolver(params, device=dev.index) as s2:
        s2.reserve(B)
        dA = torch.from_numpy(recs_np).to(dev)
        dB = torch.from_numpy(recs_np).to(dev)
        rA = torch.zeros((B, RD), dtype=torch.float64, device=dev)
        rB = torch.zeros((B, RD), dtype=torch.float64, device=dev)
        launch = [lambda: solver.solve_device(dA.data_ptr(), B, rA.data_ptr(), 0, sA.cuda_stream),
                  lambda: s2.solve_device(dB.data_ptr(), B, rB.data_ptr(), 0, sB.cuda_stream)]
        torch.cuda.synchronize()
        launch[0]()
        launch[1]()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(stream)
        sA.wait_stream(stream)
        sB.wait_stream(stream)
        nb = 2 * steps
        for k in range(nb):
            launch[k & 1]()
        stream.wait_stream(sA)
        stream.wait_stream(sB)
        ev[1].record(stream)
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / nb
        same = bool(np.array_equal(as_rows(res_of(rA)), as_rows(base_res)) and
                    np.array_equal(as_rows(res_of(rB)), as_rows(base_res)))
    ex["two_streams"] = {"value": B / (ms * 1e-3), "unit": "QP/s", "ms_per_batch": ms, "batches": nb,
                         "what": "independent %d-robot C2 batches alternating over two handles on two "
                                 "streams (HIP events around all of them)" % B,
                         "parity": {"bitwise_equal_single_stream": same}}

    # -- C5: mixed gait, per-robot contacts ~ Bernoulli(0.5)^4 and mu ~ U(0.3, 0.9), 8192 robots -
    B5 = 8192
    st5, rec5 = workload(10, B5, "mixed", True)
    with mpcqp.MpcQpSolver(mpcqp.default_params(10), device=dev.index) as s5:
        s5.reserve(B5)
        d5 = torch.from_numpy(rec5).to(dev)
        r5 = torch.zeros((B5, RD), dtype=torch.float64, device=dev)
        ms = _timed(lambda: s5.solve_device(d5.data_ptr(), B5, r5.data_ptr(), 0, sp), steps, stream)
        g5 = res_of(r5)
        h5 = s5.handoff_counts()
    ent = {"value": B5 / (ms * 1e-3), "unit": "QP/s", "ms_per_step": ms, "batch": B5, "horizon": 10,
           "workload": "C5: mixed gait, contacts ~ Bernoulli(0.5)^4, mu ~ U(0.3,0.9)",
           "mean_iters": float(g5["iters"].mean()),
           "handoff_count": {"rank_deficient_feet": h5[0], "cancellation_smax_x_amp": h5[1],
                             "smax_cap": h5[2],
                             "what": "robots the Riccati form solved in their own wave (mpcqp_handoff_counts)"}}
    if pyoracle is not None:
        idx = np.unique(np.linspace(0, B5 - 1, 512).astype(np.int64))
        ref = pyoracle.solve_batch(pyoracle.default_params(10), rec5[idx], nthreads=nthr)
        ent["parity"] = parity_of(g5[idx], ref)
    ex["c5"] = ent

    # -- C3 shard: what one of the 8 GPUs of C3 solves per step (shard 0 of the 65536-robot global
    # batch), and the batch-size curve of the same seeded global batch (dispatch-tail evidence) --
    from mpcqp.distributed import shard_range
    _, rec3 = workload(10, C3_BATCH_PER_GPU * C3_GPUS, "trot", False)
    with mpcqp.MpcQpSolver(mpcqp.default_params(10), device=dev.index) as s3:
        curve = {}
        for Bc in (C2_BATCH, C3_BATCH_PER_GPU, 16384, C3_BATCH_PER_GPU * C3_GPUS):
            s3.reserve(Bc)
            d3 = torch.from_numpy(np.ascontiguousarray(rec3[:Bc])).to(dev)
            r3 = torch.zeros((Bc, RD), dtype=torch.float64, device=dev)
            ms = _timed(lambda: s3.solve_device(d3.data_ptr(), Bc, r3.data_ptr(), 0, sp),
                        max(3, steps // (1 if Bc <= 16384 else 4)), stream)
            g3 = res_of(r3)
            curve[str(Bc)] = {"value": Bc / (ms * 1e-3), "ms_per_step": ms, "mean_iters": float(g3["iters"].mean())}
            if Bc == C3_BATCH_PER_GPU:
                b0, b1 = shard_range(C3_BATCH_PER_GPU * C3_GPUS, C3_GPUS, 0)
                assert (b0, b1) == (0, Bc)
                ent = {"value": Bc / (ms * 1e-3), "unit": "QP/s", "ms_per_step": ms, "batch": Bc, "horizon": 10,
                       "workload": "C3 shard: robots [0, 8192) of the C3 global batch (65536 trot robots, seed "
                                   "1000), i.e. rank 0's per-step solve at --gpus 8, on one GPU, no collective",
                       "mean_iters": float(g3["iters"].mean())}
                if pyoracle is not None:
                    idx = np.unique(np.linspace(0, Bc - 1, 512).astype(np.int64))
                    ref = pyoracle.solve_batch(pyoracle.default_params(10), rec3[idx], nthreads=nthr)
                    ent["parity"] = parity_of(g3[idx], ref)
                ex["c3_shard"] = ent
            del d3, r3
    ex["batch_scaling"] = {"what": "one GPU, prefixes of the C3 global batch (65536 trot robots, N = 10), "
                                   "scale_kernel + wave_kernel by HIP events; rate vs batch shows the dispatch tail",
                           "points": curve}

    # -- C4: horizon 20, 4096 trot robots --------------------------------------------------------
    B4 = 4096
    st4, rec4 = workload(20, B4, "trot", False)
    with mpcqp.MpcQpSolver(mpcqp.default_params(20), device=dev.index) as s4:
        s4.reserve(B4)
        d4 = torch.from_numpy(rec4).to(dev)
        r4 = torch.zeros((B4, RD), dtype=torch.float64, device=dev)
        ms = _timed(lambda: s4.solve_device(d4.data_ptr(), B4, r4.data_ptr(), 0, sp), max(3, steps // 2), stream)
        g4 = res_of(r4)
    fl = algorithmic_flops(20, g4["iters"], g4["rho_updates"])
    ent = {"value": B4 / (ms * 1e-3), "unit": "QP/s", "ms_per_step": ms, "batch": B4, "horizon": 20,
           "workload": "C4: horizon 20 (n=240, m=400), trot", "mean_iters": float(g4["iters"].mean()),
           "roofline_frac": fl / (ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
           **executed_fields("N20_B4096_trot", "mpcqp::wv::scale_kernel<20> + mpcqp::wv::wave_kernel<20, 0>", ms),
           # HBM bytes per launch of the N = 20 solve from its own rocprofv3 PMC pass (profiles/)
           "traffic": load_traffic("N20_B4096_trot",
                                   "mpcqp::wv::scale_kernel<20> + mpcqp::wv::wave_kernel<20, 0>"),
           "kernels": "scale_kernel<20> + wave_kernel<20, 0> (Riccati form, factorization on MFMA)"}
    if pyoracle is not None:
        idx = np.unique(np.linspace(0, B4 - 1, 256).astype(np.int64))
        ref = pyoracle.solve_batch(pyoracle.default_params(20), rec4[idx], nthreads=nthr)
        ent["parity"] = parity_of(g4[idx], ref)
    ex["c4"] = ent

    # -- warm_tick: the production tick sequence (persistent warm-started solver per robot) ------
    T = 10
    ticks = synthetic_go1_ticks(B, T, seed=31, gait="trot", swing_ticks=5)
    recs_t = np.stack([mpcqp.assemble_compute_grf(s, N) for s in ticks])
    d_t = torch.from_numpy(recs_t).to(dev)
    d_w = torch.zeros((B, solver.warm_state_size), dtype=torch.float64, device=dev)
    d_rw = torch.zeros((T, B, RD), dtype=torch.float64, device=dev)
    d_rc = torch.zeros((T, B, RD), dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record(stream)
    for t in range(T):
        solver.solve_warm_device(d_t[t].data_ptr(), B, d_w.data_ptr(), d_rw[t].data_ptr(), 0, sp)
    ev[1].record(stream)
    ev[2].record(stream)
    for t in range(T):
        solver.solve_device(d_t[t].data_ptr(), B, d_rc[t].data_ptr(), 0, sp)
    ev[3].record(stream)
    torch.cuda.synchronize()
    ms_w = ev[0].elapsed_time(ev[1]) / T
    ms_c = ev[2].elapsed_time(ev[3]) / T
    gw = np.frombuffer(d_rw.cpu().numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE).reshape(T, B)
    gc = np.frombuffer(d_rc.cpu().numpy().tobytes(), dtype=mpcqp.RESULT_DTYPE).reshape(T, B)
    ent = {"value": B / (ms_w * 1e-3), "unit": "QP/s", "ms_per_tick": ms_w, "ticks": T, "batch": B,
           "cold_ms_per_tick": ms_c, "mean_iters_warm_ticks_2_on": float(gw[1:]["iters"].mean()),
           "mean_iters_cold": float(gc[1:]["iters"].mean()),
           "what": "mpcqp_solve_batch_warm_device over consecutive ticks (OsqpEigen warm start: update_P "
                   "or re-init per robot), synthetic closed-loop trot trajectories"}
    if pyoracle is not None:
        nb = 64
        ref = pyoracle.solve_sequence(pyoracle.default_params(N), np.ascontiguousarray(recs_t[:, :nb]),
                                      nthreads=nthr)
        errs = [parity_of(gw[t, :nb], ref[t]) for t in range(T)]
        ent["parity"] = {"robots": nb, "ticks": T,
                         "max_rel_err_u0": max(e["max_rel_err_u0"] for e in errs),
                         "status_equal": all(e["status_equal"] for e in errs),
                         "iters_equal_frac": float(np.mean([e["iters_equal_frac"] for e in errs]))}
    ex["warm_tick"] = ent
    return ex


def main(argv=None):
    args = parse_args(argv)
    from mpcqp.distributed import env_rank, launch_ranks
    if (args.gpus > 1 or args.dist) and "WORLD_SIZE" not in os.environ:
        # launcher: this process never touches the GPU; the ranks each open their own device
        return launch_ranks(os.path.abspath(__file__), sys.argv[1:] if argv is None else argv, args.gpus)
    out = run_rank(args)
    if out is not None:
        print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

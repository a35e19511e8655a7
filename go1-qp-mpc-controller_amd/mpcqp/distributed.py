"""Multi-GPU sharding of a robot batch.

Robot instances are independent: GPU g solves the contiguous shard [g*B/G, (g+1)*B/G); the only
exchange is one all-gather of the solved first-step forces u0 (12 doubles per robot) so every rank
holds the whole batch's GRFs (north_star: "RCCL all-gather of solved ground-reaction forces over
xGMI").  One process per GPU; torch.distributed with backend "nccl" (= RCCL on ROCm) on the GPUs,
"gloo" in the CPU tests.

``launch_ranks`` starts those processes from a parent that never touches the GPU: it runs
``python -m torch.distributed.run`` as a CHILD process (never an exec of the current process) and
returns its exit code.
"""
import os
import socket
import subprocess
import sys

import torch
import torch.distributed as dist


def shard_range(total, world, rank):
    """Contiguous, balanced shard [begin, end) of `total` robots for `rank` of `world`."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    base, rem = divmod(total, world)
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


def allgather_forces(local, total, group=None):
    """All-gather per-rank [b_r, k] rows (u0: k = 12) into [total, k] on every rank.

    Shards may differ by one row (balanced split); they are padded to ceil(total/world) for a
    single all_gather_into_tensor and the padding is stripped.  With a balanced split into equal
    shards no padding copy is made.
    """
    world = dist.get_world_size(group)
    chunk = -(-total // world)
    if local.shape[0] == chunk and local.is_contiguous():
        pad = local
    else:
        pad = torch.zeros((chunk, local.shape[1]), dtype=local.dtype, device=local.device)
        pad[: local.shape[0]] = local
    out = torch.empty((world * chunk, local.shape[1]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, pad, group=group)
    if chunk * world == total:
        return out
    rows = []
    for r in range(world):
        b, e = shard_range(total, world, r)
        rows.append(out[r * chunk: r * chunk + (e - b)])
    return torch.cat(rows, 0)


class ForceGather:
    """Double-buffered asynchronous all-gather of the solved forces (the per-tick exchange of C3).

    ``gather(results)`` copies u0 (the first ``k`` columns of the rank's result rows) into a send
    buffer on the current stream and issues ``all_gather_into_tensor(async_op=True)``: the collective
    runs on the backend's own stream (RCCL) beside the next tick's solve, which writes the results
    again without waiting for it; a send / receive buffer pair is reused only after the collective
    that last used it has completed (``Work.wait``: a stream dependency for RCCL, a host wait for gloo).
    ``result(h)`` waits for gather ``h`` and returns the [total, k] forces (padding stripped);
    ``drain()`` waits for every gather in flight.  Shards may differ by one row (balanced split):
    the send buffer holds ceil(total / world) rows, as in ``allgather_forces``."""

    def __init__(self, total, k=12, device=None, dtype=torch.float64, group=None, depth=2):
        self.world = dist.get_world_size(group)
        self.total, self.k, self.group = total, k, group
        self.chunk = -(-total // self.world)
        self.send = [torch.zeros((self.chunk, k), dtype=dtype, device=device) for _ in range(depth)]
        self.out = [torch.empty((self.world * self.chunk, k), dtype=dtype, device=device) for _ in range(depth)]
        self.works = [None] * depth
        self.n = 0

    def _wait(self, i):
        if self.works[i] is not None:
            self.works[i].wait()
            self.works[i] = None

    def gather(self, results):
        i = self.n % len(self.send)
        self._wait(i)
        self.send[i][: results.shape[0]].copy_(results[:, : self.k])
        self.works[i] = dist.all_gather_into_tensor(self.out[i], self.send[i], group=self.group, async_op=True)
        self.n += 1
        return i

    def result(self, h):
        self._wait(h)
        out = self.out[h]
        if self.chunk * self.world == self.total:
            return out
        rows = []
        for r in range(self.world):
            b, e = shard_range(self.total, self.world, r)
            rows.append(out[r * self.chunk: r * self.chunk + (e - b)])
        return torch.cat(rows, 0)

    def drain(self):
        for i in range(len(self.works)):
            self._wait(i)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launcher_cmd(script, argv, nproc, port):
    """torch.distributed.run command line: one process per GPU of one node, rendezvous on
    127.0.0.1 (the container hostname may not resolve)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={int(nproc)}",
            "--master-addr", "127.0.0.1", "--master-port", str(int(port)), script] + list(argv)


def launch_ranks(script, argv, nproc, env=None, port=None):
    """Run `script argv` on `nproc` ranks as a child process tree; returns the exit code.

    The caller must not have initialised the GPU (no HIP call, no torch.cuda.is_available()):
    the ranks each open their own device."""
    e = dict(os.environ if env is None else env)
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK"):
        e.pop(k, None)
    cmd = launcher_cmd(script, argv, nproc, port or free_port())
    return subprocess.call(cmd, env=e)


def env_rank():
    """(world, rank, local_rank) from the torch.distributed.run environment (1, 0, 0 when absent)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))

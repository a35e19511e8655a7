"""One fused control tick for a fleet of robots, entirely on the device:

    raw *CtrlStates rows --assemble--> MPC records --warm solve--> mpcqp_result --torque map--> tau

i.e. the MPC branch of A1RobotControl::compute_grf (A1RobotControl.cpp:446-561, with the
persistent warm-started solver of A1RobotControl.h:67) followed by compute_joint_torques
(:289-319), three kernels on one stream with no host round trip.  ``capture()`` records the tick
as a HIP graph (torch.cuda.CUDAGraph is hipGraph on ROCm), so a simulator steps with one replay.
torch is used only to own device buffers and the capture stream.
"""
from . import _lib
from .solver import MpcQpSolver
from .torques import joint_torques_device


class ControlTick:
    def __init__(self, batch, params=None, device=0):
        import torch
        self.torch = torch
        self.B = int(batch)
        self.solver = MpcQpSolver(params if params is not None else _lib.default_params(10), device=device)
        self.solver.reserve(self.B)
        N = self.solver.horizon
        dev = f"cuda:{device}"
        f64 = dict(dtype=torch.float64, device=dev)
        self.states = torch.zeros((self.B, _lib.ST_SIZE), **f64)        # caller writes robot states here
        self.tq_records = torch.zeros((self.B, _lib.TQ_SIZE), **f64)    # and Jacobians / swing forces here
        self.records = torch.zeros((self.B, _lib.rec_size(N)), **f64)
        self.warm = torch.zeros((self.B, self.solver.warm_state_size), **f64)
        self.results = torch.zeros((self.B, _lib.RESULT_DOUBLES), **f64)
        self.counter = torch.zeros((self.B,), dtype=torch.int32, device=dev)
        self.torques = torch.zeros((self.B, 12), **f64)
        self.graph = None

    def step(self, stream=None):
        """Enqueue one tick on `stream` (default: torch's current stream)."""
        s = stream if stream is not None else self.torch.cuda.current_stream().cuda_stream
        _lib.assemble_records_device(self.solver.horizon, self.states.data_ptr(), self.B, self.records.data_ptr(), s)
        self.solver.solve_warm_device(self.records.data_ptr(), self.B, self.warm.data_ptr(), self.results.data_ptr(),
                                      0, s)
        joint_torques_device(self.tq_records.data_ptr(), self.results.data_ptr(), self.B, self.counter.data_ptr(),
                             self.torques.data_ptr(), s)

    def capture(self):
        """Record step() as a graph.  Warm slots, counters and torques keep evolving on replay,
        exactly as with eager steps; capture itself launches nothing."""
        torch = self.torch
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.step()
        self.graph = g
        return g

    def replay(self):
        self.graph.replay()

    def close(self):
        self.solver.close()

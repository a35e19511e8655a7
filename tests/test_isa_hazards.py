"""Static check of the product kernels' gfx950 ISA (tools/isa_hazards.py): the inline-asm DPP blocks
wait only where the compiled code needs it (mpcqp_wave_common.h, DPP wait states), so every build
must show no DPP / permlane / transcendental / untracked-load hazard.  Every horizon the product
library instantiates is checked (each N is scheduled separately; the round-6 check found
two real DPP hazards at N = 7 and 8 that the N = 10 / 20 check could not see): wave_kernel<N, 1> for
N <= 10, wave_kernel<N, 0> and scale_kernel<N> for N = 1..20.  CPU only (hipcc -S, one compile per
horizon, in parallel)."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _kernels(n):
    # wave_kernel<N, KS>: the Schur form (KS = 1, N <= 10) and the Riccati form (KS = 0)
    return ([f"wave_kernelILi{n}ELi1E"] if n <= 10 else []) + [f"wave_kernelILi{n}ELi0E", f"scale_kernelILi{n}E"]


def _check(n):
    kernels = _kernels(n)
    cmd = [sys.executable, os.path.join(REPO, "tools", "isa_hazards.py"), "--n", str(n), "--kernels"] + kernels
    return subprocess.run(cmd, capture_output=True, text=True, timeout=1200)


def test_product_kernels_have_no_isa_hazards():
    horizons = list(range(20, 0, -1))  # the long compiles first
    with ThreadPoolExecutor(min(8, os.cpu_count() or 1)) as ex:
        outs = list(ex.map(_check, horizons))
    for n, o in zip(horizons, outs):
        assert o.returncode == 0, f"N={n}:\n{o.stdout[-3000:]}{o.stderr[-2000:]}"
        assert o.stdout.count("hazards none") == len(_kernels(n)), f"N={n}:\n{o.stdout}"


def test_scalar_sweep_build_has_no_isa_hazards():
    """The in-register scalar Gauss-Jordan (-DMPCQP_GJ_MFMA=0, the pre-round-6 default kept as a
    build option) still compiles hazard-free at N = 10."""
    cmd = [sys.executable, os.path.join(REPO, "tools", "isa_hazards.py"), "--n", "10", "--defs=-DMPCQP_GJ_MFMA=0",
           "--kernels", "wave_kernelILi10ELi1E"]
    o = subprocess.run(cmd, capture_output=True, text=True, timeout=1200)
    assert o.returncode == 0 and "hazards none" in o.stdout, o.stdout[-3000:] + o.stderr[-2000:]

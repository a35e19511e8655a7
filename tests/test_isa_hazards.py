"""Static check of the product kernels' gfx950 ISA (tools/isa_hazards.py): the inline-asm DPP blocks
wait only where the compiled code needs it (mpcqp_wave_common.h, DPP wait states), so every build
must show no DPP / permlane / transcendental / untracked-load hazard at the horizons the benchmarks
run (N = 10: Schur form with the Riccati hand-off; N = 20: Riccati form).  CPU only (hipcc -S)."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _check(n, kernels):
    cmd = [sys.executable, os.path.join(REPO, "tools", "isa_hazards.py"), "--n", str(n), "--kernels"] + kernels
    return subprocess.run(cmd, capture_output=True, text=True, timeout=900)


def test_product_kernels_have_no_isa_hazards():
    jobs = [(10, ["wave_kernelILi10ELi1E", "wave_kernelILi10ELi0E", "scale_kernelILi10E"]),
            (20, ["wave_kernelILi20ELi0E", "scale_kernelILi20E"])]
    with ThreadPoolExecutor(2) as ex:
        outs = list(ex.map(lambda j: _check(*j), jobs))
    for (n, _), o in zip(jobs, outs):
        assert o.returncode == 0, f"N={n}:\n{o.stdout[-3000:]}{o.stderr[-2000:]}"
        assert "hazards none" in o.stdout

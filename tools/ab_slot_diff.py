"""Compare two warm-start slot dumps of tools/ab_warm.py (AB_SLOT_OUT) region by region."""
import sys

import numpy as np

sys.path.insert(0, "go1-qp-mpc-controller_amd")
a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
n, m, N = 120, 200, 10
MW = (n + 63) // 64
off = {"flag": 0, "rho": 1, "c": 2, "mu": 3, "D": 4, "E": 4 + n, "QT": 4 + n + m, "AK": 4 + 2 * n + m,
       "X": 4 + 2 * n + 3 * m, "Z": 4 + 3 * n + 3 * m, "Y": 4 + 3 * n + 4 * m, "MASK": 4 + 3 * n + 5 * m}
keys = list(off)
for i, k in enumerate(keys):
    lo = off[k]
    hi = off[keys[i + 1]] if i + 1 < len(keys) else lo + MW * n
    d = np.abs(a[:, lo:hi] - b[:, lo:hi])
    print(f"{k:5s} max|diff| {np.nanmax(d):.3e}  first bad robot/idx {np.argwhere(d > 1e-9)[:3].tolist()}")

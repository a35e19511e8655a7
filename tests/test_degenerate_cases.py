"""CPU checks of the degenerate-feet fixtures (tests/degenerate_cases.py): the host Gram screen's
threshold is the kernel's, exactly rank-deficient feet give a ratio of ~0, the synthetic Go1
workloads sit far above the threshold, and the near-degenerate families shrink as eps^2 (once eps sets the smallest pivot)."""
import os
import re

import numpy as np

import mpcqp
from degenerate_cases import SCHUR_GRAM_TOL, degenerate, gram_ratio, near_degenerate

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_threshold_matches_the_kernel():
    src = open(os.path.join(REPO, "go1-qp-mpc-controller_amd", "csrc", "mpcqp_wave_common.h")).read()
    m = re.search(r"#define MPCQP_SCHUR_GRAM_TOL\s+([0-9.eE+-]+)", src)
    assert m and float(m.group(1)) == SCHUR_GRAM_TOL


def test_rank_deficient_kinds_and_go1_margin():
    N = 10
    for gait, mu in (("trot", False), ("stance", False), ("mixed", True)):
        recs = mpcqp.assemble_compute_grf(mpcqp.synthetic_go1(128, seed=3, gait=gait, mixed_mu=mu), N)
        assert gram_ratio(recs, N).min() > 0.1  # C2-C5 feet: 5 orders above the threshold
        g = gram_ratio(degenerate(recs[:12], N), N)
        kinds = np.arange(12) % 4
        assert np.all(g[kinds <= 2] < 1e-12)
        assert np.all((g[kinds == 3] > 1e-8) & (g[kinds == 3] < 1e-4))  # near-collinear, not singular


def test_near_degenerate_ratio_shrinks_with_eps():
    N = 5
    recs = mpcqp.assemble_compute_grf(mpcqp.synthetic_go1(8, seed=4, gait="trot"), N)
    for kind in ("inplane", "outplane", "point"):
        a = gram_ratio(near_degenerate(recs, N, 1e-5, kind), N)
        b = gram_ratio(near_degenerate(recs, N, 1e-6, kind), N)
        assert np.all((b > 0) & (b < a / 50.0)), kind

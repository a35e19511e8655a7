#!/usr/bin/env python3
"""Executed binary64 FLOPs per solve from a rocprofv3 counter pass (VERDICT r05 "do this" 3).

Collect in its own pass (no tracing flags with --pmc; at most 8 SQ counters):

  rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 \\
      SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVE_CYCLES \\
      --kernel-include-regex "scale_kernel|wave_kernel" --output-format csv -d gpurun_out/flops/h10 -o pmc \\
      -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extras
  python3 tools/pmc_flops.py gpurun_out/flops/h10 --key N10_B4096_trot --parts 3 [--calib CALIB_DIR]

Units.  The SQ_INSTS_VALU_* counters count wave-level instructions (one per wave, whatever the exec
mask): the calibration pass over tools/mb/mb_valu (k_fma: 201 x 128 v_fmac_f64 per wave x 1024 waves
per timed launch; k_max: 64 v_add_f64) checks that, and the result records the ratio it measured.
A wave instruction is counted as 64 lanes: FMA = 2 FLOP per lane, ADD / MUL = 1, so the figure is an
UPPER bound on useful FLOPs (masked lanes and padding lanes are counted).  SQ_INSTS_VALU_MFMA_MOPS_F64
counts matrix FLOPs in units of 512 (checked against SQ_INSTS_MFMA x 2048 FLOP per
v_mfma_f64_16x16x4f64 where the kernel issues only that MFMA).  Transcendentals (rcp / sqrt / rsq)
are listed but not counted as FLOPs.
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COUNTERS = ["SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_TRANS_F64",
            "SQ_INSTS_VALU_MFMA_MOPS_F64", "SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_WAVE_CYCLES"]


def parse(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {d}")
    per = defaultdict(dict)
    names = {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                did = (fn, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                per[did][row["Counter_Name"]] = per[did].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
                names[did] = row.get("Kernel_Name", "")
    return per, names


def means(per, names, substr):
    ds = sorted([d for d in per if substr in names[d]], key=lambda d: (d[0], int(d[1]) if str(d[1]).isdigit() else 0))
    if len(ds) > 1:
        ds = ds[1:]  # the first (cold) dispatch
    out = {}
    for c in COUNTERS:
        vals = [per[d][c] for d in ds if c in per[d]]
        if vals:
            out[c] = sum(vals) / len(vals)
    return out, len(ds), (sorted({names[d] for d in ds}) or [""])[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--key", required=True)
    ap.add_argument("--kernel", default="scale_kernel,wave_kernel")
    ap.add_argument("--parts", type=int, default=1, help="launches of each kernel per solve (batch split)")
    ap.add_argument("--calib", default=None, help="counter pass over tools/mb/mb_valu (k_fma, k_max)")
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "pmc_flops.json"))
    a = ap.parse_args()
    per, names = parse(a.dir)
    tot = defaultdict(float)
    kn = []
    for k in [k for k in a.kernel.split(",") if k]:
        m, nd, name = means(per, names, k)
        if not m:
            raise SystemExit(f"no dispatch of {k}")
        kn.append({"kernel": name, "dispatches": nd, "per_dispatch": m})
        for c, v in m.items():
            tot[c] += v * a.parts
    lane = 64.0
    valu_flop = lane * (2.0 * tot["SQ_INSTS_VALU_FMA_F64"] + tot["SQ_INSTS_VALU_ADD_F64"] + tot["SQ_INSTS_VALU_MUL_F64"])
    mfma_flop = 512.0 * tot.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0)
    entry = {"kernels": kn, "parts": a.parts, "per_solve": dict(tot),
             "valu_f64_flop_per_solve": valu_flop, "mfma_f64_flop_per_solve": mfma_flop,
             "executed_f64_flop_per_solve": valu_flop + mfma_flop,
             "units": "VALU: wave instructions x 64 lanes (FMA 2 FLOP); MFMA: MOPS x 512 FLOP"}
    if a.calib:
        cp, cn = parse(a.calib)
        cal = {}
        for k, fma, add in (("k_fma", 201 * 128 * 1024, 0), ("k_max", 0, 201 * 64 * 1024)):
            ds = [d for d in cp if cn[d].startswith(k) or (k + "(") in cn[d] or cn[d].endswith(k)]
            best = None
            for d in ds:  # the timed launch (iters = 200) is the one with the larger count
                v = cp[d]
                if best is None or v.get("SQ_INSTS_VALU", 0) > best.get("SQ_INSTS_VALU", 0):
                    best = v
            if best:
                cal[k] = {"expected_fma_wave_insts": fma, "expected_add_wave_insts": add,
                          "SQ_INSTS_VALU_FMA_F64": best.get("SQ_INSTS_VALU_FMA_F64"),
                          "SQ_INSTS_VALU_ADD_F64": best.get("SQ_INSTS_VALU_ADD_F64")}
        entry["calibration"] = cal
    try:
        with open(a.out) as f:
            allj = json.load(f)
    except (OSError, ValueError):
        allj = {}
    allj[a.key] = entry
    with open(a.out, "w") as f:
        json.dump(allj, f, indent=1)
    print(json.dumps({a.key: {k: v for k, v in entry.items() if k != "kernels"}}, indent=1))


if __name__ == "__main__":
    sys.exit(main())

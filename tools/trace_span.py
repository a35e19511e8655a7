#!/usr/bin/env python3
"""Per-solve spans from a rocprofv3 kernel trace (run_kernel_trace.csv): the solve kernels of one
bench step (scale_kernel + wave_kernel per batch part, the parts on concurrent streams) are grouped
by time — a step starts with a solve-kernel launch that begins after every earlier solve kernel
ended — and each step's span is its first start to its last end.  This is what bench.py's
roofline.kernel_ms measures with HIP events on the caller's stream.

  python tools/trace_span.py TRACE_CSV [--skip 2]
"""
import argparse
import csv
import json

import numpy as np


def spans(path, pattern=("scale_kernel", "wave_kernel")):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if any(p in r["Kernel_Name"] for p in pattern):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]))
    rows.sort()
    steps, cur, end = [], [], -1
    for s, e, name, q in rows:
        if cur and s > end:
            steps.append(cur)
            cur = []
        cur.append((s, e, name, q))
        end = max(end, e)
    if cur:
        steps.append(cur)
    return steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=2, help="leading steps to drop (warmup)")
    a = ap.parse_args()
    steps = spans(a.trace)
    use = steps[a.skip:]
    sp = [(max(e for _, e, _, _ in st) - min(s for s, _, _, _ in st)) * 1e-6 for st in use]
    out = {"steps": len(use), "launches_per_step": sorted({len(st) for st in use}),
           "queues_per_step": sorted({len({q for *_, q in st}) for st in use}),
           "span_ms_mean": float(np.mean(sp)) if sp else None, "span_ms_median": float(np.median(sp)) if sp else None}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

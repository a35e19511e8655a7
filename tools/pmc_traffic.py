#!/usr/bin/env python3
"""Per-launch HBM traffic of the solve kernel from a rocprofv3 counter pass.

Collect in its own pass (no --sys-trace / --runtime-trace with --pmc):

  rocprofv3 --pmc FETCH_SIZE --kernel-include-regex wave_kernel --output-format csv \\
      -d gpurun_out/pmc/fetch -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu
  rocprofv3 --pmc WRITE_SIZE ... -d gpurun_out/pmc/write ...   (FETCH_SIZE and WRITE_SIZE do not
                                                               fit one pass on gfx950's TCC)
  python3 tools/pmc_traffic.py gpurun_out/pmc --key N10_B4096_trot

Corrections per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads, so it is
doubled.  Access widths other than 16 B/lane are uncalibrated there: the result is an estimate
(the JSON records both the raw and the corrected numbers).
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parse(d, kernel_substr):
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {d}")
    per = defaultdict(dict)  # dispatch id -> counter -> value
    names = {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                kname = row.get("Kernel_Name", "")
                if kernel_substr not in kname:
                    continue
                did = (fn, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                per[did][row["Counter_Name"]] = float(row["Counter_Value"])
                names[did] = kname
    return per, names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--key", default="N10_B4096_trot")
    ap.add_argument("--kernel", default="scale_kernel,wave_kernel",
                    help="comma-separated kernel-name substrings; per-launch means are summed (one solve)")
    ap.add_argument("--parts", type=int, default=1,
                    help="launches of each kernel per solve (the wave path's batch split): the per-dispatch "
                         "means are multiplied by it, so the entry is per solve")
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    kernels = [k for k in a.kernel.split(",") if k]
    fetch_kib = write_kib = 0.0
    knames, ndisp = [], []
    for kname in kernels:
        per, names = parse(a.dir, kname)

        def mean_of(counter):
            vals = [v[counter] for v in per.values() if counter in v]
            if not vals:
                print(f"no dispatch of {kname} with {counter}", file=sys.stderr)
                sys.exit(1)
            vals = vals[1:] if len(vals) > 1 else vals  # drop the first (cold) dispatch
            return sum(vals) / len(vals), len(vals)

        f_kib, nf = mean_of("FETCH_SIZE")
        w_kib, nw = mean_of("WRITE_SIZE")
        fetch_kib += f_kib
        write_kib += w_kib
        knames.append(sorted(set(names.values()))[0])
        ndisp.append(min(nf, nw))
    fetch_b = fetch_kib * 1024.0 * 2.0 * a.parts  # gfx950: FETCH_SIZE counts half of the bytes
    write_b = write_kib * 1024.0 * a.parts
    entry = {
        "kernel": " + ".join(knames),
        "dispatches": min(ndisp),
        "fetch_size_kib_raw_per_dispatch": fetch_kib,
        "write_size_kib_raw_per_dispatch": write_kib,
        "fetch_bytes_corrected": fetch_b,
        "write_bytes": write_b,
        "hbm_bytes_per_launch": fetch_b + write_b,
        "parts": a.parts,
        "per": "one solve call (the per-dispatch means of each kernel times `parts`)",
        "correction": "FETCH_SIZE x2 (gfx950 half-count of wide reads), KiB -> B; other widths uncalibrated",
    }
    data = {}
    if os.path.exists(a.out):
        with open(a.out) as f:
            data = json.load(f)
    data[a.key] = entry
    with open(a.out, "w") as f:
        json.dump(data, f, indent=1)
    print(json.dumps({a.key: entry}, indent=1))


if __name__ == "__main__":
    main()

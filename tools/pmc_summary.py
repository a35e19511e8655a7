"""Per-dispatch means of rocprofv3 --pmc csv files: python tools/pmc_summary.py DIR..."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    for f in sorted(glob.glob(d + "/**/pmc_counter_collection.csv", recursive=True)):
        rows = list(csv.DictReader(open(f)))
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in rows:
            per[(r["Kernel_Name"][:40], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        agg = collections.defaultdict(list)
        for (k, _), cs in per.items():
            for c, v in cs.items():
                agg[(k, c)].append(v)
        print(f)
        for (k, c), vs in sorted(agg.items()):
            print("  %-40s %-24s %.4g" % (k, c, sum(vs) / len(vs)))

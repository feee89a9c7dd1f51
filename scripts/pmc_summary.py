"""Summarise rocprofv3 --pmc counter CSVs: per-dispatch sums for kernels whose
name contains a pattern (last matching dispatch).  usage: pmc_summary.py DIR PATTERN"""
import collections
import csv
import glob
import sys

d, pat = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    if agg:
        did = list(agg)[-1]
        print(f.split("/")[-2], did, {k: round(v) for k, v in sorted(agg[did].items())})

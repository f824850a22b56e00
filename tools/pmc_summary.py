"""Median per-dispatch counter values of the coupling kernel from gpu_pmc.sh output."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "k_valu"
out = {}
for p in sorted(glob.glob(root + "/p*/run_counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(p)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        v = sorted(v[len(v) // 4:])
        out[k] = v[len(v) // 2]
for k, v in out.items():
    print("%-28s %14.6g" % (k, v))

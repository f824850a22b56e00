"""HBM traffic per launch of the bench kernel from rocprofv3 PMC passes
(tools/gpu_pmc.sh FETCH_SIZE / WRITE_SIZE), corrected per
MI355X_MICROARCH.md section HBM: on gfx950 FETCH_SIZE reports half the bytes of
a wide coalesced streaming read, so read bytes = 2 x FETCH_SIZE (KiB);
WRITE_SIZE reads exactly for 16-B-per-lane streaming stores.
usage: pmc_traffic.py <pmc dir> <out json> <workload> <B> [kernel substring]"""
import collections
import csv
import glob
import json
import sys

root, out, workload, B = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
pat = sys.argv[5] if len(sys.argv) > 5 else "k_valu"
vals = collections.defaultdict(list)
name = None
for p in sorted(glob.glob(root + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(p)):
        if pat in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            name = r["Kernel_Name"]


def med(v):
    v = sorted(v[len(v) // 4:])  # drop warm-up dispatches
    return v[len(v) // 2]


fetch, write = med(vals["FETCH_SIZE"]), med(vals["WRITE_SIZE"])
res = {
    "workload": workload, "B": B, "kernel": name,
    "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write,
    "read_bytes": 2 * fetch * 1024, "write_bytes": write * 1024,
    "traffic_bytes_per_launch": (2 * fetch + write) * 1024,
    "correction": "read = 2 x FETCH_SIZE (gfx950 streaming-read undercount), write = WRITE_SIZE",
    "dispatches": len(vals["FETCH_SIZE"]),
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))

"""Per-kernel statistics of a rocprofv3 --kernel-trace run over its LAST
dispatches only: tools/prof_target.py settles the clock for --settle-s first
(as bench.py does), and those settle launches must not enter the averages
(round 5's traces were taken cold, so a kernel's average could exceed the
bench's whole step).  usage:
  trace_stats.py <kernel_trace.csv> <last_n_calls> [out.csv|-] [first kernel of a call]
For each kernel name: the number of its dispatches among the last
last_n_calls * (dispatches per call) of the trace, their mean / median /
min / max duration (ns), and the mean start-to-start spacing of the kernel
that occurs first in a call (the per-call wall on the device timeline)."""
import csv
import statistics
import sys


def main():
    path, last = sys.argv[1], int(sys.argv[2])
    out = sys.argv[3] if len(sys.argv) > 3 and sys.argv[3] != "-" else None
    # optional: a substring of the name of the kernel that starts each call
    # (a cfg4 training step is 39 dispatches whose tail repeats itself)
    first_kernel = sys.argv[4] if len(sys.argv) > 4 else None
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    # dispatches per call: the trailing period of the kernel-name sequence
    per = 1
    for p in range(1, 65):
        reps = 4 if p <= 8 else 2  # a cfg4 training step is 39 dispatches
        tail = names[-reps * p:]
        if len(tail) == reps * p and all(tail[i] == tail[i % p] for i in range(len(tail))):
            per = p
            break
    sel = rows[-last * per:]
    if first_kernel:
        starts = [i for i, r in enumerate(rows) if first_kernel in r["Kernel_Name"]]
        sel = rows[starts[-last]:]
        per = round(len(sel) / last)
    by = {}
    for r in sel:
        by.setdefault(r["Kernel_Name"], []).append(
            (int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    first = sel[0]["Kernel_Name"]
    starts = [s for s, _ in by[first]]
    spacing = (starts[-1] - starts[0]) / (len(starts) - 1) if len(starts) > 1 else None
    def short(k):  # the kernel's name with its template arguments, no parameter list
        k = k.replace("(anonymous namespace)::", "")
        depth = 0
        for i, c in enumerate(k):
            depth += c == "<"
            depth -= c == ">"
            if c == "(" and depth == 0 and i > 0:
                return k[:i].replace("void ", "")
        return k
    table = []
    for k, v in by.items():
        d = [e - s for s, e in v]
        table.append({"Name": short(k), "Calls": len(d), "AverageNs": round(statistics.mean(d), 1),
                      "MedianNs": statistics.median(d), "MinNs": min(d), "MaxNs": max(d),
                      "DispatchesPerCall": per,
                      "CallSpacingNs": round(spacing, 1) if k == first and spacing else ""})
    table.sort(key=lambda t: -t["AverageNs"] * t["Calls"])
    w = csv.DictWriter(open(out, "w") if out else sys.stdout, fieldnames=list(table[0]))
    w.writeheader()
    w.writerows(table)


if __name__ == "__main__":
    main()

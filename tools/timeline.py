"""Print the GPU timeline of the last evaluations in a rocprofv3 kernel trace.

usage: python tools/timeline.py <kernel_trace.csv> [anchor_kernel] [n_evals]

Each evaluation is the run of dispatches that ends with `anchor_kernel`
(default k_emit); for the last n_evals of them it prints every dispatch with
its grid size, duration and the idle gap before it, so the per-evaluation
device cost of the drop-in loop can be split into kernels and dispatch gaps.
"""
import csv
import sys


def main():
    path = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "k_emit"
    n_ev = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    if len(ends) < n_ev + 1:
        print("not enough evaluations", len(ends))
        return
    for k in range(len(ends) - n_ev, len(ends)):
        lo, hi = ends[k - 1] + 1, ends[k]
        t0 = int(rows[lo - 1]["End_Timestamp"])
        print("--- evaluation", k, "dispatches", hi - lo + 1)
        prev = t0
        busy = 0
        for r in rows[lo:hi + 1]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            name = r["Kernel_Name"].split("(")[0]
            grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
            print("%-28s grid %8s  gap %8.2f us  dur %8.2f us" % (name[:28], grid, (s - prev) / 1e3, (e - s) / 1e3))
            busy += e - s
            prev = e
        print("span %.2f us  busy %.2f us" % ((prev - t0) / 1e3, busy / 1e3))


if __name__ == "__main__":
    main()

"""Per-dispatch and per-unit averages of rocprofv3 --pmc counters for one
kernel, over any number of pass directories (measurement aid).

usage: pmc_summary.py <kernel-substring> <units-per-dispatch> <pass dir>...
Prints JSON: for every counter the mean value per dispatch of the kernel and
per unit (e.g. per placement of a count loop)."""
import csv
import glob
import json
import os
import sys


def main():
    key, units = sys.argv[1], float(sys.argv[2])
    per = {}
    kernels = set()
    for d in sys.argv[3:]:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                if key not in r["Kernel_Name"]:
                    continue
                kernels.add(r["Kernel_Name"])
                per.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
                per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    out = {"kernel": sorted(kernels), "units_per_dispatch": units, "counters": {}}
    for name, d in sorted(per.items()):
        vals = list(d.values())
        m = sum(vals) / len(vals)
        out["counters"][name] = {"dispatches": len(vals), "per_dispatch": m, "per_unit": m / units}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

"""Summarise the FETCH_SIZE / WRITE_SIZE calibration passes over
tools/fetch_calib (known unique bytes per pattern): counted bytes / unique bytes
for every pattern, averaged over its dispatches after the first (warm
Infinity Cache, as in the headline loop).

usage: fetch_calib.py <fetch.csv> <write.csv> <fetch_calib stdout> [<out.json>]
"""
import csv
import json
import sys


def counters(path, name):
    per = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != name:
            continue
        k = r["Kernel_Name"]
        per.setdefault(k, {}).setdefault(r["Dispatch_Id"], 0.0)
        per[k][r["Dispatch_Id"]] += float(r["Counter_Value"]) * 1024.0
    return per


def main():
    fetch_csv, write_csv, info = sys.argv[1:4]
    meta = json.loads(open(info).read().strip().splitlines()[-1])
    f = counters(fetch_csv, "FETCH_SIZE")
    w = counters(write_csv, "WRITE_SIZE")
    out = {"rows": meta["rows"], "patterns": {}}
    for pat, (ur, uw) in meta["unique"].items():
        def pick(per):
            for k, d in per.items():
                if k.split("(")[0].replace("void ", "").strip().endswith(pat):
                    v = [d[i] for i in sorted(d, key=int)]
                    warm = v[1:] or v
                    return sum(warm) / len(warm)
            return None
        fb, wb = pick(f), pick(w)
        out["patterns"][pat] = {"unique_read": ur, "unique_write": uw, "fetch_size_bytes": fb,
                                "write_size_bytes": wb,
                                "fetch_over_unique": (fb / ur) if (fb is not None and ur) else None,
                                "write_over_unique": (wb / uw) if (wb is not None and uw) else None}
    s = json.dumps(out, indent=1)
    if len(sys.argv) > 4:
        open(sys.argv[4], "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()

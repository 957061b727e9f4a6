"""Per-launch HBM traffic from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE
in separate runs, MI355X_MICROARCH.md: both in KiB; gfx950 FETCH_SIZE counts
half of the bytes of wide coalesced streaming reads, so it is doubled).

usage: pmc_traffic.py <fetch.csv> <write.csv> <kernel-substring> <nodes> <bytes_per_node> [<out.json>] [<fetch factor>]
The fetch factor (default 2.0, the guide's 16 B/lane streaming correction)
converts FETCH_SIZE into bytes; profiles/r04/fetch_calib_*.json hold the
factors measured on known-byte gathers (64-B record gathers count ~0.93 of
their bytes: factor ~1.08).
Averages over the dispatches of the kernel whose name contains the substring,
keeping only the largest grid (the batched launches the bench times; a run
also holds single-evaluation launches of the same kernel).
"""
import csv
import json
import sys


def per_dispatch(path, counter, key):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter and key in r["Kernel_Name"]]
    if not rows:
        return []
    grid = max(int(r["Grid_Size"]) for r in rows)
    vals = {}
    for r in rows:
        if int(r["Grid_Size"]) != grid:
            continue
        vals.setdefault(r["Dispatch_Id"], 0.0)
        vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return list(vals.values())


def main():
    fetch_csv, write_csv, key, nodes, bpn = sys.argv[1:6]
    factor = float(sys.argv[7]) if len(sys.argv) > 7 else 2.0
    f = per_dispatch(fetch_csv, "FETCH_SIZE", key)
    w = per_dispatch(write_csv, "WRITE_SIZE", key)
    assert f and w, "kernel %r not found in the PMC passes" % key
    fetch_b = sum(f) / len(f) * 1024.0 * factor
    write_b = sum(w) / len(w) * 1024.0
    algo = int(nodes) * int(bpn)
    out = {"kernel": key, "nodes": int(nodes), "bytes_per_node": int(bpn), "dispatches": len(f),
           "fetch_bytes_per_launch": fetch_b, "write_bytes_per_launch": write_b,
           "bytes_per_launch": fetch_b + write_b, "algorithmic_bytes_per_launch": algo,
           "traffic_over_algorithmic": (fetch_b + write_b) / algo,
           "fetch_counted_bytes_per_launch": sum(f) / len(f) * 1024.0, "fetch_factor": factor,
           "correction": "FETCH_SIZE KiB x 1024 x %.3f (calibrated on known-byte accesses of the kernel's "
                         "pattern, tools/fetch_calib.hip), WRITE_SIZE KiB x 1024" % factor}
    s = json.dumps(out, indent=1)
    if len(sys.argv) > 6 and sys.argv[6] != "-":
        with open(sys.argv[6], "w") as fh:
            fh.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()

"""Per-launch HBM traffic of the engine's kernels from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

Corrections per MI355X_MICROARCH.md §HBM: counter values are in KB; on gfx950 FETCH_SIZE reports half the
bytes of a wide coalesced (16 B/lane) streaming read, so it is doubled; WRITE_SIZE is taken as is.  Writes
a JSON summary (bytes per launch, averaged over the launches of each kernel) that bench.py attaches as
roofline.traffic.

usage: python scripts/pmc_traffic.py gpurun_out/pmc_fetch/run_counter_collection.csv \
                                     gpurun_out/pmc_write/run_counter_collection.csv  out.json
"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    """Group dispatches by kernel and grid; launches of one kernel+grid whose duration differs by more than
    2x (e.g. the SYRK main wave and its split-K tail, same grid size) are kept apart as '/long', '/short'."""
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    groups = defaultdict(list)
    for r in rows:
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        groups[r["Kernel_Name"].split("(")[0] + "@grid" + r["Grid_Size"]].append(
            (dur, float(r["Counter_Value"]) * 1024.0))  # KB -> B
    acc = defaultdict(list)
    for name, v in groups.items():
        dmax = max(d for d, _ in v)
        split = any(d < dmax / 2 for d, _ in v)
        for d, b in v:
            acc[name + (("/long" if d >= dmax / 2 else "/short") if split else "")].append(b)
    return acc


def main(fetch_csv, write_csv, out):
    f = per_kernel(fetch_csv, "FETCH_SIZE")
    w = per_kernel(write_csv, "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        fa = f.get(k, [])
        wa = w.get(k, [])
        fb = 2.0 * sum(fa) / len(fa) if fa else None
        wb = sum(wa) / len(wa) if wa else None
        res[k] = {"launches": max(len(fa), len(wa)), "fetch_bytes_per_launch": fb,
                  "write_bytes_per_launch": wb,
                  "hbm_bytes_per_launch": (fb or 0.0) + (wb or 0.0)}
    doc = {"source": [fetch_csv, write_csv],
           "correction": "FETCH_SIZE x2 (gfx950 wide-read tally), WRITE_SIZE x1; KB -> bytes",
           "kernels": res}
    json.dump(doc, open(out, "w"), indent=1)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"])[:12]:
        print(f"{k:52s} n={v['launches']:5d} fetch={v['fetch_bytes_per_launch'] or 0:14.4g} "
              f"write={v['write_bytes_per_launch'] or 0:14.4g}")


if __name__ == "__main__":
    main(*sys.argv[1:4])

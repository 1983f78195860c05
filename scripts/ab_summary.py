"""Summarise same-box bench A/B runs: value and phase means per variant (files <dir>/ab_<variant><i>.json)."""
import glob
import json
import os
import re
import sys
from collections import defaultdict


def main(d):
    rows = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "ab_*.json"))):
        m = re.match(r"ab_(.*?)(\d+)\.json$", os.path.basename(f))
        if not m:
            continue
        for line in open(f):
            if line.startswith("{"):
                rows[m.group(1)].append(json.loads(line))
    for v, rs in rows.items():
        val = [r["value"] for r in rs]
        ph = defaultdict(list)
        for r in rs:
            for k, x in r.get("phases_ms", {}).items():
                ph[k].append(x)
        print(f"{v:8s} n={len(rs)} value {' '.join(f'{x:6.1f}' for x in val)}  mean {sum(val) / len(val):6.1f} | " +
              " ".join(f"{k[:8]} {sum(x) / len(x):.3f}" for k, x in ph.items()) +
              f" | kkt/s {sum(r.get('kkt_factor_solve_per_s', 0) for r in rs) / len(rs):.0f}")


if __name__ == "__main__":
    main(sys.argv[1])

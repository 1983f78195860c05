"""Recompute the bench's rooflines from a rocprofv3 kernel trace of `bench.py --steps K --warmup W` (C3).

Each Newton step assembles H once (k_syrk_direct main wave + split-K tail + k_syrk_reduce, launched at the end of the
previous step, or at the start of the first one) and factors it once or more (k_chol_dataflow; a second launch when
the Ruiz lookahead fell short or the factor was regularized).  Assembly i belongs to step i; the factorizations between
assembly i's first launch and assembly i + 1's first launch belong to step i.  Steps W .. W + K - 1 are the timed ones.

Prints (and with --json writes) per-assembly and per-step Cholesky kernel time (sums of kernel durations) over the
timed steps and the fractions of the FP64 MFMA peak: assembly m n (n + 1) flop, Cholesky n^3/3 + n^2/2 + n/6, combined.

  python scripts/trace_roofline.py <run_kernel_trace.csv> --warmup 5 --steps 20 [--n 4096 --m 8192] [--json out]
"""
import argparse
import csv
import json
import sys

PEAK = 78.6e12


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    return rows


def analyse(rows, warmup, steps, n, m):
    is_syrk = lambda k: "k_syrk_direct" in k or "k_syrk_reduce" in k  # noqa: E731
    # assemblies: maximal runs of SYRK launches (nothing else on the trace between them but s2 work is interleaved,
    # so group by "a k_syrk_direct launch that follows a k_syrk_reduce / non-SYRK main-stream kernel")
    asm = []  # [start, [durations]]
    cur = None
    for s, e, k in rows:
        if "k_syrk_direct" in k:
            if cur is None or cur["closed"]:
                cur = {"start": s, "dur": [], "closed": False}
                asm.append(cur)
            cur["dur"].append(e - s)
        elif "k_syrk_reduce" in k and cur is not None:
            cur["dur"].append(e - s)
            cur["closed"] = True
    chol = [(s, e - s) for s, e, k in rows if "k_chol_dataflow" in k]
    if len(asm) < warmup + steps:
        raise SystemExit(f"trace holds {len(asm)} assemblies, fewer than warmup + steps = {warmup + steps}")
    a_ms, c_ms, c_n = [], [], []
    for i in range(warmup, warmup + steps):
        a_ms.append(sum(asm[i]["dur"]) * 1e-6)
        lo = asm[i]["start"]
        hi = asm[i + 1]["start"] if i + 1 < len(asm) else float("inf")
        cs = [d for s, d in chol if lo <= s < hi]
        c_ms.append(sum(cs) * 1e-6)
        c_n.append(len(cs))
    fa = m * n * (n + 1.0)
    fc = n ** 3 / 3.0 + n * n / 2.0 + n / 6.0
    am, cm = sum(a_ms) / steps, sum(c_ms) / steps
    out = {
        "assemblies_in_trace": len(asm), "timed_steps": steps, "warmup": warmup,
        "assembly_ms": am, "assembly_frac": fa / (am * 1e-3) / PEAK,
        "cholesky_ms": cm, "cholesky_launches": sum(c_n), "cholesky_frac": fc / (cm * 1e-3) / PEAK,
        "combined_frac": (fa + fc) / ((am + cm) * 1e-3) / PEAK,
        "assembly_ms_per_step": a_ms, "cholesky_ms_per_step": c_ms,
    }
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    out = analyse(load(a.trace), a.warmup, a.steps, a.n, a.m)
    out["source"] = a.trace
    print(f"assembly {out['assembly_ms']:.4f} ms/step (frac {out['assembly_frac']:.4f}), cholesky "
          f"{out['cholesky_ms']:.4f} ms/step over {out['cholesky_launches']} launches (frac {out['cholesky_frac']:.4f}), "
          f"combined frac {out['combined_frac']:.4f}")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())

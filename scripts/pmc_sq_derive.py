"""Derive the Cholesky's MFMA utilisation from two rocprofv3 SQ counter passes (scripts/pmc_sq.sh with the regex
"k_chol_dataflow|k_syrk_direct"): per-launch means of the counters of the factorization (launches longer than 100 us;
the short ones are attempts voided by an open Ruiz lookahead) and of the assembly SYRK's main wave (launches longer
than 1 ms), then
  * the MFMA work of the factorization against the algorithmic n^3/3 (SQ_INSTS_VALU_MFMA_MOPS_F64 x 512 flop);
  * its MFMA-busy rate (SQ_VALU_MFMA_BUSY_CYCLES per us) against the SYRK main wave's, and scaled by the main
    wave's measured fraction of the clock-limited peak (0.93) against that peak;
  * the fraction of wave cycles spent waiting (SQ_WAIT_ANY / SQ_WAVE_CYCLES) and the LDS bank-conflict cycles.

  python scripts/pmc_sq_derive.py pass1.csv pass2.csv out.json [n]
"""
import csv
import json
import sys
from collections import defaultdict


def means(paths, name, min_us):
    acc = defaultdict(list)
    for path in paths:
        for r in csv.DictReader(open(path)):
            if name not in r["Kernel_Name"]:
                continue
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
            if dur < min_us:
                continue
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
            acc["_dur_us"].append(dur)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main(p1, p2, out, n=4096):
    ch = means([p1, p2], "k_chol_dataflow", 100.0)
    sy = means([p1, p2], "k_syrk_direct", 1000.0)
    alg = n ** 3 / 3.0
    d = {}
    if "SQ_INSTS_VALU_MFMA_MOPS_F64" in ch:
        d["mfma_flops (SQ_INSTS_VALU_MFMA_MOPS_F64 x 512)"] = ch["SQ_INSTS_VALU_MFMA_MOPS_F64"] * 512
        d["algorithmic_flops (n^3/3)"] = alg
        d["mfma_work_over_algorithmic"] = ch["SQ_INSTS_VALU_MFMA_MOPS_F64"] * 512 / alg
    if "SQ_VALU_MFMA_BUSY_CYCLES" in ch and "SQ_VALU_MFMA_BUSY_CYCLES" in sy:
        rate = (ch["SQ_VALU_MFMA_BUSY_CYCLES"] / ch["_dur_us"]) / (sy["SQ_VALU_MFMA_BUSY_CYCLES"] / sy["_dur_us"])
        d["mfma_busy_rate_vs_syrk_main_wave"] = rate
        d["mfma_busy_vs_clock_limited_peak (x 0.93, the SYRK main wave's measured fraction)"] = rate * 0.93
    if "SQ_WAIT_ANY" in ch and "SQ_WAVE_CYCLES" in ch:
        d["wave_wait_fraction (SQ_WAIT_ANY / SQ_WAVE_CYCLES)"] = ch["SQ_WAIT_ANY"] / ch["SQ_WAVE_CYCLES"]
    if "SQ_LDS_BANK_CONFLICT" in ch and "SQ_WAVE_CYCLES" in ch:
        d["lds_bank_conflict_cycles_over_wave_cycles"] = ch["SQ_LDS_BANK_CONFLICT"] / ch["SQ_WAVE_CYCLES"]
    doc = {"source": f"rocprofv3 --pmc passes {p1}, {p2} (scripts/pmc_sq.sh 'k_chol_dataflow|k_syrk_direct')",
           "kernel": "cvxg::k_chol_dataflow (C3 Cholesky + fused forward solve)",
           "counters": ch, "syrk_main_wave_counters": sy, "derived": d}
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], *(int(a) for a in sys.argv[4:5]))

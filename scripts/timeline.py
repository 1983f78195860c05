"""Print the kernel timeline of one Newton step from a rocprofv3 kernel trace (csv), with the GPU idle gaps.

  python scripts/timeline.py gpurun_out/prof/run_kernel_trace.csv [step_index]

A step starts at a `k_syrk_direct` launch on the main queue; the step index counts them from the end of the trace
(default: the third-to-last step, clear of the run's tail).
"""
import csv
import sys


def main():
    path = sys.argv[1]
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0],
                         r.get("Queue_Id", "")))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "k_syrk_direct" in r[2] and "short" not in r[2]]
    # one assembly = two k_syrk_direct launches (main wave + tail); a step begins at the first of each pair
    firsts = [starts[i] for i in range(0, len(starts), 2)]
    a, b = firsts[-back - 1], firsts[-back]
    t0 = rows[a][0]
    busy_end = t0
    idle = 0
    for s, e, name, q in rows[a:b]:
        gap = s - busy_end
        if gap > 0:
            idle += gap
        print(f"{(s - t0) / 1e3:9.1f} us  {((e - s) / 1e3):8.1f} us  gap {max(gap, 0) / 1e3:6.1f}  q{q:>3}  {name[:70]}")
        busy_end = max(busy_end, e)
    total = rows[b][0] - t0
    print(f"step {total / 1e3:.1f} us, GPU idle {idle / 1e3:.1f} us")


if __name__ == "__main__":
    main()

#!/bin/bash
# Kernel statistics of one complete C3 barrier solve (bench.py --workload C3FULL) under rocprofv3 --kernel-trace
# --stats: where the late path's time goes (the speculative regularized pairs, the certified line search's fresh
# trials).  Output under gpurun_out/$TAG/c3full_prof.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
TAG=${TAG:-c3fullprof}
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/c3full_prof" -o run -- python3 "$R/bench.py" --workload C3FULL > "$R/$O/c3full_prof.log" 2>&1
rc=$?
cd "$R"
# the full trace of a 3 124-step solve is far above gpurun_out's 64 MiB: keep the statistics and a per-step digest
python3 - "$O/c3full_prof/run_kernel_trace.csv" > "$O/c3full_digest.txt" 2>&1 <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float); cnt = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0]
    tot[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    cnt[k] += 1
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:30]:
    print(f"{v:10.1f} ms  {cnt[k]:7d} launches  {k}")
PY
rm -f "$O/c3full_prof/run_kernel_trace.csv"
echo "[$TAG] c3full_prof exit=$rc" | tee -a "$O/status.log"
exit $rc

#!/bin/bash
# Side workloads of bench.py (C2, C3B with and without the sparse-row split, C4, PD, C3EQ with p = 8 / 64, the
# direct KL solve C4P), one line each into
# gpurun_out/wl_<name>.json.  Each run has its own time limit; a fault or timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # $1 = label, rest = env + args
  local label=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/wl_$label.log 2>&1
  local rc=$?
  tail -1 gpurun_out/wl_$label.log > gpurun_out/wl_$label.json
  echo "[bench_workloads] $label rc=$rc $(python -c "import json; d=json.load(open('gpurun_out/wl_$label.json')); print(round(d['value'],1), 'steps/s', {k: round(v,3) for k, v in d['phases_ms'].items()})" 2>/dev/null)"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run C2 python bench.py --workload C2 --no-cpu-baseline --steps 50 --warmup 5
run C3B python bench.py --workload C3B --no-cpu-baseline --steps 10 --warmup 2
run C3B_dense python bench.py --workload C3B --no-cpu-baseline --steps 10 --warmup 2 --opt sparse_rows=0
run C4 python bench.py --workload C4 --no-cpu-baseline --steps 50 --warmup 5
run C2PD python bench.py --workload C2PD --no-cpu-baseline --steps 50
run C3PD python bench.py --workload C3PD --no-cpu-baseline --steps 20
run C3EQ8 python bench.py --workload C3EQ --p 8 --no-cpu-baseline --steps 10 --warmup 2
run C3EQ64 python bench.py --workload C3EQ --p 64 --no-cpu-baseline --steps 10 --warmup 2
run C4P python bench.py --workload C4P --no-cpu-baseline --steps 30 --warmup 3

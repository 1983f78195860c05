#!/bin/bash
# Round-5 side workloads (scripts/bench_workloads.sh -> gpurun_out/wl_*.json) and C3X2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/bench_workloads.sh || exit $?
timeout -k 10 300 python bench.py --workload C3X2 --steps 30 --warmup 3 > gpurun_out/wl_C3X2.log 2>&1 || exit $?
tail -1 gpurun_out/wl_C3X2.log > gpurun_out/wl_C3X2.json

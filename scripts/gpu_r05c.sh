#!/bin/bash
# Round-5 session C: late C3 states for the oracle fixture, the GPU suite, bench, a kernel trace of the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05c; mkdir -p $O
fault() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python -u scripts/c3_late_states.py > $O/c3_late_states.log 2>&1; rc=$?; echo "late $rc"; fault $rc && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest $rc"; fault $rc && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.log 2>&1; rc=$?; echo "bench $rc"; fault $rc && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/$O/prof.log" 2>&1; rc=$?; echo "prof $rc"
exit 0

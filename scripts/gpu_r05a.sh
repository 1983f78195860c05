#!/bin/bash
# Round-5 session A: smoke, the KL direct-solve diagnostic (new and round-4 trial kernel), the GPU suite, a bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05a
O=gpurun_out/r05a
fault() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke $rc"; fault $rc && exit $rc
timeout -k 10 400 python -u scripts/kl_direct_diag.py 2048 > $O/kl_new.log 2>&1; rc=$?; echo "kl_new $rc"; fault $rc && exit $rc
CVXG_LIB=$PWD/exp_build/libcvxg_oldklp.so timeout -k 10 400 python -u scripts/kl_direct_diag.py 2048 > $O/kl_old.log 2>&1; rc=$?; echo "kl_old $rc"; fault $rc && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest $rc"; fault $rc && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.log 2>&1; rc=$?; echo "bench $rc"
exit 0

#!/bin/bash
# A/B of two library builds on one box (cvx_amd/libcvxg_base.so vs cvx_amd/libcvxg.so): a chain trace of each, then
# ROUNDS alternating bench runs.  Output under gpurun_out/$TAG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
TAG=${TAG:-ab}
O=gpurun_out/$TAG
mkdir -p $O
chk() { local rc=$1; echo "[$TAG] $2 exit=$rc" | tee -a $O/status.log; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread -k "$PYTEST_K" > $O/pytest_gpu.log 2>&1
  rc=$?; echo "[$TAG] tests exit=$rc" | tee -a $O/status.log; if [ "$rc" -ge 124 ]; then exit $rc; fi
fi
CVXG_LIB=$R/cvx_amd/libcvxg_base.so CVXG_DF_TRACE=$R/$O/df_base.bin timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/trace_base.log 2>&1; chk $? trace_base
CVXG_DF_TRACE=$R/$O/df_new.bin timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/trace_new.log 2>&1; chk $? trace_new
for r in $(seq 1 ${ROUNDS:-2}); do
  CVXG_LIB=$R/cvx_amd/libcvxg_base.so timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/ab_base$r.log 2>&1; chk $? base$r
  timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/ab_new$r.log 2>&1; chk $? new$r
done
echo "[$TAG] done" | tee -a $O/status.log

#!/bin/bash
# A/B of two library builds on one box: cvx_amd/libcvxg_base.so (baseline) vs cvx_amd/libcvxg.so, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  CVXG_LIB=$PWD/cvx_amd/libcvxg_base.so timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/ab_base$r.log 2>&1 || exit $?
  timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/ab_new$r.log 2>&1 || exit $?
done

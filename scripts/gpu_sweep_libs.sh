#!/bin/bash
# Bench every library build in cvx_amd/vlibs/ on one box, two interleaved rounds (CVXG_LIB), C3 Cholesky phase.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/vl
for r in 1 2; do
  for f in cvx_amd/vlibs/*.so; do
    n=$(basename $f .so)
    CVXG_LIB=$PWD/$f timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/vl/${n}_$r.log 2>&1 || exit $?
  done
done

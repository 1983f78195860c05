#!/bin/bash
# A/B/n of several library builds on one box (cvx_amd/libcvxg_$v.so for v in $LIBS): a chain trace of each, then
# ROUNDS rounds of bench runs in rotation.  Output under gpurun_out/$TAG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
TAG=${TAG:-abn}
O=gpurun_out/$TAG
mkdir -p $O
chk() { local rc=$1; echo "[$TAG] $2 exit=$rc" | tee -a $O/status.log; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
for v in $LIBS; do
  CVXG_LIB=$R/cvx_amd/libcvxg_$v.so CVXG_DF_TRACE=$R/$O/df_$v.bin timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/trace_$v.log 2>&1; chk $? trace_$v
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $LIBS; do
    CVXG_LIB=$R/cvx_amd/libcvxg_$v.so timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/ab_$v$r.log 2>&1; chk $? $v$r
  done
done
echo "[$TAG] done" | tee -a $O/status.log

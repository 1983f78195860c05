#!/bin/bash
# Round-5 session R: what made the worker change fast.  default = abort word on its own cache line, no abort poll at
# the claim, df_wait3; sep = the same with the abort poll at the claim (CVXG_DF_ABORT_AT_CLAIM=1); il = default with the
# interleaved reciprocal in the DPP sweep (P64W_INTERLEAVE=1); base5 = the head before the worker change.
# POTRF microbench with / without the interleave, bitwise fingerprints of default / il / sep, chain tests, A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r05r; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
for v in dpp_true il; do timeout -k 10 120 ./microbench/potrf64w_bench_$v 400 > $O/p64_$v.log 2>&1; chk $? p64_$v; done
for v in - il sep; do
  lib=$R/cvx_amd/libcvxg.so; [ "$v" != "-" ] && lib=$R/cvx_amd/libcvxg_$v.so
  CVXG_LIB=$lib timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_${v/-/default}.txt 2>&1; chk $? fp_$v
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -k "chain_owned or speculative or batch" --timeout 200 --timeout-method thread > $O/pytest_sel.log 2>&1; chk $? seltests
TAG=r05r/ab VARIANTS="base5=base5 def=- sep=sep il=il" ROUNDS=3 bash scripts/gpu_abv.sh; chk $? abv
exit 0

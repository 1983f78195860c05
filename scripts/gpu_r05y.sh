#!/bin/bash
# Round-5 session Y: POTRF micro-changes on wave 0's path.  nomask (the default build now) = the DPP sweep loads the
# diagonal block without masking the entries above the diagonal; tu = nomask + T and U of each step with T in registers
# (P64W_TU_FUSED=1); head = before both.  POTRF microbench stamps, fingerprints, chain test on tu, A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r05y; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
for v in dpp_true tu; do timeout -k 10 120 ./microbench/potrf64w_bench_$v 400 > $O/p64_$v.log 2>&1; chk $? p64_$v; done
timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_nomask.txt 2>&1; chk $? fp_nomask
CVXG_LIB=$R/cvx_amd/libcvxg_tu.so timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_tu.txt 2>&1; chk $? fp_tu
CVXG_LIB=$R/cvx_amd/libcvxg_head.so timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_head.txt 2>&1; chk $? fp_head
CVXG_LIB=$R/cvx_amd/libcvxg_tu.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -k "chain_owned or batch or regularized_first or golden_baseline" --timeout 300 --timeout-method thread > $O/pytest_tu.log 2>&1; chk $? tests_tu
TAG=r05y/ab VARIANTS="head=head nomask=- tu=tu" ROUNDS=3 bash scripts/gpu_abv.sh; chk $? abv
exit 0

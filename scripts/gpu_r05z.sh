#!/bin/bash
# Round-5 session Z: the DPP sweep's bookkeeping off wave-uniform branches (the first bad pivot by one ballot after the
# sweep) and the diagonal block of S stored unmasked; POTRF microbench, fingerprints (must equal head's), chain and
# failure-path tests, A/B against head.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r05z; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
timeout -k 10 120 ./microbench/potrf64w_bench_dpp_true 400 > $O/p64_new.log 2>&1; chk $? p64
timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_new.txt 2>&1; chk $? fp_new
CVXG_LIB=$R/cvx_amd/libcvxg_head.so timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_head.txt 2>&1; chk $? fp_head
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -k "chain_owned or batch or regularized or golden_baseline or fail or indefinite or fallback" --timeout 300 --timeout-method thread > $O/pytest_sel.log 2>&1; chk $? seltests
TAG=r05z/ab VARIANTS="head=head new=-" ROUNDS=3 bash scripts/gpu_abv.sh; chk $? abv
exit 0

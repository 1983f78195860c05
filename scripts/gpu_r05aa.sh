#!/bin/bash
# Round-5 session AA: the chain reads its flag while the batch's MFMAs run, so the next L^-1 row-block's load goes out
# without a poll round trip after the batch; fingerprints, chain tests, A/B against head.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r05aa; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_new.txt 2>&1; chk $? fp_new
CVXG_LIB=$R/cvx_amd/libcvxg_head.so timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_head.txt 2>&1; chk $? fp_head
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -k "chain_owned or batch or regularized or golden_baseline" --timeout 300 --timeout-method thread > $O/pytest_sel.log 2>&1; chk $? seltests
TAG=r05aa/ab VARIANTS="head=head new=-" ROUNDS=3 bash scripts/gpu_abv.sh; chk $? abv
exit 0

#!/bin/bash
# Round-5 session T: wave 0 of the chain goes from its last slice straight into POTRF's first sweep (its only diagonal
# block is D_00; waves 1..3 store the other nine and count them into ps.cntD, no barrier).  Fingerprints new / head,
# chain + parity tests, A/B head vs new with chain traces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r05t; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_new.txt 2>&1; chk $? fp_new
CVXG_LIB=$R/cvx_amd/libcvxg_head.so timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_head.txt 2>&1; chk $? fp_head
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -k "chain_owned or golden_baseline or speculative or batch or lookahead or regularized_first" --timeout 300 --timeout-method thread > $O/pytest_sel.log 2>&1; chk $? seltests
TAG=r05t/ab VARIANTS="head=head new=-" ROUNDS=3 bash scripts/gpu_abv.sh; chk $? abv
exit 0

#!/bin/bash
# Round-5 session BB: tree = the DPP sweep's pivots kept and their minimum taken as a tree after the sweep, min diag(L)
# folded after T / U, the early-stop test's exact value formed only near the threshold (the default build now);
# nobatch = tree with every L^-1 row-block in its own slice (CVXG_DF_NOBATCH=1); head = the ballot commit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r05bb; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_tree.txt 2>&1; chk $? fp_tree
CVXG_LIB=$R/cvx_amd/libcvxg_nobatch.so timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_nobatch.txt 2>&1; chk $? fp_nobatch
CVXG_LIB=$R/cvx_amd/libcvxg_head.so timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_head.txt 2>&1; chk $? fp_head
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -k "chain_owned or batch or regularized or golden_baseline or fallback" --timeout 300 --timeout-method thread > $O/pytest_sel.log 2>&1; chk $? seltests
TAG=r05bb/ab VARIANTS="head=head tree=- nobatch=nobatch" ROUNDS=3 bash scripts/gpu_abv.sh; chk $? abv
exit 0

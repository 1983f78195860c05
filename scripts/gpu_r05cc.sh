#!/bin/bash
# Round-5 session CC: every L^-1 row-block in its own slice (CVXG_DF_NOBATCH=1) on the ballot head, against it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r05cc; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
CVXG_LIB=$R/cvx_amd/libcvxg_nobatch.so timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_nobatch.txt 2>&1; chk $? fp_nobatch
TAG=r05cc/ab VARIANTS="head=- nobatch=nobatch" ROUNDS=4 bash scripts/gpu_abv.sh; chk $? abv
exit 0

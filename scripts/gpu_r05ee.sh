#!/bin/bash
# Round-5 session EE: eight-panel update groups only on the tiles of the first block columns (CVXG_DF_GROUP8 = n: block
# columns j < n), where the middle of the factorization is worker-bound; the last blocks keep four-panel groups.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05ee; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
CVXG_DF_GROUP8=40 timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_g40.txt 2>&1; chk $? fp_g40
TAG=r05ee/ab VARIANTS="def=- g24=-,CVXG_DF_GROUP8=24 g32=-,CVXG_DF_GROUP8=32 g40=-,CVXG_DF_GROUP8=40 g48=-,CVXG_DF_GROUP8=48" ROUNDS=2 bash scripts/gpu_abv.sh; chk $? abv
exit 0

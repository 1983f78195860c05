#!/bin/bash
# Round-5 session DD: eight-panel update groups (CVXG_DF_GROUP8=1) re-measured under the round-5 schedule estimates.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05dd; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
CVXG_DF_GROUP8=1 timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_g8.txt 2>&1; chk $? fp_g8
TAG=r05dd/ab VARIANTS="def=- g8=-,CVXG_DF_GROUP8=1" ROUNDS=3 bash scripts/gpu_abv.sh; chk $? abv
exit 0

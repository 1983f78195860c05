#!/bin/bash
# Round-5 session FF: eight-panel groups on the first block columns only, around n = 24 (CVXG_DF_GROUP8 = n).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05ff; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
TAG=r05ff/ab VARIANTS="def=- g16=-,CVXG_DF_GROUP8=16 g20=-,CVXG_DF_GROUP8=20 g24=-,CVXG_DF_GROUP8=24 g28=-,CVXG_DF_GROUP8=28" ROUNDS=3 bash scripts/gpu_abv.sh; chk $? abv
exit 0

#!/bin/bash
# Round-5 session B: the KL direct solves over sizes and direction-bit variants, trial kernel of this round vs round 4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05b; mkdir -p $O
fault() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
NS=1024,1536,2048,2560,3072,4096
timeout -k 10 500 python -u scripts/kl_direct_diag.py $NS kl_1 > $O/kl_new.log 2>&1; rc=$?; echo "kl_new $rc"; fault $rc && exit $rc
CVXG_LIB=$PWD/exp_build/libcvxg_oldklp.so timeout -k 10 500 python -u scripts/kl_direct_diag.py $NS kl_1 > $O/kl_old.log 2>&1; rc=$?; echo "kl_old $rc"
exit 0

#!/bin/bash
# Round-5 session P: worker start-up round trips and update grouping.  polls = dependency polls loaded together
# (df_wait3), claim at the loop top; drain = the same plus the next claim taken during the previous task's drain (the
# default build); g8 = drain with eight-panel update groups (CVXG_DF_GROUP8=1).  Chain / parity tests on drain and on
# g8, then the A/B with a chain trace of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05p; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
K="chain_owned or golden_baseline or speculative or batch or lookahead"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -k "$K" --timeout 200 --timeout-method thread > $O/pytest_sel.log 2>&1; chk $? seltests
CVXG_DF_GROUP8=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -k "$K" --timeout 200 --timeout-method thread > $O/pytest_sel_g8.log 2>&1; chk $? seltests_g8
TAG=r05p/ab VARIANTS="base5=base5 polls=polls drain=- g8=-,CVXG_DF_GROUP8=1" ROUNDS=3 bash scripts/gpu_abv.sh; chk $? abv
exit 0

#!/bin/bash
# Round-5 session O: the worker claim-ahead with batched dependency polls (k_dataflow.hip): the chain / parity tests on
# the new default library, then the A/B of base5 (head before the change) against it, with a chain trace of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05o; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -k "chain_owned or golden_baseline or speculative or batch or lookahead or regularized" --timeout 200 --timeout-method thread > $O/pytest_sel.log 2>&1; chk $? seltests
TAG=r05o/ab LIBS="base5 new" ROUNDS=3 bash scripts/gpu_abn.sh; chk $? abn
exit 0

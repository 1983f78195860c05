#!/bin/bash
# Round-5 session S: the last L_kk^-1 row-block handed to the chain as data-tagged granules (CVXG_CHAIN_TAG3=1, variant
# 27): chain bitwise test (all variants), fingerprints, A/B against the default with a chain trace of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r05s; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -k "chain_owned" --timeout 300 --timeout-method thread > $O/pytest_sel.log 2>&1; chk $? seltests
timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_default.txt 2>&1; chk $? fp_def
CVXG_CHAIN_TAG3=1 timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_tag3.txt 2>&1; chk $? fp_t3
TAG=r05s/ab VARIANTS="def=- t3=-,CVXG_CHAIN_TAG3=1" ROUNDS=3 bash scripts/gpu_abv.sh; chk $? abv
exit 0

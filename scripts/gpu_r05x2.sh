#!/bin/bash
# Round-5 session X2: four polls of the chain's flag waits in flight (CVXG_DF_POLL_DEPTH=4) and the pipelined worker
# MFMA loop (CVXG_DF_MFMA_PIPE=1), alone and together, against the default; fingerprints; chain test on pp4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r05x2; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
for v in poll4 pp4; do CVXG_LIB=$R/cvx_amd/libcvxg_$v.so timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_$v.txt 2>&1; chk $? fp_$v; done
CVXG_LIB=$R/cvx_amd/libcvxg_pp4.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -k "chain_owned or batch or regularized_first" --timeout 300 --timeout-method thread > $O/pytest_pp4.log 2>&1; chk $? tests_pp4
TAG=r05x2/ab VARIANTS="def=- pipe=pipe poll4=poll4 pp4=pp4" ROUNDS=3 bash scripts/gpu_abv.sh; chk $? abv
exit 0

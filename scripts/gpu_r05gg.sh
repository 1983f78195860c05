#!/bin/bash
# Round-5 session GG: the last L^-1 row-block stored by the waves that compute it, each drained before it counts
# itself (P64W_DIRECT3=1); fingerprints, chain tests, A/B against head.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r05gg; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
CVXG_LIB=$R/cvx_amd/libcvxg_d3.so timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_d3.txt 2>&1; chk $? fp_d3
CVXG_LIB=$R/cvx_amd/libcvxg_d3.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -k "chain_owned or batch or regularized or golden_baseline" --timeout 300 --timeout-method thread > $O/pytest_d3.log 2>&1; chk $? tests_d3
TAG=r05gg/ab VARIANTS="head=head d3=d3" ROUNDS=3 bash scripts/gpu_abv.sh; chk $? abv
exit 0

#!/bin/bash
# Round-5 session N: the speculative regularized pair: bitwise test, C3FULL with and without it, the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05n; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
timeout -k 10 60 ./microbench/sweep_abl > $O/sweep_abl.log 2>&1; chk $? sweep_abl
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -k "speculative_regularized or regularized_first or golden_baseline_sizes or batch_full or full_c3" --timeout 200 --timeout-method thread > $O/pytest_sel.log 2>&1; chk $? seltests
timeout -k 10 300 python bench.py --workload C3FULL > $O/full_spec.log 2>&1; chk $? full_spec
CVXG_SPEC_REG=0 timeout -k 10 300 python bench.py --workload C3FULL > $O/full_seq.log 2>&1; chk $? full_seq
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/ab_def1.json 2>&1; chk $? def1
exit 0

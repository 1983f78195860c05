#!/bin/bash
# ad-hoc GPU session: each GPU step under its own time limit, chained with &&
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "baseline_sizes" -v -s --timeout 240 --timeout-method thread > gpurun_out/pt_big.log 2>&1 ; echo "rc=$?" >> gpurun_out/pt_big.log
timeout -k 10 60 ./microbench/potrf64_bench 200 1 > gpurun_out/potrf64_stamps.log 2>&1; echo "rc=$?" >> gpurun_out/potrf64_stamps.log

#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "kkt or equality or batch or regularized or infeasible or host_t_loop or reduced or simplex" -v --timeout 200 --timeout-method thread > gpurun_out/pt.log 2>&1 ; echo "rc=$?" >> gpurun_out/pt.log

#!/bin/bash
# ad-hoc GPU session: each GPU step under its own time limit
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread > gpurun_out/pt_all.log 2>&1 ; echo "rc=$?" >> gpurun_out/pt_all.log

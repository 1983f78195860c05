#!/bin/bash
# Round-5 session Q: the sweep ablation (M7: interleaved reciprocal), then the full GPU suite, smoke and the default
# bench on the batched-poll head.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05q; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
timeout -k 10 60 ./microbench/sweep_abl > $O/sweep_abl.log 2>&1; chk $? sweep_abl
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; chk $? tests
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; chk $? smoke
timeout -k 10 400 python bench.py > $O/bench.log 2>&1; chk $? bench
exit 0

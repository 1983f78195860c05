#!/bin/bash
# Round-4 baseline session: smoke, GPU tests, bench, rocprof kernel trace of the exact bench command, one chain trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r04a
O=gpurun_out/r04a
chk() { local rc=$1; echo "[r04a] $2 exit=$rc" | tee -a $O/status.log; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; chk $? smoke
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; chk $? tests
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench.log 2>&1; chk $? bench
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$R/$O/prof.log" 2>&1; chk $? prof
cd "$R"
CVXG_DF_TRACE=$R/$O/df_trace.bin timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/bench_trace.log 2>&1; chk $? trace
echo "[r04a] done" | tee -a $O/status.log

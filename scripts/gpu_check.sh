#!/bin/bash
# One gpurun session: smoke -> gpu tests -> bench -> rocprof kernel stats.  Each GPU step has its own
# time limit; a fault / abort / timeout (exit >= 124 or 134/139) ends the session, test failures do not.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STAGES="${STAGES:-smoke tests bench prof}"
stop_if_fault() {  # $1 = exit code, $2 = stage
  local rc=$1
  echo "[gpu_check] $2 exit=$rc" | tee -a gpurun_out/status.log
  if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then
    echo "[gpu_check] stopping after $2 (fault/timeout)" | tee -a gpurun_out/status.log
    exit "$rc"
  fi
}
for st in $STAGES; do
  case $st in
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      stop_if_fault $? smoke ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
      stop_if_fault $? tests ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
      stop_if_fault $? bench ;;
    prof)
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --steps 10 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
      rc=$?; cd "$GRAFT_REPO_ROOT"; stop_if_fault $rc prof ;;
    pmc)
      # HBM traffic counters, one counter group per pass (FETCH_SIZE and WRITE_SIZE do not fit together)
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_fetch" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --steps 3 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/pmc_fetch.log" 2>&1
      rc=$?; cd "$GRAFT_REPO_ROOT"; stop_if_fault $rc pmc_fetch
      cd /tmp
      timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_write" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --steps 3 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/pmc_write.log" 2>&1
      rc=$?; cd "$GRAFT_REPO_ROOT"; stop_if_fault $rc pmc_write ;;
  esac
done
echo "[gpu_check] done" | tee -a gpurun_out/status.log

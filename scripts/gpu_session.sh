#!/bin/bash
# One gpurun session under gpurun_out/$TAG: STAGES (default "tests bench prof trace") each with its own time limit;
# a fault / abort / time limit (exit >= 124, 134, 139) ends the session.  PYTEST_K selects GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
TAG=${TAG:-run}
O=gpurun_out/$TAG
mkdir -p $O
chk() { local rc=$1; echo "[$TAG] $2 exit=$rc" | tee -a $O/status.log; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
for st in ${STAGES:-tests bench prof trace}; do
  case $st in
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; chk $? smoke ;;
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1; chk $? tests ;;
    bench) timeout -k 10 400 python bench.py ${BENCH_ARGS:---no-cpu-baseline --steps 20 --warmup 5} > $O/bench.log 2>&1; chk $? bench ;;
    bench2) timeout -k 10 400 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench2.log 2>&1; chk $? bench2 ;;
    prof) cd /tmp && export TMPDIR=/tmp
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$R/$O/prof.log" 2>&1; rc=$?; cd "$R"; chk $rc prof ;;
    trace) CVXG_DF_TRACE=$R/$O/df_trace.bin timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/bench_trace.log 2>&1; chk $? trace ;;
    *) bash -c "$st" > $O/extra.log 2>&1; chk $? extra ;;
  esac
done
echo "[$TAG] done" | tee -a $O/status.log

#!/bin/bash
# Round-5 session L: Ruiz loop with interleaved DPP sums and no spills: bitwise tests, trace, A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r05l; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -k "ruiz_loop_bitwise or ruiz_lookahead or golden_baseline" --timeout 200 --timeout-method thread > $O/pytest_sel.log 2>&1; chk $? seltests
CVXG_RUIZ_LOOP=1 CVXG_RUIZ_TRACE=$R/$O/ruiz.bin timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/trace_ruiz.log 2>&1; chk $? ruiztrace
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline"
for i in 1 2; do
  timeout -k 10 300 $B > $O/ab_def$i.json 2>&1; chk $? def$i
  CVXG_RUIZ_LOOP=1 timeout -k 10 300 $B > $O/ab_rl$i.json 2>&1; chk $? rl$i
  CVXG_CHAIN_DPP=1 timeout -k 10 300 $B > $O/ab_dpp$i.json 2>&1; chk $? dpp$i
  CVXG_CHAIN_DPP=1 CVXG_RUIZ_LOOP=1 timeout -k 10 300 $B > $O/ab_rldpp$i.json 2>&1; chk $? rldpp$i
done
exit 0

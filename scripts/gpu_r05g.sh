#!/bin/bash
# Round-5 session G: tagged Ruiz loop v2 and the b-2 staging fix: bitwise tests, the multi-context tests, same-box
# bench A/B, one dataflow task trace and a kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r05g; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -k "ruiz_loop_bitwise or chain_owned or batch or full_c3 or lookahead" --timeout 200 --timeout-method thread > $O/pytest_sel.log 2>&1; rc=$?; chk $rc seltests
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline"
for i in 1 2; do
  timeout -k 10 300 $B > $O/ab_def$i.json 2>&1; chk $? def$i
  CVXG_CHAIN_B2=0 CVXG_CHAIN_DEFER=0 CVXG_RUIZ_LOOP=0 timeout -k 10 300 $B > $O/ab_old$i.json 2>&1; chk $? old$i
  CVXG_CHAIN_B2=0 CVXG_CHAIN_DEFER=0 timeout -k 10 300 $B > $O/ab_rl$i.json 2>&1; chk $? rl$i
  CVXG_CHAIN_DPP=1 timeout -k 10 300 $B > $O/ab_dpp$i.json 2>&1; chk $? dpp$i
  CVXG_CHAIN_B2=0 timeout -k 10 300 $B > $O/ab_dfonly$i.json 2>&1; chk $? dfonly$i
done
CVXG_DF_TRACE=$R/$O/df_1100.bin timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/trace_1100.log 2>&1; chk $? trace
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$R/$O/prof.log" 2>&1; chk $? prof
exit 0

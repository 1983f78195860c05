#!/bin/bash
# Round-5 session J: chain with the prefetched b-2 staging (A/B vs the round-4 chain and the DPP sweep), chain trace,
# Ruiz loop trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r05j; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -k "chain_owned or ruiz_loop_bitwise" --timeout 200 --timeout-method thread > $O/pytest_sel.log 2>&1; chk $? seltests
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline"
for i in 1 2 3; do
  timeout -k 10 300 $B > $O/ab_def$i.json 2>&1; chk $? def$i
  CVXG_CHAIN_B2=0 CVXG_CHAIN_DEFER=0 timeout -k 10 300 $B > $O/ab_ch0$i.json 2>&1; chk $? ch0$i
  CVXG_CHAIN_DPP=1 timeout -k 10 300 $B > $O/ab_dpp$i.json 2>&1; chk $? dpp$i
done
for v in 1100 1101; do
  CVXG_CHAIN_B2=${v:0:1} CVXG_CHAIN_DEFER=${v:1:1} CVXG_CHAIN_TAG=${v:2:1} CVXG_CHAIN_DPP=${v:3:1} CVXG_DF_TRACE=$R/$O/df_$v.bin timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/trace_$v.log 2>&1; chk $? trace$v
done
CVXG_RUIZ_LOOP=1 CVXG_RUIZ_TRACE=$R/$O/ruiz.bin timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/trace_ruiz.log 2>&1; chk $? ruiztrace
exit 0

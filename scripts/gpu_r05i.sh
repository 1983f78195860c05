#!/bin/bash
# Round-5 session I: Ruiz loop (fixed streamed claims, one-round-trip polls): selected tests; chain A/B incl. the
# tagged hand-off; dataflow traces with the row-block flag stamps; kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r05i; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -k "ruiz_loop_bitwise or batch or full_c3 or chain_owned" --timeout 200 --timeout-method thread > $O/pytest_sel.log 2>&1; chk $? seltests
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline"
for i in 1 2; do
  timeout -k 10 300 $B > $O/ab_def$i.json 2>&1; chk $? def$i
  CVXG_RUIZ_LOOP=0 timeout -k 10 300 $B > $O/ab_rloff$i.json 2>&1; chk $? rloff$i
  CVXG_CHAIN_B2=0 CVXG_CHAIN_DEFER=0 timeout -k 10 300 $B > $O/ab_ch0$i.json 2>&1; chk $? ch0$i
  CVXG_CHAIN_TAG=1 timeout -k 10 300 $B > $O/ab_tag$i.json 2>&1; chk $? tag$i
  CVXG_CHAIN_TAG=1 CVXG_CHAIN_DPP=1 timeout -k 10 300 $B > $O/ab_tagdpp$i.json 2>&1; chk $? tagdpp$i
done
for v in 1100 0000 1110; do
  CVXG_CHAIN_B2=${v:0:1} CVXG_CHAIN_DEFER=${v:1:1} CVXG_CHAIN_TAG=${v:2:1} CVXG_CHAIN_DPP=${v:3:1} CVXG_DF_TRACE=$R/$O/df_$v.bin timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/trace_$v.log 2>&1; chk $? trace$v
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$R/$O/prof.log" 2>&1; chk $? prof
exit 0

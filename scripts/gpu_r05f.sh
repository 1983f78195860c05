#!/bin/bash
# Round-5 session F: chain variants (CVXG_CHAIN_B2 / _DEFER / _TAG / _DPP) and the one-launch Ruiz loop
# (CVXG_RUIZ_LOOP): POTRF microbench (v_readlane vs DPP sweep), their bitwise tests first, GPU suite, same-box bench
# A/B and dataflow task traces, kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r05f; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
for v in false true; do timeout -k 10 120 ./microbench/potrf64w_bench_dpp_$v 400 > $O/p64_dpp_$v.log 2>&1; chk $? p64_$v; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -k "ruiz_loop_bitwise or chain_owned" --timeout 200 --timeout-method thread > $O/pytest_new.log 2>&1; rc=$?; chk $rc newtests
[ $rc -ne 0 ] && exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; chk $? pytest
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline"
for i in 1 2; do
  timeout -k 10 300 $B > $O/ab_def$i.json 2>&1; chk $? def$i
  CVXG_CHAIN_B2=0 CVXG_CHAIN_DEFER=0 CVXG_RUIZ_LOOP=0 timeout -k 10 300 $B > $O/ab_old$i.json 2>&1; chk $? old$i
  CVXG_CHAIN_B2=0 timeout -k 10 300 $B > $O/ab_b2off$i.json 2>&1; chk $? b2off$i
  CVXG_CHAIN_DEFER=0 CVXG_CHAIN_B2=0 timeout -k 10 300 $B > $O/ab_dfoff$i.json 2>&1; chk $? dfoff$i
  CVXG_CHAIN_TAG=1 timeout -k 10 300 $B > $O/ab_tag$i.json 2>&1; chk $? tag$i
  CVXG_CHAIN_DPP=1 timeout -k 10 300 $B > $O/ab_dpp$i.json 2>&1; chk $? dpp$i
  CVXG_CHAIN_DPP=1 CVXG_CHAIN_TAG=1 timeout -k 10 300 $B > $O/ab_all$i.json 2>&1; chk $? all$i
  CVXG_RUIZ_LOOP=0 timeout -k 10 300 $B > $O/ab_rloff$i.json 2>&1; chk $? rloff$i
done
for v in 1100 0000 1111; do
  CVXG_CHAIN_B2=${v:0:1} CVXG_CHAIN_DEFER=${v:1:1} CVXG_CHAIN_TAG=${v:2:1} CVXG_CHAIN_DPP=${v:3:1} CVXG_DF_TRACE=$R/$O/df_$v.bin timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/trace_$v.log 2>&1; chk $? trace$v
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$R/$O/prof.log" 2>&1; chk $? prof
exit 0

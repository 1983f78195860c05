#!/bin/bash
# Round-5 session F: chain-owned panel b-2 updates (CVXG_CHAIN_B2) and the one-launch Ruiz loop (CVXG_RUIZ_LOOP):
# their bitwise tests first, GPU suite, same-box bench A/B (default / b2 off / Ruiz loop off) and dataflow task traces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r05f; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s -k "ruiz_loop_bitwise or chain_owned" --timeout 120 --timeout-method thread > $O/pytest_new.log 2>&1; rc=$?; chk $rc newtests
[ $rc -ne 0 ] && exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; chk $? pytest
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline"
for i in 1 2 3; do
  timeout -k 10 300 $B > $O/ab_def$i.json 2>&1; chk $? def$i
  CVXG_CHAIN_B2=0 timeout -k 10 300 $B > $O/ab_b2off$i.json 2>&1; chk $? b2off$i
  CVXG_CHAIN_DEFER=0 timeout -k 10 300 $B > $O/ab_dfoff$i.json 2>&1; chk $? dfoff$i
  CVXG_CHAIN_TAG=1 timeout -k 10 300 $B > $O/ab_tag$i.json 2>&1; chk $? tag$i
  CVXG_RUIZ_LOOP=0 timeout -k 10 300 $B > $O/ab_rloff$i.json 2>&1; chk $? rloff$i
done
for v in 110 000 111; do
  CVXG_CHAIN_B2=${v:0:1} CVXG_CHAIN_DEFER=${v:1:1} CVXG_CHAIN_TAG=${v:2:1} CVXG_DF_TRACE=$R/$O/df_$v.bin timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/trace_$v.log 2>&1; chk $? trace$v
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$R/$O/prof.log" 2>&1; chk $? prof
exit 0

#!/bin/bash
# Round-5 session E: GPU suite; same-box A/B of the evaluation tail (P x bounded beside the SYRK / unbounded / before
# it on the main stream) and of the lower-only assembly (CVXG_H_LOWER=0: mirrored); kernel trace + HBM PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r05e; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; chk $? pytest
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline"
for i in 1 2 3; do
  timeout -k 10 300 $B > $O/ab_prod$i.json 2>&1; chk $? prod$i
  CVXG_LIB=$R/exp_build/libcvxg_pxfull.so timeout -k 10 300 $B > $O/ab_pxfull$i.json 2>&1; chk $? pxfull$i
  CVXG_LIB=$R/exp_build/libcvxg_pxmain.so timeout -k 10 300 $B > $O/ab_pxmain$i.json 2>&1; chk $? pxmain$i
  CVXG_H_LOWER=0 timeout -k 10 300 $B > $O/ab_hfull$i.json 2>&1; chk $? hfull$i
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$R/$O/prof.log" 2>&1; chk $? prof
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/pmc_fetch" -o run -- python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 > "$R/$O/pmc_fetch.log" 2>&1; chk $? fetch
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$O/pmc_write" -o run -- python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 > "$R/$O/pmc_write.log" 2>&1; chk $? write
exit 0

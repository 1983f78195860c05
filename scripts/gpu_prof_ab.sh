#!/bin/bash
# rocprofv3 kernel stats of bench.py for several library builds (cvx_amd/libcvxg_$v.so, v in $LIBS) -> gpurun_out/$TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
TAG=${TAG:-profab}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in $LIBS; do
  CVXG_LIB=$R/cvx_amd/libcvxg_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/$v.log 2>&1
  rc=$?; echo "[$TAG] $v exit=$rc" | tee -a $O/status.log; [ $rc -ne 0 ] && exit $rc
done
echo "[$TAG] done" | tee -a $O/status.log

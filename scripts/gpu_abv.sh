#!/bin/bash
# A/B/n of variants on one box: VARIANTS="name=lib[,ENV=value...] ..." (lib: cvx_amd/libcvxg_<lib>.so, "-" for the
# default libcvxg.so).  A chain trace of each, then ROUNDS rounds of bench runs in rotation.  Output under
# gpurun_out/$TAG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
TAG=${TAG:-abv}
O=gpurun_out/$TAG
mkdir -p $O
chk() { local rc=$1; echo "[$TAG] $2 exit=$rc" | tee -a $O/status.log; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
run() {  # run <variant spec> <command...>
  local spec=$1; shift
  local name=${spec%%=*} rest=${spec#*=}
  local lib=${rest%%,*} envs=""
  [ "$rest" != "$lib" ] && envs=${rest#*,}
  local libpath=$R/cvx_amd/libcvxg.so
  [ "$lib" != "-" ] && libpath=$R/cvx_amd/libcvxg_$lib.so
  env CVXG_LIB=$libpath ${envs//,/ } "$@"
}
for v in $VARIANTS; do
  n=${v%%=*}
  run "$v" env CVXG_DF_TRACE=$R/$O/df_$n.bin timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/trace_$n.log 2>&1; chk $? trace_$n
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    n=${v%%=*}
    run "$v" timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/ab_$n$r.log 2>&1; chk $? $n$r
  done
done
echo "[$TAG] done" | tee -a $O/status.log

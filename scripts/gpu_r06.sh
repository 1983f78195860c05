#!/bin/bash
# Round-6 session under gpurun_out/$TAG: smoke, the GPU suite (-s: every printed parity number), and a same-box A/B of
# library builds cvx_amd/libcvxg_$v.so for v in $LIBS (a chain trace of each, then ROUNDS rounds of 30-step benches in
# rotation).  STAGES selects; a fault, abort or timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
TAG=${TAG:-r06}
O=gpurun_out/$TAG
mkdir -p $O
chk() { local rc=$1; echo "[$TAG] $2 exit=$rc" | tee -a $O/status.log; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
for st in ${STAGES:-smoke tests ab}; do
  case $st in
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; chk $? smoke ;;
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1; chk $? tests ;;
    ab)
      for v in ${LIBS:-}; do
        CVXG_LIB=$R/cvx_amd/libcvxg_$v.so CVXG_DF_TRACE=$R/$O/df_$v.bin timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/trace_$v.log 2>&1; chk $? trace_$v
        python scripts/chain_offsets.py $O/df_$v.bin > $O/chain_offsets_$v.txt 2>&1
        python scripts/df_util.py $O/df_$v.bin > $O/df_util_$v.txt 2>&1
      done
      for r in $(seq 1 ${ROUNDS:-2}); do
        for v in ${LIBS:-}; do
          CVXG_LIB=$R/cvx_amd/libcvxg_$v.so timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/ab_$v$r.json 2>$O/ab_$v$r.err; chk $? $v$r
        done
      done
      python scripts/ab_summary.py $O > $O/ab_summary.txt 2>&1 ;;
    abfull)  # whole C3 solves (regularized steps: the speculative pair) with each library, in rotation
      for r in $(seq 1 ${ROUNDS:-2}); do
        for v in ${LIBS:-}; do
          CVXG_LIB=$R/cvx_amd/libcvxg_$v.so timeout -k 10 300 python bench.py --workload C3FULL > $O/full_$v$r.json 2>$O/full_$v$r.err; chk $? full_$v$r
        done
      done ;;
    bench) timeout -k 10 500 python bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1; chk $? bench ;;
    full) timeout -k 10 300 python bench.py --workload C3FULL > $O/bench_full.log 2>&1; chk $? full ;;
    ruizloop)  # the one-launch Ruiz loop against the launch pairs at C2 and C4
      for wl in C2 C4; do
        for o in 0 1; do
          timeout -k 10 200 python bench.py --workload $wl --steps 50 --warmup 5 --no-cpu-baseline --opt ruiz_loop=$o > $O/ruiz_${wl}_$o.json 2>$O/ruiz_${wl}_$o.err; chk $? ruiz_${wl}_$o
        done
      done ;;
    side)  # the side workloads on the current build
      for wl in C2 C4 C3B C4P C2PD C3PD; do
        timeout -k 10 300 python bench.py --workload $wl --steps 30 --warmup 3 --no-cpu-baseline > $O/wl_$wl.json 2>$O/wl_$wl.err; chk $? wl_$wl
      done ;;
    c2x)  # C2 instances sharing one GPU
      for k in 4 8; do
        timeout -k 10 300 python bench.py --workload C2X --instances $k --steps 60 --warmup 5 > $O/wl_C2x$k.json 2>$O/wl_C2x$k.err; chk $? c2x$k
      done ;;
    old)  # whole C3 solves with the libraries of two round-5 commits (exp6/c<sha>: each commit's own bench.py)
      for c in ${OLD:-}; do
        (cd exp6/c$c && timeout -k 10 300 python bench.py --workload C3FULL > $R/$O/c3full_$c.json 2>$R/$O/c3full_$c.err); chk $? old_$c
      done ;;
  esac
done
echo "[$TAG] done" | tee -a $O/status.log

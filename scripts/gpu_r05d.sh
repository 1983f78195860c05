#!/bin/bash
# Round-5 session D: sweep / POTRF64 microbenchmarks (DPP column sweep vs round 4), GPU suite on the DPP POTRF,
# same-box bench A/B against the round-4 POTRF build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05d; mkdir -p $O
fault() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
run() { local name=$1; shift; timeout -k 10 120 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name $rc"; fault $rc && exit $rc; return 0; }
run sweep ./microbench/sweep
run sweep_dpp ./microbench/sweep_dpp
run p64_new ./microbench/potrf64w_bench 400
run p64_r04 ./microbench/potrf64w_bench_r04 400
run p64lf_new ./microbench/potrf64w_bench_lf 400
run p64lf_r04 ./microbench/potrf64w_bench_lf_r04 400
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest $rc"; fault $rc && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_new$i.log 2>&1; rc=$?; echo "bench_new$i $rc"; fault $rc && exit $rc
  CVXG_LIB=$PWD/exp_build/libcvxg_r04potrf.so timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_r04$i.log 2>&1; rc=$?; echo "bench_r04$i $rc"; fault $rc && exit $rc
done
exit 0

cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_all.log 2>&1
echo "rc=$?" >> gpurun_out/pt_all.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_q.log 2>&1
echo "rc=$?" >> gpurun_out/bench_q.log

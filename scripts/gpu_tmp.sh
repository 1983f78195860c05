#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -c "
import sys, time
sys.argv=['bench.py']
import bench
from cvx_amd import problems as Z
spec = Z.random_qp(4096, 8192, instance=0)
for nw in (1, 4):
    t=time.time(); r = bench.cpu_baseline(spec, 60.0, fraction=0.02 * nw, workers=nw); print(nw, r['sample'], time.time()-t, flush=True)
" > gpurun_out/cpu_contention.log 2>&1; echo rc=$? >> gpurun_out/cpu_contention.log

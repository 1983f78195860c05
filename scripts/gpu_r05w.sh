#!/bin/bash
# Round-5 session W: schedule estimates around the new default (6:5:4:12.5) and the pipelined worker MFMA loop
# (CVXG_DF_MFMA_PIPE=1: negated tile, the next k-pair's LDS reads after the first two MFMAs); fingerprint of pipe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r05w; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_def.txt 2>&1; chk $? fp_def
CVXG_LIB=$R/cvx_amd/libcvxg_pipe.so timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_pipe.txt 2>&1; chk $? fp_pipe
TAG=r05w/ab VARIANTS="def=- pipe=pipe b=-,CVXG_DF_SCHED=7:4:3.5:12.5:100:3:2 g=-,CVXG_DF_SCHED=6:5:4:13:100:3:2 h=-,CVXG_DF_SCHED=6.5:4.5:3.5:12.5:100:3:2 i=-,CVXG_DF_SCHED=6:4.5:4:12:100:3:2" ROUNDS=2 bash scripts/gpu_abv.sh; chk $? abv
exit 0

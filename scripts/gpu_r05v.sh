#!/bin/bash
# Round-5 session V: the list-schedule estimates around the new default (7:5:4:12.5:100:3:2); fingerprints of the new
# default and the old estimates (the task order changes, the arithmetic per tile does not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05v; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_new.txt 2>&1; chk $? fp_new
CVXG_DF_SCHED=10:6:5.5:16:100:3:2 timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_old.txt 2>&1; chk $? fp_old
TAG=r05v/ab VARIANTS="def=- a=-,CVXG_DF_SCHED=6:5:4:12.5:100:3:2 b=-,CVXG_DF_SCHED=7:4:3.5:12.5:100:3:2 c=-,CVXG_DF_SCHED=7:5:4:11:100:3:2 d=-,CVXG_DF_SCHED=8:5.5:4.5:12.5:100:3:2 e=-,CVXG_DF_SCHED=5:5:4:12.5:100:3:2" ROUNDS=2 bash scripts/gpu_abv.sh; chk $? abv
exit 0

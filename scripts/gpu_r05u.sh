#!/bin/bash
# Round-5 session U: (1) the worker updates on the negated tile (no sign flip between LDS read and MFMA; same bits)
# against the head; (2) list-schedule parameters re-swept after the worker fix on the head library (CVXG_DF_SCHED =
# "potrf:trsm:upd:upd4:boost:band:singles"; default 10:6:5.5:16:100:3:2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r05u; mkdir -p $O
chk() { local rc=$1; echo "$2 $rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_neg.txt 2>&1; chk $? fp_neg
CVXG_LIB=$R/cvx_amd/libcvxg_head.so timeout -k 10 300 python scripts/lib_fingerprint.py > $O/fp_head.txt 2>&1; chk $? fp_head
TAG=r05u/ab VARIANTS="head=head neg=neg s1=head,CVXG_DF_SCHED=7:5:4:12.5:100:3:2 s2=head,CVXG_DF_SCHED=7:5:4:12.5:50:3:2 s3=head,CVXG_DF_SCHED=7:5:4:12.5:200:3:2 s4=head,CVXG_DF_SCHED=7:5:4:12.5:100:4:2 s5=head,CVXG_DF_SCHED=10:6:5.5:16:100:3:3" ROUNDS=2 bash scripts/gpu_abv.sh; chk $? abv
exit 0

#!/bin/bash
# Round-5 session U: list-schedule parameters re-swept after the worker fix (CVXG_DF_SCHED =
# "potrf:trsm:upd:upd4:boost:band:singles"; default 10:6:5.5:16:100:3:2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r05u/ab VARIANTS="def=- s1=-,CVXG_DF_SCHED=7:5:4:12.5:100:3:2 s2=-,CVXG_DF_SCHED=7:5:4:12.5:50:3:2 s3=-,CVXG_DF_SCHED=7:5:4:12.5:200:3:2 s4=-,CVXG_DF_SCHED=7:5:4:12.5:100:4:2 s5=-,CVXG_DF_SCHED=10:6:5.5:16:100:3:3" ROUNDS=2 bash scripts/gpu_abv.sh

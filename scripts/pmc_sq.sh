#!/bin/bash
# SQ counters of one kernel (regex $1) over a short bench run, two passes (8 SQ slots each).
set -u
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
K=${1:-k_syrk_assemble}
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_CYCLES --kernel-include-regex "$K" --output-format csv -d $R/gpurun_out/pmc_sq1 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 0 > $R/gpurun_out/pmc_sq1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_F64 SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_ADDR_CONFLICT --kernel-include-regex "$K" --output-format csv -d $R/gpurun_out/pmc_sq2 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 0 > $R/gpurun_out/pmc_sq2.log 2>&1

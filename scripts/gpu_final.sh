#!/bin/bash
# Round-end evidence session under gpurun_out/$TAG: smoke, the GPU suite (-s), the default bench (with the CPU
# baselines), a rocprofv3 kernel trace of `bench.py --steps 20 --warmup 5 --no-cpu-baseline`, HBM traffic passes
# (FETCH_SIZE, WRITE_SIZE), SQ passes for the Cholesky and the SYRK, a chain trace, C3FULL and C3X2.  STAGES selects.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
TAG=${TAG:-final}
O=gpurun_out/$TAG
mkdir -p $O
chk() { local rc=$1; echo "[$TAG] $2 exit=$rc" | tee -a $O/status.log; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
SQ1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_CYCLES"
SQ2="SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_F64 SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_ADDR_CONFLICT"
for st in ${STAGES:-smoke tests bench prof fetch write sq1 sq2 trace full x2}; do
  case $st in
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; chk $? smoke ;;
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; chk $? tests ;;
    bench) timeout -k 10 500 python bench.py > $O/bench.log 2>&1; chk $? bench ;;
    prof) cd /tmp && export TMPDIR=/tmp
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$R/$O/prof.log" 2>&1; rc=$?; cd "$R"; chk $rc prof ;;
    fetch) cd /tmp && export TMPDIR=/tmp
      timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/pmc_fetch" -o run -- python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 > "$R/$O/pmc_fetch.log" 2>&1; rc=$?; cd "$R"; chk $rc fetch ;;
    write) cd /tmp && export TMPDIR=/tmp
      timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$O/pmc_write" -o run -- python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 > "$R/$O/pmc_write.log" 2>&1; rc=$?; cd "$R"; chk $rc write ;;
    sq1) cd /tmp && export TMPDIR=/tmp
      timeout -k 10 300 rocprofv3 --pmc $SQ1 --kernel-include-regex "k_chol_dataflow|k_syrk_direct" --output-format csv -d "$R/$O/pmc_sq1" -o run -- python3 "$R/bench.py" --no-cpu-baseline --steps 2 --warmup 0 > "$R/$O/pmc_sq1.log" 2>&1; rc=$?; cd "$R"; chk $rc sq1 ;;
    sq2) cd /tmp && export TMPDIR=/tmp
      timeout -k 10 300 rocprofv3 --pmc $SQ2 --kernel-include-regex "k_chol_dataflow|k_syrk_direct" --output-format csv -d "$R/$O/pmc_sq2" -o run -- python3 "$R/bench.py" --no-cpu-baseline --steps 2 --warmup 0 > "$R/$O/pmc_sq2.log" 2>&1; rc=$?; cd "$R"; chk $rc sq2 ;;
    trace) CVXG_DF_TRACE=$R/$O/df_trace.bin timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/bench_trace.log 2>&1; chk $? trace ;;
    full) timeout -k 10 300 python bench.py --workload C3FULL > $O/bench_full.log 2>&1; chk $? full ;;
    x2) timeout -k 10 300 python bench.py --workload C3X2 --steps 30 --warmup 3 > $O/bench_x2.log 2>&1; chk $? x2 ;;
  esac
done
echo "[$TAG] done" | tee -a $O/status.log

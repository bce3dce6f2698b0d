#!/bin/bash
# PMC counters for the top kernels (separate passes; --pmc only with --kernel-trace)
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  tag=$(echo $set | cut -d' ' -f1)
  [ "$tag" = "SQ_VALU_MFMA_BUSY_CYCLES" ] && tag=MFMA_BUSY
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/pmc/$tag -o run -f csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > gpurun_out/pmc/$tag.log 2>&1 || exit $?
done

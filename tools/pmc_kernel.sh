#!/bin/bash
# SQ counters for the kernels matching $KERNEL (regex), one pass each set,
# --kernel-trace only; extra env (e.g. VOXEMB_NO_CONV3_RW=1) passes through.
export TMPDIR=/tmp
K=${KERNEL:-conv3x3}
O=gpurun_out/pmck_${TAG:-x}
mkdir -p $O
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_WAVES" \
           ${EXTRA_SETS}; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --kernel-include-regex "$K" --pmc $set -d $O/p$i -o run -f csv \
    -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $O/p$i.log 2>&1 || exit $?
done

#!/bin/bash
# PMC passes for one kernel (default gemm1x1_pipe), grouped later by launch
# position with tools/pmc_by_position.py.  Separate passes, --kernel-trace only.
export TMPDIR=/tmp
K=${KERNEL:-gemm1x1_pipe}
O=gpurun_out/pmck
mkdir -p $O
i=0
for set in "GRBM_GUI_ACTIVE TA_BUSY_avr" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" \
           "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU" "FETCH_SIZE" "WRITE_SIZE" \
           "TCP_PENDING_STALL_CYCLES_sum TD_TD_BUSY_sum" "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex "$K" --pmc $set -d $O/p$i -o run -f csv \
    -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $O/p$i.log 2>&1 || exit $?
done

#!/bin/bash
# gemm1x1_pipe diagnostics: per-op times with the normal kernel, without MFMAs
# (VOXEMB_GEMM_VAR=2) and without operand DMA (3)
export TMPDIR=/tmp
for v in 0 2 3; do
  VOXEMB_GEMM_VAR=$v timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --dump-ops \
    > gpurun_out/diag_v$v.json 2> gpurun_out/diag_v$v.ops || exit $?
done

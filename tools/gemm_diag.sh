#!/bin/bash
# 1x1 GEMM diagnostics: per-op times of the product kernel and of diagnostic
# variants (VOXEMB_GEMM_VAR: wide kernel 11 = no MFMA, 12 = no operand DMA,
# 14 = no stores, 13/15/16 = combinations; pipe kernel 2 = no MFMA, 3 = no DMA)
# diagnostic variants live in the VOX_DIAG build (python -m voxsrc2020_speaker_verification_amd.build_native --diag)
export VOXEMB_LIB=${VOXEMB_LIB:-$PWD/voxsrc2020_speaker_verification_amd/libvoxemb_diag.so}
export TMPDIR=/tmp
for v in ${VARS:-0 11 12 14 13 15 16}; do
  VOXEMB_GEMM_VAR=$v timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --dump-ops \
    > gpurun_out/diag_v$v.json 2> gpurun_out/diag_v$v.ops || exit $?
done

#!/bin/bash
# per-op times of the gemm1x1_wide launches under its diagnostic variants
# diagnostic variants live in the VOX_DIAG build (python -m voxsrc2020_speaker_verification_amd.build_native --diag)
export VOXEMB_LIB=${VOXEMB_LIB:-$PWD/voxsrc2020_speaker_verification_amd/libvoxemb_diag.so}
O=gpurun_out/gvar
mkdir -p $O
for v in ${VALUES:-0 11 12 14 15 16}; do
  VOXEMB_GEMM_VAR=$v timeout -k 10 120 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --dump-ops \
    > $O/v$v.json 2> $O/v$v.txt || exit $?
  echo "var $v: $(grep gemmwide $O/v$v.txt | awk '{print $1}' | tr '\n' ' ')"
done

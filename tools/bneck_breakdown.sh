#!/bin/bash
# Time the fused bottleneck with parts skipped (VOXEMB_BNECK_DBG bits: 1 A, 2 C, 4 chain, 8 global loads)
# diagnostic variants live in the VOX_DIAG build (python -m voxsrc2020_speaker_verification_amd.build_native --diag)
export VOXEMB_LIB=${VOXEMB_LIB:-$PWD/voxsrc2020_speaker_verification_amd/libvoxemb_diag.so}
for d in 0 1 2 4 8 3 7 15; do
  echo "dbg=$d $(VOXEMB_BNECK_DBG=$d python bench.py --steps 3 --warmup 1 --no-cpu-baseline | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernels"]["bneck_fused"])')"
done

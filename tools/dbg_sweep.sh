#!/bin/bash
# Time one kernel family under debug-variant env settings (results are wrong
# for dbg != 0; timing only).  ENVVAR=VOXEMB_BNECK_DBG VALUES="0 1 2" KEY=bneck_fused
# diagnostic variants live in the VOX_DIAG build (python -m voxsrc2020_speaker_verification_amd.build_native --diag)
export VOXEMB_LIB=${VOXEMB_LIB:-$PWD/voxsrc2020_speaker_verification_amd/libvoxemb_diag.so}
O=gpurun_out/sweep_${TAG:-x}
mkdir -p $O
for v in ${VALUES:-0}; do
  env ${ENVVAR:-VOXEMB_BNECK_DBG}=$v timeout -k 10 120 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline \
    > $O/v$v.json 2> $O/v$v.err || exit $?
  python3 -c "import json,sys; d=json.load(open('$O/v$v.json')); k=d['kernels']; print('$v', d['value'], {n: round(k[n]['ms'],4) for n in k if '${KEY:-bneck}' in n})"
done

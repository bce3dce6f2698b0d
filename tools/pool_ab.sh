#!/bin/bash
# In-situ A/B of stats_pool_col variants at the headline (the pool reads the map
# the last 1x1c just wrote): product library (VOX_POOL_VAR 0 = 4 channels per
# thread) vs libvoxemb_pool{1,2,3}.so built with -DVOX_POOL_VAR=1 (2 channels),
# 2 (4 channels, non-temporal loads), 3 (2 channels, non-temporal); per-op pool
# time from bench --dump-ops, alternating, twice each; pool tests per variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pool
P=$PWD/voxsrc2020_speaker_verification_amd
for v in 1 2 3; do
  VOXEMB_LIB=$P/libvoxemb_pool$v.so timeout -k 10 200 python -u -m pytest tests -q -m gpu -k "stats_pool or headline" \
    --timeout 120 --timeout-method thread > gpurun_out/pool/t$v.log 2>&1 || { echo "tests v$v rc=$?"; tail -20 gpurun_out/pool/t$v.log; exit 1; }
  echo "v$v tests: $(tail -1 gpurun_out/pool/t$v.log)"
done
for r in 0 1; do for v in 0 1 2 3; do
  L=$P/libvoxemb.so; [ $v -gt 0 ] && L=$P/libvoxemb_pool$v.so
  VOXEMB_LIB=$L timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --dump-ops \
    > gpurun_out/pool/b${v}_$r.json 2> gpurun_out/pool/o${v}_$r.txt || { echo "bench v$v rc=$?"; exit 1; }
  echo "v$v run$r: $(python3 -c "import json; d=json.load(open('gpurun_out/pool/b${v}_$r.json')); print(d['value'], d['ms_per_step'])") pool: $(grep -i ' pool' gpurun_out/pool/o${v}_$r.txt | awk '{printf "%s ", $1}')"
done; done

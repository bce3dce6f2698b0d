#!/bin/bash
# per-op times of the gemm1x1_wide launches under its diagnostic variants
O=gpurun_out/gvar
mkdir -p $O
for v in ${VALUES:-0 11 12 14 15 16}; do
  VOXEMB_GEMM_VAR=$v timeout -k 10 120 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --dump-ops \
    > $O/v$v.json 2> $O/v$v.txt || exit $?
  echo "var $v: $(grep gemmwide $O/v$v.txt | awk '{print $1}' | tr '\n' ' ')"
done

#!/bin/bash
# Same-box A/B of two libvoxemb builds: tools/libvoxemb_a.so (A) vs the
# in-tree library (B), alternating, bench per-kernel ms for $KEY.
for i in 1 2; do
  for v in A B; do
    if [ $v = A ]; then export VOXEMB_LIB=$PWD/tools/libvoxemb_a.so; else unset VOXEMB_LIB; fi
    timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -5 gpurun_out/ab_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); k=d['kernels']; print('$v', round(d['value']), {n: round(k[n]['ms'],4) for n in k if '${KEY:-bneck}' in n})"
  done
done

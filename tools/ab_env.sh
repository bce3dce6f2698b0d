#!/bin/bash
# Same-box A/B of one library with an environment switch: A = "$ABENV" set
# (e.g. ABENV=VOXEMB_NO_WBLK=1), B = unset; alternating bench runs, per-kernel ms for $KEY.
for i in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then envs="$ABENV"; else envs=""; fi
    env $envs timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -5 gpurun_out/ab_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); k=d['kernels']; print('$v', round(d['value']), {n: round(k[n]['ms'],4) for n in k if '${KEY:-gemm}' in n})"
  done
done

#!/bin/bash
# sweep split_chain row-tile R and WPX; report chain op time and step time
for cfg in "0 0 8" "0 2 8"; do
  set -- $cfg; export VOXEMB_CHAIN_NW=$3
  VOXEMB_CHAIN_R=$1 VOXEMB_CHAIN_WPX=$2 timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --dump-ops > gpurun_out/ch_$1_$2.json 2> gpurun_out/ch_$1_$2.ops || exit $?
  python - "$1" "$2" <<'PY'
import json, sys, re
r, wpx = sys.argv[1:3]
d = json.load(open(f"gpurun_out/ch_{r}_{wpx}.json"))
tot = {}
for line in open(f"gpurun_out/ch_{r}_{wpx}.ops"):
    m = re.match(r"\s*([\d.]+) us\s+chain .* W=(\d+) w=(\d+) .*R=(\d+)", line)
    if m:
        k = (m.group(2), m.group(4)); tot[k] = tot.get(k, 0) + float(m.group(1))
print(f"R={r} wpx={wpx} nw={__import__('os').environ.get('VOXEMB_CHAIN_NW')}: step {d['ms_per_step']} ms value {d['value']} chain(W,R)->us {tot}")
PY
done

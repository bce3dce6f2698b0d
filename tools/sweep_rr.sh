#!/bin/bash
# A/B sweep of conv1x1_rr tile configs (one bench per config), summary of rr op times
for cfg in "4 4" "4 2" "2 4" "2 2" "1 4" "1 2"; do
  set -- $cfg
  VOXEMB_RR_WPX=$1 VOXEMB_RR_WCO=$2 timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --dump-ops > gpurun_out/rr_$1_$2.json 2> gpurun_out/rr_$1_$2.ops || exit $?
  python - "$1" "$2" <<'PY'
import json, sys, re
wpx, wco = sys.argv[1:3]
d = json.load(open(f"gpurun_out/rr_{wpx}_{wco}.json"))
tot = 0.0
for line in open(f"gpurun_out/rr_{wpx}_{wco}.ops"):
    m = re.match(r"\s*([\d.]+) us\s+rr ", line)
    if m: tot += float(m.group(1))
print(f"wpx={wpx} wco={wco}: step {d['ms_per_step']} ms, rr total {tot/1e3:.3f} ms, value {d['value']}")
PY
done

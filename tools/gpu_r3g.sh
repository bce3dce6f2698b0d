#!/bin/bash
# full -m gpu suite + smoke + headline bench, then the DPN68 / TDNN benches with
# per-op dumps (each step time-limited, chained so a failure ends the call)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-g}
bash tools/gpu_suite.sh || exit $?
timeout -k 10 300 python3 bench.py --model dpn68 --frames 600 --batch 64 --steps 10 --warmup 3 \
  --no-cpu-baseline --dump-ops > gpurun_out/${TAG}_dpn68.json 2> gpurun_out/${TAG}_dpn68_ops.txt || { echo "dpn68 rc=$?"; exit 1; }
timeout -k 10 300 python3 bench.py --model tdnn --batch 64 --no-cpu-baseline --dump-ops \
  > gpurun_out/${TAG}_tdnn.json 2> gpurun_out/${TAG}_tdnn_ops.txt || { echo "tdnn rc=$?"; exit 1; }
for f in dpn68 tdnn; do
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_$f.json')); print('$f', d['value'], d['ms_per_step'], d['conv_stack']['frac'])"
done

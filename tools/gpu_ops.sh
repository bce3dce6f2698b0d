#!/bin/bash
# per-op timing of the headline plan (+ optional extra bench args)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --dump-ops "$@" > gpurun_out/ops.json 2> gpurun_out/ops.txt
echo "bench rc=$?"

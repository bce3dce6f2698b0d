#!/bin/bash
# per-op timing of the side configurations (C2 TDNN, C5 DPN68 80x600)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --model tdnn --batch 64 --steps 20 --warmup 5 --no-cpu-baseline --dump-ops > gpurun_out/tdnn_ops.json 2> gpurun_out/tdnn_ops.txt || exit 1
timeout -k 10 300 python3 bench.py --model dpn68 --frames 600 --batch 64 --steps 5 --warmup 2 --no-cpu-baseline --dump-ops > gpurun_out/dpn_ops.json 2> gpurun_out/dpn_ops.txt || exit 1
echo ok

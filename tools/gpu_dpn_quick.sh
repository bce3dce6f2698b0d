#!/bin/bash
# DPN68 kernels: gconv unit tests + DPN GPU tests, then the C5 bench with per-op dump
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-dq}
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
  -k "${TESTK:-gconv or dpn}" > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python3 bench.py --model dpn68 --frames 600 --batch 64 --steps 10 --warmup 3 \
  --no-cpu-baseline --dump-ops > gpurun_out/${TAG}_dpn68.json 2> gpurun_out/${TAG}_dpn68_ops.txt || { echo "dpn68 rc=$?"; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_dpn68.json')); print('dpn68', d['value'], d['ms_per_step'], d['conv_stack']['frac'])"

#!/bin/bash
# DPN68 parity tests + C5 bench with the per-op dump
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-dpn}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_bf16_oracle.py -q -x \
  --timeout 300 --timeout-method thread -k "${TESTK:-dpn or nw or prologue}" > gpurun_out/${TAG}_tests.log 2>&1 \
  || { echo "tests rc=$?"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python3 bench.py --model dpn68 --frames 600 --batch 64 --steps 10 --warmup 3 \
  --no-cpu-baseline --dump-ops > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_ops.txt \
  || { echo "bench rc=$?"; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print(d['value'], d['ms_per_step'])"

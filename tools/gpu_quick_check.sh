#!/bin/bash
# selected GPU tests (TESTK) + two headline benches with the per-op dump
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-q}
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
  -k "${TESTK}" > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --dump-ops \
    > gpurun_out/${TAG}_bench$i.json 2> gpurun_out/${TAG}_ops$i.txt || { echo "bench rc=$?"; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench$i.json')); print(d['value'], d['ms_per_step'])"
done

#!/bin/bash
# full -m gpu suite + smoke + one bench line (per-op dump), each step time-limited
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-suite}
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=${MAXFAIL:-1} --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke rc=$?"; exit 1; }
echo "smoke ok"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --dump-ops \
  > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_ops.txt || { echo "bench rc=$?"; exit 1; }
cat gpurun_out/${TAG}_bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"

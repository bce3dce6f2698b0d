#!/bin/bash
# selected GPU tests (TESTK) + TDNN / DPN68 / headline benches with per-op dumps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-sq}
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
  -k "${TESTK}" > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python3 bench.py --model tdnn --batch 64 --no-cpu-baseline --dump-ops \
  > gpurun_out/${TAG}_tdnn.json 2> gpurun_out/${TAG}_tdnn_ops.txt || { echo "tdnn rc=$?"; exit 1; }
timeout -k 10 300 python3 bench.py --model dpn68 --frames 600 --batch 64 --steps 10 --warmup 3 \
  --no-cpu-baseline --dump-ops > gpurun_out/${TAG}_dpn68.json 2> gpurun_out/${TAG}_dpn68_ops.txt || { echo "dpn68 rc=$?"; exit 1; }
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --dump-ops \
  > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_ops.txt || { echo "bench rc=$?"; exit 1; }
for f in tdnn dpn68 bench; do
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_$f.json')); print('$f', d['value'], d['ms_per_step'], d['conv_stack']['frac'])"
done

#!/bin/bash
# GPU check for one change: selected -m gpu tests (TESTK, all when empty), then the
# headline bench with the per-op dump.  Every step time-limited; stops at the first
# failure.  Outputs under gpurun_out/$TAG*.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-chk}
if [ -n "${TESTK+x}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    ${TESTK:+-k "$TESTK"} > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -2 gpurun_out/${TAG}_tests.log
fi
for i in $(seq 1 ${NBENCH:-1}); do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --dump-ops ${BENCH_ARGS} \
    > gpurun_out/${TAG}_bench$i.json 2> gpurun_out/${TAG}_ops$i.txt || { echo "bench rc=$?"; tail -5 gpurun_out/${TAG}_ops$i.txt; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench$i.json')); print('bench', d['value'], d['ms_per_step'])"
done
if [ -n "$EXTRA" ]; then bash -c "$EXTRA" || { echo "extra rc=$?"; exit 1; }; fi

#!/bin/bash
# One GPU session of round artefacts: bench JSON, rocprofv3 kernel stats,
# PMC counter passes (incl. FETCH_SIZE / WRITE_SIZE), AS-norm timing.
# Outputs under gpurun_out/round/; copy the summaries into profiles/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/round
mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run -f csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/stats.log 2>&1 || exit $?
bash tools/pmc_chain.sh || exit $?
timeout -k 10 300 python3 tools/bench_asnorm.py > $O/asnorm.json 2> $O/asnorm.err || exit $?

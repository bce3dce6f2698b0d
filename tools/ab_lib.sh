#!/bin/bash
# A/B of one kernel change on the headline bench, one box: the product library
# (new code) against libvoxemb_old.so (the product objects with the changed
# source's object from before the change), alternating, twice each; compare the
# per-op dump (--dump-ops) of the changed kernel.  TESTS (a pytest -k
# expression) run first on the new library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${TAG:-ab}
P=$PWD/voxsrc2020_speaker_verification_amd
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -q -m gpu -k "$TESTS" --timeout 200 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
fi
run() { local name=$1 lib=$2
  VOXEMB_LIB=$lib timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --dump-ops ${BENCH_ARGS} \
    > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_${name}_ops.txt || { echo "$name rc=$?"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_$name.json')); print('$name', d['value'], d['ms_per_step'])"; }
run old0 $P/libvoxemb_old.so && run new0 $P/libvoxemb.so && run old1 $P/libvoxemb_old.so && run new1 $P/libvoxemb.so

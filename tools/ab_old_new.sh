#!/bin/bash
# A/B of a kernel change on the headline bench, one box: the product library
# (new code) against the diagnostic library built before the change (old code;
# compare the per-op dump of the changed kernel only -- the diagnostic build's
# other kernels carry switch reads of their own), alternating, twice each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
D=$PWD/voxsrc2020_speaker_verification_amd/libvoxemb_diag.so
TAG=${TAG:-on}
run() { local name=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --dump-ops ${BENCH_ARGS} \
    > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_${name}_ops.txt || { echo "$name rc=$?"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_$name.json')); print('$name', d['value'], d['ms_per_step'])"; }
run old0 VOXEMB_LIB=$D && run new0 X=1 && run old1 VOXEMB_LIB=$D && run new1 X=1

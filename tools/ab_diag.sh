#!/bin/bash
# A/B of diagnostic-build switches on the headline bench, one box: for each
# "NAME=ENV ..." argument one bench run with the per-op dump; a control run
# (diagnostic build, no switch) first and last.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
D=$PWD/voxsrc2020_speaker_verification_amd/libvoxemb_diag.so
TAG=${TAG:-ab}
run() {
  local name=$1; shift
  env VOXEMB_LIB=$D "$@" timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --dump-ops ${BENCH_ARGS} \
    > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_${name}_ops.txt || { echo "$name rc=$?"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_$name.json')); print('$name', d['value'], d['ms_per_step'])"
}
run ctl0
for spec in "$@"; do
  name=${spec%%=*}; envs=${spec#*=}
  run $name $envs
done
run ctl1

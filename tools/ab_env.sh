#!/bin/bash
# A/B of plan/env switches on the headline bench with the product library, one
# box: for each "NAME=ENV ..." argument one bench run with the per-op dump; a
# control run (no switch) first and last.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-abe}
run() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --dump-ops ${BENCH_ARGS} \
    > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_${name}_ops.txt || { echo "$name rc=$?"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_$name.json')); print('$name', d['value'], d['ms_per_step'])"
}
run ctl0 X=0
for spec in "$@"; do
  name=${spec%%=*}; envs=${spec#*=}
  run $name $envs
done
run ctl1 X=0

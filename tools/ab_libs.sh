#!/bin/bash
# A/B of several library builds on one box: LIBS="name ..." names
# voxsrc2020_speaker_verification_amd/libvoxemb_<name>.so ("cur" = libvoxemb.so); each
# runs the headline bench (BENCH_ARGS appended) with --dump-ops, ROUNDS times in
# alternation; prints utt/s and the summed per-op time of OPS (an awk regex on
# the --dump-ops lines, e.g. "conv3ks").
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-abl}; ROUNDS=${ROUNDS:-2}; OPS=${OPS:-conv3ks}
mkdir -p gpurun_out/$TAG
P=$PWD/voxsrc2020_speaker_verification_amd
for r in $(seq 1 $ROUNDS); do
  for name in $LIBS; do
    lib=$P/libvoxemb_$name.so; [ "$name" = cur ] && lib=$P/libvoxemb.so
    out=gpurun_out/$TAG/${name}_$r
    VOXEMB_LIB=$lib timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --dump-ops ${BENCH_ARGS} \
      > $out.json 2> ${out}_ops.txt || { echo "$name rc=$?"; exit 1; }
    ops=$(awk -v re="$OPS" '$0 ~ re {s+=$1; n++} END {printf "%d ops %.1f us", n, s}' ${out}_ops.txt)
    python3 -c "import json; d=json.load(open('$out.json')); print('$name', $r, d['value'], d['ms_per_step'], '$ops')"
  done
done

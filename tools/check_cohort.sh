# cohort assembly at VoxCeleb2-dev scale on the box (tools/bench_cohort.py), world 1 over RCCL
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/${TAG:-cohort}
timeout -k 10 300 python3 -u tools/bench_cohort.py ${COHORT_ARGS:---old} > gpurun_out/${TAG:-cohort}/cohort.json 2> gpurun_out/${TAG:-cohort}/cohort.err || { echo "cohort rc=$?"; tail -5 gpurun_out/${TAG:-cohort}/cohort.err; exit 1; }
tail -1 gpurun_out/${TAG:-cohort}/cohort.json

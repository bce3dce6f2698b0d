# One-box A/B of plan switches with a test gate first:
#   TAG=x K="pytest -k expr" bash tools/gpu_ab.sh name=ENV=val ...   (see ab_env.sh)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/${TAG:-gab}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "$K" --timeout 300 --timeout-method thread > gpurun_out/${TAG:-gab}/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${TAG:-gab}/tests.log; exit 1; }
  tail -3 gpurun_out/${TAG:-gab}/tests.log
fi
TAG=${TAG:-gab}/ab bash tools/ab_env.sh "$@" || exit 1
O=gpurun_out/${TAG:-gab}
python3 tools/ops_compare.py $O/ab_ctl0_ops.txt $(for s in "$@"; do echo $O/ab_${s%%=*}_ops.txt; done) $O/ab_ctl1_ops.txt
echo done

# Quick GPU check: selected -m gpu tests (K = pytest -k expression), then
# optional extra commands in EXTRA (each under its own time limit).
#   TAG=r05a K="pool_prologue or resident" EXTRA="python tools/shape_sweep.py" bash tools/gpu_quick.sh
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-quick}; mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 ${TT:-600} python -u -m pytest tests -m gpu -x -v -k "$K" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
fi
if [ -n "$EXTRA" ]; then
  timeout -k 10 ${ET:-300} bash -c "$EXTRA" > $O/extra.log 2>&1 || { echo "extra rc=$?"; tail -30 $O/extra.log; exit 1; }
  tail -40 $O/extra.log
fi
echo done

set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/rag
timeout -k 10 600 python -u -m pytest tests/test_ragged.py -x -v --timeout 300 --timeout-method thread > gpurun_out/rag/tests.log 2>&1; rc=$?
tail -30 gpurun_out/rag/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/rag/bench.json 2> gpurun_out/rag/bench.err || { tail -5 gpurun_out/rag/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/rag/bench.json')); print('bench', d['value'], d['ms_per_step'])"

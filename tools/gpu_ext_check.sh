# ragged-batch extraction: GPU tests of the streaming path, then bench_extract in both modes
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-ext}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ragged.py tests/test_gpu_parity.py -k "ragged or stream" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 python3 -u tools/bench_extract.py --utts 4096 --lanes ${LANES:-1,2,4} --mode ragged --out $O/extract_ragged.json > $O/extract_ragged.log 2>&1 || { tail -20 $O/extract_ragged.log; exit 1; }
tail -1 $O/extract_ragged.log | cut -c1-1500
timeout -k 10 900 python3 -u tools/bench_extract.py --utts 4096 --lanes 1,4 --mode exact --out $O/extract_exact.json > $O/extract_exact.log 2>&1 || { tail -20 $O/extract_exact.log; exit 1; }
tail -1 $O/extract_exact.log | cut -c1-1500

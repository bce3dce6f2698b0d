# lane pipeline change: stream/extract GPU tests, then TDNN + res2net ragged extraction
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-lane}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "stream or extract or ragged or dp_" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 python3 -u tools/bench_extract.py --model tdnn --utts 4096 --lanes 1,4 --mode ragged --out $O/extract_ragged_tdnn.json > $O/extract_tdnn.log 2>&1 || { tail -20 $O/extract_tdnn.log; exit 1; }
timeout -k 10 900 python3 -u tools/bench_extract.py --utts 4096 --lanes 1 --mode ragged --out $O/extract_ragged_r2n.json > $O/extract_r2n.log 2>&1 || { tail -20 $O/extract_r2n.log; exit 1; }
python3 -c "
import json
for m in ('tdnn', 'r2n'):
    d=json.load(open('$O/extract_ragged_%s.json' % m))
    print(m, d['fixed_shape_frames_per_s'], [(r['utts'], r['lanes'], r['frames_per_s'], r['frac_of_fixed_shape']) for r in d['runs']])"
python3 -c "
import json
for m in ('tdnn', 'r2n'):
    d=json.load(open('$O/extract_ragged_%s.json' % m))
    for r in d['runs']: print(m, r['utts'], r['lanes'], r['frames_per_s'], r['warm_frames_per_s'], r['lane_phase_s'], r['warm_lane_phase_s'], r['plans_built'])"

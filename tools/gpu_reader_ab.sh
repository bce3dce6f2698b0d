# host reader A/B (thread pool) + TDNN ragged extraction, one box
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-reader}; mkdir -p $O
LIBS="${LIBS:-cur}" timeout -k 10 600 python3 -u tools/bench_reader.py --utts 2048 --threads 1,4,8,16 --out $O/reader.json > $O/reader.log 2>&1 || { tail -20 $O/reader.log; exit 1; }
cat $O/reader.log
timeout -k 10 900 python3 -u tools/bench_extract.py --model tdnn --utts 4096 --lanes 1,4 --mode ragged --out $O/extract_ragged_tdnn.json > $O/extract_tdnn.log 2>&1 || { tail -20 $O/extract_tdnn.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/extract_ragged_tdnn.json'))
print('tdnn', d['fixed_shape_frames_per_s'], [(r['lanes'], r['frames_per_s'], r['frac_of_fixed_shape']) for r in d['runs']])"

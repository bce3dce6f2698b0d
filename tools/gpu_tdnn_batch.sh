# TDNN extraction vs chunk batch size (1 lane, ragged, host and device reader)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-tdnnb}; mkdir -p $O
for b in 64 256 512; do for r in host device; do
timeout -k 10 900 python3 -u tools/bench_extract.py --model tdnn --utts 4096 --lanes 1 --batch $b --mode ragged --reader $r --out $O/b${b}_$r.json > $O/b${b}_$r.log 2>&1 || { tail -20 $O/b${b}_$r.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/b${b}_$r.json'))
for x in d['runs']: print($b, '$r', x['utts'], x['frames_per_s'], x['warm_frames_per_s'], x['warm_lane_phase_s'])"
done; done

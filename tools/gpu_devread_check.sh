# device reader: its GPU tests, then TDNN / res2net extraction with the host and the device reader
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-devread}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_device_reader.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "device or stream or extract" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for m in tdnn res2net50_w24_s4_c32; do for r in host device; do
timeout -k 10 900 python3 -u tools/bench_extract.py --model $m --utts 4096 --lanes 1 --mode ragged --reader $r --out $O/ext_${m}_$r.json > $O/ext_${m}_$r.log 2>&1 || { tail -20 $O/ext_${m}_$r.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ext_${m}_$r.json'))
for x in d['runs']: print('$m', '$r', x['reader'], x['utts'], x['lanes'], x['frames_per_s'], x['warm_frames_per_s'], x['warm_lane_phase_s'])"
done; done

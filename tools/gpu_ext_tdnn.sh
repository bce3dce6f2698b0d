# ragged vs equal-length extraction for the TDNN (C1/C2 model), one box
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-ext_tdnn}; mkdir -p $O
timeout -k 10 900 python3 -u tools/bench_extract.py --model tdnn --utts 4096 --lanes 1,4 --mode ragged --out $O/extract_ragged.json > $O/extract_ragged.log 2>&1 || { tail -20 $O/extract_ragged.log; exit 1; }
timeout -k 10 900 python3 -u tools/bench_extract.py --model tdnn --utts 4096 --lanes 1,4 --mode exact --out $O/extract_exact.json > $O/extract_exact.log 2>&1 || { tail -20 $O/extract_exact.log; exit 1; }
python3 - <<'PY'
import json
for m in ("ragged", "exact"):
    d = json.load(open(f"gpurun_out/ext_tdnn/extract_{m}.json"))
    print(m, d["fixed_shape_frames_per_s"], [(r["utts"], r["lanes"], r["frames_per_s"], r["frac_of_fixed_shape"], r["plans_built"], r["plan_hits"]) for r in d["runs"]])
PY

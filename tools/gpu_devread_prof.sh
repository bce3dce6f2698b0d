# kernel times of the device reader (rocprofv3 over one extraction child)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-devprof}; mkdir -p $O
timeout -k 10 600 python3 -u tools/bench_extract.py --model ${MODEL:-tdnn} --utts 4096 --lanes 1 --mode ragged --reader device --out $O/ext.json > $O/ext.log 2>&1 || { tail -20 $O/ext.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -f csv -- python3 tools/bench_extract.py --child --scp /tmp/voxemb_bench_extract/feats4096.scp --wspec /tmp/xv_prof --lanes 1 --batch 64 --model ${MODEL:-tdnn} --mode ragged --reader device > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 - <<PY
import csv, glob
f = glob.glob("$O/prof/**/run_kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:90]}')
PY

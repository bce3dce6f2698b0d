set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/${TAG:-r04c}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG:-r04c}/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/${TAG:-r04c}/tests.log; exit 1; }
tail -1 gpurun_out/${TAG:-r04c}/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG:-r04c}/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/${TAG:-r04c}/smoke.log; exit 1; }
tail -3 gpurun_out/${TAG:-r04c}/smoke.log
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG:-r04c}/bench.json 2> gpurun_out/${TAG:-r04c}/bench.err || { echo "bench rc=$?"; tail -5 gpurun_out/${TAG:-r04c}/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG:-r04c}/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['conv_stack']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG:-r04c}/stats -o run -f csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG:-r04c}/stats.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
echo done

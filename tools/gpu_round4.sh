# GPU session: full GPU suite, headline bench x4 (fault check), rocprofv3 kernel stats
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "t_gpu::700::python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bench1::300::python bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err" \
 "bench2::300::python bench.py --no-cpu-baseline > gpurun_out/bench2.json 2> gpurun_out/bench2.err" \
 "bench3::300::python bench.py --no-cpu-baseline > gpurun_out/bench3.json 2> gpurun_out/bench3.err" \
 "prof::300::rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --steps 10 > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err"

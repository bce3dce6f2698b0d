# GPU session: bitwise/parity tests first, then the bench (+ per-op timing)
# and a rocprofv3 kernel-stats pass of the same command
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "t_pipe::300::python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread -k 'conv3 or gemm_pipe or fused_kernels'" \
 "t_gpu::600::python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bench::400::python bench.py --dump-ops > gpurun_out/bench.json 2> gpurun_out/bench.err" \
 "stats::300::rocprofv3 --kernel-trace --stats -d gpurun_out/stats -o run -f csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline"

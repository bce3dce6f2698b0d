# GPU session: prologue-GEMM bitwise test, full GPU suite, DPN68 C5 and headline benches
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "t_pro::300::python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread -k 'prologue or dpn68'" \
 "t_gpu::600::python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bench_dpn::400::python bench.py --model dpn68 --frames 600 --batch 64 --steps 10 --warmup 3 --no-cpu-baseline --dump-ops > gpurun_out/bench_dpn68.json 2> gpurun_out/bench_dpn68.err" \
 "bench::400::python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err"

#!/bin/bash
# one-step residual prefetch bneck (with the unconsumed-set wait) + stats_pool_col:
# bneck / pool tests, then 5 bench runs with per-op timing; stop at the first failure
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_bneck_unit.py "tests/test_gpu_parity.py::test_stats_pool_kernel" "tests/test_gpu_parity.py::test_fused_kernels_bitwise_equal_unfused" "tests/test_gpu_parity.py::test_bneck_segments_bitwise" "tests/test_bf16_oracle.py::test_bf16_layers_match_oracle" -q --timeout 300 --timeout-method thread > gpurun_out/r3b_tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
echo "tests ok"
for i in 1 2 3 4 5; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --dump-ops > gpurun_out/r3b_bench$i.json 2> gpurun_out/r3b_ops$i.txt || { echo "bench $i rc=$?"; exit 1; }
done
echo "bench ok"

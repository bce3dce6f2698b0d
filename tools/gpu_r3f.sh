#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "tests/test_gpu_parity.py::test_conv3_s2r_bitwise_pipe" "tests/test_gpu_parity.py::test_fused_kernels_bitwise_equal_unfused" "tests/test_bf16_oracle.py::test_bf16_layers_match_oracle" -q -x --timeout 300 --timeout-method thread -k "s2r or res2net50_w24" > gpurun_out/r3f_tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
echo "tests ok"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --dump-ops > gpurun_out/r3f_bench.json 2> gpurun_out/r3f_ops.txt || exit 1
echo ok

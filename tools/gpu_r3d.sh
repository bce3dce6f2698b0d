#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "tests/test_gpu_parity.py::test_gemm_ws_prologue_bitwise" "tests/test_gpu_parity.py::test_gemm_ws_taps_bitwise" "tests/test_gpu_parity.py::test_stats_pool_kernel" "tests/test_bf16_oracle.py::test_bf16_layers_match_oracle" "tests/test_gpu_parity.py::test_forward_matches_oracle" -q --timeout 300 --timeout-method thread > gpurun_out/r3d_tests.log 2>&1
echo "tests rc=$?"
timeout -k 10 300 python3 bench.py --model dpn68 --frames 600 --batch 64 --steps 5 --warmup 2 --no-cpu-baseline --dump-ops > gpurun_out/dpn_ops.json 2> gpurun_out/dpn_ops.txt || exit 1
VOXEMB_PRO_MIN_COUT=128 timeout -k 10 300 python3 bench.py --model dpn68 --frames 600 --batch 64 --steps 5 --warmup 2 --no-cpu-baseline --dump-ops > gpurun_out/dpn128_ops.json 2> gpurun_out/dpn128_ops.txt || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --dump-ops > gpurun_out/r3d_bench.json 2> gpurun_out/r3d_ops.txt || exit 1
echo ok

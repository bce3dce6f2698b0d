#!/bin/bash
# round 3: bf16 oracle layer tests + graph rebuild race test
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_bf16_oracle.py "tests/test_gpu_parity.py::test_run_device_new_buffers_without_sync" -v -s --timeout 400 --timeout-method thread > gpurun_out/r3a_tests.log 2>&1
echo "pytest rc=$?"

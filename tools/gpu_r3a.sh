#!/bin/bash
# round 3: bf16 oracle layer tests + graph rebuild race test, then the whole GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_bf16_oracle.py "tests/test_gpu_parity.py::test_run_device_new_buffers_without_sync" tests/test_bneck_unit.py -v -s --timeout 400 --timeout-method thread > gpurun_out/r3a_tests.log 2>&1
rc=$?
echo "new tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --deselect tests/test_bf16_oracle.py > gpurun_out/r3a_suite.log 2>&1
echo "suite rc=$?"

#!/bin/bash
# FETCH_SIZE calibration per access shape (tools/ubench/fetch_calib.hip): one
# rocprofv3 pass per kernel; prints the raw FETCH_SIZE (KB) of the 2nd dispatch
# against the 1 GiB each kernel reads.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fetch_calib
mkdir -p $O
for k in ${KERNELS:-lds16 lds64 reg16 reg8 dupx dupy}; do
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/$k -o run -f csv -- ./tools/ubench/fetch_calib $k > $O/$k.log 2>&1 || exit $?
  f=$(find $O/$k -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$k" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Counter_Name"] == "FETCH_SIZE"]
v = float(rows[-1]["Counter_Value"]) * 1024
print(f"{sys.argv[2]}: FETCH_SIZE {v/2**30:.3f} GiB for 1 GiB read -> correction x{2**30/v:.2f}")
PY
done

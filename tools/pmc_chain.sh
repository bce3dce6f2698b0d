#!/bin/bash
# PMC counters of one bench configuration, one rocprofv3 pass per counter set
# (--pmc only with --kernel-trace).  usage: OUT=dir BENCH_ARGS="..." tools/pmc_chain.sh
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}
mkdir -p $OUT
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
SETS=${PMC_SETS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS|SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES|SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY|FETCH_SIZE|WRITE_SIZE|SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"}
IFS='|' read -ra SETARR <<< "$SETS"
for set in "${SETARR[@]}"; do
  tag=$(echo $set | cut -d' ' -f1)
  [ "$tag" = "SQ_VALU_MFMA_BUSY_CYCLES" ] && tag=MFMA_BUSY
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $set -d $OUT/$tag -o run -f csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $OUT/$tag.log 2>&1 || exit $?
done

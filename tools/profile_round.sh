#!/bin/bash
# Round artefacts: headline bench (with the CPU baseline) + fp32 line, rocprofv3
# kernel stats, PMC passes (HBM bytes, MFMA busy), AS-norm timing, side-config
# benches + their PMC.  Outputs under $O (default gpurun_out/round); summaries go to profiles/.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/round}
mkdir -p $O
# (the first import on a fresh box pages the image in: print as it lands)
timeout -k 10 300 python3 -c "import torch; print('torch', torch.__version__, flush=True)" || exit $?
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python3 bench.py --precision fp32 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_fp32.json 2> $O/bench_fp32.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run -f csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/stats.log 2>&1 || exit $?
OUT=$O/pmc bash tools/pmc_chain.sh || exit $?
timeout -k 10 300 python3 tools/bench_asnorm.py > $O/asnorm.json 2> $O/asnorm.err || exit $?
timeout -k 10 300 python3 bench.py --model tdnn --batch 64 --no-cpu-baseline > $O/bench_tdnn.json 2> $O/bench_tdnn.err || exit $?
timeout -k 10 300 python3 bench.py --model dpn68 --frames 600 --batch 64 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_dpn68.json 2> $O/bench_dpn68.err || exit $?
timeout -k 10 300 python3 bench.py --model res2net101_w24_s4_c32_att --no-cpu-baseline > $O/bench_r101att.json 2> $O/bench_r101att.err || exit $?
PMC_SETS="FETCH_SIZE|WRITE_SIZE|SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" OUT=$O/pmc_tdnn BENCH_ARGS="--model tdnn --batch 64" bash tools/pmc_chain.sh || exit $?
PMC_SETS="FETCH_SIZE|WRITE_SIZE|SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" OUT=$O/pmc_dpn68 BENCH_ARGS="--model dpn68 --frames 600 --batch 64" bash tools/pmc_chain.sh || exit $?
echo done

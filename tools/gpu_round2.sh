# second GPU session of the round: PMC passes over the headline bench (HBM
# bytes per kernel for roofline.traffic), then the other BASELINE configs
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "pmc::900::bash tools/pmc_chain.sh" \
 "bench_dpn::400::python bench.py --model dpn68 --frames 600 --batch 64 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_dpn68.json" \
 "bench_tdnn::300::python bench.py --model tdnn --frames 200 --batch 64 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_tdnn.json" \
 "bench_att::300::python bench.py --model res2net101_w24_s4_c32_att --batch 128 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_r101att.json"

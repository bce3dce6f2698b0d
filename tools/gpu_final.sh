# Round artefacts at the final state: headline bench + rocprofv3 stats + PMC passes +
# AS-norm (tools/profile_round.sh), then the side-configuration benches
export TMPDIR=/tmp
bash tools/profile_round.sh || exit $?
O=gpurun_out/round
timeout -k 10 300 python3 bench.py --model tdnn --batch 64 --no-cpu-baseline > $O/bench_tdnn.json 2> $O/bench_tdnn.err || exit $?
timeout -k 10 300 python3 bench.py --model dpn68 --frames 600 --batch 64 --no-cpu-baseline > $O/bench_dpn68.json 2> $O/bench_dpn68.err || exit $?
timeout -k 10 300 python3 bench.py --model res2net101_w24_s4_c32_att --no-cpu-baseline > $O/bench_r101att.json 2> $O/bench_r101att.err || exit $?

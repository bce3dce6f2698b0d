# per-CU intake model check: the 1x1 group with 128-pixel tiles (diag VOXEMB_GEMM_VAR=37)
# against the product's 192/256-pixel tiles, diagnostic build, alternating
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TAG=bm bash tools/ab_diag.sh "bm128=VOXEMB_GEMM_VAR=37" "ws=VOXEMB_GEMM_VAR=1" "bm128b=VOXEMB_GEMM_VAR=37" || exit 1
for n in ctl0 bm128 ws bm128b ctl1; do
  awk -v n=$n '/gemmwide/ {s+=$1; c++} END {printf "%s gemmwide %d ops %.1f us\n", n, c, s}' gpurun_out/bm_${n}_ops.txt
done

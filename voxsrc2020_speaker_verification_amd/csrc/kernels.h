// Internal kernel interface of libvoxemb (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Diagnostic variants (parts of a kernel skipped for timing; wrong results) are
// compiled only into the VOX_DIAG build (build_native.py --diag ->
// libvoxemb_diag.so); in the product library VOX_DBG(q) is a constant 0 and
// those paths do not exist.
#ifdef VOX_DIAG
#define VOX_DBG(q) ((q).dbg)
#else
#define VOX_DBG(q) 0
#endif

namespace vox {

enum DType { F32 = 0, BF16 = 1 };

// Epilogue flags, applied in this order:
//   PRE_RELU  v = max(v,0)                (TDNN conv->ReLU->BN, tdnn_model.py:24-30)
//   AFFINE    v = (v - mean[c]) * inv[c]  (inference BN, models.py:62-67)
//   RES       v += res[p][c]              (residual, res2net_model.py:100), only c < ysplit
//   RELU      v = max(v,0)
//   PARTIAL   raw accumulator -> split-K slab (no other flag applies)
// EPI_BN2D: TF1's non-fused inference BN of the 2-D head (tf.nn.batch_normalization,
// what tf.compat.v1.layers picks for a 2-D input): x * inv + (-mean * inv), the
// `mean` table holding -mean * inv (bn2d below); EPI_AFFINE is the fused form
// (x - mean) * inv of the 4-D BNs
enum EpiFlags { EPI_PRE_RELU = 1, EPI_AFFINE = 2, EPI_RES = 4, EPI_RELU = 8, EPI_PARTIAL = 16,
                EPI_BN2D = 32 };

// NHWC implicit-GEMM convolution, C[cout][pixel] = W[cout][k] * im2col[k][pixel].
struct ConvParams {
  const void* x;  int ldx;                 // input, channel stride (elements)
  const void* x2; int ldx2;                // optional addend of identical geometry
  const float* in_mean; const float* in_inv;  // optional prologue relu((x-m)*inv)
  const void* w;  int kp;                  // weights [coutp][kp]
  void* y;  int ldy;                       // output (channel offset pre-applied)
  void* y2; int ldy2; int ysplit;          // channels >= ysplit go to y2[c - ysplit]
  const void* res; int ldr;                // residual
  const float* mean; const float* inv;     // epilogue BN
  float* partial;                          // split-K slabs [z][M][coutp]
  int N, H, W, Cin, Ho, Wo, Cout, coutp;
  int kh, kw, sh, sw, dh, dw, ph, pw;
  int cinp;                                // per-tap padded Cin (vector path)
  int kchunk;                              // split-K Cin range per blockIdx.z
  int flags;
  int fast4;                               // 4-channel vector epilogue allowed
  int groups;                              // grouped conv (Cin/Cout are per group)
  int cblocks;                             // cout blocks per group (gridDim.y = groups*cblocks)
  // window-staged kernel (conv_win) geometry, see launch_conv_win
  int win_lo, win_len, win_kc, win_astr, win_wstr, win_lds;
  // gemm1x1_ws: paired-row bf16 weights re-blocked as [rows/16][kp/32][1 KB], each
  // 1-KB block one DMA piece in LDS order (swizzle applied), or null
  const void* wblk;
  // gemm1x1_ws at any tile count (the plan fixes the route per model, not per
  // batch: the TDNN's bits must not depend on how many utterances share a batch)
  int any_m;
  // ragged batches: per-utterance frame counts (device) and this layer's
  // downsampling shift (device_common.h valid_rows); null = every row valid
  const int* vlen; int vsh;
};

struct ConvLaunch {
  int wco, wpx;       // 16-row cout tiles / 16-pixel tiles per wave
  int vec;            // 1: vector (tap-major, Cin % VEC == 0) path
  int splitk;         // blockIdx.z count
};

// Returns hipSuccess or the launch error.
hipError_t launch_conv(DType t, const ConvParams& p, const ConvLaunch& l, hipStream_t s);
// Fused Res2Net split-scale chain (stride 1, res2net_model.py:53-75):
//   y_0 = relu(bn_0(conv_0(x_0))), y_k = relu(bn_k(conv_k(x_k + y_{k-1})))
// for k < nst = split-1, x_k = a[:, k*w:(k+1)*w], y_k -> b[:, k*w:(k+1)*w].
struct ChainParams {
  const void* a; int lda;
  void* b; int ldb;
  const void* wt[8];                // per stage [coutp][9*w] bf16
  const float* mean[8];
  const float* inv[8];
  int N, H, W, w, nst, R, coutp;
  int astr, wstr, kcp, buf_bytes, lds;
  int nwaves;                       // 4 or 8 waves per block
  // s2_fused only: the block input and its 1x1a (paired-row weights + BN)
  const void* x; int ldx; int cin;
  const void* wa; const float* ma; const float* ia;
  int dbg;                          // diagnostics (VOXEMB_BNECK_DBG): skip parts, garbage out
                                    // (read only in VOX_DIAG builds, see VOX_DBG)
  const int* vlen; int vsh;         // ragged batches (ConvParams::vlen); vsh of the input rows
};
hipError_t launch_split_chain(const ChainParams& q, int wco, int wpx, hipStream_t s);
// Row-streamed split chain (bneck.hip): utterance segments of q.R rows, q.nwaves
// segments per utterance (grid N * q.nwaves); LDS bytes or -1 if no instance.
int chain_rows_lds(int w, int split, int W);
hipError_t launch_chain_rows(const ChainParams& q, hipStream_t s);
// Identity-block front half (bneck.hip): 1x1a + BN + ReLU of q.x (q.cin
// channels, weights q.wa) feeding chain_rows' stages in the same launch; x_S
// is written to q.b at channel (S-1)*w.  LDS bytes or -1.
int chain_fused_lds(int cin, int wid, int split, int W);
// diagnostics: bneck_fused's per-step clock stamps of block 0 (VOXEMB_BNECK_DBG & 256)
hipError_t bneck_trace_read(void* dst, size_t bytes);
hipError_t ks_trace_read(void* dst, size_t bytes);   // conv3x3_ks stamps (diagnostic build)
hipError_t launch_chain_fused(const ChainParams& q, hipStream_t s);
// Stride-2 split (bneck.hip): branches k < split-1 (3x3 s2 + BN + ReLU) and the
// last split's 3x3/2 average pool, q.R output rows per segment, q.nwaves
// segments per utterance; q.H/q.W are the INPUT dims.  LDS bytes or -1.
int split_s2_lds(int w, int split, int W);
hipError_t launch_split_s2(const ChainParams& q, hipStream_t s);
// Stride-2 block front half (bneck.hip): 1x1a + BN + ReLU on the full-res
// input q.x (q.cin channels, weights q.wa) feeding split_s2_rows' branches and
// pool in the same launch; q.H/q.W are the INPUT dims.  LDS bytes or -1.
int s2_fused_lds(int cin, int wid, int split, int W);
hipError_t launch_s2_fused(const ChainParams& q, hipStream_t s);

// Fused Res2Net bottleneck (stride 1): 1x1a + split chain + 1x1c + identity
// or 1x1-projection shortcut in one launch, intermediates in LDS ring
// buffers (bneck.hip).
// One workgroup per (utterance, segment of `seg` rows); blocks = N * nseg.
struct BneckParams {
  const void* x;                    // block input [N][H][W][Cin] bf16
  void* y;                          // block output [N][H][W][C]
  int N, H, W, seg, nseg;
  const void* wa;                   // 1x1a paired-row weights [split*w][C]
  const float* ma; const float* ia;
  const void* wb[8];                // 3x3 stage k [coutp][9*w] (tap-major)
  const float* mb[8]; const float* ib[8];
  const void* wc;                   // 1x1c paired-row weights [C][split*w]
  const float* mc; const float* ic;
  const void* wp;                   // projection shortcut [C][Cin] paired rows (Cin != C)
  const float* mp; const float* ip;
  int dbg;                          // timing experiments only: skip parts (0 = normal)
  const int* vlen; int vsh;         // ragged batches (ConvParams::vlen)
};
// LDS bytes of the instantiated shape, or -1 when (C, w, split, W) has none.
int bneck_lds(int Cin, int C, int w, int split, int W);
hipError_t launch_bneck(const BneckParams& q, int Cin, int C, int w, int split, hipStream_t s);

// Stride-1 bf16 conv with the input window staged in LDS (weights in the
// [coutp][taps*Cin] layout).
hipError_t launch_conv_win(const ConvParams& p, const ConvLaunch& l, hipStream_t s);
// bf16 1x1 conv (any stride), cinp/32 in {1,2,3,4,6,8,12,16,24,32}:
// activations register-resident, all cout tiles swept per wave.  Weights in
// the paired-row layout (see kernels.hip), Cout % 8 == 0, ysplit % 8 == 0.
// l.wco in {2,4}; l.wpx <= conv1x1_rr_max_wpx(ks); l.splitk = cout ranges.
hipError_t launch_conv1x1_rr(const ConvParams& p, const ConvLaunch& l, hipStream_t s);
int conv1x1_rr_max_wpx(int ks);
// bf16 1x1 conv as an LDS-tiled GEMM (128x128 tile, BK 64): cinp % 64 == 0,
// coutp % 128 == 0, paired-row weights, Cout/ysplit/ld multiples of 8.
hipError_t launch_gemm1x1(const ConvParams& p, hipStream_t s);
// Persistent LDS-DMA pipelined 1x1 GEMM (gemm.hip): 256-pixel x 128-cout tiles,
// one workgroup per CU.  gemm_pipe_ok: K % 64 == 0, K >= 192, coutp % 128 == 0.
int gemm_pipe_ok(const ConvParams& p);
hipError_t launch_gemm_pipe(const ConvParams& p, int num_cu, int variant, hipStream_t s);
// Register-weight 3x3 (conv3r.hip): w = 96 stride-1 branches, weights in
// registers, the input window staged once per 128-pixel tile.
int conv3_rw_ok(const ConvParams& p);
hipError_t launch_conv3_rw(const ConvParams& p, int num_cu, hipStream_t s);
// K-split register-weight 3x3 (conv3k.hip): the same branches with 32x32x16
// MFMA tiles, each wave holding half the K of a 32-cout group
int conv3_ks_ok(const ConvParams& p);
hipError_t launch_conv3_ks(const ConvParams& p, int num_cu, hipStream_t s);
// Utterance-band window 3x3 conv for the w = 192 stride-1 branches (conv3u.hip)
int conv3_utt_ok(const ConvParams& p);
hipError_t launch_conv3_utt(const ConvParams& p, int num_cu, hipStream_t s);
// Register-weight stride-2 3x3 (conv3s.hip): w = 96 branches of a stride-2
// block at 40 -> 20 columns, output tiles of 3 rows with their input window
// staged once in LDS.
int conv3_s2r_ok(const ConvParams& p);
// Narrow 1x1 GEMM with the weights resident in LDS (gemm_nw.hip): K <= 256,
// Cout <= 192 (DPN68's bn_relu_conv 1x1s), prologue / residual / ysplit as
// conv1x1_rr, persistent 8-wave workgroups streaming 64-pixel chunks.
int conv1x1_nw_ok(const ConvParams& p);
hipError_t launch_conv1x1_nw(const ConvParams& p, int num_cu, hipStream_t s);
hipError_t launch_conv3_s2r(const ConvParams& p, int num_cu, hipStream_t s);
// Wide-tile variant (gemm_wide.hip): 256 x BN tiles, BN = 256 (Cout % 256 == 0)
// or 192 (Cout % 192 == 0, no residual), K % 32 == 0, K >= 96, no prologue.
// gemm_wide_bn returns BN or 0 when it does not apply.
int gemm_wide_bn(const ConvParams& p);
int gemm_wide_bm(const ConvParams& p, int num_cu);
// ksub_on: gemm1x1_ws's 128-pixel tiles take two 32-deep k-steps per ring slot
// and barrier where they fit (bitwise the same outputs)
hipError_t launch_gemm_wide(const ConvParams& p, int num_cu, int variant, hipStream_t s, int ksub_on = 1);
// Persistent LDS-DMA pipelined 3x3 implicit GEMM (conv3.hip) for the Res2Net
// branch convs with Cin in {96, 192}: stride 1 (SAME) or 2 (fixed pad 1),
// Cout % 96 == 0, epilogue BN + ReLU; with y2 set (stride 1) it also writes
// z = bf16(res + y) to y2 (the next branch's input, in place over res).
int conv3_pipe_ok(const ConvParams& p);
hipError_t launch_conv3_pipe(const ConvParams& p, int num_cu, hipStream_t s);
// 1-input-channel 3x3 SAME stem + BN + ReLU from the fp32 features;
// wts = [9][Cout] fp32 (bf16-rounded values in bf16 mode), Cout <= 64.
hipError_t launch_stem(DType t, const float* x, int N, int H, int W, const float* wts, int Cout,
                       const float* mean, const float* inv, void* y, hipStream_t s,
                       const int* vlen = nullptr);
int conv_kstep(DType t);   // 32 (bf16) / 16 (fp32)
// Attentive statistics pooling glue (fp32): bf16 -> fp32 copy; h = tanh(h +
// b[n][w]) over [N][H][W][A]; softmax-over-time weighted mean/std (+ optional
// head BN) into the NHWC-flattened [N][W*2C] feature vector.
hipError_t launch_convert_bf16(const void* x, float* y, int64_t n, hipStream_t s);
hipError_t launch_att_bias_tanh(float* h, const float* b, int N, int H, int W, int A, hipStream_t s);
hipError_t launch_att_pool(DType t, const void* x, const float* lg, int N, int H, int W, int C,
                           float eps, const float* mean, const float* inv, float* out,
                           hipStream_t s);
int conv_vec(DType t);     // elements per 16-byte lane load: 8 / 4

// Row-streamed grouped 3x3 conv + BN/ReLU input prologue (gconv.hip), DPN
// cardinality-32 convs: group width gw in {4,8,16,32}, C % 64 == 0, stride 1
// (SAME) or 2 (TF SAME, pad-begin ph/pw in {0,1}), Wo <= 80.  Weights
// expanded to [C/16][NM][64][8] bf16 (NM = 9 for gw 32, else 5; see gconv.hip).
// Grid: N * nseg workgroups x C/64 chunks; `seg` output rows per segment.
struct GconvParams {
  const void* x; int ldx;
  const float* in_mean; const float* in_inv;   // prologue relu((x-m)*inv) or null
  const void* w;
  void* y; int ldy;
  int N, H, W, C, Ho, Wo, gw;
  int sh, ph, pw;
  int seg, nseg;
  int rs_force;   // output rows per step (0 = gconv_rs's choice; plan switch VOXEMB_GCONV_RS)
};
int gconv_ok(const GconvParams& p);
int gconv_rs(const GconvParams& p);
int gconv_lds(const GconvParams& p);
hipError_t launch_gconv(const GconvParams& p, hipStream_t s);

// Fused DPN stage-1 dual-path block (dpnblk.hip): 1x1a (cin -> 128, BN+ReLU
// prologue m1/i1) -> grouped 3x3 (gconv3x3_rows' expanded weights, gw <= 16,
// prologue m2/i2) -> 1x1c (128 -> cout <= 96, prologue m3/i3); channels < bw
// get the residual x[.., c] and go to y (in place over x allowed), the rest to
// y2[c - bw].  Stride 1, 65 <= W <= 80.  Two launches: the segment-halo rows'
// 1x1a into `halo` (dpn_block_halo_bytes), then the row-streamed block.
// from_a: x is the block's 1x1a output (cin = 128, w1/m1/i1 unused, one launch,
// no halo): the grouped 3x3 + 1x1c only.  The residual is res[.., c < bw].
struct DpnBlockParams {
  const void* x; int ldx; int cin;
  const void* res; int ldr;
  int from_a;
  const void* w1; int kp1; const float* m1; const float* i1;   // paired-row [>=128][kp1]
  const void* wg; const float* m2; const float* i2;            // [8][5][64][8]
  const void* w3; int kp3; const float* m3; const float* i3;   // paired-row [>=96][kp3 = 128]
  void* y; void* y2; int ldy; int bw, cout;
  void* halo;
  int N, H, W, seg, nseg;
  int dbg;   // diagnostics (VOXEMB_DPN_DBG, VOX_DIAG builds): 256 = clock stamps
};
hipError_t dpn_trace_read(void* dst, size_t bytes);
// 1x1a + grouped 3x3 of a DPN block in one launch (dpnblk.hip): 1x1a (cin ->
// r, prologue m1/i1, paired-row weights) at the input resolution + grouped
// 3x3 (gconv3x3_rows' weights, gw <= 16, prologue m2/i2) -> y (bf16, r
// channels, ld ldy) at Ho x Wo.  Stride 2 (the projection block of stages 2
// and 3: W 80 or 40, even H and W) or stride 1 (stage 2: W 40, cin <= 288).
struct DpnDownParams {
  const void* x; int ldx; int cin;
  const void* w1; int kp1; const float* m1; const float* i1;
  const void* wg; const float* m2; const float* i2;
  void* y; int ldy; int r;
  int N, H, W, Ho, Wo, seg, nseg;
  int stride;   // 2: the projection block front; 1: a stride-1 block's 1x1a + 3x3 (stage 2)
};
int dpn_down_ok(const DpnDownParams& p);
hipError_t launch_dpn_down(const DpnDownParams& p, hipStream_t s);
int dpn_block_ok(const DpnBlockParams& p);
size_t dpn_block_halo_bytes(const DpnBlockParams& p);
hipError_t launch_dpn_block(const DpnBlockParams& p, hipStream_t s);

// DPN68's 10-channel 1x1 convs with the BN+ReLU prologue (kernels.hip)
int conv1x1_smallk_ok(const ConvParams& p);
hipError_t launch_conv1x1_smallk(const ConvParams& p, hipStream_t s, int v1 = 0);

hipError_t launch_splitk_reduce(const float* partial, int S, int M, int coutp, int cout,
                                const float* mean, const float* inv, int flags,
                                float* out, int ldo, hipStream_t s);

// in_mean / in_inv: optional input BN+ReLU (DPN68's concat_bn_relu) fused into the read
// vlen / vsh (ragged batches): utterance n pools its valid_rows only
hipError_t launch_stats_pool(DType t, const void* x, int N, int H, int W, int C,
                             const float* mean, const float* inv, float* out, hipStream_t s,
                             const float* in_mean = nullptr, const float* in_inv = nullptr,
                             const int* vlen = nullptr, int vsh = 0);

hipError_t launch_avgpool3s2(DType t, const void* x, int ldx, int N, int H, int W, int C,
                             void* y, int ldy, int Ho, int Wo, hipStream_t s,
                             const int* vlen = nullptr, int vsh = 0);

// vlen (ragged batches, n = N * H * rowlen): rows past an utterance's frames -> 0
hipError_t launch_convert_f32(DType t, const float* x, void* y, int64_t n, hipStream_t s,
                              const int* vlen = nullptr, int H = 1, int rowlen = 1);

hipError_t launch_copy_channels(DType t, const void* x, int ldx, void* y, int ldy,
                                int64_t npix, int C, hipStream_t s);

hipError_t launch_bnrelu_inplace(DType t, void* x, int ld, int64_t npix, int C, const float* mean,
                                 const float* inv, hipStream_t s);

}  // namespace vox

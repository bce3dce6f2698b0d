// Fused DPN68 stage-1 dual-path block (stride 1, no projection): 1x1a + grouped
// 3x3 + 1x1c + residual/dense outputs in one row-streamed launch
// (dpn_model.py:57-87: three bn_relu_conv, :40-45, and the [res + h | dense |
// h_dense] concat; the unfused plan is conv1x1_nw -> gconv3x3_rows -> conv1x1_nw).
//
// Stage 1 runs at full resolution (80 x T pixels, r = 128 channels): unfused,
// each block writes and re-reads two 128-channel maps (the 1x1a and grouped-3x3
// outputs, 4 x 256 B per pixel) around its 80-channel result.  Here a
// workgroup owns one utterance segment of `seg` rows and streams it one output
// row per step; the intermediates stay in LDS:
//   X1    the block input row o+1 after the 1x1a's BN+ReLU prologue
//         (prefetched into registers two rows ahead, transformed once)
//   ring  three rows of h1 = relu(bn2(bf16(1x1a))) in gconv3x3_rows' ring
//         layout (8 sub-planes of 2-unit column slots, pad columns zero)
//   H2    the grouped 3x3 output of row o after the 1x1c's BN+ReLU prologue
// and only the block input (read once, plus an L2-hot re-read of its first bw
// channels for the residual) and the 80 output channels touch HBM.
//
// In place: the block's residual channels [0, bw) are rewritten in the stage
// buffer it reads.  Within a workgroup row o is written only after row o+1 has
// been read, but the 3x3 window of a segment's first and last rows reaches
// one row into each neighbour segment, which that segment rewrites at some
// unknown time.  So the halo rows' h1 (rows s0 - 1 and s1 of every segment)
// come from a pre-pass launch of the same kernel (HALO = true) that writes
// their ring images to `halo` before the main launch starts.
//
// Arithmetic is that of the unfused kernels, step by step, so the outputs are
// bit-identical to the unfused plan: conv1x1_nw's prologue
// bf16(max((x - m) * inv, 0)) and K order (chunks of 32 ascending, paired-row
// weights), bf16 rounding of the 1x1a output, gconv3x3_rows' prologue
// ((x + (-m)) * inv, rounded, ReLU on the bf16 bits), its MFMA tap pairing and
// zero tap, the bf16 rounding of its output, and the 1x1c's prologue,
// residual add (+0.0 on the dense channels, as conv1x1_nw) and rounding.
//
// Work split (8 waves, two per SIMD):
//   1x1a   wave w: couts pair w & 3 (32 channels), pixel tiles [0, 3) for
//          w < 4 and [3, 5) for w >= 4 (40 MFMAs per SIMD per row)
//   3x3    wave w: 16-channel slab w, every tile (25 MFMAs per wave)
//   1x1c   (pair, tiles) per wave from the table c3_* below (<= 32 per SIMD)
// All weights are register-resident (84 VGPRs per lane).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "device_common.h"
#include "kernels.h"

namespace vox {

__device__ uint4 g_db_zero[2] = {};   // source of masked loads (channels >= cin, pixels >= W)
__device__ uint4 g_db_sink[64];       // destination of masked lanes' stores
// diagnostics (VOXEMB_DPN_DBG & 256, VOX_DIAG builds): per-step shader-clock
// stamps of workgroup 0's waves [8 waves][256 steps][8 stamps]
__device__ unsigned long long g_db_trace[8 * 256 * 8];

namespace {
constexpr int DB_THREADS = 512;
constexpr int DB_R = 128;   // 1x1a / grouped 3x3 width
constexpr int DB_PXS = 18;  // X1 / H2 units per pixel (16 + 2: 18 = 2 mod 16, conflict-free b128 reads)
constexpr int DB_KS = 4;    // k-steps of 32: 1x1a (cin <= 128) and 1x1c (K = 128)
constexpr int DB_TPR = 5;   // 16-pixel tiles per row (65 <= W <= 80)
constexpr int DB_RXS = 10;  // RES units per pixel (8 + 2: 10 = 10 mod 16, conflict-free b128 reads)

struct DbGeo {
  int spw, rowb, zero, x1, h2, res, tb, lds;
};
__host__ __device__ inline DbGeo db_geo(int W) {
  DbGeo g{};
  int spw = 2 * (W + 2);
  spw += ((2 - spw) % 16 + 16) % 16;   // == 2 (mod 16), as gconv3x3_rows
  g.spw = spw;
  g.rowb = 8 * spw * 16;
  g.zero = 3 * g.rowb;                 // zero line of the paired tap 9 (512 B per tile)
  g.x1 = g.zero + 512 * DB_TPR + 1024; // + slack: masked tail columns read past the ring
  g.h2 = g.x1 + 16 * DB_TPR * DB_PXS * 16;
  g.res = g.h2 + 16 * DB_TPR * DB_PXS * 16;  // residual rows (bw <= 64 channels), 3 slots
  g.tb = g.res + 3 * 16 * DB_TPR * DB_RXS * 16;   // BN tables: m1 i1 -m2 i2 m3 i3 (128 floats each)
  g.lds = g.tb + 6 * DB_R * 4;
  return g;
}

// 1x1c work per wave: couts pair, first pixel tile, tile count (15 units of
// 2 x 4 MFMAs; waves w and w + 4 share a SIMD: 4, 3, 4, 4 units per SIMD)
__device__ constexpr int c3_pair(int w) { return w < 3 ? 0 : (w < 6 ? 1 : 2); }
__device__ constexpr int c3_t0(int w) {
  return w == 0 ? 0 : w == 1 ? 2 : w == 2 ? 4 : w == 3 ? 0 : w == 4 ? 2 : w == 5 ? 4 : w == 6 ? 0 : 3;
}
__device__ constexpr int c3_nt(int w) { return (w == 2 || w == 5) ? 1 : (w == 6 ? 3 : 2); }
}  // namespace

#pragma clang fp contract(off)
// MODE 0: the block (1x1a computed here); 1: halo pre-pass of mode 0; 2: the
// ring rows are read from a 1x1a output map (p.x, 128 channels) and only the
// grouped 3x3 + 1x1c run here (stage 1's projection block, whose 1x1a reads
// the 10-channel stem: conv1x1_smallk's exact fp32 sums stay in that launch)
template <int MODE>
__global__ __launch_bounds__(DB_THREADS) void dpn_block_rows(DpnBlockParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr bool HALO = MODE == 1, FROM_A = MODE == 2;
  constexpr int TPR = DB_TPR;
  constexpr int U = (256 * TPR + DB_THREADS - 1) / DB_THREADS;   // input units per thread
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int W = p.W, H = p.H;
  const DbGeo geo = db_geo(W);
  const int SPW = geo.spw, ROWB = geo.rowb;
  const int n = blockIdx.x / p.nseg;
  const int s0 = (blockIdx.x - n * p.nseg) * p.seg;
  const int s1 = min(s0 + p.seg, H);
  if (s0 >= s1) return;
  const size_t rowe = (size_t)W * p.ldx;                          // elements per input row
  const bf16_t* __restrict__ Xn = reinterpret_cast<const bf16_t*>(p.x) + (size_t)n * H * rowe;
  char* halo = reinterpret_cast<char*>(p.halo) + (size_t)blockIdx.x * 2 * ROWB;

  // ---- input staging roles: unit u = tid + 512 i -> (pixel u / 16, chunk tid % 16)
  const int ch8 = tid & 15;
  int upx[U], uoff[U];
#pragma unroll
  for (int i = 0; i < U; ++i) {
    const int px = (tid + DB_THREADS * i) >> 4;
    upx[i] = px < W ? px : -1;
    uoff[i] = px * p.ldx + 8 * ch8;
  }
  const bool cval = 8 * ch8 < p.cin;
  // BN tables in LDS (1x1a prologue 0 past cin: relu(0 * 0) = 0)
  float* tb = reinterpret_cast<float*>(smem + geo.tb);
  for (int c = tid; c < DB_R; c += DB_THREADS) {
    tb[c] = (!FROM_A && c < p.cin) ? p.m1[c] : 0.f;
    tb[DB_R + c] = (!FROM_A && c < p.cin) ? p.i1[c] : 0.f;
    tb[2 * DB_R + c] = -p.m2[c];
    tb[3 * DB_R + c] = p.i2[c];
    tb[4 * DB_R + c] = p.m3[c];
    tb[5 * DB_R + c] = p.i3[c];
  }
  __syncthreads();
  const uint4* zl = g_db_zero;
  const bool trace = (VOX_DBG(p) & 256) && blockIdx.x == 0 && lane == 0;
  auto stamp = [&](int o, int i) __attribute__((always_inline)) {
    if (trace && o - s0 < 256) g_db_trace[(wave * 256 + (o - s0)) * 8 + i] = __builtin_amdgcn_s_memtime();
  };
  auto load_row = [&](int r, uint4 (&v)[U]) __attribute__((always_inline)) {
    const bf16_t* __restrict__ Xr = Xn + (size_t)r * rowe;   // wave-uniform base
#pragma unroll
    for (int i = 0; i < U; ++i)
      v[i] = *((upx[i] >= 0 && cval) ? reinterpret_cast<const uint4*>(Xr + uoff[i]) : zl);
  };
  // (mode 0) the row's raw first bw channels also go to RES[par] for its 1x1c residual
  auto stage_x1 = [&](const uint4 (&v)[U], int par) __attribute__((always_inline)) {
    float pm[8], pi[8];
    *reinterpret_cast<f32x4*>(pm) = *reinterpret_cast<const f32x4*>(tb + 8 * ch8);
    *reinterpret_cast<f32x4*>(pm + 4) = *reinterpret_cast<const f32x4*>(tb + 8 * ch8 + 4);
    *reinterpret_cast<f32x4*>(pi) = *reinterpret_cast<const f32x4*>(tb + DB_R + 8 * ch8);
    *reinterpret_cast<f32x4*>(pi + 4) = *reinterpret_cast<const f32x4*>(tb + DB_R + 8 * ch8 + 4);
#pragma unroll
    for (int i = 0; i < U; ++i) {
      if (upx[i] < 0) continue;
      const bf16x8 b = __builtin_bit_cast(bf16x8, v[i]);
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (bf16_t)fmaxf(((float)b[e] - pm[e]) * pi[e], 0.f);
      *reinterpret_cast<bf16x8*>(smem + geo.x1 + (upx[i] * DB_PXS + ch8) * 16) = o;
      if (8 * ch8 < p.bw)
        *reinterpret_cast<uint4*>(smem + geo.res + ((par * 16 * TPR + upx[i]) * DB_RXS + ch8) * 16) = v[i];
    }
  };

  // mode 2: a 1x1a output row into ring slot `slot` with gconv3x3_rows' prologue
  auto stage_ring = [&](const uint4 (&v)[U], int slot) __attribute__((always_inline)) {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    float nm[8], iv[8];
    *reinterpret_cast<f32x4*>(nm) = *reinterpret_cast<const f32x4*>(tb + 2 * DB_R + 8 * ch8);
    *reinterpret_cast<f32x4*>(nm + 4) = *reinterpret_cast<const f32x4*>(tb + 2 * DB_R + 8 * ch8 + 4);
    *reinterpret_cast<f32x4*>(iv) = *reinterpret_cast<const f32x4*>(tb + 3 * DB_R + 8 * ch8);
    *reinterpret_cast<f32x4*>(iv + 4) = *reinterpret_cast<const f32x4*>(tb + 3 * DB_R + 8 * ch8 + 4);
    const int cu = (ch8 >> 1) * geo.spw + (ch8 & 1);
#pragma unroll
    for (int i = 0; i < U; ++i) {
      if (upx[i] < 0) continue;
      const vu32x4 w = __builtin_bit_cast(vu32x4, v[i]);
      bf16x8 r;
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        f32x2 xv = {__builtin_bit_cast(float, w[h] << 16), __builtin_bit_cast(float, w[h] & 0xFFFF0000u)};
        const f32x2 m2 = {nm[2 * h], nm[2 * h + 1]};
        const f32x2 i2 = {iv[2 * h], iv[2 * h + 1]};
        xv = (xv + m2) * i2;
        r[2 * h] = (bf16_t)xv[0];
        r[2 * h + 1] = (bf16_t)xv[1];
      }
      *reinterpret_cast<bf16x8*>(smem + slot + (cu + 2 * (upx[i] + 1)) * 16) = relu_bf16(r);
    }
  };

  // ---- 1x1a: couts pair q1 (paired-row weights: lane channels 32 q1 + 8 g + 0..7)
  const int q1 = wave & 3;
  constexpr int T1A = (TPR + 1) / 2, T1B = TPR / 2;
  bf16x8 a1[2][DB_KS];
  if constexpr (!FROM_A) {
    const bf16_t* w1 = reinterpret_cast<const bf16_t*>(p.w1);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int s = 0; s < DB_KS; ++s) {
        const int c = 32 * s + 8 * g;
        a1[u][s] = c < p.kp1 ? ld16(w1 + (size_t)((2 * q1 + u) * 16 + col) * p.kp1 + c) : bf16x8{};
      }
  }
  // h1 unit of chunk 4 q1 + g at column slot x (= pixel + 1)
  const int h1u = ((4 * q1 + g) >> 1) * SPW + ((4 * q1 + g) & 1);
  auto gemm1a_t = [&](auto NT_, int t0, int slot) __attribute__((always_inline)) {
    constexpr int NT = decltype(NT_)::value;
    f32x4 acc[2][NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[0][j] = acc[1][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < DB_KS; ++s)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(
            smem + geo.x1 + ((16 * (t0 + j) + col) * DB_PXS + 4 * s + g) * 16);
        acc[0][j] = mfma_step(a1[0][s], b, acc[0][j]);
        acc[1][j] = mfma_step(a1[1][s], b, acc[1][j]);
      }
    // gconv prologue of the lane's channels (negated means)
    float nm2[8], iv2[8];
    {
      const float* t2 = tb + 2 * DB_R + 32 * q1 + 8 * g;
      *reinterpret_cast<f32x4*>(nm2) = *reinterpret_cast<const f32x4*>(t2);
      *reinterpret_cast<f32x4*>(nm2 + 4) = *reinterpret_cast<const f32x4*>(t2 + 4);
      *reinterpret_cast<f32x4*>(iv2) = *reinterpret_cast<const f32x4*>(t2 + DB_R);
      *reinterpret_cast<f32x4*>(iv2 + 4) = *reinterpret_cast<const f32x4*>(t2 + DB_R + 4);
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int px = 16 * (t0 + j) + col;
      if (px >= W) continue;   // the pad column slots stay zero
      typedef float f32x2 __attribute__((ext_vector_type(2)));
      bf16x8 r;
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        // bf16 1x1a output, then relu((x + (-m)) * inv) on fp32 pairs as gconv3x3_rows
        const int e0 = 2 * h, e1 = 2 * h + 1;
        const float v0 = (float)(bf16_t)(e0 < 4 ? acc[0][j][e0] : acc[1][j][e0 - 4]);
        const float v1 = (float)(bf16_t)(e1 < 4 ? acc[0][j][e1] : acc[1][j][e1 - 4]);
        f32x2 xv = {v0, v1};
        const f32x2 m2 = {nm2[e0], nm2[e1]};
        const f32x2 i2 = {iv2[e0], iv2[e1]};
        xv = (xv + m2) * i2;
        r[e0] = (bf16_t)xv[0];
        r[e1] = (bf16_t)xv[1];
      }
      *reinterpret_cast<bf16x8*>(smem + slot + (h1u + 2 * (px + 1)) * 16) = relu_bf16(r);
    }
  };
  using NA = std::integral_constant<int, T1A>;
  using NB = std::integral_constant<int, T1B>;
  auto gemm1a = [&](int slot) __attribute__((always_inline)) {
    if (wave < 4) gemm1a_t(NA{}, 0, slot);
    else gemm1a_t(NB{}, T1A, slot);
  };

  // zero the pad column slots of the ring rows, and the zero line
  for (int u = tid; u < 3 * 8 * 4; u += DB_THREADS) {
    const int row = u >> 5, sp = (u >> 2) & 7, e = u & 3;
    const int xs = (e >> 1) ? W + 1 : 0;
    *reinterpret_cast<uint4*>(smem + row * ROWB + (sp * SPW + 2 * xs + (e & 1)) * 16) = uint4{0u, 0u, 0u, 0u};
  }
  for (int u = tid; u < 32 * TPR; u += DB_THREADS)
    *reinterpret_cast<uint4*>(smem + geo.zero + u * 16) = uint4{0u, 0u, 0u, 0u};

  if constexpr (HALO) {
    // h1 of rows s0 - 1 and s1 (those inside the image) -> halo[0], halo[1]
#pragma unroll 1
    for (int j = 0; j < 2; ++j) {
      const int r = j == 0 ? s0 - 1 : s1;
      if (r < 0 || r >= H) continue;
      uint4 v[U];
      load_row(r, v);
      stage_x1(v, 0);
      __syncthreads();
      gemm1a(0);
      __syncthreads();
      for (int u = tid; u < ROWB / 16; u += DB_THREADS)
        reinterpret_cast<uint4*>(halo + (size_t)j * ROWB)[u] = reinterpret_cast<const uint4*>(smem)[u];
      __syncthreads();
    }
    return;
  } else {
    auto ring_off = [&](int r) { return ((r - s0 + 3) % 3) * ROWB; };   // r >= s0 - 1
    auto fill_row = [&](int slot, int j) __attribute__((always_inline)) {
      // halo image j, or zeros for a row outside the image
      const bool z = j < 0;
      for (int u = tid; u < ROWB / 16; u += DB_THREADS)
        reinterpret_cast<uint4*>(smem + slot)[u] =
            z ? uint4{0u, 0u, 0u, 0u} : reinterpret_cast<const uint4*>(halo + (size_t)j * ROWB)[u];
    };

    // ---- grouped 3x3: slab `wave` (output channels 16 wave + 4 g + 0..3)
    bf16x8 ag[5];
    {
      const bf16_t* wp = reinterpret_cast<const bf16_t*>(p.wg) + ((size_t)wave * 5 * 64 + lane) * 8;
#pragma unroll
      for (int m = 0; m < 5; ++m) ag[m] = ld16(wp + m * 512);
    }
    int lofs[5];
#pragma unroll
    for (int m = 0; m < 5; ++m) {
      const int tap = 2 * m + (g >> 1);
      const int kx = (tap < 9 ? tap : 8) % 3;
      const int chunk = 2 * wave + (g & 1);
      lofs[m] = ((chunk >> 1) * SPW + 2 * (col + kx) + (chunk & 1)) * 16;
    }
    auto gconv_row = [&](int o) __attribute__((always_inline)) {
      const int r0 = __builtin_amdgcn_readfirstlane(ring_off(o - 1));
      const int r1 = __builtin_amdgcn_readfirstlane(ring_off(o));
      const int r2 = __builtin_amdgcn_readfirstlane(ring_off(o + 1));
      f32x4 acc[TPR];
#pragma unroll
      for (int t = 0; t < TPR; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int m = 0; m < 5; ++m) {
        int addr;
        if (m == 0) addr = r0 + lofs[0];                          // taps 0, 1
        else if (m == 1) addr = ((g >> 1) ? r1 : r0) + lofs[1];   // taps 2 (row 0), 3 (row 1)
        else if (m == 2) addr = r1 + lofs[2];                     // taps 4, 5
        else if (m == 3) addr = r2 + lofs[3];                     // taps 6, 7
        else addr = (g >> 1) ? geo.zero : r2 + lofs[4];           // tap 8, zero tap
#pragma unroll
        for (int t = 0; t < TPR; ++t) {
          const bf16x8 b = *reinterpret_cast<const bf16x8*>(smem + addr + 512 * t);
          acc[t] = mfma_step(ag[m], b, acc[t]);
        }
      }
      // 1x1c prologue of the lane's channels
      const f32x4 m3g = *reinterpret_cast<const f32x4*>(tb + 4 * DB_R + 16 * wave + 4 * g);
      const f32x4 i3g = *reinterpret_cast<const f32x4*>(tb + 5 * DB_R + 16 * wave + 4 * g);
#pragma unroll
      for (int t = 0; t < TPR; ++t) {
        const int px = 16 * t + col;
        bf16x4 o4;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          o4[e] = (bf16_t)fmaxf(((float)(bf16_t)acc[t][e] - m3g[e]) * i3g[e], 0.f);
        *reinterpret_cast<bf16x4*>(smem + geo.h2 + (px * DB_PXS + 2 * wave + (g >> 1)) * 16 + (g & 1) * 8) = o4;
      }
    };

    // ---- 1x1c: couts pair q3 (lane channels 32 q3 + 8 g + 0..7), tiles [t3, t3 + nt3)
    const int q3 = c3_pair(wave), t3 = c3_t0(wave), nt3 = c3_nt(wave);
    bf16x8 a3[2][DB_KS];
    {
      const bf16_t* w3 = reinterpret_cast<const bf16_t*>(p.w3);
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int s = 0; s < DB_KS; ++s)
          a3[u][s] = ld16(w3 + (size_t)((2 * q3 + u) * 16 + col) * p.kp3 + 32 * s + 8 * g);
    }
    const int ch3 = 32 * q3 + 8 * g;
    bf16_t* __restrict__ Yn = reinterpret_cast<bf16_t*>(p.y) + (size_t)n * H * W * p.ldy;
    bf16_t* __restrict__ Y2n = reinterpret_cast<bf16_t*>(p.y2) + (size_t)n * H * W * p.ldy;
    // mode 2: the residual rows (p.res, first bw channels) are prefetched with
    // the ring rows: unit u = tid + 512 i -> (pixel u / 8, chunk u % 8)
    const bf16_t* __restrict__ Rn = reinterpret_cast<const bf16_t*>(p.res) + (size_t)n * H * W * p.ldr;
    // mode 2: the residual (p.res rows, first bw channels) straight into the
    // 1x1c lanes' registers, requested before the staging of the step
    uint4 rv[3];
    auto load_rv = [&](int o) __attribute__((always_inline)) {
      const bf16_t* __restrict__ Rr = Rn + (size_t)o * W * p.ldr;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int px = 16 * (t3 + j) + col;
        const bool ok = j < nt3 && px < W && ch3 < p.bw;
        rv[j] = *(ok ? reinterpret_cast<const uint4*>(Rr + (size_t)px * p.ldr + ch3) : zl);
      }
    };
    auto gemm1c_t = [&](auto NT_, int o) __attribute__((always_inline)) {
      constexpr int NT = decltype(NT_)::value;
      f32x4 acc[2][NT];
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[0][j] = acc[1][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < DB_KS; ++s)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const bf16x8 b = *reinterpret_cast<const bf16x8*>(
              smem + geo.h2 + ((16 * (t3 + j) + col) * DB_PXS + 4 * s + g) * 16);
          acc[0][j] = mfma_step(a3[0][s], b, acc[0][j]);
          acc[1][j] = mfma_step(a3[1][s], b, acc[1][j]);
        }
      const int par = (o - s0) % 3;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int px = 16 * (t3 + j) + col;
        // residual below bw (RES row o), +0.0 on the dense channels (conv1x1_nw)
        bf16x8 r;
        if constexpr (FROM_A)
          r = __builtin_bit_cast(bf16x8, rv[j]);
        else
          r = ch3 < p.bw ? *reinterpret_cast<const bf16x8*>(
                               smem + geo.res + ((par * 16 * TPR + px) * DB_RXS + (ch3 >> 3)) * 16)
                         : bf16x8{};
        bf16x8 o8;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float v = e < 4 ? acc[0][j][e] : acc[1][j][e - 4];
          v += (float)r[e];
          o8[e] = (bf16_t)v;
        }
        // every lane stores (masked ones into the sink): no divergent store
        // branches, so the compiler's vmcnt counts stay exact
        const size_t pix = (size_t)o * W + px;
        bf16_t* dst = ch3 < p.bw ? Yn + pix * p.ldy + ch3 : Y2n + pix * p.ldy + (ch3 - p.bw);
        void* d = (ch3 < p.cout && px < W) ? (void*)dst : (void*)&g_db_sink[lane];
        *reinterpret_cast<bf16x8*>(d) = o8;
      }
    };
    using N1 = std::integral_constant<int, 1>;
    using N2 = std::integral_constant<int, 2>;
    using N3 = std::integral_constant<int, 3>;
    auto gemm1c = [&](int o) __attribute__((always_inline)) {
      if (nt3 == 1) gemm1c_t(N1{}, o);
      else if (nt3 == 2) gemm1c_t(N2{}, o);
      else gemm1c_t(N3{}, o);
    };

    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    if constexpr (FROM_A) {
      // ring rows straight from the (immutable) 1x1a map: rows s0 - 1 .. s1,
      // zeros outside the image.  Ring row o + 2 is staged
      // in step o between the 3x3 and the 1x1c (their register prefetch, two
      // rows ahead, has long landed; the wait then covers no fresh stores).
      const int last = min(s1, H - 1);
      uint4 pf[2][U];
      if (s0 > 0) {
        load_row(s0 - 1, pf[1]);
        stage_ring(pf[1], ring_off(s0 - 1));
      } else {
        fill_row(ring_off(s0 - 1), -1);
      }
      load_row(s0, pf[0]);
      if (s0 + 1 <= last) load_row(s0 + 1, pf[1]);
      stage_ring(pf[0], ring_off(s0));
      if (s0 + 2 <= last) load_row(s0 + 2, pf[0]);
      if (s0 + 1 < H) stage_ring(pf[1], ring_off(s0 + 1));
      else fill_row(ring_off(s0 + 1), -1);
      if (s0 + 3 <= last) load_row(s0 + 3, pf[1]);
      __syncthreads();
      auto step = [&](auto PS, int o) __attribute__((always_inline)) {
        constexpr int PI = decltype(PS)::value;
        gconv_row(o);      // ring rows o - 1 .. o + 1
        __syncthreads();   // H2 complete; ring slot of row o - 1 free
        if (o + 2 <= s1) {
          if (o + 2 < H) {
            stage_ring(pf[PI], ring_off(o + 2));
            if (o + 4 <= last) load_row(o + 4, pf[PI]);
          } else {
            fill_row(ring_off(o + 2), -1);
          }
        }
        load_rv(o);   // the youngest loads: the 1x1c epilogue's wait covers nothing else
        gemm1c(o);
        __syncthreads();   // ring row o + 2 staged; H2 free
      };
      for (int o = s0; o < s1; o += 2) {
        step(P0{}, o);
        if (o + 1 < s1) step(P1{}, o + 1);
      }
      return;
    }
    // ---- prologue: ring rows s0 - 1 (halo / zeros) and s0 (computed), X1 = row s0 + 1
    fill_row(ring_off(s0 - 1), s0 > 0 ? 0 : -1);
    uint4 pf[2][U];
    load_row(s0, pf[0]);
    if (s0 + 1 < s1) load_row(s0 + 1, pf[1]);
    stage_x1(pf[0], 0);
    if (s0 + 2 < s1) load_row(s0 + 2, pf[0]);
    __syncthreads();
    gemm1a(ring_off(s0));
    __syncthreads();
    if (s0 + 1 < s1) {
      stage_x1(pf[1], 1);
      if (s0 + 3 < s1) load_row(s0 + 3, pf[1]);
    }
    __syncthreads();

    // step o: h1 of row o + 1 (X1) into the ring, 3x3 of row o into H2, then
    // row o + 2 into X1 / RES (its register prefetch, two rows ahead, has long
    // landed, and the wait for it covers no fresh stores) and the 1x1c of row
    // o to HBM.  Row o + 2's input is in pf[PI] (PI = (o - s0) & 1).
    auto step = [&](auto PS, int o) __attribute__((always_inline)) {
      constexpr int PI = decltype(PS)::value;
      stamp(o, 0);
      if (o + 1 < s1) gemm1a(ring_off(o + 1));
      else fill_row(ring_off(o + 1), o + 1 < H ? 1 : -1);
      stamp(o, 1);
      __syncthreads();   // ring rows o - 1 .. o + 1 complete; X1 free
      stamp(o, 2);
      gconv_row(o);
      stamp(o, 3);
      __syncthreads();   // H2 complete
      stamp(o, 4);
      if (o + 2 < s1) {
        stage_x1(pf[PI], (o + 2 - s0) % 3);
        if (o + 4 < s1) load_row(o + 4, pf[PI]);
      }
      stamp(o, 5);
      gemm1c(o);
      stamp(o, 6);
      __syncthreads();   // X1 = row o + 2; H2 free
      stamp(o, 7);
    };
    for (int o = s0; o < s1; o += 2) {
      step(P0{}, o);
      if (o + 1 < s1) step(P1{}, o + 1);
    }
  }
}


// ---------------------------------------------------------------------------
// Projection block front of a stride-2 stage (dpn_model.py:57-87 with
// stride 2; stage 2 of DPN68): the 1x1a (cin -> r, BN+ReLU prologue) at the
// full input resolution and the grouped 3x3 with stride 2 (TF SAME, pad_beg 0)
// in one row-streamed launch.  Unfused, the 1x1a writes its r-channel map at
// full resolution (1.57 GB at B = 64, 80 x 600) and the 3x3 reads it back.
// Workgroup = (utterance segment of output rows, 128-channel slice of r; the
// groups lie inside a slice).  Step = output row o: the 1x1a of input rows
// 2o+1 and 2o+2 (waves 0-3 / 4-7, one 32-cout pair each) into a 3-row ring
// (row 2o stays from the previous step; segments share one input row and
// recompute it, nothing is written in place), then the 3x3 of row o to HBM.
// Bit-identical to gemm1x1_ws<.., GS_PRO> -> gconv3x3_rows<.., 2, ..>: the
// 1x1a prologue and K order, the bf16 1x1a output, the 3x3's staging
// prologue, its stride-2 column-slot layout and tap pairing.
// Shapes (compile time): KS 1x1a k-steps (cin <= 32 KS), TPI / TPO input /
// output 16-pixel tiles per row, PXS X1 units per pixel (4 KS + 2, = 2 mod 4:
// conflict-free b128 fragment reads), PL staging pixel lanes (4 KS x PL <= 512
// threads each own one 8-channel chunk).
//   stage 2 of DPN68: 80 -> 40 columns, cin 144: <5, 5, 3, 22, 25>
//   stage 3:          40 -> 20 columns, cin 320: <10, 3, 2, 42, 12>
//   stage-2 stride-1 blocks (S = 1): 40 columns, cin <= 288: <9, 3, 3, 38, 14, 1>
// With S = 1 a step adds input rows o+1, o+2 and produces output rows o, o+1
// (4-row ring; the segment's first window row o-1 is computed by the segment
// itself: the block's 1x1c writes its output in place only after this launch).
template <int KS, int TPI, int TPO, int PXS, int PL, int S = 2>
struct DdShape {
  static constexpr int ks = KS, tpi = TPI, tpo = TPO, pxs = PXS, pl = PL, st = S;
  static constexpr int nring = S == 2 ? 3 : 4;
};
using DdS2 = DdShape<5, 5, 3, 22, 25>;
using DdS3 = DdShape<10, 3, 2, 42, 12>;
using DdF2 = DdShape<9, 3, 3, 38, 14, 1>;
namespace {
struct DdGeo {
  int spw, rowb, zero, x1, tb, lds;
};
template <class SH>
__host__ __device__ inline DdGeo dd_geo(int W) {
  DdGeo g{};
  int spw = 2 * (W + 2);
  spw += ((2 - spw) % 16 + 16) % 16;
  g.spw = spw;
  g.rowb = 8 * spw * 16;
  g.zero = SH::nring * g.rowb;
  g.x1 = g.zero + 512 * SH::tpo + 1024;
  g.tb = g.x1 + 2 * 16 * SH::tpi * SH::pxs * 16;   // m1 i1 (32 KS each) -m2 i2 (128 each)
  g.lds = g.tb + (2 * 32 * SH::ks + 2 * DB_R) * 4;
  return g;
}
}  // namespace

template <class SH>
__global__ __launch_bounds__(DB_THREADS) void dpn_down_rows(DpnDownParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int DD_KS = SH::ks, DD_TPI = SH::tpi, DD_TPO = SH::tpo, DD_PXS = SH::pxs, PL = SH::pl;
  constexpr int CPX = 4 * DD_KS;                 // 8-channel chunks per pixel
  static_assert(CPX * PL <= DB_THREADS, "staging threads");
  constexpr int KW = 32 * DD_KS;                 // padded K of the 1x1a
  constexpr int UP = (16 * DD_TPI + PL - 1) / PL;   // pixels per staging thread per row
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int W = p.W, H = p.H, Ho = p.Ho, Wo = p.Wo;
  const DdGeo geo = dd_geo<SH>(W);
  const int SPW = geo.spw, ROWB = geo.rowb;
  constexpr int S = SH::st, NR = SH::nring;
  const int E = (W + 3) >> 1;                    // stride 2: even padded columns come first
  auto slot_of = [&](int xp) { return S == 1 ? xp : ((xp & 1) ? E + (xp >> 1) : (xp >> 1)); };
  // blockIdx -> (segment id, slice): the slices of a segment 8 apart (one XCD,
  // one L2 for their shared input rows)
  const int b = blockIdx.x;
  const int nsl = p.r / DB_R;
  const int sid = (b >> 3) / nsl * 8 + (b & 7), slice = (b >> 3) % nsl;
  const int n = sid / p.nseg;
  if (n >= p.N) return;
  const int s0 = (sid - n * p.nseg) * p.seg;
  const int s1 = min(s0 + p.seg, Ho);
  if (s0 >= s1) return;
  const int c0 = slice * DB_R;
  const size_t rowe = (size_t)W * p.ldx;
  const bf16_t* __restrict__ Xn = reinterpret_cast<const bf16_t*>(p.x) + (size_t)n * H * rowe;

  // ---- BN tables
  float* tb = reinterpret_cast<float*>(smem + geo.tb);
  for (int c = tid; c < KW; c += DB_THREADS) {
    tb[c] = c < p.cin ? p.m1[c] : 0.f;
    tb[KW + c] = c < p.cin ? p.i1[c] : 0.f;
  }
  for (int c = tid; c < DB_R; c += DB_THREADS) {
    tb[2 * KW + c] = -p.m2[c0 + c];
    tb[2 * KW + DB_R + c] = p.i2[c0 + c];
  }
  // zero the pad column slots of the ring rows, and the zero line
  for (int u = tid; u < NR * 8 * 4; u += DB_THREADS) {
    const int row = u >> 5, sp = (u >> 2) & 7, e = u & 3;
    const int xs = slot_of((e >> 1) ? W + 1 : 0);
    *reinterpret_cast<uint4*>(smem + row * ROWB + (sp * SPW + 2 * xs + (e & 1)) * 16) = uint4{0u, 0u, 0u, 0u};
  }
  for (int u = tid; u < 32 * DD_TPO; u += DB_THREADS)
    *reinterpret_cast<uint4*>(smem + geo.zero + u * 16) = uint4{0u, 0u, 0u, 0u};
  __syncthreads();

  // ---- staging roles: thread t < CPX PL -> chunk t % CPX (8 channels) of
  // pixels t / CPX + PL j, both rows of a step
  const bool sact = tid < CPX * PL;
  const int sch = tid % CPX, spl = tid / CPX;
  const bool cval = sact && 8 * sch < p.cin;
  const uint4* zl = g_db_zero;
  // rows ra, ra + 1 (each only if < H and < rlim)
  auto load_rows = [&](int ra, int rlim, uint4 (&v)[2][UP]) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int r = ra + k;
      const bf16_t* __restrict__ Xr = Xn + (size_t)r * rowe;
#pragma unroll
      for (int j = 0; j < UP; ++j) {
        const int px = spl + PL * j;
        const bool ok = cval && px < W && r >= 0 && r < H && r < rlim;
        v[k][j] = *(ok ? reinterpret_cast<const uint4*>(Xr + (size_t)px * p.ldx + 8 * sch) : zl);
      }
    }
  };
  auto stage = [&](const uint4 (&v)[2][UP]) __attribute__((always_inline)) {
    if (!sact) return;
    float pm[8], pi[8];
    *reinterpret_cast<f32x4*>(pm) = *reinterpret_cast<const f32x4*>(tb + 8 * sch);
    *reinterpret_cast<f32x4*>(pm + 4) = *reinterpret_cast<const f32x4*>(tb + 8 * sch + 4);
    *reinterpret_cast<f32x4*>(pi) = *reinterpret_cast<const f32x4*>(tb + KW + 8 * sch);
    *reinterpret_cast<f32x4*>(pi + 4) = *reinterpret_cast<const f32x4*>(tb + KW + 8 * sch + 4);
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int j = 0; j < UP; ++j) {
        const int px = spl + PL * j;
        if (px >= W) continue;
        const bf16x8 bv = __builtin_bit_cast(bf16x8, v[k][j]);
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (bf16_t)fmaxf(((float)bv[e] - pm[e]) * pi[e], 0.f);
        *reinterpret_cast<bf16x8*>(smem + geo.x1 + ((k * 16 * DD_TPI + px) * DD_PXS + sch) * 16) = o;
      }
  };

  // ---- 1x1a: wave -> (row k = wave / 4 of the step, couts pair q1 = wave % 4 of the slice)
  const int q1 = wave & 3, kr = wave >> 2;
  bf16x8 a1[2][DD_KS];
  {
    const bf16_t* w1 = reinterpret_cast<const bf16_t*>(p.w1);
    const int q = c0 / 32 + q1;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int s = 0; s < DD_KS; ++s) {
        const int c = 32 * s + 8 * g;
        a1[u][s] = c < p.kp1 ? ld16(w1 + (size_t)((2 * q + u) * 16 + col) * p.kp1 + c) : bf16x8{};
      }
  }
  const int h1u = ((4 * q1 + g) >> 1) * SPW + ((4 * q1 + g) & 1);
  // first input row of the segment's windows: 2 s0 (stride 2, pad_beg 0) or s0 - 1
  const int rfirst = S == 2 ? 2 * s0 : s0 - 1;
  auto ring_off = [&](int r) { return ((r - rfirst) % NR) * ROWB; };   // input row r >= rfirst
  // input row r (waves of row part kr) -> its ring slot; zeros outside the image
  auto gemm1a = [&](int r) __attribute__((always_inline)) {
    const int slot = ring_off(r);
    if (r < 0 || r >= H) {
#pragma unroll
      for (int t = 0; t < DD_TPI; ++t) {
        const int px = 16 * t + col;
        if (px < W)
          *reinterpret_cast<uint4*>(smem + slot + (h1u + 2 * slot_of(px + 1)) * 16) = uint4{0u, 0u, 0u, 0u};
      }
      return;
    }
    f32x4 acc[2][DD_TPI];
#pragma unroll
    for (int t = 0; t < DD_TPI; ++t) acc[0][t] = acc[1][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < DD_KS; ++s) {
      if (32 * s >= p.kp1) break;   // (uniform) the unfused GEMM's k-steps, no more
#pragma unroll
      for (int t = 0; t < DD_TPI; ++t) {
        const bf16x8 bv = *reinterpret_cast<const bf16x8*>(
            smem + geo.x1 + ((kr * 16 * DD_TPI + 16 * t + col) * DD_PXS + 4 * s + g) * 16);
        acc[0][t] = mfma_step(a1[0][s], bv, acc[0][t]);
        acc[1][t] = mfma_step(a1[1][s], bv, acc[1][t]);
      }
    }
    float nm2[8], iv2[8];
    {
      const float* t2 = tb + 2 * KW + 32 * q1 + 8 * g;
      *reinterpret_cast<f32x4*>(nm2) = *reinterpret_cast<const f32x4*>(t2);
      *reinterpret_cast<f32x4*>(nm2 + 4) = *reinterpret_cast<const f32x4*>(t2 + 4);
      *reinterpret_cast<f32x4*>(iv2) = *reinterpret_cast<const f32x4*>(t2 + DB_R);
      *reinterpret_cast<f32x4*>(iv2 + 4) = *reinterpret_cast<const f32x4*>(t2 + DB_R + 4);
    }
#pragma unroll
    for (int t = 0; t < DD_TPI; ++t) {
      const int px = 16 * t + col;
      if (px >= W) continue;
      typedef float f32x2 __attribute__((ext_vector_type(2)));
      bf16x8 rr;
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const int e0 = 2 * h, e1 = 2 * h + 1;
        const float v0 = (float)(bf16_t)(e0 < 4 ? acc[0][t][e0] : acc[1][t][e0 - 4]);
        const float v1 = (float)(bf16_t)(e1 < 4 ? acc[0][t][e1] : acc[1][t][e1 - 4]);
        f32x2 xv = {v0, v1};
        const f32x2 m2 = {nm2[e0], nm2[e1]};
        const f32x2 i2 = {iv2[e0], iv2[e1]};
        xv = (xv + m2) * i2;
        rr[e0] = (bf16_t)xv[0];
        rr[e1] = (bf16_t)xv[1];
      }
      *reinterpret_cast<bf16x8*>(smem + slot + (h1u + 2 * slot_of(px + 1)) * 16) = relu_bf16(rr);
    }
  };

  // ---- grouped 3x3 stride 2: slab `wave` of the slice (channels c0 + 16 wave + 4 g + 0..3)
  bf16x8 ag[5];
  {
    const bf16_t* wp = reinterpret_cast<const bf16_t*>(p.wg) + ((size_t)(c0 / 16 + wave) * 5 * 64 + lane) * 8;
#pragma unroll
    for (int m = 0; m < 5; ++m) ag[m] = ld16(wp + m * 512);
  }
  int lofs[5];
#pragma unroll
  for (int m = 0; m < 5; ++m) {
    const int tap = 2 * m + (g >> 1);
    const int kx = (tap < 9 ? tap : 8) % 3;
    const int chunk = 2 * wave + (g & 1);
    lofs[m] = ((chunk >> 1) * SPW + 2 * slot_of(S * col + kx + (S == 2 ? 1 : 0)) + (chunk & 1)) * 16;
  }
  bf16_t* __restrict__ Y = reinterpret_cast<bf16_t*>(p.y) + (size_t)n * Ho * Wo * p.ldy + c0 + 16 * wave + 4 * g;
  const bool wide = (p.ldy & 7) == 0;   // 16-B aligned rows
  auto gconv_row = [&](int o) __attribute__((always_inline)) {
    const int wr = S == 2 ? 2 * o : o - 1;   // window row 0
    const int r0 = __builtin_amdgcn_readfirstlane(ring_off(wr));
    const int r1 = __builtin_amdgcn_readfirstlane(ring_off(wr + 1));
    const int r2 = __builtin_amdgcn_readfirstlane(ring_off(wr + 2));
    f32x4 acc[DD_TPO];
#pragma unroll
    for (int t = 0; t < DD_TPO; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int m = 0; m < 5; ++m) {
      int addr;
      if (m == 0) addr = r0 + lofs[0];
      else if (m == 1) addr = ((g >> 1) ? r1 : r0) + lofs[1];
      else if (m == 2) addr = r1 + lofs[2];
      else if (m == 3) addr = r2 + lofs[3];
      else addr = (g >> 1) ? geo.zero : r2 + lofs[4];
#pragma unroll
      for (int t = 0; t < DD_TPO; ++t) {
        const bf16x8 bv = *reinterpret_cast<const bf16x8*>(smem + addr + 512 * t);
        acc[t] = mfma_step(ag[m], bv, acc[t]);
      }
    }
    auto cvt = [&](int t) __attribute__((always_inline)) {
      bf16x4 o4;
#pragma unroll
      for (int e = 0; e < 4; ++e) o4[e] = (bf16_t)acc[t][e];
      return __builtin_bit_cast(uint2, o4);
    };
    if (wide) {
      // tiles t, t + 1: a half-row exchange per dword gives lane (col, g) 8
      // contiguous channels 8 (g / 2) of tile t + g % 2, one 16-B store
      // (8-B stores were 16 pixels x 32 B per instruction)
#pragma unroll
      for (int t = 0; t + 1 < DD_TPO; t += 2) {
        const uint2 d0 = cvt(t), d1 = cvt(t + 1);
        const auto s0 = __builtin_amdgcn_permlane16_swap(d0.x, d1.x, false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(d0.y, d1.y, false, false);
        const int oc = 16 * (t + (g & 1)) + col;
        if (oc < Wo)
          *reinterpret_cast<uint4*>(Y - 4 * g + 8 * (g >> 1) + ((size_t)o * Wo + oc) * p.ldy) =
              make_uint4(s0[0], s1[0], s0[1], s1[1]);
      }
      if constexpr (DD_TPO % 2 == 1) {
        const int oc = 16 * (DD_TPO - 1) + col;
        if (oc < Wo) *reinterpret_cast<uint2*>(Y + ((size_t)o * Wo + oc) * p.ldy) = cvt(DD_TPO - 1);
      }
    } else {
#pragma unroll
      for (int t = 0; t < DD_TPO; ++t) {
        const int oc = 16 * t + col;
        void* d = oc < Wo ? (void*)(Y + ((size_t)o * Wo + oc) * p.ldy) : (void*)&g_db_sink[lane];
        *reinterpret_cast<uint2*>(d) = cvt(t);
      }
    }
  };

  uint4 pf[2][UP];               // one step ahead
  if constexpr (S == 2) {
    // ---- prologue: input row 2 s0 (the first window row) into the ring
    const int rlim = 2 * s1 + 1;   // input rows this segment needs: [2 s0, 2 s1]
    load_rows(2 * s0, 2 * s0 + 1, pf);             // row 2 s0 only
    stage(pf);
    load_rows(2 * s0 + 1, rlim, pf);               // step s0: rows 2 s0 + 1, 2 s0 + 2
    __syncthreads();
    if (kr == 0) gemm1a(2 * s0);
    __syncthreads();
    for (int o = s0; o < s1; ++o) {
      // X1 is free: the previous step's 1x1a finished before its second barrier
      stage(pf);         // rows 2o+1, 2o+2
      if (o + 1 < s1) load_rows(2 * o + 3, rlim, pf);
      __syncthreads();   // X1 = rows 2o+1, 2o+2; ring slots of rows 2o-2, 2o-1 free (3x3 of o-1 done)
      gemm1a(2 * o + 1 + kr);
      __syncthreads();   // ring rows 2o .. 2o+2 complete
      gconv_row(o);
    }
  } else {
    // ---- prologue: input rows s0 - 1, s0 into the ring
    const int rlim = s1 + 1;       // input rows this segment needs: [s0 - 1, s1]
    load_rows(s0 - 1, rlim, pf);
    stage(pf);
    load_rows(s0 + 1, rlim, pf);                   // step s0: rows s0 + 1, s0 + 2
    __syncthreads();
    gemm1a(s0 - 1 + kr);
    __syncthreads();
    for (int o = s0; o < s1; o += 2) {
      stage(pf);         // rows o+1, o+2
      if (o + 2 < s1) load_rows(o + 3, rlim, pf);
      __syncthreads();   // X1 = rows o+1, o+2; ring slots of rows o-3, o-2 free (3x3 of o-2, o-1 done)
      gemm1a(o + 1 + kr);
      __syncthreads();   // ring rows o-1 .. o+2 complete
      gconv_row(o);
      if (o + 1 < s1) gconv_row(o + 1);
    }
  }
}

template <class SH>
static bool dd_fits(const DpnDownParams& p, int cin_lo) {
  return p.W > 16 * (SH::tpi - 1) && p.W <= 16 * SH::tpi && p.Wo <= 16 * SH::tpo &&
         p.cin <= 32 * SH::ks && p.kp1 <= 32 * SH::ks && p.cin > cin_lo;
}

// 0: no instance; 2 / 3: the stride-2 stage-2 / stage-3 shapes; 1: stride-1 stage 2
static int dd_shape(const DpnDownParams& p) {
  if (!(p.cin > 0 && p.cin % 8 == 0 && p.cin <= p.ldx && p.ldx % 8 == 0 && p.kp1 >= p.cin &&
        p.r % DB_R == 0 && p.ldy % 4 == 0 && p.N > 0 && p.seg > 0 && p.nseg > 0 &&
        (long)p.seg * p.nseg >= p.Ho))
    return 0;
  if (p.stride == 2) {
    if (!(p.Wo == (p.W + 1) / 2 && p.Ho == (p.H + 1) / 2 && p.H % 2 == 0 && p.W % 2 == 0))  // pad_beg 0
      return 0;
    if (dd_fits<DdS2>(p, 96)) return 2;
    if (dd_fits<DdS3>(p, 256)) return 3;
    return 0;
  }
  if (p.stride == 1 && p.Wo == p.W && p.Ho == p.H && dd_fits<DdF2>(p, 160)) return 1;
  return 0;
}

int dpn_down_ok(const DpnDownParams& p) { return dd_shape(p) != 0; }

hipError_t launch_dpn_down(const DpnDownParams& p, hipStream_t s) {
  const int sh = dd_shape(p);
  if (!sh || !p.x || !p.y || !p.w1 || !p.m1 || !p.i1 || !p.wg || !p.m2 || !p.i2)
    return hipErrorInvalidValue;
  const int segs = p.N * p.nseg;
  const int nsl = p.r / DB_R;
  const dim3 grid((segs + 7) / 8 * 8 * nsl);
  if (sh == 2)
    hipLaunchKernelGGL(dpn_down_rows<DdS2>, grid, dim3(DB_THREADS), dd_geo<DdS2>(p.W).lds, s, p);
  else if (sh == 3)
    hipLaunchKernelGGL(dpn_down_rows<DdS3>, grid, dim3(DB_THREADS), dd_geo<DdS3>(p.W).lds, s, p);
  else
    hipLaunchKernelGGL(dpn_down_rows<DdF2>, grid, dim3(DB_THREADS), dd_geo<DdF2>(p.W).lds, s, p);
  return hipGetLastError();
}

int dpn_block_ok(const DpnBlockParams& p) {
  return p.W > 16 * (DB_TPR - 1) && p.W <= 16 * DB_TPR && p.cin > 0 && p.cin <= 128 &&
         p.cin % 8 == 0 && p.cin <= p.ldx && p.kp3 == DB_R &&
         (p.from_a ? p.cin == DB_R : (p.kp1 >= p.cin && p.kp1 <= 128)) &&
         p.ldx % 8 == 0 && p.ldy % 8 == 0 && p.ldr % 8 == 0 && p.bw <= p.ldr &&
         p.bw <= 8 * (DB_RXS - 2) && p.bw % 8 == 0 && p.bw <= p.cout && p.cout <= 96 && p.cout % 8 == 0 && p.H > 0 &&
         p.N > 0 && p.seg > 0 && p.nseg > 0 && (long)p.seg * p.nseg >= p.H;
}

size_t dpn_block_halo_bytes(const DpnBlockParams& p) {
  return (size_t)p.N * p.nseg * 2 * db_geo(p.W).rowb;
}

hipError_t dpn_trace_read(void* dst, size_t bytes) {
  if (bytes > sizeof(g_db_trace)) bytes = sizeof(g_db_trace);
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_db_trace), bytes, 0, hipMemcpyDeviceToHost);
}

hipError_t launch_dpn_block(const DpnBlockParams& p, hipStream_t s) {
  if (!dpn_block_ok(p) || !p.x || !p.res || !p.y || !p.y2 || !p.wg || !p.w3 || !p.m2 || !p.i2 ||
      !p.m3 || !p.i3 || (!p.from_a && (!p.halo || !p.w1 || !p.m1 || !p.i1)))
    return hipErrorInvalidValue;
  const int lds = db_geo(p.W).lds;
  const dim3 grid(p.N * p.nseg);
  if (p.from_a) {
    hipLaunchKernelGGL(dpn_block_rows<2>, grid, dim3(DB_THREADS), lds, s, p);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(dpn_block_rows<1>, grid, dim3(DB_THREADS), lds, s, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(dpn_block_rows<0>, grid, dim3(DB_THREADS), lds, s, p);
  return hipGetLastError();
}

}  // namespace vox

// Row-streamed grouped 3x3 convolution with a BN+ReLU input prologue: the
// DPN68 `bn_relu_conv(..., cardinality=32)` of every dual-path block
// (dpn_model.py:40-45,49; conv2d with cardinality, models.py:173-203).
//
// Group widths are tiny (DPN68: 4, 8, 16, 32 channels per group), so the op is
// bound by memory and instruction issue, never by the MFMAs (~9..72 MAC per
// byte).  Structure:
//   * a workgroup (4 waves) owns one utterance, a 64-channel chunk (aligned
//     to whole groups) and a segment of output rows, and streams the segment
//     RS output rows at a time.  Input rows pass through a ring of NR LDS row
//     slots; each input element is read from HBM once per segment and gets
//     its BN+ReLU (TF pads AFTER the activation, so halo columns / rows
//     outside the image stay exact zeros) once, while staged;
//   * the new input rows of step j+2 are requested into VGPRs (two register
//     sets) before step j's MFMAs; step j+1's rows are written to the ring
//     after step j's outputs are stored (one barrier per step; NR >= window
//     + new rows keeps the two sets disjoint);
//   * wave w computes output channels [16w, 16w+16) of the chunk with bf16
//     MFMA 16x16x32: for group width <= 16 the 16x16 per-tap weight block is
//     block-diagonal (zeros between groups) and one MFMA covers two taps
//     (K = 2 taps x 16 channels, 5 MFMAs per 16x16 output tile); for group
//     width 32 one MFMA covers one tap of the group's 32 channels (9 MFMAs);
//   * weights are expanded once at load into [C/16][NM][64 lanes][8] so each
//     lane's A fragments are one coalesced 16-B load, kept in registers.
//
// Addressing is built so that a step costs few VALU instructions (the first
// version spent ~490 VALU per wave-step on 64-bit row arithmetic, per-read ring
// modulos and the prologue, and ran VALU-bound at 3.3 TB/s on DPN68 stage 1):
//   * output pixel tiles are 16 columns of ONE output row (TPR tiles per row,
//     the tail lanes of a row masked), so a tile's fragment address is a
//     per-(row, MFMA) base plus a compile-time offset;
//   * ring-row offsets of the step's window rows are wave-uniform (scalar);
//   * LDS image (16-B units): chunk c (8 channels) of column slot x sits in
//     sub-plane c/2 at unit 2x + c%2 (sub-plane stride SPW = 2 mod 16 units):
//     the two lane groups a gfx950 ds_read_b128 pairs read chunks c, c+1 of 8
//     distinct pixels, so fragment reads and the staging stores are
//     conflict-free.  For stride 2 the even padded input columns come first,
//     then the odd ones, so a tap reads 16 consecutive slots;
//   * the prologue runs on packed fp32 pairs, ReLU on the rounded bf16 pairs.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "device_common.h"
#include "kernels.h"

namespace vox {

__device__ uint4 g_gc_zero[1] = {};   // source of the row loads outside the image

namespace {
constexpr int GC_THREADS = 256;

constexpr int GC_MAXT = 8;        // 16-pixel output tiles per step

// geometry shared by the kernel and the host (LDS size)
struct GcGeo {
  int spw, rowb, zero_off, lds;
};
__host__ __device__ constexpr int gc_nr(int S, int RS) { return S == 1 ? 2 * RS + 2 : 4 * RS + 1; }
__host__ __device__ inline GcGeo gc_geo(int W, int S, int RS, int TPR) {
  GcGeo g{};
  int spw = 2 * (W + 2);
  spw += ((2 - spw) % 16 + 16) % 16;   // == 2 (mod 16): conflict-free staging stores
  g.spw = spw;
  g.rowb = 4 * spw * 16;
  g.zero_off = gc_nr(S, RS) * g.rowb;
  // zero line for the invalid tap of the paired-tap MFMA (+ tile offsets), then
  // slack for the masked tail lanes of a row's last tile
  g.lds = g.zero_off + 512 * TPR + 1024;
  return g;
}
}  // namespace

#pragma clang fp contract(off)
template <bool G32, int S, int RS, int TPR>
__global__ __launch_bounds__(GC_THREADS) void gconv3x3_rows(GconvParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NM = G32 ? 9 : 5;                  // MFMAs per 16x16 output tile
  constexpr int NR = gc_nr(S, RS);                 // ring rows
  constexpr int NEW = S * RS;                      // input rows entering per step
  constexpr int WLEN = S * (RS - 1) + 3;           // window rows of a step
  constexpr int NT = RS * TPR;
  static_assert(NT <= GC_MAXT, "tiles per step");
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int col = lane & 15, q = lane >> 4;
  const int n = blockIdx.x / p.nseg;
  const int sgi = blockIdx.x - n * p.nseg;
  const int c0 = blockIdx.y * 64;
  const int ho0 = sgi * p.seg;
  const int ho1 = min(ho0 + p.seg, p.Ho);
  if (ho0 >= ho1) return;
  const int Wi = p.W, H = p.H;
  const GcGeo geo = gc_geo(Wi, S, RS, TPR);
  const int ROWB = geo.rowb, SPW = geo.spw;
  const int E = (Wi + 3) >> 1;                     // even padded columns (stride 2)
  // LDS column slot of padded input column xp (0 = left pad, Wi + 1 = right pad)
  auto slot_of = [&](int xp) { return S == 1 ? xp : ((xp & 1) ? E + (xp >> 1) : (xp >> 1)); };

  // ---- staging roles: unit u = tid + 256 i -> (new row rr, column x, chunk sub)
  // units per thread: NEW rows of at most min(80, 16 S TPR) columns, 8 units each
  constexpr int WMAX = 16 * S * TPR < 80 ? 16 * S * TPR : 80;
  constexpr int U = (NEW * WMAX * 8 + GC_THREADS - 1) / GC_THREADS;
  const int upr = Wi * 8;                          // units per input row
  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(p.x) + (size_t)n * H * Wi * p.ldx + c0;
  // per unit: new-row index (-1: none), element offset within the utterance
  // (32 bits: H * W * ldx of one utterance stays far below 2^31), LDS offset
  int srr[U], soff[U], slds[U];
#pragma unroll
  for (int i = 0; i < U; ++i) {
    const int u = tid + GC_THREADS * i;
    const int rr = u / upr, rem = u - rr * upr;
    const int x = rem >> 3, sub = rem & 7;
    srr[i] = rr < NEW ? rr : -1;
    soff[i] = (rr * Wi + x) * p.ldx + sub * 8;
    slds[i] = ((sub >> 1) * SPW + 2 * slot_of(x + 1) + (sub & 1)) * 16;
  }
  // this thread's prologue channels: sub = tid & 7 for every unit (256 % 8 == 0)
  f32x4 bm0, bm1, bi0, bi1;
  const bool pro = p.in_mean != nullptr;
  {
    const int cb = c0 + (tid & 7) * 8;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      bm0[e] = pro ? -p.in_mean[cb + e] : 0.f;
      bm1[e] = pro ? -p.in_mean[cb + 4 + e] : 0.f;
      bi0[e] = pro ? p.in_inv[cb + e] : 1.f;
      bi1[e] = pro ? p.in_inv[cb + 4 + e] : 1.f;
    }
  }
  const int rstride = Wi * p.ldx;                  // elements per input row
  // load the NEW input rows starting at r0.  Every load is issued (rows outside
  // the image read a zero line): a conditional load merges into the prefetch
  // registers through a copy, and the copy waits for the data at once
  // (s_waitcnt vmcnt(0) right after the loads: no prefetch at all).
  const uint4* zline = g_gc_zero;
  auto load_rows = [&](int r0, uint4 (&v)[U]) __attribute__((always_inline)) {
    const bf16_t* __restrict__ Xr = X + (ptrdiff_t)r0 * rstride;   // wave-uniform base
#pragma unroll
    for (int i = 0; i < U; ++i) {
      const int row = r0 + srr[i];
      const bool ok = srr[i] >= 0 && (unsigned)row < (unsigned)H;
      v[i] = *(ok ? reinterpret_cast<const uint4*>(Xr + soff[i]) : zline);
    }
  };
  // ring byte offset of input row r (r >= -2)
  auto ring_off = [&](int r) { return ((r + 2 * NR) % NR) * ROWB; };
  auto store_rows = [&](int r0, const uint4 (&v)[U]) __attribute__((always_inline)) {
    const int rb = (r0 + 2 * NR) % NR;
#pragma unroll
    for (int i = 0; i < U; ++i) {
      if (srr[i] < 0) continue;
      int sl = rb + srr[i];
      sl = sl >= NR ? sl - NR : sl;
      const int row = r0 + srr[i];
      bf16x8 o = __builtin_bit_cast(bf16x8, v[i]);
      if (pro && (unsigned)row < (unsigned)H) {
        // relu((x - m) * inv) on fp32 pairs, rounded to bf16, ReLU on the bf16 bits
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        const vu32x4 w = __builtin_bit_cast(vu32x4, v[i]);
        bf16x8 r;
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          f32x2 xv = {__builtin_bit_cast(float, w[h] << 16), __builtin_bit_cast(float, w[h] & 0xFFFF0000u)};
          const f32x4& bm = h < 2 ? bm0 : bm1;
          const f32x4& bi = h < 2 ? bi0 : bi1;
          const f32x2 m2 = {bm[2 * (h & 1)], bm[2 * (h & 1) + 1]};
          const f32x2 i2 = {bi[2 * (h & 1)], bi[2 * (h & 1) + 1]};
          xv = (xv + m2) * i2;
          r[2 * h] = (bf16_t)xv[0];
          r[2 * h + 1] = (bf16_t)xv[1];
        }
        o = relu_bf16(r);
      }
      *reinterpret_cast<bf16x8*>(smem + sl * ROWB + slds[i]) = o;
    }
  };

  // ---- compute roles: wave = 16-channel slab; lane column = pixel of a tile
  const int sgw = blockIdx.y * 4 + wave;
  bf16x8 a[NM];
  {
    const bf16_t* wp = reinterpret_cast<const bf16_t*>(p.w) + ((size_t)sgw * NM * 64 + lane) * 8;
#pragma unroll
    for (int m = 0; m < NM; ++m) a[m] = ld16(wp + m * 512);
  }
  // per MFMA slot m: byte offset of this lane's B fragment within a ring row
  // (its tap's column, output column col of the row's first tile)
  int lofs[NM];
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    const int tap = G32 ? m : 2 * m + (q >> 1);
    const int tt = tap < 9 ? tap : 8;
    const int kx = tt % 3;
    const int chunk = G32 ? 4 * (wave >> 1) + q : 2 * wave + (q & 1);
    lofs[m] = ((chunk >> 1) * SPW + 2 * slot_of(col * S + kx - p.pw + 1) + (chunk & 1)) * 16;
  }

  // zero the pad columns of every ring row, and the zero line
  for (int u = tid; u < NR * 16; u += GC_THREADS) {
    const int row = u >> 4, sp = (u >> 2) & 3, e = u & 3;
    const int xp = (e >> 1) ? Wi + 1 : 0;
    *reinterpret_cast<uint4*>(smem + row * ROWB + (sp * SPW + 2 * slot_of(xp) + (e & 1)) * 16) =
        uint4{0u, 0u, 0u, 0u};
  }
  for (int u = tid; u < 32 * TPR; u += GC_THREADS)
    *reinterpret_cast<uint4*>(smem + geo.zero_off + u * 16) = uint4{0u, 0u, 0u, 0u};
  // the first step's window: input rows [ho0*S - ph, ho0*S - ph + WLEN), in
  // groups of NEW rows (a group's rows past the window go to ring slots of
  // later steps, rewritten before they are read)
  {
    const int win0 = ho0 * S - p.ph;
    for (int r = 0; r < WLEN; r += NEW) {
      uint4 v[U];
      load_rows(win0 + r, v);
      store_rows(win0 + r, v);
    }
  }
  __syncthreads();

  bf16_t* __restrict__ Y = reinterpret_cast<bf16_t*>(p.y) + (size_t)n * p.Ho * p.Wo * p.ldy + c0 +
                           16 * wave + 4 * q;
  const int Wo = p.Wo;
  // Input rows are requested two steps before they enter the ring (register
  // sets pf[j & 1] hold step j's new rows); the ring receives step j+1's rows
  // at the end of step j.
  uint4 pf[2][U];
  // first input row step hs adds to the window
  auto nxt_of = [&](int hs) { return hs * S - p.ph + WLEN - NEW; };
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  // (rows past the segment are fetched too -- unconditional, see load_rows --
  // and never staged)
  load_rows(nxt_of(ho0 + RS), pf[1]);
  auto step = [&](auto PS, int hs) __attribute__((always_inline)) {
    constexpr int PI = decltype(PS)::value;
    load_rows(nxt_of(hs + 2 * RS), pf[PI]);   // step j+2: same parity
    // the scheduler would otherwise sink the loads below the MFMAs, next to
    // the wait for them
    __builtin_amdgcn_sched_barrier(0);

    const int wb = hs * S - p.ph;                  // window row 0
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int orow = 0; orow < RS; ++orow) {
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        // the lane's fragment address for tile (orow, 0); the row's tiles
        // follow at 512 B (16 column slots)
        int addr;
        if (G32 || (m != 1 && m != 4)) {
          const int ky = G32 ? m / 3 : (2 * m) / 3;
          addr = __builtin_amdgcn_readfirstlane(ring_off(wb + orow * S + ky)) + lofs[m];
        } else if (m == 1) {
          // taps 2 (window row 0) and 3 (row 1) of the two lane halves
          const int r0 = __builtin_amdgcn_readfirstlane(ring_off(wb + orow * S));
          const int r1 = __builtin_amdgcn_readfirstlane(ring_off(wb + orow * S + 1));
          addr = ((q >> 1) ? r1 : r0) + lofs[m];
        } else {
          // taps 8 (window row 2) and 9 (none: the zero line) of the two halves
          const int r2 = __builtin_amdgcn_readfirstlane(ring_off(wb + orow * S + 2));
          addr = (q >> 1) ? geo.zero_off : r2 + lofs[m];
        }
#pragma unroll
        for (int tc = 0; tc < TPR; ++tc) {
          const bf16x8 b = *reinterpret_cast<const bf16x8*>(smem + addr + 512 * tc);
          acc[orow * TPR + tc] = mfma_step(a[m], b, acc[orow * TPR + tc]);
        }
      }
    }
#pragma unroll
    for (int orow = 0; orow < RS; ++orow) {
      const int ho = hs + orow;
      if (ho >= ho1) break;   // uniform
      auto cvt = [&](int tc) __attribute__((always_inline)) {
        const f32x4& v = acc[orow * TPR + tc];
        bf16x4 o;
        o[0] = (bf16_t)v[0]; o[1] = (bf16_t)v[1];
        o[2] = (bf16_t)v[2]; o[3] = (bf16_t)v[3];
        return __builtin_bit_cast(uint2, o);
      };
      if ((p.ldy & 7) != 0) {   // (8-B aligned rows only: one 8-B store per tile)
#pragma unroll
        for (int tc = 0; tc < TPR; ++tc) {
          const int oc = 16 * tc + col;
          if (oc < Wo) *reinterpret_cast<uint2*>(Y + ((size_t)ho * Wo + oc) * p.ldy) = cvt(tc);
        }
        continue;
      }
#pragma unroll
      for (int tc = 0; tc + 1 < TPR; tc += 2) {
        // tiles tc, tc + 1: a half-row exchange per dword gives lane (col, q)
        // 8 contiguous channels 8 (q / 2) of tile tc + q % 2 (16-B stores)
        const uint2 d0 = cvt(tc), d1 = cvt(tc + 1);
        const auto s0 = __builtin_amdgcn_permlane16_swap(d0.x, d1.x, false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(d0.y, d1.y, false, false);
        const int oc = 16 * (tc + (q & 1)) + col;
        if (oc < Wo)
          *reinterpret_cast<uint4*>(Y - 4 * q + 8 * (q >> 1) + ((size_t)ho * Wo + oc) * p.ldy) =
              make_uint4(s0[0], s1[0], s0[1], s1[1]);
      }
      if constexpr (TPR % 2 == 1) {
        const int oc = 16 * (TPR - 1) + col;
        if (oc < Wo) *reinterpret_cast<uint2*>(Y + ((size_t)ho * Wo + oc) * p.ldy) = cvt(TPR - 1);
      }
    }
    // step j+1's rows enter the ring (staging them before the stores above,
    // so that the wait for them has fewer younger stores, measured slower)
    if (hs + RS < ho1) store_rows(nxt_of(hs + RS), pf[PI ^ 1]);
    __syncthreads();
  };
  for (int hs = ho0; hs < ho1; hs += 2 * RS) {
    step(P0{}, hs);
    if (hs + RS < ho1) step(P1{}, hs + RS);
  }
}

// 16-column tiles of one output row, TPR per row, RS rows per step (<= 8 tiles)
static int gconv_tpr(const GconvParams& p) { return (p.Wo + 15) / 16; }

int gconv_rs(const GconvParams& p) {
  const int tpr = gconv_tpr(p);
  if (p.rs_force > 0 && p.sh == 1 && p.rs_force * tpr <= GC_MAXT) return p.rs_force;
  if (p.sh == 2) return tpr >= 2 ? 1 : 2;
  // one-tile rows (DPN68 stage 4, W = 10): 2 rows per step, 138 vs 155 us at 8
  // (VOXEMB_GCONV_RS A/B, gpurun_out/gcrs)
  return tpr >= 5 ? 1 : tpr >= 3 ? 2 : tpr == 2 ? 4 : 2;
}

int gconv_ok(const GconvParams& p) {
  return p.C % 64 == 0 && (p.gw == 4 || p.gw == 8 || p.gw == 16 || p.gw == 32) &&
         p.Wo >= 1 && p.Wo <= 80 && p.W <= 80 && (p.sh == 1 || p.sh == 2) && p.ph >= 0 &&
         p.ph <= 1 && p.pw >= 0 && p.pw <= 1 && p.ldx % 8 == 0 && p.ldy % 4 == 0 &&
         (p.sh == 1 ? (p.W == p.Wo && p.H == p.Ho)
                    : (p.Wo == (p.W + 1) / 2 && p.Ho == (p.H + 1) / 2));
}

int gconv_lds(const GconvParams& p) {
  return gc_geo(p.W, p.sh, gconv_rs(p), gconv_tpr(p)).lds;
}

template <bool G32, int S, int RS, int TPR>
static hipError_t gconv_t(const GconvParams& p, hipStream_t s) {
  const dim3 grid(p.N * p.nseg, p.C / 64);
  hipLaunchKernelGGL((gconv3x3_rows<G32, S, RS, TPR>), grid, dim3(GC_THREADS), gconv_lds(p), s, p);
  return hipGetLastError();
}

template <bool G32>
static hipError_t gconv_g(const GconvParams& p, hipStream_t s) {
  const int tpr = gconv_tpr(p), rs = gconv_rs(p);
#define GC_CASE(S_, RS_, TPR_) \
  if (p.sh == S_ && rs == RS_ && tpr == TPR_) return gconv_t<G32, S_, RS_, TPR_>(p, s);
  GC_CASE(1, 1, 5) GC_CASE(1, 2, 4) GC_CASE(1, 2, 3) GC_CASE(1, 4, 2) GC_CASE(1, 8, 1)
  GC_CASE(1, 2, 2) GC_CASE(1, 1, 2) GC_CASE(1, 1, 1) GC_CASE(1, 1, 3) GC_CASE(1, 1, 4)
  GC_CASE(1, 2, 1) GC_CASE(1, 4, 1)
  GC_CASE(2, 1, 5) GC_CASE(2, 1, 4) GC_CASE(2, 1, 3) GC_CASE(2, 1, 2) GC_CASE(2, 2, 1)
#undef GC_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_gconv(const GconvParams& p, hipStream_t s) {
  if (!gconv_ok(p) || p.seg <= 0 || p.nseg <= 0 || (long)p.seg * p.nseg < p.Ho)
    return hipErrorInvalidValue;
  return p.gw == 32 ? gconv_g<true>(p, s) : gconv_g<false>(p, s);
}

}  // namespace vox

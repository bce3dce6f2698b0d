// Row-streamed grouped 3x3 convolution with a BN+ReLU input prologue: the
// DPN68 `bn_relu_conv(..., cardinality=32)` of every dual-path block
// (dpn_model.py:40-45,49; conv2d with cardinality, models.py:173-203).
//
// Group widths are tiny (DPN68: 4, 8, 16, 32 channels per group), so the op is
// HBM-bound (~9..72 MAC per byte); the generic implicit GEMM spent 17 ms on a
// 28 GFLOP stage-1 launch because a 16-row MFMA tile carried one 4-channel
// group.  Here:
//   * a workgroup (4 waves) owns one utterance, a 64-channel chunk (aligned
//     to whole groups) and a segment of output rows, and streams the segment
//     RS output rows at a time.  Input rows pass through a ring of NR LDS row
//     slots; each input element is read from HBM once per segment and gets
//     its BN+ReLU (TF pads AFTER the activation, so halo columns / rows
//     outside the image stay exact zeros) once, while staged;
//   * the next step's new input rows are fetched into VGPRs before the
//     current step's MFMAs and written to the ring afterwards (one barrier per
//     step; NR >= window + new rows keeps the two sets disjoint);
//   * wave w computes output channels [16w, 16w+16) of the chunk with bf16
//     MFMA 16x16x32: for group width <= 16 the 16x16 per-tap weight block is
//     block-diagonal (zeros between groups) and one MFMA covers two taps
//     (K = 2 taps x 16 channels, 5 MFMAs per 16x16 output tile); for group
//     width 32 one MFMA covers one tap of the group's 32 channels (9 MFMAs).
//     The wasted zero products are free: the op is bound by HBM, not MFMA.
//   * weights are expanded once at load into [C/16][NM][64 lanes][8] so each
//     lane's A fragments are one coalesced 16-B load, kept in registers.
// LDS pixel stride is 144 B (128 data + 16 pad, an odd number of 16-B units)
// so the 16 pixels of a ds_read_b128 quarter-wave hit distinct banks.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_common.h"
#include "kernels.h"

namespace vox {

namespace {
constexpr int GC_NT = 5;        // 16-pixel output tiles per step (RS * Wo <= 80)
constexpr int GC_PSTR = 144;    // LDS bytes per staged pixel (64 channels + pad)
constexpr int GC_THREADS = 256;
}  // namespace

#pragma clang fp contract(off)
template <bool G32, int S, int RS>
__global__ __launch_bounds__(GC_THREADS) void gconv3x3_rows(GconvParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NM = G32 ? 9 : 5;                  // MFMAs per 16x16 output tile
  constexpr int NR = S == 1 ? 2 * RS + 2 : 4 * RS + 1;   // ring rows
  constexpr int NEW = S * RS;                       // input rows entering per step
  constexpr int RPC = S == 1 ? RS : 2;              // rows per staging call
  constexpr int U = S == 1 ? 3 : 5;                 // 16-B units per thread per call
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
  const int Wi = p.W;
  const int SLOT = (Wi + 2) * GC_PSTR;
  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(p.x) + (size_t)n * p.H * Wi * p.ldx + c0;

  // ---- staging roles: thread owns channel unit `sub` of pixels pidx_i
  const int sub = tid & 7;
  int prow[U], pcol[U];
#pragma unroll
  for (int i = 0; i < U; ++i) {
    const int pidx = (tid >> 3) + 32 * i;
    prow[i] = pidx / Wi;
    pcol[i] = pidx - prow[i] * Wi;
  }
  float bm[8], bi[8];
  const bool pro = p.in_mean != nullptr;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    bm[e] = pro ? p.in_mean[c0 + sub * 8 + e] : 0.f;
    bi[e] = pro ? p.in_inv[c0 + sub * 8 + e] : 1.f;
  }
  auto load_call = [&](int r0, int nr, uint4 (&v)[U]) {
#pragma unroll
    for (int i = 0; i < U; ++i) {
      const int row = r0 + prow[i];
      v[i] = uint4{0u, 0u, 0u, 0u};
      if (prow[i] < nr && row >= 0 && row < p.H)
        v[i] = *reinterpret_cast<const uint4*>(X + ((size_t)row * Wi + pcol[i]) * p.ldx + sub * 8);
    }
  };
  auto store_call = [&](int r0, int nr, const uint4 (&v)[U]) {
#pragma unroll
    for (int i = 0; i < U; ++i) {
      if (prow[i] >= nr) continue;
      const int row = r0 + prow[i];
      bf16x8 o = __builtin_bit_cast(bf16x8, v[i]);
      if (pro) {
        if (row >= 0 && row < p.H) {
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = (bf16_t)fmaxf(((float)o[e] - bm[e]) * bi[e], 0.f);
        }  // else: zero padding stays zero (v was zero-filled)
      }
      const int slot = (row + NR) % NR;
      *reinterpret_cast<bf16x8*>(smem + slot * SLOT + (pcol[i] + 1) * GC_PSTR + sub * 16) = o;
    }
  };

  // ---- compute roles: wave = 16-channel slab; lane column = pixel of a tile
  const int sg = blockIdx.y * 4 + wave;
  bf16x8 a[NM];
  {
    const bf16_t* wp = reinterpret_cast<const bf16_t*>(p.w) + ((size_t)sg * NM * 64 + lane) * 8;
#pragma unroll
    for (int m = 0; m < NM; ++m) a[m] = ld16(wp + m * 512);
  }
  const int P = RS * p.Wo;   // output pixels per step
  int orow[GC_NT], ocol[GC_NT];
#pragma unroll
  for (int j = 0; j < GC_NT; ++j) {
    const int pp = min(16 * j + col, P - 1);
    orow[j] = pp / p.Wo;
    ocol[j] = pp - orow[j] * p.Wo;
  }
  // per (tap-slot m): row offset and byte offset within the slot
  int kyq[NM], cofs[NM];
  bool tapok[NM];
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    const int tap = G32 ? m : 2 * m + (q >> 1);
    tapok[m] = tap < 9;
    const int tt = tap < 9 ? tap : 0;
    kyq[m] = tt / 3;
    const int kx = tt - 3 * (tt / 3);
    const int coff = G32 ? (32 * (wave >> 1) + 8 * q) * 2 : (16 * wave + 8 * (q & 1)) * 2;
    cofs[m] = (kx - p.pw + 1) * GC_PSTR + coff;
  }

  // zero the halo columns of every ring slot (never written by staging)
  for (int u = tid; u < NR * 2 * 8; u += GC_THREADS) {
    const int slot = u >> 4, side = (u >> 3) & 1, c = u & 7;
    *reinterpret_cast<uint4*>(smem + slot * SLOT + (side ? (Wi + 1) * GC_PSTR : 0) + c * 16) =
        uint4{0u, 0u, 0u, 0u};
  }
  // the first step's window: input rows [ho0*S - ph, ho0*S - ph + S*(RS-1) + 2]
  const int win0 = ho0 * S - p.ph;
  const int wlen = S * (RS - 1) + 3;
  for (int r = 0; r < wlen; r += RPC) {
    uint4 v[U];
    load_call(win0 + r, min(RPC, wlen - r), v);
    store_call(win0 + r, min(RPC, wlen - r), v);
  }
  __syncthreads();

  bf16_t* __restrict__ Y = reinterpret_cast<bf16_t*>(p.y) + (size_t)n * p.Ho * p.Wo * p.ldy + c0 +
                           16 * wave + 4 * q;
  for (int hs = ho0; hs < ho1; hs += RS) {
    // prefetch the rows the next step adds: [win_end(hs)+1, win_end(hs)+NEW]
    const int nxt = hs * S - p.ph + wlen;
    const bool more = hs + RS < ho1;
    uint4 pf[(NEW + RPC - 1) / RPC][U];
#pragma unroll
    for (int c = 0; c < (NEW + RPC - 1) / RPC; ++c)
      if (more) load_call(nxt + c * RPC, min(RPC, NEW - c * RPC), pf[c]);

    f32x4 acc[GC_NT];
#pragma unroll
    for (int j = 0; j < GC_NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < GC_NT; ++j) {
      if (16 * j >= P) break;   // uniform
      const int rbase = (hs + orow[j]) * S - p.ph + NR;
      const int cbase = ocol[j] * S * GC_PSTR;
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        const int slot = (rbase + kyq[m]) % NR;
        bf16x8 b = *reinterpret_cast<const bf16x8*>(smem + slot * SLOT + cbase + cofs[m]);
        if (!G32 && !tapok[m]) b = bf16x8{};
        acc[j] = mfma_step(a[m], b, acc[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < GC_NT; ++j) {
      if (16 * j >= P) break;
      const int pp = 16 * j + col;
      const int ho = hs + orow[j];
      if (pp < P && ho < ho1) {
        bf16x4 o;
        o[0] = (bf16_t)acc[j][0]; o[1] = (bf16_t)acc[j][1];
        o[2] = (bf16_t)acc[j][2]; o[3] = (bf16_t)acc[j][3];
        *reinterpret_cast<bf16x4*>(Y + ((size_t)ho * p.Wo + ocol[j]) * p.ldy) = o;
      }
    }
#pragma unroll
    for (int c = 0; c < (NEW + RPC - 1) / RPC; ++c)
      if (more) store_call(nxt + c * RPC, min(RPC, NEW - c * RPC), pf[c]);
    __syncthreads();
  }
}

int gconv_ok(const GconvParams& p) {
  const int rs = p.Wo > 0 ? 80 / p.Wo : 0;
  return p.C % 64 == 0 && (p.gw == 4 || p.gw == 8 || p.gw == 16 || p.gw == 32) &&
         p.Wo >= 1 && p.Wo <= 80 && (p.sh == 1 || p.sh == 2) && p.ph >= 0 && p.ph <= 1 &&
         p.pw >= 0 && p.pw <= 1 && p.ldx % 8 == 0 && p.ldy % 4 == 0 &&
         (p.sh == 1 ? (p.W == p.Wo && p.H == p.Ho && rs >= 1)
                    : (p.Wo == (p.W + 1) / 2 && p.Ho == (p.H + 1) / 2 && p.W + 2 <= 162));
}

// rows per step: RS * Wo <= 80 (5 tiles); stride 2 streams one output row
int gconv_rs(const GconvParams& p) {
  if (p.sh == 2) return 1;
  const int r = 80 / p.Wo;
  return r >= 8 ? 8 : r >= 4 ? 4 : r >= 2 ? 2 : 1;
}

int gconv_lds(const GconvParams& p) {
  const int rs = gconv_rs(p);
  const int nr = p.sh == 1 ? 2 * rs + 2 : 4 * rs + 1;
  return nr * (p.W + 2) * GC_PSTR;
}

template <bool G32, int S, int RS>
static hipError_t gconv_t(const GconvParams& p, hipStream_t s) {
  const dim3 grid(p.N * p.nseg, p.C / 64);
  hipLaunchKernelGGL((gconv3x3_rows<G32, S, RS>), grid, dim3(GC_THREADS), gconv_lds(p), s, p);
  return hipGetLastError();
}

template <bool G32>
static hipError_t gconv_g(const GconvParams& p, hipStream_t s) {
  if (p.sh == 2) return gconv_t<G32, 2, 1>(p, s);
  switch (gconv_rs(p)) {
    case 8: return gconv_t<G32, 1, 8>(p, s);
    case 4: return gconv_t<G32, 1, 4>(p, s);
    case 2: return gconv_t<G32, 1, 2>(p, s);
    default: return gconv_t<G32, 1, 1>(p, s);
  }
}

hipError_t launch_gconv(const GconvParams& p, hipStream_t s) {
  if (!gconv_ok(p) || p.seg <= 0 || p.nseg <= 0 || (long)p.seg * p.nseg < p.Ho)
    return hipErrorInvalidValue;
  return p.gw == 32 ? gconv_g<true>(p, s) : gconv_g<false>(p, s);
}

}  // namespace vox

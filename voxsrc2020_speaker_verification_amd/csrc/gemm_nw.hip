// Narrow 1x1 GEMM with weights resident in LDS, for the DPN68 1x1 convs whose
// whole weight matrix is small (K <= 256 input channels, <= 192 output
// channels: the bn_relu_conv 1x1a/1x1c of dpn_model.py:40-87 with their
// BN+ReLU input prologue, the residual add into the [res | dense] prefix and
// the dense channels appended past `ysplit`).
//
// conv1x1_rr (kernels.hip) handles these with one 64-pixel tile per wave and
// streams every weight fragment from L2 per tile pair: for K = 256 x 160 couts
// that is 80 KB of L2 reads per 32 KB of activations, and each wave's tile
// pairs wait on those loads in turn (1.9 TB/s).  Here a persistent workgroup
// copies the weights (paired-row layout, rows padded to an odd number of 16-B
// units so fragment reads are conflict-free) and the BN / prologue tables into
// LDS once; its 8 waves then stream 16*WPX-pixel chunks: input fragments
// global -> registers with the prologue applied in registers, every cout tile
// pair from the LDS weights, the epilogue (BN, residual below ysplit, ReLU) and
// 16-B stores of 8 consecutive channels per lane.  Accumulation order (K
// chunks of 32 in increasing order) and the epilogue roundings (BN, residual
// and ReLU as separate steps, no contraction) are those of the other 1x1
// kernels.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_common.h"
#include "kernels.h"

namespace vox {

namespace {
constexpr int NW_NT = 512;   // 8 waves
}

#pragma clang fp contract(off)
// KS = k-steps of 32 (K <= 32 KS), NP = cout tile pairs (coutp <= 32 NP),
// WPX = 16-pixel tiles per chunk
template <int KS, int NP, int WPX>
__global__ __launch_bounds__(NW_NT) void conv1x1_nw(ConvParams p) {
  constexpr int KW = KS * 32;          // padded K of an LDS weight row
  constexpr int WSTR = KW + 8;         // row stride (elements): odd 16-B units
  constexpr int ROWS = NP * 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* wl = reinterpret_cast<bf16_t*>(smem);
  float* bnm = reinterpret_cast<float*>(smem + ROWS * WSTR * 2);
  float* bni = bnm + ROWS;
  float* pm = bni + ROWS;               // prologue tables [KW]
  float* pi = pm + KW;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4, kl = 8 * g;

  // ---- resident operands: weights (zero past kp / past the padded rows), BN, prologue
  const bf16_t* __restrict__ Wt = reinterpret_cast<const bf16_t*>(p.w);
  for (int i = tid; i < ROWS * (KW / 8); i += NW_NT) {
    const int r = i / (KW / 8), c = 8 * (i - r * (KW / 8));
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r < p.coutp && c < p.kp) v = *reinterpret_cast<const uint4*>(Wt + (size_t)r * p.kp + c);
    *reinterpret_cast<uint4*>(wl + r * WSTR + c) = v;
  }
  const bool aff = (p.flags & EPI_AFFINE) != 0;
  for (int c = tid; c < ROWS; c += NW_NT) {
    bnm[c] = (aff && c < p.Cout) ? p.mean[c] : 0.f;
    bni[c] = (aff && c < p.Cout) ? p.inv[c] : 0.f;
  }
  const bool pro = p.in_mean != nullptr;
  for (int c = tid; c < KW; c += NW_NT) {
    pm[c] = (pro && c < p.Cin) ? p.in_mean[c] : 0.f;
    pi[c] = (pro && c < p.Cin) ? p.in_inv[c] : 0.f;
  }
  __syncthreads();

  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(p.x);
  const bf16_t* __restrict__ R = reinterpret_cast<const bf16_t*>(p.res);
  bf16_t* __restrict__ Y = reinterpret_cast<bf16_t*>(p.y);
  bf16_t* __restrict__ Y2 = reinterpret_cast<bf16_t*>(p.y2);
  const int flags = p.flags;
  const int M = p.N * p.Ho * p.Wo;
  const int HoWo = p.Ho * p.Wo;
  const int nchunks = (M + 16 * WPX - 1) / (16 * WPX);
  const int npair = (p.Cout + 31) / 32;   // pairs holding real channels

  for (int ck = blockIdx.x * 8 + wave; ck < nchunks; ck += gridDim.x * 8) {
    bool pv[WPX];
    size_t pix[WPX];
    bf16x8 b[KS][WPX];
#pragma unroll
    for (int j = 0; j < WPX; ++j) {
      const int pp = ck * 16 * WPX + 16 * j + col;
      pv[j] = pp < M;
      const int q = pv[j] ? pp : 0;
      pix[j] = (size_t)q;
      const int n = q / HoWo, r = q - n * HoWo;
      const int ho = r / p.Wo, wo = r - ho * p.Wo;
      const bf16_t* xp = X + (((size_t)n * p.H + ho * p.sh) * p.W + wo * p.sw) * p.ldx;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int c = 32 * s + kl;
        b[s][j] = (pv[j] && c < p.Cin) ? ld16(xp + c) : bf16x8{};
      }
    }
    if (pro) {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int c = 32 * s + kl;
        const f32x4 m0 = *reinterpret_cast<const f32x4*>(pm + c);
        const f32x4 m1 = *reinterpret_cast<const f32x4*>(pm + c + 4);
        const f32x4 i0 = *reinterpret_cast<const f32x4*>(pi + c);
        const f32x4 i1 = *reinterpret_cast<const f32x4*>(pi + c + 4);
#pragma unroll
        for (int j = 0; j < WPX; ++j) {
          // channels past Cin stay zero (m = inv = 0: relu(0) = 0)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            b[s][j][e] = (bf16_t)fmaxf(((float)b[s][j][e] - m0[e]) * i0[e], 0.f);
            b[s][j][4 + e] = (bf16_t)fmaxf(((float)b[s][j][4 + e] - m1[e]) * i1[e], 0.f);
          }
        }
      }
    }
    // every residual fragment of the chunk requested with its inputs, so
    // their latencies overlap (the pairs below do not wait one by one)
    bf16x8 rvs[NP][WPX];
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const int ch = 32 * q + 8 * g;
#pragma unroll
      for (int j = 0; j < WPX; ++j)
        rvs[q][j] = ((flags & EPI_RES) && q < npair && pv[j] && ch < p.Cout && ch < p.ysplit)
                        ? ld16(R + pix[j] * p.ldr + ch) : bf16x8{};
    }
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      if (q >= npair) break;
      const int ch = 32 * q + 8 * g;
      const bf16x8* rv = rvs[q];
      f32x4 acc[2][WPX];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int j = 0; j < WPX; ++j) acc[u][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      const bf16_t* w0 = wl + ((2 * q) * 16 + col) * WSTR + kl;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(w0 + 32 * s);
        const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(w0 + 16 * WSTR + 32 * s);
#pragma unroll
        for (int j = 0; j < WPX; ++j) {
          acc[0][j] = mfma_step(a0, b[s][j], acc[0][j]);
          acc[1][j] = mfma_step(a1, b[s][j], acc[1][j]);
        }
      }
      if (ch >= p.Cout) continue;
      const f32x4 m0 = *reinterpret_cast<const f32x4*>(bnm + ch);
      const f32x4 m1 = *reinterpret_cast<const f32x4*>(bnm + ch + 4);
      const f32x4 i0 = *reinterpret_cast<const f32x4*>(bni + ch);
      const f32x4 i1 = *reinterpret_cast<const f32x4*>(bni + ch + 4);
#pragma unroll
      for (int j = 0; j < WPX; ++j) {
        if (!pv[j]) continue;
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[0][j][e];
          v[4 + e] = acc[1][j][e];
        }
        if (flags & EPI_PRE_RELU) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        if (aff) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = (v[e] - m0[e]) * i0[e];
            v[4 + e] = (v[4 + e] - m1[e]) * i1[e];
          }
        }
        if (flags & EPI_RES) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += (float)rv[j][e];
        }
        if (flags & EPI_RELU) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (bf16_t)v[e];
        bf16_t* dst = ch < p.ysplit ? Y + pix[j] * p.ldy + ch : Y2 + pix[j] * p.ldy2 + (ch - p.ysplit);
        *reinterpret_cast<uint4*>(dst) = __builtin_bit_cast(uint4, o);
      }
    }
  }
}

namespace {
int nw_lds(int ks, int np) { return np * 32 * (ks * 32 + 8) * 2 + 8 * np * 32 + 8 * ks * 32; }
}

int conv1x1_nw_ok(const ConvParams& p) {
  if (p.kh != 1 || p.kw != 1 || p.groups != 1 || p.ph || p.pw) return 0;
  if (p.flags & EPI_PARTIAL) return 0;
  if (p.x2 || p.Cout % 8 || p.ldy % 8 || p.ldx % 8) return 0;
  if (p.ysplit < (1 << 30) && (p.ysplit % 8 || p.ldy2 % 8)) return 0;
  if ((p.flags & EPI_RES) && (!p.res || p.ldr % 8)) return 0;
  if ((p.flags & EPI_AFFINE) && (!p.mean || !p.inv)) return 0;
  if (p.in_mean && !p.in_inv) return 0;
  const int ks = (p.Cin + 31) / 32, np = (p.Cout + 31) / 32;
  if (!((ks == 4 && np <= 4) || (ks == 8 && np <= 6))) return 0;
  return nw_lds(ks, np) <= 160 * 1024;
}

hipError_t launch_conv1x1_nw(const ConvParams& p, int num_cu, hipStream_t s) {
  if (!conv1x1_nw_ok(p)) return hipErrorInvalidValue;
  const int ks = (p.Cin + 31) / 32, np = (p.Cout + 31) / 32;
  const int lds = nw_lds(ks, np);
  const int per_cu = (160 * 1024) / lds >= 2 ? 2 : 1;
  const int M = p.N * p.Ho * p.Wo;
  // 32-pixel chunks (input fragments KS * WPX * 4 VGPRs, residuals NP * WPX * 4)
  const int wpx = 2;
  const int nchunks = (M + 16 * wpx - 1) / (16 * wpx);
  int G = num_cu * per_cu;
  const int need = (nchunks + 7) / 8;
  if (G > need) G = need;
#define NW_L(K, P)                                                                          \
  if (ks == K && np == P) {                                                                 \
    hipLaunchKernelGGL((conv1x1_nw<K, P, 2>), dim3(G), dim3(NW_NT), lds, s, p);         \
    return hipGetLastError();                                                               \
  }
  NW_L(4, 1) NW_L(4, 2) NW_L(4, 3) NW_L(4, 4)
  NW_L(8, 1) NW_L(8, 2) NW_L(8, 3) NW_L(8, 4) NW_L(8, 5) NW_L(8, 6)
#undef NW_L
  return hipErrorInvalidValue;
}

}  // namespace vox

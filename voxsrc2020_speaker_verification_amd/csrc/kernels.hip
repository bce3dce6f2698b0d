// gfx950 (CDNA4) kernels of the embedding-extraction hot path.
//
//  * conv_igemm   -- NHWC implicit-GEMM convolution on MFMA (bf16 16x16x32 or
//                    f32 16x16x4), BN/ReLU/residual epilogues, split outputs
//                    (free channel concat), hierarchical-add and BN+ReLU
//                    prologues, split-K partial slabs.  Replaces TF Conv2D +
//                    FusedBatchNormV3 + Relu + AddV2 + Split/ConcatV2
//                    (models.py:155-203, res2net_model.py:26-103,
//                    tdnn_model.py:24-30, dpn_model.py:40-87).
//  * stats_pool   -- wave-parallel mean/std over time + head BN
//                    (models.py:262-269, res2net_model.py:239).
//  * splitk_reduce-- deterministic fixed-order split-K combine + BN (head dense,
//                    res2net_model.py:240-241).
//  * avgpool3s2   -- AvgPool 3x3/2 VALID over the fixed-padded tensor, divisor 9
//                    (res2net_model.py:27-28,77).
#include <cstdlib>
#include "kernels.h"
#include "device_common.h"

namespace vox {

template <typename T> struct Tr;
template <> struct Tr<bf16_t> {
  static constexpr int VEC = 8;     // elements per 16-byte lane load
  static constexpr int KSTEP = 32;  // K per MFMA step (16x16x32)
  typedef bf16x8 frag;
};
template <> struct Tr<float> {
  static constexpr int VEC = 4;
  static constexpr int KSTEP = 16;  // 4 x mfma 16x16x4 over a permuted K
  typedef f32x4 frag;
};

__device__ __forceinline__ bf16x8 frag_bnrelu(bf16x8 a, const float* m, const float* iv) {
  bf16x8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = (bf16_t)fmaxf(((float)a[e] - m[e]) * iv[e], 0.f);
  return r;
}
__device__ __forceinline__ f32x4 frag_bnrelu(f32x4 a, const float* m, const float* iv) {
  f32x4 r;
#pragma unroll
  for (int e = 0; e < 4; ++e) r[e] = fmaxf((a[e] - m[e]) * iv[e], 0.f);
  return r;
}

// f32: lane l holds k = 4*(l>>4)+j in element j of both operands; MFMA j uses
// element j, i.e. internal k index kk <-> real k = 4*kk + j for A and B alike.
__device__ __forceinline__ f32x4 mfma_step(f32x4 a, f32x4 b, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], c, 0, 0, 0);
  return c;
}

__device__ __forceinline__ void store4(bf16_t* p, const float* v) {
  bf16x4 r;
  r[0] = (bf16_t)v[0]; r[1] = (bf16_t)v[1]; r[2] = (bf16_t)v[2]; r[3] = (bf16_t)v[3];
  *reinterpret_cast<bf16x4*>(p) = r;
}
__device__ __forceinline__ void store4(float* p, const float* v) {
  *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
}
__device__ __forceinline__ void load4(const bf16_t* p, float* v) {
  bf16x4 r = *reinterpret_cast<const bf16x4*>(p);
  v[0] = (float)r[0]; v[1] = (float)r[1]; v[2] = (float)r[2]; v[3] = (float)r[3];
}
__device__ __forceinline__ void load4(const float* p, float* v) {
  f32x4 r = *reinterpret_cast<const f32x4*>(p);
  v[0] = r[0]; v[1] = r[1]; v[2] = r[2]; v[3] = r[3];
}

// Shared epilogue: lane holds couts co0+16i+4*(lane>>4)+r (r<4) of pixel
// pbase+16j+(lane&15).  Applies EPI_* flags, writes y / y2 / split-K slab.
template <typename T, int WCO, int WPX>
__device__ __forceinline__ void conv_epilogue(const ConvParams& p, f32x4 (&acc)[WCO][WPX],
                                              const bool (&pv)[WPX], int pbase, int co0, int grp,
                                              int M) {
  const int lane = threadIdx.x & 63;
  const int col = lane & 15;
  const int goff = grp * p.Cout;
  T* __restrict__ Y = reinterpret_cast<T*>(p.y) + goff;
  T* __restrict__ Y2 = reinterpret_cast<T*>(p.y2);
  const T* __restrict__ R = p.res ? reinterpret_cast<const T*>(p.res) + goff : nullptr;
  const float* __restrict__ bnm = p.mean ? p.mean + goff : nullptr;
  const float* __restrict__ bni = p.inv ? p.inv + goff : nullptr;
  const int flags = p.flags;
#pragma unroll
  for (int i = 0; i < WCO; ++i) {
    const int co = co0 + 16 * i + 4 * (lane >> 4);
    if (co >= p.Cout) continue;
#pragma unroll
    for (int j = 0; j < WPX; ++j) {
      if (!pv[j]) continue;
      const size_t pix = (size_t)(pbase + 16 * j + col);
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (flags & EPI_PARTIAL) {
        float* dst = p.partial + ((size_t)blockIdx.z * M + pix) * p.coutp + co;
        *reinterpret_cast<f32x4*>(dst) = f32x4{v[0], v[1], v[2], v[3]};
        continue;
      }
      if (p.fast4 && co + 3 < p.Cout) {
        if (flags & EPI_PRE_RELU) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
        }
        if (flags & EPI_AFFINE) {
          f32x4 m = *reinterpret_cast<const f32x4*>(bnm + co);
          f32x4 s = *reinterpret_cast<const f32x4*>(bni + co);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (v[r] - m[r]) * s[r];
        }
        const bool primary = co < p.ysplit;
        if ((flags & EPI_RES) && primary) {
          float rv[4];
          load4(R + pix * p.ldr + co, rv);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += rv[r];
        }
        if (flags & EPI_RELU) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
        }
        if (primary) store4(Y + pix * p.ldy + co, v);
        else store4(Y2 + pix * p.ldy2 + (co - p.ysplit), v);
      } else {
        for (int r = 0; r < 4; ++r) {
          const int c = co + r;
          if (c >= p.Cout) break;
          float x = v[r];
          if (flags & EPI_PRE_RELU) x = fmaxf(x, 0.f);
          if (flags & EPI_AFFINE) x = (x - bnm[c]) * bni[c];
          const bool primary = c < p.ysplit;
          if ((flags & EPI_RES) && primary) x += (float)R[pix * p.ldr + c];
          if (flags & EPI_RELU) x = fmaxf(x, 0.f);
          if (primary) Y[pix * p.ldy + c] = (T)x;
          else Y2[pix * p.ldy2 + (c - p.ysplit)] = (T)x;
        }
      }
    }
  }
}

// ----------------------------------------------------------------------------
// Implicit-GEMM conv.  MFMA rows = output channels (A = weights [coutp][kp]),
// MFMA columns = output pixels (B = im2col, gathered straight from NHWC).
// Block = 4 waves stacked along pixels; a wave owns WCO x WPX 16x16 tiles.
// The accumulator layout (col = lane&15 = pixel, rows 4*(lane>>4)+r = couts)
// gives every lane 4 consecutive channels of one pixel in the epilogue.
template <typename T, int WCO, int WPX, bool VEC>
__global__ __launch_bounds__(256) void conv_igemm(ConvParams p) {
  typedef typename Tr<T>::frag frag;
  constexpr int VN = Tr<T>::VEC;
  constexpr int KS = Tr<T>::KSTEP;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int M = p.N * p.Ho * p.Wo;
  const int HoWo = p.Ho * p.Wo;
  const int grp = blockIdx.y / p.cblocks;
  const int co0 = (blockIdx.y - grp * p.cblocks) * (16 * WCO);
  const int pbase = (blockIdx.x * 4 + wave) * (16 * WPX);
  if (pbase >= M) return;
  const int col = lane & 15;
  const int kl = (lane >> 4) * VN;

  int pn[WPX], pho[WPX], pwo[WPX];
  bool pv[WPX];
#pragma unroll
  for (int j = 0; j < WPX; ++j) {
    int pix = pbase + 16 * j + col;
    pv[j] = pix < M;
    int q = pv[j] ? pix : 0;
    pn[j] = q / HoWo;
    int r = q - pn[j] * HoWo;
    pho[j] = r / p.Wo;
    pwo[j] = r - pho[j] * p.Wo;
  }

  f32x4 acc[WCO][WPX];
#pragma unroll
  for (int i = 0; i < WCO; ++i)
#pragma unroll
    for (int j = 0; j < WPX; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // grouped conv: per-group channel offsets (groups == 1 -> all zero)
  const T* __restrict__ X = reinterpret_cast<const T*>(p.x) + grp * p.Cin;
  const T* __restrict__ X2 = p.x2 ? reinterpret_cast<const T*>(p.x2) + grp * p.Cin : nullptr;
  const float* in_mean = p.in_mean ? p.in_mean + grp * p.Cin : nullptr;
  const float* in_inv = p.in_inv ? p.in_inv + grp * p.Cin : nullptr;
  const T* __restrict__ Wt = reinterpret_cast<const T*>(p.w) + (size_t)grp * p.coutp * p.kp;
  const T* wrow[WCO];
#pragma unroll
  for (int i = 0; i < WCO; ++i) wrow[i] = Wt + (size_t)(co0 + 16 * i + col) * p.kp;

  if constexpr (VEC) {
    const int taps = p.kh * p.kw;
    int cbeg = 0, cend = p.cinp;
    if (gridDim.z > 1) {
      cbeg = blockIdx.z * p.kchunk;
      cend = min(cbeg + p.kchunk, p.cinp);
    }
    for (int tap = 0; tap < taps; ++tap) {
      const int ky = tap / p.kw, kx = tap - (tap / p.kw) * p.kw;
      const T* xb[WPX];
      const T* xb2[WPX];
#pragma unroll
      for (int j = 0; j < WPX; ++j) {
        int hi = pho[j] * p.sh - p.ph + ky * p.dh;
        int wi = pwo[j] * p.sw - p.pw + kx * p.dw;
        bool ok = pv[j] && hi >= 0 && hi < p.H && wi >= 0 && wi < p.W;
        size_t pix = ((size_t)pn[j] * p.H + hi) * p.W + wi;
        xb[j] = ok ? X + pix * p.ldx : nullptr;
        xb2[j] = (ok && X2) ? X2 + pix * p.ldx2 : nullptr;
      }
      const int woff = tap * p.cinp;
      for (int c0 = cbeg; c0 < cend; c0 += KS) {
        const int c = c0 + kl;
        frag a[WCO], b[WPX];
#pragma unroll
        for (int i = 0; i < WCO; ++i) a[i] = ld16(wrow[i] + woff + c);
        const bool cin_ok = c < p.Cin;
        float im[VN], ii[VN];
        if (in_mean && cin_ok) {
#pragma unroll
          for (int e = 0; e < VN; ++e) { im[e] = in_mean[c + e]; ii[e] = in_inv[c + e]; }
        }
#pragma unroll
        for (int j = 0; j < WPX; ++j) {
          if (xb[j] && cin_ok) {
            frag v = ld16(xb[j] + c);
            if (xb2[j]) v = frag_add(v, ld16(xb2[j] + c));
            if (in_mean) v = frag_bnrelu(v, im, ii);
            b[j] = v;
          } else {
            b[j] = zero_frag<frag>();
          }
        }
#pragma unroll
        for (int i = 0; i < WCO; ++i)
#pragma unroll
          for (int j = 0; j < WPX; ++j) acc[i][j] = mfma_step(a[i], b[j], acc[i][j]);
      }
    }
  } else {
    // Gather path (Cin not a multiple of VN, e.g. the 1-channel stem): K is
    // flattened as k = tap*Cin + ci and padded to kp.
    const int K = p.kh * p.kw * p.Cin;
    for (int k0 = 0; k0 < p.kp; k0 += KS) {
      frag a[WCO], b[WPX];
#pragma unroll
      for (int i = 0; i < WCO; ++i) a[i] = ld16(wrow[i] + k0 + kl);
#pragma unroll
      for (int j = 0; j < WPX; ++j) {
        frag v;
#pragma unroll
        for (int e = 0; e < VN; ++e) {
          int k = k0 + kl + e;
          float val = 0.f;
          if (pv[j] && k < K) {
            int tap = k / p.Cin, ci = k - (k / p.Cin) * p.Cin;
            int ky = tap / p.kw, kx = tap - (tap / p.kw) * p.kw;
            int hi = pho[j] * p.sh - p.ph + ky * p.dh;
            int wi = pwo[j] * p.sw - p.pw + kx * p.dw;
            if (hi >= 0 && hi < p.H && wi >= 0 && wi < p.W) {
              size_t pix = ((size_t)pn[j] * p.H + hi) * p.W + wi;
              val = (float)X[pix * p.ldx + ci];
              if (X2) val += (float)X2[pix * p.ldx2 + ci];
              if (in_mean) val = fmaxf((val - in_mean[ci]) * in_inv[ci], 0.f);
            }
          }
          v[e] = (T)val;
        }
        b[j] = v;
      }
#pragma unroll
      for (int i = 0; i < WCO; ++i)
#pragma unroll
        for (int j = 0; j < WPX; ++j) acc[i][j] = mfma_step(a[i], b[j], acc[i][j]);
    }
  }

  conv_epilogue<T, WCO, WPX>(p, acc, pv, pbase, co0, grp, M);
}

// ----------------------------------------------------------------------------
// Window-staged implicit GEMM for stride-1 convolutions (bf16).  A block owns
// BP = 64*WPX consecutive output pixels and BCO = 16*WCO output channels.
// For each chunk of kc input channels it stages into LDS
//   * the input window: flattened pixels [p0 + lo, p0 + BP + hi) x kc channels
//     (every tap of every output pixel is a constant flattened offset
//     dy*W + dx away in this window; out-of-image taps are masked), with the
//     optional hierarchical addend x2 added on the way in;
//   * the weights of the chunk for all taps, rows [tap][kc] flattened;
//   * a k-step table q -> (window offset, channel byte offset, dy, dx).
// Each input pixel is read from HBM once per block instead of once per tap.
// LDS pixel / weight-row strides are padded to an odd number of 16-B units so
// the 16 lanes of a ds_read_b128 group hit distinct banks.
template <int WCO, int WPX>
__global__ __launch_bounds__(256) void conv_win(ConvParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BCO = 16 * WCO;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int col = lane & 15;
  const int M = p.N * p.Ho * p.Wo;           // output pixels
  const int Min = p.N * p.H * p.W;           // input pixels
  const int HoWo = p.Ho * p.Wo;
  const int p0 = blockIdx.x * (64 * WPX);
  const int co0 = blockIdx.y * BCO;
  const int taps = p.kh * p.kw;
  char* act = smem;
  char* wts = smem + p.win_len * p.win_astr;
  int4* ktab = reinterpret_cast<int4*>(wts + BCO * p.win_wstr);
  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(p.x);
  const bf16_t* __restrict__ X2 = reinterpret_cast<const bf16_t*>(p.x2);
  const bf16_t* __restrict__ Wt = reinterpret_cast<const bf16_t*>(p.w);
  const int pbase = p0 + wave * 16 * WPX;
  // window in input-flattened coordinates: tap (dy,dx) of the output pixel
  // whose centre input pixel is c sits at c + dy*W + dx (stride 1 or 2)
  auto in_flat = [&](int pix) {
    const int n = pix / HoWo, r = pix - (pix / HoWo) * HoWo;
    const int ho = r / p.Wo, wo = r - (r / p.Wo) * p.Wo;
    return (n * p.H + ho * p.sh) * p.W + wo * p.sw;
  };
  const int wstart = in_flat(min(p0, M - 1)) + p.win_lo;

  int hh[WPX], ww[WPX], li[WPX];
  bool pv[WPX];
#pragma unroll
  for (int j = 0; j < WPX; ++j) {
    const int pix = pbase + 16 * j + col;
    pv[j] = pix < M;
    const int q = pv[j] ? pix : 0;
    const int r = q % HoWo;
    const int ho = r / p.Wo, wo = r - (r / p.Wo) * p.Wo;
    hh[j] = ho * p.sh;
    ww[j] = wo * p.sw;
    li[j] = in_flat(q) - wstart;
  }
  f32x4 acc[WCO][WPX];
#pragma unroll
  for (int i = 0; i < WCO; ++i)
#pragma unroll
    for (int j = 0; j < WPX; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int c0 = 0; c0 < p.Cin; c0 += p.win_kc) {
    const int kc = min(p.win_kc, p.Cin - c0);
    const int kflat = taps * kc;
    const int kcp = (kflat + 31) & ~31;
    const int units = kcp >> 3;
    // k-step table
    for (int q = tid; q < units; q += 256) {
      const int k = q * 8;
      int4 e = make_int4(0, 0, 1 << 20, 1 << 20);
      if (k < kflat) {
        const int tap = k / kc, ch = k - (k / kc) * kc;
        const int ky = tap / p.kw, kx = tap - (tap / p.kw) * p.kw;
        const int dy = ky * p.dh - p.ph, dx = kx * p.dw - p.pw;
        e = make_int4(dy * p.W + dx, ch * 2, dy, dx);
      }
      ktab[q] = e;
    }
    // weights [BCO][taps*kc] (global layout [coutp][taps*Cin])
    {
      const int total = BCO * units;
      const int rowlen = taps * p.Cin;
      for (int idx = tid; idx < total; idx += 256) {
        const int r = idx / units, u = idx - (idx / units) * units;
        const int k = u * 8;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (k < kflat) {
          const int tap = k / kc, ch = k - (k / kc) * kc;
          v = *reinterpret_cast<const uint4*>(Wt + (size_t)(co0 + r) * rowlen + tap * p.Cin + c0 + ch);
        }
        *reinterpret_cast<uint4*>(wts + r * p.win_wstr + u * 16) = v;
      }
    }
    // input window (+ addend)
    {
      const int cu = kc >> 3;
      const int total = p.win_len * cu;
      const int gbase = wstart;
      for (int b0 = tid; b0 < total; b0 += 4 * 256) {
        uint4 v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int idx = b0 + r * 256;
          v[r] = make_uint4(0, 0, 0, 0);
          if (idx < total) {
            const int wp = idx / cu, u = idx - (idx / cu) * cu;
            const int gp = gbase + wp;
            if (gp >= 0 && gp < Min) {
              v[r] = *reinterpret_cast<const uint4*>(X + (size_t)gp * p.ldx + c0 + u * 8);
              if (X2) {
                bf16x8 a = __builtin_bit_cast(bf16x8, v[r]);
                bf16x8 b = ld16(X2 + (size_t)gp * p.ldx2 + c0 + u * 8);
                v[r] = __builtin_bit_cast(uint4, frag_add(a, b));
              }
            }
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int idx = b0 + r * 256;
          if (idx < total) {
            const int wp = idx / cu, u = idx - (idx / cu) * cu;
            *reinterpret_cast<uint4*>(act + wp * p.win_astr + u * 16) = v[r];
          }
        }
      }
    }
    __syncthreads();
    for (int k0 = 0; k0 < kcp; k0 += 32) {
      const int4 t = ktab[(k0 >> 3) + (lane >> 4)];
      bf16x8 a[WCO], b[WPX];
#pragma unroll
      for (int i = 0; i < WCO; ++i)
        a[i] = *reinterpret_cast<const bf16x8*>(wts + (16 * i + col) * p.win_wstr +
                                                (k0 + 8 * (lane >> 4)) * 2);
#pragma unroll
      for (int j = 0; j < WPX; ++j) {
        const int y = hh[j] + t.z, x = ww[j] + t.w;
        const bool ok = pv[j] && (unsigned)y < (unsigned)p.H && (unsigned)x < (unsigned)p.W;
        b[j] = ok ? *reinterpret_cast<const bf16x8*>(act + (li[j] + t.x) * p.win_astr + t.y)
                  : bf16x8{};
      }
#pragma unroll
      for (int i = 0; i < WCO; ++i)
#pragma unroll
        for (int j = 0; j < WPX; ++j) acc[i][j] = mfma_step(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
  conv_epilogue<bf16_t, WCO, WPX>(p, acc, pv, pbase, co0, 0, M);
}

template <int WCO, int WPX>
static hipError_t launch_win_t(const ConvParams& p, hipStream_t s) {
  const int M = p.N * p.Ho * p.Wo;
  dim3 grid((M + 64 * WPX - 1) / (64 * WPX), p.cblocks, 1);
  hipLaunchKernelGGL((conv_win<WCO, WPX>), grid, dim3(256), p.win_lds, s, p);
  return hipGetLastError();
}

template <int WPX>
static hipError_t launch_win_wco(const ConvParams& p, int wco, hipStream_t s) {
  switch (wco) {
    case 1: return launch_win_t<1, WPX>(p, s);
    case 2: return launch_win_t<2, WPX>(p, s);
    case 3: return launch_win_t<3, WPX>(p, s);
    case 4: return launch_win_t<4, WPX>(p, s);
    case 6: return launch_win_t<6, WPX>(p, s);
    case 8: return launch_win_t<8, WPX>(p, s);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_conv_win(const ConvParams& p, const ConvLaunch& l, hipStream_t s) {
  switch (l.wpx) {
    case 1: return launch_win_wco<1>(p, l.wco, s);
    case 2: return launch_win_wco<2>(p, l.wco, s);
    case 4: return launch_win_wco<4>(p, l.wco, s);
  }
  return hipErrorInvalidValue;
}

// ----------------------------------------------------------------------------
// Register-resident 1x1 conv (any stride) for K = Cin <= 32*KS: a wave loads
// its 16*WPX pixels' whole input vector into registers once (B fragments,
// optional BN+ReLU prologue applied in registers), then sweeps every output
// channel tile pair, WCO tiles (WCO/2 pairs) at a time, streaming weight
// fragments from L1/L2.  Activations are read from HBM exactly once; no LDS.
//
// Paired-row weight layout (built on the host): within each 32-channel pair of
// tiles (2q, 2q+1), MFMA row 4g+e of tile 2q+u holds output channel
// 32q + 8g + 4u + e.  Lane group g = lane>>4 therefore ends up with 8
// consecutive channels 32q+8g .. +7 of its pixel, so every epilogue access
// (BN mean/inv, residual, output) is one 16-byte load/store per lane.  The
// residual and BN operands of a tile group are fetched before its MFMAs.
template <int KS, int WPX, int WCO>
__global__ __launch_bounds__(256) void conv1x1_rr(ConvParams p) {
  static_assert(WCO % 2 == 0, "paired tiles");
  constexpr int NP = WCO / 2;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int col = lane & 15;
  const int g = lane >> 4;
  const int kl = g * 8;
  const int M = p.N * p.Ho * p.Wo;
  const int HoWo = p.Ho * p.Wo;
  const int pbase = (blockIdx.x * 4 + wave) * (16 * WPX);
  if (pbase >= M) return;
  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(p.x);
  const bf16_t* __restrict__ Wt = reinterpret_cast<const bf16_t*>(p.w);
  const bf16_t* __restrict__ R = reinterpret_cast<const bf16_t*>(p.res);
  bf16_t* __restrict__ Y = reinterpret_cast<bf16_t*>(p.y);
  bf16_t* __restrict__ Y2 = reinterpret_cast<bf16_t*>(p.y2);
  const int flags = p.flags;

  bool pv[WPX];
  size_t pix[WPX];
  bf16x8 b[KS][WPX];
#pragma unroll
  for (int j = 0; j < WPX; ++j) {
    const int pp = pbase + 16 * j + col;
    pv[j] = pp < M;
    const int q = pv[j] ? pp : 0;
    pix[j] = (size_t)q;
    const int n = q / HoWo;
    const int r = q - n * HoWo;
    const int ho = r / p.Wo, wo = r - (r / p.Wo) * p.Wo;
    const bf16_t* xp = X + (((size_t)n * p.H + ho * p.sh) * p.W + wo * p.sw) * p.ldx;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int c = s * 32 + kl;
      b[s][j] = (pv[j] && c < p.Cin) ? ld16(xp + c) : bf16x8{};
    }
  }
  if (p.in_mean) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int c = s * 32 + kl;
      if (c < p.Cin) {
        float im[8], ii[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) { im[e] = p.in_mean[c + e]; ii[e] = p.in_inv[c + e]; }
#pragma unroll
        for (int j = 0; j < WPX; ++j)
          if (pv[j]) b[s][j] = frag_bnrelu(b[s][j], im, ii);
      }
    }
  }
  const int tiles = p.coutp / 16;
  const int per = ((tiles + gridDim.y - 1) / gridDim.y + WCO - 1) / WCO * WCO;
  const int t0 = blockIdx.y * per, t1 = min(tiles, t0 + per);
  for (int t = t0; t < t1; t += WCO) {
    // epilogue operands first (independent of the MFMAs)
    f32x4 bm[NP][2], bi[NP][2];
    bf16x8 rv[NP][WPX];
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const int ch = (t / 2 + q) * 32 + 8 * g;
      const bool cok = ch < p.Cout;
      if ((flags & EPI_AFFINE) && cok) {
        bm[q][0] = *reinterpret_cast<const f32x4*>(p.mean + ch);
        bm[q][1] = *reinterpret_cast<const f32x4*>(p.mean + ch + 4);
        bi[q][0] = *reinterpret_cast<const f32x4*>(p.inv + ch);
        bi[q][1] = *reinterpret_cast<const f32x4*>(p.inv + ch + 4);
      }
#pragma unroll
      for (int j = 0; j < WPX; ++j)
        rv[q][j] = ((flags & EPI_RES) && cok && pv[j] && ch < p.ysplit)
                       ? ld16(R + pix[j] * p.ldr + ch) : bf16x8{};
    }
    f32x4 acc[WCO][WPX];
#pragma unroll
    for (int i = 0; i < WCO; ++i)
#pragma unroll
      for (int j = 0; j < WPX; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      bf16x8 a[WCO];
#pragma unroll
      for (int i = 0; i < WCO; ++i) {
        const int row = min(t + i, tiles - 1) * 16 + col;
        a[i] = ld16(Wt + (size_t)row * p.kp + s * 32 + kl);
      }
#pragma unroll
      for (int i = 0; i < WCO; ++i)
#pragma unroll
        for (int j = 0; j < WPX; ++j) acc[i][j] = mfma_step(a[i], b[s][j], acc[i][j]);
    }
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const int ch = (t / 2 + q) * 32 + 8 * g;
      if (ch >= p.Cout) continue;
#pragma unroll
      for (int j = 0; j < WPX; ++j) {
        if (!pv[j]) continue;
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[2 * q][j][e];
          v[4 + e] = acc[2 * q + 1][j][e];
        }
        if (flags & EPI_PRE_RELU) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        if (flags & EPI_AFFINE) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = (v[e] - bm[q][0][e]) * bi[q][0][e];
            v[4 + e] = (v[4 + e] - bm[q][1][e]) * bi[q][1][e];
          }
        }
        if (flags & EPI_RES) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += (float)rv[q][j][e];
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

template <int KS, int WPX>
static hipError_t launch_rr_t(const ConvParams& p, int wco, int ysplit_blocks, hipStream_t s) {
  const int M = p.N * p.Ho * p.Wo;
  dim3 grid((M + 64 * WPX - 1) / (64 * WPX), ysplit_blocks, 1);
  if (wco == 4)
    hipLaunchKernelGGL((conv1x1_rr<KS, WPX, 4>), grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((conv1x1_rr<KS, WPX, 2>), grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

int conv1x1_rr_max_wpx(int ks) {
  // keep the B fragments (KS*WPX*4 VGPRs) within ~128 registers
  if (ks <= 8) return 4;
  if (ks <= 16) return 2;
  return 1;
}

hipError_t launch_conv1x1_rr(const ConvParams& p, const ConvLaunch& l, hipStream_t s) {
  const int ks = (p.cinp + 31) / 32;
  const int ys = l.splitk > 0 ? l.splitk : 1;  // reused as the cout-split count
#define RR_CASE(K)                                                        \
  case K:                                                                 \
    return l.wpx == 4 ? launch_rr_t<K, 4>(p, l.wco, ys, s)                \
                      : (l.wpx == 2 ? launch_rr_t<K, 2>(p, l.wco, ys, s)  \
                                    : launch_rr_t<K, 1>(p, l.wco, ys, s));
#define RR_CASE2(K)                                                       \
  case K:                                                                 \
    return l.wpx == 2 ? launch_rr_t<K, 2>(p, l.wco, ys, s)                \
                      : launch_rr_t<K, 1>(p, l.wco, ys, s);
#define RR_CASE1(K) \
  case K:           \
    return launch_rr_t<K, 1>(p, l.wco, ys, s);
  switch (ks) {
    RR_CASE(1)
    RR_CASE(2)
    RR_CASE(3)
    RR_CASE(4)
    RR_CASE(6)
    RR_CASE(8)
    RR_CASE2(12)
    RR_CASE2(16)
    RR_CASE1(24)
    RR_CASE1(32)
  }
#undef RR_CASE
#undef RR_CASE2
#undef RR_CASE1
  return hipErrorInvalidValue;
}

// ----------------------------------------------------------------------------
// LDS-tiled GEMM for compute-bound 1x1 convs (K = cinp % 64 == 0, any stride):
// block tile 128 output channels x 128 pixels, BK = 64, 4 waves in 2x2, each
// wave 64x64 = 4x4 MFMA 16x16x32 tiles.  Both operands are K-contiguous rows
// staged global -> registers -> LDS (double-buffered; the next tile's global
// loads are issued before the current tile's MFMAs).  LDS rows are 128 B with
// 16-B chunk c of row r stored at chunk c ^ ((r>>1)&7): every ds_read_b128
// lane group (rows 0-3,12-15 at chunk c, rows 4-11 at c+1) then covers all
// 64 banks exactly once.  Weights use the paired-row layout so the epilogue
// does 16-byte accesses (see conv1x1_rr).
__device__ __forceinline__ int swz(int r, int c) { return r * 64 + ((c ^ ((r >> 1) & 7)) << 3); }

__global__ __launch_bounds__(256) void gemm1x1_lds(ConvParams p) {
  __shared__ __attribute__((aligned(16))) bf16_t As[2][128 * 64];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[2][128 * 64];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int col = lane & 15, g = lane >> 4;
  const int M = p.N * p.Ho * p.Wo;
  const int HoWo = p.Ho * p.Wo;
  // XCD-aware bijective remap (blocks are dealt round-robin over the 8 XCDs):
  // each XCD gets a contiguous range of logical ids, and within it the cout
  // blocks of one pixel tile are consecutive, so the activation tile is
  // fetched into that XCD's L2 once and reused by all cout blocks.
  const int nwg = gridDim.x;
  const int cblocks = p.coutp / 128;
  int lid;
  {
    const int bid = blockIdx.x, xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    lid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int co0 = (lid % cblocks) * 128;
  const int px0 = (lid / cblocks) * 128;
  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(p.x);
  const bf16_t* __restrict__ Wt = reinterpret_cast<const bf16_t*>(p.w);
  // staging assignment: 1024 16-B chunks per operand tile, 4 per thread
  const bf16_t* ga[4];
  const bf16_t* gb[4];
  int lr[4], lc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i;
    lr[i] = c >> 3;
    lc[i] = c & 7;
    ga[i] = Wt + (size_t)(co0 + lr[i]) * p.kp + lc[i] * 8;
    // rows past M load pixel M-1 (any valid address): their output columns
    // are never stored, and unconditional loads keep the pipeline branch-free
    const int pix = min(px0 + lr[i], M - 1);
    const int n = pix / HoWo, r = pix - (pix / HoWo) * HoWo;
    const int ho = r / p.Wo, wo = r - (r / p.Wo) * p.Wo;
    gb[i] = X + (((size_t)n * p.H + ho * p.sh) * p.W + wo * p.sw) * p.ldx + lc[i] * 8;
  }
  // staging registers as named scalars (arrays captured by a lambda were
  // promoted to LDS by the compiler).  Two register sets x/y give a 2-deep
  // prefetch: while tile k is computed from LDS, tile k+1 waits in one set
  // (loaded an iteration earlier) and tile k+2 is in flight into the other.
  uint4 xa0, xa1, xa2, xa3, xb0, xb1, xb2, xb3;
  uint4 ya0, ya1, ya2, ya3, yb0, yb1, yb2, yb3;
  const int so0 = swz(lr[0], lc[0]), so1 = swz(lr[1], lc[1]), so2 = swz(lr[2], lc[2]),
            so3 = swz(lr[3], lc[3]);
#define GEMM_GLOAD(P, k0)                                     \
  do {                                                        \
    P##a0 = *reinterpret_cast<const uint4*>(ga[0] + (k0));    \
    P##a1 = *reinterpret_cast<const uint4*>(ga[1] + (k0));    \
    P##a2 = *reinterpret_cast<const uint4*>(ga[2] + (k0));    \
    P##a3 = *reinterpret_cast<const uint4*>(ga[3] + (k0));    \
    P##b0 = *reinterpret_cast<const uint4*>(gb[0] + (k0));    \
    P##b1 = *reinterpret_cast<const uint4*>(gb[1] + (k0));    \
    P##b2 = *reinterpret_cast<const uint4*>(gb[2] + (k0));    \
    P##b3 = *reinterpret_cast<const uint4*>(gb[3] + (k0));    \
  } while (0)
#define GEMM_LSTORE(P, buf)                                   \
  do {                                                        \
    *reinterpret_cast<uint4*>(&As[buf][so0]) = P##a0;         \
    *reinterpret_cast<uint4*>(&As[buf][so1]) = P##a1;         \
    *reinterpret_cast<uint4*>(&As[buf][so2]) = P##a2;         \
    *reinterpret_cast<uint4*>(&As[buf][so3]) = P##a3;         \
    *reinterpret_cast<uint4*>(&Bs[buf][so0]) = P##b0;         \
    *reinterpret_cast<uint4*>(&Bs[buf][so1]) = P##b1;         \
    *reinterpret_cast<uint4*>(&Bs[buf][so2]) = P##b2;         \
    *reinterpret_cast<uint4*>(&Bs[buf][so3]) = P##b3;         \
  } while (0)
#define GEMM_COMPUTE(cur)                                                                    \
  do {                                                                                       \
    _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) {                                       \
      const int c = ks * 4 + g;                                                              \
      bf16x8 a[4], b[4];                                                                     \
      _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                        \
        a[i] = *reinterpret_cast<const bf16x8*>(&As[cur][swz(wm * 64 + 16 * i + col, c)]);   \
        b[i] = *reinterpret_cast<const bf16x8*>(&Bs[cur][swz(wn * 64 + 16 * i + col, c)]);   \
      }                                                                                      \
      _Pragma("unroll") for (int i = 0; i < 4; ++i)                                          \
        _Pragma("unroll") for (int j = 0; j < 4; ++j) acc[i][j] = mfma_step(a[i], b[j], acc[i][j]); \
    }                                                                                        \
  } while (0)
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int KT = p.kp / 64;
  const int last = (KT - 1) * 64;
  // loads past the last tile re-read it: harmless, and keeps the loop
  // branch-free (a branch lets the compiler fuse the load and store blocks)
  GEMM_GLOAD(x, 0);
  GEMM_LSTORE(x, 0);
  GEMM_GLOAD(x, min(64, last));
  __syncthreads();
  int kt = 0;
  for (; kt + 1 < KT; kt += 2) {
    GEMM_GLOAD(y, min((kt + 2) * 64, last));
    __builtin_amdgcn_sched_barrier(0);
    GEMM_COMPUTE(0);
    __builtin_amdgcn_sched_barrier(0);
    GEMM_LSTORE(x, 1);
    __syncthreads();
    GEMM_GLOAD(x, min((kt + 3) * 64, last));
    __builtin_amdgcn_sched_barrier(0);
    GEMM_COMPUTE(1);
    __builtin_amdgcn_sched_barrier(0);
    GEMM_LSTORE(y, 0);
    __syncthreads();
  }
  if (kt < KT) GEMM_COMPUTE(0);  // odd KT: the final tile is in buffer 0

#undef GEMM_GLOAD
#undef GEMM_LSTORE
#undef GEMM_COMPUTE
  // paired epilogue: m-tiles (2q, 2q+1) of this wave -> 8 consecutive channels
  const bf16_t* __restrict__ R = reinterpret_cast<const bf16_t*>(p.res);
  bf16_t* __restrict__ Y = reinterpret_cast<bf16_t*>(p.y);
  bf16_t* __restrict__ Y2 = reinterpret_cast<bf16_t*>(p.y2);
  const int flags = p.flags;
  bf16x8 rvs[2][4];  // residual operands first, off the dependent path
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int ch = co0 + wm * 64 + 32 * q + 8 * g;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int pix = px0 + wn * 64 + 16 * j + col;
      rvs[q][j] = ((flags & EPI_RES) && ch < p.Cout && ch < p.ysplit && pix < M)
                      ? ld16(R + (size_t)pix * p.ldr + ch) : bf16x8{};
    }
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int ch = co0 + wm * 64 + 32 * q + 8 * g;
    if (ch >= p.Cout) continue;
    f32x4 bm0, bm1, bi0, bi1;
    if (flags & EPI_AFFINE) {
      bm0 = *reinterpret_cast<const f32x4*>(p.mean + ch);
      bm1 = *reinterpret_cast<const f32x4*>(p.mean + ch + 4);
      bi0 = *reinterpret_cast<const f32x4*>(p.inv + ch);
      bi1 = *reinterpret_cast<const f32x4*>(p.inv + ch + 4);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int pix = px0 + wn * 64 + 16 * j + col;
      if (pix >= M) continue;
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc[2 * q][j][e];
        v[4 + e] = acc[2 * q + 1][j][e];
      }
      if (flags & EPI_PRE_RELU) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      if (flags & EPI_AFFINE) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = (v[e] - bm0[e]) * bi0[e];
          v[4 + e] = (v[4 + e] - bm1[e]) * bi1[e];
        }
      }
      if (flags & EPI_RES) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += (float)rvs[q][j][e];
      }
      if (flags & EPI_RELU) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (bf16_t)v[e];
      bf16_t* dst = ch < p.ysplit ? Y + (size_t)pix * p.ldy + ch
                                  : Y2 + (size_t)pix * p.ldy2 + (ch - p.ysplit);
      *reinterpret_cast<uint4*>(dst) = __builtin_bit_cast(uint4, o);
    }
  }
}

hipError_t launch_gemm1x1(const ConvParams& p, hipStream_t s) {
  const int M = p.N * p.Ho * p.Wo;
  dim3 grid(((M + 127) / 128) * (p.coutp / 128), 1, 1);
  hipLaunchKernelGGL(gemm1x1_lds, grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------
// Fused hierarchical split-scale chain (Res2Net, stride 1).  A block owns R
// full-width output rows of one utterance and runs all nst = split-1 branch
// convolutions on them, keeping every intermediate in LDS:
//   buffer rows map to image rows r0-nst .. r0+R+nst (zeros outside the image);
//   stage k reads rows [r0-(nst-k), r0+R+(nst-k)) and produces rows
//   [r0-(nst-1-k), r0+R+(nst-1-k)) -- the halo shrinks by one row per stage;
//   before stage k the next input x_{k+1} is staged into the other buffer and
//   stage k's epilogue adds y_k into it (z_{k+1} = x_{k+1} + y_k, rounded to
//   bf16 like the unfused path); y_k for the R central rows goes to HBM.
// Only x_0..x_{nst-1} are read and y_0..y_{nst-1} written: the intermediate
// branch tensors and the hierarchical adds never touch HBM.
template <int WCO, int WPX, int NW>
__global__ __launch_bounds__(64 * NW) void split_chain(ChainParams q) {
  constexpr int NT = 64 * NW;
  constexpr int XREG = 8;                 // prefetched x chunks per thread (host-checked)
  // weight chunks per thread, sized for the widest branch this tile count
  // serves (w <= 16*WCO): BCO rows x roundup(9*w, 32)/8 16-byte units
  constexpr int WREG = (16 * WCO * (((9 * 16 * WCO + 31) / 32) * 4) + NT - 1) / NT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BCO = 16 * WCO;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, g = lane >> 4;
  const int W = q.W, H = q.H, w = q.w, nst = q.nst, R = q.R;
  const int WP = W + 2;                             // LDS row: zero column | W | zero column
  const int rowb = WP * q.astr;                     // bytes per LDS row
  const int tiles_img = (H + R - 1) / R;
  const int n = blockIdx.x / tiles_img;
  const int r0 = (blockIdx.x - n * tiles_img) * R;
  const int rbase = r0 - nst;                       // image row of buffer row 0
  const int nrows = R + 2 * nst;
  char* buf0 = smem;
  char* buf1 = smem + q.buf_bytes;
  char* wts = smem + 2 * q.buf_bytes;
  int* ktab = reinterpret_cast<int*>(wts + BCO * q.wstr);
  const bf16_t* __restrict__ A = reinterpret_cast<const bf16_t*>(q.a);
  bf16_t* __restrict__ Bo = reinterpret_cast<bf16_t*>(q.b);
  const size_t img = (size_t)n * H * W;
  const int kflat = 9 * w;
  const int units = q.kcp >> 3;
  // k-step table: byte offset of chunk u's tap/channel relative to the
  // centre pixel (padded K points at a zero pad column of row 0 .. harmless:
  // the matching weights are zero)
  for (int u = tid; u < units; u += NT) {
    const int k = u * 8;
    int off = 0;
    if (k < kflat) {
      const int tap = k / w, ch = k - (k / w) * w;
      const int dy = tap / 3 - 1, dx = tap % 3 - 1;
      off = dy * rowb + dx * q.astr + ch * 2;
    }
    ktab[u] = off;
  }
  // zero the pad columns of both buffers once (staging and the epilogue only
  // ever write interior pixels)
  for (int i = tid; i < 2 * nrows * 2 * (q.astr >> 4); i += NT) {
    const int per_row = 2 * (q.astr >> 4);
    const int bsel = i / (nrows * per_row);
    const int rem = i - bsel * nrows * per_row;
    const int row = rem / per_row, cix = rem - (rem / per_row) * per_row;
    const int side = cix / (q.astr >> 4), u = cix - side * (q.astr >> 4);
    char* bb = bsel ? buf1 : buf0;
    *reinterpret_cast<uint4*>(bb + row * rowb + (side ? (W + 1) : 0) * q.astr + u * 16) =
        make_uint4(0, 0, 0, 0);
  }
  // copy channels [c0, c0+w) of image rows [ra, rb) into an LDS buffer.
  // Thread t owns 16-B chunk t of every row (computed once); rows unrolled 8-deep.
  const int cu = w >> 3;
  const int rowchunks = W * cu;
  auto stage_rows = [&](char* dst, int c0, int ra, int rb) __attribute__((always_inline)) {
    for (int c = tid; c < rowchunks; c += NT) {
      const int px = c / cu, uu = c - (c / cu) * cu;
      const bf16_t* src = A + (img + px) * q.lda + c0 + uu * 8;
      char* d = dst + (px + 1) * q.astr + uu * 16;
      for (int row = ra; row < rb; row += 8) {
        uint4 v[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int rr = row + r;
          v[r] = (rr < rb && rr >= 0 && rr < H)
                     ? *reinterpret_cast<const uint4*>(src + (size_t)rr * W * q.lda)
                     : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 8; ++r)
          if (row + r < rb) *reinterpret_cast<uint4*>(d + (row + r - rbase) * rowb) = v[r];
      }
    }
  };
  stage_rows(buf0, 0, r0 - nst, r0 + R + nst);

  // weights of stage 0 straight into LDS
  auto load_w = [&](int k, uint4 (&v)[WREG]) __attribute__((always_inline)) {
    const bf16_t* __restrict__ Wt = reinterpret_cast<const bf16_t*>(q.wt[k]);
#pragma unroll
    for (int r = 0; r < WREG; ++r) {
      const int idx = tid + r * NT;
      const int rw = idx / units, u = idx - (idx / units) * units;
      v[r] = (idx < BCO * units && u * 8 < kflat)
                 ? *reinterpret_cast<const uint4*>(Wt + (size_t)rw * kflat + u * 8)
                 : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_w = [&](const uint4 (&v)[WREG]) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < WREG; ++r) {
      const int idx = tid + r * NT;
      if (idx < BCO * units) {
        const int rw = idx / units, u = idx - (idx / units) * units;
        *reinterpret_cast<uint4*>(wts + rw * q.wstr + u * 16) = v[r];
      }
    }
  };
  uint4 wr[WREG];
  load_w(0, wr);
  store_w(wr);
  __syncthreads();

  for (int k = 0; k < nst; ++k) {
    const int ext = nst - 1 - k;
    const int oa = r0 - ext, ob = r0 + R + ext;     // output image rows of this stage
    char* in = (k & 1) ? buf1 : buf0;
    char* out = (k & 1) ? buf0 : buf1;
    const bool more = k + 1 < nst;
    // prefetch x_{k+1} rows [oa, ob) and the next stage's weights into
    // registers; they land while this stage computes
    const int xchunks = (ob - oa) * rowchunks;
    uint4 xr[XREG];
    if (more) {
#pragma unroll
      for (int r = 0; r < XREG; ++r) {
        const int c = tid + r * NT;
        xr[r] = make_uint4(0, 0, 0, 0);
        if (c < xchunks) {
          const int rr = oa + c / rowchunks;
          const int cc = c - (c / rowchunks) * rowchunks;
          const int px = cc / cu, uu = cc - (cc / cu) * cu;
          if (rr >= 0 && rr < H)
            xr[r] = *reinterpret_cast<const uint4*>(A + (img + (size_t)rr * W + px) * q.lda +
                                                    (k + 1) * w + uu * 8);
        }
      }
      load_w(k + 1, wr);
    }
    const float* __restrict__ bm = q.mean[k];
    const float* __restrict__ bi = q.inv[k];
    const int npix = (ob - oa) * W;
    const int ntiles = (npix + 15) >> 4;
    const char* wrow = wts + col * q.wstr + 16 * g;
    for (int t0 = wave * WPX; t0 < ntiles; t0 += NW * WPX) {
      int prow[WPX], pcol[WPX], base[WPX];
      bool pv[WPX];
#pragma unroll
      for (int j = 0; j < WPX; ++j) {
        const int lp = (t0 + j) * 16 + col;
        pv[j] = lp < npix;
        const int l = pv[j] ? lp : npix - 1;       // clamp: reads stay in the buffer
        prow[j] = oa + l / W;
        pcol[j] = l - (l / W) * W;
        pv[j] = pv[j] && prow[j] >= 0 && prow[j] < H;
        base[j] = (prow[j] - rbase) * rowb + (pcol[j] + 1) * q.astr;
      }
      f32x4 acc[WCO][WPX];
#pragma unroll
      for (int i = 0; i < WCO; ++i)
#pragma unroll
        for (int j = 0; j < WPX; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int k0 = 0; k0 < q.kcp; k0 += 32) {
        const int off = ktab[(k0 >> 3) + g];
        bf16x8 a[WCO], b[WPX];
#pragma unroll
        for (int i = 0; i < WCO; ++i)
          a[i] = *reinterpret_cast<const bf16x8*>(wrow + 16 * i * q.wstr + k0 * 2);
#pragma unroll
        for (int j = 0; j < WPX; ++j) b[j] = *reinterpret_cast<const bf16x8*>(in + base[j] + off);
#pragma unroll
        for (int i = 0; i < WCO; ++i)
#pragma unroll
          for (int j = 0; j < WPX; ++j) acc[i][j] = mfma_step(a[i], b[j], acc[i][j]);
      }
      // epilogue: y = relu(bn(acc)) -> HBM (central rows) and -> LDS (next input)
#pragma unroll
      for (int i = 0; i < WCO; ++i) {
        const int co = 16 * i + 4 * g;
        if (co >= w) continue;
        const f32x4 m = *reinterpret_cast<const f32x4*>(bm + co);
        const f32x4 sc = *reinterpret_cast<const f32x4*>(bi + co);
#pragma unroll
        for (int j = 0; j < WPX; ++j) {
          if (!pv[j]) continue;
          bf16x4 y;
#pragma unroll
          for (int r = 0; r < 4; ++r) y[r] = (bf16_t)fmaxf((acc[i][j][r] - m[r]) * sc[r], 0.f);
          if (prow[j] >= r0 && prow[j] < r0 + R)
            *reinterpret_cast<bf16x4*>(Bo + (img + (size_t)prow[j] * W + pcol[j]) * q.ldb + k * w + co) = y;
          if (more) *reinterpret_cast<bf16x4*>(out + base[j] + co * 2) = y;
        }
      }
    }
    __syncthreads();
    if (more) {
      // combine pass: z_{k+1} = x_{k+1} + y_k (bf16, as the unfused path);
      // rows outside the image stay zero
#pragma unroll
      for (int r = 0; r < XREG; ++r) {
        const int c = tid + r * NT;
        if (c < xchunks) {
          const int rr = oa + c / rowchunks;
          const int cc = c - (c / rowchunks) * rowchunks;
          const int px = cc / cu, uu = cc - (cc / cu) * cu;
          uint4* zp = reinterpret_cast<uint4*>(out + (rr - rbase) * rowb + (px + 1) * q.astr + uu * 16);
          if (rr >= 0 && rr < H) {
            const bf16x8 x = __builtin_bit_cast(bf16x8, xr[r]);
            const bf16x8 y = __builtin_bit_cast(bf16x8, *zp);
            *zp = __builtin_bit_cast(uint4, frag_add(x, y));
          } else {
            *zp = make_uint4(0, 0, 0, 0);  // SAME zero padding of the next stage
          }
        }
      }
      store_w(wr);
      __syncthreads();
    }
  }
}

template <int WCO, int WPX>
static hipError_t launch_chain_t(const ChainParams& q, hipStream_t s) {
  const int blocks = q.N * ((q.H + q.R - 1) / q.R);
  if (q.nwaves == 8)
    hipLaunchKernelGGL((split_chain<WCO, WPX, 8>), dim3(blocks), dim3(512), q.lds, s, q);
  else
    hipLaunchKernelGGL((split_chain<WCO, WPX, 4>), dim3(blocks), dim3(256), q.lds, s, q);
  return hipGetLastError();
}

hipError_t launch_split_chain(const ChainParams& q, int wco, int wpx, hipStream_t s) {
#define CH_CASE(C)                                                        \
  case C:                                                                 \
    return wpx == 4 ? launch_chain_t<C, 4>(q, s)                          \
                    : (wpx == 2 ? launch_chain_t<C, 2>(q, s) : launch_chain_t<C, 1>(q, s));
  switch (wco) {
    CH_CASE(1)
    CH_CASE(2)
    CH_CASE(3)
    CH_CASE(4)
    CH_CASE(6)
  }
#undef CH_CASE
  return hipErrorInvalidValue;
}

// ----------------------------------------------------------------------------
// Stem: 3x3 SAME conv from one input channel (res2net_model.py:192-203,
// dpn_model.py:113) + BN + ReLU.  One thread per output pixel, all Cout
// channels 8 at a time, weights (bf16-rounded in bf16 mode, like the MFMA
// path) and BN in LDS.  Reads the fp32 features directly; in bf16 mode each
// tap is rounded to bf16 first, exactly as the separate cast would.
template <typename T>
__global__ __launch_bounds__(256) void stem_conv1(const float* __restrict__ x, int N, int H,
                                                  int W, const float* __restrict__ wts, int Cout,
                                                  const float* __restrict__ mean,
                                                  const float* __restrict__ inv,
                                                  T* __restrict__ y) {
  __shared__ float sw[9 * 64];
  __shared__ float sm[64], si[64];
  for (int i = threadIdx.x; i < 9 * Cout; i += blockDim.x) sw[i] = wts[i];
  for (int i = threadIdx.x; i < Cout; i += blockDim.x) { sm[i] = mean[i]; si[i] = inv[i]; }
  __syncthreads();
  const int64_t pix = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= (int64_t)N * H * W) return;
  // (h, w) with 32-bit divisions whenever the pixel count allows (the 64-bit
  // ones cost more than the stem's loads)
  const int64_t npix = (int64_t)N * H * W;
  const unsigned hw = npix < ((int64_t)1 << 32) ? (unsigned)pix % (unsigned)(H * W)
                                                : (unsigned)(pix % ((int64_t)H * W));
  const int hi = (int)(hw / (unsigned)W);
  const int wi = (int)(hw - (unsigned)hi * (unsigned)W);
  float v[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int yy = hi + t / 3 - 1, xx = wi + t % 3 - 1;
    float a = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? x[pix + (t / 3 - 1) * W + (t % 3 - 1)] : 0.f;
    if constexpr (sizeof(T) == 2) a = (float)(bf16_t)a;
    v[t] = a;
  }
  T* out = y + pix * Cout;
  for (int c0 = 0; c0 < Cout; c0 += 8) {
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = min(c0 + e, Cout - 1);
      float sacc = 0.f;
#pragma unroll
      for (int t = 0; t < 9; ++t) sacc = fmaf(v[t], sw[t * Cout + c], sacc);
      acc[e] = fmaxf((sacc - sm[c]) * si[c], 0.f);
    }
    if (c0 + 8 <= Cout && (Cout % 8) == 0) {
      if constexpr (sizeof(T) == 2) {
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (bf16_t)acc[e];
        *reinterpret_cast<uint4*>(out + c0) = __builtin_bit_cast(uint4, o);
      } else {
        *reinterpret_cast<f32x4*>(out + c0) = f32x4{acc[0], acc[1], acc[2], acc[3]};
        *reinterpret_cast<f32x4*>(out + c0 + 4) = f32x4{acc[4], acc[5], acc[6], acc[7]};
      }
    } else {
      for (int e = 0; e < 8 && c0 + e < Cout; ++e) out[c0 + e] = (T)acc[e];
    }
  }
}

// The stem with a small even Cout (DPN68: 10): the generic kernel computed
// 8-channel groups (16 channels for 10) and wrote each channel with its own
// 2-byte store.  Here a thread computes its pixel's COUT channels (pairs on
// v_pk_fma_f32, each element the fmaf chain of stem_conv1 in the same tap
// order), packs them into COUT / 2 dwords in LDS, and the workgroup writes its
// 256 pixels' rows (contiguous in y) as 16-B stores.  Bitwise equal to stem_conv1.
template <int COUT>
__global__ __launch_bounds__(256) void stem_conv1_small(const float* __restrict__ x, int N, int H,
                                                       int W, const float* __restrict__ wts,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ inv,
                                                       bf16_t* __restrict__ y) {
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  static_assert(COUT % 2 == 0 && (256 * COUT * 2) % 16 == 0, "channel pairs, 16-B rows");
  constexpr int DW = COUT / 2;   // dwords per pixel
  __shared__ __attribute__((aligned(16))) float sw[9 * COUT];
  __shared__ float sm[COUT], si[COUT];
  __shared__ __attribute__((aligned(16))) unsigned st[256 * DW];
  for (int i = threadIdx.x; i < 9 * COUT; i += blockDim.x) sw[i] = wts[i];
  for (int i = threadIdx.x; i < COUT; i += blockDim.x) { sm[i] = mean[i]; si[i] = inv[i]; }
  __syncthreads();
  const int64_t pix0 = (int64_t)blockIdx.x * 256;
  const int64_t npix = (int64_t)N * H * W;
  const int64_t pix = min(pix0 + threadIdx.x, npix - 1);
  const unsigned hw = npix < ((int64_t)1 << 32) ? (unsigned)pix % (unsigned)(H * W)
                                                : (unsigned)(pix % ((int64_t)H * W));
  const int hi = (int)(hw / (unsigned)W);
  const int wi = (int)(hw - (unsigned)hi * (unsigned)W);
  const float* xi = x + (pix - (int64_t)hw);
  float v[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int yy = hi + t / 3 - 1, xx = wi + t % 3 - 1;
    const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
    const int yc = min(max(yy, 0), H - 1), xc = min(max(xx, 0), W - 1);
    const float a = xi[yc * W + xc];
    v[t] = ok ? (float)(bf16_t)a : 0.f;
  }
#pragma unroll
  for (int k = 0; k < DW; ++k) {
    f32x2 acc = {0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 9; ++t)
      acc = __builtin_elementwise_fma(f32x2{v[t], v[t]}, *reinterpret_cast<const f32x2*>(sw + t * COUT + 2 * k), acc);
    const f32x2 tt = (acc - f32x2{sm[2 * k], sm[2 * k + 1]}) * f32x2{si[2 * k], si[2 * k + 1]};
    bf16x4 o = {(bf16_t)tt[0], (bf16_t)tt[1], (bf16_t)0.f, (bf16_t)0.f};
    o = relu_bf16(o);   // == bf16(relu(x)) bit for bit (device_common.h)
    st[threadIdx.x * DW + k] = __builtin_bit_cast(uint2, o).x;   // odd DW: conflict-free
  }
  __syncthreads();
  // the block's rows are contiguous in y: 16-B pieces, a partial last block by dwords
  const int64_t nb = min((int64_t)256, npix - pix0) * DW;   // dwords this block owns
  unsigned* yo = reinterpret_cast<unsigned*>(y + pix0 * COUT);
  for (int i = threadIdx.x; 4 * i < nb; i += 256) {
    if (4 * i + 4 <= nb)
      *reinterpret_cast<uint4*>(yo + 4 * i) = *reinterpret_cast<const uint4*>(st + 4 * i);
    else
      for (int e = 4 * i; e < nb; ++e) yo[e] = st[e];
  }
}

// The stem with Cout = 32 (Res2Net): the weights as [tap][Cout] and BN in LDS
// are read 4 channels per 16-B broadcast (ds_read_b128) instead of one float per
// FMA -- the per-FMA LDS reads bounded the generic kernel (122 us at 256 x 200 x
// 80) -- and each wave's 64 output pixels are staged in LDS so that a store
// instruction writes 1 KB contiguous (lane l: chunk l % 4 of pixel l / 4 + 16 s)
// instead of 16 B at a 64-B lane stride (4x the L2 write requests: 111 -> 91
// us); channel pairs on v_pk_fma_f32 and branch-free tap loads: 91 -> 78 us.
// Same products, same tap order, same roundings: bitwise equal to stem_conv1.
#ifndef STEM_PP
#define STEM_PP 1   // pixels per thread (2: half the weight reads, measured 78 -> 84 us)
#endif
__global__ __launch_bounds__(256) void stem_conv1_c32(const float* __restrict__ x, int N, int H,
                                                     int W, const float* __restrict__ wts,
                                                     const float* __restrict__ mean,
                                                     const float* __restrict__ inv,
                                                     bf16_t* __restrict__ y,
                                                     const int* __restrict__ vlen) {
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  constexpr int COUT = 32, PP = STEM_PP;   // PP pixels per thread, 256 apart
  __shared__ __attribute__((aligned(16))) float sw[9 * COUT];
  __shared__ __attribute__((aligned(16))) float sm[COUT], si[COUT];
  __shared__ __attribute__((aligned(16))) uint4 st[PP * 256 * 4];
  for (int i = threadIdx.x; i < 9 * COUT; i += blockDim.x) sw[i] = wts[i];
  for (int i = threadIdx.x; i < COUT; i += blockDim.x) { sm[i] = mean[i]; si[i] = inv[i]; }
  __syncthreads();
  const int64_t pix0 = (int64_t)blockIdx.x * (PP * 256);
  const int64_t npix = (int64_t)N * H * W;
  const int lane = threadIdx.x & 63, wb = threadIdx.x & ~63;
  // taps loaded unconditionally from clamped coordinates, then masked (the
  // bounds-checked loads compiled to a branch per tap)
  float v[PP][9];
#pragma unroll
  for (int u = 0; u < PP; ++u) {
    const int64_t pix = min(pix0 + 256 * u + threadIdx.x, npix - 1);
    const unsigned hw = npix < ((int64_t)1 << 32) ? (unsigned)pix % (unsigned)(H * W)
                                                  : (unsigned)(pix % ((int64_t)H * W));
    const int hi = (int)(hw / (unsigned)W);
    const int wi = (int)(hw - (unsigned)hi * (unsigned)W);
    const float* xi = x + (pix - (int64_t)hw);
    // ragged batch: rows past the utterance's frames are its SAME padding
    const int Hn = vlen ? valid_rows(vlen, 0, (int)((pix - (int64_t)hw) / ((int64_t)H * W)), H) : H;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int yy = hi + t / 3 - 1, xx = wi + t % 3 - 1;
      const bool ok = yy >= 0 && yy < Hn && xx >= 0 && xx < W;
      const int yc = min(max(yy, 0), H - 1), xc = min(max(xx, 0), W - 1);
      const float a = xi[yc * W + xc];
      v[u][t] = ok ? (float)(bf16_t)a : 0.f;
    }
  }
#pragma unroll
  for (int c = 0; c < COUT / 8; ++c) {
    const int c0 = 8 * c;
    // channel pairs on v_pk_fma_f32 (each element the fmaf of the scalar
    // chain, same tap order): the kernel was bound by VALU issue
    f32x2 acc[PP][4] = {};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const f32x4 w0 = *reinterpret_cast<const f32x4*>(sw + t * COUT + c0);
      const f32x4 w1 = *reinterpret_cast<const f32x4*>(sw + t * COUT + c0 + 4);
#pragma unroll
      for (int u = 0; u < PP; ++u) {
        const f32x2 vv = {v[u][t], v[u][t]};
        acc[u][0] = __builtin_elementwise_fma(vv, f32x2{w0[0], w0[1]}, acc[u][0]);
        acc[u][1] = __builtin_elementwise_fma(vv, f32x2{w0[2], w0[3]}, acc[u][1]);
        acc[u][2] = __builtin_elementwise_fma(vv, f32x2{w1[0], w1[1]}, acc[u][2]);
        acc[u][3] = __builtin_elementwise_fma(vv, f32x2{w1[2], w1[3]}, acc[u][3]);
      }
    }
    const f32x4 m0 = *reinterpret_cast<const f32x4*>(sm + c0);
    const f32x4 m1 = *reinterpret_cast<const f32x4*>(sm + c0 + 4);
    const f32x4 i0 = *reinterpret_cast<const f32x4*>(si + c0);
    const f32x4 i1 = *reinterpret_cast<const f32x4*>(si + c0 + 4);
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const f32x2 t0 = (acc[u][0] - f32x2{m0[0], m0[1]}) * f32x2{i0[0], i0[1]};
      const f32x2 t1 = (acc[u][1] - f32x2{m0[2], m0[3]}) * f32x2{i0[2], i0[3]};
      const f32x2 t2 = (acc[u][2] - f32x2{m1[0], m1[1]}) * f32x2{i1[0], i1[1]};
      const f32x2 t3 = (acc[u][3] - f32x2{m1[2], m1[3]}) * f32x2{i1[2], i1[3]};
      bf16x8 o;
      o[0] = (bf16_t)t0[0]; o[1] = (bf16_t)t0[1]; o[2] = (bf16_t)t1[0]; o[3] = (bf16_t)t1[1];
      o[4] = (bf16_t)t2[0]; o[5] = (bf16_t)t2[1]; o[6] = (bf16_t)t3[0]; o[7] = (bf16_t)t3[1];
      o = relu_bf16(o);   // == bf16(relu(x)) bit for bit (device_common.h)
      // chunk c of pixel lane at unit 4 lane + (c + lane / 2) % 4: conflict-free
      // 8-lane store groups and 16-lane read groups
      st[4 * (256 * u + wb + lane) + ((c + (lane >> 1)) & 3)] = __builtin_bit_cast(uint4, o);
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < PP; ++u)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int p = 16 * s + (lane >> 2), c = lane & 3;   // wave pixel, chunk
      const int64_t q = pix0 + 256 * u + wb + p;
      if (q < npix)
        *reinterpret_cast<uint4*>(y + q * COUT + 8 * c) = st[4 * (256 * u + wb + p) + ((c + (p >> 1)) & 3)];
    }
}

hipError_t launch_stem(DType t, const float* x, int N, int H, int W, const float* wts, int Cout,
                       const float* mean, const float* inv, void* y, hipStream_t s,
                       const int* vlen) {
  if (Cout > 64) return hipErrorInvalidValue;
  const int64_t n = (int64_t)N * H * W;
  const unsigned g = (unsigned)((n + 255) / 256);
  if (t == BF16 && Cout == 32) {
    hipLaunchKernelGGL(stem_conv1_c32, dim3((unsigned)((n + 256 * STEM_PP - 1) / (256 * STEM_PP))),
                       dim3(256), 0, s, x, N, H, W, wts, mean, inv,
                       (bf16_t*)y, vlen);
    return hipGetLastError();
  }
  if (vlen) return hipErrorInvalidValue;   // ragged batches: the c32 stem only
  if (t == BF16 && Cout == 10) {
    hipLaunchKernelGGL(stem_conv1_small<10>, dim3(g), dim3(256), 0, s, x, N, H, W, wts, mean, inv,
                       (bf16_t*)y);
    return hipGetLastError();
  }
  if (t == BF16)
    hipLaunchKernelGGL(stem_conv1<bf16_t>, dim3(g), dim3(256), 0, s, x, N, H, W, wts, Cout, mean,
                       inv, (bf16_t*)y);
  else
    hipLaunchKernelGGL(stem_conv1<float>, dim3(g), dim3(256), 0, s, x, N, H, W, wts, Cout, mean,
                       inv, (float*)y);
  return hipGetLastError();
}

int conv_kstep(DType t) { return t == BF16 ? Tr<bf16_t>::KSTEP : Tr<float>::KSTEP; }
int conv_vec(DType t) { return t == BF16 ? Tr<bf16_t>::VEC : Tr<float>::VEC; }

template <typename T, int WCO, int WPX>
static hipError_t launch_t(const ConvParams& p, const ConvLaunch& l, hipStream_t s) {
  const int M = p.N * p.Ho * p.Wo;
  dim3 grid((M + 64 * WPX - 1) / (64 * WPX), p.groups * p.cblocks, l.splitk > 0 ? l.splitk : 1);
  if (l.vec)
    hipLaunchKernelGGL((conv_igemm<T, WCO, WPX, true>), grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((conv_igemm<T, WCO, WPX, false>), grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

template <typename T, int WPX>
static hipError_t launch_wco(const ConvParams& p, const ConvLaunch& l, hipStream_t s) {
  switch (l.wco) {
    case 1: return launch_t<T, 1, WPX>(p, l, s);
    case 2: return launch_t<T, 2, WPX>(p, l, s);
    case 3: return launch_t<T, 3, WPX>(p, l, s);
    case 4: return launch_t<T, 4, WPX>(p, l, s);
    case 6: return launch_t<T, 6, WPX>(p, l, s);
    case 8: return launch_t<T, 8, WPX>(p, l, s);
  }
  return hipErrorInvalidValue;
}

template <typename T>
static hipError_t launch_wpx(const ConvParams& p, const ConvLaunch& l, hipStream_t s) {
  switch (l.wpx) {
    case 1: return launch_wco<T, 1>(p, l, s);
    case 2: return launch_wco<T, 2>(p, l, s);
    case 4: return launch_wco<T, 4>(p, l, s);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_conv(DType t, const ConvParams& p, const ConvLaunch& l, hipStream_t s) {
  return t == BF16 ? launch_wpx<bf16_t>(p, l, s) : launch_wpx<float>(p, l, s);
}

// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void splitk_reduce(const float* __restrict__ partial, int S,
                                                     int M, int coutp, int cout,
                                                     const float* __restrict__ mean,
                                                     const float* __restrict__ inv, int flags,
                                                     float* __restrict__ out, int ldo) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)M * cout) return;
  const int pix = (int)(idx / cout), c = (int)(idx - (int64_t)pix * cout);
  // fixed order z = 0, 1, ..., S-1; the slab loads of 8 consecutive z issued
  // together (a load -> add chain per slab waited out S L2 round trips)
  const float* src = partial + (size_t)pix * coutp + c;
  const size_t zs = (size_t)M * coutp;
  float v = 0.f;
  int z = 0;
  for (; z + 8 <= S; z += 8) {
    float t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = src[(size_t)(z + u) * zs];
#pragma unroll
    for (int u = 0; u < 8; ++u) v += t[u];
  }
  for (; z < S; ++z) v += src[(size_t)z * zs];
  if (flags & EPI_PRE_RELU) v = fmaxf(v, 0.f);
  if (flags & EPI_AFFINE) v = (v - mean[c]) * inv[c];
  if (flags & EPI_BN2D) v = bn2d(v, inv[c], mean[c]);
  if (flags & EPI_RELU) v = fmaxf(v, 0.f);
  out[(size_t)pix * ldo + c] = v;
}

hipError_t launch_splitk_reduce(const float* partial, int S, int M, int coutp, int cout,
                                const float* mean, const float* inv, int flags, float* out,
                                int ldo, hipStream_t s) {
  int64_t n = (int64_t)M * cout;
  hipLaunchKernelGGL(splitk_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, partial,
                     S, M, coutp, cout, mean, inv, flags, out, ldo);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------
// Stats pool over H (time) of NHWC [N,H,W,C] + head BN on the pooled vector.
// Block = (64 column-chunks) x TS time-slices.  A column chunk is VN
// consecutive channels of one (n, w); slices sum strided rows, then the
// slice partials are combined in fixed order through LDS (deterministic),
// first for the mean and then for the centred second moment (two-pass, as
// tf.nn.moments).  out[n][w*2C + c] = mean, out[n][w*2C + C + c] = std.
// in_mean / in_inv (optional): an input BN+ReLU applied to every element as it
// is read, rounded to T: the bits of DPN68's in-place concat_bn_relu pass
// (bnrelu_k, dpn_model.py:24-29) followed by the pool, without the extra
// read + write of the map.
// RAG (ragged batches, vlen): utterance n pools its valid_rows Hn, in the
// order the unpadded run (H = Hn) takes -- stats_pool_ts' slice count for Hn
// (bf16 / 8 channels: the sequential stats_pool_col up to 32 rows) -- the
// slices past it idle (their zero partials add exactly)
template <typename T, int VN, int TS, bool PRO = false, bool RAG = false>
__global__ __launch_bounds__(64 * TS, PRO ? 4 : 1) void stats_pool_k(const T* __restrict__ x, int N, int H,
                                                        int W, int C,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ inv,
                                                        float* __restrict__ out,
                                                        const float* __restrict__ in_mean,
                                                        const float* __restrict__ in_inv,
                                                        const int* __restrict__ vlen = nullptr,
                                                        int vsh = 0) {
  __shared__ float red[TS][64][VN];
  __shared__ float mu_s[64][VN];
  const int cx = threadIdx.x & 63, ts = threadIdx.x >> 6;
  const int chunks = C / VN;
  const int64_t gcol = (int64_t)blockIdx.x * 64 + cx;  // over N*W*chunks
  const bool valid = gcol < (int64_t)N * W * chunks;
  int n = 0, w = 0, ch = 0;
  if (valid) {
    n = (int)(gcol / ((int64_t)W * chunks));
    int r = (int)(gcol - (int64_t)n * W * chunks);
    w = r / chunks;
    ch = r - w * chunks;
  }
  // rows pooled and time slices (RAG: per utterance; the block's 64 columns
  // may span utterances, so per thread)
  int Hp = H, tsn = TS;
  if constexpr (RAG) {
    Hp = valid_rows(vlen, vsh, n, H);
    tsn = (sizeof(T) == 2 && VN == 8 && Hp <= 32) ? 1 : (Hp >= 64 ? 8 : (Hp >= 16 ? 4 : 1));
    if (tsn > TS) tsn = TS;
  }
  const bool mine = valid && ts < tsn;
  const size_t rowstride = (size_t)W * C;
  const T* base = x + ((size_t)n * H * W + w) * C + (size_t)ch * VN;
  constexpr bool pro = PRO;
  float pm[VN], pi[VN];
#pragma unroll
  for (int e = 0; e < VN; ++e) {
    pm[e] = pro ? in_mean[ch * VN + e] : 0.f;
    pi[e] = pro ? in_inv[ch * VN + e] : 1.f;
  }
  // element e of a row as the pool sees it (bnrelu_k's rounding when pro)
  auto elt = [&](float raw, int e) __attribute__((always_inline)) {
    return pro ? (float)(T)fmaxf((raw - pm[e]) * pi[e], 0.f) : raw;
  };
  // the first RM rows of this slice stay in registers for the second pass (the
  // re-read was the kernel's second HBM/L2 stream); same summation order
  constexpr int RM = 8;
  constexpr bool PK = sizeof(T) == 2 && VN == 8;   // rows kept as packed bf16 (exact either way)
  float v[PK ? 1 : RM][VN];
  bf16x8 vb[PK ? RM : 1];
  float s[VN];
#pragma unroll
  for (int e = 0; e < VN; ++e) s[e] = 0.f;
  const int tstep = RAG ? tsn : TS;
  if (mine) {
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const int h = ts + i * tstep;
      if (h < Hp) {
        const T* q = base + (size_t)h * rowstride;
        if constexpr (PK) {
          const bf16x8 r = ld16(q);
          bf16x8 t;
#pragma unroll
          for (int e = 0; e < VN; ++e) t[e] = (bf16_t)elt((float)r[e], e);
          vb[i] = t;
#pragma unroll
          for (int e = 0; e < VN; ++e) s[e] += (float)t[e];
        } else {
#pragma unroll
          for (int e = 0; e < VN; ++e) v[i][e] = elt((float)q[e], e);
#pragma unroll
          for (int e = 0; e < VN; ++e) s[e] += v[i][e];
        }
      }
    }
    // (unrolled: the loads of 4 rows issue together, the sums keep their order)
#pragma unroll 4
    for (int h = ts + RM * tstep; h < Hp; h += tstep) {
      const T* q = base + (size_t)h * rowstride;
#pragma unroll
      for (int e = 0; e < VN; ++e) s[e] += elt((float)q[e], e);
    }
  }
#pragma unroll
  for (int e = 0; e < VN; ++e) red[ts][cx][e] = s[e];
  __syncthreads();
  if (ts == 0) {
#pragma unroll
    for (int e = 0; e < VN; ++e) {
      float t = RAG ? red[0][cx][e] : 0.f;
      for (int k = RAG ? 1 : 0; k < (RAG ? tsn : TS); ++k) t += red[k][cx][e];
      mu_s[cx][e] = t / (float)Hp;
    }
  }
  __syncthreads();
  float mu[VN];
#pragma unroll
  for (int e = 0; e < VN; ++e) { mu[e] = mu_s[cx][e]; s[e] = 0.f; }
  if (mine) {
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      if (ts + i * tstep < Hp) {
#pragma unroll
        for (int e = 0; e < VN; ++e) {
          float x;
          if constexpr (PK) x = (float)vb[i][e];
          else x = v[i][e];
          const float d = x - mu[e];
          s[e] = __builtin_fmaf(d, d, s[e]);   // explicit: one rounding in every pool variant
        }
      }
    }
#pragma unroll 4
    for (int h = ts + RM * tstep; h < Hp; h += tstep) {
      const T* q = base + (size_t)h * rowstride;
#pragma unroll
      for (int e = 0; e < VN; ++e) {
        float d = elt((float)q[e], e) - mu[e];
        s[e] = __builtin_fmaf(d, d, s[e]);
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < VN; ++e) red[ts][cx][e] = s[e];
  __syncthreads();
  if (ts == 0 && valid) {
    float* o = out + (size_t)n * W * 2 * C + (size_t)w * 2 * C + (size_t)ch * VN;
#pragma unroll
    for (int e = 0; e < VN; ++e) {
      float t = RAG ? red[0][cx][e] : 0.f;
      for (int k = RAG ? 1 : 0; k < (RAG ? tsn : TS); ++k) t += red[k][cx][e];
      float sd = sqrtf(t / (float)Hp + 1e-5f);
      float m = mu[e];
      const int fm = w * 2 * C + ch * VN + e, fs = fm + C;
      if (mean) {
        m = bn2d(m, inv[fm], mean[fm]);
        sd = bn2d(sd, inv[fs], mean[fs]);
      }
      o[e] = m;
      o[C + e] = sd;
    }
  }
}

// Short utterance axis (H <= HM, bf16): one thread per 8-channel column of
// one (n, w), all H rows requested at once into registers (raw bf16, 4 VGPRs
// a row), both passes of tf.nn.moments from those registers, no LDS and no
// barrier: every byte is read once with H loads in flight per thread.
// Sequential summation over h (a fixed order per column, batch-independent).
template <int VN> struct PoolRaw { typedef unsigned t __attribute__((ext_vector_type(VN / 2))); };
template <> struct PoolRaw<2> { typedef unsigned t; };
// PRO: DPN68's concat_bn_relu applied to each row as it lands (bnrelu_k's
// rounding, as stats_pool_k<..., true>), the rows kept packed after it.
template <int HM, int VN, bool PRO = false>
__global__ __launch_bounds__(256) void stats_pool_col(const bf16_t* __restrict__ x, int N, int H,
                                                      int W, int C,
                                                      const float* __restrict__ mean,
                                                      const float* __restrict__ inv,
                                                      float* __restrict__ out,
                                                      const float* __restrict__ in_mean = nullptr,
                                                      const float* __restrict__ in_inv = nullptr) {
  typedef __bf16 bfv __attribute__((ext_vector_type(VN)));
  typedef typename PoolRaw<VN>::t uv;
  typedef float fv __attribute__((ext_vector_type(VN)));
  const int chunks = C / VN;
  const int64_t gcol = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gcol >= (int64_t)N * W * chunks) return;
  const int n = (int)(gcol / ((int64_t)W * chunks));
  const int r = (int)(gcol - (int64_t)n * W * chunks);
  const int w = r / chunks, ch = r - (r / chunks) * chunks;
  const bf16_t* base = x + ((size_t)n * H * W + w) * C + (size_t)ch * VN;
  const size_t rowstride = (size_t)W * C;
  uv v[HM];
#pragma unroll
  for (int h = 0; h < HM; ++h)
    if (h < H) v[h] = *reinterpret_cast<const uv*>(base + (size_t)h * rowstride);
  if constexpr (PRO) {
    float pm[VN], pi[VN];
#pragma unroll
    for (int e = 0; e < VN; ++e) {
      pm[e] = in_mean[ch * VN + e];
      pi[e] = in_inv[ch * VN + e];
    }
#pragma unroll
    for (int h = 0; h < HM; ++h)
      if (h < H) {
        bfv b = __builtin_bit_cast(bfv, v[h]);
#pragma unroll
        for (int e = 0; e < VN; ++e) b[e] = (bf16_t)fmaxf(((float)b[e] - pm[e]) * pi[e], 0.f);
        v[h] = __builtin_bit_cast(uv, b);
      }
  }
  float s[VN], q[VN];
#pragma unroll
  for (int e = 0; e < VN; ++e) s[e] = q[e] = 0.f;
#pragma unroll
  for (int h = 0; h < HM; ++h)
    if (h < H) {
      const bfv b = __builtin_bit_cast(bfv, v[h]);
#pragma unroll
      for (int e = 0; e < VN; ++e) s[e] += (float)b[e];
    }
  float mu[VN];
#pragma unroll
  for (int e = 0; e < VN; ++e) mu[e] = s[e] / (float)H;
  // the rows stay packed bf16 between the passes: without this the compiler
  // keeps every converted float of pass 1 live for pass 2
#pragma unroll
  for (int h = 0; h < HM; ++h) asm volatile("" : "+v"(v[h]));
#pragma unroll
  for (int h = 0; h < HM; ++h)
    if (h < H) {
      const bfv b = __builtin_bit_cast(bfv, v[h]);
#pragma unroll
      for (int e = 0; e < VN; ++e) {
        const float d = (float)b[e] - mu[e];
        q[e] = __builtin_fmaf(d, d, q[e]);   // as stats_pool_k (ragged batches pool there)
      }
    }
  float* o = out + (size_t)n * W * 2 * C + (size_t)w * 2 * C + (size_t)ch * VN;
  fv om, os;
#pragma unroll
  for (int e = 0; e < VN; ++e) {
    float sd = sqrtf(q[e] / (float)H + 1e-5f);
    float m = mu[e];
    const int fm = w * 2 * C + ch * VN + e, fs = fm + C;
    if (mean) {
      m = bn2d(m, inv[fm], mean[fm]);
      sd = bn2d(sd, inv[fs], mean[fs]);
    }
    om[e] = m;
    os[e] = sd;
  }
  *reinterpret_cast<fv*>(o) = om;
  *reinterpret_cast<fv*>(o + C) = os;
}

template <typename T, int VN>
static hipError_t stats_pool_ts(const T* x, int N, int H, int W, int C, const float* mean,
                                const float* inv, float* out, const float* in_mean,
                                const float* in_inv, hipStream_t s, const int* vlen, int vsh) {
  const int64_t cols = (int64_t)N * W * (C / VN);
  if (vlen) {   // ragged batch: per-utterance rows and slice counts (stats_pool_k RAG)
    if (in_mean) return hipErrorInvalidValue;
    hipLaunchKernelGGL((stats_pool_k<T, VN, 8, false, true>), dim3((unsigned)((cols + 63) / 64)),
                       dim3(64 * 8), 0, s, x, N, H, W, C, mean, inv, out, in_mean, in_inv, vlen, vsh);
    return hipGetLastError();
  }
  if constexpr (sizeof(T) == 2 && VN == 8) {
    if (H <= 32) {
      const unsigned b = (unsigned)((cols * 2 + 255) / 256);
      // 2 channels (4 B) per thread: at the headline (H = 25, T = 200) 2.5 grid
      // rounds of 8 waves per SIMD instead of 1.25 rounds at 7 (68 VGPRs with 4
      // channels), 35 -> 31 us in place; <16, 4> had compiled to 248 VGPRs.
      // Same per-element summation order as 4 channels per thread: same bits.
      // With DPN68's prologue (in_mean) the PRO form, so the fused pool sums the
      // same bnrelu_k-rounded rows in the same order as bnrelu + stats_pool_col
      if (in_mean) {
        if (H <= 16)
          hipLaunchKernelGGL((stats_pool_col<16, 2, true>), dim3(2 * b), dim3(256), 0, s, x, N, H, W, C, mean, inv, out, in_mean, in_inv);
        else if (H <= 25)
          hipLaunchKernelGGL((stats_pool_col<25, 2, true>), dim3(2 * b), dim3(256), 0, s, x, N, H, W, C, mean, inv, out, in_mean, in_inv);
        else
          hipLaunchKernelGGL((stats_pool_col<32, 2, true>), dim3(2 * b), dim3(256), 0, s, x, N, H, W, C, mean, inv, out, in_mean, in_inv);
        return hipGetLastError();
      }
      if (H <= 16)
        hipLaunchKernelGGL((stats_pool_col<16, 2>), dim3(2 * b), dim3(256), 0, s, x, N, H, W, C, mean, inv, out, nullptr, nullptr);
      else if (H <= 25)
        hipLaunchKernelGGL((stats_pool_col<25, 2>), dim3(2 * b), dim3(256), 0, s, x, N, H, W, C, mean, inv, out, nullptr, nullptr);
      else
        hipLaunchKernelGGL((stats_pool_col<32, 2>), dim3(2 * b), dim3(256), 0, s, x, N, H, W, C, mean, inv, out, nullptr, nullptr);
      return hipGetLastError();
    }
  }
  const unsigned blocks = (unsigned)((cols + 63) / 64);
  // more time-slices for many frames.  The slice count fixes the summation
  // order, so it depends on H only -- never on the batch (it used to drop to 4
  // past 2,048 blocks, i.e. a TDNN utterance's pooled bits changed with the
  // batch size past ~680 utterances)
  if (in_mean) {   // DPN68's concat_bn_relu on the read (time slices as below)
    if (H >= 64)
      hipLaunchKernelGGL((stats_pool_k<T, VN, 8, true>), dim3(blocks), dim3(64 * 8), 0, s, x, N, H, W,
                         C, mean, inv, out, in_mean, in_inv);
    else if (H >= 16)
      hipLaunchKernelGGL((stats_pool_k<T, VN, 4, true>), dim3(blocks), dim3(64 * 4), 0, s, x, N, H, W,
                         C, mean, inv, out, in_mean, in_inv);
    else
      hipLaunchKernelGGL((stats_pool_k<T, VN, 1, true>), dim3(blocks), dim3(64), 0, s, x, N, H, W, C,
                         mean, inv, out, in_mean, in_inv);
    return hipGetLastError();
  }
  if (H >= 64) {
    hipLaunchKernelGGL((stats_pool_k<T, VN, 8>), dim3(blocks), dim3(64 * 8), 0, s, x, N, H, W, C,
                       mean, inv, out, in_mean, in_inv);
  } else if (H >= 16) {
    hipLaunchKernelGGL((stats_pool_k<T, VN, 4>), dim3(blocks), dim3(64 * 4), 0, s, x, N, H, W, C,
                       mean, inv, out, in_mean, in_inv);
  } else {
    hipLaunchKernelGGL((stats_pool_k<T, VN, 1>), dim3(blocks), dim3(64), 0, s, x, N, H, W, C,
                       mean, inv, out, in_mean, in_inv);
  }
  return hipGetLastError();
}

hipError_t launch_stats_pool(DType t, const void* x, int N, int H, int W, int C,
                             const float* mean, const float* inv, float* out, hipStream_t s,
                             const float* in_mean, const float* in_inv, const int* vlen, int vsh) {
  if (t == BF16) {
    if (C % 8 == 0)
      return stats_pool_ts<bf16_t, 8>((const bf16_t*)x, N, H, W, C, mean, inv, out, in_mean, in_inv, s, vlen, vsh);
    if (C % 2 == 0)
      return stats_pool_ts<bf16_t, 2>((const bf16_t*)x, N, H, W, C, mean, inv, out, in_mean, in_inv, s, vlen, vsh);
    return stats_pool_ts<bf16_t, 1>((const bf16_t*)x, N, H, W, C, mean, inv, out, in_mean, in_inv, s, vlen, vsh);
  }
  if (C % 4 == 0)
    return stats_pool_ts<float, 4>((const float*)x, N, H, W, C, mean, inv, out, in_mean, in_inv, s, vlen, vsh);
  return stats_pool_ts<float, 1>((const float*)x, N, H, W, C, mean, inv, out, in_mean, in_inv, s, vlen, vsh);
}

// ----------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void avgpool3s2_k(const T* __restrict__ x, int ldx, int N,
                                                    int H, int W, int C, T* __restrict__ y,
                                                    int ldy, int Ho, int Wo) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)N * Ho * Wo * C) return;
  const int c = (int)(idx % C);
  const int64_t pix = idx / C;
  const int wo = (int)(pix % Wo);
  const int ho = (int)((pix / Wo) % Ho);
  const int n = (int)(pix / ((int64_t)Wo * Ho));
  float s = 0.f;
  for (int ky = 0; ky < 3; ++ky) {
    const int hi = 2 * ho - 1 + ky;
    if (hi < 0 || hi >= H) continue;
    for (int kx = 0; kx < 3; ++kx) {
      const int wi = 2 * wo - 1 + kx;
      if (wi < 0 || wi >= W) continue;
      s += (float)x[(((size_t)n * H + hi) * W + wi) * ldx + c];
    }
  }
  y[pix * ldy + c] = (T)(s / 9.0f);
}

// bf16, C % 8 == 0: 8 channels per thread with 16-byte loads/stores (same sum order)
__device__ uint4 g_pool_zero[1] = {};
__global__ __launch_bounds__(256) void avgpool3s2_v8(const bf16_t* __restrict__ x, int ldx, int N,
                                                     int H, int W, int C8, bf16_t* __restrict__ y,
                                                     int ldy, int Ho, int Wo,
                                                     const int* __restrict__ vlen, int vsh) {
  // 32-bit index math (the launcher guarantees N*Ho*Wo*C8 < 2^31): the 64-bit
  // divisions cost more than the loads
  const unsigned idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (unsigned)(N * Ho * Wo * C8)) return;
  const unsigned pix = idx / (unsigned)C8;
  const int c = (int)(idx - pix * (unsigned)C8) * 8;
  const unsigned nh = pix / (unsigned)Wo;
  const int wo = (int)(pix - nh * (unsigned)Wo);
  const int n = (int)(nh / (unsigned)Ho);
  const int ho = (int)(nh - (unsigned)n * (unsigned)Ho);
  const int Hn = valid_rows(vlen, vsh, n, H);   // ragged batch: padding past the utterance
  // all nine taps requested at once (padding taps read a zero line and add an
  // exact +0: the same sums in the same order as skipping them)
  bf16x8 v[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int hi = 2 * ho - 1 + t / 3, wi = 2 * wo - 1 + t % 3;
    const bool ok = hi >= 0 && hi < Hn && wi >= 0 && wi < W;
    v[t] = ld16(ok ? x + (((size_t)n * H + hi) * W + wi) * ldx + c
                   : reinterpret_cast<const bf16_t*>(g_pool_zero));
  }
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int hi = 2 * ho - 1 + t / 3, wi = 2 * wo - 1 + t % 3;
    if (hi >= 0 && hi < Hn && wi >= 0 && wi < W) {
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += (float)v[t][e];
    }
  }
  bf16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = (bf16_t)(s[e] / 9.0f);
  *reinterpret_cast<uint4*>(y + (size_t)pix * ldy + c) = __builtin_bit_cast(uint4, o);
}

hipError_t launch_avgpool3s2(DType t, const void* x, int ldx, int N, int H, int W, int C,
                             void* y, int ldy, int Ho, int Wo, hipStream_t s, const int* vlen,
                             int vsh) {
  if (t == BF16 && C % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0 &&
      (int64_t)N * Ho * Wo * (C / 8) < (int64_t)1 << 31) {
    const int64_t n = (int64_t)N * Ho * Wo * (C / 8);
    hipLaunchKernelGGL(avgpool3s2_v8, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       (const bf16_t*)x, ldx, N, H, W, C / 8, (bf16_t*)y, ldy, Ho, Wo, vlen, vsh);
    return hipGetLastError();
  }
  if (vlen) return hipErrorInvalidValue;   // ragged batches: the 8-channel kernel only
  const int64_t n = (int64_t)N * Ho * Wo * C;
  const unsigned g = (unsigned)((n + 255) / 256);
  if (t == BF16)
    hipLaunchKernelGGL(avgpool3s2_k<bf16_t>, dim3(g), dim3(256), 0, s, (const bf16_t*)x, ldx, N,
                       H, W, C, (bf16_t*)y, ldy, Ho, Wo);
  else
    hipLaunchKernelGGL(avgpool3s2_k<float>, dim3(g), dim3(256), 0, s, (const float*)x, ldx, N, H,
                       W, C, (float*)y, ldy, Ho, Wo);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------
// vlen (ragged batches): n = N * H * rowlen elements; the rows of utterance u
// past its vlen[u] frames are written as zeros -- a kernel whose K is padded
// past a row's channels (the TDNN's first layer: 80 of 96) reads the start of
// the next row against zero weights, and NaN padding times zero is NaN
__global__ void convert_f32_bf16(const float* __restrict__ x, bf16_t* __restrict__ y, int64_t n,
                                 const int* __restrict__ vlen, int H, int rowlen) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float v = x[i];
  if (vlen) {
    const int64_t r = i / rowlen;              // row over the batch
    const int u = (int)(r / H), h = (int)(r - (int64_t)u * H);
    if (h >= vlen[u]) v = 0.f;
  }
  y[i] = (bf16_t)v;
}

hipError_t launch_convert_f32(DType t, const float* x, void* y, int64_t n, hipStream_t s,
                              const int* vlen, int H, int rowlen) {
  if (t == F32) {
    if (vlen) return hipErrorInvalidValue;   // ragged batches run bf16 plans only
    return hipMemcpyAsync(y, x, n * 4, hipMemcpyDeviceToDevice, s);
  }
  hipLaunchKernelGGL(convert_f32_bf16, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x,
                     (bf16_t*)y, n, vlen, H, rowlen);
  return hipGetLastError();
}

template <typename T>
__global__ void copy_channels_k(const T* __restrict__ x, int ldx, T* __restrict__ y, int ldy,
                                int64_t npix, int C) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix * C) return;
  const int64_t p = i / C;
  const int c = (int)(i - p * C);
  y[p * ldy + c] = x[p * ldx + c];
}

hipError_t launch_copy_channels(DType t, const void* x, int ldx, void* y, int ldy, int64_t npix,
                                int C, hipStream_t s) {
  const int64_t n = npix * C;
  const unsigned g = (unsigned)((n + 255) / 256);
  if (t == BF16)
    hipLaunchKernelGGL(copy_channels_k<bf16_t>, dim3(g), dim3(256), 0, s, (const bf16_t*)x, ldx,
                       (bf16_t*)y, ldy, npix, C);
  else
    hipLaunchKernelGGL(copy_channels_k<float>, dim3(g), dim3(256), 0, s, (const float*)x, ldx,
                       (float*)y, ldy, npix, C);
  return hipGetLastError();
}

// In-place BN+ReLU over a channel prefix [npix][C] of a buffer with stride ld
// (DPN concat_bn_relu, dpn_model.py:24-29).
template <typename T>
__global__ void bnrelu_k(T* __restrict__ x, int ld, int64_t npix, int C,
                         const float* __restrict__ mean, const float* __restrict__ inv) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix * C) return;
  const int64_t p = i / C;
  const int c = (int)(i - p * C);
  T* q = x + p * ld + c;
  *q = (T)fmaxf(((float)*q - mean[c]) * inv[c], 0.f);
}

hipError_t launch_bnrelu_inplace(DType t, void* x, int ld, int64_t npix, int C, const float* mean,
                                 const float* inv, hipStream_t s) {
  const int64_t n = npix * C;
  const unsigned g = (unsigned)((n + 255) / 256);
  if (t == BF16)
    hipLaunchKernelGGL(bnrelu_k<bf16_t>, dim3(g), dim3(256), 0, s, (bf16_t*)x, ld, npix, C, mean,
                       inv);
  else
    hipLaunchKernelGGL(bnrelu_k<float>, dim3(g), dim3(256), 0, s, (float*)x, ld, npix, C, mean,
                       inv);
  return hipGetLastError();
}

}  // namespace vox

namespace vox {

// ----------------------------------------------------------------------------
// Attentive statistics pooling (models.py:273-303), fp32.  The attention MLP
// runs as fp32 1x1 convs on the conv path; these kernels are the glue:
//   conv1x1([x, tile(mean), tile(std)], W1) = x W1[:C] + [mean, std] W1[C:]
// so the (time-invariant) second term is one small GEMM per (n, w) and is
// added here before the tanh.
__global__ void convert_bf16_f32_k(const bf16_t* __restrict__ x, float* __restrict__ y, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = (float)x[i];
}

hipError_t launch_convert_bf16(const void* x, float* y, int64_t n, hipStream_t s) {
  const int64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(convert_bf16_f32_k, dim3((unsigned)blocks), dim3(256), 0, s,
                     reinterpret_cast<const bf16_t*>(x), y, n);
  return hipGetLastError();
}

// h[n][t][w][a] = tanh(h + b[n][w][a])
__global__ void att_bias_tanh_k(float* __restrict__ h, const float* __restrict__ b, int H, int W,
                                int A, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int a = (int)(i % A);
  const int64_t pix = i / A;
  const int w = (int)(pix % W);
  const int64_t n = pix / ((int64_t)H * W);
  h[i] = tanhf(h[i] + b[(n * W + w) * A + a]);
}

hipError_t launch_att_bias_tanh(float* h, const float* b, int N, int H, int W, int A,
                                hipStream_t s) {
  const int64_t total = (int64_t)N * H * W * A;
  hipLaunchKernelGGL(att_bias_tanh_k, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, h, b,
                     H, W, A, total);
  return hipGetLastError();
}

// Softmax over time of the logits, weighted mean and std of x, head BN, NHWC
// flatten (feature w*2C + j).  One thread per (n, w, c): coalesced over c.
template <typename T>
__global__ void att_pool_k(const T* __restrict__ x, const float* __restrict__ lg, int N, int H,
                           int W, int C, float eps, const float* __restrict__ mean,
                           const float* __restrict__ inv, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * W * C) return;
  const int c = (int)(i % C);
  const int64_t nw = i / C;
  const int w = (int)(nw % W);
  const int64_t n = nw / W;
  const int64_t base = (n * H * W + w) * C + c, st = (int64_t)W * C;
  float mx = -INFINITY;
  for (int t = 0; t < H; ++t) mx = fmaxf(mx, lg[base + t * st]);
  float sum = 0.f;
  for (int t = 0; t < H; ++t) sum += expf(lg[base + t * st] - mx);
  float wm = 0.f, wss = 0.f;
  for (int t = 0; t < H; ++t) {
    const float wt = expf(lg[base + t * st] - mx) / sum;
    const float xv = (float)x[base + t * st];
    wm += xv * wt;
    wss += xv * xv * wt;
  }
  const float sd = sqrtf(wss - wm * wm + eps);
  float* o = out + n * W * 2 * C + (int64_t)w * 2 * C;
  const int j0 = w * 2 * C + c, j1 = j0 + C;
  o[c] = mean ? bn2d(wm, inv[j0], mean[j0]) : wm;
  o[C + c] = mean ? bn2d(sd, inv[j1], mean[j1]) : sd;
}

hipError_t launch_att_pool(DType t, const void* x, const float* lg, int N, int H, int W, int C,
                           float eps, const float* mean, const float* inv, float* out,
                           hipStream_t s) {
  const int64_t total = (int64_t)N * W * C;
  const dim3 grid((unsigned)((total + 255) / 256));
  if (t == BF16)
    hipLaunchKernelGGL((att_pool_k<bf16_t>), grid, dim3(256), 0, s,
                       reinterpret_cast<const bf16_t*>(x), lg, N, H, W, C, eps, mean, inv, out);
  else
    hipLaunchKernelGGL((att_pool_k<float>), grid, dim3(256), 0, s,
                       reinterpret_cast<const float*>(x), lg, N, H, W, C, eps, mean, inv, out);
  return hipGetLastError();
}

}  // namespace vox

namespace vox {
// ----------------------------------------------------------------------------
// Small-K 1x1 conv with the BN + ReLU input prologue (DPN68's first projection
// and 1x1a read the 10-channel stem output, dpn_model.py:40-45,111-130): too
// narrow a K for the MFMA paths (one 32-step of which 22 are zero).  Thread =
// (pixel, 8 output channels): x -> relu((x - m) * inv) rounded to bf16 (the
// MFMA operand the other paths feed), products with the bf16 weights exact in
// fp32, summed over k in order, one bf16 rounding of the sum.  Weights
// [Cout][kp] (the generic layout).
//
// Thread = (pixel, 8-channel output chunk), the chunk fixed per thread so its
// 8 x K weights stay in registers: the NC = Cout / 8 lanes of a pixel store its
// Cout channels as one contiguous run.  Each thread takes PXU pixels per pass
// (their inputs requested together as dwords) so a wave waits out one memory
// round trip per PXU pixels: the thread-per-pixel form stored 16 B per
// ldy-strided pixel per instruction, a one-pixel loop waited per pixel, and
// both ran at 1.5-1.8 TB/s on DPN68's 3 M-pixel stage-1 maps.
constexpr int SMALLK_PX = 16;   // pixel slots of a workgroup
constexpr int SMALLK_PXU = 8;   // pixels per thread per pass
template <int K>
__global__ __launch_bounds__(256) void conv1x1_smallk(ConvParams p) {
  static_assert(K % 2 == 0, "dword input loads");
  const int nc = p.Cout >> 3;
  const int tid = threadIdx.x;
  const int c = tid % nc, pl = tid / nc;
  const int co = 8 * c;
  const bf16_t* __restrict__ Wt = reinterpret_cast<const bf16_t*>(p.w);
  float w[8][K];
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int k = 0; k < K; ++k) w[e][k] = (float)Wt[(size_t)(co + e) * p.kp + k];
  float bm[K], bi[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    bm[k] = p.in_mean ? p.in_mean[k] : 0.f;
    bi[k] = p.in_mean ? p.in_inv[k] : 1.f;
  }
  const int64_t npx = (int64_t)p.N * p.H * p.W;
  const bf16_t* __restrict__ X0 = reinterpret_cast<const bf16_t*>(p.x);
  bf16_t* Y = reinterpret_cast<bf16_t*>(p.y);
  bf16_t* Y2 = reinterpret_cast<bf16_t*>(p.y2);
  const bool lo = co < p.ysplit;
  constexpr int PASS = SMALLK_PX * SMALLK_PXU;
  for (int64_t base = (int64_t)blockIdx.x * PASS + pl; base < npx;
       base += (int64_t)gridDim.x * PASS) {
    unsigned raw[SMALLK_PXU][K / 2];
#pragma unroll
    for (int u = 0; u < SMALLK_PXU; ++u) {
      const int64_t pix = base + SMALLK_PX * u;
      const unsigned* src = reinterpret_cast<const unsigned*>(X0 + (pix < npx ? pix : 0) * p.ldx);
#pragma unroll
      for (int k = 0; k < K / 2; ++k) raw[u][k] = src[k];
    }
#pragma unroll
    for (int u = 0; u < SMALLK_PXU; ++u) {
      const int64_t pix = base + SMALLK_PX * u;
      if (pix >= npx) break;
      float xv[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        float v = __builtin_bit_cast(float, (k & 1) ? raw[u][k / 2] & 0xFFFF0000u : raw[u][k / 2] << 16);
        if (p.in_mean) v = fmaxf((v - bm[k]) * bi[k], 0.f);
        xv[k] = (float)(bf16_t)v;   // the bf16 operand the MFMA paths feed
      }
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) acc = fmaf(xv[k], w[e][k], acc);
        o[e] = (bf16_t)acc;
      }
      bf16_t* dst = lo ? Y + pix * p.ldy + co : Y2 + pix * p.ldy2 + (co - p.ysplit);
      *reinterpret_cast<uint4*>(dst) = __builtin_bit_cast(uint4, o);
    }
  }
}

// Version 2 (the product kernel; version 1 above behind VOXEMB_SMALLK_V1, bitwise
// equal): version 1 ran at 2.8 TB/s, instruction-bound -- each of the Cout / 8
// threads of a pixel re-loaded its 10 inputs and re-ran their BN + ReLU prologue
// (about 140 VALU per thread-pixel).  Here a workgroup pass of SMALLK_PX x
// SMALLK_PXU pixels first stages the pass's prologued inputs once (thread = one
// (pixel, channel pair), the fixed pair's mean / inverse in registers) as fp32
// rows in LDS, then every thread reads its pixel's row back (LDS broadcast) and
// runs the same fma chain, k = 0..K-1 in order, on packed pairs of output
// channels (v_pk_fma_f32: per element the same rounding as the scalar chain).
constexpr int SMALLK_ROW = 12;   // floats per staged pixel row (K = 10, 16-B aligned rows)
template <int K, int NC>
__global__ __launch_bounds__(256) void conv1x1_smallk2(ConvParams p) {
  static_assert(K % 2 == 0 && K <= SMALLK_ROW, "dword input loads, one staged row");
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  constexpr int PASS = SMALLK_PX * SMALLK_PXU;
  constexpr int NT = SMALLK_PX * NC;    // threads (Cout = 8 NC)
  __shared__ __attribute__((aligned(16))) float xs[PASS * SMALLK_ROW];
  const int tid = threadIdx.x;
  const int c = tid % NC, pl = tid / NC;
  const int co = 8 * c;
  const bf16_t* __restrict__ Wt = reinterpret_cast<const bf16_t*>(p.w);
  f32x2 w[4][K];   // output channel pairs (co + 2h, co + 2h + 1)
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int k = 0; k < K; ++k)
      w[h][k] = f32x2{(float)Wt[(size_t)(co + 2 * h) * p.kp + k], (float)Wt[(size_t)(co + 2 * h + 1) * p.kp + k]};
  // staging role: thread -> channel pair kq (fixed), pixels sp0 + i SPP of the pass
  constexpr int KQ = K / 2;
  constexpr int SPP = NT / KQ;                  // pixels staged per sweep
  constexpr int NS = (PASS + SPP - 1) / SPP;    // sweeps per pass
  const int kq = tid % KQ, sp0 = tid / KQ;
  const bool stager = sp0 < SPP;
  float bm0 = 0.f, bm1 = 0.f, bi0 = 1.f, bi1 = 1.f;
  if (p.in_mean) {
    bm0 = p.in_mean[2 * kq]; bm1 = p.in_mean[2 * kq + 1];
    bi0 = p.in_inv[2 * kq]; bi1 = p.in_inv[2 * kq + 1];
  }
  const int64_t npx = (int64_t)p.N * p.H * p.W;
  const bf16_t* __restrict__ X0 = reinterpret_cast<const bf16_t*>(p.x);
  bf16_t* Y = reinterpret_cast<bf16_t*>(p.y);
  bf16_t* Y2 = reinterpret_cast<bf16_t*>(p.y2);
  const bool lo = co < p.ysplit;
  const int64_t gstep = (int64_t)gridDim.x * PASS;
  // the next pass's inputs are requested before this pass's outputs are computed
  unsigned raw[NS];
  auto fetch = [&](int64_t base) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const int sp = sp0 + i * SPP;
      const int64_t pix = base + sp;
      raw[i] = (stager && sp < PASS && pix < npx)
                   ? *reinterpret_cast<const unsigned*>(X0 + pix * p.ldx + 2 * kq) : 0u;
    }
  };
  int64_t base = (int64_t)blockIdx.x * PASS;
  if (base < npx) fetch(base);
  for (; base < npx; base += gstep) {
    if (stager) {
#pragma unroll
      for (int i = 0; i < NS; ++i) {
        const int sp = sp0 + i * SPP;
        if (sp >= PASS) break;
        float v0 = __builtin_bit_cast(float, raw[i] << 16);
        float v1 = __builtin_bit_cast(float, raw[i] & 0xFFFF0000u);
        if (p.in_mean) {
          v0 = fmaxf((v0 - bm0) * bi0, 0.f);
          v1 = fmaxf((v1 - bm1) * bi1, 0.f);
        }
        // the bf16 operand the MFMA paths feed
        *reinterpret_cast<f32x2*>(&xs[sp * SMALLK_ROW + 2 * kq]) = f32x2{(float)(bf16_t)v0, (float)(bf16_t)v1};
      }
    }
    __syncthreads();
    if (base + gstep < npx) fetch(base + gstep);
#pragma unroll 2
    for (int u = 0; u < SMALLK_PXU; ++u) {
      const int sp = pl + SMALLK_PX * u;
      const int64_t pix = base + sp;
      if (pix >= npx) break;
      float xv[SMALLK_ROW];
      *reinterpret_cast<f32x4*>(&xv[0]) = *reinterpret_cast<const f32x4*>(&xs[sp * SMALLK_ROW]);
      *reinterpret_cast<f32x4*>(&xv[4]) = *reinterpret_cast<const f32x4*>(&xs[sp * SMALLK_ROW + 4]);
      *reinterpret_cast<f32x4*>(&xv[8]) = *reinterpret_cast<const f32x4*>(&xs[sp * SMALLK_ROW + 8]);
      f32x2 acc[4];
#pragma unroll
      for (int h = 0; h < 4; ++h) acc[h] = f32x2{0.f, 0.f};
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int h = 0; h < 4; ++h) acc[h] = __builtin_elementwise_fma(f32x2{xv[k], xv[k]}, w[h][k], acc[h]);
      bf16x8 o;
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        o[2 * h] = (bf16_t)acc[h][0];
        o[2 * h + 1] = (bf16_t)acc[h][1];
      }
      bf16_t* dst = lo ? Y + pix * p.ldy + co : Y2 + pix * p.ldy2 + (co - p.ysplit);
      *reinterpret_cast<uint4*>(dst) = __builtin_bit_cast(uint4, o);
    }
    __syncthreads();
  }
}

int conv1x1_smallk_ok(const ConvParams& p) {
  return p.kh == 1 && p.kw == 1 && p.sh == 1 && p.sw == 1 && p.ph == 0 && p.pw == 0 &&
         p.groups == 1 && p.Cin == 10 && p.Cout % 8 == 0 && p.Cout <= 128 && p.flags == 0 &&
         !p.x2 && !p.res &&
         p.ldy % 8 == 0 && (p.ysplit >= (1 << 30) || (p.ysplit % 8 == 0 && p.ldy2 % 8 == 0)) &&
         p.Ho == p.H && p.Wo == p.W && p.ldx % 2 == 0 && (uintptr_t)p.x % 4 == 0;
}

hipError_t launch_conv1x1_smallk(const ConvParams& p, hipStream_t s, int v1) {
  if (!conv1x1_smallk_ok(p)) return hipErrorInvalidValue;
  const int64_t n = (int64_t)p.N * p.H * p.W;
  const int64_t blocks = (n + SMALLK_PX * SMALLK_PXU - 1) / (SMALLK_PX * SMALLK_PXU);
  // a few passes per workgroup (the weight loads amortised)
  const unsigned G = (unsigned)(blocks < 4096 ? blocks : 4096);
  if (v1)
    hipLaunchKernelGGL((conv1x1_smallk<10>), dim3(G), dim3(SMALLK_PX * (p.Cout / 8)), 0, s, p);
  else if (p.Cout == 96)
    hipLaunchKernelGGL((conv1x1_smallk2<10, 12>), dim3(G), dim3(SMALLK_PX * 12), 0, s, p);
  else if (p.Cout == 128)
    hipLaunchKernelGGL((conv1x1_smallk2<10, 16>), dim3(G), dim3(SMALLK_PX * 16), 0, s, p);
  else
    hipLaunchKernelGGL((conv1x1_smallk<10>), dim3(G), dim3(SMALLK_PX * (p.Cout / 8)), 0, s, p);
  return hipGetLastError();
}
}  // namespace vox

// Kaldi-compatible FBANK front end and sliding-window CMN on the GPU -- the
// wav -> features half of the reference pipeline (prepare_data.sh:66-70:
// `compute-fbank-feats --config=conf/fbank80.conf`, tensorflow/tf_extract.py:63:
// `apply-cmvn-sliding --norm-vars=false --center=true --cmn-window=300`), so
// that wav -> embedding can run entirely on the device.
//
// fbank_k: one wavefront per frame (a 64-thread workgroup, 4 KB of LDS), all
// of Kaldi's per-frame steps in registers/LDS: frame extraction (snip_edges),
// optional Gaussian dither, DC-offset removal, pre-emphasis 0.97, "povey"
// window, zero padding to NFFT, real FFT as an NFFT/2-point complex radix-2
// FFT in LDS + the real-spectrum unpack, power spectrum, the triangular mel
// filterbank (Kaldi's MelBanks weights, built on the host in float32 exactly
// as Kaldi builds them) and log(max(e, FLT_EPSILON)).  float32 throughout, as
// Kaldi's BaseFloat; FFT and sum orders differ from Kaldi's split-radix / BLAS,
// so agreement with an exact-arithmetic restatement is to float32 rounding.
// HBM traffic is ~1.6 B per sample read + 4 B per output value: the kernel is
// latency-bound on its FFT, a few microseconds per batch of utterances.
//
// cmn_k: one thread per (utterance, feature bin) runs Kaldi's sliding-window
// recursion (SlidingWindowCmnInternal, double-precision running sums) over the
// utterance's frames: bit-identical to the host vox_sliding_cmn.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <mutex>
#include <string>
#include <deque>
#include <vector>

#include "../../include/voxemb.h"

int vox_set_error(int code, const char* msg);

namespace vox {

struct FbankDev {
  int frame_len, frame_shift, num_bins, remove_dc;
  float preemph, dither;
  unsigned long long seed;
  const float* win;     // [frame_len] povey window
  const float* mel;     // [num_bins][NFFT/2] dense MelBanks weights
  const int* mel_lo;    // first nonzero FFT bin per mel bin
  const int* mel_n;     // nonzero count per mel bin
  const float* tw;      // [NFFT/4] x (cos, sin) of -2 pi k / (NFFT/2)
  const float* utw;     // [NFFT/2 + 1] x (cos, sin) of -2 pi k / NFFT (real unpack)
};

// counter-based Gaussian for the dither: splitmix64 -> two uniforms -> Box-Muller
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float gauss(unsigned long long key) {
  const unsigned long long r = mix64(key);
  const float u1 = ((float)(r >> 40) + 1.0f) * (1.0f / 16777217.0f);   // (0, 1]
  const float u2 = (float)((r >> 16) & 0xFFFFFF) * (1.0f / 16777216.0f);
  return sqrtf(-2.0f * logf(u1)) * cosf(6.28318530717958647692f * u2);
}

#pragma clang fp contract(off)
template <int NFFT>
__global__ __launch_bounds__(64) void fbank_k(const float* __restrict__ wav,
                                              const int64_t* __restrict__ samp_off,
                                              const int64_t* __restrict__ frame_off,
                                              const uint64_t* __restrict__ utt_key, int n_utt,
                                              FbankDev d, float* __restrict__ out) {
  constexpr int NC = NFFT / 2;          // complex FFT size
  constexpr int LOGNC = NC == 256 ? 8 : 7;
  __shared__ float xr[NFFT + 1];        // time samples (+1: x[-1] slot at index 0)
  __shared__ float cre[NC], cim[NC];    // complex FFT buffers
  __shared__ float pw[NC + 1];          // power spectrum
  const int lane = threadIdx.x;
  const int64_t f = blockIdx.x;         // global frame index
  // utterance of this frame (frame_off is sorted, n_utt + 1 entries)
  int lo = 0, hi = n_utt;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (frame_off[mid] <= f) lo = mid;
    else hi = mid;
  }
  const int u = lo;
  const int64_t t = f - frame_off[u];
  const float* src = wav + samp_off[u] + t * d.frame_shift;
  const int L = d.frame_len;
  // per-utterance stream: the caller's key (a hash of the utterance id) keeps the
  // noise independent across utterances yet the same at any batch position
  const unsigned long long dkey = d.seed ^ (utt_key ? mix64(utt_key[u] ^ 0xD1B54A32D192ED03ull) : 0ull);

  // 1. extract (+ dither), 2. DC offset
  float v[(NFFT + 63) / 64];
  float part = 0.f;
#pragma unroll
  for (int k = 0; k < (NFFT + 63) / 64; ++k) {
    const int i = lane + 64 * k;
    float x = 0.f;
    if (i < L) {
      x = src[i];
      if (d.dither != 0.f)
        x += d.dither * gauss(dkey ^ mix64(((unsigned long long)t << 16) ^ (unsigned)i));
    }
    v[k] = x;
    part += x;
  }
  if (d.remove_dc) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
    const float mean = part / (float)L;
#pragma unroll
    for (int k = 0; k < (NFFT + 63) / 64; ++k)
      if (lane + 64 * k < L) v[k] -= mean;
  }
  // 3. pre-emphasis x[i] -= c x[i-1] (x[0] -= c x[0]), 4. window
#pragma unroll
  for (int k = 0; k < (NFFT + 63) / 64; ++k) xr[1 + lane + 64 * k] = v[k];
  if (lane == 0) xr[0] = v[0];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < (NFFT + 63) / 64; ++k) {
    const int i = lane + 64 * k;
    float y = 0.f;
    if (i < L) {
      y = v[k];
      if (d.preemph != 0.f) y = y - d.preemph * xr[i];   // xr[i] = x[i-1] (x[0] for i = 0)
      y = y * d.win[i];
    }
    v[k] = y;
  }
  __syncthreads();
  // 5. pack y[2n] + i y[2n+1] in bit-reversed order for the radix-2 DIT FFT
#pragma unroll
  for (int k = 0; k < (NFFT + 63) / 64; ++k) xr[lane + 64 * k] = v[k];
  __syncthreads();
  for (int n = lane; n < NC; n += 64) {
    const int r = (int)(__builtin_bitreverse32((unsigned)n) >> (32 - LOGNC));
    cre[r] = xr[2 * n];
    cim[r] = xr[2 * n + 1];
  }
  __syncthreads();
  // 6. NC-point complex FFT, exp(-2 pi i nk / NC)
  for (int m = 1; m < NC; m <<= 1) {
    for (int b = lane; b < NC / 2; b += 64) {
      const int j = b & (m - 1);
      const int i1 = ((b - j) << 1) + j, i2 = i1 + m;
      const int ti = j * (NC / (2 * m));
      const float wr = d.tw[2 * ti], wi = d.tw[2 * ti + 1];
      const float br = cre[i2], bi = cim[i2];
      const float cr = br * wr - bi * wi, ci = br * wi + bi * wr;
      const float ar = cre[i1], ai = cim[i1];
      cre[i1] = ar + cr;
      cim[i1] = ai + ci;
      cre[i2] = ar - cr;
      cim[i2] = ai - ci;
    }
    __syncthreads();
  }
  // 7. real-spectrum unpack X[k] = (Z[k] + Z*[NC-k])/2 - i W^k (Z[k] - Z*[NC-k])/2,
  //    power |X[k]|^2 for k = 0..NC
  for (int k = lane; k <= NC; k += 64) {
    const int k1 = k & (NC - 1), k2 = (NC - k) & (NC - 1);
    const float zr = cre[k1], zi = cim[k1], yr = cre[k2], yi = -cim[k2];
    const float er = 0.5f * (zr + yr), ei = 0.5f * (zi + yi);   // even part
    const float or_ = 0.5f * (zr - yr), oi = 0.5f * (zi - yi);  // (Z - Z*)/2
    const float wr = d.utw[2 * k], wi = d.utw[2 * k + 1];
    // -i * W * o
    const float tr = wr * or_ - wi * oi, ti = wr * oi + wi * or_;
    const float xr_ = er + ti, xi_ = ei - tr;
    pw[k] = xr_ * xr_ + xi_ * xi_;
  }
  __syncthreads();
  // 8. mel filterbank, 9. log
  for (int b = lane; b < d.num_bins; b += 64) {
    const int k0 = d.mel_lo[b], n = d.mel_n[b];
    const float* w = d.mel + (size_t)b * NC + k0;
    float e = 0.f;
    for (int i = 0; i < n; ++i) e += w[i] * pw[k0 + i];
    e = fmaxf(e, 1.1920928955078125e-07f);   // FLT_EPSILON
    out[f * d.num_bins + b] = logf(e);
  }
}

// Kaldi SlidingWindowCmnInternal (center = true: window [t - W/2, t - W/2 + W)
// shifted into [0, T); center = false: [t - W, t], at least min_window frames),
// double running sums, output = x + (-1/n) * sum: one thread per (utt, bin).
__global__ void cmn_k(const float* __restrict__ in, const int64_t* __restrict__ frame_off,
                      int n_utt, int F, int W, int center, float* __restrict__ out) {
  const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (long)n_utt * F) return;
  const int u = (int)(id / F), c = (int)(id - (long)u * F);
  const int64_t base = frame_off[u];
  const int T = (int)(frame_off[u + 1] - base);
  const float* x = in + base * F + c;
  float* y = out + base * F + c;
  const int min_window = 100;
  double s = 0.0;
  int last_start = -1, last_end = -1;
  for (int t = 0; t < T; ++t) {
    int ws, we;
    if (center) {
      ws = t - W / 2;
      we = ws + W;
    } else {
      ws = t - W;
      we = t + 1;
    }
    if (ws < 0) {
      we -= ws;
      ws = 0;
    }
    if (!center && we < min_window) we = min_window;
    if (we > T) {
      ws -= we - T;
      we = T;
      if (ws < 0) ws = 0;
    }
    if (last_start == -1) {
      for (int r = ws; r < we; ++r) s += (double)x[(long)r * F];
    } else {
      if (ws > last_start) s -= (double)x[(long)last_start * F];
      if (we > last_end) s += (double)x[(long)last_end * F];
    }
    const int n = we - ws;
    last_start = ws;
    last_end = we;
    const double alpha = -1.0 / n;
    y[(long)t * F] = (float)((double)x[(long)t * F] + alpha * s);
  }
}

// cmn_k's recursion (center = true) with its loads issued ahead: the windows
// advance by at most one row per frame, so the rows a block of CMN_B frames
// subtracts, adds and centres are known before any of its sums -- all 3 CMN_B
// loads go out first, then the CMN_B dependent double updates run in cmn_k's
// order.  One thread per (utterance, bin) still, so the frames are a serial
// chain; cmn_k waited out a load round trip per frame.
constexpr int CMN_B = 32;   // <= 64: the per-frame flags are 64-bit masks
static_assert(CMN_B <= 64, "flag masks");
__global__ __launch_bounds__(256) void cmn_fast_k(const float* __restrict__ in,
                                                  const int64_t* __restrict__ frame_off,
                                                  int n_utt, int F, int W,
                                                  float* __restrict__ out) {
  const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (long)n_utt * F) return;
  const int u = (int)(id / F), c = (int)(id - (long)u * F);
  const int64_t base = frame_off[u];
  const int T = (int)(frame_off[u + 1] - base);
  if (T <= 0) return;
  const float* __restrict__ x = in + base * F + c;   // row r at x[r * F] (T * F < 2^31)
  float* __restrict__ y = out + base * F + c;
  // Kaldi's centred window of frame t, branch-free: [max(t - W/2, 0), + W),
  // shifted left (not below 0) to end at T
  auto win = [&](int t, int& ws, int& we) {
    const int a = max(t - W / 2, 0);
    const bool over = a + W > T;
    ws = over ? max(T - W, 0) : a;
    we = over ? T : a + W;
  };
  int ls, le;
  win(0, ls, le);
  double s = 0.0;
  for (int r = ls; r < le; r += CMN_B) {   // the first window, in row order
    float v[CMN_B];
#pragma unroll
    for (int k = 0; k < CMN_B; ++k) v[k] = x[min(r + k, T - 1) * F];
#pragma unroll
    for (int k = 0; k < CMN_B; ++k)
      if (r + k < le) s += (double)v[k];
  }
  int n_prev = -1;
  double alpha = 0.0;
  for (int t = 0; t < T; t += CMN_B) {
    // every row this block of frames subtracts, adds and centres, requested first
    float xs[CMN_B], xa[CMN_B], xt[CMN_B];
    uint64_t dsub = 0, dadd = 0, nchg = 0;   // one bit per frame of the block
    int ps = ls, pe = le, pn = le - ls;
#pragma unroll
    for (int k = 0; k < CMN_B; ++k) {
      const int tt = t + k;
      int ws = ps, we = pe;
      if (tt > 0) win(min(tt, T - 1), ws, we);
      dsub |= (uint64_t)(ws > ps) << k;
      dadd |= (uint64_t)(we > pe) << k;
      xs[k] = x[ps * F];
      xa[k] = x[min(pe, T - 1) * F];
      xt[k] = x[min(tt, T - 1) * F];
      nchg |= (uint64_t)(we - ws != pn) << k;
      pn = we - ws;
      ps = ws;
      pe = we;
    }
#pragma unroll
    for (int k = 0; k < CMN_B; ++k) {
      if (t + k >= T) break;
      if ((dsub >> k) & 1) s -= (double)xs[k];
      if ((dadd >> k) & 1) s += (double)xa[k];
      // the window size is W away from the utterance edges: its -1/n (an IEEE
      // double division, a long dependent sequence) only when it changes
      if (n_prev < 0 || ((nchg >> k) & 1)) {
        int ws, we;
        win(t + k, ws, we);
        n_prev = we - ws;
        alpha = -1.0 / n_prev;
      }
      y[(t + k) * F] = (float)((double)xt[k] + alpha * s);
    }
    ls = ps;
    le = pe;
  }
}

// ---- Kaldi CompressedMatrix round trip (`copy-feats --compress=true`,
// prepare_data.sh:69; Kaldi compressed-matrix.cc, not vendored: its published
// kAutomaticMethod -> kSpeechFeature for rows > 8, kTwoByteAuto otherwise).
// Per utterance the blob is what follows the "CM " / "CM2 " token:
//   float min, float range, int32 rows, int32 cols,
//   rows > 8:  uint16 [cols][4] percentiles (0, 25, 75, 100), uint8 [cols][rows]
//   rows <= 8: uint16 [rows][cols]
// cm_head_k writes the global header; cm_col_k one column: the four order
// statistics by a 4 x 8-bit radix select (exact, as Kaldi's nth_element
// chain), the column header, the bytes, and the decoded values in Kaldi C++
// CopyToMat order (the one apply-cmvn-sliding sees, tf_extract.py:63).
__device__ __forceinline__ unsigned cm_key(float v) {
  const unsigned u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float cm_unkey(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
// FloatToUint16: float ratio, clamp, + 0.499 in double, truncate
__device__ __forceinline__ int cm_u16(float mn, float range, float v) {
  float f = (v - mn) / range;
  if (f > 1.0f) f = 1.0f;
  if (f < 0.0f) f = 0.0f;
  return (int)((double)(f * 65535.0f) + 0.499);
}
// Uint16ToFloat: min + range * 1.52590218966964e-05f * v, float, left to right
__device__ __forceinline__ float cm_f16(float mn, float range, int v) {
  return mn + (range * 1.52590218966964e-05f) * (float)v;
}
__device__ __forceinline__ int cm_char(float p0, float p25, float p75, float p100, float v) {
  int a;
  if (v < p25) {
    const float f = (v - p0) / (p25 - p0);
    a = (int)((double)(f * 64.0f) + 0.5);
    a = a < 0 ? 0 : (a > 64 ? 64 : a);
  } else if (v < p75) {
    const float f = (v - p25) / (p75 - p25);
    a = 64 + (int)((double)(f * 128.0f) + 0.5);
    a = a < 64 ? 64 : (a > 192 ? 192 : a);
  } else {
    const float f = (v - p75) / (p100 - p75);
    a = 192 + (int)((double)(f * 63.0f) + 0.5);
    a = a < 192 ? 192 : (a > 255 ? 255 : a);
  }
  return a;
}
__device__ __forceinline__ float cm_unchar(float p0, float p25, float p75, float p100, int v) {
  double x;
  if (v <= 64) x = (double)p0 + (double)((p25 - p0) * (float)v) * (1 / 64.0);
  else if (v <= 192) x = (double)p25 + (double)((p75 - p25) * (float)(v - 64)) * (1 / 128.0);
  else x = (double)p75 + (double)((p100 - p75) * (float)(v - 192)) * (1 / 63.0);
  return (float)x;
}

__global__ __launch_bounds__(256) void cm_head_k(const float* __restrict__ in,
                                                 const int64_t* __restrict__ frame_off, int F,
                                                 uint8_t* __restrict__ blob,
                                                 const int64_t* __restrict__ blob_off) {
  const int u = blockIdx.x;
  const int64_t base = frame_off[u];
  const int T = (int)(frame_off[u + 1] - base);
  const float* x = in + base * F;
  float mn = INFINITY, mx = -INFINITY;
  for (long i = threadIdx.x; i < (long)T * F; i += 256) {
    const float v = x[i];
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, o, 64));
    mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  }
  __shared__ float smn[4], smx[4];
  if ((threadIdx.x & 63) == 0) {
    smn[threadIdx.x >> 6] = mn;
    smx[threadIdx.x >> 6] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    mn = fminf(fminf(smn[0], smn[1]), fminf(smn[2], smn[3]));
    mx = fmaxf(fmaxf(smx[0], smx[1]), fmaxf(smx[2], smx[3]));
    if (T == 0) mn = mx = 0.f;
    // ComputeGlobalHeader: a constant matrix gets max = min + (1 + |min|)
    if (mx == mn) mx = (float)((double)mn + (1.0 + fabs((double)mn)));
    const float hdr[2] = {mn, mx - mn};
    const int dims[2] = {T, F};
    uint8_t* b = blob + blob_off[u];
    __builtin_memcpy(b, hdr, 8);
    __builtin_memcpy(b + 8, dims, 8);
  }
}

__global__ __launch_bounds__(256) void cm_col_k(const float* __restrict__ in,
                                                const int64_t* __restrict__ frame_off, int F,
                                                uint8_t* __restrict__ blob,
                                                const int64_t* __restrict__ blob_off,
                                                float* __restrict__ out) {
  const int c = blockIdx.x, u = blockIdx.y, tid = threadIdx.x;
  const int64_t base = frame_off[u];
  const int T = (int)(frame_off[u + 1] - base);
  if (T == 0) return;
  const float* x = in + base * F + c;
  uint8_t* b = blob + blob_off[u];
  float hdr[2];
  __builtin_memcpy(hdr, b, 8);
  const float mn = hdr[0], range = hdr[1];
  if (T <= 8) {   // kTwoByteAuto ("CM2"): uint16 row-major, min + v * (range / 65535)
    const float inc = (float)((double)range * (1.0 / 65535.0));
    for (int t = tid; t < T; t += 256) {
      const int q = cm_u16(mn, range, x[(long)t * F]);
      const uint16_t q16 = (uint16_t)q;
      __builtin_memcpy(b + 16 + 2 * ((long)t * F + c), &q16, 2);
      if (out) out[(base + t) * F + c] = mn + (float)q16 * inc;
    }
    return;
  }
  __shared__ unsigned hist[4][256];
  __shared__ unsigned pref[4];
  __shared__ int want[4];
  __shared__ float pf[4];
  const int qr = T / 4;
  if (tid < 4) {
    pref[tid] = 0;
    want[tid] = tid == 0 ? 0 : tid == 1 ? qr : tid == 2 ? 3 * qr : T - 1;
  }
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    const unsigned hi = pass == 0 ? 0u : (0xFFFFFFFFu << (32 - 8 * pass));
    for (int i = tid; i < 4 * 256; i += 256) (&hist[0][0])[i] = 0;
    __syncthreads();
    for (int t = tid; t < T; t += 256) {
      const unsigned k = cm_key(x[(long)t * F]);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if ((k & hi) == pref[r]) atomicAdd(&hist[r][(k >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid < 4) {
      unsigned cum = 0;
      int d = 0;
      for (; d < 255; ++d) {
        if (cum + hist[tid][d] > (unsigned)want[tid]) break;
        cum += hist[tid][d];
      }
      want[tid] -= (int)cum;
      pref[tid] |= (unsigned)d << shift;
    }
    __syncthreads();
  }
  if (tid == 0) {
    // ComputeColHeader (rows >= 5): strictly increasing uint16 percentiles
    int p[4];
    p[0] = min(cm_u16(mn, range, cm_unkey(pref[0])), 65532);
    p[1] = min(max(cm_u16(mn, range, cm_unkey(pref[1])), p[0] + 1), 65533);
    p[2] = min(max(cm_u16(mn, range, cm_unkey(pref[2])), p[1] + 1), 65534);
    p[3] = max(cm_u16(mn, range, cm_unkey(pref[3])), p[2] + 1);
    uint16_t h16[4];
    for (int r = 0; r < 4; ++r) {
      h16[r] = (uint16_t)p[r];
      pf[r] = cm_f16(mn, range, h16[r]);
    }
    __builtin_memcpy(b + 16 + 8 * c, h16, 8);
  }
  __syncthreads();
  const float p0 = pf[0], p25 = pf[1], p75 = pf[2], p100 = pf[3];
  uint8_t* col = b + 16 + 8 * (long)F + (long)c * T;
  for (int t = tid; t < T; t += 256) {
    const int a = cm_char(p0, p25, p75, p100, x[(long)t * F]);
    col[t] = (uint8_t)a;
    if (out) out[(base + t) * F + c] = cm_unchar(p0, p25, p75, p100, a);
  }
}

namespace {
// MelBanks (mel-computations.cc) in float32, Kaldi's operation order
inline float mel_scale(float f) { return 1127.0f * logf(1.0f + f / 700.0f); }

struct FbankTables {
  int device = -1, nfft = 0, frame_len = 0, num_bins = 0;
  float samp = 0.f, low = 0.f, high = 0.f;
  float *win = nullptr, *mel = nullptr, *tw = nullptr, *utw = nullptr;
  int *lo = nullptr, *n = nullptr;
  void release() {
    for (void* p : {(void*)win, (void*)mel, (void*)tw, (void*)utw, (void*)lo, (void*)n})
      if (p) (void)hipFree(p);
    win = mel = tw = utw = nullptr;
    lo = n = nullptr;
  }
};
std::mutex g_tab_mu;
std::deque<FbankTables> g_tabs;   // one per (device, shape); deque: push_back keeps references valid

template <typename T>
hipError_t upload(T** dst, const std::vector<T>& v) {
  hipError_t e = hipMalloc((void**)dst, v.size() * sizeof(T));
  if (e == hipSuccess) e = hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
  return e;
}

int fbank_geometry(const vox_fbank_opts* o, int* frame_len, int* shift, int* nfft) {
  if (!o || o->sample_frequency <= 0 || o->frame_length_ms <= 0 || o->frame_shift_ms <= 0 ||
      o->num_mel_bins <= 0 || o->num_mel_bins > 256)
    return vox_set_error(VOX_EINVAL, "bad fbank options");
  // FrameExtractionOptions::WindowSize/WindowShift: int(samp_freq * 0.001 * ms)
  *frame_len = (int)(o->sample_frequency * 0.001 * o->frame_length_ms);
  *shift = (int)(o->sample_frequency * 0.001 * o->frame_shift_ms);
  int p = 1;
  while (p < *frame_len) p <<= 1;   // round_to_power_of_two
  *nfft = p;
  if (p != 256 && p != 512)
    return vox_set_error(VOX_EINVAL, "fbank: padded window must be 256 or 512 samples");
  if (*shift <= 0) return vox_set_error(VOX_EINVAL, "fbank: frame shift < 1 sample");
  return VOX_OK;
}

int get_tables(int device, const vox_fbank_opts* o, int frame_len, int nfft, FbankTables** out) {
  std::lock_guard<std::mutex> lk(g_tab_mu);
  for (auto& t : g_tabs)
    if (t.device == device && t.nfft == nfft && t.frame_len == frame_len &&
        t.num_bins == o->num_mel_bins && t.samp == o->sample_frequency && t.low == o->low_freq &&
        t.high == o->high_freq) {
      *out = &t;
      return VOX_OK;
    }
  const int nb = o->num_mel_bins, nfb = nfft / 2;
  // povey window (FeatureWindowFunction, double then float)
  std::vector<float> win(frame_len);
  const double a = 2.0 * M_PI / (frame_len - 1);
  for (int i = 0; i < frame_len; ++i) win[i] = (float)std::pow(0.5 - 0.5 * std::cos(a * i), 0.85);
  // MelBanks
  const float samp = o->sample_frequency;
  const float nyquist = 0.5f * samp;
  const float high = o->high_freq > 0.f ? o->high_freq : nyquist + o->high_freq;
  if (o->low_freq < 0.f || o->low_freq >= nyquist || high <= 0.f || high > nyquist ||
      high <= o->low_freq)
    return vox_set_error(VOX_EINVAL, "fbank: bad low/high frequency");
  const float bin_w = samp / (float)nfft;
  const float mel_lo = mel_scale(o->low_freq), mel_hi = mel_scale(high);
  const float delta = (mel_hi - mel_lo) / (float)(nb + 1);
  std::vector<float> mel((size_t)nb * nfb, 0.f);
  std::vector<int> first(nb, 0), cnt(nb, 0);
  for (int b = 0; b < nb; ++b) {
    const float left = mel_lo + (float)b * delta, center = mel_lo + (float)(b + 1) * delta,
                right = mel_lo + (float)(b + 2) * delta;
    int f0 = -1, f1 = -1;
    for (int i = 0; i < nfb; ++i) {
      const float m = mel_scale(bin_w * (float)i);
      if (m > left && m < right) {
        mel[(size_t)b * nfb + i] = m <= center ? (m - left) / (center - left) : (right - m) / (right - center);
        if (f0 < 0) f0 = i;
        f1 = i;
      }
    }
    if (f0 < 0) return vox_set_error(VOX_EINVAL, "fbank: a mel bin has no FFT bins (too many bins)");
    first[b] = f0;
    cnt[b] = f1 + 1 - f0;
  }
  // FFT twiddles exp(-2 pi i k / (nfft/2)) and unpack twiddles exp(-2 pi i k / nfft)
  std::vector<float> tw(nfft / 2), utw(2 * (nfb + 1));
  for (int k = 0; k < nfft / 4; ++k) {
    tw[2 * k] = (float)std::cos(-2.0 * M_PI * k / nfb);
    tw[2 * k + 1] = (float)std::sin(-2.0 * M_PI * k / nfb);
  }
  for (int k = 0; k <= nfb; ++k) {
    utw[2 * k] = (float)std::cos(-2.0 * M_PI * k / nfft);
    utw[2 * k + 1] = (float)std::sin(-2.0 * M_PI * k / nfft);
  }
  FbankTables t;
  t.device = device; t.nfft = nfft; t.frame_len = frame_len; t.num_bins = nb;
  t.samp = samp; t.low = o->low_freq; t.high = o->high_freq;
  hipError_t e = upload(&t.win, win);
  if (e == hipSuccess) e = upload(&t.mel, mel);
  if (e == hipSuccess) e = upload(&t.lo, first);
  if (e == hipSuccess) e = upload(&t.n, cnt);
  if (e == hipSuccess) e = upload(&t.tw, tw);
  if (e == hipSuccess) e = upload(&t.utw, utw);
  if (e != hipSuccess) {
    t.release();
    return vox_set_error(VOX_EHIP, (std::string("fbank tables: ") + hipGetErrorString(e)).c_str());
  }
  g_tabs.push_back(t);
  *out = &g_tabs.back();
  return VOX_OK;
}
}  // namespace

}  // namespace vox

using namespace vox;

extern "C" void vox_fbank_default_opts(vox_fbank_opts* o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->sample_frequency = 16000.f;
  o->frame_length_ms = 25.f;
  o->frame_shift_ms = 10.f;
  o->dither = 1.f;
  o->preemphasis_coefficient = 0.97f;
  o->remove_dc_offset = 1;
  o->num_mel_bins = 23;
  o->low_freq = 20.f;
  o->high_freq = 0.f;
  o->seed = 0;
}

extern "C" int64_t vox_fbank_num_frames(int64_t num_samples, const vox_fbank_opts* o) {
  int L, S, nfft;
  int rc = fbank_geometry(o, &L, &S, &nfft);
  if (rc) return rc;
  if (num_samples < L) return 0;   // snip_edges
  return 1 + (num_samples - L) / S;
}

extern "C" int vox_fbank_device_keyed(const float* d_wav, const int64_t* d_samp_off,
                                      const int64_t* d_frame_off, const uint64_t* d_utt_key,
                                      int n_utt, int64_t total_frames, const vox_fbank_opts* o,
                                      float* d_out, void* stream) {
  if (!d_wav || !d_samp_off || !d_frame_off || !d_out || n_utt <= 0 || total_frames < 0)
    return vox_set_error(VOX_EINVAL, "bad fbank arguments");
  int L, S, nfft;
  int rc = fbank_geometry(o, &L, &S, &nfft);
  if (rc) return rc;
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, d_wav) != hipSuccess || at.type != hipMemoryTypeDevice)
    return vox_set_error(VOX_EINVAL, "fbank: waveform must be device memory");
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(at.device) != hipSuccess)
    return vox_set_error(VOX_EHIP, "fbank: cannot select the waveform's device");
  FbankTables* t = nullptr;
  rc = get_tables(at.device, o, L, nfft, &t);
  if (rc == VOX_OK && total_frames > 0) {
    FbankDev d;
    d.frame_len = L; d.frame_shift = S; d.num_bins = o->num_mel_bins;
    d.remove_dc = o->remove_dc_offset; d.preemph = o->preemphasis_coefficient;
    d.dither = o->dither; d.seed = o->seed;
    d.win = t->win; d.mel = t->mel; d.mel_lo = t->lo; d.mel_n = t->n; d.tw = t->tw; d.utw = t->utw;
    hipStream_t s = (hipStream_t)stream;
    if (nfft == 512)
      hipLaunchKernelGGL(fbank_k<512>, dim3((unsigned)total_frames), dim3(64), 0, s, d_wav,
                         d_samp_off, d_frame_off, d_utt_key, n_utt, d, d_out);
    else
      hipLaunchKernelGGL(fbank_k<256>, dim3((unsigned)total_frames), dim3(64), 0, s, d_wav,
                         d_samp_off, d_frame_off, d_utt_key, n_utt, d, d_out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) rc = vox_set_error(VOX_EHIP, (std::string("fbank_k: ") + hipGetErrorString(e)).c_str());
  }
  (void)hipSetDevice(prev);
  return rc;
}

extern "C" int vox_fbank_device(const float* d_wav, const int64_t* d_samp_off,
                                const int64_t* d_frame_off, int n_utt, int64_t total_frames,
                                const vox_fbank_opts* o, float* d_out, void* stream) {
  return vox_fbank_device_keyed(d_wav, d_samp_off, d_frame_off, nullptr, n_utt, total_frames, o,
                                d_out, stream);
}

extern "C" int vox_sliding_cmn_device(const float* d_in, const int64_t* d_frame_off, int n_utt,
                                      int f, int cmn_window, int center, float* d_out,
                                      void* stream) {
  if (!d_in || !d_frame_off || !d_out || n_utt <= 0 || f <= 0 || cmn_window <= 0)
    return vox_set_error(VOX_EINVAL, "bad cmn arguments");
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, d_in) != hipSuccess || at.type != hipMemoryTypeDevice)
    return vox_set_error(VOX_EINVAL, "cmn: features must be device memory");
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(at.device) != hipSuccess)
    return vox_set_error(VOX_EHIP, "cmn: cannot select the features' device");
  const long threads = (long)n_utt * f;
  if (center)
    hipLaunchKernelGGL(cmn_fast_k, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, d_in, d_frame_off, n_utt, f, cmn_window, d_out);
  else
    hipLaunchKernelGGL(cmn_k, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, d_in, d_frame_off, n_utt, f, cmn_window, center, d_out);
  hipError_t e = hipGetLastError();
  (void)hipSetDevice(prev);
  if (e != hipSuccess) return vox_set_error(VOX_EHIP, (std::string("cmn_k: ") + hipGetErrorString(e)).c_str());
  return VOX_OK;
}

// ---- device side of the extraction reader: CM payloads -> decoded rows ->
// sliding CMN -> the padded chunk batch (tf_extract.py:63, the values
// apply-cmvn-sliding computes from `copy-feats --compress` arks; the host
// reader's arithmetic, kaldi_host.cpp parse_payload with cm_kaldi = 1).
// meta (int64): blob_off[U+1] | frame_off[U+1] | rows[U] | item_utt[n] | item_start[n] | item_len[n]
// Utterance u: its payload at blob + blob_off[u] (rows[u] rows, column-major
// bytes), rows [0, frame_off[u+1] - frame_off[u]) of it decoded.

// rows [64 blockIdx.x, +64) of utterance blockIdx.y: the column percentiles to
// LDS, the bytes read column-major (coalesced per column), the floats written
// row-major through an LDS tile
constexpr int CMD_R = 64;
__global__ __launch_bounds__(256) void cm_rows_k(const uint8_t* __restrict__ blob,
                                                 const int64_t* __restrict__ meta, int U, int F,
                                                 float* __restrict__ out) {
  const int u = blockIdx.y, tid = threadIdx.x;
  const int64_t* blob_off = meta;
  const int64_t* frame_off = meta + U + 1;
  const int64_t* rows = meta + 2 * (U + 1);
  const int64_t base = frame_off[u];
  const int need = (int)(frame_off[u + 1] - base);
  const int r0 = blockIdx.x * CMD_R;
  if (r0 >= need) return;
  const int T = (int)rows[u];
  const uint8_t* b = blob + blob_off[u];
  extern __shared__ float cm_lds[];
  float* pc = cm_lds;                 // [F][4] column percentiles
  float* tile = cm_lds + 4 * F;       // [CMD_R][F + 1]
  float hdr[2];
  __builtin_memcpy(hdr, b, 8);
  for (int i = tid; i < 4 * F; i += 256) {
    uint16_t v;
    __builtin_memcpy(&v, b + 16 + 2 * i, 2);
    pc[i] = cm_f16(hdr[0], hdr[1], v);
  }
  __syncthreads();
  const int nr = min(CMD_R, need - r0);
  const uint8_t* data = b + 16 + 8 * F;
  for (int i = tid; i < F * CMD_R; i += 256) {
    const int c = i / CMD_R, r = i - c * CMD_R;
    if (r < nr) {
      const int v = data[(int64_t)c * T + r0 + r];
      tile[r * (F + 1) + c] = cm_unchar(pc[4 * c], pc[4 * c + 1], pc[4 * c + 2], pc[4 * c + 3], v);
    }
  }
  __syncthreads();
  for (int i = tid; i < F * nr; i += 256) {
    const int r = i / F, c = i - r * F;
    out[(base + r0 + r) * F + c] = tile[r * (F + 1) + c];
  }
}

// item i's rows [start, start + len) of its utterance into rows [i stride, + len)
// of the batch, zero up to the stride
__global__ __launch_bounds__(256) void chunk_gather_k(const float* __restrict__ feats,
                                                      const int64_t* __restrict__ meta, int U, int n,
                                                      int stride, int F, float* __restrict__ out) {
  const int64_t* frame_off = meta + U + 1;
  const int64_t* it = meta + 3 * U + 2;   // item_utt | item_start | item_len
  const int64_t total = (int64_t)n * stride * F;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t row = e / F;
    const int c = (int)(e - row * F);
    const int i = (int)(row / stride), t = (int)(row - (int64_t)i * stride);
    const int u = (int)it[i];
    out[e] = t < it[2 * n + i] ? feats[(frame_off[u] + it[n + i] + t) * F + c] : 0.f;
  }
}

extern "C" int64_t vox_cm_blob_bytes(int rows, int cols) {
  if (rows < 0 || cols <= 0) return vox_set_error(VOX_EINVAL, "cm: bad matrix shape");
  if (rows > 8) return 16 + 8 * (int64_t)cols + (int64_t)rows * cols;
  return 16 + 2 * (int64_t)rows * cols;
}

extern "C" int vox_cm_compress_device(const float* d_in, const int64_t* d_frame_off, int n_utt,
                                      int f, uint8_t* d_blob, const int64_t* d_blob_off,
                                      float* d_out, void* stream) {
  if (!d_in || !d_frame_off || !d_blob || !d_blob_off || n_utt <= 0 || f <= 0 || n_utt > 65535)
    return vox_set_error(VOX_EINVAL, "bad cm arguments");
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, d_in) != hipSuccess || at.type != hipMemoryTypeDevice)
    return vox_set_error(VOX_EINVAL, "cm: features must be device memory");
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(at.device) != hipSuccess)
    return vox_set_error(VOX_EHIP, "cm: cannot select the features' device");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(cm_head_k, dim3(n_utt), dim3(256), 0, s, d_in, d_frame_off, f, d_blob,
                     d_blob_off);
  hipLaunchKernelGGL(cm_col_k, dim3(f, n_utt), dim3(256), 0, s, d_in, d_frame_off, f, d_blob,
                     d_blob_off, d_out);
  hipError_t e = hipGetLastError();
  (void)hipSetDevice(prev);
  if (e != hipSuccess)
    return vox_set_error(VOX_EHIP, (std::string("cm kernels: ") + hipGetErrorString(e)).c_str());
  return VOX_OK;
}

extern "C" int vox_cm_chunks_device(const uint8_t* d_blob, const int64_t* d_meta, int n_utt,
                                    int64_t total_rows, int max_need, int n_items, int stride,
                                    int f, int cmn_window, float* d_work, float* d_out,
                                    void* stream) {
  if (!d_blob || !d_meta || !d_work || !d_out || n_utt <= 0 || n_utt > 65535 || total_rows <= 0 ||
      max_need <= 0 || n_items <= 0 || stride <= 0 || f <= 0 || f > 2048 || cmn_window < 0)
    return vox_set_error(VOX_EINVAL, "bad cm chunk arguments");
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, d_out) != hipSuccess || at.type != hipMemoryTypeDevice)
    return vox_set_error(VOX_EINVAL, "cm chunks: the batch must be device memory");
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(at.device) != hipSuccess)
    return vox_set_error(VOX_EHIP, "cm chunks: cannot select the batch's device");
  hipStream_t s = (hipStream_t)stream;
  const size_t lds = (size_t)(4 * f + CMD_R * (f + 1)) * 4;
  hipLaunchKernelGGL(cm_rows_k, dim3((unsigned)((max_need + CMD_R - 1) / CMD_R), (unsigned)n_utt),
                     dim3(256), lds, s, d_blob, d_meta, n_utt, f, d_work);
  const float* feats = d_work;
  if (cmn_window > 0) {
    float* cm = d_work + (size_t)total_rows * f;   // the CMN'd rows follow the decoded ones
    const long threads = (long)n_utt * f;
    hipLaunchKernelGGL(cmn_fast_k, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, d_work,
                       d_meta + n_utt + 1, n_utt, f, cmn_window, cm);
    feats = cm;
  }
  const int64_t total = (int64_t)n_items * stride * f;
  const unsigned g = (unsigned)std::min<int64_t>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(chunk_gather_k, dim3(g), dim3(256), 0, s, feats, d_meta, n_utt, n_items,
                     stride, f, d_out);
  hipError_t e = hipGetLastError();
  (void)hipSetDevice(prev);
  if (e != hipSuccess)
    return vox_set_error(VOX_EHIP, (std::string("cm chunk kernels: ") + hipGetErrorString(e)).c_str());
  return VOX_OK;
}

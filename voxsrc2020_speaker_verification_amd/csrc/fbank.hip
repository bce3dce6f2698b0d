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

#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <mutex>
#include <string>
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
                                              const int64_t* __restrict__ frame_off, int n_utt,
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
        x += d.dither * gauss(d.seed ^ mix64(((unsigned long long)t << 16) ^ (unsigned)i));
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
std::vector<FbankTables> g_tabs;   // one per (device, shape)

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

extern "C" int vox_fbank_device(const float* d_wav, const int64_t* d_samp_off,
                                const int64_t* d_frame_off, int n_utt, int64_t total_frames,
                                const vox_fbank_opts* o, float* d_out, void* stream) {
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
                         d_samp_off, d_frame_off, n_utt, d, d_out);
    else
      hipLaunchKernelGGL(fbank_k<256>, dim3((unsigned)total_frames), dim3(64), 0, s, d_wav,
                         d_samp_off, d_frame_off, n_utt, d, d_out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) rc = vox_set_error(VOX_EHIP, (std::string("fbank_k: ") + hipGetErrorString(e)).c_str());
  }
  (void)hipSetDevice(prev);
  return rc;
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
  hipLaunchKernelGGL(cmn_k, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, d_in, d_frame_off, n_utt, f, cmn_window, center, d_out);
  hipError_t e = hipGetLastError();
  (void)hipSetDevice(prev);
  if (e != hipSuccess) return vox_set_error(VOX_EHIP, (std::string("cmn_k: ") + hipGetErrorString(e)).c_str());
  return VOX_OK;
}

// Adaptive score normalisation statistics on the GPU (snorm.py:83-109,
// get_cohort_mean_std): for every trial embedding, cosine scores against the
// cohort speaker means (fp32 GEMM on the MFMA conv path), then the mean and
// population std of its top-k scores.
//
// The reference sorts every full score row (np.sort of ~6k values per trial).
// Here one workgroup per row finds the k-th largest score by an exact 4-pass
// 8-bit radix select on order-preserving float keys; the top-k multiset is
// then {x > T} plus (k - #{x > T}) copies of T, identical to the sorted
// prefix including ties.  Mean and std are two-pass, accumulated in double.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>

#include "../../include/voxemb.h"
#include "kernels.h"

namespace vox {

__device__ __forceinline__ uint32_t f2key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

template <int NT>
__global__ __launch_bounds__(NT) void topk_stats_k(const float* __restrict__ s, int m, int lds_row,
                                                   int k, float* __restrict__ mean_out,
                                                   float* __restrict__ std_out, int row0) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem);        // 256 bins
  double* red = reinterpret_cast<double*>(smem + 256 * 4);   // NT/64 partials
  __shared__ uint32_t sel_digit, sel_above;
  const int tid = threadIdx.x;
  const float* row = s + (size_t)blockIdx.x * lds_row;
  uint32_t prefix = 0, pmask = 0;
  int kr = k;   // rank still to place inside the current prefix bucket
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    for (int i = tid; i < 256; i += NT) hist[i] = 0;
    __syncthreads();
    for (int i = tid; i < m; i += NT) {
      const uint32_t key = f2key(row[i]);
      if ((key & pmask) == prefix) atomicAdd(&hist[(key >> shift) & 255], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t above = 0;
      int d = 255;
      for (; d > 0; --d) {
        if (above + hist[d] >= (uint32_t)kr) break;
        above += hist[d];
      }
      sel_digit = d;
      sel_above = above;
    }
    __syncthreads();
    prefix |= sel_digit << shift;
    pmask |= 255u << shift;
    kr -= (int)sel_above;
    __syncthreads();
  }
  // threshold key = prefix; kr copies of it belong to the top-k
  const uint32_t tkey = prefix;
  const uint32_t tbits = (tkey & 0x80000000u) ? (tkey & 0x7fffffffu) : ~tkey;
  const float tval = __uint_as_float(tbits);
  auto block_sum = [&](double v) -> double {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    if ((tid & 63) == 0) red[tid >> 6] = v;
    __syncthreads();
    double t = 0;
    if (tid == 0)
      for (int w = 0; w < NT / 64; ++w) t += red[w];
    __syncthreads();
    return t;   // valid on thread 0
  };
  double acc = 0;
  for (int i = tid; i < m; i += NT) {
    const float x = row[i];
    if (f2key(x) > tkey) acc += x;
  }
  const double sum = block_sum(acc) + (tid == 0 ? (double)kr * tval : 0.0);
  __shared__ double mu_s;
  if (tid == 0) mu_s = sum / k;
  __syncthreads();
  const double mu = mu_s;
  acc = 0;
  for (int i = tid; i < m; i += NT) {
    const float x = row[i];
    if (f2key(x) > tkey) acc += (x - mu) * (x - mu);
  }
  const double ss = block_sum(acc);
  if (tid == 0) {
    const double var = (ss + (double)kr * (tval - mu) * (tval - mu)) / k;
    mean_out[row0 + blockIdx.x] = (float)mu;
    std_out[row0 + blockIdx.x] = (float)std::sqrt(var);
  }
}

}  // namespace vox

using namespace vox;

int vox_set_error(int code, const char* msg);

#define AS_HIPCHK(x)                                                               \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      rc = vox_set_error(VOX_EHIP, (std::string(#x) + ": " + hipGetErrorString(e_)).c_str()); \
      goto done;                                                                   \
    }                                                                              \
  } while (0)

extern "C" int vox_asnorm_stats(const float* d_trial, int n, const float* d_cohort, int m, int d,
                                int topk, float* d_mean, float* d_std, void* stream) {
  if (!d_trial || !d_cohort || !d_mean || !d_std || n <= 0 || m <= 0 || d <= 0 || topk <= 0)
    return vox_set_error(VOX_EINVAL, "bad asnorm arguments");
  if (d % 4) return vox_set_error(VOX_EINVAL, "embedding dim must be a multiple of 4");
  hipStream_t s = (hipStream_t)stream;
  // the buffers and kernels go to the device that holds the trial matrix (the
  // caller's stream belongs to it), not to this thread's current device
  int dev = -1, prev = -1;
  {
    hipPointerAttribute_t at, ac;
    if (hipPointerGetAttributes(&at, d_trial) != hipSuccess ||
        hipPointerGetAttributes(&ac, d_cohort) != hipSuccess || at.type != hipMemoryTypeDevice ||
        ac.type != hipMemoryTypeDevice)
      return vox_set_error(VOX_EINVAL, "asnorm operands must be device memory");
    if (at.device != ac.device)
      return vox_set_error(VOX_EINVAL, "asnorm trial and cohort matrices on different devices");
    dev = at.device;
  }
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(dev) != hipSuccess)
    return vox_set_error(VOX_EHIP, "asnorm: cannot select the operands' device");
  const int k = topk < m ? topk : m;
  // cohort as fp32 1x1-conv weights [coutp][kp] (zero-padded rows / columns)
  const int KS = conv_kstep(F32);
  const int kp = (d + KS - 1) / KS * KS;
  const int tiles = (m + 15) / 16;
  const int wco = tiles <= 4 ? tiles : (tiles <= 6 ? 6 : 8);
  const int coutp = (m + 16 * wco - 1) / (16 * wco) * (16 * wco);
  const int R = 4096;   // trial rows per GEMM + select pass
  const int ldrow = (m + 3) / 4 * 4;
  float* wbuf = nullptr;
  float* sbuf = nullptr;
  int rc = VOX_OK;
  AS_HIPCHK(hipMalloc(&wbuf, (size_t)coutp * kp * 4));
  AS_HIPCHK(hipMalloc(&sbuf, (size_t)R * ldrow * 4));
  AS_HIPCHK(hipMemsetAsync(wbuf, 0, (size_t)coutp * kp * 4, s));
  AS_HIPCHK(hipMemcpy2DAsync(wbuf, (size_t)kp * 4, d_cohort, (size_t)d * 4, (size_t)d * 4, m,
                             hipMemcpyDeviceToDevice, s));
  for (int r0 = 0; r0 < n; r0 += R) {
    const int rows = n - r0 < R ? n - r0 : R;
    ConvParams p;
    std::memset(&p, 0, sizeof(p));
    p.x = d_trial + (size_t)r0 * d; p.ldx = d;
    p.w = wbuf; p.kp = kp;
    p.y = sbuf; p.ldy = ldrow; p.ysplit = 1 << 30;
    p.N = rows; p.H = 1; p.W = 1; p.Cin = d; p.Ho = 1; p.Wo = 1; p.Cout = m; p.coutp = coutp;
    p.kh = 1; p.kw = 1; p.sh = p.sw = p.dh = p.dw = 1;
    p.cinp = kp; p.flags = 0; p.groups = 1; p.cblocks = coutp / (16 * wco);
    p.fast4 = (m % 4 == 0) ? 1 : 0;
    ConvLaunch l;
    l.wco = wco; l.wpx = rows >= 64 * 2 * 256 ? 2 : 1; l.vec = 1; l.splitk = 1;
    AS_HIPCHK(launch_conv(F32, p, l, s));
    constexpr int NT = 256;
    hipLaunchKernelGGL(topk_stats_k<NT>, dim3(rows), dim3(NT), 256 * 4 + (NT / 64) * 8, s, sbuf,
                       m, ldrow, k, d_mean, d_std, r0);
    AS_HIPCHK(hipGetLastError());
  }
  AS_HIPCHK(hipStreamSynchronize(s));
done:
  if (wbuf) (void)hipFree(wbuf);
  if (sbuf) (void)hipFree(sbuf);
  (void)hipSetDevice(prev);
  return rc;
}

// Stats-pool variants at the headline shape (layer-4 map of res2net50_w24_s4_c32,
// 80x200, B = 256: N = 256 utterances, H = 25 frames, W = 10, C = 1024 bf16):
// mean and std over H per (n, w, c), fp32 out [N][W][2C] (models.py:262-269).
// The product kernel is stats_pool_col<25, 4> (csrc/kernels.hip): one thread per
// VN-channel column, all H rows in registers, sequential sum over h.  Every
// variant here keeps that per-element summation order, so all outputs must be
// bitwise equal; only the channels per thread (VN) and the load flavour change:
//   v4   VN = 4, 8-B loads (the product kernel's mapping)
//   v2   VN = 2, 4-B loads (2.5 grid rounds of 8 waves per SIMD instead of 1.25)
//   v1   VN = 1, 2-B loads (5 rounds)
//   v4nt VN = 4 with non-temporal loads (streamed once)
//   v4o8 VN = 4 with the registers capped for 8 waves per SIMD (v4 takes 68: 7)
// usage: pool_variants [reps]  -- prints avg us per launch and the TB/s of the
// algorithmic bytes (input + output) per variant, and checks bitwise equality.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

template <int VN> struct Raw;
template <> struct Raw<1> { typedef unsigned short t; };
template <> struct Raw<2> { typedef unsigned t; };
template <> struct Raw<4> { typedef unsigned t __attribute__((ext_vector_type(2))); };

template <int HM, int VN, bool NT>
__device__ __forceinline__ void pool_body(const __bf16* __restrict__ x, int N, int H, int W,
                                                int C, float* __restrict__ out) {
  typedef __bf16 bfv __attribute__((ext_vector_type(VN)));
  typedef typename Raw<VN>::t uv;
  // (body shared by the occupancy variants below)
  const int chunks = C / VN;
  const int64_t gcol = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gcol >= (int64_t)N * W * chunks) return;
  const int n = (int)(gcol / ((int64_t)W * chunks));
  const int r = (int)(gcol - (int64_t)n * W * chunks);
  const int w = r / chunks, ch = r - (r / chunks) * chunks;
  const __bf16* base = x + ((size_t)n * H * W + w) * C + (size_t)ch * VN;
  const size_t rowstride = (size_t)W * C;
  uv v[HM];
#pragma unroll
  for (int h = 0; h < HM; ++h)
    if (h < H) {
      const uv* p = reinterpret_cast<const uv*>(base + (size_t)h * rowstride);
      v[h] = NT ? __builtin_nontemporal_load(p) : *p;
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
#pragma unroll
  for (int h = 0; h < HM; ++h) asm volatile("" : "+v"(v[h]));
#pragma unroll
  for (int h = 0; h < HM; ++h)
    if (h < H) {
      const bfv b = __builtin_bit_cast(bfv, v[h]);
#pragma unroll
      for (int e = 0; e < VN; ++e) {
        const float d = (float)b[e] - mu[e];
        q[e] += d * d;
      }
    }
  float* o = out + (size_t)n * W * 2 * C + (size_t)w * 2 * C + (size_t)ch * VN;
#pragma unroll
  for (int e = 0; e < VN; ++e) {
    o[e] = mu[e];
    o[C + e] = sqrtf(q[e] / (float)H + 1e-5f);
  }
}

template <int HM, int VN, bool NT>
__global__ __launch_bounds__(256) void pool_col(const __bf16* __restrict__ x, int N, int H, int W,
                                                int C, float* __restrict__ out) {
  pool_body<HM, VN, NT>(x, N, H, W, C, out);
}
// the same with the register budget capped at 8 waves per SIMD (<= 64 VGPRs)
template <int HM, int VN, bool NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8)))
void pool_col8(const __bf16* __restrict__ x, int N, int H, int W, int C, float* __restrict__ out) {
  pool_body<HM, VN, NT>(x, N, H, W, C, out);
}

typedef void (*Launch)(const __bf16*, int, int, int, int, float*);
template <int VN, bool NT, bool O8 = false>
static void launch(const __bf16* x, int N, int H, int W, int C, float* out) {
  const int64_t threads = (int64_t)N * W * (C / VN);
  if (O8)
    hipLaunchKernelGGL((pool_col8<25, VN, NT>), dim3((unsigned)((threads + 255) / 256)), dim3(256),
                       0, 0, x, N, H, W, C, out);
  else
    hipLaunchKernelGGL((pool_col<25, VN, NT>), dim3((unsigned)((threads + 255) / 256)), dim3(256),
                       0, 0, x, N, H, W, C, out);
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 50;
  const int N = 256, H = 25, W = 10, C = 1024;
  const size_t nin = (size_t)N * H * W * C, nout = (size_t)N * W * 2 * C;
  std::vector<uint16_t> hx(nin);
  uint32_t st = 12345;
  for (size_t i = 0; i < nin; ++i) {
    st = st * 1664525u + 1013904223u;
    // post-ReLU-like bf16 values in [0, 4): sign 0, exponent 126..128
    hx[i] = (uint16_t)(0x3F00 + ((st >> 9) % 0x180));
  }
  __bf16* dx;
  float* dout[5];
  CK(hipMalloc(&dx, nin * 2));
  CK(hipMemcpy(dx, hx.data(), nin * 2, hipMemcpyHostToDevice));
  for (auto& d : dout) CK(hipMalloc(&d, nout * 4));
  // a buffer larger than L2 + MALL, rewritten between timed launches so every
  // launch reads its input from HBM as in the forward (the input map is
  // written by the previous layer and partly cache-resident there; this is the
  // colder case)
  const size_t flush_bytes = 1ull << 30;
  void* flush;
  CK(hipMalloc(&flush, flush_bytes));
  const char* names[5] = {"v4", "v2", "v1", "v4nt", "v4o8"};
  Launch fns[5] = {launch<4, false>, launch<2, false>, launch<1, false>, launch<4, true>,
                   launch<4, false, true>};
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double bytes = nin * 2.0 + nout * 4.0;
  for (int pass = 0; pass < 2; ++pass)   // pass 0: cold input (flushed), 1: warm
  for (int v = 0; v < 5; ++v) {
    fns[v](dx, N, H, W, C, dout[v]);
    CK(hipDeviceSynchronize());
    double tot = 0, best = 1e30;
    for (int r = 0; r < reps; ++r) {
      if (pass == 0) CK(hipMemsetAsync(flush, r & 0xFF, flush_bytes, 0));
      CK(hipEventRecord(a, 0));
      fns[v](dx, N, H, W, C, dout[v]);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      tot += ms;
      best = ms < best ? ms : best;
    }
    const double us = 1e3 * tot / reps;
    printf("%s %-5s avg %.2f us  best %.2f us  %.2f TB/s (algorithmic %.1f MB)\n", pass ? "warm" : "cold", names[v], us,
           1e3 * best, bytes / (us * 1e-6) / 1e12, bytes / 1e6);
  }
  std::vector<float> r0(nout), r1(nout);
  CK(hipMemcpy(r0.data(), dout[0], nout * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int v = 1; v < 5; ++v) {
    CK(hipMemcpy(r1.data(), dout[v], nout * 4, hipMemcpyDeviceToHost));
    const bool eq = memcmp(r0.data(), r1.data(), nout * 4) == 0;
    printf("%s bitwise == v4: %s\n", names[v], eq ? "yes" : "NO");
    bad += !eq;
  }
  return bad ? 2 : 0;
}

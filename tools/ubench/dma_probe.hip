// Microbenchmark: LDS-DMA (global_load_lds_dwordx4) ring throughput/latency per CU
// on gfx950, the fill pattern of gemm1x1_wide / conv3x3_pipe with no compute.
// Each workgroup (8 waves) runs S steps: wait until the step issued D-1 steps
// ago landed (vmcnt), barrier, issue P 1-KB pieces per wave into ring slot s%D+...
// Sources: a buffer of `span` bytes walked linearly per workgroup (span >> L2:
// HBM stream; small span: L2/MALL hits).  Reports ns per step -> GB/s per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ void glds16(const void* src, uint32_t lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
}
#define W_(n) case n: asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory"); break;
__device__ __forceinline__ void wait_vm(int n) {
  switch (n) { W_(0) W_(1) W_(2) W_(3) W_(4) W_(5) W_(6) W_(7) W_(8) W_(9) W_(10) W_(11) W_(12)
    W_(13) W_(14) W_(15) W_(16) W_(17) W_(18) W_(19) W_(20) W_(21) W_(22) W_(23) W_(24) W_(28) W_(32)
    W_(36) W_(40) W_(48) W_(56) default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512) void probe(const char* buf, size_t span, int S, int D, int P, int nwaves_issue,
                                             int nmfma, float* sink, int mfma_wave_lo, int stagger) {
  extern __shared__ char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  const bool iss = wave < nwaves_issue;
  const size_t slot_bytes = (size_t)nwaves_issue * P * 1024;
  const size_t mask = span - 1;   // span is a power of two
  const char* base = buf;
  size_t off = ((size_t)blockIdx.x * 7919 * 1024) & mask;
  auto issue = [&](int s) {
    if (!iss) return;
    const uint32_t l = lds0 + (uint32_t)((s % D) * slot_bytes + wave * P * 1024);
    for (int i = 0; i < P; ++i) {
      const char* src = base + ((off + (size_t)(wave * P + i) * 1024 + lane * 16) & mask);
      glds16(src, l + i * 1024);
    }
    off = (off + slot_bytes) & mask;
  };
  for (int s = 0; s < D - 1; ++s) issue(s);
  bf16x8 a = {}, b = {};
  for (int e = 0; e < 8; ++e) { a[e] = (__bf16)(lane * 0.01f + e); b[e] = (__bf16)(wave * 0.1f - e); }
  f32x4 acc[8] = {};
  for (int s = 0; s < S; ++s) {
    if (iss) wait_vm((D - 2) * P);
    __builtin_amdgcn_s_barrier();
    const bool late = stagger && wave >= 4;   // waves 4-7: MFMAs first, then their DMA
    if (!late) issue(s + D - 1);
    // nmfma independent 16x16x32 MFMAs per wave (8 accumulators round robin)
    for (int m = 0; m < (wave >= mfma_wave_lo ? nmfma : 0); m += 8) {
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[k], 0, 0, 0);
    }
    if (late) issue(s + D - 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float t = 0.f;
  for (int k = 0; k < 8; ++k) t += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
  if (t == 12345.f) sink[threadIdx.x] = t;   // keep the MFMAs alive
}

int main(int argc, char** argv) {
  size_t big = (size_t)4 << 30;
  char* buf;
  hipMalloc(&buf, big);
  hipMemset(buf, 1, big);
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  printf("{\"cus\": %d, \"runs\": [\n", ncu);
  bool first = true;
  float* sink;
  hipMalloc(&sink, 4096);
  struct Cfg { int nw, P, nm, lo, st; const char* name; };
  const Cfg cfgs[] = {
      {8, 4, 32, 0, 0, "all8: dma4+mfma32"}, {8, 4, 32, 0, 1, "all8 staggered: dma4+mfma32"},
      {8, 4, 0, 0, 0, "all8: dma4 only"}, {8, 0, 32, 0, 0, "all8: mfma32 only"},
      {4, 8, 64, 4, 0, "split: w0-3 dma8, w4-7 mfma64"},
      {8, 2, 32, 0, 0, "all8: dma2+mfma32"}, {8, 2, 32, 0, 1, "all8 staggered: dma2+mfma32"},
      {8, 4, 64, 0, 0, "all8: dma4+mfma64"}, {8, 4, 64, 0, 1, "all8 staggered: dma4+mfma64"}};
  for (size_t span : {(size_t)4 << 30, (size_t)64 << 20, (size_t)2 << 20}) {
    for (const Cfg& c : cfgs) {
      const int D = 4;
      const size_t lds = (size_t)D * (c.nw ? c.nw : 1) * (c.P ? c.P : 1) * 1024;
      const int S = 400;
      hipLaunchKernelGGL(probe, dim3(ncu), dim3(512), lds, 0, buf, span, 50, D, c.P, c.P ? c.nw : 0, c.nm, sink, c.lo, c.st);
      hipEventRecord(e0);
      hipLaunchKernelGGL(probe, dim3(ncu), dim3(512), lds, 0, buf, span, S, D, c.P, c.P ? c.nw : 0, c.nm, sink, c.lo, c.st);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      printf("%s{\"span_mb\": %zu, \"cfg\": \"%s\", \"ns_step\": %.1f}", first ? "" : ",\n", span >> 20, c.name, ms * 1e6 / S);
      first = false;
    }
  }
  printf("\n]}\n");
  return 0;
}

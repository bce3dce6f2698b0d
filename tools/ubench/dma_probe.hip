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

__global__ __launch_bounds__(512) void probe(const char* buf, size_t span, int S, int D, int P, int nwaves_issue) {
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
  for (int s = 0; s < S; ++s) {
    if (iss) wait_vm((D - 2) * P);
    __builtin_amdgcn_s_barrier();
    issue(s + D - 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
  for (size_t span : {(size_t)4 << 30, (size_t)64 << 20, (size_t)2 << 20}) {
    for (int nw : {8, 4}) {
      for (int P : {1, 2, 4, 8}) {
        for (int D : {2, 3, 4}) {
          const size_t lds = (size_t)D * nw * P * 1024;
          if (lds > 160 * 1024 || (D - 2) * P > 56) continue;
          const int S = 400;
          hipLaunchKernelGGL(probe, dim3(ncu), dim3(512), lds, 0, buf, span, 50, D, P, nw);
          hipEventRecord(e0);
          hipLaunchKernelGGL(probe, dim3(ncu), dim3(512), lds, 0, buf, span, S, D, P, nw);
          hipEventRecord(e1);
          hipEventSynchronize(e1);
          float ms;
          hipEventElapsedTime(&ms, e0, e1);
          const double per_step_ns = ms * 1e6 / S;
          const double gbs_cu = (double)nw * P * 1024 / per_step_ns;
          printf("%s{\"span_mb\": %zu, \"waves\": %d, \"P\": %d, \"D\": %d, \"inflight_kb\": %d, \"ns_step\": %.1f, \"gbs_cu\": %.1f, \"tbs_chip\": %.2f}",
                 first ? "" : ",\n", span >> 20, nw, P, D, (D - 1) * nw * P, per_step_ns, gbs_cu, gbs_cu * ncu / 1000);
          first = false;
        }
      }
    }
  }
  printf("\n]}\n");
  return 0;
}

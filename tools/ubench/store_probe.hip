// Microbenchmark: global_store_dwordx4 throughput per CU by the shape one wave
// instruction covers: rows x bytes-per-row (the 1x1 GEMM epilogue writes 16
// pixel rows x 64 B per instruction; full 128-B lines would be 8 x 128 B).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int SEG>   // bytes per row segment covered by consecutive lanes (64, 128, 256, 1024)
__global__ __launch_bounds__(512) void stores(char* out, size_t row_bytes, int tiles, int nstore) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int LPR = SEG / 16;            // lanes per row segment
  const int r = lane / LPR, c = lane % LPR;
  u32x4 v = {(unsigned)lane, 1u, 2u, 3u};
  for (int t = 0; t < tiles; ++t) {
    const size_t tile = (size_t)t * gridDim.x + blockIdx.x;
    // a tile = 256 rows x 256 B (a 256-pixel x 128-channel bf16 output block)
    char* base = out + tile * 256 * row_bytes;
    for (int i = 0; i < nstore; ++i) {
      const int q = wave * nstore + i;             // instruction index within the tile
      // instruction q covers rows [q*(64/LPR) ...) of the tile, segment (q % (256/SEG))
      const int rows_per = 64 / LPR;
      const int seg_per_row = 256 / SEG;
      const int row = (q / seg_per_row) * rows_per + r;
      const int col = (q % seg_per_row) * SEG + c * 16;
      asm volatile("global_store_dwordx4 %0, %1, off" : : "v"(base + row * row_bytes + col), "v"(v) : "memory");
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const size_t row_bytes = 1024;           // a 512-channel bf16 output row
  const int tiles = 64;
  const size_t bytes = (size_t)tiles * ncu * 256 * row_bytes;
  char* out;
  hipMalloc(&out, bytes);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  // every tile: 256 rows x 256 B = 64 KB = 64 wave-instructions of 1 KB -> 8 per wave
  const int nstore = 8;
  printf("{\"runs\": [\n");
  auto run = [&](auto kern, const char* name, bool last) {
    hipLaunchKernelGGL(kern, dim3(ncu), dim3(512), 0, 0, out, row_bytes, tiles, nstore);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(ncu), dim3(512), 0, 0, out, row_bytes, tiles, nstore);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double b = (double)tiles * ncu * 256 * 256;
    printf("{\"shape\": \"%s\", \"us\": %.1f, \"tbs\": %.2f}%s\n", name, ms * 1e3, b / (ms * 1e-3) / 1e12, last ? "" : ",");
  };
  run(stores<64>, "16 rows x 64 B", false);
  run(stores<128>, "8 rows x 128 B", false);
  run(stores<256>, "4 rows x 256 B", true);
  printf("]}\n");
  return 0;
}

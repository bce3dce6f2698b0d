// Calibration of rocprofv3's FETCH_SIZE on gfx950 for the access shapes the
// library's kernels use (MI355X_MICROARCH.md "HBM": the x2 correction is
// measured for 16-B/lane streaming reads only; other widths are uncalibrated).
// Each kernel reads every byte of a 1 GiB buffer (far beyond L2 + MALL)
// exactly once, so the expected fetch is 1,073,741,824 B:
//   lds16   LDS-DMA, 1 KB contiguous per wave instruction (16 B / lane)
//   lds64   LDS-DMA, 16 segments of 64 B per wave instruction, segments 1 KB
//           apart (gemm1x1_ws's activation pieces: 16 pixel rows x 32 channels);
//           the 16 segments of each 1 KB row come from 16 instructions, issued
//           back to back by the same wave (consecutive k-steps)
//   reg16   global_load_dwordx4 into registers (16 B / lane)
//   reg8    global_load_dwordx2 into registers (8 B / lane)
//   dupx    lds16 over the first 512 MiB, read by TWO workgroups at the same
//           time: blocks b and b + 8 (the same XCD under round-robin placement)
//   dupy    the same with blocks b and b + 1 (different XCDs)
//           (unique bytes 512 MiB, requested 1 GiB: does FETCH_SIZE count a
//           line that two CUs miss on at once twice?)
// usage: fetch_calib <kernel>   (run one per rocprofv3 --pmc FETCH_SIZE pass)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

__device__ __forceinline__ void glds16(const void* src, uint32_t lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
}

constexpr size_t BYTES = 1ull << 30;

// one wave instruction = 1 KB; wave w of block b handles KB units u = (b * 8 + w) + k * (grid * 8)
__global__ __launch_bounds__(512) void lds16(const char* buf, int units_per_wave) {
  extern __shared__ char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t stride = (size_t)gridDim.x * 8;
  const uint32_t l = (uint32_t)(uintptr_t)smem + wave * 1024;
  for (int k = 0; k < units_per_wave; ++k) {
    const size_t u = (size_t)blockIdx.x * 8 + wave + k * stride;
    glds16(buf + u * 1024 + lane * 16, l);
    if ((k & 7) == 7) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// a "row block" = 16 rows x 1 KB = 16 KB; one instruction reads 64 B of each of
// the 16 rows (lane: row lane / 4, 16 B chunk lane % 4 within the 64-B
// segment); 16 instructions (segments 0..15) cover the block
__global__ __launch_bounds__(512) void lds64(const char* buf, int blocks_per_wave) {
  extern __shared__ char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t stride = (size_t)gridDim.x * 8;
  const uint32_t l = (uint32_t)(uintptr_t)smem + wave * 1024;
  for (int k = 0; k < blocks_per_wave; ++k) {
    const size_t blk = (size_t)blockIdx.x * 8 + wave + k * stride;
    const char* base = buf + blk * 16384 + (lane >> 2) * 1024 + (lane & 3) * 16;
    for (int seg = 0; seg < 16; ++seg) glds16(base + seg * 64, l);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// pairs of blocks read the same units: partner = b ^ pbit
__global__ __launch_bounds__(512) void dup(const char* buf, int units_per_wave, int pbit) {
  extern __shared__ char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int bb = blockIdx.x & ~pbit;                       // both partners use bb
  const int nb = gridDim.x / 2;                            // distinct block ids
  const int bi = (bb & (pbit - 1)) | ((bb / (2 * pbit)) * pbit);
  const size_t stride = (size_t)nb * 8;
  const uint32_t l = (uint32_t)(uintptr_t)smem + wave * 1024;
  for (int k = 0; k < units_per_wave; ++k) {
    const size_t u = (size_t)bi * 8 + wave + k * stride;
    glds16(buf + u * 1024 + lane * 16, l);
    if ((k & 7) == 7) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__global__ __launch_bounds__(512) void reg16(const uint4* buf, int per_thread, uint4* sink) {
  const size_t n = (size_t)gridDim.x * blockDim.x;
  uint4 acc = {0, 0, 0, 0};
  for (int k = 0; k < per_thread; ++k) {
    const uint4 v = buf[(size_t)blockIdx.x * blockDim.x + threadIdx.x + k * n];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if (acc.x == 0x12345678u) sink[threadIdx.x] = acc;
}

__global__ __launch_bounds__(512) void reg8(const uint2* buf, int per_thread, uint2* sink) {
  const size_t n = (size_t)gridDim.x * blockDim.x;
  uint2 acc = {0, 0};
  for (int k = 0; k < per_thread; ++k) {
    const uint2 v = buf[(size_t)blockIdx.x * blockDim.x + threadIdx.x + k * n];
    acc.x ^= v.x; acc.y ^= v.y;
  }
  if (acc.x == 0x12345678u) sink[threadIdx.x] = acc;
}

int main(int argc, char** argv) {
  const char* which = argc > 1 ? argv[1] : "lds16";
  char* buf = nullptr;
  void* sink = nullptr;
  if (hipMalloc(&buf, BYTES) != hipSuccess || hipMalloc(&sink, 1 << 16) != hipSuccess) return 1;
  hipMemset(buf, 1, BYTES);
  hipDeviceSynchronize();
  const int G = 1024;   // blocks of 512 threads
  for (int rep = 0; rep < 2; ++rep) {
    if (!strcmp(which, "lds16"))
      hipLaunchKernelGGL(lds16, dim3(G), dim3(512), 8192, 0, buf, (int)(BYTES / 1024 / (G * 8)));
    else if (!strcmp(which, "lds64"))
      hipLaunchKernelGGL(lds64, dim3(G), dim3(512), 8192, 0, buf, (int)(BYTES / 16384 / (G * 8)));
    else if (!strcmp(which, "dupx") || !strcmp(which, "dupy"))
      hipLaunchKernelGGL(dup, dim3(G), dim3(512), 8192, 0, buf, (int)(BYTES / 2 / 1024 / (G / 2 * 8)),
                         which[3] == 'x' ? 8 : 1);
    else if (!strcmp(which, "reg16"))
      hipLaunchKernelGGL(reg16, dim3(G), dim3(512), 0, 0, (const uint4*)buf,
                         (int)(BYTES / 16 / (G * 512)), (uint4*)sink);
    else if (!strcmp(which, "reg8"))
      hipLaunchKernelGGL(reg8, dim3(G), dim3(512), 0, 0, (const uint2*)buf,
                         (int)(BYTES / 8 / (G * 512)), (uint2*)sink);
    else return 2;
    if (hipDeviceSynchronize() != hipSuccess) return 3;
  }
  printf("%s: read %zu bytes per launch\n", which, BYTES);
  hipFree(buf);
  hipFree(sink);
  return 0;
}

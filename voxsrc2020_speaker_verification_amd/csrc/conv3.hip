// Persistent LDS-DMA pipelined implicit GEMM for the bf16 3x3 branch convs of
// the wide Res2Net stages (res2net_pad_conv_bn_relu, res2net_model.py:26-78:
// split width w = 96 (L3) and 192 (L4), stride 1 SAME or stride 2 with the
// fixed (1,1) pad) -- the second-largest kernel group of the extraction
// forward after the 1x1 GEMMs.
//
// Same machine as gemm1x1_pipe (gemm.hip): one workgroup per CU walks a
// contiguous list of (256-pixel x 96-cout) tiles with one continuous
// global_load_lds stream over all (tile, K-step) pairs into a 3-slot LDS
// ring, every global access counted by hand.  What differs:
//   * the B operand is gathered im2col-style: K runs tap-major (k = tap*Cin +
//     ci, the generic conv path's order), a 64-wide K-step is 8 chunks of 8
//     channels, and each lane's DMA source is its pixel shifted by the chunk's
//     tap (dy, dx) -- out-of-image taps (and k >= 9*Cin) read a zero line;
//   * the 96 couts of a tile are the six 16-row MFMA tiles of every wave
//     (8 waves x 32 pixels); LDS weight row r holds output channel
//     32(r/32) + 8((r%16)/4) + 4((r/16)%2) + r%4 (the paired-row permutation,
//     applied on the DMA source), so a lane ends up with 8 consecutive
//     channels of a pixel: 16-B epilogue loads and stores;
//   * the hierarchical addend of the next branch (z_{k+1} = x_{k+1} + y_k,
//     res2net_model.py:62-65) is produced in this kernel's epilogue, in place
//     over x_{k+1}, with the same bf16 roundings as the unfused path
//     (y_k rounded to bf16, the sum in fp32, rounded to bf16), so the next
//     branch's DMA reads a plain tensor.
// Accumulation order per output = K chunks of 32 in increasing order, as in
// conv_igemm: results are bitwise identical to the generic conv path.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_common.h"
#include "kernels.h"

namespace vox {

namespace {
constexpr int C3_BM = 256;                 // pixels per tile
constexpr int C3_BN = 96;                  // output channels per tile
constexpr int C3_AR = 128;                 // LDS weight rows per slot (96 used)
constexpr int C3_ROWS = C3_AR + C3_BM;     // 128-B rows per ring slot
constexpr int C3_SLOT = C3_ROWS * 128;     // 48 KB
constexpr int C3_NST = 3;                  // ring slots
constexpr int C3_NT = 512;                 // 8 waves
constexpr int C3_NA = C3_AR * 8 / C3_NT;   // weight DMA pieces per thread per step (2)
constexpr int C3_NB = C3_BM * 8 / C3_NT;   // pixel DMA pieces per thread per step (4)
constexpr int C3_NL = C3_NA + C3_NB;       // DMA instructions per wave per step (6)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void c3_glds16(const void* src, uint32_t lds) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds)
      : "memory");
}

// an ordinary (compiler-visible) load: the compiler's waitcnt pass covers
// every use and copy of the destination (see device_common.h vld16); the
// counted wait before the epilogue stays as the place the values are needed
__device__ __forceinline__ void c3_gld16(u32x4& v, const void* src) {
  v = *reinterpret_cast<const u32x4*>(src);
}

// the trailing s_nop keeps the next instruction from overwriting the data
// registers before the store has read them
__device__ __forceinline__ void c3_gst16(void* dst, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" : : "v"(dst), "v"(v) : "memory");
}

template <int N> __device__ __forceinline__ void c3_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" : : "n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
}  // namespace

__device__ uint4 g_conv3_zero[4] = {};     // source of padded taps / k >= 9*Cin
__device__ uint4 g_conv3_sink[64];         // destination of masked lanes' stores

#pragma clang fp contract(off)
// ConvParams use: x/ldx input (one split slice), w = [Cout][9*Cin] tap-major
// bf16, y/ldy output slice, mean/inv BN; res/ldr = x_{k+1} and y2/ldy2 = where
// z_{k+1} goes (the same slice, in place) when HAS_Z.
template <int CIN, bool HAS_Z>
__global__ __launch_bounds__(C3_NT) __attribute__((amdgpu_waves_per_eu(2, 2)))
void conv3x3_pipe(ConvParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int K = 9 * CIN;
  constexpr int KT = (K + 63) / 64;
  constexpr int NST_ST = HAS_Z ? 12 : 6;   // epilogue stores per wave
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int M = p.N * p.Ho * p.Wo;
  const int HoWo = p.Ho * p.Wo;
  const int cblocks = p.Cout / C3_BN;
  const int T = ((M + C3_BM - 1) / C3_BM) * cblocks;
  // XCD-contiguous tile ranges, as gemm1x1_pipe
  int t_first, t_step, ntiles;
  {
    const int G = gridDim.x;
    if ((G & 7) == 0) {
      const int x = blockIdx.x & 7, bi = blockIdx.x >> 3, nb = G >> 3;
      const int b0 = (int)((long)x * T / 8), b1 = (int)((long)(x + 1) * T / 8);
      t_first = b0 + bi;
      t_step = nb;
      ntiles = t_first < b1 ? (b1 - t_first + nb - 1) / nb : 0;
    } else {
      t_first = blockIdx.x;
      t_step = G;
      ntiles = t_first < T ? (T - t_first + G - 1) / G : 0;
    }
  }
  if (ntiles == 0) return;
  const int S = ntiles * KT;

  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(p.x);
  const bf16_t* __restrict__ Wt = reinterpret_cast<const bf16_t*>(p.w);
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  // DMA piece i of this thread: ring row i*64 + tid/8, slot tid%8, holding
  // source chunk cch = (tid%8) ^ ((row>>1)&7) -- the same for every piece
  const int rsub = tid >> 3;
  const int cch = (tid & 7) ^ ((rsub >> 1) & 7);
  const uint32_t lds_wave = lds0 + (uint32_t)wave * 1024u;
  const bf16_t* zero = reinterpret_cast<const bf16_t*>(g_conv3_zero);

  const bf16_t* pa[C3_NA];
  const bf16_t* pb[C3_NB];
  int hin[C3_NB], win[C3_NB], hl[C3_NB];   // hl: the pixel's utterance's valid input rows
  auto set_load_tile = [&](int tj) {
    const int lid = t_first + tj * t_step;
    const int co0 = (lid % cblocks) * C3_BN;
    const int px0 = (lid / cblocks) * C3_BM;
#pragma unroll
    for (int i = 0; i < C3_NA; ++i) {
      int r = i * 64 + rsub;
      r = r < C3_BN ? r : 0;   // rows 96..127 are never read: re-fetch row 0
      const int ch = 32 * (r >> 5) + 8 * ((r & 15) >> 2) + 4 * ((r >> 4) & 1) + (r & 3);
      pa[i] = Wt + (size_t)(co0 + ch) * K + cch * 8;
    }
#pragma unroll
    for (int i = 0; i < C3_NB; ++i) {
      // rows past M re-read pixel M-1: their outputs are never stored
      const int pix = min(px0 + i * 64 + rsub, M - 1);
      const int n = pix / HoWo, rr = pix - n * HoWo;
      const int ho = rr / p.Wo, wo = rr - ho * p.Wo;
      hin[i] = ho * p.sh;
      win[i] = wo * p.sw;
      hl[i] = valid_rows(p.vlen, p.vsh, n, p.H);   // ragged batch: rows past it are padding
      pb[i] = X + (((size_t)n * p.H + hin[i]) * p.W + win[i]) * p.ldx;
    }
  };
  int l_tile = 0, l_k = 0;
  auto issue = [&](int s_slot) {
    const uint32_t base = lds_wave + (uint32_t)s_slot * C3_SLOT;
    const int k = l_k * 64 + cch * 8;
    const bool kin = k < K;
    const int tap = kin ? k / CIN : 0;
    const int ci = k - tap * CIN;
    const int ky = tap / 3;
    const int dy = ky - 1, dx = tap - 3 * ky - 1;
    const long off = ((long)dy * p.W + dx) * p.ldx + ci;
#pragma unroll
    for (int i = 0; i < C3_NA; ++i) c3_glds16(kin ? pa[i] + l_k * 64 : zero, base + i * 8192u);
#pragma unroll
    for (int i = 0; i < C3_NB; ++i) {
      const bool ok = kin && (unsigned)(hin[i] + dy) < (unsigned)hl[i] &&
                      (unsigned)(win[i] + dx) < (unsigned)p.W;
      c3_glds16(ok ? pb[i] + off : zero, base + (C3_NA + i) * 8192u);
    }
    // advance; past the last tile the final step is re-read (never consumed)
    if (l_k + 1 < KT) {
      ++l_k;
    } else if (l_tile + 1 < ntiles) {
      ++l_tile;
      l_k = 0;
      set_load_tile(l_tile);
    }
  };

  set_load_tile(0);
  issue(0);
  issue(1);

  f32x4 acc[6][2];
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bf16_t* __restrict__ XZ = reinterpret_cast<const bf16_t*>(p.res);
  bf16_t* __restrict__ Y = reinterpret_cast<bf16_t*>(p.y);
  bf16_t* __restrict__ Z = reinterpret_cast<bf16_t*>(p.y2);

  int c_tile = 0, c_k = 0;
  int epi_age = 8;   // steps since the last epilogue's stores
  int offa[6], offb[2];
#pragma unroll
  for (int i = 0; i < 6; ++i) offa[i] = (16 * i + col) * 128;
#pragma unroll
  for (int j = 0; j < 2; ++j) offb[j] = (C3_AR + wave * 32 + 16 * j + col) * 128;
  const int swa = (col >> 1) & 7;   // (row>>1)&7 of every fragment row

  // epilogue operands (BN, x_{k+1}) are fetched right after the DMA issue of
  // step L0 = KT-1-LEAD, so LEAD steps of MFMAs cover their latency
  constexpr int LEAD = 2;
  constexpr int L0 = KT - 1 - LEAD;
  static_assert(L0 >= 0, "K too short for the epilogue lead");
  constexpr int EPI_LD = HAS_Z ? 18 : 12;  // epilogue loads per wave
  u32x4 bm[3][2] = {}, bi[3][2] = {}, xz[3][2] = {};
  for (int s = 0; s < S; ++s) {
    // step s's operands landed; younger: step s+1's DMA, the epilogue loads
    // while they are in flight (steps L0+1 .. KT-1) and, in the two steps
    // after an epilogue, its stores -- exactly the ops issued after step s's DMA
    const bool el = c_k > L0;
    if (epi_age <= 1) {
      if (el) c3_wait_vm<C3_NL + NST_ST + EPI_LD>(); else c3_wait_vm<C3_NL + NST_ST>();
    } else {
      if (el) c3_wait_vm<C3_NL + EPI_LD>(); else c3_wait_vm<C3_NL>();
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const bool last = (c_k == KT - 1);
    const int lid = t_first + c_tile * t_step;
    const int co0 = (lid % cblocks) * C3_BN;
    const int px0 = (lid / cblocks) * C3_BM;
    issue((s + 2) % C3_NST);
    if (c_k == L0) {
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int ch = co0 + 32 * q + 8 * g;
        c3_gld16(bm[q][0], p.mean + ch);
        c3_gld16(bm[q][1], p.mean + ch + 4);
        c3_gld16(bi[q][0], p.inv + ch);
        c3_gld16(bi[q][1], p.inv + ch + 4);
        if (HAS_Z) {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int pix = min(px0 + wave * 32 + 16 * j + col, M - 1);
            c3_gld16(xz[q][j], XZ + (size_t)pix * p.ldr + ch);
          }
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    const char* L = smem + (s % C3_NST) * C3_SLOT;
    {
      // both half-steps' fragments are read before the first MFMA (the LDS
      // latency exposed once per step, counted lgkmcnt waits in issue order);
      // the all-zero half-step past K (K % 64 == 32) is skipped, as in the
      // generic path's K loop
      const bool two = !((K % 64) != 0 && last);
      bf16x8 a[2][6], b[2][2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int cs = ((ks * 4 + g) ^ swa) << 4;
#pragma unroll
        for (int j = 0; j < 2; ++j) b[ks][j] = *reinterpret_cast<const bf16x8*>(L + offb[j] + cs);
#pragma unroll
        for (int i = 0; i < 6; ++i) a[ks][i] = *reinterpret_cast<const bf16x8*>(L + offa[i] + cs);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if (ks == 1 && !two) break;
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma_step(a[ks][i], b[ks][j], acc[i][j]);
      }
    }
    ++epi_age;
    if (last) {
      // the epilogue loads precede LEAD DMA issues (steps KT-1-LEAD+2 ..)
      if (HAS_Z) {
        asm volatile("s_waitcnt vmcnt(%18)"
                     : "+v"(bm[0][0]), "+v"(bm[0][1]), "+v"(bm[1][0]), "+v"(bm[1][1]),
                       "+v"(bm[2][0]), "+v"(bm[2][1]), "+v"(bi[0][0]), "+v"(bi[0][1]),
                       "+v"(bi[1][0]), "+v"(bi[1][1]), "+v"(bi[2][0]), "+v"(bi[2][1]),
                       "+v"(xz[0][0]), "+v"(xz[0][1]), "+v"(xz[1][0]), "+v"(xz[1][1]),
                       "+v"(xz[2][0]), "+v"(xz[2][1])
                     : "n"(C3_NL * LEAD)
                     : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(%12)"
                     : "+v"(bm[0][0]), "+v"(bm[0][1]), "+v"(bm[1][0]), "+v"(bm[1][1]),
                       "+v"(bm[2][0]), "+v"(bm[2][1]), "+v"(bi[0][0]), "+v"(bi[0][1]),
                       "+v"(bi[1][0]), "+v"(bi[1][1]), "+v"(bi[2][0]), "+v"(bi[2][1])
                     : "n"(C3_NL * LEAD)
                     : "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int ch = co0 + 32 * q + 8 * g;
        const f32x4 m0 = __builtin_bit_cast(f32x4, bm[q][0]);
        const f32x4 m1 = __builtin_bit_cast(f32x4, bm[q][1]);
        const f32x4 i0 = __builtin_bit_cast(f32x4, bi[q][0]);
        const f32x4 i1 = __builtin_bit_cast(f32x4, bi[q][1]);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int pix = px0 + wave * 32 + 16 * j + col;
          float v[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = (acc[2 * q][j][e] - m0[e]) * i0[e];
            v[4 + e] = (acc[2 * q + 1][j][e] - m1[e]) * i1[e];
          }
          bf16x8 o;
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = (bf16_t)fmaxf(v[e], 0.f);
          const bool in = pix < M;
          c3_gst16(in ? (void*)(Y + (size_t)pix * p.ldy + ch) : (void*)&g_conv3_sink[lane],
                   __builtin_bit_cast(u32x4, o));
          if (HAS_Z) {
            const bf16x8 xv = __builtin_bit_cast(bf16x8, xz[q][j]);
            bf16x8 zv;
#pragma unroll
            for (int e = 0; e < 8; ++e) zv[e] = (bf16_t)((float)xv[e] + (float)o[e]);
            c3_gst16(in ? (void*)(Z + (size_t)pix * p.ldy2 + ch) : (void*)&g_conv3_sink[lane],
                     __builtin_bit_cast(u32x4, zv));
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      epi_age = 0;
      c_k = 0;
      ++c_tile;
    } else {
      ++c_k;
    }
  }
  // drain: the trailing (never consumed) DMA must land before the workgroup
  // releases its LDS
  c3_wait_vm<0>();
}

int conv3_pipe_ok(const ConvParams& p) {
  if (!(p.Cin == 96 || p.Cin == 192) || p.kh != 3 || p.kw != 3 || p.groups != 1) return 0;
  if (p.dh != 1 || p.dw != 1 || p.ph != 1 || p.pw != 1 || p.sh != p.sw) return 0;
  if (!(p.sh == 1 || p.sh == 2)) return 0;
  if (p.Ho != (p.H + p.sh - 1) / p.sh || p.Wo != (p.W + p.sw - 1) / p.sw) return 0;
  if (p.Cout % C3_BN != 0 || p.ldx % 8 || p.ldy % 8 || p.ldr % 8 || p.ldy2 % 8) return 0;
  if (p.flags != (EPI_AFFINE | EPI_RELU) || p.in_mean || p.x2) return 0;
  return p.N * p.Ho * p.Wo > 0;
}

template <int CIN, bool Z>
static void launch_c3(const ConvParams& p, int G, hipStream_t s) {
  hipLaunchKernelGGL((conv3x3_pipe<CIN, Z>), dim3(G), dim3(C3_NT), C3_NST * C3_SLOT, s, p);
}

hipError_t launch_conv3_pipe(const ConvParams& p, int num_cu, hipStream_t s) {
  if (!conv3_pipe_ok(p) || !p.mean || !p.inv) return hipErrorInvalidValue;
  const bool z = p.y2 != nullptr;
  if (z && (!p.res || p.sh != 1)) return hipErrorInvalidValue;
  const int M = p.N * p.Ho * p.Wo;
  const int T = ((M + C3_BM - 1) / C3_BM) * (p.Cout / C3_BN);
  int G = num_cu < T ? num_cu : T;
  if (G >= 8) G = G / 8 * 8;   // XCD-contiguous mapping needs a multiple of 8
  if (p.Cin == 96) {
    if (z) launch_c3<96, true>(p, G, s); else launch_c3<96, false>(p, G, s);
  } else {
    if (z) launch_c3<192, true>(p, G, s); else launch_c3<192, false>(p, G, s);
  }
  return hipGetLastError();
}

}  // namespace vox

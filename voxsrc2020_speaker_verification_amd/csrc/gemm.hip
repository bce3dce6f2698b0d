// Persistent, LDS-DMA pipelined GEMM for the bf16 1x1 convolutions of the
// Res2Net bottlenecks (conv1x1a / conv1x1c / projection shortcut,
// res2net_model.py:90-127 via tf_extract.py) -- the largest kernel group of
// the extraction forward.
//
// Why a second GEMM: the 1x1 convs have short K (192..1024, i.e. 3..16
// K-steps of 64) and big M (64K..1M pixels).  gemm1x1_lds (kernels.hip) pays a
// pipeline prologue and an unoverlapped epilogue (residual read + stores) on
// every 128x128 tile and keeps only one K-tile of loads ahead of the MFMAs.
// Here one workgroup per CU walks a contiguous list of tiles with ONE
// continuous load stream over all (tile, K-step) pairs:
//   * 8 waves, tile 256 pixels x 128 output channels, BK = 64; wave (wm, wn)
//     owns 64 couts x 64 pixels = 4x4 MFMA 16x16x32 accumulators;
//   * operands go global -> LDS by global_load_lds_dwordx4 (no staging VGPRs)
//     into a 3-slot ring (3 x 48 KB): the loads of K-steps s+1 and s+2 are in
//     flight while step s is computed, including across tile boundaries, so the
//     next tile's first operands arrive during this tile's epilogue;
//   * every global access of the loop is inline asm and counted by hand
//     (s_waitcnt vmcnt(6) or (14) at the top of a step): the compiler never
//     sees a VGPR load beside the in-flight DMA and never drains it;
//   * residual tile and BN parameters are fetched at the start of a tile's
//     last K-step, so their latency hides under that step's MFMAs;
//   * lanes whose output is masked store into a sink, so every wave issues a
//     fixed number of stores and the vmcnt arithmetic stays exact.
// LDS rows are 128 B; 16-B chunk c of ring row r sits at slot c ^ ((r>>1)&7)
// (the gemm1x1_lds swizzle: conflict-free ds_read_b128).  DMA writes are
// lane-linear, so the swizzle is applied to the per-lane SOURCE chunk.
// Accumulation order per output = K chunks of 32 in increasing order, same as
// every other bf16 1x1 path: results are bitwise identical to gemm1x1_lds.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_common.h"
#include "kernels.h"

namespace vox {

namespace {
constexpr int GP_BM = 256;                 // pixels per tile
constexpr int GP_BN = 128;                 // output channels per tile
constexpr int GP_ROWS = GP_BM + GP_BN;     // 128-B rows per ring slot
constexpr int GP_SLOT = GP_ROWS * 128;     // bytes per slot (48 KB)
constexpr int GP_NST = 3;                  // ring slots
constexpr int GP_NT = 512;                 // threads (8 waves)
constexpr int GP_NA = GP_BN * 8 / GP_NT;   // weight DMA pieces per thread per step (2)
constexpr int GP_NB = GP_BM * 8 / GP_NT;   // pixel DMA pieces per thread per step (4)
constexpr int GP_NL = GP_NA + GP_NB;       // DMA instructions per wave per step (6)
}  // namespace

__device__ uint4 g_gemm_sink[64];          // destination of masked lanes' stores
__device__ uint4 g_gemm_zero[4] = {};      // DMA source of the K tail past kp (PRO)

__device__ __forceinline__ void glds16(const void* src, uint32_t lds) {
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

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// an ordinary (compiler-visible) load: the compiler's waitcnt pass covers
// every use and copy of the destination (see device_common.h vld16); the
// counted wait before the epilogue stays as the place the values are needed
__device__ __forceinline__ void gld16(u32x4& v, const void* src) {
  v = *reinterpret_cast<const u32x4*>(src);
}

// the trailing s_nop keeps the next instruction from overwriting the data
// registers before the store has read them
__device__ __forceinline__ void gst16(void* dst, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" : : "v"(dst), "v"(v) : "memory");
}

template <int N> __device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" : : "n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

#pragma clang fp contract(off)
// PRO: BN+ReLU input prologue relu((x - in_mean[k]) * in_inv[k]) (DPN68
// bn_relu_conv, dpn_model.py:40-54), applied once per element to each step's
// pixel rows in LDS after the DMA lands (prologue table staged in LDS at
// start, one extra barrier per step); channels k >= Cin are zero, as in the
// generic conv.  K may end on a half step (kp % 64 = 32): the tail DMA reads
// a zero line and the all-zero MFMA half step is skipped.
// DBG (diagnostics only, VOXEMB_GEMM_VAR=2/3): 1 = no MFMA / fragment reads,
// 2 = no operand DMA (MFMAs on whatever the ring holds); results are garbage
template <int SWZ, bool PRO, int DBG = 0>
__global__ __launch_bounds__(GP_NT) __attribute__((amdgpu_waves_per_eu(2, 2)))
void gemm1x1_pipe(ConvParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int col = lane & 15, g = lane >> 4;
  const int M = p.N * p.Ho * p.Wo;
  const int HoWo = p.Ho * p.Wo;
  const int KT = (p.kp + 63) / 64;
  const int cblocks = p.coutp / GP_BN;
  const int T = ((M + GP_BM - 1) / GP_BM) * cblocks;
  // tiles of this workgroup: XCD x (blocks x, x+8, ...) owns the contiguous
  // range [x*T/8, (x+1)*T/8) and its nb workgroups take every nb-th tile, so at
  // any moment one XCD works on nb consecutive tiles (the cout blocks of a
  // pixel block share its L2 lines)
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
  const int S = ntiles * KT;   // (tile, K-step) pairs of this workgroup

  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(p.x);
  const bf16_t* __restrict__ Wt = reinterpret_cast<const bf16_t*>(p.w);
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  // DMA piece i of this thread: ring row r = i*64 + tid/8 at slot tid%8, which
  // holds source chunk (tid%8) ^ ((r>>1)&7); rows 0..127 weights, 128.. pixels
  const int slot = tid & 7;
  const int rsub = tid >> 3;
  // source chunk of every DMA piece of this thread (see set_load_tile)
  const int cch = SWZ ? slot ^ ((rsub >> 1) & 7) : slot;
  const bf16_t* gzero = reinterpret_cast<const bf16_t*>(g_gemm_zero);
  const uint32_t lds_wave = lds0 + (uint32_t)wave * 1024u;

  // load-side state: the tile whose operands are being fetched
  const bf16_t* pa[GP_NA];
  const bf16_t* pb[GP_NB];
  auto set_load_tile = [&](int tj) {
    const int lid = t_first + tj * t_step;
    const int co0 = (lid % cblocks) * GP_BN;
    const int px0 = (lid / cblocks) * GP_BM;
#pragma unroll
    for (int i = 0; i < GP_NA; ++i) {
      const int r = i * 64 + rsub;
      const int c = SWZ ? slot ^ ((r >> 1) & 7) : slot;
      pa[i] = Wt + (size_t)(co0 + r) * p.kp + c * 8;
    }
#pragma unroll
    for (int i = 0; i < GP_NB; ++i) {
      const int r = (GP_NA + i) * 64 + rsub;
      const int c = SWZ ? slot ^ ((r >> 1) & 7) : slot;
      // rows past M re-read pixel M-1: their outputs are never stored
      const int pix = min(px0 + r - GP_BN, M - 1);
      const int n = pix / HoWo, rr = pix - n * HoWo;
      const int ho = rr / p.Wo, wo = rr - ho * p.Wo;
      pb[i] = X + (((size_t)n * p.H + ho * p.sh) * p.W + wo * p.sw) * p.ldx + c * 8;
    }
  };
  int l_tile = 0, l_k = 0;
  auto issue = [&](int s_slot) {
    const uint32_t base = lds_wave + (uint32_t)s_slot * GP_SLOT;
    const int ko = l_k * 64;
    const bool kin = !PRO || ko + cch * 8 < p.kp;
    if (DBG == 2) goto advance;
#pragma unroll
    for (int i = 0; i < GP_NA; ++i) glds16(kin ? pa[i] + ko : gzero, base + i * 8192u);
#pragma unroll
    for (int i = 0; i < GP_NB; ++i) glds16(kin ? pb[i] + ko : gzero, base + (GP_NA + i) * 8192u);
    // advance; past the last tile the final step is re-read (never consumed)
  advance:
    if (l_k + 1 < KT) {
      ++l_k;
    } else if (l_tile + 1 < ntiles) {
      ++l_tile;
      l_k = 0;
      set_load_tile(l_tile);
    }
  };

  const float* ptab = reinterpret_cast<const float*>(smem + GP_NST * GP_SLOT);
  if (PRO) {
    float* tab = reinterpret_cast<float*>(smem + GP_NST * GP_SLOT);
    for (int k = tid; k < p.kp; k += GP_NT) {
      tab[k] = k < p.Cin ? p.in_mean[k] : 0.f;
      tab[p.kp + k] = k < p.Cin ? p.in_inv[k] : 0.f;
    }
    __syncthreads();   // no DMA in flight yet
  }

  set_load_tile(0);
  issue(0);
  issue(1);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int flags = p.flags;
  const bf16_t* __restrict__ R = reinterpret_cast<const bf16_t*>(p.res);
  bf16_t* __restrict__ Y = reinterpret_cast<bf16_t*>(p.y);
  bf16_t* __restrict__ Y2 = reinterpret_cast<bf16_t*>(p.y2);

  int c_tile = 0, c_k = 0;
  int epi_age = 8;   // steps since the last epilogue's stores
  // per-wave LDS byte offsets of the A / B fragment rows (slot 0)
  int offa[4], offb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ra = wm * 64 + 16 * i + col;
    const int rb = GP_BN + wn * 64 + 16 * i + col;
    offa[i] = ra * 128;
    offb[i] = rb * 128;
  }
  const int swa = SWZ ? (col >> 1) & 7 : 0;   // (r>>1)&7 for every fragment row (rows differ by multiples of 16)

  // epilogue operands (BN, residual tile) are fetched right after the DMA
  // issue of step L0 = KT-1-LEAD, so LEAD steps of MFMAs cover their latency
  // (K >= 192: KT >= 3)
  constexpr int LEAD = 2;
  const int L0 = KT - 1 - LEAD;
  const int EPI_LD = ((flags & EPI_AFFINE) ? 8 : 0) + ((flags & EPI_RES) ? 8 : 0);
  u32x4 rv[2][4] = {};
  u32x4 bm[2][2] = {}, bi[2][2] = {};
  for (int s = 0; s < S; ++s) {
    // operands of step s landed (this wave's DMA); younger: exactly the ops
    // issued after that DMA -- step s+1's six pieces, the epilogue loads while
    // in flight (steps L0+1 .. KT-1), and in the two steps after an epilogue
    // its eight stores
    const bool el = c_k > L0 && EPI_LD > 0;
    if (epi_age <= 1) {
      if (!el) wait_vm<GP_NL + 8>();
      else if (EPI_LD == 16) wait_vm<GP_NL + 8 + 16>();
      else wait_vm<GP_NL + 8 + 8>();
    } else {
      if (!el) wait_vm<GP_NL>();
      else if (EPI_LD == 16) wait_vm<GP_NL + 16>();
      else wait_vm<GP_NL + 8>();
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (PRO) {
      // prologue once per element, in place in this step's LDS pixel rows:
      // chunk (row r, slot sl) holds input channels k .. k+7 of the step,
      // bf16(relu((x - m) * inv)), zero for k >= Cin (and for the zero tail)
      char* Lw = smem + (s % GP_NST) * GP_SLOT;
#pragma unroll
      for (int i = 0; i < (GP_BM * 8) / GP_NT; ++i) {
        const int chunk = tid + GP_NT * i;
        const int r = chunk >> 3, sl = chunk & 7;
        const int src = SWZ ? sl ^ ((r >> 1) & 7) : sl;
        const int k = c_k * 64 + src * 8;
        bf16x8* q = reinterpret_cast<bf16x8*>(Lw + (GP_BN + r) * 128 + sl * 16);
        bf16x8 v = *q;
        if (k < p.Cin) {
          const f32x4 m0 = *reinterpret_cast<const f32x4*>(ptab + k);
          const f32x4 m1 = *reinterpret_cast<const f32x4*>(ptab + k + 4);
          const f32x4 i0 = *reinterpret_cast<const f32x4*>(ptab + p.kp + k);
          const f32x4 i1 = *reinterpret_cast<const f32x4*>(ptab + p.kp + k + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = (bf16_t)fmaxf(((float)v[e] - m0[e]) * i0[e], 0.f);
            v[4 + e] = (bf16_t)fmaxf(((float)v[4 + e] - m1[e]) * i1[e], 0.f);
          }
        } else {
          v = bf16x8{};
        }
        *q = v;
      }
      // LDS writes visible to every wave; the DMA stays in flight (no vmcnt)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    const bool last = (c_k == KT - 1);
    const int lid = t_first + c_tile * t_step;
    const int co0 = (lid % cblocks) * GP_BN;
    const int px0 = (lid / cblocks) * GP_BM;
    issue((s + 2) % GP_NST);
    if (c_k == L0) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int ch = co0 + wm * 64 + 32 * q + 8 * g;
        const int chc = ch < p.Cout ? ch : 0;
        if (flags & EPI_AFFINE) {
          gld16(bm[q][0], p.mean + chc);
          gld16(bm[q][1], p.mean + chc + 4);
          gld16(bi[q][0], p.inv + chc);
          gld16(bi[q][1], p.inv + chc + 4);
        }
        if (flags & EPI_RES) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int pix = min(px0 + wn * 64 + 16 * j + col, M - 1);
            gld16(rv[q][j], R + (size_t)pix * p.ldr + chc);
          }
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    const int sb = (s % GP_NST) * GP_SLOT;
    const char* L = smem + sb;
    if (PRO) {   // (register budget: the prologue variant reads per half step)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if (ks == 1 && last && (p.kp & 63)) break;   // zero half step past kp
        const int cs = ((ks * 4 + g) ^ swa) << 4;
        bf16x8 a[4], b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          a[i] = *reinterpret_cast<const bf16x8*>(L + offa[i] + cs);
          b[i] = *reinterpret_cast<const bf16x8*>(L + offb[i] + cs);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma_step(a[i], b[j], acc[i][j]);
      }
    } else if (DBG != 1) {
      // both half-steps' fragments are read before the first MFMA (the LDS
      // latency exposed once per step, counted lgkmcnt waits in issue order)
      const bool two = true;
      bf16x8 a[2][4], b[2][4];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int cs = ((ks * 4 + g) ^ swa) << 4;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          b[ks][i] = *reinterpret_cast<const bf16x8*>(L + offb[i] + cs);
          a[ks][i] = *reinterpret_cast<const bf16x8*>(L + offa[i] + cs);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if (ks == 1 && !two) break;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma_step(a[ks][i], b[ks][j], acc[i][j]);
      }
    }
    ++epi_age;
    if (last) {
      // the epilogue loads precede LEAD DMA issues (steps L0+1 .. KT-1).
      // The wait names every asm-load destination, so nothing reads (or
      // copies) those registers before the data has landed.
      asm volatile("s_waitcnt vmcnt(%16)"
                   : "+v"(rv[0][0]), "+v"(rv[0][1]), "+v"(rv[0][2]), "+v"(rv[0][3]),
                     "+v"(rv[1][0]), "+v"(rv[1][1]), "+v"(rv[1][2]), "+v"(rv[1][3]),
                     "+v"(bm[0][0]), "+v"(bm[0][1]), "+v"(bm[1][0]), "+v"(bm[1][1]),
                     "+v"(bi[0][0]), "+v"(bi[0][1]), "+v"(bi[1][0]), "+v"(bi[1][1])
                   : "n"(GP_NL * LEAD)
                   : "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int ch = co0 + wm * 64 + 32 * q + 8 * g;
        f32x4 m0, m1, i0, i1;
        if (flags & EPI_AFFINE) {
          m0 = __builtin_bit_cast(f32x4, bm[q][0]);
          m1 = __builtin_bit_cast(f32x4, bm[q][1]);
          i0 = __builtin_bit_cast(f32x4, bi[q][0]);
          i1 = __builtin_bit_cast(f32x4, bi[q][1]);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int pix = px0 + wn * 64 + 16 * j + col;
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
              v[e] = (v[e] - m0[e]) * i0[e];
              v[4 + e] = (v[4 + e] - m1[e]) * i1[e];
            }
          }
          if ((flags & EPI_RES) && ch < p.ysplit) {   // the dual-destination part has none
            const bf16x8 r8 = __builtin_bit_cast(bf16x8, rv[q][j]);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += (float)r8[e];
          }
          if (flags & EPI_RELU) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
          }
          bf16x8 o;
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = (bf16_t)v[e];
          void* dst;
          if (ch < p.Cout && pix < M)
            dst = ch < p.ysplit ? (void*)(Y + (size_t)pix * p.ldy + ch)
                                : (void*)(Y2 + (size_t)pix * p.ldy2 + (ch - p.ysplit));
          else
            dst = &g_gemm_sink[lane];
          gst16(dst, __builtin_bit_cast(u32x4, o));
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      epi_age = 0;
      c_k = 0;
      ++c_tile;
    } else {
      ++c_k;
    }
  }
  // drain: the trailing (never consumed) DMA must land before the workgroup
  // releases its LDS
  wait_vm<0>();
}

int gemm_pipe_ok(const ConvParams& p) {
  const int M = p.N * p.Ho * p.Wo;
  const int T = ((M + GP_BM - 1) / GP_BM) * (p.coutp / GP_BN);
  if (p.in_mean) {
    // prologue variant: K in 32-steps, at least three 64-steps, table in LDS
    if (p.kp % 32 || (p.kp + 63) / 64 < 3 || p.kp > 1024 || p.Cin > p.kp || p.Cin % 8 ||
        !p.in_inv)
      return 0;
  } else if (p.kp % 64 || p.kp / 64 < 3) {
    return 0;
  }
  return p.coutp % GP_BN == 0 && T >= 8;
}

hipError_t launch_gemm_pipe(const ConvParams& p, int num_cu, int variant, hipStream_t s) {
  if (!gemm_pipe_ok(p)) return hipErrorInvalidValue;
  const int M = p.N * p.Ho * p.Wo;
  const int T = ((M + GP_BM - 1) / GP_BM) * (p.coutp / GP_BN);
  int G = num_cu < T ? num_cu : T;
  G = G / 8 * 8;
  if (p.in_mean)
    hipLaunchKernelGGL((gemm1x1_pipe<1, true>), dim3(G), dim3(GP_NT),
                       GP_NST * GP_SLOT + 8 * p.kp, s, p);
  else if (variant == 1)
    hipLaunchKernelGGL((gemm1x1_pipe<0, false>), dim3(G), dim3(GP_NT), GP_NST * GP_SLOT, s, p);
#ifdef VOX_DIAG
  else if (variant == 2)
    hipLaunchKernelGGL((gemm1x1_pipe<1, false, 1>), dim3(G), dim3(GP_NT), GP_NST * GP_SLOT, s, p);
  else if (variant == 3)
    hipLaunchKernelGGL((gemm1x1_pipe<1, false, 2>), dim3(G), dim3(GP_NT), GP_NST * GP_SLOT, s, p);
#endif
  else
    hipLaunchKernelGGL((gemm1x1_pipe<1, false>), dim3(G), dim3(GP_NT), GP_NST * GP_SLOT, s, p);
  return hipGetLastError();
}

}  // namespace vox

// Wide-tile persistent LDS-DMA GEMM for the bf16 1x1 convolutions of the
// Res2Net bottlenecks (conv1x1a / conv1x1c / projection shortcut,
// res2net_model.py:90-127 via tf_extract.py) and the TDNN 1x1 layers.
//
// Why: gemm1x1_pipe (gemm.hip) is bound by what a CU can pull through its
// memory pipe, not by MFMA (profiles: removing its MFMAs saves ~4 %, removing
// its operand DMA ~25 %).  Its 256-pixel x 128-cout tile re-reads every pixel
// row once per 128 output channels.  Here a tile is 256 pixels x BN couts
// (BN = 256, or 192 for the 192/384/768-channel 1x1a), so per output element
// the operand bytes a CU moves drop by a third (L3 1x1c: 6.5 -> 4.3 KB per
// pixel including the epilogue), and:
//   * BK = 32: a ring slot is (BN + 256) rows x 64 B (<= 32 KB), 4 slots,
//     three K-steps in flight (96 KB per CU) while one is computed;
//   * 8 waves as 2 (cout halves) x 4 (64-pixel quarters): a wave owns
//     BN/2 couts x 64 pixels = (BN/32) x 4 MFMA 16x16x32 accumulators;
//   * the residual tile of the 1x1c (res2net_model.py:100) is streamed by the
//     same DMA ring as four extra "phase" steps after the K-steps (64 pixels x
//     256 couts = 32 KB each): no residual registers, its latency covered like
//     an operand's, and the epilogue of 16-pixel column j runs in phase j;
//   * BN parameters of all output channels sit in LDS for the whole kernel.
// LDS operand rows are 64 B; 16-B chunk c of row r is stored at position
// c ^ f((r >> 2) & 3), f(a) = (4 - a) & 3, which makes the ds_read_b128
// fragment reads conflict-free under gfx950's 4 x 16-lane read groups (DMA
// writes are lane-linear, so the swizzle is applied to each lane's SOURCE
// chunk).  Residual rows are 512 B, chunk c at c ^ (r & 15).
// Accumulation order per output = K chunks of 32 in increasing order, and the
// epilogue is the same sequence of roundings: bitwise identical to
// gemm1x1_pipe / gemm1x1_lds.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <cstdint>
#include <type_traits>

#include "device_common.h"
#include "kernels.h"

namespace vox {

namespace {
constexpr int GW_BM = 256;      // pixels per tile
constexpr int GW_NT = 512;      // 8 waves
constexpr int GW_NST = 4;       // ring slots
constexpr int GW_SLOT = 32768;  // bytes per ring slot
constexpr int GW_NR = 4;        // residual phases per tile

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void gw_glds16(const void* src, uint32_t lds) {
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

// (diagnostics) the same with the non-temporal policy
__device__ __forceinline__ void gw_glds16_nt(const void* src, uint32_t lds) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds)
      : "memory");
}

// the trailing s_nop keeps the next instruction from overwriting the data
// registers before the store has read them
__device__ __forceinline__ void gw_st16(void* dst, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" : : "v"(dst), "v"(v) : "memory");
}
__device__ __forceinline__ void gw_st16_nt(void* dst, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" : : "v"(dst), "v"(v) : "memory");
}
__device__ __forceinline__ void gw_st16_sc1(void* dst, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" : : "v"(dst), "v"(v) : "memory");
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
// a - b on two lanes of a pair (v_pk_add_f32 with b negated: the rounding of two v_sub_f32)
__device__ __forceinline__ f32x2 gw_pk_sub(f32x2 a, f32x2 b) {
  f32x2 r;
  asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// max(0, v) as the one instruction fmaxf(v, 0.f) ends in (without its canonicalising
// v_max_f32 v, v, v: the operands here are arithmetic results, never signalling NaNs)
__device__ __forceinline__ float gw_relu(float v) {
  float r;
  asm("v_max_f32 %0, 0, %1" : "=v"(r) : "v"(v));
  return r;
}

#define GW_W(n) \
  case n: asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory"); break;
// s_waitcnt with a wave-uniform count (a scalar branch to the immediate form)
__device__ __forceinline__ void gw_wait_vm(int n) {
  switch (n) {
    GW_W(0) GW_W(1) GW_W(2) GW_W(3) GW_W(4) GW_W(5) GW_W(6) GW_W(7) GW_W(8) GW_W(9)
    GW_W(10) GW_W(11) GW_W(12) GW_W(13) GW_W(14) GW_W(15) GW_W(16) GW_W(17) GW_W(18)
    GW_W(19) GW_W(20) GW_W(21) GW_W(22) GW_W(23) GW_W(24) GW_W(25) GW_W(26) GW_W(27)
    GW_W(28) GW_W(29) GW_W(30) GW_W(31) GW_W(32)
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
  __builtin_amdgcn_sched_barrier(0);
}
#undef GW_W

__device__ __forceinline__ int gw_swz(int r) { return (4 - ((r >> 2) & 3)) & 3; }
}  // namespace

__device__ uint4 g_gw_sink[64];   // destination of masked lanes' stores
__device__ uint4 g_gw_zero[4] = {};   // source of the B rows outside an utterance (1-D taps)

#pragma clang fp contract(off)
// DBG (diagnostics only, VOXEMB_GEMM_VAR): 1 = no MFMA / fragment reads,
// 2 = no operand DMA, 4 = no output stores, 32 = non-temporal stores (same
// results), 64 = every store to one sink line; results are garbage
template <int BN, bool RES, int DBG = 0>
__global__ __launch_bounds__(GW_NT) __attribute__((amdgpu_waves_per_eu(2, 2)))
void gemm1x1_wide(ConvParams p) {
  constexpr int NI = BN / 32;                // 16-cout MFMA blocks per wave (BN/2 couts)
  constexpr int NQ = NI / 2;                 // 32-cout groups per wave
  constexpr int GRP = (BN + GW_BM) / 16;     // 1-KB DMA groups per operand step
  constexpr int NLMAX = (GRP + 7) / 8;
  constexpr int NR = RES ? GW_NR : 0;
  static_assert(!RES || GRP == 32, "residual phases need 4 DMA groups per wave");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int col = lane & 15, g = lane >> 4;
  const int NLw = (wave + 8 * (NLMAX - 1) < GRP) ? NLMAX : NLMAX - 1;   // wave-uniform
  const int M = p.N * p.Ho * p.Wo;
  const int HoWo = p.Ho * p.Wo;
  const int KT = p.kp / 32;
  const int SPT = KT + NR;                   // ring steps per tile
  const int cblocks = p.coutp / BN;
  const int T = ((M + GW_BM - 1) / GW_BM) * cblocks;
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
  const int S = ntiles * SPT;

  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(p.x);
  const bf16_t* __restrict__ Wt = reinterpret_cast<const bf16_t*>(p.w);
  const bf16_t* __restrict__ R = reinterpret_cast<const bf16_t*>(p.res);
  bf16_t* __restrict__ Y = reinterpret_cast<bf16_t*>(p.y);
  bf16_t* __restrict__ Y2 = reinterpret_cast<bf16_t*>(p.y2);
  const int flags = p.flags;
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  const uint32_t lds_wave = lds0 + (uint32_t)wave * 1024u;

  // BN tables (mean | inv) of every output channel, for the whole kernel
  float* tab = reinterpret_cast<float*>(smem + GW_NST * GW_SLOT);
  if (flags & EPI_AFFINE) {
    for (int k = tid; k < p.coutp; k += GW_NT) {
      tab[k] = k < p.Cout ? p.mean[k] : 0.f;
      tab[p.coutp + k] = k < p.Cout ? p.inv[k] : 0.f;
    }
  }
  __syncthreads();   // no DMA in flight yet

  // ---- load side: the (tile, step) whose operands are being fetched
  const bf16_t* src[NLMAX];
  int l_tile = 0, l_k = 0, l_co0 = 0, l_px0 = 0;
  auto set_load_tile = [&](int tj) {
    const int lid = t_first + tj * t_step;
    l_co0 = (lid % cblocks) * BN;
    l_px0 = (lid / cblocks) * GW_BM;
#pragma unroll
    for (int i = 0; i < NLMAX; ++i) {
      if (i >= NLw) break;
      // group gi = 16 rows of the slot; lane -> row 16gi + lane/4, position lane%4
      const int row = 16 * (wave + 8 * i) + (lane >> 2);
      const int c = (lane & 3) ^ gw_swz(row);
      if (row < BN) {
        src[i] = Wt + (size_t)(l_co0 + row) * p.kp + c * 8;
      } else {
        // rows past M re-read pixel M-1: their outputs are never stored
        const int pix = min(l_px0 + row - BN, M - 1);
        const int n = pix / HoWo, rr = pix - n * HoWo;
        const int ho = rr / p.Wo, wo = rr - ho * p.Wo;
        src[i] = X + (((size_t)n * p.H + ho * p.sh) * p.W + wo * p.sw) * p.ldx + c * 8;
      }
    }
  };
  // DMA piece i (1 KB per wave) of the step being fetched into ring slot `slot`
  auto issue_piece = [&](int slot, int i) {
    const uint32_t base = lds_wave + (uint32_t)slot * GW_SLOT + (uint32_t)i * 8192u;
    if (l_k < KT) {
      if (i < NLw && !(DBG & 2)) gw_glds16(src[i] + l_k * 32, base);
    } else if (RES) {
      // residual phase ph: slot row r (512 B) = pixel l_px0 + 64(r/16) + 16 ph + r%16
      const int ph = l_k - KT;
      const int row = 2 * (wave + 8 * i) + (lane >> 5);
      const int c = (lane & 31) ^ (row & 15);
      const int pix = min(l_px0 + 64 * i + 16 * ph + (row & 15), M - 1);
      gw_glds16(R + (size_t)pix * p.ldr + l_co0 + c * 8, base);
    }
  };
  // advance; past the last tile the final step is re-read (never consumed)
  auto advance = [&]() {
    if (l_k + 1 < SPT) {
      ++l_k;
    } else if (l_tile + 1 < ntiles) {
      ++l_tile;
      l_k = 0;
      set_load_tile(l_tile);
    }
  };
  auto issue = [&](int slot) {
#pragma unroll
    for (int i = 0; i < NLMAX; ++i) issue_piece(slot, i);
    advance();
  };

  set_load_tile(0);
  issue(0);
  issue(1);
  issue(2);

  f32x4 acc[NI][4];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int cs = (g ^ gw_swz(col)) << 4;   // fragment chunk byte offset (rows 16 | base)
  const int offa = (wm * (BN / 2) + col) * 64 + cs;
  const int offb = (BN + wn * 64 + col) * 64 + cs;

  // epilogue of 16-pixel column J for every 32-cout group (rl: residual slot or null)
  auto epi = [&](auto jc, int co0, int px0, const char* rl) {
    constexpr int J = decltype(jc)::value;
    const int pix = px0 + wn * 64 + 16 * J + col;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int chl = wm * (BN / 2) + 32 * q + 8 * g;
      const int ch = co0 + chl;
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc[2 * q][J][e];
        v[4 + e] = acc[2 * q + 1][J][e];
      }
      if (flags & EPI_PRE_RELU) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      if (flags & EPI_AFFINE) {
        const f32x4 m0 = *reinterpret_cast<const f32x4*>(tab + ch);
        const f32x4 m1 = *reinterpret_cast<const f32x4*>(tab + ch + 4);
        const f32x4 i0 = *reinterpret_cast<const f32x4*>(tab + p.coutp + ch);
        const f32x4 i1 = *reinterpret_cast<const f32x4*>(tab + p.coutp + ch + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = (v[e] - m0[e]) * i0[e];
          v[4 + e] = (v[4 + e] - m1[e]) * i1[e];
        }
      }
      if (RES && rl && ch < p.ysplit) {   // the dual-destination part has none
        const int row = wn * 16 + col;
        const bf16x8 r8 = *reinterpret_cast<const bf16x8*>(
            rl + row * 512 + ((((chl >> 3) ^ (row & 15))) << 4));
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
        dst = &g_gw_sink[lane];
      if (DBG & 64) dst = &g_gw_sink[lane];
      if (DBG & 32) gw_st16_nt(dst, __builtin_bit_cast(u32x4, o));
      else if (!(DBG & 4)) gw_st16(dst, __builtin_bit_cast(u32x4, o));
    }
  };

  int c_tile = 0, c_k = 0;
  int st1 = 0, st2 = 0, st3 = 0;   // stores issued in steps s-1, s-2, s-3
  for (int s = 0; s < S; ++s) {
    // operands of step s landed (this wave's DMA); younger: steps s+1, s+2's
    // DMA and the stores of the last three steps (issued after step s's DMA)
    gw_wait_vm(2 * NLw + st1 + st2 + st3);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // the next DMA goes into the slot every wave released at this barrier, as
    // early as possible (measured: spreading its pieces between the MFMA row
    // blocks is 6 % slower -- the stream is latency-bound, not issue-bound)
    issue((s + 3) & 3);
    __builtin_amdgcn_sched_barrier(0);
    const int lid = t_first + c_tile * t_step;
    const int co0 = (lid % cblocks) * BN;
    const int px0 = (lid / cblocks) * GW_BM;
    const char* L = smem + (s & 3) * GW_SLOT;
    int nst = 0;
    if (c_k < KT && (DBG & 1)) {
      if (!RES && c_k == KT - 1) nst = (DBG & 4) ? 0 : 4 * NQ;
    } else if (c_k < KT) {
      // every fragment read of the step is issued before the first MFMA, so the
      // LDS latency is exposed once per step (counted lgkmcnt waits follow the
      // issue order), not once per MFMA group
      bf16x8 a[NI], b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const bf16x8*>(L + offb + j * 1024);
#pragma unroll
      for (int i = 0; i < NI; ++i) a[i] = *reinterpret_cast<const bf16x8*>(L + offa + i * 1024);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma_step(a[i], b[j], acc[i][j]);
      if (!RES && c_k == KT - 1) {
        epi(std::integral_constant<int, 0>{}, co0, px0, nullptr);
        epi(std::integral_constant<int, 1>{}, co0, px0, nullptr);
        epi(std::integral_constant<int, 2>{}, co0, px0, nullptr);
        epi(std::integral_constant<int, 3>{}, co0, px0, nullptr);
        nst = (DBG & 4) ? 0 : 4 * NQ;
      }
    } else if (RES) {
      const int ph = c_k - KT;
      if (ph == 0) epi(std::integral_constant<int, 0>{}, co0, px0, L);
      else if (ph == 1) epi(std::integral_constant<int, 1>{}, co0, px0, L);
      else if (ph == 2) epi(std::integral_constant<int, 2>{}, co0, px0, L);
      else epi(std::integral_constant<int, 3>{}, co0, px0, L);
      nst = (DBG & 4) ? 0 : NQ;
    }
    st3 = st2;
    st2 = st1;
    st1 = nst;
    if (c_k + 1 == SPT) {
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      c_k = 0;
      ++c_tile;
    } else {
      ++c_k;
    }
  }
  // drain: the trailing (never consumed) DMA must land before the workgroup
  // releases its LDS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ----------------------------------------------------------------------------
// Wave-specialised variant: the same tiles, ring, K order and epilogue, with
// the operand DMA moved to 4 loader waves (waves 8..11) so the 8 compute waves
// never issue or wait on a global_load_lds.  In gemm1x1_wide every wave issues
// its share of a K-step's DMA and then runs its MFMAs, and on these L2-fed
// streams the two add (DESIGN.md "What bounds the DMA-fed kernels"); here a
// loader wave only waits for its own pieces before the step's barrier.
// 12 waves (3 per SIMD) cap the VGPRs at 168.  Bitwise equal to gemm1x1_wide.
constexpr int GS_NT = 768;
constexpr int GS_NL = 4;   // loader waves

// BM = pixels per tile: 256, or 192 for the 256-wide tiles (their compute waves
// then hold 96 accumulators and fit the cap; the residual takes 3 phases)
// DBG (diagnostics, VOXEMB_GEMM_VAR 21/22): 1 = compute waves skip fragment
// reads and MFMAs (stores kept), 2 = loaders issue no DMA, 8 = loaders skip
// the weight pieces (operand + residual DMA only), 64 = no output stores,
// 128 = loaders skip the residual pieces; results garbage.  Same results, other
// policies: 256 / 512 = nt / sc1 output stores, 1024 / 2048 = nt residual /
// activation DMA (VOXEMB_GEMM_VAR 33 / 34 / 35 / 36)
// MODE (operand variants; 0 = the Res2Net 1x1s):
//   GS_PRO : BN + ReLU prologue on the B operand, relu((x - m[k]) * inv[k])
//            rounded to bf16, as gemm1x1_pipe<.., PRO> (DPN bn_relu_conv,
//            dpn_model.py:40-45), applied in LDS by the loader waves to the
//            pieces they loaded; channels k >= Cin of a padded K get m = inv = 0
//   GS_TAPS: 1-D dilated conv along H (W = 1, the TDNN layers,
//            tdnn_model.py:24-30): K = taps x cinp, k-step -> (tap, channel
//            chunk), B row of pixel (n, h) at tap t = input row h + t dh - ph of
//            the same utterance, a zero row outside it (SAME padding)
constexpr int GS_PRO = 1, GS_TAPS = 2;
// KSUB = 32-deep k-steps per ring slot and barrier: 1 (4 slots of 32 KB,
// three in flight), or 2 for the 128-pixel tiles of the few-tile launches
// (TDNN): 3 slots of 2 x (BN + BM) x 64 B, half the barrier-separated steps
template <int BN, bool RES, int BM = GW_BM, int DBG = 0, int MODE = 0, int KSUB = 1>
__global__ __launch_bounds__(GS_NT) void gemm1x1_ws(ConvParams p) {
  constexpr bool PRO = (MODE & GS_PRO) != 0, TAPS = (MODE & GS_TAPS) != 0;
  static_assert(!(PRO && TAPS), "one operand variant");
  static_assert(KSUB == 1 || (KSUB == 2 && !PRO), "two k-steps per slot: plain or taps operands");
  constexpr int SUBB = (BN + BM) * 64;                    // one k-step's operands
  constexpr int SLOTB = KSUB == 1 ? GW_SLOT : KSUB * SUBB;
  // ring slots: 4 of 32 KB at one k-step per slot, 3 at two (the 128-pixel tiles;
  // 64-deep steps on the 448-row tiles fit only 2 slots, one step in flight, and
  // measured 2 % slower: DESIGN.md, Round 5)
  constexpr int NSTR = KSUB == 1 ? GW_NST : 3;
  static_assert(NSTR * SLOTB <= 147456, "ring slots");
  constexpr int NI = BN / 32;
  constexpr int NQ = NI / 2;
  constexpr int NJ = BM / 64;                // 16-pixel columns per wave
  constexpr int GRP = (BN + BM) / 16;        // 1-KB DMA groups per operand step
  constexpr int NLL = GRP / GS_NL;           // per loader wave
  constexpr int NR = RES ? NJ : 0;           // residual phases (64 pixels x 256 couts each)
  constexpr int NLR = 32 / GS_NL;            // residual pieces per loader wave
  static_assert(GRP % GS_NL == 0, "groups per loader");
  static_assert(BN % 64 == 0, "weight pieces are the first BN/64 of a loader");
  // residual phases carry 256 couts; the 320-wide tile (DPN68's 288-cout
  // stage-3 1x1c, one cout block) takes its residual from those 256 only
  // (the host checks ysplit <= 256 and a single cout block)
  static_assert(!RES || BN == 256 || BN == 320, "residual phases: 256 couts");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool loader = wave >= 8;
  const int lw = wave - 8;
  const int wm = (wave >> 2) & 1, wn = wave & 3;
  const int col = lane & 15, g = lane >> 4;
  const int M = p.N * p.Ho * p.Wo;
  const int HoWo = p.Ho * p.Wo;
  const int KT = p.kp / 32;
  const int KTS = KT / KSUB;          // ring steps of the K loop (the host checks KT % KSUB == 0)
  const int SPT = KTS + NR;
  const int cblocks = p.coutp / BN;
  const int T = ((M + BM - 1) / BM) * cblocks;
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
  const int S = ntiles * SPT;

  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(p.x);
  const bf16_t* __restrict__ Wt = reinterpret_cast<const bf16_t*>(p.w);
  const bf16_t* __restrict__ R = reinterpret_cast<const bf16_t*>(p.res);
  bf16_t* __restrict__ Y = reinterpret_cast<bf16_t*>(p.y);
  bf16_t* __restrict__ Y2 = reinterpret_cast<bf16_t*>(p.y2);
  const int flags = p.flags;
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;

  float* tab = reinterpret_cast<float*>(smem + NSTR * SLOTB);
  if (flags & EPI_AFFINE) {
    for (int k = tid; k < p.coutp; k += GS_NT) {
      tab[k] = k < p.Cout ? p.mean[k] : 0.f;
      tab[p.coutp + k] = k < p.Cout ? p.inv[k] : 0.f;
    }
  }
  // prologue table [kp] means, [kp] inverses (zero past Cin: padded K reads
  // finite neighbouring channels, relu((x - 0) * 0) = 0)
  float* ptab = tab + 2 * p.coutp;
  if constexpr (PRO) {
    for (int k = tid; k < p.kp; k += GS_NT) {
      ptab[k] = k < p.Cin ? p.in_mean[k] : 0.f;
      ptab[p.kp + k] = k < p.Cin ? p.in_inv[k] : 0.f;
    }
  }
  __syncthreads();

  // (diagnostics: DBG 16 / 32 = static priority 1 for the loader / compute waves)
  if ((DBG & 16) && loader) __builtin_amdgcn_s_setprio(1);
  if ((DBG & 32) && !loader) __builtin_amdgcn_s_setprio(1);
  if (loader) {
    // ---- loader waves: groups gi = lw + 4 i of every step
    const bf16_t* src[NLL];
    // weight pieces (i < BN/64: groups gi < BN/16) from the re-blocked copy when
    // present: one contiguous 1-KB block per (16 rows, k-step), already in LDS order
    const bf16_t* __restrict__ Wb = reinterpret_cast<const bf16_t*>(p.wblk);
    const bool blk = Wb != nullptr && !(DBG & 4);
    const int wstep = blk ? 512 : 32;   // elements per k-step of a weight piece
    int l_tile = 0, l_k = 0, l_co0 = 0, l_px0 = 0;
    int tho[NLL];   // GS_TAPS: the B row's time index (its utterance base is in src)
    int thn[NLL];   // GS_TAPS: its utterance's valid rows (ragged batches; H otherwise)
    const bf16_t* zero = reinterpret_cast<const bf16_t*>(g_gw_zero);
    auto set_load_tile = [&](int tj) {
      const int lid = t_first + tj * t_step;
      l_co0 = (lid % cblocks) * BN;
      l_px0 = (lid / cblocks) * BM;
#pragma unroll
      for (int i = 0; i < NLL; ++i) {
        const int gi = lw + GS_NL * i;
        // DBG 4 (timing only): 8 rows x 128 B per piece instead of 16 x 64 B
        const int row = (DBG & 4) ? 16 * gi + 2 * (lane >> 3) : 16 * gi + (lane >> 2);
        const int c = (DBG & 4) ? (lane & 7) : ((lane & 3) ^ gw_swz(row));
        if (row < BN && blk) {
          src[i] = Wb + ((size_t)((l_co0 >> 4) + gi) * KT) * 512 + lane * 8;
        } else if (row < BN) {
          src[i] = Wt + (size_t)(l_co0 + row) * p.kp + c * 8;
        } else {
          const int pix = min(l_px0 + row - BN, M - 1);
          const int n = pix / HoWo, rr = pix - n * HoWo;
          const int ho = rr / p.Wo, wo = rr - ho * p.Wo;
          if constexpr (TAPS) {
            src[i] = X + (size_t)n * p.H * p.ldx + c * 8;   // W = 1: row h at h * ldx
            tho[i] = ho;
            thn[i] = valid_rows(p.vlen, p.vsh, n, p.H);
          } else {
            src[i] = X + (((size_t)n * p.H + ho * p.sh) * p.W + wo * p.sw) * p.ldx + c * 8;
          }
        }
      }
    };
    // returns the pieces issued (an operand step NLL, a residual phase NLR)
    // GS_PRO: the k-step each ring slot was filled with (16-bit fields, 0xFFFF =
    // a residual phase), for the prologue pass below
    uint64_t kinfo = ~0ull;
    auto issue = [&](int slot) -> int {
      int n = 0;
      if constexpr (PRO) {
        const uint64_t v = l_k < KTS ? (uint64_t)l_k : 0xFFFFull;
        kinfo = (kinfo & ~(0xFFFFull << (16 * slot))) | (v << (16 * slot));
      }
      if (l_k < KTS) {
#pragma unroll
        for (int u = 0; u < KSUB; ++u) {
          const int kk = l_k * KSUB + u;   // the k-step of sub-slot u
          // GS_TAPS: this k-step's tap and channel chunk (wave-uniform)
          const int tap = TAPS ? (32 * kk) / p.cinp : 0;
          const int ci0 = TAPS ? 32 * kk - tap * p.cinp : 0;
          const int sh_t = TAPS ? tap * p.dh - p.ph : 0;
#pragma unroll
          for (int i = 0; i < NLL; ++i) {
            const int gi = lw + GS_NL * i;
            const int kst = i < BN / 64 ? wstep : 32;   // gi < BN/16 <=> i < BN/64
            const bf16_t* a = src[i] + kk * kst;
            if (TAPS && i >= BN / 64) {
              const int hi = tho[i] + sh_t;
              a = (hi >= 0 && hi < thn[i]) ? src[i] + (size_t)hi * p.ldx + ci0 : zero;
            }
            if ((DBG & 2048) && i >= BN / 64)   // (diagnostics: activation pieces nt)
              gw_glds16_nt(a, lds0 + (uint32_t)slot * SLOTB + (uint32_t)(u * SUBB) + (uint32_t)gi * 1024u);
            else if (!(DBG & 2) && !((DBG & 8) && i < BN / 64))
              gw_glds16(a, lds0 + (uint32_t)slot * SLOTB + (uint32_t)(u * SUBB) + (uint32_t)gi * 1024u);
          }
        }
        n = KSUB * ((DBG & 2) ? 0 : (DBG & 8) ? NLL - BN / 64 : NLL);
      } else if (RES) {
        // residual phase ph: slot row r (512 B) = pixel l_px0 + (BM/4) (r / 16) + 16 ph + r % 16
        const int ph = l_k - KTS;
#pragma unroll
        for (int i = 0; i < NLR; ++i) {
          const int gi = lw + GS_NL * i;
          const int row = 2 * gi + (lane >> 5);
          const int c = (lane & 31) ^ (row & 15);
          const int pix = min(l_px0 + (BM / 4) * (gi >> 3) + 16 * ph + (row & 15), M - 1);
          if (DBG & 1024)   // (diagnostics: residual pieces nt)
            gw_glds16_nt(R + (size_t)pix * p.ldr + l_co0 + c * 8,
                         lds0 + (uint32_t)slot * SLOTB + (uint32_t)gi * 1024u);
          else if (!(DBG & 2) && !(DBG & 128))
            gw_glds16(R + (size_t)pix * p.ldr + l_co0 + c * 8,
                      lds0 + (uint32_t)slot * SLOTB + (uint32_t)gi * 1024u);
        }
        n = ((DBG & 2) || (DBG & 128)) ? 0 : NLR;
      }
      if (l_k + 1 < SPT) {
        ++l_k;
      } else if (l_tile + 1 < ntiles) {
        ++l_tile;
        l_k = 0;
        set_load_tile(l_tile);
      }
      return n;
    };
    set_load_tile(0);
    issue(0);
    // pieces of the NSTR - 2 steps after the awaited one (n1 unused with 3 slots)
    int n1 = NSTR == 4 ? issue(1) : 0;
    int n2 = issue(NSTR - 2);
    // GS_PRO: this lane's K chunk within a k-step (the DMA swizzle of an
    // activation row depends only on the lane: row = 16 gi + lane / 4)
    const int pc = (lane & 3) ^ ((4 - ((lane >> 4) & 3)) & 3);
    for (int s = 0; s < S; ++s) {
      gw_wait_vm(n1 + n2);   // step s landed; steps s+1, s+2 in flight
      if constexpr (PRO) {
        // the BN + ReLU prologue, applied once to the activation pieces this
        // wave loaded, in LDS before the barrier: the compute waves read
        // finished B fragments (each used to transform them itself, twice
        // over -- both cout halves read the same fragment -- and that VALU
        // work bound the DPN68 prologue GEMMs)
        const int slot = s & 3;
        const int ks = (int)((kinfo >> (16 * slot)) & 0xFFFFull);
        if (ks != 0xFFFF) {
          const int kb = 32 * ks + 8 * pc;
          const f32x4 m0 = *reinterpret_cast<const f32x4*>(ptab + kb);
          const f32x4 m1 = *reinterpret_cast<const f32x4*>(ptab + kb + 4);
          const f32x4 i0 = *reinterpret_cast<const f32x4*>(ptab + p.kp + kb);
          const f32x4 i1 = *reinterpret_cast<const f32x4*>(ptab + p.kp + kb + 4);
#pragma unroll
          for (int i = BN / 64; i < NLL; ++i) {
            const int gi = lw + GS_NL * i;
            bf16x8* q = reinterpret_cast<bf16x8*>(smem + slot * SLOTB + gi * 1024 + lane * 16);
            bf16x8 b = *q;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              b[e] = (bf16_t)fmaxf(((float)b[e] - m0[e]) * i0[e], 0.f);
              b[4 + e] = (bf16_t)fmaxf(((float)b[4 + e] - m1[e]) * i1[e], 0.f);
            }
            *q = b;
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
      }
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      const int n3 = issue((s + NSTR - 1) % NSTR);
      n1 = NSTR == 4 ? n2 : 0;
      n2 = n3;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }

  // ---- compute waves (2 cout halves x 4 pixel quarters), as gemm1x1_wide
  f32x4 acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int cs = (g ^ gw_swz(col)) << 4;
  const int offa = (wm * (BN / 2) + col) * 64 + cs;
  const int offb = (BN + wn * (BM / 4) + col) * 64 + cs;

  // epilogue of one 16-pixel column J: FL = the EPI flags as a compile-time set for the
  // common ones (-1 = read p.flags).  Packed pairs and a hoisted row address: the
  // per-column VALU work, not the MFMAs, filled most of the residual phases.
  auto epi_f = [&](auto jc, auto flc, int co0, int px0, const char* rl) {
    constexpr int J = decltype(jc)::value;
    constexpr int FL = decltype(flc)::value;
    const int fl = FL >= 0 ? FL : flags;
    const int pix = px0 + wn * (BM / 4) + 16 * J + col;
    const bool pok = pix < M;
    const int pixc = pok ? pix : M - 1;
    bf16_t* const yrow = Y + (size_t)pixc * p.ldy;
    const bool split = p.ysplit < p.Cout;   // two destinations (DPN dense channels)
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int chl = wm * (BN / 2) + 32 * q + 8 * g;
      const int ch = co0 + chl;
      f32x2 v[4];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        v[e] = f32x2{acc[2 * q][J][2 * e], acc[2 * q][J][2 * e + 1]};
        v[2 + e] = f32x2{acc[2 * q + 1][J][2 * e], acc[2 * q + 1][J][2 * e + 1]};
      }
      if (fl & EPI_PRE_RELU) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = f32x2{gw_relu(v[e].x), gw_relu(v[e].y)};
      }
      if (fl & EPI_AFFINE) {
        // BN values re-read per column: not kept live across the 4 columns
        int tch = ch;
        asm volatile("" : "+v"(tch));
        const f32x4 m0 = *reinterpret_cast<const f32x4*>(tab + tch);
        const f32x4 m1 = *reinterpret_cast<const f32x4*>(tab + tch + 4);
        const f32x4 i0 = *reinterpret_cast<const f32x4*>(tab + p.coutp + tch);
        const f32x4 i1 = *reinterpret_cast<const f32x4*>(tab + p.coutp + tch + 4);
        v[0] = gw_pk_sub(v[0], f32x2{m0[0], m0[1]}) * f32x2{i0[0], i0[1]};
        v[1] = gw_pk_sub(v[1], f32x2{m0[2], m0[3]}) * f32x2{i0[2], i0[3]};
        v[2] = gw_pk_sub(v[2], f32x2{m1[0], m1[1]}) * f32x2{i1[0], i1[1]};
        v[3] = gw_pk_sub(v[3], f32x2{m1[2], m1[3]}) * f32x2{i1[2], i1[3]};
      }
      if (RES && rl && (!split || ch < p.ysplit)) {
        const int row = wn * 16 + col;
        const u32x4 r4 = *reinterpret_cast<const u32x4*>(
            rl + row * 512 + ((((chl >> 3) ^ (row & 15))) << 4));
#pragma unroll
        for (int e = 0; e < 4; ++e)
          v[e] += f32x2{__builtin_bit_cast(float, r4[e] << 16), __builtin_bit_cast(float, r4[e] & 0xFFFF0000u)};
      }
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[2 * e] = (bf16_t)v[e].x;
        o[2 * e + 1] = (bf16_t)v[e].y;
      }
      // relu(bf16(x)) == bf16(relu(x)) bit for bit (device_common.h)
      if (fl & EPI_RELU) o = relu_bf16(o);
      void* dst;
      if (!split) {
        dst = (ch < p.Cout && pok) ? (void*)(yrow + ch) : (void*)&g_gw_sink[lane];
      } else if (ch < p.Cout && pok) {
        dst = ch < p.ysplit ? (void*)(yrow + ch)
                            : (void*)(Y2 + (size_t)pix * p.ldy2 + (ch - p.ysplit));
      } else {
        dst = &g_gw_sink[lane];
      }
      if (DBG & 64) asm volatile("" ::"v"(o), "v"(dst));   // (diagnostics: no output stores)
      else if (DBG & 256) gw_st16_nt(dst, __builtin_bit_cast(u32x4, o));    // (nt stores)
      else if (DBG & 512) gw_st16_sc1(dst, __builtin_bit_cast(u32x4, o));   // (sc1 stores)
      else gw_st16(dst, __builtin_bit_cast(u32x4, o));
    }
  };
  // the flag sets of the Res2Net / TDNN / DPN 1x1s as compile-time epilogues
  auto epi = [&](auto jc, int co0, int px0, const char* rl) {
    using IC10 = std::integral_constant<int, EPI_AFFINE | EPI_RELU>;
    using IC14 = std::integral_constant<int, EPI_AFFINE | EPI_RES | EPI_RELU>;
    using IC2 = std::integral_constant<int, EPI_AFFINE>;
    using IC3 = std::integral_constant<int, EPI_PRE_RELU | EPI_AFFINE>;
    const int f = flags & (EPI_PRE_RELU | EPI_AFFINE | EPI_RES | EPI_RELU);
    if (RES && f == (EPI_AFFINE | EPI_RES | EPI_RELU)) epi_f(jc, IC14{}, co0, px0, rl);
    else if (!RES && f == (EPI_AFFINE | EPI_RELU)) epi_f(jc, IC10{}, co0, px0, rl);
    else if (!RES && f == EPI_AFFINE) epi_f(jc, IC2{}, co0, px0, rl);
    else if (!RES && f == (EPI_PRE_RELU | EPI_AFFINE)) epi_f(jc, IC3{}, co0, px0, rl);
    else epi_f(jc, std::integral_constant<int, -1>{}, co0, px0, rl);
  };

  int c_tile = 0, c_k = 0;
  for (int s = 0; s < S; ++s) {
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const int lid = t_first + c_tile * t_step;
    const int co0 = (lid % cblocks) * BN;
    const int px0 = (lid / cblocks) * BM;
    const char* L = smem + (s % NSTR) * SLOTB;
    if (c_k < KTS && (DBG & 1)) {
      if (!RES && c_k == KTS - 1) {
        epi(std::integral_constant<int, 0>{}, co0, px0, nullptr);
        epi(std::integral_constant<int, 1>{}, co0, px0, nullptr);
        if constexpr (NJ > 2) epi(std::integral_constant<int, 2>{}, co0, px0, nullptr);
        if constexpr (NJ > 3) epi(std::integral_constant<int, 3>{}, co0, px0, nullptr);
      }
    } else if (c_k < KTS) {
#pragma unroll
      for (int u = 0; u < KSUB; ++u) {
        const char* Lu = L + u * SUBB;
        // B fragments for the k-step, A fragments two cout blocks ahead (register budget)
        bf16x8 a[NI], b[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) b[j] = *reinterpret_cast<const bf16x8*>(Lu + offb + j * 1024);
        // (GS_PRO: the loader waves applied the prologue to these fragments)
        a[0] = *reinterpret_cast<const bf16x8*>(Lu + offa);
        a[1] = *reinterpret_cast<const bf16x8*>(Lu + offa + 1024);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          if (i + 2 < NI) a[i + 2] = *reinterpret_cast<const bf16x8*>(Lu + offa + (i + 2) * 1024);
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] = mfma_step(a[i], b[j], acc[i][j]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (!RES && c_k == KTS - 1) {
        epi(std::integral_constant<int, 0>{}, co0, px0, nullptr);
        epi(std::integral_constant<int, 1>{}, co0, px0, nullptr);
        if constexpr (NJ > 2) epi(std::integral_constant<int, 2>{}, co0, px0, nullptr);
        if constexpr (NJ > 3) epi(std::integral_constant<int, 3>{}, co0, px0, nullptr);
      }
    } else if (RES) {
      const int ph = c_k - KTS;
      if (ph == 0) epi(std::integral_constant<int, 0>{}, co0, px0, L);
      else if (ph == 1) epi(std::integral_constant<int, 1>{}, co0, px0, L);
      else if (ph == 2) {
        if constexpr (NJ > 2) epi(std::integral_constant<int, 2>{}, co0, px0, L);
      } else {
        if constexpr (NJ > 3) epi(std::integral_constant<int, 3>{}, co0, px0, L);
      }
    }
    if (c_k + 1 == SPT) {
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      c_k = 0;
      ++c_tile;
    } else {
      ++c_k;
    }
  }
}

// BN of the wide tile for this conv, or 0 if gemm1x1_wide does not apply
int gemm_wide_bn(const ConvParams& p) {
  if (p.kp % 32 || p.kp / 32 < 3 || p.Cout % 8) return 0;
  if (p.in_mean && (!p.in_inv || (p.kh != 1 || p.kw != 1))) return 0;
  if (p.kh > 1 && (p.in_mean || p.kw != 1 || p.W != 1 || p.Wo != 1 || p.sh != 1 || p.cinp % 32 ||
                   p.kp != p.kh * p.cinp || p.Ho != p.H))
    return 0;
  const int M = p.N * p.Ho * p.Wo;
  int bn = 0;
  if (p.Cout % 256 == 0) bn = 256;
  else if (p.Cout % 192 == 0 && !(p.flags & EPI_RES)) bn = 192;
  // DPN68 stage-3 1x1c: 256 residual couts + 32 dense ones in one 320-wide
  // block (two 256-wide blocks re-read the activations for 32 couts)
  else if (p.in_mean && p.Cout > 256 && p.Cout <= 320 && (!(p.flags & EPI_RES) || p.ysplit <= 256))
    bn = 320;
  // DPN prologue convs: partial last cout tile (the weights hold 256-row multiples)
  else if (p.in_mean && p.Cout >= 128) bn = 256;
  if (!bn || p.Cout > 2048) return 0;
  if ((p.flags & EPI_RES) && (!p.res || p.ldr % 8)) return 0;
  const int T = ((M + GW_BM - 1) / GW_BM) * ((p.Cout + bn - 1) / bn);
  return (T >= 8 || p.any_m) ? bn : 0;
}

template <int DBG>
static void launch_wide_t(const ConvParams& p, int bn, int G, size_t lds, hipStream_t s) {
  if (bn == 192)
    hipLaunchKernelGGL((gemm1x1_wide<192, false, DBG>), dim3(G), dim3(GW_NT), lds, s, p);
  else if (p.flags & EPI_RES)
    hipLaunchKernelGGL((gemm1x1_wide<256, true, DBG>), dim3(G), dim3(GW_NT), lds, s, p);
  else
    hipLaunchKernelGGL((gemm1x1_wide<256, false, DBG>), dim3(G), dim3(GW_NT), lds, s, p);
}

// pixels per tile: the default (192 for 256-wide tiles, 256 for 192-wide) or
// 128 when the launch has too few tiles to fill the chip -- per tile the DMA
// moves (BM + BN) rows per k-step, and ceil(tiles / CUs) rounds run in turn
static int ws_bm(int M, int cblocks, int bn, int num_cu) {
  const int big = bn == 256 ? 192 : 256;
  auto cost = [&](int bm) {
    const long t = (long)((M + bm - 1) / bm) * cblocks;
    return ((t + num_cu - 1) / num_cu) * (long)(bm + bn);
  };
  return cost(128) < cost(big) ? 128 : big;
}

// pixels per tile launch_gemm_wide picks for this conv (plan descriptions, tests)
int gemm_wide_bm(const ConvParams& p0, int num_cu) {
  const int bn = gemm_wide_bn(p0);
  if (!bn) return 0;
  const int coutp = (p0.Cout + bn - 1) / bn * bn;
  return bn == 320 ? 128 : ws_bm(p0.N * p0.Ho * p0.Wo, coutp / bn, bn, num_cu);
}

hipError_t launch_gemm_wide(const ConvParams& p0, int num_cu, int variant, hipStream_t s, int ksub_on) {
  const int bn = gemm_wide_bn(p0);
  if (!bn) return hipErrorInvalidValue;
  ConvParams p = p0;
  // whole BN blocks (the weights hold roundup256(Cout) rows; extra couts are masked)
  p.coutp = (p.Cout + bn - 1) / bn * bn;
  const int M = p.N * p.Ho * p.Wo;
  const int T = ((M + GW_BM - 1) / GW_BM) * (p.coutp / bn);
  int G = num_cu < T ? num_cu : T;
  G = G >= 8 ? G / 8 * 8 : G;   // small launches (any_m) keep their few tiles
  const size_t lds = GW_NST * GW_SLOT + 8 * (size_t)p.coutp + (p.in_mean ? 8 * (size_t)p.kp : 0);
  // (the 320-wide tile holds 80 accumulators per compute wave at 128 pixels)
  int bm = bn == 320 ? 128 : ws_bm(M, p.coutp / bn, bn, num_cu);
#ifdef VOX_DIAG
  // (diagnostic VOXEMB_GEMM_VAR 37: 128-pixel tiles, one k-step per slot, on
  // every launch -- the same results; tests the per-CU intake model, whose
  // operand bytes per output grow by (128 + BN) / (BM + BN) * BM / 128)
  if (variant == 37 && bn != 320) bm = 128;
#endif
  auto grid_for = [&](int bmx) {
    const int t = ((M + bmx - 1) / bmx) * (p.coutp / bn);
    int g = num_cu < t ? num_cu : t;
    return g >= 8 ? g / 8 * 8 : g;
  };
  const int Gb = grid_for(bm);
  // two k-steps per ring slot on the 128-pixel tiles (few-tile launches) when
  // the three 2 x (BN + 128) x 64 B slots fit
  const size_t lds2 = 3 * 2 * (size_t)(bn + 128) * 64 + 8 * (size_t)p.coutp;
  const bool two = ksub_on && variant != 37 && bm == 128 && bn <= 256 && !p.in_mean &&
                   (p.kp / 32) % 2 == 0 && lds2 <= 163840;
  if (p.in_mean || p.kh > 1) {
    // operand variants (GS_PRO / GS_TAPS): wave-specialised only
#define WS_L(BN_, RES_, BM_, MODE_) \
  hipLaunchKernelGGL((gemm1x1_ws<BN_, RES_, BM_, 0, MODE_>), dim3(Gb), dim3(GS_NT), lds, s, p)
    if (p.in_mean) {
      if (bn == 320) {
        if (p.flags & EPI_RES) WS_L(320, true, 128, GS_PRO); else WS_L(320, false, 128, GS_PRO);
      } else if (p.flags & EPI_RES) {
        if (bm == 128) WS_L(256, true, 128, GS_PRO); else WS_L(256, true, 192, GS_PRO);
      } else if (bn == 192) {
        if (bm == 128) WS_L(192, false, 128, GS_PRO); else WS_L(192, false, 256, GS_PRO);
      } else {
        if (bm == 128) WS_L(256, false, 128, GS_PRO); else WS_L(256, false, 192, GS_PRO);
      }
    } else if (two) {
      if (bn == 192)
        hipLaunchKernelGGL((gemm1x1_ws<192, false, 128, 0, GS_TAPS, 2>), dim3(Gb), dim3(GS_NT), lds2, s, p);
      else
        hipLaunchKernelGGL((gemm1x1_ws<256, false, 128, 0, GS_TAPS, 2>), dim3(Gb), dim3(GS_NT), lds2, s, p);
    } else {
      if (bn == 192) {
        if (bm == 128) WS_L(192, false, 128, GS_TAPS); else WS_L(192, false, 256, GS_TAPS);
      } else {
        if (bm == 128) WS_L(256, false, 128, GS_TAPS); else WS_L(256, false, 192, GS_TAPS);
      }
    }
#undef WS_L
    return hipGetLastError();
  }
  // wave-specialised by default (4-11 % faster per launch; the 256-wide tiles
  // with 192 pixels so the compute waves fit the 12-wave register cap);
  // VOXEMB_GEMM_VAR=-1 selects gemm1x1_wide
  if (variant == 0) variant = 1;
  if (variant == -1) variant = 0;
  if (variant == 1 || (variant >= 21 && variant <= 37)) {   // wave-specialised
    auto go = [&](auto dbgc) {
      constexpr int D = decltype(dbgc)::value;
      if (two && bn == 192) {
        hipLaunchKernelGGL((gemm1x1_ws<192, false, 128, 0, 0, 2>), dim3(Gb), dim3(GS_NT), lds2, s, p);
      } else if (two && (p.flags & EPI_RES)) {
        hipLaunchKernelGGL((gemm1x1_ws<256, true, 128, 0, 0, 2>), dim3(Gb), dim3(GS_NT), lds2, s, p);
      } else if (two) {
        hipLaunchKernelGGL((gemm1x1_ws<256, false, 128, 0, 0, 2>), dim3(Gb), dim3(GS_NT), lds2, s, p);
      } else if (bm == 128) {
        // too few tiles to fill the chip at the default size (small batches, TDNN)
        if (bn == 192)
          hipLaunchKernelGGL((gemm1x1_ws<192, false, 128, 0>), dim3(Gb), dim3(GS_NT), lds, s, p);
        else if (p.flags & EPI_RES)
          hipLaunchKernelGGL((gemm1x1_ws<256, true, 128, 0>), dim3(Gb), dim3(GS_NT), lds, s, p);
        else
          hipLaunchKernelGGL((gemm1x1_ws<256, false, 128, 0>), dim3(Gb), dim3(GS_NT), lds, s, p);
      } else if (bn == 192) {
        hipLaunchKernelGGL((gemm1x1_ws<192, false, 256, D>), dim3(Gb), dim3(GS_NT), lds, s, p);
      } else {
        // 256-wide: 192-pixel tiles (their own tile count and grid)
        if (p.flags & EPI_RES)
          hipLaunchKernelGGL((gemm1x1_ws<256, true, 192, D>), dim3(Gb), dim3(GS_NT), lds, s, p);
        else
          hipLaunchKernelGGL((gemm1x1_ws<256, false, 192, D>), dim3(Gb), dim3(GS_NT), lds, s, p);
      }
    };
#ifdef VOX_DIAG
    if (variant == 21) go(std::integral_constant<int, 1>{});
    else if (variant == 22) go(std::integral_constant<int, 2>{});
    else if (variant == 25) go(std::integral_constant<int, 5>{});
    else if (variant == 24) go(std::integral_constant<int, 4>{});
    else if (variant == 28) go(std::integral_constant<int, 8>{});
    else if (variant == 29) go(std::integral_constant<int, 9>{});
    else if (variant == 30) go(std::integral_constant<int, 16>{});
    else if (variant == 31) go(std::integral_constant<int, 32>{});
    else if (variant == 26) go(std::integral_constant<int, 64>{});
    else if (variant == 27) go(std::integral_constant<int, 65>{});
    else if (variant == 23) go(std::integral_constant<int, 128>{});
    else if (variant == 33) go(std::integral_constant<int, 256>{});
    else if (variant == 34) go(std::integral_constant<int, 512>{});
    else if (variant == 35) go(std::integral_constant<int, 1024>{});
    else if (variant == 36) go(std::integral_constant<int, 2048>{});
    else
#endif
      go(std::integral_constant<int, 0>{});
    return hipGetLastError();
  }
  switch (variant) {   // 0 = the product kernel; 11..17 = diagnostics (DBG = variant - 10)
#ifdef VOX_DIAG
    case 11: launch_wide_t<1>(p, bn, G, lds, s); break;
    case 12: launch_wide_t<2>(p, bn, G, lds, s); break;
    case 14: launch_wide_t<4>(p, bn, G, lds, s); break;
    case 13: launch_wide_t<3>(p, bn, G, lds, s); break;
    case 16: launch_wide_t<6>(p, bn, G, lds, s); break;
    case 42: launch_wide_t<32>(p, bn, G, lds, s); break;
    case 74: launch_wide_t<64>(p, bn, G, lds, s); break;
    case 15: launch_wide_t<5>(p, bn, G, lds, s); break;
#endif
    default: launch_wide_t<0>(p, bn, G, lds, s); break;
  }
  return hipGetLastError();
}

}  // namespace vox

// K-split register-weight 3x3 conv for the w = 96 stride-1 Res2Net branches
// (res2net_pad_conv_bn_relu, res2net_model.py:53-75, layer 3): y_k =
// relu(bn(conv3x3(z_k))), and for k < S-1 the next branch's input
// z_{k+1} = x_{k+1} + y_k formed in place over x_{k+1}.
//
// conv3x3_rw (conv3r.hip) holds one 16-cout tile's weights per wave and feeds
// every v_mfma_f32_16x16x32_bf16 (16 cycles) a fresh 1-KB pixel fragment from
// LDS: 12 waves x 108 fragments per 128-pixel tile = 1.3 MB of LDS reads, the
// CU's whole LDS bandwidth at the MFMA rate, so the k-loop runs at the LDS
// (with bank conflicts) rather than the matrix pipe.  Here every wave uses
// v_mfma_f32_32x32x16_bf16 (32 cycles, 32 couts x 32 pixels x 16 k): the same
// 1-KB pixel fragment now feeds twice the MFMA work, halving the LDS reads per
// FLOP.  A 32-cout tile's full-K weights (216 VGPRs) do not fit the 12-wave
// register budget, so K is split in halves:
//
//   wave = (cout group cg of 32, K half kh, pixel half ph): weights
//   W[32 cg .. +32][432 kh .. +432] in 108 VGPRs; pixel groups 2 ph, 2 ph + 1
//   (32 pixels each) of the 128-pixel tile, two accumulators of 16 VGPRs.
//
// After the k-loop the two K halves of a (cg, ph) pair meet in LDS: each wave
// writes the partial sums of the pixel group its partner finishes (fp32, 4 KB)
// and adds the partner's partial of its own group, so every output is
// (half 0) + (half 1) in fp32 -- one fixed order, whatever wave finishes it.
//
// Window layout: pixel-major, 13 16-B units per pixel slot (12 chunks of 8
// channels + 1 pad unit).  The odd 208-B pitch gives 16 consecutive slots 16
// disjoint 4-bank sets, and a window DMA piece reads 192 contiguous bytes per
// pixel.  One zero slot between window rows serves as both rows' SAME padding
// column (SW = W + 1); its row breaks would put two lanes of a ds_read_b128
// lane group on one bank set, so lanes take their group's pixels in a
// permuted order (g_ks_perm).  Tiles are utterance-aligned (the padding is per
// utterance); the window is double-buffered so the next tile's rows stream in
// under this tile's MFMAs, and the y staging + deferred row-contiguous store
// pass are conv3x3_rw's.
// Not bitwise equal to conv3x3_pipe (K halves summed at the end, 16-deep MFMA
// k-steps): the per-layer bf16 oracle check holds it (tests/test_bf16_oracle.py)
// and tests/test_gpu_parity.py compares it with conv3x3_rw on the same input.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_common.h"
#include "kernels.h"

namespace vox {

namespace {
constexpr int KS_C = 96;               // Cin = Cout = branch width
constexpr int KS_TP = 128;             // pixels per tile (4 groups of 32)
constexpr int KS_NW = 12;              // 3 cout groups x 2 K halves x 2 pixel halves
constexpr int KS_NT = 64 * KS_NW;
constexpr int KS_SH = 9 * KS_C / 32;   // 27 k16-steps per K half (54 in all)
constexpr int KS_NCH = KS_C / 8;       // 12 chunks per pixel
constexpr int KS_PU = KS_NCH + 1;      // units per window slot (odd: conflict-free reads)
constexpr int KS_PB = KS_PU * 16;      // 208 B
constexpr int KS_XCH = KS_NW * 4096;   // partial-sum exchange: 4 KB per wave
#ifndef KS_STAGE
#define KS_STAGE 1                     // y / z stores staged through LDS (0: from registers)
#endif
#ifndef KS_PD
#define KS_PD 2                        // B fragments read ahead of their MFMA
#endif

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
// a - b on a pair (v_pk_add_f32, b negated: the rounding of two v_sub_f32)
__device__ __forceinline__ f32x2 ks_pk_sub(f32x2 a, f32x2 b) {
  f32x2 r;
  asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// two floats to a bf16 pair (round to nearest even, as a scalar conversion)
__device__ __forceinline__ unsigned ks_cvt_pk(f32x2 v) {
  unsigned r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(v[0]), "v"(v[1]));
  return r;
}

__device__ __forceinline__ void ks_glds16(const void* src, uint32_t lds) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds))
      : "memory");
}
// the trailing s_nop keeps the next instruction from overwriting the data
// registers before the store has read them
__device__ __forceinline__ void ks_st16(void* dst, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" : : "v"(dst), "v"(v) : "memory");
}
__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
}  // namespace

__device__ uint4 g_ks_zero[4] = {};
// diagnostics (libvoxemb_diag.so only): shader-clock stamps of workgroup 0 of
// the z-forming launches, [wave][tile < 16][stamp < 8] (tools/ks_trace.py)
__device__ unsigned long long g_ks_trace[KS_NW * 16 * 8];
__device__ uint4 g_ks_sink[64];   // destination of masked lanes' stores
// lane -> pixel of a 32-pixel group, [W = 20, 10][(first pixel % W) / (W / 5)][lane]
// (tools/ks_lane_perm.py): each pixel on the ds_read_b128 lane group that still lacks
// its 4-bank quad; the window's row breaks put two lanes of a group on one quad when
// pixel i sits on lane i (8 LDS cycles per fragment read instead of 5.6 for W = 20).
// The MFMA column of a lane is its output pixel in the B operand and the accumulator
// alike, so the permutation changes no arithmetic.
__device__ const unsigned char g_ks_perm[2][5][32] = {
    {  // W = 20
        {0, 5, 10, 15, 16, 20, 25, 30, 24, 29, 19, 23, 9, 14, 3, 8, 28, 18, 22, 27, 13, 2, 7, 12, 1, 6, 11, 31, 17, 21, 26, 4},
        {12, 1, 6, 11, 27, 16, 21, 26, 31, 20, 25, 30, 0, 5, 10, 15, 19, 24, 29, 18, 4, 9, 14, 3, 8, 13, 2, 7, 23, 28, 17, 22},
        {0, 8, 12, 2, 15, 23, 28, 17, 22, 16, 21, 26, 7, 1, 6, 11, 20, 25, 30, 19, 5, 10, 14, 4, 9, 13, 3, 31, 24, 29, 18, 27},
        {1, 0, 4, 8, 16, 15, 19, 24, 28, 18, 17, 22, 13, 3, 2, 7, 27, 21, 26, 20, 11, 6, 10, 5, 9, 14, 31, 30, 25, 29, 23, 12},
        {0, 1, 4, 9, 15, 16, 20, 24, 29, 28, 18, 23, 14, 13, 3, 7, 27, 17, 22, 26, 12, 2, 6, 11, 5, 10, 30, 31, 21, 25, 19, 8},
    },
    {  // W = 10
        {2, 1, 0, 14, 17, 16, 15, 29, 19, 23, 28, 18, 4, 9, 13, 3, 22, 27, 21, 26, 8, 12, 7, 11, 6, 10, 31, 30, 20, 25, 5, 24},
        {2, 1, 0, 12, 17, 16, 15, 27, 21, 26, 20, 25, 7, 11, 6, 10, 19, 24, 28, 18, 5, 9, 14, 4, 8, 31, 30, 29, 23, 13, 3, 22},
        {0, 2, 1, 10, 15, 16, 30, 25, 19, 24, 28, 18, 5, 9, 14, 4, 23, 27, 17, 22, 8, 13, 3, 7, 12, 6, 29, 31, 26, 21, 11, 20},
        {2, 1, 0, 8, 16, 15, 14, 23, 27, 17, 22, 26, 13, 3, 7, 12, 21, 25, 20, 24, 6, 11, 5, 10, 4, 31, 30, 29, 19, 9, 28, 18},
        {1, 0, 16, 6, 15, 14, 31, 21, 25, 20, 24, 19, 11, 5, 10, 4, 23, 28, 18, 22, 9, 13, 3, 8, 12, 2, 30, 29, 27, 17, 7, 26},
    },
};

template <int W>
struct KsCfg {
  static constexpr int SW = W + 1;                                // slots per window row
  static constexpr int RMAX = (W - 1 + KS_TP - 1) / W + 1 + 2;    // rows + halo a tile touches
  static constexpr int SLOTS = RMAX * SW + 1;                     // + the last row's right pad
  static constexpr int WPC = (SLOTS * KS_PU + 63) / 64;           // window DMA pieces
  static constexpr int WBUF = WPC * 1024;
  static constexpr int XZB = KS_TP * KS_C * 2;                    // x_{k+1} rows of a tile
  static constexpr int XPC = XZB / 1024;
  static constexpr int LDS = 2 * WBUF + KS_XCH + XZB + 2 * KS_C * 4;
  static_assert(XZB % 1024 == 0, "x pieces");
  // the next tile's window is issued at the first pass's k16-steps s % 6 == 3
  // (fill() in the kernel): one piece per wave at each, so every piece must
  // have a slot there or nwin no longer matches what was issued
  static_assert(WPC <= KS_NW * ((KS_SH - 4) / 6 + 1), "window fill schedule too short");
  static_assert(LDS <= 163840, "LDS");
};

#pragma clang fp contract(off)
template <int W, bool HAS_Z>
__global__ __launch_bounds__(KS_NT) void conv3x3_ks(ConvParams p) {
  using K = KsCfg<W>;
  constexpr int SW = K::SW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, h = lane >> 5;
  const int cg = wave % 3, kh = (wave / 3) & 1, ph = wave / 6;
  const int H = p.H, HW = p.H * W;
  const int tpu = (HW + KS_TP - 1) / KS_TP;  // tiles per utterance
  const int T = p.N * tpu;
  int t_first, t_step, ntiles;
  {
    const int G = gridDim.x;
    if ((G & 7) == 0) {
      // XCD x (blocks x, x+8, ...) owns a contiguous tile range
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

  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(p.x);
  const bf16_t* __restrict__ XZ = reinterpret_cast<const bf16_t*>(p.res);
  bf16_t* __restrict__ Y = reinterpret_cast<bf16_t*>(p.y);
  bf16_t* __restrict__ Z = reinterpret_cast<bf16_t*>(p.y2);
  const bf16_t* zero = reinterpret_cast<const bf16_t*>(g_ks_zero);
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  float* xch = reinterpret_cast<float*>(smem + 2 * K::WBUF);   // 4 KB per wave
  char* xzb = smem + 2 * K::WBUF + KS_XCH;                      // x_{k+1} rows of the tile
  float* bnm = reinterpret_cast<float*>(xzb + K::XZB);
  float* bni = bnm + KS_C;
  for (int c = tid; c < KS_C; c += KS_NT) {
    bnm[c] = p.mean[c];
    bni[c] = p.inv[c];
  }

  // A operand: cout row 32 cg + r32, k = 432 kh + 16 s + 8 h .. + 8
  bf16x8 wr[KS_SH];
  {
    const bf16_t* __restrict__ Wt = reinterpret_cast<const bf16_t*>(p.w);
    const bf16_t* wrow = Wt + (size_t)(32 * cg + r32) * (9 * KS_C) + 432 * kh + 8 * h;
#pragma unroll
    for (int s = 0; s < KS_SH; ++s) wr[s] = ld16(wrow + 16 * s);
  }

  // window piece q of tile tj into buffer b: units [64q, 64q + 64), unit u =
  // chunk u % 13 of slot u / 13 (chunk 12 = the pad unit)
  // hn: the utterance's valid rows (ragged batches; H otherwise): rows past
  // them are its SAME padding
  auto issue_piece = [&](int n, int r0w, int b, int q, int hn) __attribute__((always_inline)) {
    int u = lane;
    asm volatile("" : "+v"(u));
    u += 64 * q;
    const int x = u / KS_PU, c = u - x * KS_PU;
    const int rr = x / SW, sc = x - rr * SW;
    const int row = r0w + rr;
    const bf16_t* src = zero;
    if (c < KS_NCH && sc > 0 && rr < K::RMAX && row >= 0 && row < hn)
      src = X + ((size_t)n * HW + row * W + (sc - 1)) * p.ldx + c * 8;
    ks_glds16(src, lds0 + (uint32_t)b * K::WBUF + (uint32_t)q * 1024u);
  };
  auto issue_win = [&](int tj, int b) __attribute__((always_inline)) {
    const int id = t_first + tj * t_step;
    const int n = id / tpu, t = id - n * tpu;
    const int r0w = (t * KS_TP) / W - 1;   // image row of window row 0
    const int hn = p.vlen ? valid_rows(p.vlen, p.vsh, n, H) : H;
    for (int q = wave; q < K::WPC; q += KS_NW) issue_piece(n, r0w, b, q, hn);
  };

  // the tile's x_{k+1} pixel rows (192 B each) into LDS, linear
  auto issue_xz = [&](int tj) __attribute__((always_inline)) {
    const int id = t_first + tj * t_step;
    const int n = id / tpu, t = id - n * tpu;
    const int p0 = t * KS_TP;
#pragma unroll
    for (int i = 0; i < (K::XPC + KS_NW - 1) / KS_NW; ++i) {
      const int q = wave + KS_NW * i;
      if (q < K::XPC) {
        int u = lane;
        asm volatile("" : "+v"(u));
        u += 64 * q;
        const int px = u / KS_NCH, c = u - px * KS_NCH;
        const int pix = min(p0 + px, HW - 1);
        ks_glds16(XZ + ((size_t)n * HW + pix) * p.ldr + c * 8,
                  lds0 + 2u * K::WBUF + (uint32_t)KS_XCH + (uint32_t)q * 1024u);
      }
    }
  };
  // window pieces this wave issues per tile (wave-uniform)
  const int nwin = (K::WPC - wave + KS_NW - 1) / KS_NW;

  issue_win(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // this lane's pixel offset in a group of each of the five bank patterns, 5 bits each
  unsigned lperm = 0;
#pragma unroll
  for (int q = 0; q < 5; ++q) lperm |= (unsigned)g_ks_perm[W == 20 ? 0 : 1][q][r32] << (5 * q);
  // consumed here, so the compiler's wait for these loads sits before the tile loop
  // (inside it, its vmcnt would also count the hand-counted window DMA)
  asm volatile("" : "+v"(lperm));
  auto lpx = [&](int p0, int j) __attribute__((always_inline)) {
    const int pat = ((p0 + 32 * j) % W) / (W / 5);
    return (int)((lperm >> (5 * pat)) & 31u);
  };

  // this wave finishes pixel group 2 ph + kh of every tile and hands its
  // partial of group 2 ph + (1 - kh) to its partner (cg, 1 - kh, ph)
  const int gown = 2 * ph + kh, gpart = 2 * ph + (1 - kh);
  const int partner = cg + 3 * (1 - kh) + 6 * ph;
#ifdef VOX_DIAG
  const bool trace = HAS_Z && blockIdx.x == 0 && lane == 0;
#else
  constexpr bool trace = false;
#endif
  auto stamp = [&](int tj, int i) __attribute__((always_inline)) {
    if (trace && tj < 16) g_ks_trace[(wave * 16 + tj) * 8 + i] = __builtin_amdgcn_s_memtime();
  };
  for (int tj = 0; tj < ntiles; ++tj) {
    const int b = tj & 1;
    stamp(tj, 0);
    if (HAS_Z) issue_xz(tj);
    // the next tile's window pieces go out between the first pass's MFMAs
    // (issued together here they held every wave ~2-4k clk per tile before
    // its first MFMA; conv3x3_ks 990 -> 967 us per step); same issue order
    // relative to the x rows and stores
    int n1 = 0, r0w1 = 0, hn1 = H;
    const bool more = tj + 1 < ntiles;
    if (more) {
      const int id1 = t_first + (tj + 1) * t_step;
      n1 = id1 / tpu;
      r0w1 = ((id1 - n1 * tpu) * KS_TP) / W - 1;
      if (p.vlen) hn1 = valid_rows(p.vlen, p.vsh, n1, H);
    }
    auto fill = [&](int s) __attribute__((always_inline)) {
      if (more && s % 6 == 3) {
        const int q = wave + KS_NW * (s / 6);
        if (q < K::WPC) issue_piece(n1, r0w1, b ^ 1, q, hn1);
      }
    };
    auto nofill = [](int) {};
    stamp(tj, 1);
    const int id = t_first + tj * t_step;
    const int n = id / tpu, t = id - n * tpu;
    const int p0 = t * KS_TP;
    // lane-derived values re-formed per tile from a laundered lane id: kept
    // live across the loop they cost the weights' registers (spills)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int h = ln >> 5;
    // this lane's output pixel (group gown) and its 16-B cout chunks 16 i + 8 h
    const int ro = lpx(p0, gown);
    const int pxo = p0 + 32 * gown + ro;
    const bool inpx = pxo < HW;
    const size_t pix = (size_t)n * HW + (inpx ? pxo : HW - 1);
    // byte address of the lane's pixel slot of group j shifted by (-1 row,
    // -1 column), chunk h; + a compile-time tap/chunk offset per k16-step
    auto base_of = [&](int j) __attribute__((always_inline)) {
      const int pc = min(p0 + 32 * j + lpx(p0, j), HW - 1);
      const int rr = pc / W - (p0 / W - 1);   // window row of the pixel (>= 1)
      return b * K::WBUF + KS_PB * ((rr - 1) * SW + (pc % W)) + 16 * h;
    };
    // one pass: the 27 k16-steps of K half KH over pixel group j, one
    // accumulation chain (32x32x16 needs no interleaving for throughput),
    // fragments read KS_PD steps ahead (2; 3 and 4 measured the same)
    auto kpass = [&](auto khc, int j, auto&& fl) __attribute__((always_inline)) {
      constexpr int KH = decltype(khc)::value;
      auto off = [](int s) constexpr {
        const int S = 27 * KH + s, tap = S / 6, part = S % 6;
        return KS_PB * ((tap / 3) * SW + tap % 3) + 32 * part;
      };
      const int bs = base_of(j);
      f32x16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
      bf16x8 bf[KS_PD + 1];
#pragma unroll
      for (int s = 0; s < KS_PD; ++s) bf[s] = *reinterpret_cast<const bf16x8*>(smem + bs + off(s));
#pragma unroll
      for (int s = 0; s < KS_SH; ++s) {
        // hard scheduling fences: with sched_group_barrier hints alone the
        // compiler issued each read right before its MFMA (lgkmcnt(0) per MFMA)
        if (s + KS_PD < KS_SH)
          bf[(s + KS_PD) % (KS_PD + 1)] = *reinterpret_cast<const bf16x8*>(smem + bs + off(s + KS_PD));
        __builtin_amdgcn_sched_barrier(0);
        acc = mfma32(wr[s], bf[s % (KS_PD + 1)], acc);
        fl(s);
        __builtin_amdgcn_sched_barrier(0);
      }
      return acc;
    };
    f32x16 acc;
    if (kh == 0) {
      const f32x16 give = kpass(std::integral_constant<int, 0>{}, gpart, fill);
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4)
        *reinterpret_cast<f32x4*>(xch + wave * 1024 + r4 * 256 + ln * 4) =
            f32x4{give[4 * r4], give[4 * r4 + 1], give[4 * r4 + 2], give[4 * r4 + 3]};
      stamp(tj, 2);
      acc = kpass(std::integral_constant<int, 0>{}, gown, nofill);
    } else {
      const f32x16 give = kpass(std::integral_constant<int, 1>{}, gpart, fill);
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4)
        *reinterpret_cast<f32x4*>(xch + wave * 1024 + r4 * 256 + ln * 4) =
            f32x4{give[4 * r4], give[4 * r4 + 1], give[4 * r4 + 2], give[4 * r4 + 3]};
      stamp(tj, 2);
      acc = kpass(std::integral_constant<int, 1>{}, gown, nofill);
    }
    stamp(tj, 3);
    // this tile's x rows have landed: younger are the next window's pieces
    if (HAS_Z) vm_wait(tj + 1 < ntiles ? nwin : 0);
    stamp(tj, 4);
    __syncthreads();   // B: partials and x rows visible; every wave done with window b
    stamp(tj, 5);
    // (half 0) + (half 1), BN on packed pairs (the same roundings as scalar)
    f32x2 a2[8];
#pragma unroll
    for (int r4 = 0; r4 < 4; ++r4) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(xch + partner * 1024 + r4 * 256 + ln * 4);
      a2[2 * r4] = f32x2{acc[4 * r4], acc[4 * r4 + 1]} + f32x2{v[0], v[1]};
      a2[2 * r4 + 1] = f32x2{acc[4 * r4 + 2], acc[4 * r4 + 3]} + f32x2{v[2], v[3]};
    }
    // y: register group q holds couts 32 cg + 8 q + 4 h + (0..3) of pixel pxo
    unsigned yd[4][2];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int co = 32 * cg + 8 * q + 4 * h;
      const f32x4 m = *reinterpret_cast<const f32x4*>(bnm + co);
      const f32x4 iv = *reinterpret_cast<const f32x4*>(bni + co);
      const f32x2 t0 = ks_pk_sub(a2[2 * q], f32x2{m[0], m[1]}) * f32x2{iv[0], iv[1]};
      const f32x2 t1 = ks_pk_sub(a2[2 * q + 1], f32x2{m[2], m[3]}) * f32x2{iv[2], iv[3]};
      // one v_cvt_pk_bf16_f32 per pair (element-wise the compiler converted each
      // value alone and merged the halves with v_perm_b32: 16 extra per tile)
      bf16x4 y = __builtin_bit_cast(bf16x4, uint2{ks_cvt_pk(t0), ks_cvt_pk(t1)});
      y = relu_bf16(y);
      const uint2 d = __builtin_bit_cast(uint2, y);
      yd[q][0] = d.x;
      yd[q][1] = d.y;
    }
#if KS_STAGE
    // y through the partner's partial-sum slot (this wave was its only reader):
    // row r32 (pixel ro) x 32 couts, 64 B, 16-B chunks swizzled by (r32 >> 1) & 3
    // (the b64 writes of 16 lanes then fall on 8 bank pairs, not 2); read back
    // as 16 pixels x 64 B per instruction, so each y / z store touches 16 lines
    // with 64 B instead of 32 with 32 B (stores ~17 % of the kernel, line-bound)
    char* stg = smem + 2 * K::WBUF + partner * 4096;
    {
      const int r = ln & 31, sw = (r >> 1) & 3;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<uint2*>(stg + r * 64 + ((q ^ sw) * 16) + 8 * h) = uint2{yd[q][0], yd[q][1]};
    }
    asm volatile("" ::: "memory");   // same-wave LDS: in order in hardware; keep the compiler's order
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int r = (ln >> 2) + 16 * k, c = ln & 3;
      const u32x4 yc = *reinterpret_cast<const u32x4*>(stg + r * 64 + ((c ^ ((r >> 1) & 3)) * 16));
      const int rk = __builtin_amdgcn_ds_bpermute(4 * r, ro);   // pixel of row r (lane r's)
      const int pk = p0 + 32 * gown + rk;
      const bool ink = pk < HW;
      const size_t pixk = (size_t)n * HW + (ink ? pk : HW - 1);
      // always issued (a masked pixel stores to a sink line) so every wave's
      // vmcnt count below is the same
      ks_st16(ink ? (void*)(Y + pixk * p.ldy + 32 * cg + 8 * c) : (void*)&g_ks_sink[ln], yc);
      if (HAS_Z) {
        const u32x4 xw = *reinterpret_cast<const u32x4*>(xzb + (32 * gown + rk) * (KS_C * 2) + (32 * cg + 8 * c) * 2);
        u32x4 zw;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          // bf16 pairs widened to fp32 pairs, one packed add: (float)x + (float)y
          const f32x2 z2 = f32x2{__builtin_bit_cast(float, xw[e] << 16), __builtin_bit_cast(float, xw[e] & 0xFFFF0000u)} +
                           f32x2{__builtin_bit_cast(float, yc[e] << 16), __builtin_bit_cast(float, yc[e] & 0xFFFF0000u)};
          zw[e] = ks_cvt_pk(z2);
        }
        ks_st16(ink ? (void*)(Z + pixk * p.ldy2 + 32 * cg + 8 * c) : (void*)&g_ks_sink[ln], zw);
      }
    }
#else
    // lanes l and l + 32 (same pixel) hold couts 8q..8q+3 and 8q+4..8q+7: one
    // half exchange per dword pair gives each lane 8 contiguous couts, chunk
    // i = 16 i + 8 h (T21 of the HIP guide)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const auto r0 = __builtin_amdgcn_permlane32_swap(yd[2 * i][0], yd[2 * i + 1][0], false, false);
      const auto r1 = __builtin_amdgcn_permlane32_swap(yd[2 * i][1], yd[2 * i + 1][1], false, false);
      const u32x4 yc = {r0[0], r1[0], r0[1], r1[1]};
      const size_t off = pix * p.ldy + 32 * cg + 16 * i + 8 * h;
      // always issued (a masked pixel stores to a sink line) so every wave's
      // vmcnt count below is the same
      ks_st16(inpx ? (void*)(Y + off) : (void*)&g_ks_sink[ln], yc);
      if (HAS_Z) {
        const bf16x8 xb = *reinterpret_cast<const bf16x8*>(
            xzb + (32 * gown + ro) * (KS_C * 2) + (32 * cg + 16 * i + 8 * h) * 2);
        const u32x4 xw = __builtin_bit_cast(u32x4, xb);
        bf16x8 zb;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          // bf16 pairs widened to fp32 pairs, one packed add: (float)x + (float)y
          const f32x2 z2 = f32x2{__builtin_bit_cast(float, xw[e] << 16), __builtin_bit_cast(float, xw[e] & 0xFFFF0000u)} +
                           f32x2{__builtin_bit_cast(float, yc[e] << 16), __builtin_bit_cast(float, yc[e] & 0xFFFF0000u)};
          zb[2 * e] = (bf16_t)z2[0];
          zb[2 * e + 1] = (bf16_t)z2[1];
        }
        ks_st16(inpx ? (void*)(Z + pix * p.ldy2 + 32 * cg + 16 * i + 8 * h) : (void*)&g_ks_sink[ln],
                __builtin_bit_cast(u32x4, zb));
      }
    }
#endif
    stamp(tj, 6);
    // window tj+1 has landed: younger are only this tile's stores
    // (a diagnostic stamp store above only makes this wait stricter)
    if (HAS_Z) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    __syncthreads();   // D: next window visible; partials read before they are rewritten
    stamp(tj, 7);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

hipError_t ks_trace_read(void* dst, size_t bytes) {
  if (bytes > sizeof(g_ks_trace)) bytes = sizeof(g_ks_trace);
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_ks_trace), bytes, 0, hipMemcpyDeviceToHost);
}

int conv3_ks_ok(const ConvParams& p) {
  if (p.Cin != KS_C || p.Cout != KS_C || p.kh != 3 || p.kw != 3 || p.groups != 1) return 0;
  if (p.sh != 1 || p.sw != 1 || p.dh != 1 || p.dw != 1 || p.ph != 1 || p.pw != 1) return 0;
  if (p.Ho != p.H || p.Wo != p.W || !(p.W == 20 || p.W == 10)) return 0;
  if (p.kp != 9 * KS_C) return 0;   // weights [96][9 * 96], tap-major
  if (p.ldx % 8 || p.ldy % 8 || p.ldr % 8 || p.ldy2 % 8) return 0;
  if (p.flags != (EPI_AFFINE | EPI_RELU) || p.in_mean || p.x2 || !p.mean || !p.inv) return 0;
  if (p.y2 && p.y2 != p.res) return 0;   // z_{k+1} in place over x_{k+1}
  return p.N * p.H * p.W > 0;
}

hipError_t launch_conv3_ks(const ConvParams& p, int num_cu, hipStream_t s) {
  if (!conv3_ks_ok(p)) return hipErrorInvalidValue;
  const bool z = p.y2 != nullptr;
  const int HW = p.H * p.W;
  const int T = p.N * ((HW + KS_TP - 1) / KS_TP);
  int G = num_cu < T ? num_cu : T;
  if (G >= 8) G = G / 8 * 8;
  if (p.W == 20) {
    if (z) hipLaunchKernelGGL((conv3x3_ks<20, true>), dim3(G), dim3(KS_NT), KsCfg<20>::LDS, s, p);
    else hipLaunchKernelGGL((conv3x3_ks<20, false>), dim3(G), dim3(KS_NT), KsCfg<20>::LDS, s, p);
  } else {
    if (z) hipLaunchKernelGGL((conv3x3_ks<10, true>), dim3(G), dim3(KS_NT), KsCfg<10>::LDS, s, p);
    else hipLaunchKernelGGL((conv3x3_ks<10, false>), dim3(G), dim3(KS_NT), KsCfg<10>::LDS, s, p);
  }
  return hipGetLastError();
}

}  // namespace vox

// Register-weight 3x3 conv for the w = 96 stride-1 Res2Net branches
// (res2net_pad_conv_bn_relu, res2net_model.py:53-75, layer 3): y_k =
// relu(bn(conv3x3(z_k))), and for k < S-1 the next branch's input
// z_{k+1} = x_{k+1} + y_k formed in place over x_{k+1}.
//
// conv3x3_pipe (conv3.hip) streams both operands through LDS-DMA for every
// 256-pixel tile: the 166 KB of weights and an im2col gather that moves each
// input pixel 9 times -- ~2.4 KB per output pixel at the per-CU fill rate.
// Here the weights never move after the prologue: each of the 12 waves holds
// one 16-channel output tile's 16 x 864 weights in registers (108 VGPRs), and
// a tile's input (the <= RMAX image rows its 128 pixels and their 3x3 halo
// touch, zero rows/columns for the SAME padding) is fetched once into an LDS
// window, double-buffered so the next tile's window (and its x_{k+1} rows for
// the in-place epilogue) streams in under this tile's MFMAs: ~520 B per
// output pixel.  Tiles never cross an utterance (the padding is per
// utterance), 8 pixel tiles of 16 each; wave w computes output tile w % 6 for
// pixel tiles 4 (w / 6) .. +3, with no barrier between its 27 k-steps.
//
// Window layout (16-B units): chunk c (8 channels) of pixel slot x sits in
// sub-plane c/2 at unit 2x + c%2.  The two lane groups a gfx950
// ds_read_b128 pairs read chunks c, c+1 (c even) of one tap for 8 distinct
// pixels: opposite parities, so fragment reads are conflict-free; every
// fragment address is a per-lane base plus a compile-time tap offset.
// K order = k-steps of 32 in increasing order (k = tap * 96 + ci), epilogue
// roundings as conv_igemm's: bitwise identical to conv3x3_pipe.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "device_common.h"
#include "kernels.h"

namespace vox {

namespace {
constexpr int CR_C = 96;               // Cin = Cout = branch width
constexpr int CR_TP = 128;             // pixels per tile
constexpr int CR_NW = 12;              // 6 output tiles x 2 pixel halves
constexpr int CR_NT = 64 * CR_NW;
constexpr int CR_KS = 9 * CR_C / 32;   // 27 k-steps
constexpr int CR_NCH = CR_C / 8;       // 12 chunks per pixel

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void cr_glds16(const void* src, uint32_t lds) {
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
// the trailing s_nop keeps the next instruction from overwriting the data
// registers before the store has read them
__device__ __forceinline__ void cr_st16(void* dst, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" : : "v"(dst), "v"(v) : "memory");
}
#define CR_W(n) \
  case n: asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory"); break;
__device__ __forceinline__ void cr_wait_vm(int n) {
  switch (n) {
    CR_W(0) CR_W(1) CR_W(2) CR_W(3) CR_W(4) CR_W(5) CR_W(6) CR_W(7) CR_W(8) CR_W(9)
    CR_W(10) CR_W(11) CR_W(12) CR_W(13) CR_W(14) CR_W(15) CR_W(16)
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
  __builtin_amdgcn_sched_barrier(0);
}
#undef CR_W
}  // namespace

__device__ uint4 g_cr_zero[4] = {};

template <int W>
struct CrCfg {
  static constexpr int SW = W + 2;                                // slots per window row
  static constexpr int RMAX = (W - 1 + CR_TP - 1) / W + 1 + 2;    // rows + halo a tile touches
  static constexpr int SLOTS = RMAX * SW;
  static constexpr int SPW = 2 * SLOTS;                           // units per sub-plane
  static constexpr int WIN = CR_NCH / 2 * SPW * 16;               // window bytes
  static constexpr int WPC = (WIN + 1023) / 1024;                 // window DMA pieces
  static constexpr int XZB = CR_TP * CR_C * 2;                    // x_{k+1} rows of the tile
  static constexpr int XPC = XZB / 1024;
  static constexpr int PCS = WPC + XPC;                           // pieces per tile
  static constexpr int BUF = WPC * 1024;                          // one window buffer
  static constexpr int YST = 13 * 16;                             // staged y: pixel stride (odd units)
  static constexpr int YSB = CR_TP * YST;
  static constexpr int LDS = 2 * BUF + 2 * XZB + YSB + 2 * CR_C * 4;
  static constexpr int PPW = (PCS + CR_NW - 1) / CR_NW;           // pieces per wave (max)
  static_assert(XZB % 1024 == 0, "xz pieces");
  static_assert(LDS <= 163840, "LDS");
  static_assert(CR_TP * CR_NCH % CR_NT == 0, "epilogue chunks");
};

#pragma clang fp contract(off)
// DBG (diagnostics, VOXEMB_CONV3_RW_DBG; garbage out): 1 = contiguous window
// sources, 2 = no window DMA, 4 = no MFMA, 8 = no stores, 16 = no k-loop,
// 32 = no DMA waits
template <int W, bool HAS_Z, int DBG = 0>
__global__ __launch_bounds__(CR_NT) void conv3x3_rw(ConvParams p) {
  using K = CrCfg<W>;
  constexpr int SW = K::SW, SPW = K::SPW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int ct = wave % 6, ph = wave / 6;     // output tile, pixel half
  const int H = p.H, HW = p.H * W;
  const int tpu = (HW + CR_TP - 1) / CR_TP;  // tiles per utterance
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
  const bf16_t* zero = reinterpret_cast<const bf16_t*>(g_cr_zero);
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  char* xzb = smem + 2 * K::BUF;  // x_{k+1} rows of a tile, double-buffered
  char* ys = xzb + 2 * K::XZB;    // y of a tile, pixel-major, for row-contiguous stores
  float* bnm = reinterpret_cast<float*>(ys + K::YSB);
  float* bni = bnm + CR_C;
  for (int c = tid; c < CR_C; c += CR_NT) {
    bnm[c] = p.mean[c];
    bni[c] = p.inv[c];
  }

  // weights of output tile ct: row 16 ct + col, k-step s chunk g
  bf16x8 wr[CR_KS];
  {
    const bf16_t* __restrict__ Wt = reinterpret_cast<const bf16_t*>(p.w);
#pragma unroll
    for (int s = 0; s < CR_KS; ++s)
      wr[s] = ld16(Wt + (size_t)(16 * ct + col) * (9 * CR_C) + 32 * s + 8 * g);
  }

  // DMA piece q of tile tj into buffer b: window units [64q, 64q + 64), then
  // the tile's x_{k+1} pixel rows (linear, 192 B per pixel)
  auto issue_piece = [&](int tj, int q, int b) __attribute__((always_inline)) {
    const int id = t_first + tj * t_step;
    const int n = id / tpu, t = id - n * tpu;
    const int p0 = t * CR_TP;
    const bf16_t* src = zero;
    if (q < K::WPC) {
      // recomputed per tile from the laundered lane id: no per-piece state
      // held in registers (laundering the sum instead made the compiler keep
      // each piece's sum in scratch and reload it under a vmcnt(0) that
      // serialised the DMA issue)
      int u = lane;
      asm volatile("" : "+v"(u));
      u += 64 * q;
      const int sp = u / SPW, rem = u - sp * SPW;
      const int slot = rem >> 1, c = 2 * sp + (rem & 1);
      const int wr_ = slot / SW, sc = slot - wr_ * SW;
      const int row = p0 / W - 1 + wr_, wc = sc - 1;
      if (sp < CR_NCH / 2 && row >= 0 && row < H && wc >= 0 && wc < W)
        src = X + ((size_t)n * HW + row * W + wc) * p.ldx + c * 8;
      if (DBG & 1) src = X + ((size_t)n * HW + p0) * p.ldx + u * 8;
    } else if (HAS_Z) {
      int u = lane;
      asm volatile("" : "+v"(u));
      u += 64 * (q - K::WPC);
      const int px = u / CR_NCH, c = u - px * CR_NCH;
      const int pix = min(p0 + px, HW - 1);
      src = XZ + ((size_t)n * HW + pix) * p.ldr + c * 8;
    }
    if ((DBG & 2) && q < K::WPC) return;
    const uint32_t dst = q < K::WPC ? lds0 + (uint32_t)b * K::BUF + (uint32_t)q * 1024u
                                    : lds0 + 2u * K::BUF + (uint32_t)b * K::XZB +
                                          (uint32_t)(q - K::WPC) * 1024u;
    cr_glds16(src, dst);
  };
  // this wave's window pieces of a tile (q = wave, wave + 12, ...) and its
  // x_{k+1} pieces; returns the count issued (wave-uniform)
  auto issue_win = [&](int tj, int b) __attribute__((always_inline)) {
    int c = 0;
#pragma unroll
    for (int i = 0; i < (K::WPC + CR_NW - 1) / CR_NW; ++i) {
      const int q = wave + CR_NW * i;
      if (q < K::WPC) {
        issue_piece(tj, q, b);
        ++c;
      }
    }
    return c;
  };
  auto issue_xz = [&](int tj, int b) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < (K::XPC + CR_NW - 1) / CR_NW; ++i) {
      const int q = K::WPC + wave + CR_NW * i;
      if (HAS_Z && q < K::PCS) issue_piece(tj, q, b);
    }
  };
  // store pass of tile tj (deferred into the next tile, so its HBM writes
  // drain under MFMAs): y from the staging, z = x_{k+1} + y, 16-B chunks u of
  // pixels px (192 contiguous bytes per pixel)
  auto store_pass = [&](int tj) __attribute__((always_inline)) {
    const int id = t_first + tj * t_step;
    const int n = id / tpu, t = id - n * tpu;
    const int p0 = t * CR_TP;
    const char* xzl = xzb + (tj & 1) * K::XZB;
#pragma unroll
    for (int i = 0; i < CR_TP * CR_NCH / CR_NT; ++i) {
      int c = tid;
      asm volatile("" : "+v"(c));   // nothing per-pass held in registers (or scratch)
      c += CR_NT * i;
      const int px = c / CR_NCH, u = c - px * CR_NCH;
      const bool in = p0 + px < HW && !(DBG & 8);
      const size_t pix = (size_t)n * HW + p0 + px;
      const bf16x8 y = *reinterpret_cast<const bf16x8*>(ys + px * K::YST + u * 16);
      // (masked lanes skip the store: the tile's closing vmcnt(0) needs no count)
      if (in) cr_st16(Y + pix * p.ldy + u * 8, __builtin_bit_cast(u32x4, y));
      if (HAS_Z) {
        const bf16x8 xv = *reinterpret_cast<const bf16x8*>(xzl + px * (CR_C * 2) + u * 16);
        bf16x8 zv;
#pragma unroll
        for (int e = 0; e < 8; ++e) zv[e] = (bf16_t)((float)xv[e] + (float)y[e]);
        if (in) cr_st16(Z + pix * p.ldy2 + u * 8, __builtin_bit_cast(u32x4, zv));
      }
    }
  };

  issue_win(0, 0);
  cr_wait_vm(0);
  __syncthreads();

  // chunk c = 4 part + g of a k-step lives in sub-plane 2 part + g/2, parity g%2
  int cg[3];
#pragma unroll
  for (int part = 0; part < 3; ++part) cg[part] = ((2 * part + (g >> 1)) * SPW + (g & 1)) * 16;

  // tile tj: [pass: stores of tile tj-1] [DMA: window tj+1, x rows tj] [27
  // k-steps] | barrier | [y of tile tj -> staging] [DMA landed] | barrier
  for (int tj = 0; tj < ntiles; ++tj) {
    const int b = tj & 1;
    if (tj > 0) store_pass(tj - 1);
    if (tj + 1 < ntiles) issue_win(tj + 1, b ^ 1);
    issue_xz(tj, b);
    const int id = t_first + tj * t_step;
    const int n = id / tpu, t = id - n * tpu;
    const int p0 = t * CR_TP;
    // per pixel tile: byte address of the (ky, kx) = (0, 0) tap slot of the
    // lane's pixel; + cg[part] + 32 (ky SW + kx) per k-step
    int bj[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int pc = min(p0 + 16 * (4 * ph + jj) + col, HW - 1);
      const int prow = pc / W - (p0 / W - 1);   // window row of the pixel (>= 1)
      bj[jj] = b * K::BUF + 32 * ((prow - 1) * SW + (pc % W));
    }
    f32x4 acc[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) acc[jj] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < ((DBG & 16) ? 0 : CR_KS); ++s) {
      const int tap = s / 3, part = s % 3;
      const int off = 32 * ((tap / 3) * SW + tap % 3);
      bf16x8 bf[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        int a = bj[jj] + cg[part];
        asm volatile("" : "+v"(a));   // one add per read, nothing precomputed per k-step
        bf[jj] = *reinterpret_cast<const bf16x8*>(smem + a + off);
      }
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        if (!(DBG & 4)) acc[jj] = mfma_step(wr[s], bf[jj], acc[jj]);
        else acc[jj][0] += (float)bf[jj][0];
      __builtin_amdgcn_sched_barrier(0);   // fragments of one k-step live at a time
    }
    __syncthreads();   // every thread is done with the staging (store pass tj-1)
    // y of tile tj: 4 output channels 16 ct + 4 g of pixel 16 j + col
    const int co = 16 * ct + 4 * g;
    const f32x4 m = *reinterpret_cast<const f32x4*>(bnm + co);
    const f32x4 iv = *reinterpret_cast<const f32x4*>(bni + co);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int px = 16 * (4 * ph + jj) + col;
      bf16x4 y;
#pragma unroll
      for (int e = 0; e < 4; ++e) y[e] = (bf16_t)((acc[jj][e] - m[e]) * iv[e]);
      y = relu_bf16(y);
      *reinterpret_cast<bf16x4*>(ys + px * K::YST + co * 2) = y;
    }
    // window tj+1 and x rows tj have landed (the older stores have too)
    if (!(DBG & 32)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  store_pass(ntiles - 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int conv3_rw_ok(const ConvParams& p) {
  if (p.Cin != CR_C || p.Cout != CR_C || p.kh != 3 || p.kw != 3 || p.groups != 1) return 0;
  if (p.sh != 1 || p.sw != 1 || p.dh != 1 || p.dw != 1 || p.ph != 1 || p.pw != 1) return 0;
  if (p.Ho != p.H || p.Wo != p.W || !(p.W == 20 || p.W == 10)) return 0;
  if (p.ldx % 8 || p.ldy % 8 || p.ldr % 8 || p.ldy2 % 8) return 0;
  if (p.flags != (EPI_AFFINE | EPI_RELU) || p.in_mean || p.x2 || !p.mean || !p.inv) return 0;
  if (p.y2 && p.y2 != p.res) return 0;   // z_{k+1} in place over x_{k+1}
  return p.N * p.H * p.W > 0;
}

template <int W, bool Z>
static void launch_cr(const ConvParams& p, int G, hipStream_t s) {
#ifdef VOX_DIAG
  static const int dbg = [] {
    const char* e = std::getenv("VOXEMB_CONV3_RW_DBG");
    return e ? std::atoi(e) : 0;
  }();
#else
  constexpr int dbg = 0;
#endif
  switch (dbg) {
#ifdef VOX_DIAG
#define CR_L(d) case d: hipLaunchKernelGGL((conv3x3_rw<W, Z, d>), dim3(G), dim3(CR_NT), CrCfg<W>::LDS, s, p); break;
    CR_L(1) CR_L(2) CR_L(8) CR_L(16) CR_L(32) CR_L(24) CR_L(48) CR_L(40)
#undef CR_L
#endif
    default: hipLaunchKernelGGL((conv3x3_rw<W, Z, 0>), dim3(G), dim3(CR_NT), CrCfg<W>::LDS, s, p); break;
  }
}

hipError_t launch_conv3_rw(const ConvParams& p, int num_cu, hipStream_t s) {
  if (!conv3_rw_ok(p)) return hipErrorInvalidValue;
  const bool z = p.y2 != nullptr;
  const int HW = p.H * p.W;
  const int T = p.N * ((HW + CR_TP - 1) / CR_TP);
  int G = num_cu < T ? num_cu : T;
  if (G >= 8) G = G / 8 * 8;
  if (p.W == 20) {
    if (z) launch_cr<20, true>(p, G, s); else launch_cr<20, false>(p, G, s);
  } else {
    if (z) launch_cr<10, true>(p, G, s); else launch_cr<10, false>(p, G, s);
  }
  return hipGetLastError();
}

}  // namespace vox

// Register-weight stride-2 3x3 conv for the w = 96 Res2Net branches of a
// stride-2 block (res2net_pad_conv_bn_relu, res2net_model.py:26-78 with
// stride 2: fixed_padding(1, 1) + VALID; the layer-3 block 0 at 100x40 ->
// 50x20): y = relu(bn(conv3x3_s2(x))), no hierarchical addend.
//
// conv3x3_pipe gathers an im2col operand per 256-pixel tile through the LDS-DMA
// ring (2.5x the branch input in HBM reads, PMC).  Here, as conv3x3_rw does for
// stride 1, each of the 12 waves keeps one 16-channel output tile's 16 x 864
// weights in registers (108 VGPRs), and a tile = TR output rows of one
// utterance whose input window (2 TR + 1 rows, every column) is fetched once
// into LDS, double-buffered under the previous tile's MFMAs.  The window keeps
// the odd input columns before the even ones (slot 0 = the padding column -1,
// slots 1..WO = columns 1, 3, .., slots WO+1.. = columns 0, 2, ..), so the 16
// pixels of a fragment read sit in consecutive slots for every tap, as at
// stride 1, and the sub-plane / parity chunk layout of conv3r.hip keeps the
// ds_read_b128 lane groups conflict-free.
// K order = 27 k-steps of 32 (k = tap * 96 + ci), epilogue BN -> ReLU ->
// bf16: bitwise equal to conv3x3_pipe (tests/test_gpu_parity.py).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_common.h"
#include "kernels.h"

namespace vox {

namespace {
constexpr int CS_C = 96;               // Cin = Cout = branch width
constexpr int CS_NW = 12;              // 6 output tiles x 2 pixel halves
constexpr int CS_NT = 64 * CS_NW;
constexpr int CS_KS = 9 * CS_C / 32;   // 27 k-steps
constexpr int CS_NCH = CS_C / 8;       // 12 chunks per pixel

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void cs_glds16(const void* src, uint32_t lds) {
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
__device__ __forceinline__ void cs_st16(void* dst, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" : : "v"(dst), "v"(v) : "memory");
}
}  // namespace

__device__ uint4 g_cs_zero[4] = {};

template <int WO>
struct CsCfg {
  static constexpr int WI = 2 * WO;                      // input columns
  static constexpr int TR = (64 + WO - 1) / WO > 3 ? 3 : (64 / WO);   // output rows per tile
  static constexpr int TP = TR * WO;                     // output pixels per tile (<= 64)
  static constexpr int SW = WI + 1;                      // slots per window row (pad column -1)
  static constexpr int ROWS = 2 * TR + 1;
  static constexpr int SLOTS = ROWS * SW;
  static constexpr int SPW = 2 * SLOTS;                  // units per sub-plane
  static constexpr int WIN = CS_NCH / 2 * SPW * 16;      // window bytes
  static constexpr int WPC = (WIN + 1023) / 1024;        // DMA pieces
  static constexpr int BUF = WPC * 1024;
  static constexpr int YST = 13 * 16;                    // staged y: pixel stride (odd units)
  static constexpr int YSB = 64 * YST;
  static constexpr int LDS = 2 * BUF + YSB + 2 * CS_C * 4;
  static_assert(TP <= 64, "4 pixel tiles of 16");
  static_assert(LDS <= 163840, "LDS");
};

// window slot of input column c (-1 .. WI-1): odd columns (and -1) first, then even
template <int WO>
__device__ __forceinline__ int cs_slot(int c) {
  return (c & 1) || c < 0 ? (c + 1) >> 1 : WO + 1 + (c >> 1);
}

#pragma clang fp contract(off)
template <int WO>
__global__ __launch_bounds__(CS_NT) void conv3x3_s2r(ConvParams p) {
  using K = CsCfg<WO>;
  constexpr int SW = K::SW, SPW = K::SPW, TR = K::TR, TP = K::TP;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int ct = wave % 6, ph = wave / 6;     // output tile, pixel half
  const int H = p.H, Ho = p.Ho;
  const int tpu = (Ho + TR - 1) / TR;         // tiles per utterance
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
  bf16_t* __restrict__ Y = reinterpret_cast<bf16_t*>(p.y);
  const bf16_t* zero = reinterpret_cast<const bf16_t*>(g_cs_zero);
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  char* ys = smem + 2 * K::BUF;   // y of a tile, pixel-major, for row-contiguous stores
  float* bnm = reinterpret_cast<float*>(ys + K::YSB);
  float* bni = bnm + CS_C;
  for (int c = tid; c < CS_C; c += CS_NT) {
    bnm[c] = p.mean[c];
    bni[c] = p.inv[c];
  }

  bf16x8 wr[CS_KS];
  {
    const bf16_t* __restrict__ Wt = reinterpret_cast<const bf16_t*>(p.w);
#pragma unroll
    for (int s = 0; s < CS_KS; ++s)
      wr[s] = ld16(Wt + (size_t)(16 * ct + col) * (9 * CS_C) + 32 * s + 8 * g);
  }

  // window DMA of tile tj into buffer b: piece q = units [64q, 64q + 64)
  auto issue_win = [&](int tj, int b) __attribute__((always_inline)) {
    const int id = t_first + tj * t_step;
    const int n = id / tpu, t = id - n * tpu;
    const int r0 = 2 * t * TR - 1;             // input row of window row 0
    // ragged batch: the utterance's input rows past hn are its fixed padding
    const int hn = p.vlen ? valid_rows(p.vlen, p.vsh, n, H) : H;
#pragma unroll
    for (int i = 0; i < (K::WPC + CS_NW - 1) / CS_NW; ++i) {
      const int q = wave + CS_NW * i;
      if (q < K::WPC) {
        int u = lane;
        asm volatile("" : "+v"(u));
        u += 64 * q;
        const int sp = u / SPW, rem = u - sp * SPW;
        const int slot = rem >> 1, c = 2 * sp + (rem & 1);
        const int wrow = slot / SW, sc = slot - wrow * SW;
        // slot -> input column (inverse of cs_slot)
        const int icol = sc <= WO ? 2 * sc - 1 : 2 * (sc - WO - 1);
        const int row = r0 + wrow;
        const bf16_t* src = zero;
        if (sp < CS_NCH / 2 && row >= 0 && row < hn && icol >= 0 && icol < K::WI)
          src = X + ((size_t)n * H * K::WI + (size_t)row * K::WI + icol) * p.ldx + c * 8;
        cs_glds16(src, lds0 + (uint32_t)b * K::BUF + (uint32_t)q * 1024u);
      }
    }
  };
  // store pass of tile tj: y from the staging, 16-B chunks u of pixel px
  auto store_pass = [&](int tj) __attribute__((always_inline)) {
    const int id = t_first + tj * t_step;
    const int n = id / tpu, t = id - n * tpu;
    const int o0 = t * TP;                     // first output pixel of the tile in the utterance
    const int HoWo = Ho * WO;
#pragma unroll
    for (int i = 0; i < (64 * CS_NCH + CS_NT - 1) / CS_NT; ++i) {
      int c = tid;
      asm volatile("" : "+v"(c));
      c += CS_NT * i;
      const int px = c / CS_NCH, u = c - px * CS_NCH;
      const bool in = px < TP && o0 + px < HoWo;
      if (in) {
        const bf16x8 y = *reinterpret_cast<const bf16x8*>(ys + px * K::YST + u * 16);
        cs_st16(Y + ((size_t)n * HoWo + o0 + px) * p.ldy + u * 8, __builtin_bit_cast(u32x4, y));
      }
    }
  };

  issue_win(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // chunk c = 4 part + g of a k-step lives in sub-plane 2 part + g/2, parity g%2
  int cg[3];
#pragma unroll
  for (int part = 0; part < 3; ++part) cg[part] = ((2 * part + (g >> 1)) * SPW + (g & 1)) * 16;
  // per pixel tile: slot of tap (0, 0) of the lane's output pixel (row pr, col pc)
  int bslot[2];
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int pxl = min(16 * (2 * ph + jj) + col, TP - 1);
    const int pr = pxl / WO, pc = pxl - pr * WO;
    bslot[jj] = 2 * pr * SW + pc;
  }

  for (int tj = 0; tj < ntiles; ++tj) {
    const int b = tj & 1;
    if (tj > 0) store_pass(tj - 1);
    if (tj + 1 < ntiles) issue_win(tj + 1, b ^ 1);
    f32x4 acc[2];
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) acc[jj] = f32x4{0.f, 0.f, 0.f, 0.f};
    // fragments of k-step s (both pixel tiles); read two steps ahead of their
    // MFMAs (a 3-set ring, as conv3x3_ks) so the LDS latency hides under the
    // MFMAs of the two steps before instead of stalling every step.  The six
    // (pixel tile, chunk part) base addresses are formed once per tile (the
    // tap offset is an immediate); no inline asm inside the k-loop, which
    // would split the scheduling region and undo the read-ahead order
    int ba[2][3];
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int part = 0; part < 3; ++part) {
        ba[jj][part] = b * K::BUF + 32 * bslot[jj] + cg[part];
        asm volatile("" : "+v"(ba[jj][part]));
      }
    auto rd = [&](int s, int jj) __attribute__((always_inline)) {
      const int tap = s / 3, part = s % 3;
      const int ky = tap / 3, kx = tap % 3;
      // tap (ky, kx) of output column pc: input column 2pc - 1 + kx ->
      // kx 0: odd slot pc, kx 1: even slot WO + 1 + pc, kx 2: odd slot pc + 1
      const int off = 32 * (ky * SW + (kx == 0 ? 0 : (kx == 1 ? WO + 1 : 1)));
      return *reinterpret_cast<const bf16x8*>(smem + ba[jj][part] + off);
    };
    bf16x8 bf[3][2];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) bf[s][jj] = rd(s, jj);
#pragma unroll
    for (int s = 0; s < CS_KS; ++s) {
      if (s + 2 < CS_KS) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) bf[(s + 2) % 3][jj] = rd(s + 2, jj);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) acc[jj] = mfma_step(wr[s], bf[s % 3][jj], acc[jj]);
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();   // every thread is done with the staging (store pass tj-1)
    const int co = 16 * ct + 4 * g;
    const f32x4 m = *reinterpret_cast<const f32x4*>(bnm + co);
    const f32x4 iv = *reinterpret_cast<const f32x4*>(bni + co);
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int px = 16 * (2 * ph + jj) + col;
      bf16x4 y;
#pragma unroll
      for (int e = 0; e < 4; ++e) y[e] = (bf16_t)((acc[jj][e] - m[e]) * iv[e]);
      y = relu_bf16(y);
      *reinterpret_cast<bf16x4*>(ys + px * K::YST + co * 2) = y;
    }
    // window tj+1 has landed (the older stores have too)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  store_pass(ntiles - 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int conv3_s2r_ok(const ConvParams& p) {
  if (p.Cin != CS_C || p.Cout != CS_C || p.kh != 3 || p.kw != 3 || p.groups != 1) return 0;
  if (p.sh != 2 || p.sw != 2 || p.dh != 1 || p.dw != 1 || p.ph != 1 || p.pw != 1) return 0;
  if (!(p.Wo == 20 && p.W == 40)) return 0;
  if (p.Ho != (p.H + 1) / 2) return 0;
  if (p.ldx % 8 || p.ldy % 8) return 0;
  if (p.flags != (EPI_AFFINE | EPI_RELU) || p.in_mean || p.x2 || p.res || p.y2 || !p.mean || !p.inv)
    return 0;
  return p.N * p.Ho * p.Wo > 0;
}

hipError_t launch_conv3_s2r(const ConvParams& p, int num_cu, hipStream_t s) {
  if (!conv3_s2r_ok(p)) return hipErrorInvalidValue;
  using K = CsCfg<20>;
  const int T = p.N * ((p.Ho + K::TR - 1) / K::TR);
  int G = num_cu < T ? num_cu : T;
  if (G >= 8) G = G / 8 * 8;
  hipLaunchKernelGGL((conv3x3_s2r<20>), dim3(G), dim3(CS_NT), K::LDS, s, p);
  return hipGetLastError();
}

}  // namespace vox

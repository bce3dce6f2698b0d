// Utterance-window 3x3 conv for the w = 192 stride-1 Res2Net branches
// (res2net_pad_conv_bn_relu, res2net_model.py:53-75, layer 4): y_k =
// relu(bn(conv3x3(z_k))) and, for k < S-1, z_{k+1} = x_{k+1} + y_k in place.
//
// conv3x3_pipe (conv3.hip) gathers im2col operands through LDS-DMA: at layer 4
// a 256-pixel x 96-cout tile moves 27 x 48 KB, ~5 KB per output pixel and
// cout half, and the kernel runs at the per-CU fill rate.  Layer 4 images are
// tiny (25 x 10 pixels at T = 200), so here a tile is a band of up to
// 256 / W rows of one utterance with all 192 couts: its input window (band +
// halo rows, one shared zero column between rows) is staged in LDS once
// (~115 KB), and only the weights stream, 12 KB per 32-wide k-step through a
// 3-slot ring (L2-resident, 663 KB per tile): ~3 KB per output pixel.
//
// 12 waves = 4 cout groups (48 couts, 3 MFMA tiles) x 3 pixel groups (6 pixel
// tiles of 16); waves w, w+4, w+8 (one SIMD) share a cout group.  Every wave
// issues one 1-KB weight piece per k-step (16 cout rows x 64 B, chunk swizzle
// of gemm_wide.hip); window layout as conv3r.hip (chunk c of slot x in
// sub-plane c/2, unit 2x + c%2).
// K order = k-steps of 32 in increasing order (k = tap * 192 + ci) and the
// epilogue roundings of conv3x3_pipe: bitwise identical to it.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_common.h"
#include "kernels.h"

namespace vox {

namespace {
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int CU_C = 192;                // Cin = Cout = branch width
constexpr int CU_NW = 12;
constexpr int CU_NT = 64 * CU_NW;
constexpr int CU_KS = 9 * CU_C / 32;     // 54 k-steps
constexpr int CU_NCH = CU_C / 8;         // 24 chunks per pixel
constexpr int CU_PXT = 16;               // pixel tiles per band (<= 256 pixels)
constexpr int CU_PG = 6;                 // pixel tiles per wave (3 groups, 18 >= 16)
constexpr int CU_WSLOT = CU_C * 64;      // 12 KB weight ring slot
constexpr int CU_NST = 3;

__device__ __forceinline__ void cu_glds16(const void* src, uint32_t lds) {
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
template <int N> __device__ __forceinline__ void cu_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" : : "n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ int cu_swz(int r) { return (4 - ((r >> 2) & 3)) & 3; }
}  // namespace

__device__ uint4 g_cu_zero[4] = {};

template <int W>
struct CuCfg {
  static constexpr int R = 256 / W;                 // band rows (pixels <= 256)
  static constexpr int SW = W + 1;                  // slots per row (shared zero column)
  static constexpr int SLOTS = (R + 2) * SW + 1;    // halo rows above and below
  static constexpr int SPW = 2 * SLOTS;             // units per sub-plane
  static constexpr int WIN = CU_NCH / 2 * SPW * 16;
  static constexpr int WPC = (WIN + 1023) / 1024;   // window DMA pieces
  static constexpr int WBUF = WPC * 1024;
  static constexpr int LDS = WBUF + CU_NST * CU_WSLOT;
  static_assert(LDS <= 163840, "LDS");
  static_assert(R * W <= 16 * CU_PXT, "band pixels");
};

#pragma clang fp contract(off)
// ConvParams use as conv3x3_pipe: x/ldx input slice, w = [192][9*192] tap-major
// bf16, y/ldy output slice, mean/inv BN; res/ldr = x_{k+1} and y2 = res when HAS_Z
template <int W, bool HAS_Z>
__global__ __launch_bounds__(CU_NT) void conv3x3_utt(ConvParams p) {
  using K = CuCfg<W>;
  constexpr int R = K::R, SW = K::SW, SPW = K::SPW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int cg = wave & 3, pg = wave >> 2;
  const int H = p.H;
  const int nb = (H + R - 1) / R;                   // bands per utterance
  const int T = p.N * nb;
  int t_first, t_step, ntiles;
  {
    const int G = gridDim.x;
    if ((G & 7) == 0) {
      const int x = blockIdx.x & 7, bi = blockIdx.x >> 3, nbk = G >> 3;
      const int b0 = (int)((long)x * T / 8), b1 = (int)((long)(x + 1) * T / 8);
      t_first = b0 + bi;
      t_step = nbk;
      ntiles = t_first < b1 ? (b1 - t_first + nbk - 1) / nbk : 0;
    } else {
      t_first = blockIdx.x;
      t_step = G;
      ntiles = t_first < T ? (T - t_first + G - 1) / G : 0;
    }
  }
  if (ntiles == 0) return;

  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(p.x);
  const bf16_t* __restrict__ Wt = reinterpret_cast<const bf16_t*>(p.w);
  const bf16_t* __restrict__ XZ = reinterpret_cast<const bf16_t*>(p.res);
  bf16_t* __restrict__ Y = reinterpret_cast<bf16_t*>(p.y);
  bf16_t* __restrict__ Z = reinterpret_cast<bf16_t*>(p.y2);
  const bf16_t* zero = reinterpret_cast<const bf16_t*>(g_cu_zero);
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  const uint32_t ring0 = lds0 + (uint32_t)K::WBUF;
  const char* ring = smem + K::WBUF;

  // weight piece of k-step s: cout rows 16 wave + lane/4, LDS position lane%4
  // holds source chunk (lane%4) ^ swz(row)
  const int wrow = 16 * wave + (lane >> 2);
  const bf16_t* wsrc = Wt + (size_t)wrow * (9 * CU_C) + 8 * ((lane & 3) ^ cu_swz(wrow));
  auto issue_w = [&](int s) __attribute__((always_inline)) {
    // the k offset laundered into a VGPR: otherwise the compiler precomputes a
    // 64-bit source per unrolled step and spills them (reloads wait vmcnt(0))
    int ko = 32 * s;
    asm volatile("" : "+v"(ko));
    cu_glds16(wsrc + ko, ring0 + (uint32_t)(s % CU_NST) * CU_WSLOT + (uint32_t)wave * 1024u);
  };
  // A fragment offsets (cout tile i of this wave's group), chunk g swizzled
  int aoff[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int r = 48 * cg + 16 * i + col;
    aoff[i] = r * 64 + ((g ^ cu_swz(r)) << 4);
  }
  // B fragment base of pixel tile j (window slot of the lane's pixel, sub-plane
  // g/2, parity g%2); + per k-step 2 (s%6) SPW units and the tap's slot shift
  const int cb = ((g >> 1) * SPW + (g & 1)) * 16;

  for (int tj = 0; tj < ntiles; ++tj) {
    const int id = t_first + tj * t_step;
    const int n = id / nb, band = id - n * nb;
    const int r0 = band * R;
    const int rb = min(R, H - r0);                  // rows of this band
    const int npx = rb * W;
    const int hn = p.vlen ? valid_rows(p.vlen, p.vsh, n, H) : H;   // ragged batch: padding past hn
    // ---- window of the band: rows r0-1 .. r0+rb (zero outside the image)
    for (int q = wave; q < K::WPC; q += CU_NW) {
      int u = lane;
      asm volatile("" : "+v"(u));
      u += 64 * q;
      const int sp = u / SPW, rem = u - sp * SPW;
      const int slot = rem >> 1, c = 2 * sp + (rem & 1);
      const int rr = slot / SW, cc = slot - rr * SW;
      const int r = r0 - 1 + rr, wc = cc - 1;
      const bf16_t* src = zero;
      if (sp < CU_NCH / 2 && cc > 0 && rr <= rb + 1 && r >= 0 && r < hn)
        src = X + (((size_t)n * H + r) * W + wc) * p.ldx + c * 8;
      cu_glds16(src, lds0 + (uint32_t)q * 1024u);
    }
    issue_w(0);
    issue_w(1);
    cu_wait_vm<1>();   // window + step 0 landed (this wave's pieces)
    __syncthreads();

    int bb[CU_PG];
    int tcol = col;
    asm volatile("" : "+v"(tcol));   // (formed per tile, not hoisted out of the tile loop)
#pragma unroll
    for (int j = 0; j < CU_PG; ++j) {
      const int px = min(16 * (CU_PG * pg + j) + tcol, npx - 1);
      const int slot = (px / W + 1) * SW + (px % W) + 1;
      bb[j] = cb + 32 * slot;
    }
    f32x4 acc[3][CU_PG];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < CU_PG; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // taps as a rolled loop (a fully unrolled K loop let the scheduler hoist
    // reads across k-steps and spill), the 6 k-steps of a tap unrolled.  The
    // window (B operand) is fixed for the band, so step s + 1's B fragments are
    // requested at the end of step s, after its MFMAs (same registers), and
    // land while the waves meet at the next step's barrier.
    bf16x8 b[CU_PG];
    auto read_b = [&](int toff) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < CU_PG; ++j) {
        int ad = bb[j] + toff;
        asm volatile("" : "+v"(ad));   // one add per read, nothing precomputed per k-step
        b[j] = *reinterpret_cast<const bf16x8*>(smem + ad);
      }
    };
    read_b(32 * (-SW - 1));   // tap 0, part 0
    for (int tap = 0; tap < 9; ++tap) {
      const int tsh = 32 * ((tap / 3 - 1) * SW + (tap % 3 - 1));
      const int tn = tap < 8 ? tap + 1 : tap;   // (the last prefetch is unused)
      const int tsh_n = 32 * ((tn / 3 - 1) * SW + (tn % 3 - 1));
#pragma unroll
      for (int part = 0; part < 6; ++part) {
        const int s = tap * 6 + part;
        __builtin_amdgcn_sched_barrier(0);
        // (also at s = 0, where it is a no-op: a peeled first step spilled an
        // accumulator through the whole first tap)
        if (s + 1 < CU_KS) cu_wait_vm<1>(); else cu_wait_vm<0>();
        __syncthreads();   // step s landed for every wave; slot (s+2)%3 released
        if (s + 2 < CU_KS) issue_w(s + 2);
        const char* L = ring + (s % CU_NST) * CU_WSLOT;
        bf16x8 a[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) a[i] = *reinterpret_cast<const bf16x8*>(L + aoff[i]);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < CU_PG; ++j) acc[i][j] = mfma_step(a[i], b[j], acc[i][j]);
        __builtin_amdgcn_sched_barrier(0);
        read_b(part < 5 ? tsh + (part + 1) * 2 * SPW * 16 : tsh_n);   // B of step s + 1
      }
    }

    // ---- epilogue: lane (col, g) holds couts co .. co+3 of pixel 16 t + col.
    // The lane indices are laundered here so the epilogue's addresses are
    // formed after the k-loop: loop-invariant, they were hoisted out of the
    // tile loop and held live across it (spilled: 92 / 76 B of scratch per lane)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int ecol = ln & 15, eg = ln >> 4;
    const size_t pbase = ((size_t)n * H + r0) * W;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int co = 48 * cg + 16 * i + 4 * eg;
      const f32x4 m = *reinterpret_cast<const f32x4*>(p.mean + co);
      const f32x4 iv = *reinterpret_cast<const f32x4*>(p.inv + co);
#pragma unroll
      for (int jj = 0; jj < CU_PG / 2; ++jj) {
        // pixel tiles 2 jj, 2 jj + 1: one half-row exchange per dword gives each
        // lane 8 contiguous couts (g even: tile 2 jj, couts 16 i + 8 (g / 2);
        // g odd: tile 2 jj + 1), so y and z go out as 16-B stores, half the
        // store instructions of the 8-B ones (T21 with v_permlane16_swap)
        unsigned d[2][2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          bf16x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = (bf16_t)fmaxf((acc[i][2 * jj + t][e] - m[e]) * iv[e], 0.f);
          const uint2 u = __builtin_bit_cast(uint2, o);
          d[t][0] = u.x;
          d[t][1] = u.y;
        }
        const auto s0 = __builtin_amdgcn_permlane16_swap(d[0][0], d[1][0], false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(d[0][1], d[1][1], false, false);
        const u32x4 yc = {s0[0], s1[0], s0[1], s1[1]};
        const int px = 16 * (CU_PG * pg + 2 * jj + (eg & 1)) + ecol;
        const int cq = 48 * cg + 16 * i + 8 * (eg >> 1);
        if (px < npx) {
          *reinterpret_cast<u32x4*>(Y + (pbase + px) * p.ldy + cq) = yc;
          if (HAS_Z) {
            const bf16x8 xv = *reinterpret_cast<const bf16x8*>(XZ + (pbase + px) * p.ldr + cq);
            const bf16x8 ov = __builtin_bit_cast(bf16x8, yc);
            bf16x8 zv;
#pragma unroll
            for (int e = 0; e < 8; ++e) zv[e] = (bf16_t)((float)xv[e] + (float)ov[e]);
            *reinterpret_cast<bf16x8*>(Z + (pbase + px) * p.ldy2 + cq) = zv;
          }
        }
      }
    }
    // the next band's window and ring reuse the LDS every wave has just read
    cu_wait_vm<0>();
    __syncthreads();
  }
}

int conv3_utt_ok(const ConvParams& p) {
  if (p.Cin != CU_C || p.Cout != CU_C || p.kh != 3 || p.kw != 3 || p.groups != 1) return 0;
  if (p.sh != 1 || p.sw != 1 || p.dh != 1 || p.dw != 1 || p.ph != 1 || p.pw != 1) return 0;
  if (p.Ho != p.H || p.Wo != p.W || p.W != 10) return 0;
  if (p.ldx % 8 || p.ldy % 8 || p.ldr % 8 || p.ldy2 % 8) return 0;   // 16-B epilogue stores
  if (p.flags != (EPI_AFFINE | EPI_RELU) || p.in_mean || p.x2 || !p.mean || !p.inv) return 0;
  if (p.y2 && p.y2 != p.res) return 0;   // z_{k+1} in place over x_{k+1}
  return p.N * p.H * p.W > 0;
}

hipError_t launch_conv3_utt(const ConvParams& p, int num_cu, hipStream_t s) {
  if (!conv3_utt_ok(p)) return hipErrorInvalidValue;
  using K = CuCfg<10>;
  const int T = p.N * ((p.H + K::R - 1) / K::R);
  int G = num_cu < T ? num_cu : T;
  if (G >= 8) G = G / 8 * 8;
  if (p.y2)
    hipLaunchKernelGGL((conv3x3_utt<10, true>), dim3(G), dim3(CU_NT), K::LDS, s, p);
  else
    hipLaunchKernelGGL((conv3x3_utt<10, false>), dim3(G), dim3(CU_NT), K::LDS, s, p);
  return hipGetLastError();
}

}  // namespace vox

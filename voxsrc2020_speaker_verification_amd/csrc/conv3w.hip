// Window-staged pipelined 3x3 conv for the w = 96 stride-1 Res2Net branches
// (res2net_pad_conv_bn_relu, res2net_model.py:53-75, layer 3): the same tile
// (256 pixels x 96 couts), MFMA layout, K order and epilogue as
// conv3x3_pipe (conv3.hip), with a different operand stream.
//
// conv3x3_pipe gathers the im2col operand by DMA: every K-step fetches 256
// shifted pixel rows, so each input pixel crosses the CU's memory pipe 9
// times (608 KB per tile with the weights), and the kernel runs at the
// per-CU fill rate (~25-30 GB/s measured).  Here each tile's input rows are
// fetched ONCE into an LDS window (the <= 16 image rows the 256 pixels and
// their 3x3 halo touch, zero-padded columns, 3 planes of 32 channels with
// 64-B pixel slots), double-buffered so the next tile's window streams in
// under this tile's K-steps; only the weights (6 KB per K-step) go through
// the 4-slot DMA ring.  The B fragments of K-step (tap, plane) are read
// straight from the window at the tap's offset; taps outside the utterance
// read a zero pad slot.  243 KB per tile instead of 608 KB.
//
// DMA bookkeeping: a K-step's ring fill is 6 pieces (waves 0-5) plus, in
// load-steps 3..24 of a tile, 3 pieces of the next tile's window (piece i of
// a step goes to wave i % 8); every wave counts what it issued per step and
// waits with vmcnt = its ops issued after the awaited weight piece.
// LDS slot swizzle: 16-B chunk c of 64-B slot r sits at c ^ f(r & 15 >> 2).
// Accumulation order = K chunks of 32 increasing: bitwise equal to
// conv3x3_pipe and the generic conv.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_common.h"
#include "kernels.h"

namespace vox {

namespace {
constexpr int CW_BM = 256;      // pixels per tile
constexpr int CW_CIN = 96;      // branch width (= Cout)
constexpr int CW_NT = 512;      // 8 waves x 32 pixels
constexpr int CW_NST = 4;       // weight ring slots
constexpr int CW_WSLOT = CW_CIN * 64;   // 6 KB: 96 cout rows x 32 K
constexpr int CW_KT = 9 * CW_CIN / 32;  // 27 K-steps
constexpr int CW_WIN_LS0 = 3;   // load-steps of a tile that carry next-window pieces
constexpr int CW_WIN_PER = 3;   // window pieces per such load-step

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void cw_glds16(const void* src, uint32_t lds) {
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
__device__ __forceinline__ u32x4 cw_gld16(const void* src) {
  u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(src) : "memory");
  return v;
}
__device__ __forceinline__ void cw_gst16(void* dst, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" : : "v"(dst), "v"(v) : "memory");
}
#define CW_W(n) \
  case n: asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory"); break;
__device__ __forceinline__ void cw_wait_vm(int n) {
  switch (n) {
    CW_W(0) CW_W(1) CW_W(2) CW_W(3) CW_W(4) CW_W(5) CW_W(6) CW_W(7) CW_W(8) CW_W(9)
    CW_W(10) CW_W(11) CW_W(12) CW_W(13) CW_W(14) CW_W(15) CW_W(16) CW_W(17) CW_W(18)
    CW_W(19) CW_W(20) CW_W(21) CW_W(22) CW_W(23) CW_W(24) CW_W(25) CW_W(26) CW_W(27)
    CW_W(28) CW_W(29) CW_W(30) CW_W(31) CW_W(32) CW_W(33) CW_W(34) CW_W(35) CW_W(36)
    CW_W(37) CW_W(38) CW_W(39) CW_W(40) CW_W(41) CW_W(42) CW_W(43) CW_W(44) CW_W(45)
    CW_W(46) CW_W(47) CW_W(48) CW_W(49) CW_W(50) CW_W(51) CW_W(52) CW_W(53) CW_W(54)
    CW_W(55) CW_W(56) CW_W(57) CW_W(58) CW_W(59) CW_W(60) CW_W(61) CW_W(62)
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
  __builtin_amdgcn_sched_barrier(0);
}
#undef CW_W
__device__ __forceinline__ int cw_swz(int r) { return (4 - ((r >> 2) & 3)) & 3; }
}  // namespace

__device__ uint4 g_cw_zero[4] = {};
__device__ uint4 g_cw_sink[64];

template <int W>
struct CwCfg {
  static constexpr int SW = W + 2;                         // slots per window row
  static constexpr int RMAX = (CW_BM + W - 1 + W - 1) / W + 2;   // rows a tile + halo touches
  static constexpr int PLANE = RMAX * SW * 64;             // bytes per 32-channel plane
  static constexpr int WIN = 3 * PLANE;                    // one window
  static constexpr int WPIECES = (WIN + 1023) / 1024;      // 1-KB DMA pieces per window
  static constexpr int WINA = WPIECES * 1024;               // window buffer stride
  static constexpr int LDS = 2 * WINA + CW_NST * CW_WSLOT;
  static_assert(WPIECES <= CW_WIN_PER * (CW_KT - 2 - CW_WIN_LS0), "window must land in time");
  static_assert(LDS <= 163840, "LDS");
};

#pragma clang fp contract(off)
template <int W, bool HAS_Z>
__global__ __launch_bounds__(CW_NT) __attribute__((amdgpu_waves_per_eu(2, 2)))
void conv3x3_win(ConvParams p) {
  using K = CwCfg<W>;
  constexpr int SW = K::SW, PLANE = K::PLANE, WIN = K::WIN, WINA = K::WINA;
  constexpr int KT = CW_KT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int H = p.H;
  const int M = p.N * H * W;
  const int TR = p.N * H;                 // rows of the tall image (utterances stacked)
  const int T = (M + CW_BM - 1) / CW_BM;
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
  const bf16_t* zero = reinterpret_cast<const bf16_t*>(g_cw_zero);
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  const uint32_t ring0 = lds0 + 2 * WINA;
  const int ldx = p.ldx;

  // ---- DMA sources
  // weight piece (wave < 6): 16 ring rows 16*wave + lane/4, position lane%4 ->
  // source chunk (lane%4) ^ f(row); row r holds output channel perm(r)
  const bf16_t* wsrc = zero;
  if (wave < 6) {
    const int r = 16 * wave + (lane >> 2);
    const int ch = 32 * (r >> 5) + 8 * ((r & 15) >> 2) + 4 * ((r >> 4) & 1) + (r & 3);
    wsrc = Wt + (size_t)ch * (9 * CW_CIN) + ((lane & 3) ^ cw_swz(r)) * 8;
  }
  // window piece q of tile tj: LDS bytes [1024 q, 1024 q + 1024) of its window
  auto win_src = [&](int tj, int q) -> const bf16_t* {
    const int idx = q * 64 + lane;              // 16-B unit of the window
    if (idx * 16 >= WIN) return zero;
    const int plane = idx / (PLANE / 16);
    const int rem = idx - plane * (PLANE / 16);
    const int slot = rem >> 2, pos = rem & 3;   // slot = row * SW + column
    const int row = slot / SW, sc = slot - row * SW;
    const int px0 = (t_first + tj * t_step) * CW_BM;
    const int tr = px0 / W - 1 + row;           // tall-image row
    const int wc = sc - 1;                      // image column
    if (tr < 0 || tr >= TR || wc < 0 || wc >= W) return zero;
    return X + ((size_t)tr * W + wc) * ldx + plane * 32 + ((pos ^ cw_swz(slot)) * 8);
  };

  // per-step op counts of this wave for steps s-1, s-2, s-3: a = ops after
  // its weight piece (all ops when it has none), t = all ops
  int a1 = 0, a2 = 0, a3 = 0, t1 = 0, t2 = 0;
  int l_tile = 0, l_k = 0;
  // issue load-step (l_tile, l_k): weight piece into ring slot, next-window
  // pieces into window buffer (l_tile + 1) & 1; returns (after, total)
  auto issue = [&](int rslot, int& na, int& nt) {
    na = nt = 0;
    if (wave < 6) {
      cw_glds16(wsrc + (size_t)l_k * 32, ring0 + (uint32_t)rslot * CW_WSLOT + (uint32_t)wave * 1024u);
      ++nt;
    }
    if (l_k >= CW_WIN_LS0 && l_tile + 1 < ntiles) {
      const int q0 = (l_k - CW_WIN_LS0) * CW_WIN_PER;
#pragma unroll
      for (int i = 0; i < CW_WIN_PER; ++i) {
        const int pi = 6 + i;                   // piece index within the step
        const int q = q0 + i;
        if ((pi & 7) == wave && q < K::WPIECES) {
          cw_glds16(win_src(l_tile + 1, q), lds0 + (uint32_t)((l_tile + 1) & 1) * WINA + (uint32_t)q * 1024u);
          ++na;
          ++nt;
        }
      }
    }
    if (wave >= 6) na = nt;
    // advance; past the last tile the final step is re-read (never consumed)
    if (l_k + 1 < KT) {
      ++l_k;
    } else if (l_tile + 1 < ntiles) {
      ++l_tile;
      l_k = 0;
    }
  };

  // prologue: tile 0's window (all pieces, waves round-robin), then load-steps 0..2
  for (int q = wave; q < K::WPIECES; q += 8) cw_glds16(win_src(0, q), lds0 + (uint32_t)q * 1024u);
  {
    int na, nt;
    issue(0, na, nt);   // these three are older than anything the loop waits past
    issue(1, na, nt);
    issue(2, na, nt);
  }

  f32x4 acc[6][2];
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bf16_t* __restrict__ XZ = reinterpret_cast<const bf16_t*>(p.res);
  bf16_t* __restrict__ Y = reinterpret_cast<bf16_t*>(p.y);
  bf16_t* __restrict__ Z = reinterpret_cast<bf16_t*>(p.y2);
  const int offa = col * 64 + ((g ^ cw_swz(col)) << 4);   // + 1024 i per A fragment

  // per-lane geometry of the two pixel blocks of the current tile
  int wrow[2], wcol[2], okm[2];   // okm bit0: row above in utterance, bit1: below, bit2: pixel < M
  auto set_tile_geom = [&](int tj) {
    const int px0 = (t_first + tj * t_step) * CW_BM;
    const int rt0 = px0 / W;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int pix = min(px0 + 32 * wave + 16 * j + col, M - 1);
      const int rt = pix / W, wc = pix - rt * W, h = rt % H;
      wrow[j] = rt - rt0;
      wcol[j] = wc;
      okm[j] = (h > 0 ? 1 : 0) | (h < H - 1 ? 2 : 0);
    }
  };
  set_tile_geom(0);

  constexpr int LEAD = 2;
  constexpr int L0 = KT - 1 - LEAD;
  u32x4 bm[3][2], bi[3][2], xz[3][2];
  int c_tile = 0, c_k = 0;
  for (int s = 0; s < S; ++s) {
    // step s's weight piece landed (and, at a tile start, the tile's window:
    // its pieces are older); younger = ops after it in step s-3 + steps s-2, s-1
    if (s >= 3) cw_wait_vm(a3 + t2 + t1);
    else if (s == 0) cw_wait_vm(0);   // prologue: window 0 and load-steps 0..2 (drained once)
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const int lid = t_first + c_tile * t_step;
    const int px0 = lid * CW_BM;
    int na, nt;
    issue((s + 3) & 3, na, nt);
    if (c_k == L0) {
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int ch = 32 * q + 8 * g;
        bm[q][0] = cw_gld16(p.mean + ch);
        bm[q][1] = cw_gld16(p.mean + ch + 4);
        bi[q][0] = cw_gld16(p.inv + ch);
        bi[q][1] = cw_gld16(p.inv + ch + 4);
        if (HAS_Z) {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int pix = min(px0 + wave * 32 + 16 * j + col, M - 1);
            xz[q][j] = cw_gld16(XZ + (size_t)pix * p.ldr + ch);
          }
        }
      }
      na += HAS_Z ? 18 : 12;
      nt += HAS_Z ? 18 : 12;
    }
    __builtin_amdgcn_sched_barrier(0);
    {
      // K-step c_k = (tap, plane): A from the ring, B from the window
      const char* L = smem + 2 * WINA + (s & 3) * CW_WSLOT;
      const int tap = c_k / 3, plane = c_k - 3 * (c_k / 3);
      const int ky = tap / 3, kx = tap - 3 * ky;
      const char* Wn = smem + (c_tile & 1) * WINA + plane * PLANE;
      bf16x8 a[6], b[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bool ok = (ky == 0 ? (okm[j] & 1) : (ky == 2 ? (okm[j] & 2) : 1)) != 0;
        const int slot = ok ? (wrow[j] + ky) * SW + wcol[j] + kx : 0;
        b[j] = *reinterpret_cast<const bf16x8*>(Wn + slot * 64 + ((g ^ cw_swz(slot)) << 4));
      }
#pragma unroll
      for (int i = 0; i < 6; ++i) a[i] = *reinterpret_cast<const bf16x8*>(L + offa + i * 1024);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma_step(a[i], b[j], acc[i][j]);
    }
    if (c_k == KT - 1) {
      // epilogue operands: younger than them = everything issued in steps
      // L0+1 .. KT-1 (this step's DMA included)
      {
        static_assert(LEAD == 2, "ops younger than the epilogue loads: this step's and step s-1's");
        cw_wait_vm(nt + t1);
        asm volatile("" : "+v"(bm[0][0]), "+v"(bm[0][1]), "+v"(bm[1][0]), "+v"(bm[1][1]),
                          "+v"(bm[2][0]), "+v"(bm[2][1]), "+v"(bi[0][0]), "+v"(bi[0][1]),
                          "+v"(bi[1][0]), "+v"(bi[1][1]), "+v"(bi[2][0]), "+v"(bi[2][1]));
        if (HAS_Z)
          asm volatile("" : "+v"(xz[0][0]), "+v"(xz[0][1]), "+v"(xz[1][0]), "+v"(xz[1][1]),
                            "+v"(xz[2][0]), "+v"(xz[2][1]));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int ch = 32 * q + 8 * g;
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
          cw_gst16(in ? (void*)(Y + (size_t)pix * p.ldy + ch) : (void*)&g_cw_sink[lane],
                   __builtin_bit_cast(u32x4, o));
          if (HAS_Z) {
            const bf16x8 xv = __builtin_bit_cast(bf16x8, xz[q][j]);
            bf16x8 zv;
#pragma unroll
            for (int e = 0; e < 8; ++e) zv[e] = (bf16_t)((float)xv[e] + (float)o[e]);
            cw_gst16(in ? (void*)(Z + (size_t)pix * p.ldy2 + ch) : (void*)&g_cw_sink[lane],
                     __builtin_bit_cast(u32x4, zv));
          }
        }
      }
      na += HAS_Z ? 12 : 6;
      nt += HAS_Z ? 12 : 6;
#pragma unroll
      for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      c_k = 0;
      ++c_tile;
      if (c_tile < ntiles) set_tile_geom(c_tile);
    } else {
      ++c_k;
    }
    a3 = a2;
    a2 = a1;
    a1 = na;
    t2 = t1;
    t1 = nt;
  }
  // drain: the trailing (never consumed) DMA must land before the workgroup
  // releases its LDS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int conv3_win_ok(const ConvParams& p) {
  if (p.Cin != CW_CIN || p.Cout != CW_CIN || p.kh != 3 || p.kw != 3 || p.groups != 1) return 0;
  if (p.sh != 1 || p.sw != 1 || p.dh != 1 || p.dw != 1 || p.ph != 1 || p.pw != 1) return 0;
  if (p.Ho != p.H || p.Wo != p.W || !(p.W == 20 || p.W == 10)) return 0;
  if (p.ldx % 8 || p.ldy % 8 || p.ldr % 8 || p.ldy2 % 8) return 0;
  if (p.flags != (EPI_AFFINE | EPI_RELU) || p.in_mean || p.x2 || !p.mean || !p.inv) return 0;
  if (p.y2 && !p.res) return 0;
  return p.N * p.H * p.W > 0;
}

template <int W, bool Z>
static void launch_cw(const ConvParams& p, int G, hipStream_t s) {
  hipLaunchKernelGGL((conv3x3_win<W, Z>), dim3(G), dim3(CW_NT), CwCfg<W>::LDS, s, p);
}

hipError_t launch_conv3_win(const ConvParams& p, int num_cu, hipStream_t s) {
  if (!conv3_win_ok(p)) return hipErrorInvalidValue;
  const bool z = p.y2 != nullptr;
  const int M = p.N * p.H * p.W;
  const int T = (M + CW_BM - 1) / CW_BM;
  int G = num_cu < T ? num_cu : T;
  if (G >= 8) G = G / 8 * 8;
  if (p.W == 20) {
    if (z) launch_cw<20, true>(p, G, s); else launch_cw<20, false>(p, G, s);
  } else {
    if (z) launch_cw<10, true>(p, G, s); else launch_cw<10, false>(p, G, s);
  }
  return hipGetLastError();
}

}  // namespace vox

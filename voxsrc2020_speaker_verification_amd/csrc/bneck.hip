// Fused Res2Net identity bottleneck (stride 1, identity shortcut), bf16:
//
//   x   = relu(bn_a(conv1x1_a(in)))                  split into S planes x_1..x_S
//   y_1 = relu(bn_1(conv3x3_1(x_1)))
//   y_k = relu(bn_k(conv3x3_k(x_k + y_{k-1})))       k = 2..S-1
//   out = relu(bn_c(conv1x1_c([y_1 .. y_{S-1}, x_S])) + in)
//
// (res2net_model.py:26-103, one `block` with stype 'normal'.)  The unfused
// path moves every intermediate through HBM three times (1x1a -> split chain
// -> 1x1c, ~1.5 KB per pixel at 128 channels); here a workgroup streams one
// utterance segment row by row (time = image rows) and keeps every
// intermediate in LDS ring buffers, so HBM sees the block input once and the
// block output once (~0.5 KB per pixel).
//
// Row pipeline, two phases (one barrier each) per step; step t handles
// A-row a = h0-(S-1)+t:
//   phase 0 : 1x1a on row a (input row staged in LDS)       -> rings x_1..x_S
//             1x1c on row a-2(S-1) (rings y_1..y_{S-1}, x_S) -> HBM (+ residual)
//   phase 1 : every 3x3 stage k at once, on row a-2k+1 (ring z_k rows
//             a-2k..a-2k+2, all written in earlier steps or phase 0)
//             -> ring y_k, and z_{k+1} = x_{k+1} + y_k (bf16, as unfused)
// Ring depths follow from the lags: z_k 4 rows, x_k 2k-2, x_S 2S-1,
// y_k 2S-1-2k.  Rows outside the image are zero (SAME padding).  Segments
// recompute 3(S-1) warm-up rows.
//
// Work split (8 waves): phase 0 -- waves 0..NPA-1 own one 32-channel pair of
// 1x1a outputs, waves NW-NPC..NW-1 one pair of 1x1c outputs, each across all
// pixel tiles, with that pair's weights held in registers for the whole
// kernel; phase 1 -- wave w < (S-1)*WCO owns 3x3 stage w/WCO+1, cout tile
// w % WCO (its weights in registers) across all pixel tiles, two pixel tiles'
// MFMA chains interleaved.
// Accumulation orders (K chunks of 32, paired-row 1x1 weights, flattened
// tap-major 3x3 K) equal the unfused kernels', so results are bit-identical.
#include "kernels.h"
#include "device_common.h"

namespace vox {

template <int CI, int C, int WID, int S, int PT>
struct BneckCfg {
  static constexpr int NW = 8, NT = 64 * NW;
  static constexpr bool PROJ = CI != C;              // projection shortcut (block 0)
  static constexpr int KSP = CI / 32;                // its k-steps
  static constexpr int SW = S * WID;
  static constexpr int NPA = SW / 32, KSA = CI / 32; // 1x1a: output pairs, k-steps
  static constexpr int NPC = C / 32, KSC = SW / 32;  // 1x1c
  static constexpr int KSW = KSA > KSC ? KSA : KSC;
  static constexpr int WCO = (WID + 15) / 16;        // 3x3 cout tiles
  static constexpr int KFLAT = 9 * WID;
  static constexpr int KCP = (KFLAT + 31) / 32 * 32;
  static constexpr int KST = KCP / 32;
  static constexpr int AU = ((WID / 8) & 1) ? WID / 8 : WID / 8 + 1;  // odd 16-B units
  static constexpr int ASTR = AU * 16;                                // ring pixel stride
  static constexpr int IU = ((CI / 8) & 1) ? CI / 8 : CI / 8 + 1;
  static constexpr int ISTR = IU * 16;                                // input-row pixel stride
  static constexpr int WR = 16 * PT + 2;  // ring row: pad | pixels | pad (+ tile slack)
  static constexpr int ROWB = WR * ASTR;
  // ring planes (one image row each) and depths
  // z_k: 4 rows each (k = 1..S-1), so a stage's three tap rows wrap with a mask
  static constexpr int ZB(int k) { return 4 * (k - 1); }
  static constexpr int ZEND = 4 * (S - 1);
  static constexpr int XD(int k) { return k == S ? 2 * S - 1 : 2 * k - 2; }
  static constexpr int XB(int k) { return ZEND + (k - 2) * (k - 1); }       // x_k, k = 2..S
  static constexpr int XEND = XB(S) + 2 * S - 1;
  static constexpr int YD(int k) { return 2 * S - 1 - 2 * k; }
  static constexpr int YB(int k) { return XEND + (k - 1) * (2 * S - 1 - k); } // y_k, k = 1..S-1
  static constexpr int NPLANES = XEND + (S - 1) * (S - 1);
  static constexpr int LAG_C = 2 * (S - 1);  // 1x1c row = A row - LAG_C
  static constexpr int RING_BYTES = NPLANES * ROWB;
  static constexpr int IN_BYTES = 16 * PT * ISTR;
  static constexpr int BN_FLOATS = 2 * (S - 1) * 16 * WCO + 2 * SW + 2 * C + (PROJ ? 2 * C : 0);
  static constexpr int KP = (KST + 1) / 2;
  static constexpr int KTB = 64 * KP * 4;   // tap table [lane][k-step] u16
  static constexpr int LDS = RING_BYTES + IN_BYTES + KTB + 4 * BN_FLOATS;
  static_assert(4 * ROWB < 65536, "tap offsets in 16 bits");
  static_assert(LDS <= 163840, "LDS");
  static constexpr int CU = CI / 8;                           // 16-B chunks per input pixel
  static constexpr int IREG = (16 * PT * CU + NT - 1) / NT;   // input-row chunks per thread
};

// ring slot of image row r (r >= -840) in a ring of `depth` rows
template <int D> __device__ __forceinline__ int slot(int r) { return (r + 840) % D; }

__device__ __forceinline__ bf16x4 add4(bf16x4 a, bf16x4 b) {
  bf16x4 r;
#pragma unroll
  for (int e = 0; e < 4; ++e) r[e] = (bf16_t)((float)a[e] + (float)b[e]);
  return r;
}

__device__ uint4 g_vox_zero[4] = {};   // source of the row loads outside the image

// diagnostics (VOXEMB_BNECK_DBG bit 256): per-step shader-clock stamps of
// block 0, [wave][step][start, phase-0 done, phase 1 start, phase-1 done]
__device__ unsigned long long g_vox_trace[8 * 512 * 4];

template <int CI, int C, int WID, int S, int PT>
__global__ __launch_bounds__(512) void bneck_fused(BneckParams q) {
  using K = BneckCfg<CI, C, WID, S, PT>;
  static_assert(!K::PROJ || K::KSP == 1, "projection shortcut: one k-step (Cin 32)");
  constexpr int NW = K::NW, NT = K::NT, WCO = K::WCO, KST = K::KST;
  constexpr int ASTR = K::ASTR, ROWB = K::ROWB;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar ring math
  const int col = lane & 15, g = lane >> 4;
  const int H = q.H, W = q.W;
  const int n = blockIdx.x / q.nseg;
  const int h0 = (blockIdx.x - n * q.nseg) * q.seg;
  const int h1 = min(H, h0 + q.seg);
  // ragged batch: rows at or past Hn are this utterance's padding (zeros in the rings)
  const int Hn = valid_rows(q.vlen, q.vsh, n, H);
  char* rings = smem;
  char* inb = smem + K::RING_BYTES;
  unsigned short* ktl = reinterpret_cast<unsigned short*>(inb + K::IN_BYTES);
  float* bmb = reinterpret_cast<float*>(inb + K::IN_BYTES + K::KTB);   // [S-1][16*WCO]
  float* bib = bmb + (S - 1) * 16 * WCO;
  float* bma = bib + (S - 1) * 16 * WCO;                      // 1x1a BN [SW]
  float* bia = bma + K::SW;
  float* bmc = bia + K::SW;                                   // 1x1c BN [C]
  float* bic = bmc + C;
  float* bmp = bic + C;                                       // projection BN [C]
  float* bip = bmp + C;
  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(q.x);
  bf16_t* __restrict__ Y = reinterpret_cast<bf16_t*>(q.y);
  const size_t img = (size_t)n * H * W;

  for (int i = tid; i < K::RING_BYTES / 16; i += NT)
    reinterpret_cast<uint4*>(rings)[i] = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int k = 0; k < S - 1; ++k)
    for (int c = tid; c < 16 * WCO; c += NT) {
      bmb[k * 16 * WCO + c] = c < WID ? -q.mb[k][c] : 0.f;
      bib[k * 16 * WCO + c] = c < WID ? q.ib[k][c] : 0.f;
    }
  for (int c = tid; c < K::SW; c += NT) { bma[c] = -q.ma[c]; bia[c] = q.ia[c]; }
  for (int c = tid; c < C; c += NT) { bmc[c] = -q.mc[c]; bic[c] = q.ic[c]; }
  if (K::PROJ)
    for (int c = tid; c < C; c += NT) { bmp[c] = -q.mp[c]; bip[c] = q.ip[c]; }

  // ---- per-wave constant operands
  const bool is_a = wave < K::NPA;
  const bool is_c = wave >= NW - K::NPC;
  // (diagnostics: VOXEMB_BNECK_DBG 2048 = static priority 1 for the 1x1c waves,
  // the longest phase-0 role)
  if ((VOX_DBG(q) & 2048) && is_c) __builtin_amdgcn_s_setprio(1);
  const int pq = is_a ? wave : wave - (NW - K::NPC);   // 1x1 pair of this wave
  bf16x8 w1[K::KSW][2];
  {
    const bf16_t* __restrict__ Wp = reinterpret_cast<const bf16_t*>(is_a ? q.wa : q.wc);
    const int kp = is_a ? CI : K::SW;
    const int ks = is_a ? K::KSA : K::KSC;
#pragma unroll
    for (int s = 0; s < K::KSW; ++s)
#pragma unroll
      for (int u = 0; u < 2; ++u)
        w1[s][u] = ((is_a || is_c) && s < ks)
                       ? ld16(Wp + (size_t)((2 * pq + u) * 16 + col) * kp + 32 * s + 8 * g)
                       : bf16x8{};
  }
  // this lane's 8 BN channels of its 1x1 pair (LDS)
  const float* bn1m = (is_a ? bma : bmc) + 32 * pq + 8 * g;
  const float* bn1i = (is_a ? bia : bic) + 32 * pq + 8 * g;
  // projection shortcut pair of a 1x1c wave (block 0): weights in registers
  bf16x8 wp[2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
    wp[u] = (K::PROJ && is_c)
                ? ld16(reinterpret_cast<const bf16_t*>(q.wp) + (size_t)((2 * pq + u) * 16 + col) * CI + 8 * g)
                : bf16x8{};
  static_assert((S - 1) * WCO <= NW, "one (stage, cout tile) per wave");
  const bool chain_wave = wave < (S - 1) * WCO;
  const int ck = chain_wave ? wave / WCO + 1 : 1;     // 3x3 stage of this wave
  const int ci = wave % WCO;                          // its cout tile
  bf16x8 wb[KST];
  {
    const void* wk = q.wb[0];
#pragma unroll
    for (int k = 1; k < S - 1; ++k)
      if (ck == k + 1) wk = q.wb[k];
    const bf16_t* __restrict__ Wk = reinterpret_cast<const bf16_t*>(wk);
#pragma unroll
    for (int s = 0; s < KST; ++s) {
      const int kk = 32 * s + 8 * g;
      wb[s] = (chain_wave && kk < K::KFLAT)
                  ? ld16(Wk + (size_t)(ci * 16 + col) * K::KFLAT + kk) : bf16x8{};
    }
  }
  // tap table: for lane l and k-step s, the byte offset of its B fragment (pixel
  // tile 0) in a 4-row z ring, counted from the ring row of tap row 0
  for (int e = tid; e < 64 * KST; e += NT) {
    const int l = e / KST, st = e - l * KST;
    const int kk = 32 * st + 8 * (l >> 4);
    int dyi = 1, off = 0;
    if (kk < K::KFLAT) {
      const int tap = kk / WID, ch = kk - tap * WID;
      dyi = tap / 3;
      off = (tap % 3 - 1) * ASTR + ch * 2;
    }
    ktl[l * K::KP * 2 + st] = (unsigned short)(dyi * ROWB + off + ASTR + (l & 15) * ASTR);
  }

  // ---- input rows: global -> registers (prefetch) -> LDS
  // two register sets for the input rows: a row is requested two steps before
  // it is used (HBM latency under load exceeds a step)
  vu32x4 inr[2][K::IREG] = {};
  const int nres = PT;                                          // residual loads per step
  const int nst = ((VOX_DBG(q) & 256) && blockIdx.x == 0) ? 1 : 0;  // trace stamps (stores)
  // The row loop's stores are inline asm and its waits counted by hand
  // (device_common.h vst16 / vm_wait): compiler-placed waits fell back to
  // vmcnt(0) before the staging writes, holding every wave on its in-flight
  // 1x1c stores and residual prefetches.  The loads are ordinary loads
  // (vld16), so the compiler's own waits also cover every use and copy of
  // their destinations (tests/test_vmcnt_audit.py).  Each load is always
  // issued (rows outside the image read a zero line), so the per-step op
  // counts are wave-uniform:
  //   phase 0: 1x1c waves: ns stores (PT when row c is owned, else 0) then PT
  //            residual loads (row c+1); phase 1: IREG input loads (row a+3).
  const bf16_t* zline = reinterpret_cast<const bf16_t*>(g_vox_zero);
  auto load_in = [&](auto P, int r) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < K::IREG; ++i) {
      int c = tid + i * NT;
      const int px = c / K::CU, u = c - px * K::CU;
      const bool ok = c < 16 * PT * K::CU && px < W && r >= 0 && r < H;
      vld16(inr[P][i], ok ? (const void*)(X + (img + (size_t)r * W + px) * CI + u * 8) : zline);
    }
  };
  auto store_in = [&](auto P) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < K::IREG; ++i) {
      const int c = tid + i * NT;
      const int px = c / K::CU, u = c - px * K::CU;
      vm_launder(inr[P][i]);
      if (c < 16 * PT * K::CU) *reinterpret_cast<vu32x4*>(inb + px * K::ISTR + u * 16) = inr[P][i];
    }
  };
  // the residual row is requested one step ahead (a second register set would
  // push the chain's fragment reads onto the registers they are consumed from)
  vu32x4 resb[PT] = {};
  // addresses of residual row r, formed while the previous row's values are
  // still live: the register allocator then has no reason to build them in
  // resb's registers, and the loads land in resb's registers directly (no
  // copy -- a copy would wait for the loads at once, vld16)
  auto res_addr = [&](int r, const void* (&ra)[PT]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      const int px = 16 * j + col;
      // identity: this lane's 8 residual channels; projection: its B chunk of
      // the (CI = 32)-channel input row, for the shortcut MFMAs
      const int cho = K::PROJ ? 8 * g : 32 * pq + 8 * g;
      const bool ok = r >= h0 && r < h1 && px < W;
      ra[j] = ok ? (const void*)(X + (img + (size_t)r * W + px) * CI + cho) : (const void*)zline;
    }
  };
  // issued by every wave (the others read the zero line): one definition of
  // resb on every path, so no merge copy of in-flight values at the join
  auto load_res_at = [&](const void* const (&ra)[PT]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < PT; ++j)
      vld16(resb[j], (is_c && !(VOX_DBG(q) & 512)) ? ra[j] : (const void*)zline);
  };
  auto load_res = [&](int r) __attribute__((always_inline)) {
    const void* ra[PT];
    res_addr(r, ra);
    load_res_at(ra);
  };

  const int a0 = h0 - (S - 1);
  const int steps = (h1 - h0) + 3 * (S - 1);
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  // the weights land here: otherwise the compiler, which does not see the asm
  // loads, re-places its waits for them inside the row loop every step, where
  // they drain the row prefetches too
#pragma unroll
  for (int s = 0; s < K::KSW; ++s) { vm_launder(w1[s][0]); vm_launder(w1[s][1]); }
  vm_launder(wp[0]);
  vm_launder(wp[1]);
#pragma unroll
  for (int s = 0; s < KST; ++s) vm_launder(wb[s]);
  load_in(P0{}, a0);
  vm_wait(0);
  store_in(P0{});
  load_in(P0{}, a0 + 1);
  load_in(P1{}, a0 + 2);
  load_res(a0 - K::LAG_C);
  __syncthreads();
  int ns_prev = 0;   // stores this wave issued in the previous step

  // step t (register set P = t & 1): input row a + 1 was requested two steps
  // earlier, residual row c one step earlier
  const bool trace = (VOX_DBG(q) & 256) && blockIdx.x == 0 && lane == 0;
  auto stamp = [&](int t, int i) __attribute__((always_inline)) {
    if (trace && t < 512) g_vox_trace[(wave * 512 + t) * 4 + i] = __builtin_amdgcn_s_memtime();
  };
  auto step = [&](auto P, int t) __attribute__((always_inline)) {
    const int a = a0 + t;
    const int c = a - K::LAG_C;
    auto& res = resb;
    const bool cstep = is_c && c >= h0 && c < h1 && !(VOX_DBG(q) & 2);
    const int ns_cur = cstep ? PT : 0;
    const void* rnext[PT];
    res_addr(c + 1, rnext);
    stamp(t, 0);
    // ---------------- phase 0: 1x1a (row a) | 1x1c (row c)
    if (is_a && !(VOX_DBG(q) & 1)) {
      const bool inimg = a >= 0 && a < Hn;
      const int ch = 32 * pq + 8 * g;
      const int p = ch / WID, off = ch - p * WID;
      int sl = K::ZB(1) + (a & 3);                   // plane 0 -> z_1 = x_1
#pragma unroll
      for (int d = 2; d <= S; ++d)
        if (p + 1 == d) sl = K::XB(d) + (a + 840) % K::XD(d);
      char* dst = rings + sl * ROWB + off * 2;
      const f32x4 m0 = *reinterpret_cast<const f32x4*>(bn1m);
      const f32x4 m1 = *reinterpret_cast<const f32x4*>(bn1m + 4);
      const f32x4 i0 = *reinterpret_cast<const f32x4*>(bn1i);
      const f32x4 i1 = *reinterpret_cast<const f32x4*>(bn1i + 4);
      auto epi = [&](const f32x4& acc0, const f32x4& acc1, int px) __attribute__((always_inline)) {
        // BN as (acc + (-mean)) * inv on packed fp32 pairs: x + (-m) == x - m
        // exactly; the tables hold the negated means
        const f32x4 t0 = (acc0 + m0) * i0, t1 = (acc1 + m1) * i1;
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o[e] = (bf16_t)t0[e];
          o[4 + e] = (bf16_t)t1[e];
        }
        o = relu_bf16(o);
        if (!inimg) o = bf16x8{};
        if (px < W) *reinterpret_cast<bf16x8*>(dst + (px + 1) * ASTR) = o;
      };
#pragma unroll
      for (int j = 0; j < PT; j += 2) {
        const bool two = j + 1 < PT;
        const int px = 16 * j + col;
        bf16x8 b[K::KSA], bq[K::KSA];
#pragma unroll
        for (int s = 0; s < K::KSA; ++s) {
          b[s] = *reinterpret_cast<const bf16x8*>(inb + px * K::ISTR + (32 * s + 8 * g) * 2);
          bq[s] = two ? *reinterpret_cast<const bf16x8*>(inb + (px + 16) * K::ISTR + (32 * s + 8 * g) * 2)
                      : bf16x8{};
        }
        f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, c0 = a0, c1 = a0;
#pragma unroll
        for (int s = 0; s < K::KSA; ++s) {
          a0 = mfma_step(w1[s][0], b[s], a0);
          a1 = mfma_step(w1[s][1], b[s], a1);
          if (two) {
            c0 = mfma_step(w1[s][0], bq[s], c0);
            c1 = mfma_step(w1[s][1], bq[s], c1);
          }
        }
        epi(a0, a1, px);
        if (two) epi(c0, c1, px + 16);
      }
    } else if (cstep) {
      // residual row c (loaded at step t-1, after its stores): younger are
      // that step's input loads and 3 trace stamps, and this step's first stamp
      vm_wait(t < 1 ? 0 : K::IREG + 4 * nst);
#pragma unroll
      for (int j = 0; j < PT; ++j) vm_launder(res[j]);
      if (VOX_DBG(q) & 2048) stamp(t, 1);   // (residual row landed)
      // B chunk s of lane group g: concat channel 32s+8g -> (plane, offset)
      const char* src[K::KSC];
#pragma unroll
      for (int s = 0; s < K::KSC; ++s) {
        const int ch = 32 * s + 8 * g;
        const int p = ch / WID, off = ch - p * WID;
        int sl = K::XB(S) + (c + 840) % K::XD(S);
#pragma unroll
        for (int d = 1; d < S; ++d)
          if (p + 1 == d) sl = K::YB(d) + (c + 840) % K::YD(d);
        src[s] = rings + sl * ROWB + off * 2;
      }
      const int ch = 32 * pq + 8 * g;
      const f32x4 m0 = *reinterpret_cast<const f32x4*>(bn1m);
      const f32x4 m1 = *reinterpret_cast<const f32x4*>(bn1m + 4);
      const f32x4 i0 = *reinterpret_cast<const f32x4*>(bn1i);
      const f32x4 i1 = *reinterpret_cast<const f32x4*>(bn1i + 4);
      auto epi = [&](const f32x4& acc0, const f32x4& acc1, bf16x8 rv, int px)
                     __attribute__((always_inline)) {
        if (K::PROJ) {
          // shortcut = bf16(bn_p(conv1x1_p(in))), as the unfused projection writes it
          const f32x4 z = {0.f, 0.f, 0.f, 0.f};
          const f32x4 s0 = mfma_step(wp[0], rv, z), s1 = mfma_step(wp[1], rv, z);
          // (negated means in the table, as below)
          const f32x4 pm0 = *reinterpret_cast<const f32x4*>(bmp + ch);
          const f32x4 pm1 = *reinterpret_cast<const f32x4*>(bmp + ch + 4);
          const f32x4 pi0 = *reinterpret_cast<const f32x4*>(bip + ch);
          const f32x4 pi1 = *reinterpret_cast<const f32x4*>(bip + ch + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            rv[e] = (bf16_t)((s0[e] + pm0[e]) * pi0[e]);
            rv[4 + e] = (bf16_t)((s1[e] + pm1[e]) * pi1[e]);
          }
        }
        // BN, then the residual add, each rounded like the unfused epilogue (no
        // FMA); BN on packed pairs with the negated means of the table
        const f32x4 t0 = (acc0 + m0) * i0, t1 = (acc1 + m1) * i1;
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
#pragma clang fp contract(off)
          float v0 = t0[e] + (float)rv[e];
          float v1 = t1[e] + (float)rv[4 + e];
          o[e] = (bf16_t)v0;
          o[4 + e] = (bf16_t)v1;
        }
        o = relu_bf16(o);
        // lane col 0 (px = 16 j < W) is always active: one store per tile
        if (px < W) vst16(Y + (img + (size_t)c * W + px) * C + ch, __builtin_bit_cast(vu32x4, o));
      };
#pragma unroll
      for (int j = 0; j < PT; j += 2) {
        const bool two = j + 1 < PT;
        const int px = 16 * j + col;
        bf16x8 b[K::KSC], bq[K::KSC];
#pragma unroll
        for (int s = 0; s < K::KSC; ++s) {
          b[s] = *reinterpret_cast<const bf16x8*>(src[s] + (px + 1) * ASTR);
          bq[s] = two ? *reinterpret_cast<const bf16x8*>(src[s] + (px + 17) * ASTR) : bf16x8{};
        }
        f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, c0 = a0, c1 = a0;
#pragma unroll
        for (int s = 0; s < K::KSC; ++s) {
          a0 = mfma_step(w1[s][0], b[s], a0);
          a1 = mfma_step(w1[s][1], b[s], a1);
          if (two) {
            c0 = mfma_step(w1[s][0], bq[s], c0);
            c1 = mfma_step(w1[s][1], bq[s], c1);
          }
        }
        epi(a0, a1, __builtin_bit_cast(bf16x8, res[j]), px);
        if (two) epi(c0, c1, __builtin_bit_cast(bf16x8, res[(j + 1) < PT ? j + 1 : j]), px + 16);
      }
    } else if (is_c) {
      // row c is outside the segment: the residual row requested at step t-1 is
      // not consumed, but load_res below reuses its registers.  Retire it first
      // on this path too -- otherwise those registers are dead to the compiler
      // while the loads are in flight, it builds the next addresses in them, and
      // the late data (the zero line at the segment start) lands on an address:
      // the intermittent illegal-address fault of 9c1d9bf (DESIGN.md "vmcnt")
      vm_wait(t < 1 ? 0 : K::IREG + 4 * nst);
#pragma unroll
      for (int j = 0; j < PT; ++j) vm_launder(res[j]);
    }
    // (VOXEMB_BNECK_DBG bit 2048: stamps 1, 2, 3 after the 1x1c's residual wait,
    // after the phase-0 work and after barrier 1, to split phase 0)
    if (VOX_DBG(q) & 2048) stamp(t, 2);
    if (!(VOX_DBG(q) & 8)) load_res_at(rnext);
    if (!(VOX_DBG(q) & 2048)) stamp(t, 1);
    __syncthreads();
    if (VOX_DBG(q) & 2048) stamp(t, 3);
    // (VOXEMB_BNECK_DBG bit 1024: stamps 2 and 3 after the input staging and
    // after the chain's MFMA loop instead, to split phase 1)
    if (!(VOX_DBG(q) & 1024) && !(VOX_DBG(q) & 2048)) stamp(t, 2);
    // ---------------- phase 1: all 3x3 stages, stage k on row a-2k+1
    if (!(VOX_DBG(q) & 8)) {
      // input row a+1 (loaded at step t-2): younger are step t-1's and this
      // step's stores and residual loads, step t-1's input loads, 8 stamps
      vm_wait(t < 2 ? 0 : K::IREG + ns_prev + ns_cur + 2 * nres + 8 * nst);
      store_in(P);
      load_in(P, a + 3);
    }
    if (VOX_DBG(q) & 1024) stamp(t, 2);
    ns_prev = ns_cur;
    if (chain_wave && !(VOX_DBG(q) & 4)) {
      const int k = ck;
      const int co = 16 * ci + 4 * g;
      const int r = a - 2 * k + 1;
      const bool inimg = r >= 0 && r < Hn;
      // ring geometry of stage k (wave-uniform -> scalar registers); tap row dy
      // of output row r is ring row (r - 1 + dy) & 3 of z_k
      const char* zring = rings + K::ZB(k) * ROWB;
      const int rbase = __builtin_amdgcn_readfirstlane(((r - 1 + 840) & 3) * ROWB);
      const int ysl = __builtin_amdgcn_readfirstlane(
          (K::XEND + (k - 1) * (2 * S - 1 - k) + (r + 840) % (2 * S - 1 - 2 * k)) * ROWB);
      const bool chain_next = k < S - 1;
      const int zsl = __builtin_amdgcn_readfirstlane((K::ZB(k + 1) + ((r + 840) & 3)) * ROWB);
      const int xsl = __builtin_amdgcn_readfirstlane(
          (K::ZEND + (k - 1) * k + (r + 840) % (2 * k)) * ROWB);
      const f32x4 m = *reinterpret_cast<const f32x4*>(bmb + (k - 1) * 16 * WCO + co);
      const f32x4 sc = *reinterpret_cast<const f32x4*>(bib + (k - 1) * 16 * WCO + co);
      unsigned bpk[K::KP];
      {
        const unsigned* kt = reinterpret_cast<const unsigned*>(ktl) + lane * K::KP;
#pragma unroll
        for (int i = 0; i < K::KP; ++i) bpk[i] = kt[i];
      }
      int boff[KST];
#pragma unroll
      for (int s = 0; s < KST; ++s) {
        const int e = (s & 1) ? (int)(bpk[s >> 1] >> 16) : (int)(bpk[s >> 1] & 0xFFFFu);
        const int v = rbase + e;
        boff[s] = v >= 4 * ROWB ? v - 4 * ROWB : v;
      }
      auto epilogue = [&](const f32x4& acc, int px) __attribute__((always_inline)) {
        if (!(co < WID && px < W)) return;
        const int pxo = px * ASTR + co * 2 + ASTR;
        const f32x4 t = (acc + m) * sc;   // negated means in the table
        bf16x4 y;
#pragma unroll
        for (int e = 0; e < 4; ++e) y[e] = (bf16_t)t[e];
        y = relu_bf16(y);
        if (!inimg) y = bf16x4{};
        *reinterpret_cast<bf16x4*>(rings + ysl + pxo) = y;
        if (chain_next) {
          const bf16x4 x = *reinterpret_cast<const bf16x4*>(rings + xsl + pxo);
          // SAME padding of the next stage: z_{k+1} = 0 outside the image
          *reinterpret_cast<bf16x4*>(rings + zsl + pxo) = inimg ? add4(x, y) : bf16x4{};
        }
      };
      // the PT pixel tiles as independent accumulators, fragments read one
      // k-step ahead into the other of two register sets (same K order per
      // tile); a single set rotated by copies let the compiler merge the two
      // and issue each read only after the MFMA that freed its register
      f32x4 acc[PT];
      bf16x8 fr[2][PT];
#pragma unroll
      for (int j = 0; j < PT; ++j) {
        acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        fr[0][j] = *reinterpret_cast<const bf16x8*>(zring + boff[0] + 16 * j * ASTR);
      }
#pragma unroll
      for (int s = 0; s < KST; ++s) {
        if (s + 1 < KST) {
#pragma unroll
          for (int j = 0; j < PT; ++j)
            fr[(s + 1) & 1][j] = *reinterpret_cast<const bf16x8*>(zring + boff[s + 1] + 16 * j * ASTR);
          __builtin_amdgcn_sched_group_barrier(0x100, PT, 0);   // the reads first
        }
#pragma unroll
        for (int j = 0; j < PT; ++j) acc[j] = mfma_step(wb[s], fr[s & 1][j], acc[j]);
        if (s + 1 < KST) __builtin_amdgcn_sched_group_barrier(0x008, PT, 0);   // then the MFMAs
        __builtin_amdgcn_sched_barrier(0);
      }
      if (VOX_DBG(q) & 1024) stamp(t, 3);
#pragma unroll
      for (int j = 0; j < PT; ++j) epilogue(acc[j], 16 * j + col);
    } else if (VOX_DBG(q) & 1024) {
      stamp(t, 3);
    }
    if (!(VOX_DBG(q) & 1024) && !(VOX_DBG(q) & 2048)) stamp(t, 3);
    __syncthreads();
  };
  for (int t = 0; t < steps; t += 2) {
    step(P0{}, t);
    if (t + 1 < steps) step(P1{}, t + 1);
  }
  // the last prefetches (rows past the segment) retire before the wave ends
  vm_wait(0);
#pragma unroll
  for (int i = 0; i < K::IREG; ++i) { vm_launder(inr[0][i]); vm_launder(inr[1][i]); }
#pragma unroll
  for (int j = 0; j < PT; ++j) vm_launder(resb[j]);
}

template <int CI, int C, int WID, int S, int PT>
static hipError_t launch_bneck_t(const BneckParams& q, hipStream_t s) {
  using K = BneckCfg<CI, C, WID, S, PT>;
  hipLaunchKernelGGL((bneck_fused<CI, C, WID, S, PT>), dim3(q.N * q.nseg), dim3(512), K::LDS, s, q);
  return hipGetLastError();
}

// Instantiated shapes: (Cin, C, w, split, pixel tiles of the frequency axis).
#define BNECK_SHAPES(X) \
  X(128, 128, 24, 4, 5) /* res2net50_w24_s4_c32 layer 1, identity blocks, 80-d */ \
  X(128, 128, 24, 4, 3) /* ... 40-d features */                                   \
  X(32, 128, 24, 4, 5)  /* ... layer-1 block 0 (projection shortcut), 80-d */     \
  X(32, 128, 24, 4, 3)  /* ... 40-d */

int bneck_lds(int CI, int C, int wid, int s, int W) {
  const int pt = (W + 15) / 16;
#define X_LDS(ci_, c_, w_, s_, p_)                                            \
  if (CI == ci_ && C == c_ && wid == w_ && s == s_ && pt == p_)               \
    return BneckCfg<ci_, c_, w_, s_, p_>::LDS;
  BNECK_SHAPES(X_LDS)
#undef X_LDS
  return -1;
}

hipError_t launch_bneck(const BneckParams& q, int CI, int C, int wid, int s, hipStream_t st) {
  const int pt = (q.W + 15) / 16;
#define X_LAUNCH(ci_, c_, w_, s_, p_)                                         \
  if (CI == ci_ && C == c_ && wid == w_ && s == s_ && pt == p_)               \
    return launch_bneck_t<ci_, c_, w_, s_, p_>(q, st);
  BNECK_SHAPES(X_LAUNCH)
#undef X_LAUNCH
  return hipErrorInvalidValue;
}

}  // namespace vox

namespace vox {

// ----------------------------------------------------------------------------
// Row-streamed Res2Net split chain (stride 1) for blocks the whole-bottleneck
// kernel cannot hold (wider branches): the 1x1a output planes x_1..x_{S-1}
// stream in row by row, every 3x3 stage runs in one phase on its own lagged
// row (stage k on row a-2k+1, as in bneck_fused), z_{k+1} = x_{k+1} + y_k
// stays in LDS rings and y_k goes to HBM.  No halo rows are recomputed
// (split_chain's row tiles recompute 2(S-2) of every R+... rows).
// Waves: one per (stage, cout tile) with its weights in registers; NW is the
// role count rounded up to whole SIMDs (spare waves only move data).
template <int WID, int S, int PT>
struct ChainRowsCfg {
  static constexpr int WCO = (WID + 15) / 16;
  static constexpr int ROLES = (S - 1) * WCO;
  static constexpr int NW = (ROLES + 3) / 4 * 4;
  static constexpr int NT = 64 * NW;
  static constexpr int KFLAT = 9 * WID;
  static constexpr int KST = (KFLAT + 31) / 32;
  static constexpr int AU = ((WID / 8) & 1) ? WID / 8 : WID / 8 + 1;
  static constexpr int ASTR = AU * 16;
  static constexpr int WR = 16 * PT + 2;
  static constexpr int ROWB = WR * ASTR;
  // z_1: 3 rows, z_k: 4 rows (k = 2..S-1); x_k: 2k-2 rows (k = 2..S-1)
  static constexpr int ZEND = 3 + 4 * (S - 2);
  static constexpr int NPLANES = ZEND + (S - 2) * (S - 1);
  static constexpr int RING_BYTES = NPLANES * ROWB;
  static constexpr int LDS = RING_BYTES + 4 * 2 * (S - 1) * 16 * WCO;
  static constexpr int CU = (S - 1) * WID / 8;               // 16-B chunks of x_1..x_{S-1}
  static constexpr int XREG = (16 * PT * CU + NT - 1) / NT;  // per thread
};

template <int WID, int S, int PT>
__global__ __launch_bounds__((ChainRowsCfg<WID, S, PT>::NT)) void chain_rows(ChainParams q) {
  using K = ChainRowsCfg<WID, S, PT>;
  constexpr int NT = K::NT, WCO = K::WCO, KST = K::KST, ASTR = K::ASTR, ROWB = K::ROWB;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar ring math
  const int col = lane & 15, g = lane >> 4;
  const int H = q.H, W = q.W;
  const int nseg = q.nwaves;                 // segments per utterance (reused field)
  const int n = blockIdx.x / nseg;
  const int h0 = (blockIdx.x - n * nseg) * q.R;
  const int h1 = min(H, h0 + q.R);
  const int Hn = valid_rows(q.vlen, q.vsh, n, H);   // ragged batch (device_common.h)
  char* rings = smem;
  float* bmb = reinterpret_cast<float*>(smem + K::RING_BYTES);
  float* bib = bmb + (S - 1) * 16 * WCO;
  const bf16_t* __restrict__ A = reinterpret_cast<const bf16_t*>(q.a);
  bf16_t* __restrict__ Bo = reinterpret_cast<bf16_t*>(q.b);
  const size_t img = (size_t)n * H * W;

  for (int i = tid; i < K::RING_BYTES / 16; i += NT)
    reinterpret_cast<uint4*>(rings)[i] = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int k = 0; k < S - 1; ++k)
    for (int c = tid; c < 16 * WCO; c += NT) {
      bmb[k * 16 * WCO + c] = c < WID ? -q.mean[k][c] : 0.f;   // negated: BN as (x + (-m)) * inv
      bib[k * 16 * WCO + c] = c < WID ? q.inv[k][c] : 0.f;
    }

  const bool role = wave < K::ROLES;
  const int ck = role ? wave / WCO + 1 : 1;
  const int ci = wave % WCO;
  bf16x8 wb[KST];
  {
    const void* wk = q.wt[0];
#pragma unroll
    for (int k = 1; k < S - 1; ++k)
      if (ck == k + 1) wk = q.wt[k];
    const bf16_t* __restrict__ Wk = reinterpret_cast<const bf16_t*>(wk);
#pragma unroll
    for (int s = 0; s < KST; ++s) {
      const int kk = 32 * s + 8 * g;
      wb[s] = (role && kk < K::KFLAT) ? ld16(Wk + (size_t)(ci * 16 + col) * K::KFLAT + kk)
                                      : bf16x8{};
    }
  }
  int ktab[KST];
#pragma unroll
  for (int s = 0; s < KST; ++s) {
    const int kk = 32 * s + 8 * g;
    int dyi = 1, off = 0;
    if (kk < K::KFLAT) {
      const int tap = kk / WID, ch = kk - tap * WID;
      dyi = tap / 3;
      off = (tap % 3 - 1) * ASTR + ch * 2;
    }
    ktab[s] = (dyi << 24) | (off + 32768);
  }

  // x rows: global -> registers one step ahead -> LDS rings
  uint4 xr[K::XREG];
  auto load_x = [&](int r) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < K::XREG; ++i) {
      const int c = tid + i * NT;
      const int px = c / K::CU, u = c - px * K::CU;
      xr[i] = make_uint4(0, 0, 0, 0);
      if (c < 16 * PT * K::CU && px < W && r >= 0 && r < Hn)
        xr[i] = *reinterpret_cast<const uint4*>(A + (img + (size_t)r * W + px) * q.lda + u * 8);
    }
  };
  auto store_x = [&](int r) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < K::XREG; ++i) {
      const int c = tid + i * NT;
      const int px = c / K::CU, u = c - px * K::CU;
      if (c < 16 * PT * K::CU && px < W) {
        const int ch = u * 8, p = ch / WID, off = ch - p * WID;
        int sl = (r + 840) % 3;                         // plane 0 -> z_1
#pragma unroll
        for (int d = 2; d < S; ++d)
          if (p + 1 == d) sl = K::ZEND + (d - 2) * (d - 1) + (r + 840) % (2 * d - 2);
        *reinterpret_cast<uint4*>(rings + sl * ROWB + (px + 1) * ASTR + off * 2) = xr[i];
      }
    }
  };

  const int a0 = h0 - (S - 1);
  const int steps = (h1 - h0) + 3 * (S - 1) - 1;  // stage S-1 reaches row h1-1 at a = h1+2S-4
  load_x(a0);
  for (int t = 0; t < steps; ++t) {
    const int a = a0 + t;
    store_x(a);
    __syncthreads();
    load_x(a + 1);
    if (role) {
      const int k = ck;
      const int co = 16 * ci + 4 * g;
      const int r = a - 2 * k + 1;
      const bool inimg = r >= 0 && r < Hn;
      const int zd = k == 1 ? 3 : 4;
      const int zbase = k == 1 ? 0 : 3 + 4 * (k - 2);
      const int rb0 = __builtin_amdgcn_readfirstlane((zbase + (r - 1 + 840) % zd) * ROWB);
      const int rb1 = __builtin_amdgcn_readfirstlane((zbase + (r + 840) % zd) * ROWB);
      const int rb2 = __builtin_amdgcn_readfirstlane((zbase + (r + 1 + 840) % zd) * ROWB);
      const bool chain_next = k < S - 1;
      const int zsl = __builtin_amdgcn_readfirstlane((3 + 4 * (k - 1) + (r + 840) % 4) * ROWB);
      const int xsl = __builtin_amdgcn_readfirstlane(
          (K::ZEND + (k - 1) * k + (r + 840) % (2 * k)) * ROWB);
      const f32x4 m = *reinterpret_cast<const f32x4*>(bmb + (k - 1) * 16 * WCO + co);
      const f32x4 sc = *reinterpret_cast<const f32x4*>(bib + (k - 1) * 16 * WCO + co);
      const bool emit = r >= h0 && r < h1;               // rows this segment owns
      int boff[KST];
#pragma unroll
      for (int s = 0; s < KST; ++s) {
        int e = ktab[s];
        asm volatile("" : "+v"(e));
        const int dyi = e >> 24;
        boff[s] = (dyi == 0 ? rb0 : (dyi == 1 ? rb1 : rb2)) + (e & 0xFFFFFF) - 32768 + ASTR;
      }
      auto epilogue = [&](const f32x4& acc, int px) __attribute__((always_inline)) {
        if (!(co < WID && px < W)) return;
        const int pxo = px * ASTR + co * 2 + ASTR;
        bf16x4 y;
        {
          const f32x4 t = (acc + m) * sc;
#pragma unroll
          for (int e = 0; e < 4; ++e) y[e] = (bf16_t)t[e];
        }
        y = relu_bf16(y);
        if (emit)
          *reinterpret_cast<bf16x4*>(Bo + (img + (size_t)r * W + px) * q.ldb + (k - 1) * WID + co) = y;
        if (chain_next) {
          const bf16x4 x = *reinterpret_cast<const bf16x4*>(rings + xsl + pxo);
          *reinterpret_cast<bf16x4*>(rings + zsl + pxo) = inimg ? add4(x, y) : bf16x4{};
        }
      };
      for (int j = 0; j < PT; j += 2) {
        const bool two = j + 1 < PT;
        const int px0 = 16 * j + col, px1 = px0 + 16;
        bf16x8 b0[KST], b1[KST];
#pragma unroll
        for (int s = 0; s < KST; ++s) {
          b0[s] = *reinterpret_cast<const bf16x8*>(rings + boff[s] + px0 * ASTR);
          b1[s] = two ? *reinterpret_cast<const bf16x8*>(rings + boff[s] + px1 * ASTR) : bf16x8{};
        }
        f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KST; ++s) {
          acc0 = mfma_step(wb[s], b0[s], acc0);
          acc1 = mfma_step(wb[s], b1[s], acc1);
        }
        epilogue(acc0, px0);
        if (two) epilogue(acc1, px1);
      }
    }
    __syncthreads();
  }
}

// ----------------------------------------------------------------------------
// Identity-block front half in one launch (res2net_model.py:90-93 + 53-75,
// layer 2 blocks 1..): the 1x1a (+BN+ReLU, K = Cin) on the block input and
// chain_rows' row-streamed split chain, so the 1x1a output never touches HBM
// (only x_S, which the 1x1c reads, is written there).  Step for A-row a:
//   phase A: wave t computes 16 1x1a channels of row a from the staged input
//            row (weights in registers) -> rings x_1 (= z_1), x_2 .. x_{S-1};
//            x_S -> the concat buffer (global);
//   phase B: chain_rows' stage waves, stage k on row a-2k+1.
// The next input row streams global -> registers during the step and lands in
// the staging buffer at its end.  Same roundings and K orders as the unfused
// 1x1a + chain_rows: bit-identical.
template <int CI, int WID, int S, int PT>
struct ChainFusedCfg {
  using R = ChainRowsCfg<WID, S, PT>;
  static constexpr int SW = S * WID;
  static constexpr int NW = SW / 16;                   // one 1x1a 16-channel tile per wave
  static constexpr int NT = 64 * NW;
  static constexpr int KSA = CI / 32;
  // LDS images (16-B units): chunk c (8 channels) of pixel slot x sits in
  // sub-plane c/2 at unit 2x + ((c & 1) ^ bit2(x)).  gfx950 serves a
  // ds_read_b128 in lane groups that pair 8 columns of lane group g (even)
  // with 8 of g+1, which read chunks c and c+1: the two halves land on
  // opposite unit parities and 8 distinct pixel residues, so fragment reads
  // are conflict-free (the odd pixel stride of chain_rows conflicts 2-way);
  // the bit-2 flip halves the conflicts of the 8-byte epilogue stores.
  static constexpr int WR = 16 * PT + 2;                // ring slots: pad | pixels | pad
  static constexpr int NCH = WID / 8;
  static constexpr int SPR = 2 * WR;                   // units per sub-plane
  static constexpr int ROWB = NCH / 2 * SPR * 16;
  // z_k rings (k = 1..S-1) 4 rows each, so that the tap rows of a stage wrap
  // with a mask; x_k (k = 2..S-1) 2k-2 rows
  static constexpr int ZEND = 4 * (S - 1);
  static constexpr int NPLANES = ZEND + (S - 2) * (S - 1);
  static constexpr int RING_BYTES = NPLANES * ROWB;
  static constexpr int KST = R::KST;
  static constexpr int KTB = 64 * ((KST + 1) / 2) * 4;    // tap table [lane][k-step] u16
  static constexpr int CU = CI / 8;
  static constexpr int SPX = 2 * 16 * PT + 2;          // staging sub-plane (= 2 mod 8: store_x)
  static constexpr int INB = CU / 2 * SPX * 16;
  static constexpr int XREG = (16 * PT * CU + NT - 1) / NT;
  static constexpr int LDS = RING_BYTES + INB + KTB + 4 * (2 * (S - 1) * 16 * R::WCO + 2 * SW);
  static_assert(4 * ROWB < 65536, "tap offsets in 16 bits");
  static_assert(NW >= R::ROLES, "every chain role needs a wave");
  static_assert(NCH % 2 == 0 && CU % 2 == 0, "chunk pairs");
  static_assert(SPX % 8 == 2, "staging stores");
};

// byte offset of (pixel slot x, channel ch) in a chain_fused ring row
template <int SPR>
__device__ __forceinline__ int cf_off(int x, int ch) {
  const int c = ch >> 3;
  return ((c >> 1) * SPR + 2 * x + ((c & 1) ^ ((x >> 2) & 1))) * 16 + (ch & 7) * 2;
}

template <int CI, int WID, int S, int PT>
__global__ __launch_bounds__((ChainFusedCfg<CI, WID, S, PT>::NT)) void chain_fused(ChainParams q) {
  using K = ChainFusedCfg<CI, WID, S, PT>;
  using R = typename K::R;
  constexpr int NT = K::NT, WCO = R::WCO, KST = R::KST, ROWB = K::ROWB, SPR = K::SPR;
  static_assert(CI % 32 == 0 && WID % 8 == 0 && K::SW % 32 == 0, "shape");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int H = q.H, W = q.W;
  const int nseg = q.nwaves;
  const int n = blockIdx.x / nseg;
  const int h0 = (blockIdx.x - n * nseg) * q.R;
  const int h1 = min(H, h0 + q.R);
  const int Hn = valid_rows(q.vlen, q.vsh, n, H);   // ragged batch (device_common.h)
  char* rings = smem;
  char* inb = smem + K::RING_BYTES;
  unsigned short* ktl = reinterpret_cast<unsigned short*>(inb + K::INB);
  float* bmb = reinterpret_cast<float*>(inb + K::INB + K::KTB);
  float* bib = bmb + (S - 1) * 16 * WCO;
  float* bma = bib + (S - 1) * 16 * WCO;
  float* bia = bma + K::SW;
  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(q.x);
  bf16_t* __restrict__ Bo = reinterpret_cast<bf16_t*>(q.b);
  const size_t img = (size_t)n * H * W;

  for (int i = tid; i < K::RING_BYTES / 16; i += NT)
    reinterpret_cast<uint4*>(rings)[i] = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int k = 0; k < S - 1; ++k)
    for (int c = tid; c < 16 * WCO; c += NT) {
      bmb[k * 16 * WCO + c] = c < WID ? -q.mean[k][c] : 0.f;   // negated: BN as (x + (-m)) * inv
      bib[k * 16 * WCO + c] = c < WID ? q.inv[k][c] : 0.f;
    }
  for (int c = tid; c < K::SW; c += NT) {
    bma[c] = -q.ma[c];
    bia[c] = q.ia[c];
  }
  // tap table: for lane l and k-step s, the byte offset of its B fragment in
  // the 4-row z ring counted from the slot of tap row 0 (before wrapping)
  for (int e = tid; e < 64 * KST; e += NT) {
    const int l = e / KST, st = e - l * KST;
    const int kk = 32 * st + 8 * (l >> 4);
    int dyi = 1, dx = 0, ch = 0;
    if (kk < R::KFLAT) {
      const int tap = kk / WID;
      ch = kk - tap * WID;
      dyi = tap / 3;
      dx = tap % 3 - 1;
    }
    ktl[l * ((KST + 1) / 2) * 2 + st] = (unsigned short)(dyi * ROWB + cf_off<SPR>((l & 15) + 1 + dx, ch));
  }

  const bool role = wave < R::ROLES;
  const int ck = role ? wave / WCO + 1 : 1;
  const int ci = wave % WCO;
  bf16x8 wb[KST];
  {
    const void* wk = q.wt[0];
#pragma unroll
    for (int k = 1; k < S - 1; ++k)
      if (ck == k + 1) wk = q.wt[k];
    const bf16_t* __restrict__ Wk = reinterpret_cast<const bf16_t*>(wk);
#pragma unroll
    for (int s = 0; s < KST; ++s) {
      const int kk = 32 * s + 8 * g;
      wb[s] = (role && kk < R::KFLAT) ? ld16(Wk + (size_t)(ci * 16 + col) * R::KFLAT + kk)
                                      : bf16x8{};
    }
  }
  // 1x1a tile t of the paired-row weights: lane channels 32(t/2) + 8g + 4(t%2) + 0..3
  const int t16 = wave;
  bf16x8 w1[K::KSA];
  {
    const bf16_t* __restrict__ Wa = reinterpret_cast<const bf16_t*>(q.wa);
#pragma unroll
    for (int s = 0; s < K::KSA; ++s)
      w1[s] = ld16(Wa + (size_t)(t16 * 16 + col) * CI + 32 * s + 8 * g);
  }

  // input rows: global -> registers (one step ahead) -> staging
  uint4 xr[K::XREG];
  const int ldx = q.ldx;
  auto load_x = [&](int r) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < K::XREG; ++i) {
      int c = tid + i * NT;
      asm volatile("" : "+v"(c));   // recomputed per step: nothing hoisted into registers
      const int px = c / K::CU, u = c - px * K::CU;
      xr[i] = make_uint4(0, 0, 0, 0);
      if (c < 16 * PT * K::CU && px < W && r >= 0 && r < H)
        xr[i] = *reinterpret_cast<const uint4*>(X + (img + (size_t)r * W + px) * ldx + u * 8);
    }
  };
  auto store_x = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < K::XREG; ++i) {
      int c = tid + i * NT;
      asm volatile("" : "+v"(c));
      const int px = c / K::CU, u = c - px * K::CU;
      if (c < 16 * PT * K::CU)
        *reinterpret_cast<uint4*>(inb + ((u >> 1) * K::SPX + 2 * px + (u & 1)) * 16) = xr[i];
    }
  };

  const int a0 = h0 - (S - 1);
  const int steps = (h1 - h0) + 3 * (S - 1) - 1;   // as chain_rows
  load_x(a0);
  store_x();
  load_x(a0 + 1);
  __syncthreads();
  for (int t = 0; t < steps; ++t) {
    const int a = a0 + t;
    // input row a+1 was requested right after the previous step's staging
    // store, so it has phase B of step t-1 and phase A of this step to land
    // (requested at the top of the step it had phase A only)
    // ---------------- phase A: 1x1a of A-row a -> rings / x_S
    {
      const int ch = 32 * (t16 >> 1) + 8 * g + 4 * (t16 & 1);
      const int p = ch / WID, off = ch - p * WID;
      const bool inimg = a >= 0 && a < Hn;
      int sl = (a + 840) & 3;                                   // plane 0 -> z_1
#pragma unroll
      for (int d = 2; d < S; ++d)
        if (p + 1 == d) sl = K::ZEND + (d - 2) * (d - 1) + (a + 840) % (2 * d - 2);
      const bool last = p == S - 1;                             // x_S: global only
      const bool emit_s = last && inimg && a >= h0 && a < h1;
      char* dst = rings + sl * ROWB + cf_off<SPR>(col + 1, off);
      const f32x4 m0 = *reinterpret_cast<const f32x4*>(bma + ch);
      const f32x4 i0 = *reinterpret_cast<const f32x4*>(bia + ch);
      // the PT pixel tiles as independent accumulators, fragments read one
      // k-step ahead (same K order per tile as the GEMM)
      f32x4 acc[PT];
      bf16x8 bc[PT], bn[PT];
      // chunk u = 4s + g of pixel pr: sub-plane 2s + g/2, unit 2 pr + g%2
      int fb[PT];
#pragma unroll
      for (int j = 0; j < PT; ++j) {
        int pr = min(16 * j + col, W - 1);
        asm volatile("" : "+v"(pr));   // per step: not hoisted out of the row loop
        fb[j] = ((g >> 1) * K::SPX + 2 * pr + (g & 1)) * 16;
      }
      auto frag = [&](int s, int j) __attribute__((always_inline)) {
        return *reinterpret_cast<const bf16x8*>(inb + fb[j] + 2 * s * K::SPX * 16);
      };
#pragma unroll
      for (int j = 0; j < PT; ++j) {
        acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        bc[j] = frag(0, j);
      }
      if (!(VOX_DBG(q) & 128)) {   // (diagnostics: 128 = no phase-A MFMAs)
#pragma unroll
        for (int s = 0; s < K::KSA; ++s) {
          if (s + 1 < K::KSA) {
#pragma unroll
            for (int j = 0; j < PT; ++j) bn[j] = frag(s + 1, j);
          }
#pragma unroll
          for (int j = 0; j < PT; ++j) acc[j] = mfma_step(w1[s], bc[j], acc[j]);
#pragma unroll
          for (int j = 0; j < PT; ++j) bc[j] = bn[j];
          __builtin_amdgcn_sched_barrier(0);   // reads stay one k-step ahead
        }
      }
#pragma unroll
      for (int j = 0; j < PT; ++j) {
        const int px = 16 * j + col;
        bf16x4 o;
        {
          const f32x4 t = (acc[j] + m0) * i0;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = (bf16_t)t[e];
        }
        o = relu_bf16(o);
        if (!inimg) o = bf16x4{};   // SAME padding rows of the chain
        if (px < W) {
          if (!last) *reinterpret_cast<bf16x4*>(dst + 512 * j) = o;
          else if (emit_s)
            *reinterpret_cast<bf16x4*>(Bo + (img + (size_t)a * W + px) * q.ldb + ch) = o;
        }
      }
    }
    __syncthreads();
    store_x();   // input row a+1: phase A is done with the staging
    load_x(a + 2);
    // ---------------- phase B: chain_rows' stages, stage k on row a-2k+1
    // (VOXEMB_BNECK_DBG diagnostics, garbage out: 16 = wave 8 skips its role,
    // 32 = wave 1 skips its role, 64 = no phase B)
    if (role && !((VOX_DBG(q) & 16) && wave == 8) && !((VOX_DBG(q) & 32) && wave == 1) && !(VOX_DBG(q) & 64)) {
      const int k = ck;
      const int co = 16 * ci + 4 * g;
      const int r = a - 2 * k + 1;
      const bool inimg = r >= 0 && r < Hn;
      // z_k ring (4 rows): tap row dy of output row r is ring row (r - 1 + dy) & 3
      const char* zring = rings + 4 * (k - 1) * ROWB;
      const int rbase = __builtin_amdgcn_readfirstlane(((r - 1 + 840) & 3) * ROWB);
      const bool chain_next = k < S - 1;
      const int zsl = __builtin_amdgcn_readfirstlane((4 * k + ((r + 840) & 3)) * ROWB);
      const int xsl = __builtin_amdgcn_readfirstlane(
          (K::ZEND + (k - 1) * k + (r + 840) % (2 * k)) * ROWB);
      const f32x4 m = *reinterpret_cast<const f32x4*>(bmb + (k - 1) * 16 * WCO + co);
      const f32x4 sc = *reinterpret_cast<const f32x4*>(bib + (k - 1) * 16 * WCO + co);
      const bool emit = r >= h0 && r < h1;
      constexpr int KP = (KST + 1) / 2;
      unsigned bpk[KP];
      {
        const unsigned* kt = reinterpret_cast<const unsigned*>(ktl) + lane * KP;
#pragma unroll
        for (int i = 0; i < KP; ++i) bpk[i] = kt[i];
      }
      auto boff = [&](int s) __attribute__((always_inline)) {
        const int e = (s & 1) ? (int)(bpk[s >> 1] >> 16) : (int)(bpk[s >> 1] & 0xFFFFu);
        const int v = rbase + e;
        return v >= 4 * ROWB ? v - 4 * ROWB : v;
      };
      const int pxo = cf_off<SPR>(col + 1, co);   // this lane's 4 channels, tile 0
      auto epilogue = [&](const f32x4& acc, int j) __attribute__((always_inline)) {
        const int px = 16 * j + col;
        if (!(co < WID && px < W)) return;
        bf16x4 y;
        {
          const f32x4 t = (acc + m) * sc;
#pragma unroll
          for (int e = 0; e < 4; ++e) y[e] = (bf16_t)t[e];
        }
        y = relu_bf16(y);
        if (emit)
          *reinterpret_cast<bf16x4*>(Bo + (img + (size_t)r * W + px) * q.ldb + (k - 1) * WID + co) = y;
        if (chain_next) {
          const bf16x4 x = *reinterpret_cast<const bf16x4*>(rings + xsl + pxo + 512 * j);
          *reinterpret_cast<bf16x4*>(rings + zsl + pxo + 512 * j) = inimg ? add4(x, y) : bf16x4{};
        }
      };
      f32x4 acc[PT];
      bf16x8 bc[PT], bn[PT];
#pragma unroll
      for (int j = 0; j < PT; ++j) {
        acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        bc[j] = *reinterpret_cast<const bf16x8*>(zring + boff(0) + 512 * j);
      }
#pragma unroll
      for (int s = 0; s < KST; ++s) {
        if (s + 1 < KST) {
#pragma unroll
          for (int j = 0; j < PT; ++j)
            bn[j] = *reinterpret_cast<const bf16x8*>(zring + boff(s + 1) + 512 * j);
        }
#pragma unroll
        for (int j = 0; j < PT; ++j) acc[j] = mfma_step(wb[s], bc[j], acc[j]);
#pragma unroll
        for (int j = 0; j < PT; ++j) bc[j] = bn[j];
        __builtin_amdgcn_sched_barrier(0);   // reads stay one k-step ahead
      }
#pragma unroll
      for (int j = 0; j < PT; ++j) epilogue(acc[j], j);
    }
    __syncthreads();
  }
}

#define CHAIN_FUSED_SHAPES(X) \
  X(256, 48, 4, 3)  /* res2net50_w24_s4_c32 layer-2 identity blocks, 80-d features (W = 40) */ \
  X(256, 48, 4, 2)  /* ... 40-d features (W = 20) */

int chain_fused_lds(int ci, int wid, int s, int W) {
  const int pt = (W + 15) / 16;
#define X_LDS(ci_, w_, s_, p_) \
  if (ci == ci_ && wid == w_ && s == s_ && pt == p_) return ChainFusedCfg<ci_, w_, s_, p_>::LDS;
  CHAIN_FUSED_SHAPES(X_LDS)
#undef X_LDS
  return -1;
}

hipError_t launch_chain_fused(const ChainParams& q, hipStream_t st) {
  const int pt = (q.W + 15) / 16;
#define X_LAUNCH(ci_, w_, s_, p_)                                                          \
  if (q.cin == ci_ && q.w == w_ && q.nst + 1 == s_ && pt == p_) {                         \
    using K = ChainFusedCfg<ci_, w_, s_, p_>;                                             \
    hipLaunchKernelGGL((chain_fused<ci_, w_, s_, p_>), dim3(q.N * q.nwaves), dim3(K::NT), \
                       K::LDS, st, q);                                                    \
    return hipGetLastError();                                                             \
  }
  CHAIN_FUSED_SHAPES(X_LAUNCH)
#undef X_LAUNCH
  return hipErrorInvalidValue;
}

#define CHAIN_ROWS_SHAPES(X) \
  X(48, 4, 3)  /* res2net50_w24_s4_c32 layer 2, 80-d features (W = 40) */ \
  X(48, 4, 2)  /* ... 40-d features (W = 20) */

int chain_rows_lds(int wid, int s, int W) {
  const int pt = (W + 15) / 16;
#define X_LDS(w_, s_, p_) \
  if (wid == w_ && s == s_ && pt == p_) return ChainRowsCfg<w_, s_, p_>::LDS;
  CHAIN_ROWS_SHAPES(X_LDS)
#undef X_LDS
  return -1;
}

hipError_t launch_chain_rows(const ChainParams& q, hipStream_t st) {
  const int pt = (q.W + 15) / 16;
#define X_LAUNCH(w_, s_, p_)                                                             \
  if (q.w == w_ && q.nst + 1 == s_ && pt == p_) {                                      \
    using K = ChainRowsCfg<w_, s_, p_>;                                                \
    hipLaunchKernelGGL((chain_rows<w_, s_, p_>), dim3(q.N * q.nwaves), dim3(K::NT), K::LDS, \
                       st, q);                                                         \
    return hipGetLastError();                                                          \
  }
  CHAIN_ROWS_SHAPES(X_LAUNCH)
#undef X_LAUNCH
  return hipErrorInvalidValue;
}

}  // namespace vox

namespace vox {

// ----------------------------------------------------------------------------
// Stride-2 Res2Net split ('stage' blocks, res2net_model.py:53-77): branch k
// (k < S) = relu(bn(conv3x3 stride 2, fixed pad 1)(x_k)), the last split
// avg-pooled 3x3/2 (divisor 9), all from one row-streamed launch.  Output row
// ho reads input rows 2ho-1..2ho+1 of every plane from a 3-row LDS ring; the
// next two input rows stream in (global -> registers -> LDS) while the row is
// computed.  Waves: one per (branch, cout tile) with weights in registers;
// the spare waves average-pool the last plane.
template <int WID, int S, int WIN>
struct SplitS2Cfg {
  static constexpr int WOUT = (WIN + 1) / 2;
  static constexpr int PT = (WOUT + 15) / 16;
  static constexpr int WR = WIN + 2;            // ring row: pad | WIN | pad
  static constexpr int WCO = (WID + 15) / 16;
  static constexpr int ROLES = (S - 1) * WCO;
  static constexpr int NW = (ROLES + 3) / 4 * 4 + ((ROLES % 4) == 0 ? 4 : 0);  // >= 1 spare wave
  static constexpr int NT = 64 * NW;
  static constexpr int KFLAT = 9 * WID;
  static constexpr int KST = (KFLAT + 31) / 32;
  static constexpr int AU = ((WID / 8) & 1) ? WID / 8 : WID / 8 + 1;
  static constexpr int ASTR = AU * 16;
  static constexpr int CU = S * WID / 8;        // 16-B chunks per input pixel (all planes)
  static constexpr int WC8 = WID / 8;           // chunks of one plane
  static constexpr int XREG = (2 * WIN * CU + NT - 1) / NT;   // two rows per step
  static constexpr int LDS = S * 3 * WR * ASTR + 4 * 2 * (S - 1) * 16 * WCO + 4 * 4 * KST;
};

template <int WID, int S, int WIN>
__global__ __launch_bounds__((SplitS2Cfg<WID, S, WIN>::NT)) void split_s2_rows(ChainParams q) {
  using K = SplitS2Cfg<WID, S, WIN>;
  constexpr int NT = K::NT, WCO = K::WCO, KST = K::KST, ASTR = K::ASTR, CU = K::CU;
  constexpr int PT = K::PT, W = WIN, Wo = K::WOUT, ROWB = K::WR * ASTR, PLANEB = 3 * ROWB;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar ring math
  const int col = lane & 15, g = lane >> 4;
  const int H = q.H;
  const int Ho = (H + 1) / 2;
  const int nseg = q.nwaves;
  const int n = blockIdx.x / nseg;
  const int g0 = (blockIdx.x - n * nseg) * q.R;
  const int g1 = min(Ho, g0 + q.R);
  const int Hn = valid_rows(q.vlen, q.vsh, n, H);   // ragged batch: input rows past it are padding
  char* rings = smem;
  const int ring_bytes = S * PLANEB;
  float* bmb = reinterpret_cast<float*>(smem + ring_bytes);
  float* bib = bmb + (S - 1) * 16 * WCO;
  int* ktab_l = reinterpret_cast<int*>(bib + (S - 1) * 16 * WCO);   // [4 lane groups][KST]
  const bf16_t* __restrict__ A = reinterpret_cast<const bf16_t*>(q.a);
  bf16_t* __restrict__ Bo = reinterpret_cast<bf16_t*>(q.b);
  const size_t img = (size_t)n * H * W;
  const size_t imgo = (size_t)n * Ho * Wo;

  for (int i = tid; i < ring_bytes / 16; i += NT)
    reinterpret_cast<uint4*>(rings)[i] = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int k = 0; k < S - 1; ++k)
    for (int c = tid; c < 16 * WCO; c += NT) {
      bmb[k * 16 * WCO + c] = c < WID ? -q.mean[k][c] : 0.f;   // negated: BN as (x + (-m)) * inv
      bib[k * 16 * WCO + c] = c < WID ? q.inv[k][c] : 0.f;
    }

  const bool role = wave < K::ROLES;
  const int ck = role ? wave / WCO : 0;          // branch (0-based)
  const int ci = wave % WCO;
  bf16x8 wb[KST];
  {
    const void* wk = q.wt[0];
#pragma unroll
    for (int k = 1; k < S - 1; ++k)
      if (ck == k) wk = q.wt[k];
    const bf16_t* __restrict__ Wk = reinterpret_cast<const bf16_t*>(wk);
#pragma unroll
    for (int s = 0; s < KST; ++s) {
      const int kk = 32 * s + 8 * g;
      wb[s] = (role && kk < K::KFLAT) ? ld16(Wk + (size_t)(ci * 16 + col) * K::KFLAT + kk)
                                      : bf16x8{};
    }
  }
  // k-step table per lane group (LDS; read back every row): tap row << 24 |
  // (byte offset + 2^15)
  for (int i = tid; i < 4 * KST; i += NT) {
    const int gg = i / KST, s = i - gg * KST;
    const int kk = 32 * s + 8 * gg;
    int dyi = 1, off = 0;
    if (kk < K::KFLAT) {
      const int tap = kk / WID, ch = kk - tap * WID;
      dyi = tap / 3;
      off = (tap % 3 - 1) * ASTR + ch * 2;
    }
    ktab_l[i] = (dyi << 24) | (off + 32768);
  }

  // two input rows per step: global -> registers -> ring.  Chunk c of the
  // pair is (row rr, pixel px, 16-B unit u); all divisors are compile-time and
  // addresses are a scalar row base + a 32-bit lane offset (nothing to hoist).
  constexpr int XREG = K::XREG;
  uint4 xr[XREG];
  const int lda = q.lda;
  auto load_rows = [&](int r0) __attribute__((always_inline)) {
    const bf16_t* base = A + (img + (size_t)r0 * W) * lda;
#pragma unroll
    for (int i = 0; i < XREG; ++i) {
      const int c = tid + i * NT;
      const int rr = c / (W * CU), cc = c - rr * (W * CU);
      const int px = cc / CU, u = cc - px * CU;
      const int r = r0 + rr;
      xr[i] = make_uint4(0, 0, 0, 0);
      if (rr < 2 && r >= 0 && r < Hn)
        xr[i] = *reinterpret_cast<const uint4*>(base + (rr * W + px) * lda + u * 8);
    }
  };
  auto store_rows = [&](int r0, int nrows) __attribute__((always_inline)) {
    const int s0 = ((r0 + 840) % 3) * ROWB, s1 = ((r0 + 841) % 3) * ROWB;
#pragma unroll
    for (int i = 0; i < XREG; ++i) {
      const int c = tid + i * NT;
      const int rr = c / (W * CU), cc = c - rr * (W * CU);
      const int px = cc / CU, u = cc - px * CU;
      if (rr < nrows) {
        const int p = u / K::WC8, uo = u - p * K::WC8;
        *reinterpret_cast<uint4*>(rings + p * PLANEB + (rr ? s1 : s0) + (px + 1) * ASTR + uo * 16) =
            xr[i];
      }
    }
  };

  load_rows(2 * g0 - 1);       // row 2*g0-1 (first of the pair) seeds the ring
  store_rows(2 * g0 - 1, 1);
  load_rows(2 * g0);
  for (int ho = g0; ho < g1; ++ho) {
    store_rows(2 * ho, 2);
    __syncthreads();
    load_rows(2 * ho + 2);
    const int rb0 = __builtin_amdgcn_readfirstlane(((2 * ho - 1 + 840) % 3) * ROWB);
    const int rb1 = __builtin_amdgcn_readfirstlane(((2 * ho + 840) % 3) * ROWB);
    const int rb2 = __builtin_amdgcn_readfirstlane(((2 * ho + 1 + 840) % 3) * ROWB);
    if (role) {
      const int co = 16 * ci + 4 * g;
      const char* zb = rings + ck * PLANEB;
      const f32x4 m = *reinterpret_cast<const f32x4*>(bmb + ck * 16 * WCO + co);
      const f32x4 sc = *reinterpret_cast<const f32x4*>(bib + ck * 16 * WCO + co);
      int boff[KST];
#pragma unroll
      for (int s = 0; s < KST; ++s) {
        const int e = ktab_l[g * KST + s];
        const int dyi = e >> 24;
        boff[s] = (dyi == 0 ? rb0 : (dyi == 1 ? rb1 : rb2)) + (e & 0xFFFFFF) - 32768 + ASTR;
      }
      auto epilogue = [&](const f32x4& acc, int wo) __attribute__((always_inline)) {
        if (!(co < WID && wo < Wo)) return;
        bf16x4 y;
        {
          const f32x4 t = (acc + m) * sc;
#pragma unroll
          for (int e = 0; e < 4; ++e) y[e] = (bf16_t)t[e];
        }
        y = relu_bf16(y);
        *reinterpret_cast<bf16x4*>(Bo + (imgo + (size_t)ho * Wo + wo) * q.ldb + ck * WID + co) = y;
      };
      for (int j = 0; j < PT; j += 2) {
        const bool two = j + 1 < PT;
        const int wo0 = 16 * j + col, wo1 = wo0 + 16;
        f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
        constexpr int KH = (KST + 1) / 2;   // B fragments in two halves (register budget)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          bf16x8 b0[KH], b1[KH];
#pragma unroll
          for (int i = 0; i < KH; ++i) {
            const int s = h * KH + i;
            if (s < KST) {
              b0[i] = *reinterpret_cast<const bf16x8*>(zb + boff[s] + 2 * min(wo0, Wo - 1) * ASTR);
              b1[i] = two ? *reinterpret_cast<const bf16x8*>(zb + boff[s] + 2 * min(wo1, Wo - 1) * ASTR)
                          : bf16x8{};
            }
          }
#pragma unroll
          for (int i = 0; i < KH; ++i) {
            const int s = h * KH + i;
            if (s < KST) {
              acc0 = mfma_step(wb[s], b0[i], acc0);
              acc1 = mfma_step(wb[s], b1[i], acc1);
            }
          }
        }
        epilogue(acc0, wo0);
        if (two) epilogue(acc1, wo1);
      }
    } else {
      // last split: AvgPool 3x3/2 VALID over the fixed-padded plane, divisor 9
      // (taps outside the image skipped, in the order of avgpool3s2_v8)
      const char* pl = rings + (S - 1) * PLANEB;
      const int st = tid - 64 * K::ROLES, nst = NT - 64 * K::ROLES;
      for (int it = st; it < Wo * K::WC8; it += nst) {
        const int wo = it / K::WC8, u = it - wo * K::WC8;
        float sum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int hi = 2 * ho - 1 + ky;
          if (hi < 0 || hi >= H) continue;
          const int rb = ky == 0 ? rb0 : (ky == 1 ? rb1 : rb2);
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const int wi = 2 * wo - 1 + kx;
            if (wi < 0 || wi >= W) continue;
            const bf16x8 v = *reinterpret_cast<const bf16x8*>(pl + rb + (wi + 1) * ASTR + u * 16);
#pragma unroll
            for (int e = 0; e < 8; ++e) sum[e] += (float)v[e];
          }
        }
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (bf16_t)(sum[e] / 9.0f);
        *reinterpret_cast<bf16x8*>(Bo + (imgo + (size_t)ho * Wo + wo) * q.ldb + (S - 1) * WID + u * 8) = o;
      }
    }
    __syncthreads();
  }
}

// ----------------------------------------------------------------------------
// Stride-2 block front half in one launch (res2net_model.py:90-93 + 53-77,
// layer-2 block 0): the 1x1a (+BN+ReLU) on the full-resolution block input
// and split_s2_rows' stride-2 branches / average pool, so the 1x1a output
// (S*w channels at full resolution, the largest tensor of the stage) never
// touches HBM.  Output row ho needs 1x1a rows 2ho-1..2ho+1: step ho stages
// input rows 2ho, 2ho+1 (global -> registers one step ahead -> LDS), then
//   phase A: wave (pair pq, row rr) computes 32 1x1a channels of A-row
//            2ho+rr for all pixels (weights in registers) -> 3-row ring;
//   phase B: split_s2_rows' branch waves / pool waves on rows 2ho-1..2ho+1.
// A segment starts with one warm-up step (A-rows 2g0-2, 2g0-1).  Same
// roundings and K orders as the unfused 1x1a + split kernels: bit-identical.
template <int CI, int WID, int S, int WIN>
struct S2FusedCfg {
  static constexpr int WOUT = (WIN + 1) / 2;
  static constexpr int PTO = (WOUT + 15) / 16;   // output pixel tiles
  static constexpr int PTI = (WIN + 15) / 16;    // input pixel tiles
  static constexpr int WR = WIN + 2;             // ring row: pad | WIN | pad
  static constexpr int WCO = (WID + 15) / 16;
  static constexpr int ROLES = (S - 1) * WCO;    // branch (stage, cout tile) waves
  static constexpr int SW = S * WID;
  static constexpr int NPA = SW / 32;            // 1x1a channel pairs
  static constexpr int NW = SW / 16;             // one 1x1a 16-channel tile per wave
  static constexpr int NT = 64 * NW;
  static constexpr int KSA = CI / 32;
  static constexpr int KFLAT = 9 * WID;
  static constexpr int KST = (KFLAT + 31) / 32;
  static constexpr int AU = ((WID / 8) & 1) ? WID / 8 : WID / 8 + 1;
  static constexpr int ASTR = AU * 16;
  // staged input rows: chunk u (8 channels) of pixel px at 16-B unit
  // (u/2) SPX + 2 px + u%2 -- the two lane groups a ds_read_b128 pairs read
  // chunks u, u+1 of 8 distinct pixels: opposite parities, conflict-free
  // (SPX = 2 mod 8 keeps the 8-lane store groups conflict-free too)
  static constexpr int CU = CI / 8;
  static constexpr int SPX = 2 * WIN + 2;
  static constexpr int ROWB = WR * ASTR, PLANEB = 3 * ROWB;
  static constexpr int RING = S * PLANEB;
  static constexpr int INROW = CU / 2 * SPX * 16;
  static_assert(SPX % 8 == 2 && CU % 2 == 0, "staging layout");
  static constexpr int XREG = (2 * WIN * CU + NT - 1) / NT;   // two input rows per step
  static constexpr int KP = (KST + 1) / 2;
  static constexpr int KTB = 64 * KP * 4;        // tap table [lane][k-step] u16
  static constexpr int LDS = RING + 2 * INROW + 4 * (2 * (S - 1) * 16 * WCO + 2 * SW) + KTB;
  static_assert(3 * ROWB + 2 * ROWB < 65536, "tap offsets in 16 bits");
};

template <int CI, int WID, int S, int WIN>
__global__ __launch_bounds__((S2FusedCfg<CI, WID, S, WIN>::NT)) void s2_fused(ChainParams q) {
  using K = S2FusedCfg<CI, WID, S, WIN>;
  constexpr int NT = K::NT, WCO = K::WCO, KST = K::KST, ASTR = K::ASTR, CU = K::CU;
  constexpr int W = WIN, Wo = K::WOUT, ROWB = K::ROWB, PLANEB = K::PLANEB;
  static_assert(K::NW > K::ROLES, "spare waves pool the last split");
  static_assert(K::SW % 32 == 0 && WID % 8 == 0 && CI % 32 == 0, "shape");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int H = q.H;
  const int Ho = (H + 1) / 2;
  const int nseg = q.nwaves;
  const int n = blockIdx.x / nseg;
  const int g0 = (blockIdx.x - n * nseg) * q.R;
  const int g1 = min(Ho, g0 + q.R);
  const int Hn = valid_rows(q.vlen, q.vsh, n, H);   // ragged batch: input rows past it are padding
  char* rings = smem;
  char* inb = smem + K::RING;
  float* bmb = reinterpret_cast<float*>(inb + 2 * K::INROW);
  float* bib = bmb + (S - 1) * 16 * WCO;
  float* bma = bib + (S - 1) * 16 * WCO;          // 1x1a BN [SW]
  float* bia = bma + K::SW;
  unsigned short* ktl = reinterpret_cast<unsigned short*>(bia + K::SW);
  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(q.x);
  bf16_t* __restrict__ Bo = reinterpret_cast<bf16_t*>(q.b);
  const size_t img = (size_t)n * H * W;
  const size_t imgo = (size_t)n * Ho * Wo;

  for (int i = tid; i < K::RING / 16; i += NT)
    reinterpret_cast<uint4*>(rings)[i] = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int k = 0; k < S - 1; ++k)
    for (int c = tid; c < 16 * WCO; c += NT) {
      bmb[k * 16 * WCO + c] = c < WID ? -q.mean[k][c] : 0.f;   // negated: BN as (x + (-m)) * inv
      bib[k * 16 * WCO + c] = c < WID ? q.inv[k][c] : 0.f;
    }
  for (int c = tid; c < K::SW; c += NT) {
    bma[c] = -q.ma[c];
    bia[c] = q.ia[c];
  }

  // branch role weights (registers)
  const bool role = wave < K::ROLES;
  const int ck = role ? wave / WCO : 0;
  const int ci = wave % WCO;
  bf16x8 wb[KST];
  {
    const void* wk = q.wt[0];
#pragma unroll
    for (int k = 1; k < S - 1; ++k)
      if (ck == k) wk = q.wt[k];
    const bf16_t* __restrict__ Wk = reinterpret_cast<const bf16_t*>(wk);
#pragma unroll
    for (int s = 0; s < KST; ++s) {
      const int kk = 32 * s + 8 * g;
      wb[s] = (role && kk < K::KFLAT) ? ld16(Wk + (size_t)(ci * 16 + col) * K::KFLAT + kk)
                                      : bf16x8{};
    }
  }
  // 1x1a: one 16-row tile t of the paired-row weights per wave, for both
  // staged rows; lane (col, g) gets channels 32(t/2) + 8g + 4(t%2) + 0..3
  const int t16 = wave;
  bf16x8 w1[K::KSA];
  {
    const bf16_t* __restrict__ Wa = reinterpret_cast<const bf16_t*>(q.wa);
#pragma unroll
    for (int s = 0; s < K::KSA; ++s)
      w1[s] = ld16(Wa + (size_t)(t16 * 16 + col) * CI + 32 * s + 8 * g);
  }
  // tap table: for lane l and k-step s, the byte offset of its B fragment
  // (output pixel tile 0, stride-2 column 2 col) in the 3-row ring of a plane,
  // counted from the ring row of tap row 0 (before wrapping)
  for (int e = tid; e < 64 * KST; e += NT) {
    const int l = e / KST, st = e - l * KST;
    const int kk = 32 * st + 8 * (l >> 4);
    int dyi = 1, off = 0;
    if (kk < K::KFLAT) {
      const int tap = kk / WID, ch = kk - tap * WID;
      dyi = tap / 3;
      off = (tap % 3 - 1) * ASTR + ch * 2;
    }
    ktl[l * K::KP * 2 + st] = (unsigned short)(dyi * ROWB + off + ASTR + 2 * (l & 15) * ASTR);
  }

  // two input rows per step: global -> registers (one step ahead) -> LDS.
  // The row loads (device_common.h vld16; rows outside the image read a zero
  // line) are waited for by hand right after the phase-A barrier, where only
  // they and the previous step's output stores are in flight.
  vu32x4 xr[K::XREG] = {};
  const int ldx = q.ldx;
  const bf16_t* zline = reinterpret_cast<const bf16_t*>(g_vox_zero);
  auto load_x = [&](int r0) __attribute__((always_inline)) {
    const bf16_t* base = X + (img + (size_t)r0 * W) * ldx;
#pragma unroll
    for (int i = 0; i < K::XREG; ++i) {
      int c = tid + i * NT;
      asm volatile("" : "+v"(c));   // recomputed per step: nothing hoisted into registers
      const int rr = c / (W * CU), cc = c - rr * (W * CU);
      const int px = cc / CU, u = cc - px * CU;
      const int r = r0 + rr;
      const bool ok = rr < 2 && r >= 0 && r < H;
      vld16(xr[i], ok ? (const void*)(base + (rr * W + px) * ldx + u * 8) : zline);
    }
  };
  auto store_x = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < K::XREG; ++i) {
      int c = tid + i * NT;
      asm volatile("" : "+v"(c));
      const int rr = c / (W * CU), cc = c - rr * (W * CU);
      const int px = cc / CU, u = cc - px * CU;
      vm_launder(xr[i]);
      if (rr < 2)
        *reinterpret_cast<vu32x4*>(inb + rr * K::INROW + ((u >> 1) * K::SPX + 2 * px + (u & 1)) * 16) = xr[i];
    }
  };

  // the weights land here, not at a compiler wait inside the row loop
#pragma unroll
  for (int s = 0; s < KST; ++s) vm_launder(wb[s]);
#pragma unroll
  for (int s = 0; s < K::KSA; ++s) vm_launder(w1[s]);
  load_x(2 * (g0 - 1));
  vm_wait(0);
  store_x();
  __syncthreads();
  for (int ho = g0 - 1; ho < g1; ++ho) {
    if (!(VOX_DBG(q) & 8)) load_x(2 * ho + 2);   // lands during this step, goes to LDS at its end
    // ---------------- phase A: 1x1a rows 2ho, 2ho+1 -> ring
    if (!(VOX_DBG(q) & 1)) {
      const int ch = 32 * (t16 >> 1) + 8 * g + 4 * (t16 & 1);
      const int p = ch / WID, off = ch - p * WID;
      const f32x4 m0 = *reinterpret_cast<const f32x4*>(bma + ch);
      const f32x4 i0 = *reinterpret_cast<const f32x4*>(bia + ch);
      // the 2 x PTI (row, pixel tile) items in sequence, the next item's
      // fragments read before this item's MFMAs
      constexpr int NI = 2 * K::PTI;
      // chunk u = 4s + g of pixel pr: sub-plane 2s + g/2, unit 2 pr + g%2
      const int gb = ((g >> 1) * K::SPX + (g & 1)) * 16;
      auto frag = [&](int it, int s) __attribute__((always_inline)) {
        const int rr = it / K::PTI, j = it - rr * K::PTI;
        int pr = min(16 * j + col, W - 1);
        asm volatile("" : "+v"(pr));   // item bases are not hoisted out of the row loop
        return *reinterpret_cast<const bf16x8*>(inb + rr * K::INROW + gb + 32 * pr + 2 * s * K::SPX * 16);
      };
      bf16x8 bc[K::KSA], bn[K::KSA];
#pragma unroll
      for (int s = 0; s < K::KSA; ++s) bc[s] = frag(0, s);
#pragma unroll
      for (int it = 0; it < NI; ++it) {
        const int rr = it / K::PTI, j = it - rr * K::PTI;
        if (it + 1 < NI) {
#pragma unroll
          for (int s = 0; s < K::KSA; ++s) bn[s] = frag(it + 1, s);
        }
        f32x4 a0 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < K::KSA; ++s) a0 = mfma_step(w1[s], bc[s], a0);
        const int r = 2 * ho + rr;
        const bool inimg = r >= 0 && r < Hn;
        char* dst = rings + p * PLANEB + ((r + 840) % 3) * ROWB + off * 2;
        const int px = 16 * j + col;
        bf16x4 o;
        {
          const f32x4 t = (a0 + m0) * i0;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = (bf16_t)t[e];
        }
        o = relu_bf16(o);
        if (!inimg) o = bf16x4{};   // the fixed zero padding of the stride-2 convs
        if (px < W) *reinterpret_cast<bf16x4*>(dst + (px + 1) * ASTR) = o;
#pragma unroll
        for (int s = 0; s < K::KSA; ++s) bc[s] = bn[s];
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __syncthreads();
    if (!(VOX_DBG(q) & 8)) {   // input rows 2ho+2, 2ho+3: phase A is done with the staging
      vm_wait(0);
      store_x();
    }
    // ---------------- phase B: output row ho from A-rows 2ho-1 .. 2ho+1
    if (ho >= g0 && !(VOX_DBG(q) & 2)) {
      const int rb0 = __builtin_amdgcn_readfirstlane(((2 * ho - 1 + 840) % 3) * ROWB);
      const int rb1 = __builtin_amdgcn_readfirstlane(((2 * ho + 840) % 3) * ROWB);
      const int rb2 = __builtin_amdgcn_readfirstlane(((2 * ho + 1 + 840) % 3) * ROWB);
      if (role) {
        const int co = 16 * ci + 4 * g;
        const char* zb = rings + ck * PLANEB;
        const f32x4 m = *reinterpret_cast<const f32x4*>(bmb + ck * 16 * WCO + co);
        const f32x4 sc = *reinterpret_cast<const f32x4*>(bib + ck * 16 * WCO + co);
        unsigned bpk[K::KP];
        {
          const unsigned* kt = reinterpret_cast<const unsigned*>(ktl) + lane * K::KP;
#pragma unroll
          for (int i = 0; i < K::KP; ++i) bpk[i] = kt[i];
        }
        auto boff = [&](int s) __attribute__((always_inline)) {
          const int e = (s & 1) ? (int)(bpk[s >> 1] >> 16) : (int)(bpk[s >> 1] & 0xFFFFu);
          const int v = rb0 + e;
          return v >= 3 * ROWB ? v - 3 * ROWB : v;
        };
        // the PTO output tiles as independent accumulators, fragments one k-step
        // ahead (columns past Wo read the row's tail / the next row: discarded)
        constexpr int PT = K::PTO;
        f32x4 acc[PT];
        bf16x8 bc[PT], bn[PT];
#pragma unroll
        for (int j = 0; j < PT; ++j) {
          acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
          bc[j] = *reinterpret_cast<const bf16x8*>(zb + boff(0) + 32 * j * ASTR);
        }
#pragma unroll
        for (int s = 0; s < KST; ++s) {
          if (s + 1 < KST) {
#pragma unroll
            for (int j = 0; j < PT; ++j)
              bn[j] = *reinterpret_cast<const bf16x8*>(zb + boff(s + 1) + 32 * j * ASTR);
          }
#pragma unroll
          for (int j = 0; j < PT; ++j) acc[j] = mfma_step(wb[s], bc[j], acc[j]);
#pragma unroll
          for (int j = 0; j < PT; ++j) bc[j] = bn[j];
          __builtin_amdgcn_sched_barrier(0);   // reads stay one k-step ahead
        }
        auto ycv = [&](int j) __attribute__((always_inline)) {
          bf16x4 y;
          {
            const f32x4 t = (acc[j] + m) * sc;
#pragma unroll
            for (int e = 0; e < 4; ++e) y[e] = (bf16_t)t[e];
          }
          return __builtin_bit_cast(uint2, relu_bf16(y));
        };
        bf16_t* const brow = Bo + (imgo + (size_t)ho * Wo) * q.ldb + ck * WID;
        if ((q.ldb & 7) == 0) {
          // tiles j, j + 1: a half-row exchange per dword gives lane (col, g) 8
          // contiguous channels 16 ci + 8 (g / 2) of tile j + g % 2 (16-B stores)
#pragma unroll
          for (int j = 0; j + 1 < PT; j += 2) {
            const uint2 d0 = ycv(j), d1 = ycv(j + 1);
            const auto s0 = __builtin_amdgcn_permlane16_swap(d0.x, d1.x, false, false);
            const auto s1 = __builtin_amdgcn_permlane16_swap(d0.y, d1.y, false, false);
            const int wo = 16 * (j + (g & 1)) + col, cq = 16 * ci + 8 * (g >> 1);
            if (cq < WID && wo < Wo)
              *reinterpret_cast<uint4*>(brow + (size_t)wo * q.ldb + cq) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
          }
          if constexpr (PT % 2 == 1) {
            const int wo = 16 * (PT - 1) + col;
            if (co < WID && wo < Wo) *reinterpret_cast<uint2*>(brow + (size_t)wo * q.ldb + co) = ycv(PT - 1);
          }
        } else {
#pragma unroll
          for (int j = 0; j < PT; ++j) {
            const int wo = 16 * j + col;
            if (co < WID && wo < Wo) *reinterpret_cast<uint2*>(brow + (size_t)wo * q.ldb + co) = ycv(j);
          }
        }
      } else if (!(VOX_DBG(q) & 4)) {
        // last split: AvgPool 3x3/2 VALID over the fixed-padded plane, divisor 9
        // (taps outside the image skipped, in the order of avgpool3s2_v8)
        const char* pl = rings + (S - 1) * PLANEB;
        const int st = tid - 64 * K::ROLES, nst = NT - 64 * K::ROLES;
        for (int it = st; it < Wo * (WID / 8); it += nst) {
          const int wo = it / (WID / 8), u = it - wo * (WID / 8);
          float sum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ky = 0; ky < 3; ++ky) {
            const int hi = 2 * ho - 1 + ky;
            if (hi < 0 || hi >= H) continue;
            const int rb = ky == 0 ? rb0 : (ky == 1 ? rb1 : rb2);
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
              const int wi = 2 * wo - 1 + kx;
              if (wi < 0 || wi >= W) continue;
              const bf16x8 v = *reinterpret_cast<const bf16x8*>(pl + rb + (wi + 1) * ASTR + u * 16);
#pragma unroll
              for (int e = 0; e < 8; ++e) sum[e] += (float)v[e];
            }
          }
          bf16x8 o;
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = (bf16_t)(sum[e] / 9.0f);
          *reinterpret_cast<bf16x8*>(Bo + (imgo + (size_t)ho * Wo + wo) * q.ldb + (S - 1) * WID + u * 8) = o;
        }
      }
    }
    __syncthreads();
  }
}

#define S2_FUSED_SHAPES(X) \
  X(128, 48, 4, 80)  /* res2net50_w24_s4_c32 layer-2 block 0, 80-d features */ \
  X(128, 48, 4, 40)  /* ... 40-d features */

int s2_fused_lds(int ci, int wid, int s, int W) {
#define X_LDS(ci_, w_, s_, win_) \
  if (ci == ci_ && wid == w_ && s == s_ && W == win_) return S2FusedCfg<ci_, w_, s_, win_>::LDS;
  S2_FUSED_SHAPES(X_LDS)
#undef X_LDS
  return -1;
}

hipError_t launch_s2_fused(const ChainParams& q, hipStream_t st) {
#define X_LAUNCH(ci_, w_, s_, win_)                                                      \
  if (q.cin == ci_ && q.w == w_ && q.nst + 1 == s_ && q.W == win_) {                      \
    using K = S2FusedCfg<ci_, w_, s_, win_>;                                              \
    hipLaunchKernelGGL((s2_fused<ci_, w_, s_, win_>), dim3(q.N * q.nwaves), dim3(K::NT),  \
                       K::LDS, st, q);                                                    \
    return hipGetLastError();                                                             \
  }
  S2_FUSED_SHAPES(X_LAUNCH)
#undef X_LAUNCH
  return hipErrorInvalidValue;
}

#define SPLIT_S2_SHAPES(X) \
  X(48, 4, 80)  /* res2net50_w24_s4_c32 layer-2 block 0, 80-d features */ \
  X(48, 4, 40)  /* ... 40-d features */

int split_s2_lds(int wid, int s, int W) {
#define X_LDS(w_, s_, win_) \
  if (wid == w_ && s == s_ && W == win_) return SplitS2Cfg<w_, s_, win_>::LDS;
  SPLIT_S2_SHAPES(X_LDS)
#undef X_LDS
  return -1;
}

hipError_t launch_split_s2(const ChainParams& q, hipStream_t st) {
#define X_LAUNCH(w_, s_, win_)                                                             \
  if (q.w == w_ && q.nst + 1 == s_ && q.W == win_) {                                     \
    using K = SplitS2Cfg<w_, s_, win_>;                                                  \
    hipLaunchKernelGGL((split_s2_rows<w_, s_, win_>), dim3(q.N * q.nwaves), dim3(K::NT), \
                       K::LDS, st, q);                                                   \
    return hipGetLastError();                                                            \
  }
  SPLIT_S2_SHAPES(X_LAUNCH)
#undef X_LAUNCH
  return hipErrorInvalidValue;
}

}  // namespace vox

namespace vox {
// copy the bneck_fused trace (diagnostics) to host memory
hipError_t bneck_trace_read(void* dst, size_t bytes) {
  if (bytes > sizeof(g_vox_trace)) bytes = sizeof(g_vox_trace);
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_vox_trace), bytes, 0, hipMemcpyDeviceToHost);
}
}  // namespace vox

// libvoxemb host runtime: weight blob -> device weights, per-shape execution
// plans (one kernel launch per op, pointers into grow-only device slots),
// C-ABI entry points declared in include/voxemb.h.
//
// Graph semantics follow the reference TF1 builders:
//   TDNN    tensorflow/models/tdnn_model.py:24-30,128-161
//   Res2Net tensorflow/models/res2net_model.py:26-136,185-243
//   DPN     tensorflow/models/dpn_model.py:24-171
//   head    res2net_model.py:229-242 / models.py:262-269,306-309
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/voxemb.h"
#include "kernels.h"

using namespace vox;

static thread_local std::string g_err;
static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPCHK(expr)                                                                 \
  do {                                                                               \
    hipError_t e_ = (expr);                                                          \
    if (e_ != hipSuccess)                                                            \
      return fail(VOX_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_));      \
  } while (0)

extern "C" const char* vox_last_error(void) { return g_err.c_str(); }
int vox_set_error(int code, const char* msg) { return fail(code, msg); }

static const float kEps4 = 1.001e-5f;  // fused BN eps clamp (models.py:62-67)
static const float kEps2 = 1e-5f;      // non-fused 2-D head BN (models.py:20)

// ------------------------------------------------------------------ blob
struct HostTensor {
  std::string name, kind;
  std::vector<int> shape;
  std::vector<float> data;
};

struct Spec {
  std::map<std::string, std::string> kv;
  std::string get(const std::string& k) const {
    auto it = kv.find(k);
    return it == kv.end() ? std::string() : it->second;
  }
  int geti(const std::string& k, int dflt = -1) const {
    auto s = get(k);
    return s.empty() ? dflt : std::atoi(s.c_str());
  }
  std::vector<int> getv(const std::string& k) const {
    std::vector<int> v;
    std::stringstream ss(get(k));
    std::string item;
    while (std::getline(ss, item, ','))
      if (!item.empty()) v.push_back(std::atoi(item.c_str()));
    return v;
  }
};

static int parse_blob(const uint8_t* raw, size_t n, Spec& spec, std::vector<HostTensor>& ts) {
  if (n < 16 || std::memcmp(raw, "VOXEMB01", 8) != 0) return fail(VOX_EIO, "not a VOXEMB01 blob");
  uint64_t hlen;
  std::memcpy(&hlen, raw + 8, 8);
  if (16 + hlen > n) return fail(VOX_EIO, "truncated blob header");
  std::string header((const char*)raw + 16, hlen);
  size_t data_start = (16 + hlen + 63) / 64 * 64;
  std::stringstream ss(header);
  std::string line;
  int ntensors = -1;
  while (std::getline(ss, line)) {
    if (line.empty()) continue;
    if (ntensors < 0) {
      auto eq = line.find('=');
      if (eq == std::string::npos) return fail(VOX_EIO, "bad header line: " + line);
      std::string k = line.substr(0, eq), v = line.substr(eq + 1);
      if (k == "tensors") {
        ntensors = std::atoi(v.c_str());
      } else {
        spec.kv[k] = v;
      }
      continue;
    }
    // name|kind|dims|offset|nbytes
    std::vector<std::string> f;
    std::stringstream ls(line);
    std::string item;
    while (std::getline(ls, item, '|')) f.push_back(item);
    if (f.size() != 5) return fail(VOX_EIO, "bad tensor line: " + line);
    HostTensor t;
    t.name = f[0];
    t.kind = f[1];
    std::stringstream ds(f[2]);
    size_t numel = 1;
    while (std::getline(ds, item, ',')) {
      t.shape.push_back(std::atoi(item.c_str()));
      numel *= t.shape.back();
    }
    size_t off = std::strtoull(f[3].c_str(), nullptr, 10);
    size_t nb = std::strtoull(f[4].c_str(), nullptr, 10);
    if (nb != numel * 4 || data_start + off + nb > n)
      return fail(VOX_EIO, "tensor out of range: " + t.name);
    t.data.resize(numel);
    std::memcpy(t.data.data(), raw + data_start + off, nb);
    ts.push_back(std::move(t));
  }
  if (ntensors < 0 || (int)ts.size() != ntensors) return fail(VOX_EIO, "tensor count mismatch");
  return VOX_OK;
}

// ------------------------------------------------------------------ device memory
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t ensure(size_t b) {
    if (b <= bytes) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    hipError_t e = hipMalloc(&p, b);
    if (e == hipSuccess) bytes = b;
    return e;
  }
};

static uint16_t f2bf(float f) {  // round-to-nearest-even (weights only; no NaN here)
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7FFF + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}

// A convolution with its BN, in kernel-native layout.
struct ConvW {
  int kh = 1, kw = 1, cin = 0, cout = 0, groups = 1;  // cin/cout per group
  int coutp = 0, cinp = 0, kp = 0, wco = 1, vec = 1;
  std::shared_ptr<DevBuf> w;         // [groups][coutp][kp] in the model dtype
  std::shared_ptr<DevBuf> wtc;       // bf16 [coutp][taps*cin] for conv_win (groups == 1)
  std::shared_ptr<DevBuf> wpair;     // bf16 [coutp][kp] paired-row layout for conv1x1_rr
  std::shared_ptr<DevBuf> wblk;      // wpair re-blocked for gemm1x1_ws (contiguous 1-KB DMA pieces)
  std::shared_ptr<DevBuf> wstem;     // fp32 [9][cout] for the 1-channel 3x3 stem kernel
  std::shared_ptr<DevBuf> wgc;       // bf16 [C/16][NM][64][8] expanded grouped 3x3 (gconv.hip)
  std::shared_ptr<DevBuf> mean, inv; // optional epilogue BN (cout*groups)
};

struct BNW {
  int c = 0;
  std::shared_ptr<DevBuf> mean, inv;
};

static int choose_wco(int cout_tiles) {
  if (cout_tiles <= 4) return cout_tiles;
  if (cout_tiles <= 6) return 6;
  if (cout_tiles <= 8) return 8;
  if (cout_tiles % 6 == 0 && cout_tiles % 8 != 0) return 6;
  return 8;
}

// ------------------------------------------------------------------ plan
enum OpKind { OP_CONV = 0, OP_POOL = 1, OP_HEAD = 2, OP_OTHER = 3 };
struct Op {
  int kind = OP_CONV;
  int type = 0;  // 0 conv, 1 splitk reduce, 2 stats pool, 3 avgpool, 4 convert
  ConvParams cp{};
  ConvLaunch cl{};
  // reduce
  const float* part = nullptr; int S = 0, M = 0, coutp = 0, cout = 0, flags = 0;
  const float* mean = nullptr; const float* inv = nullptr; float* out = nullptr; int ldo = 0;
  // pool / avgpool / convert
  const void* src = nullptr; void* dst = nullptr; int N = 0, H = 0, W = 0, C = 0, lds = 0, ldd = 0,
             Ho = 0, Wo = 0;
  int64_t count = 0;
  ChainParams ch{};
  BneckParams bq{};  // type 12: Cin (cin), C, w (cl.wco), split (S)
  GconvParams gq{};  // type 19
  DpnBlockParams dq{};  // type 31
  DpnDownParams ddq{};  // type 32
  const float* in_mean = nullptr;  // type 2: input BN+ReLU fused into the pool (DPN68)
  const float* in_inv = nullptr;
  int cin = 0;
  // ragged batches (types 11, 2, 3): per-utterance frames + this op's shift
  const int* vlen = nullptr; int vsh = 0;
  double flops = 0, bytes = 0;
};

enum Slot { S_IN, S_X0, S_X1, S_A, S_B, S_SC, S_POOL, S_PART, S_LEN, S_NSLOTS };

// A layer output the plan exposes for layer-by-layer checks (vox_debug_taps):
// after ops [0, op_end) have run, `p` holds that layer's NHWC output.
struct Tap {
  int op_end;
  const void* p;
  int n, h, w, c, ld;
};

// A built plan kept resident (vox_model::cache): its launches, layer taps and
// captured graph, keyed by the shape and the device pointers it was built for.
struct PlanEntry {
  int n = -1, t = -1;
  bool rag = false;     // ragged-batch plan (vox_embed_device_lens)
  const float* x = nullptr;
  float* out = nullptr;
  std::vector<Op> plan;
  std::vector<Tap> taps;
  hipGraphExec_t exec = nullptr;
  int uses = 0;
  uint64_t used = 0;    // LRU stamp
};

struct vox_model {
  int device = 0;
  DType dt = BF16;
  Spec spec;
  std::string family;
  int feat_dim = 0, out_dim = 0, expand_dim = 3, pooled = 0;
  std::vector<ConvW> convs;  // consumption order
  std::vector<BNW> bns;      // standalone BNs (prologues, pool BN, DPN final)
  ConvW head;                // dense as a 1x1 conv, fp32
  bool att = false;          // attentive statistics pooling (models.py:273-303)
  ConvW att_a, att_b, att_2; // fp32 1x1: W1[:C], W1[C:3C] (mean/std rows), W2
  BNW head_bn1;
  DevBuf slots[S_NSLOTS];
  size_t slot_need[S_NSLOTS] = {};
  hipStream_t stream = nullptr;
  // plan cache
  int plan_n = -1, plan_t = -1;
  bool plan_rag = false;       // built for per-utterance lengths (S_LEN holds them)
  const float* plan_x = nullptr;
  float* plan_out = nullptr;
  std::vector<Op> plan;
  std::vector<Tap> taps;       // layer boundaries of the plan (debug / parity tests)
  // completion of the last launch of the plan: waited for before a rebuild
  // destroys the graph exec or reallocates the slots the launch still uses
  hipEvent_t done = nullptr;
  // the plan's launches captured once into a hipGraph and replayed per call
  // (VOXEMB_NO_GRAPH=1: eager launches); rebuilt with the plan
  bool use_graph = true;
  hipGraphExec_t graph_exec = nullptr;
  // other resident plans (real extraction alternates chunk lengths and ragged
  // last batches): switching to one swaps it in without re-planning or
  // re-capturing.  Every plan points into the shared grow-only slots, so a slot
  // reallocation drops them all.  VOXEMB_PLAN_CACHE = resident plans besides
  // the current one (default 64: every shape of a ragged job -- ~40 padded
  // lengths -- stays resident across passes; 0 = the single-plan behaviour)
  std::vector<PlanEntry> cache;
  int cache_max = 64;
  // calls of the current plan so far; its graph is captured on call
  // graph_after + 1 (a shape met once -- one chunk-length bucket of real
  // extraction -- launches eagerly instead of paying capture + instantiate).
  // VOXEMB_GRAPH_AFTER, default 1
  int plan_uses = 0;
  int graph_after = 1;
  uint64_t clock = 0;
  int64_t plans_built = 0, plan_hits = 0, plans_dropped = 0;
  DevBuf stage_in, stage_out, stage_len;  // host-API staging
  float eps4 = 1.001e-5f, eps2 = 1e-5f;  // BN epsilons (blob header may override)
  // Plan switches: kernel-routing A/B and parity knobs, 0 = the product plan.
  // Read once at load from the environment through kPlanEnv (below); each
  // names the kernel it turns off and the path taken instead.
  int no_win = 0;          // VOXEMB_NO_WIN: conv_win off (generic implicit GEMM)
  int no_rr = 0;           // fixed (env switch removed in round 6); when set: conv1x1_rr off
  int no_gemm = 0;         // VOXEMB_NO_GEMM: the LDS GEMMs off (conv1x1_rr)
  int no_gemm_pipe = 0;    // VOXEMB_NO_GEMM_PIPE: gemm1x1_lds instead of gemm1x1_pipe
  int no_gemm_wide = 0;    // VOXEMB_NO_GEMM_WIDE: gemm1x1_pipe instead of gemm1x1_ws
  int no_wblk = 0;         // fixed (env switch removed in round 6); when set: gemm1x1_ws reads the paired-row weights
  int no_s2_fused = 0;     // VOXEMB_NO_S2_FUSED: 1x1a + split_s2_rows instead of s2_fused
  int no_chain_fused = 0;  // VOXEMB_NO_CHAIN_FUSED: 1x1a + chain_rows instead of chain_fused
  int no_conv3_rw = 0;     // VOXEMB_NO_CONV3_RW: conv3x3_pipe for the w = 96 stride-1 branches
  int no_conv3_ks = 0;     // VOXEMB_NO_CONV3_KS: conv3x3_rw (not K-split) for them
  int no_conv3_utt = 0;    // VOXEMB_NO_CONV3_UTT: conv3x3_pipe for the w = 192 stride-1 branches
  int no_conv3_s2r = 0;    // VOXEMB_NO_CONV3_S2R: conv3x3_pipe for the w = 96 stride-2 branches
  int no_gconv = 0;        // fixed (env switch removed in round 6); when set: grouped 3x3 on the generic implicit GEMM
  int gconv_rs = 0;        // fixed (env switch removed in round 6); when set: grouped 3x3 output rows per step (0 = default)
  int gconv_wgs = 1024;    // fixed (env switch removed in round 6); when set: grouped 3x3 workgroups the row segments aim for
                           // (1,024: 2 segments per utterance at stage 3, 1,453 -> 1,424 us
                           // over its 11 launches against 2,048)
  int no_conv3 = 0;        // VOXEMB_NO_CONV3: every 3x3 branch kernel off
  int no_gemm_pro = 0;     // VOXEMB_NO_GEMM_PRO: prologue 1x1 convs off the LDS-DMA GEMMs
  int no_gemm_taps = 0;    // VOXEMB_NO_GEMM_TAPS: TDNN dilated convs off gemm1x1_ws
  int no_smallk = 0;       // fixed (env switch removed in round 6); when set: DPN 10-channel 1x1s on the generic conv
  int smallk_v1 = 0;       // VOXEMB_SMALLK_V1: conv1x1_smallk (version 1) instead of version 2
  int no_nw = 0;           // VOXEMB_NO_NW: narrow 1x1s on conv1x1_rr instead of conv1x1_nw
  int no_dpn_block = 0;    // VOXEMB_NO_DPN_BLOCK: DPN stage-1 blocks as 1x1a / gconv / 1x1c launches
  int dpn_nseg = 0;        // VOXEMB_DPN_NSEG: force dpn_block_rows' segments per utterance (tests)
  int dpn_dbg = 0;         // VOXEMB_DPN_DBG: dpn_block_rows diagnostics (VOX_DIAG builds)
  int no_pool_pro = 0;     // VOXEMB_NO_POOL_PRO: DPN68's final BN+ReLU as its own pass before the pool
  int pro_min_cout = 192;  // fixed (env switch removed in round 6); when set: narrowest prologue 1x1 on gemm1x1_ws
  int gemm_ksub1 = 0;      // VOXEMB_GEMM_KSUB1: gemm1x1_ws's 128-pixel tiles with one k-step
                           // per ring slot instead of two (bitwise A/B)
  int gemm_var = 0;        // VOXEMB_GEMM_VAR: -1 = gemm1x1_wide instead of gemm1x1_ws
                           // (bitwise A/B); other values are diagnostics (VOX_DIAG builds)
  int gemm_min_k = 128;    // fixed (env switch removed in round 6); when set: smallest K routed to the LDS GEMMs (the K = 128
                           // L2 projection: gemm1x1_ws 0.17 ms vs conv1x1_rr 0.26 ms)
  int no_chain = 0;        // VOXEMB_NO_CHAIN: unfused Res2Net branches
  int no_stem = 0;         // VOXEMB_NO_STEM: stem through the generic conv
  int no_bneck = 0;        // VOXEMB_NO_BNECK: unfused identity bottlenecks
  int no_chain_rows = 0;   // VOXEMB_NO_CHAIN_ROWS: row-tiled split_chain instead
  int no_split_s2 = 0;     // VOXEMB_NO_SPLIT_S2: stride-2 branches as separate convs
  int bneck_nseg = 0;      // fixed (env switch removed in round 6); when set: force row segments per utterance (tests)
  int bneck_dbg = 0;       // VOXEMB_BNECK_DBG: diagnostics (VOX_DIAG builds; skips work)
  int num_cu = 256;        // compute units (persistent grids)
};

// environment name -> plan switch (vox_model fields above)
struct PlanEnv {
  const char* name;
  int vox_model::*field;
};
static const PlanEnv kPlanEnv[] = {
    {"VOXEMB_NO_WIN", &vox_model::no_win},
    {"VOXEMB_NO_GEMM", &vox_model::no_gemm},
    {"VOXEMB_NO_GEMM_PIPE", &vox_model::no_gemm_pipe},
    {"VOXEMB_NO_GEMM_WIDE", &vox_model::no_gemm_wide},
    {"VOXEMB_NO_S2_FUSED", &vox_model::no_s2_fused},
    {"VOXEMB_NO_CHAIN_FUSED", &vox_model::no_chain_fused},
    {"VOXEMB_NO_CONV3_RW", &vox_model::no_conv3_rw},
    {"VOXEMB_NO_CONV3_KS", &vox_model::no_conv3_ks},
    {"VOXEMB_NO_CONV3_UTT", &vox_model::no_conv3_utt},
    {"VOXEMB_NO_CONV3_S2R", &vox_model::no_conv3_s2r},
    {"VOXEMB_NO_CONV3", &vox_model::no_conv3},
    {"VOXEMB_NO_GEMM_PRO", &vox_model::no_gemm_pro},
    {"VOXEMB_NO_GEMM_TAPS", &vox_model::no_gemm_taps},
    {"VOXEMB_SMALLK_V1", &vox_model::smallk_v1},
    {"VOXEMB_NO_NW", &vox_model::no_nw},
    {"VOXEMB_NO_DPN_BLOCK", &vox_model::no_dpn_block},
    {"VOXEMB_DPN_NSEG", &vox_model::dpn_nseg},
    {"VOXEMB_DPN_DBG", &vox_model::dpn_dbg},
    {"VOXEMB_NO_POOL_PRO", &vox_model::no_pool_pro},
    {"VOXEMB_GEMM_VAR", &vox_model::gemm_var},
    {"VOXEMB_GEMM_KSUB1", &vox_model::gemm_ksub1},
    {"VOXEMB_NO_CHAIN", &vox_model::no_chain},
    {"VOXEMB_NO_STEM", &vox_model::no_stem},
    {"VOXEMB_NO_BNECK", &vox_model::no_bneck},
    {"VOXEMB_NO_CHAIN_ROWS", &vox_model::no_chain_rows},
    {"VOXEMB_NO_SPLIT_S2", &vox_model::no_split_s2},
    {"VOXEMB_BNECK_DBG", &vox_model::bneck_dbg},
};

static size_t esize(DType t) { return t == BF16 ? 2 : 4; }

// Upload one HWIO conv kernel (+ optional BN) in kernel-native layout.
static int make_conv(vox_model* m, const HostTensor& k, int groups, const HostTensor* bm,
                     const HostTensor* bv, float eps, DType dt, ConvW& out, int col0 = 0,
                     int ncols = -1) {
  const int kh = k.shape[0], kw = k.shape[1], cin = k.shape[2];
  const int cout_all = k.shape[3];
  if (ncols < 0) ncols = cout_all;
  const int cout = ncols / groups;
  const int taps = kh * kw;
  const int KS = conv_kstep(dt), VN = conv_vec(dt);
  out.kh = kh; out.kw = kw; out.cin = cin; out.cout = cout; out.groups = groups;
  out.vec = (cin % VN == 0) ? 1 : 0;
  const int tiles = (cout + 15) / 16;
  out.wco = choose_wco(tiles);
  out.coutp = ((cout + 16 * out.wco - 1) / (16 * out.wco)) * 16 * out.wco;
  if (out.vec) {
    out.cinp = (cin + KS - 1) / KS * KS;
    out.kp = taps * out.cinp;
  } else {
    out.cinp = cin;
    out.kp = (taps * cin + KS - 1) / KS * KS;
  }
  const size_t per_g = (size_t)out.coutp * out.kp;
  std::vector<float> w(per_g * groups, 0.f);
  for (int g = 0; g < groups; ++g)
    for (int co = 0; co < cout; ++co)
      for (int t = 0; t < taps; ++t)
        for (int ci = 0; ci < cin; ++ci) {
          const int ky = t / kw, kx = t % kw;
          const float v = k.data[(((size_t)ky * kw + kx) * cin + ci) * cout_all + col0 + g * cout + co];
          const size_t kidx = out.vec ? (size_t)t * out.cinp + ci : (size_t)t * cin + ci;
          w[g * per_g + (size_t)co * out.kp + kidx] = v;
        }
  out.w = std::make_shared<DevBuf>();
  const size_t es = esize(dt);
  HIPCHK(out.w->ensure(w.size() * es));
  if (dt == BF16) {
    std::vector<uint16_t> h(w.size());
    for (size_t i = 0; i < w.size(); ++i) h[i] = f2bf(w[i]);
    HIPCHK(hipMemcpy(out.w->p, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  } else {
    HIPCHK(hipMemcpy(out.w->p, w.data(), w.size() * 4, hipMemcpyHostToDevice));
  }
  // 1-D taps along H (TDNN kernels [k,1,Cin,Cout]): the same paired / blocked
  // layouts with K = tap * cinp + ci, for gemm1x1_ws<.., GS_TAPS>
  const bool taps1d = kw == 1 && kh > 1 && out.vec && out.cinp % 32 == 0;
  if (dt == BF16 && groups == 1 && (taps == 1 || taps1d) && out.vec && out.coutp % 32 == 0) {
    // paired rows: row (2q+u)*16 + 4g + e <- channel 32q + 8g + 4u + e;
    // rows padded with zeros to a multiple of 256 (gemm1x1_lds 128-row and
    // gemm1x1_ws 256-row cout tiles, incl. a partial last tile)
    const int rows = (out.coutp + 255) / 256 * 256;
    std::vector<uint16_t> h((size_t)rows * out.kp, 0);
    for (int row = 0; row < out.coutp; ++row) {
      const int q = row / 32, u = (row / 16) & 1, g = (row & 15) / 4, e = row & 3;
      const int co = 32 * q + 8 * g + 4 * u + e;
      if (co >= cout) continue;
      for (int t = 0; t < taps; ++t)
        for (int ci = 0; ci < cin; ++ci)
          h[(size_t)row * out.kp + (size_t)t * out.cinp + ci] =
              f2bf(k.data[((size_t)t * cin + ci) * cout_all + col0 + co]);
    }
    out.wpair = std::make_shared<DevBuf>();
    HIPCHK(out.wpair->ensure(h.size() * 2));
    HIPCHK(hipMemcpy(out.wpair->p, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    if (out.kp % 32 == 0) {
      // gemm1x1_ws weight pieces: block (16-row group rb, k-step kk) is the 1 KB a
      // loader lane set writes into LDS, lane l -> row 16rb + l/4, chunk
      // (l & 3) ^ f(row), f(r) = (4 - ((r >> 2) & 3)) & 3 (gemm_wide.hip gw_swz):
      // one contiguous read of eight full cache lines instead of 16 half lines
      const int KT = out.kp / 32;
      std::vector<uint16_t> b(h.size());
      for (int rb = 0; rb < rows / 16; ++rb)
        for (int kk = 0; kk < KT; ++kk)
          for (int l = 0; l < 64; ++l) {
            const int row = 16 * rb + l / 4;
            const int c = (l & 3) ^ ((4 - ((row >> 2) & 3)) & 3);
            for (int e = 0; e < 8; ++e)
              b[(((size_t)rb * KT + kk) * 64 + l) * 8 + e] = h[(size_t)row * out.kp + kk * 32 + c * 8 + e];
          }
      out.wblk = std::make_shared<DevBuf>();
      HIPCHK(out.wblk->ensure(b.size() * 2));
      HIPCHK(hipMemcpy(out.wblk->p, b.data(), b.size() * 2, hipMemcpyHostToDevice));
    }
  }
  if (dt == BF16 && groups > 1 && kh == 3 && kw == 3 && cin == cout &&
      (cin == 4 || cin == 8 || cin == 16 || cin == 32) && (cout * groups) % 64 == 0) {
    // gconv.hip A fragments: slab sg = output channels [16sg, 16sg+16), MFMA m,
    // lane l -> row co = 16sg + (l & 15), k-group q = l >> 4, element e:
    //   gw 32: tap m, input channel 8q+e of the group;
    //   gw <= 16: tap 2m + (q>>1) (tap 9 = zero), input channel 16sg + 8(q&1) + e,
    //             zero unless it lies in co's group (block-diagonal)
    const int gw = cin, C = cout * groups, NM = gw == 32 ? 9 : 5;
    std::vector<uint16_t> h((size_t)C / 16 * NM * 64 * 8, 0);
    for (int sg = 0; sg < C / 16; ++sg)
      for (int mm = 0; mm < NM; ++mm)
        for (int l = 0; l < 64; ++l)
          for (int e = 0; e < 8; ++e) {
            const int co = 16 * sg + (l & 15), q = l >> 4;
            int tap, ci;
            if (gw == 32) {
              tap = mm;
              ci = 32 * (co / 32) + 8 * q + e;
            } else {
              tap = 2 * mm + (q >> 1);
              ci = 16 * sg + 8 * (q & 1) + e;
            }
            if (tap >= 9 || ci / gw != co / gw) continue;
            h[(((size_t)sg * NM + mm) * 64 + l) * 8 + e] =
                f2bf(k.data[((size_t)tap * cin + ci % gw) * cout_all + col0 + co]);
          }
    out.wgc = std::make_shared<DevBuf>();
    HIPCHK(out.wgc->ensure(h.size() * 2));
    HIPCHK(hipMemcpy(out.wgc->p, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  }
  if (groups == 1 && cin == 1 && kh == 3 && kw == 3 && cout <= 64) {
    std::vector<float> h(9 * (size_t)cout);
    for (int t = 0; t < 9; ++t)
      for (int co = 0; co < cout; ++co) {
        float v = k.data[(size_t)t * cout_all + col0 + co];
        if (dt == BF16) {  // the same bf16 value the MFMA path would use
          const uint32_t u = (uint32_t)f2bf(v) << 16;
          std::memcpy(&v, &u, 4);
        }
        h[(size_t)t * cout + co] = v;
      }
    out.wstem = std::make_shared<DevBuf>();
    HIPCHK(out.wstem->ensure(h.size() * 4));
    HIPCHK(hipMemcpy(out.wstem->p, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  }
  if (dt == BF16 && groups == 1 && cin % 8 == 0) {
    std::vector<uint16_t> h((size_t)out.coutp * taps * cin, 0);
    for (int co = 0; co < cout; ++co)
      for (int t = 0; t < taps; ++t)
        for (int ci = 0; ci < cin; ++ci) {
          const int ky = t / kw, kx = t % kw;
          h[((size_t)co * taps + t) * cin + ci] =
              f2bf(k.data[(((size_t)ky * kw + kx) * cin + ci) * cout_all + col0 + co]);
        }
    out.wtc = std::make_shared<DevBuf>();
    HIPCHK(out.wtc->ensure(h.size() * 2));
    HIPCHK(hipMemcpy(out.wtc->p, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  }
  if (bm) {
    const int C = (int)bm->data.size();
    std::vector<float> inv(C);
    for (int c = 0; c < C; ++c) inv[c] = 1.0f / std::sqrt(bv->data[c] + eps);
    out.mean = std::make_shared<DevBuf>();
    out.inv = std::make_shared<DevBuf>();
    HIPCHK(out.mean->ensure(C * 4));
    HIPCHK(out.inv->ensure(C * 4));
    HIPCHK(hipMemcpy(out.mean->p, bm->data.data(), C * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(out.inv->p, inv.data(), C * 4, hipMemcpyHostToDevice));
  }
  return VOX_OK;
}

static int make_bn(const HostTensor& bm, const HostTensor& bv, float eps, BNW& out, int off = 0,
                   int len = -1) {
  if (len < 0) len = (int)bm.data.size();
  std::vector<float> inv(len);
  for (int c = 0; c < len; ++c) inv[c] = 1.0f / std::sqrt(bv.data[off + c] + eps);
  out.c = len;
  out.mean = std::make_shared<DevBuf>();
  out.inv = std::make_shared<DevBuf>();
  HIPCHK(out.mean->ensure(len * 4));
  HIPCHK(out.inv->ensure(len * 4));
  HIPCHK(hipMemcpy(out.mean->p, bm.data.data() + off, len * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(out.inv->p, inv.data(), len * 4, hipMemcpyHostToDevice));
  return VOX_OK;
}

// tf.nn.batch_normalization (the non-fused inference BN TF1 uses for a 2-D
// input, models.py:62-67 via tf.compat.v1.layers): y = x * inv + (-mean * inv).
// Overwrites a BN's mean table with -mean * inv, inv computed exactly as in
// make_bn / make_conv
static int bn_nonfused_offsets(const HostTensor& bm, const HostTensor& bv, float eps, DevBuf& dst) {
  const int C = (int)bm.data.size();
  std::vector<float> nmi(C);
  for (int c = 0; c < C; ++c) {
    const float inv = 1.0f / std::sqrt(bv.data[c] + eps);
    nmi[c] = -bm.data[c] * inv;
  }
  HIPCHK(hipMemcpy(dst.p, nmi.data(), C * 4, hipMemcpyHostToDevice));
  return VOX_OK;
}

struct Cursor {
  const std::vector<HostTensor>& ts;
  size_t i = 0;
  explicit Cursor(const std::vector<HostTensor>& t) : ts(t) {}
  const HostTensor* next(const char* kind_hint) {
    if (i >= ts.size()) {
      g_err = std::string("blob exhausted, expected ") + kind_hint;
      return nullptr;
    }
    return &ts[i++];
  }
};

#define NEXT(var, hint)                                  \
  const HostTensor* var = cur.next(hint);                \
  if (!var) return VOX_EIO;

static int load_weights(vox_model* m, const std::vector<HostTensor>& ts) {
  Cursor cur(ts);
  const DType dt = m->dt;
  int rc;
  auto conv_bn = [&](float eps, ConvW& cw) -> int {
    const HostTensor* k = cur.next("conv");
    const HostTensor* bm = cur.next("bn mean");
    const HostTensor* bv = cur.next("bn var");
    if (!k || !bm || !bv) return VOX_EIO;
    return make_conv(m, *k, 1, bm, bv, eps, dt, cw);
  };
  if (m->family == "tdnn") {
    for (size_t l = 0; l < m->spec.getv("filters").size(); ++l) {
      ConvW cw;
      if ((rc = conv_bn(m->eps4, cw))) return rc;
      m->convs.push_back(cw);
    }
  } else if (m->family == "res2net") {
    const int s = m->spec.geti("split");
    auto blocks = m->spec.getv("block_sizes");
    ConvW stem;
    if ((rc = conv_bn(m->eps4, stem))) return rc;
    m->convs.push_back(stem);
    for (size_t st = 0; st < blocks.size(); ++st)
      for (int b = 0; b < blocks[st]; ++b) {
        if (b == 0) {
          ConvW pr;
          if ((rc = conv_bn(m->eps4, pr))) return rc;
          m->convs.push_back(pr);
        }
        ConvW a;
        if ((rc = conv_bn(m->eps4, a))) return rc;
        m->convs.push_back(a);
        NEXT(k, "split kernel");
        const int w = k->shape[2];
        for (int j = 0; j < s - 1; ++j) {
          NEXT(bm, "split bn mean");
          NEXT(bv, "split bn var");
          ConvW br;
          if ((rc = make_conv(m, *k, 1, bm, bv, m->eps4, dt, br, j * w, w))) return rc;
          m->convs.push_back(br);
        }
        ConvW c;
        if ((rc = conv_bn(m->eps4, c))) return rc;
        m->convs.push_back(c);
      }
    if (m->spec.get("pool") == "att") {   // att_stats_pool kernels [1,1,3C,A], [1,1,A,C]
      NEXT(k1, "attention kernel 1");
      NEXT(k2, "attention kernel 2");
      const int C3 = k1->shape[2], A = k1->shape[3], C = C3 / 3;
      if (C3 != 3 * C || k2->shape[2] != A || k2->shape[3] != C)
        return fail(VOX_EIO, "attention kernel shapes");
      HostTensor ka = *k1, kb = *k1;
      ka.shape = {1, 1, C, A};
      ka.data.assign(k1->data.begin(), k1->data.begin() + (size_t)C * A);
      kb.shape = {1, 1, 2 * C, A};
      kb.data.assign(k1->data.begin() + (size_t)C * A, k1->data.end());
      if ((rc = make_conv(m, ka, 1, nullptr, nullptr, 0.f, F32, m->att_a))) return rc;
      if ((rc = make_conv(m, kb, 1, nullptr, nullptr, 0.f, F32, m->att_b))) return rc;
      if ((rc = make_conv(m, *k2, 1, nullptr, nullptr, 0.f, F32, m->att_2))) return rc;
      m->att = true;
    }
  } else if (m->family == "dpn") {
    const int G = m->spec.geti("cardinality");
    ConvW stem;
    if ((rc = conv_bn(m->eps4, stem))) return rc;
    m->convs.push_back(stem);
    // every body conv is BN->ReLU->conv: BN becomes the conv's prologue
    auto ks = m->spec.getv("k_sec");
    for (size_t st = 0; st < ks.size(); ++st)
      for (int b = 0; b < ks[st]; ++b) {
        const int nconv = (b == 0) ? 4 : 3;
        for (int j = 0; j < nconv; ++j) {
          NEXT(bm, "bn mean");
          NEXT(bv, "bn var");
          NEXT(k, "conv");
          BNW pro;
          if ((rc = make_bn(*bm, *bv, m->eps4, pro))) return rc;
          m->bns.push_back(pro);
          ConvW cw;
          const int groups = (k->shape[0] == 3) ? G : 1;
          if ((rc = make_conv(m, *k, groups, nullptr, nullptr, m->eps4, dt, cw))) return rc;
          m->convs.push_back(cw);
        }
      }
    NEXT(fm, "final bn mean");
    NEXT(fv, "final bn var");
    BNW fin;
    if ((rc = make_bn(*fm, *fv, m->eps4, fin))) return rc;
    m->bns.push_back(fin);
  } else {
    return fail(VOX_EINVAL, "unknown family " + m->family);
  }
  // head: BN(2-D) -> dense -> BN(2-D), dense in fp32 as a 1x1 conv
  NEXT(h1m, "head bn1 mean");
  NEXT(h1v, "head bn1 var");
  NEXT(dk, "dense kernel");
  NEXT(h2m, "head bn2 mean");
  NEXT(h2v, "head bn2 var");
  if ((rc = make_bn(*h1m, *h1v, m->eps2, m->head_bn1))) return rc;
  HostTensor dk4 = *dk;  // [D, out] -> HWIO [1,1,D,out]
  dk4.shape = {1, 1, dk->shape[0], dk->shape[1]};
  if ((rc = make_conv(m, dk4, 1, h2m, h2v, m->eps2, F32, m->head))) return rc;
  // both head BNs are 2-D, so TF1 runs them non-fused: their mean tables hold
  // -mean * inv for the kernels' bn2d (EPI_BN2D)
  if ((rc = bn_nonfused_offsets(*h1m, *h1v, m->eps2, *m->head_bn1.mean))) return rc;
  if ((rc = bn_nonfused_offsets(*h2m, *h2v, m->eps2, *m->head.mean))) return rc;
  m->pooled = dk->shape[0];
  m->out_dim = dk->shape[1];
  if (cur.i != ts.size()) return fail(VOX_EIO, "blob has trailing tensors");
  return VOX_OK;
}

// ------------------------------------------------------------------ plan builder
struct Builder {
  vox_model* m;
  bool dry;
  std::vector<Op>* ops;
  // ragged batches: the device frame counts every row-aware kernel reads, and
  // the downsampling shift of the rows the ops being emitted read
  const int* vlen = nullptr;
  int vsh = 0;
  char* base(Slot s, size_t bytes) {
    m->slot_need[s] = std::max(m->slot_need[s], bytes);
    return dry ? nullptr : (char*)m->slots[s].p;
  }
  void tap(const void* p, int n, int h, int w, int c, int ld) {
    m->taps.push_back(Tap{(int)ops->size(), p, n, h, w, c, ld});
  }
};

struct Act {  // an NHWC activation view
  const void* p;
  int ld, N, H, W, C;
};

static size_t es_of(vox_model* m) { return esize(m->dt); }

static void emit_conv(Builder& B, const ConvW& cw, Act x, const void* x2, int ldx2, int sh,
                      int sw, int dh, int dw, int ph, int pw, int Ho, int Wo, void* y, int ldy,
                      int flags, const void* res = nullptr, int ldr = 0, void* y2 = nullptr,
                      int ldy2 = 0, int ysplit = 1 << 30, const float* in_mean = nullptr,
                      const float* in_inv = nullptr, DType dt_override = (DType)-1) {
  Op op;
  op.kind = OP_CONV;
  op.type = 0;
  ConvParams& p = op.cp;
  p.x = x.p; p.ldx = x.ld; p.x2 = x2; p.ldx2 = ldx2;
  p.in_mean = in_mean; p.in_inv = in_inv;
  p.w = cw.w->p; p.kp = cw.kp;
  p.y = y; p.ldy = ldy; p.y2 = y2; p.ldy2 = ldy2; p.ysplit = ysplit;
  p.res = res; p.ldr = ldr;
  p.mean = cw.mean ? (const float*)cw.mean->p : nullptr;
  p.inv = cw.inv ? (const float*)cw.inv->p : nullptr;
  p.partial = nullptr;
  p.N = x.N; p.H = x.H; p.W = x.W; p.Cin = cw.cin; p.Ho = Ho; p.Wo = Wo; p.Cout = cw.cout;
  p.coutp = cw.coutp;
  p.kh = cw.kh; p.kw = cw.kw; p.sh = sh; p.sw = sw; p.dh = dh; p.dw = dw; p.ph = ph; p.pw = pw;
  p.cinp = cw.cinp; p.kchunk = 0; p.flags = flags;
  p.groups = cw.groups;
  p.cblocks = cw.coutp / (16 * cw.wco);
  // TDNN: one kernel route per layer whatever the batch (gemm1x1_ws even for a
  // handful of tiles), so an utterance's embedding bits do not depend on its
  // batch (tf_extract.py:27 extracts every utterance on its own)
  p.any_m = B.m->family == "tdnn" ? 1 : 0;
  p.vlen = B.vlen; p.vsh = B.vsh;
  p.fast4 = (cw.cout % 4 == 0 && ldy % 4 == 0 && (ysplit >= (1 << 30) || (ysplit % 4 == 0 && ldy2 % 4 == 0)) &&
             (!res || ldr % 4 == 0) && cw.groups == 1) ? 1 : 0;
  op.cl.wco = cw.wco;
  op.cl.vec = cw.vec;
  op.cl.splitk = 1;
  const int M = x.N * Ho * Wo;
  op.cl.wpx = M >= 64 * 4 * 512 ? 4 : (M >= 64 * 2 * 256 ? 2 : 1);
  // bf16 1x1 with K <= 256: register-resident activations, all couts per wave
  const int ks_rr = (cw.cinp + 31) / 32;
  if (B.m->dt == BF16 && dt_override != F32 && cw.wpair && !(flags & EPI_PARTIAL) &&
      !B.m->no_rr && ph == 0 && pw == 0 && cw.cout % 8 == 0 && ldy % 8 == 0 &&
      (ysplit >= (1 << 30) || (ysplit % 8 == 0 && ldy2 % 8 == 0)) && (!res || ldr % 8 == 0) &&
      x.ld % 8 == 0 &&
      (ks_rr == 1 || ks_rr == 2 || ks_rr == 3 || ks_rr == 4 || ks_rr == 6 || ks_rr == 8 ||
       ks_rr == 12 || ks_rr == 16 || ks_rr == 24 || ks_rr == 32)) {
    op.type = 8;
    p.w = cw.wpair->p;
    op.cl.wco = 2;  // measured best (tools/sweep_rr.sh): occupancy over tile size
    // enough waves: pixel tiles x cout ranges >= ~2048 blocks' worth
    int wpx = conv1x1_rr_max_wpx(ks_rr);
    while (wpx > 1 && (M + 64 * wpx - 1) / (64 * wpx) < 1024) wpx /= 2;
    op.cl.wpx = wpx;
    const int gx = (M + 64 * wpx - 1) / (64 * wpx);
    const int tiles = cw.coutp / 16;
    int ys = 1;
    while (gx * ys < 1024 && tiles / (ys * 2) >= op.cl.wco) ys *= 2;
    op.cl.splitk = ys;
    // compute-bound shapes: LDS-tiled 128x128 GEMM (cout padded to 128-row
    // tiles with zero weights when that wastes at most a third of the tile)
    const int cout128 = (cw.cout + 127) / 128 * 128;
    if (!B.m->no_gemm && !in_mean && cw.cinp % 64 == 0 && cw.cinp >= B.m->gemm_min_k &&
        cw.cout >= 128 && 3 * (cout128 - cw.cout) <= cout128) {
      op.type = 9;
      p.coutp = cout128;
      // persistent LDS-DMA pipelined GEMM (gemm.hip) where its tiling applies
      if (!B.m->no_gemm_pipe && gemm_pipe_ok(p)) op.type = 18;
      // wide-tile variant (gemm_wide.hip): 256 x 256 / 256 x 192 tiles, residual
      // streamed through the DMA ring
      if (!B.m->no_gemm_wide && gemm_wide_bn(p)) {
        op.type = 21;
        p.wblk = (cw.wblk && !B.m->no_wblk) ? cw.wblk->p : nullptr;
      }
    }
  }
  // narrow 1x1s (K <= 256, <= 192 couts): weights resident in LDS (gemm_nw.hip)
  if (op.type == 8 && !B.m->no_nw && conv1x1_nw_ok(p)) op.type = 29;
  // bf16 1x1 with a BN+ReLU input prologue (DPN bn_relu_conv, >= 192 couts):
  // the wave-specialised GEMM applies it to its B fragments
  // (gemm1x1_ws<.., GS_PRO>; a padded K reads finite neighbouring channels
  // that the prologue zeroes, slots carry slack for the last row)
  if (op.type != 18 && op.type != 21 && B.m->dt == BF16 && dt_override != F32 && in_mean &&
      cw.wblk && !B.m->no_gemm_wide && !B.m->no_gemm_pro && !(flags & EPI_PARTIAL) && ph == 0 &&
      pw == 0 && cw.kh == 1 && cw.kw == 1 && cw.groups == 1 && cw.cout >= B.m->pro_min_cout &&
      cw.cout % 8 == 0 &&
      ldy % 8 == 0 && (ysplit >= (1 << 30) || (ysplit % 8 == 0 && ldy2 % 8 == 0)) &&
      (!res || ldr % 8 == 0) && x.ld % 8 == 0) {
    ConvParams q = p;
    q.w = cw.wpair->p;
    q.wblk = cw.wblk->p;
    if (gemm_wide_bn(q)) {
      p = q;
      op.type = 21;
    }
  }
  // 1-D dilated taps along time (TDNN, W = 1): the wave-specialised GEMM
  // gathers every tap's input rows itself (gemm1x1_ws<.., GS_TAPS>)
  if (op.type == 0 && B.m->dt == BF16 && dt_override != F32 && cw.wblk && cw.groups == 1 &&
      cw.kw == 1 && cw.kh > 1 && x.W == 1 && Wo == 1 && Ho == x.H && sh == 1 && sw == 1 &&
      pw == 0 && !in_mean && !x2 && !res && !(flags & EPI_PARTIAL) && !B.m->no_gemm_wide &&
      !B.m->no_gemm_taps && x.ld % 8 == 0 && ldy % 8 == 0 && ysplit >= (1 << 30)) {
    ConvParams q = p;
    q.w = cw.wpair->p;
    q.wblk = cw.wblk->p;
    if (gemm_wide_bn(q)) {
      p = q;
      op.type = 21;
    }
  }
  // bf16 1x1 with a BN+ReLU input prologue (DPN bn_relu_conv): the pipelined
  // GEMM applies the prologue to its pixel fragments (gemm1x1_pipe<.., PRO>)
  if (op.type != 18 && op.type != 21 && B.m->dt == BF16 && dt_override != F32 && in_mean && cw.wpair &&
      !B.m->no_gemm_pipe && !B.m->no_gemm_pro && !(flags & EPI_PARTIAL) && ph == 0 && pw == 0 &&
      cw.kh == 1 && cw.kw == 1 && cw.groups == 1 && cw.cout % 8 == 0 && ldy % 8 == 0 &&
      (ysplit >= (1 << 30) || (ysplit % 8 == 0 && ldy2 % 8 == 0)) && (!res || ldr % 8 == 0) &&
      x.ld % 8 == 0 && cw.kp <= x.ld) {
    const int cout128 = (cw.cout + 127) / 128 * 128;
    if (cw.cout >= 128 && 3 * (cout128 - cw.cout) <= cout128) {
      ConvParams q = p;
      q.coutp = cout128;
      q.w = cw.wpair->p;
      if (gemm_pipe_ok(q)) {
        p = q;
        op.type = 18;
      }
    }
  }
  // bf16 convs (stride 1 or 2) without prologue: window-staged LDS kernel if
  // some (pixel tile, cout tile, channel chunk) fits the LDS budget
  // stride 2 only pays off for wide inputs (measured: L4 yes, L2/L3 no)
  if (op.type == 0 && B.m->dt == BF16 && dt_override != F32 && cw.wtc && sh == sw &&
      (sh == 1 || (sh == 2 && cw.cin >= 192)) && !in_mean && !(flags & EPI_PARTIAL) &&
      !B.m->no_win) {
    const int taps = cw.kh * cw.kw;
    const int minoff = -(ph * x.W + pw);
    const int maxoff = ((cw.kh - 1) * dh - ph) * x.W + (cw.kw - 1) * dw - pw;
    const int HoWo = Ho * Wo;
    auto in_flat = [&](long pix) -> long {
      const long n = pix / HoWo, r = pix % HoWo;
      return (n * x.H + (r / Wo) * sh) * (long)x.W + (r % Wo) * sw;
    };
    auto span = [&](int bp) -> long {  // max input-index span of a block's pixels
      if (sh == 1) return bp - 1;
      long mx = 0;
      for (long b0 = 0; b0 < M; b0 += bp)
        mx = std::max(mx, in_flat(std::min<long>(b0 + bp, M) - 1) - in_flat(b0));
      return mx;
    };
    std::vector<int> wcos = {cw.wco};
    for (int w : {6, 4, 3, 2, 1})
      if (w < cw.wco && cw.coutp % (16 * w) == 0) wcos.push_back(w);
    const int kcs[] = {cw.cin, 256, 128, 64, 32, 16, 8};
    const int LDS_MAX = 64 * 1024;
    bool done = false;
    for (int wpx : {4, 2, 1}) {
      if (done) break;
      if (wpx > 1 && M < 64 * wpx * 256) continue;  // keep >= 256 blocks when possible
      const long len = span(64 * wpx) + 1 + maxoff - minoff;
      // pass 0: full K at any cout tile (same tap-major K order as every
      // other conv path, so results are bitwise identical); pass 1: channel
      // chunks, largest cout tile first
      for (int pass = 0; pass < 2 && !done; ++pass)
      for (int wco : wcos) {
        if (done) break;
        for (int kc : kcs) {
          if (pass == 0 && kc != cw.cin) continue;
          if (kc > cw.cin || kc % 8) continue;
          if (kc != cw.cin && kc > 128) continue;
          int au = kc / 8;
          if (!(au & 1)) ++au;
          const int kcp = (taps * kc + 31) / 32 * 32;
          int wu = kcp / 8;
          if (!(wu & 1)) ++wu;
          const long lds = len * au * 16 + 16L * wco * wu * 16 + (kcp / 8) * 16;
          if (lds > LDS_MAX) continue;
          p.win_lo = minoff; p.win_len = (int)len; p.win_kc = kc;
          p.win_astr = au * 16; p.win_wstr = wu * 16; p.win_lds = (int)lds;
          p.w = cw.wtc->p;
          p.cblocks = cw.coutp / (16 * wco);
          op.cl.wco = wco;
          op.cl.wpx = wpx;
          op.type = 7;
          done = true;
          break;
        }
      }
    }
  }
  // 10-channel input (DPN68 stem output) with the prologue: vector-ALU kernel
  if (op.type == 0 && B.m->dt == BF16 && dt_override != F32 && in_mean && !B.m->no_smallk &&
      conv1x1_smallk_ok(p))
    op.type = 27;
  if (dt_override == F32) op.type = 5;
  const double es = dt_override == F32 ? 4.0 : (double)es_of(B.m);
  op.flops = 2.0 * M * cw.cout * cw.groups * (double)cw.kh * cw.kw * cw.cin;
  // algorithmic input bytes = the input pixels the conv samples: a kernel
  // narrower than its stride (the stride-2 1x1 projections,
  // res2net_model.py:125-127) reads only min(k, s) of every s rows / columns
  const double rows_in = std::min<double>(x.H, (double)Ho * std::min(cw.kh, sh) + (cw.kh > sh ? cw.kh - sh : 0));
  const double cols_in = std::min<double>(x.W, (double)Wo * std::min(cw.kw, sw) + (cw.kw > sw ? cw.kw - sw : 0));
  op.bytes = es * ((double)x.N * rows_in * cols_in * cw.cin * cw.groups * (x2 ? 2 : 1) +
                   (double)M * cw.cout * cw.groups * (res ? 2 : 1));
  // + the weights once per XCD: each of the 8 XCDs' L2s fetches a layer's
  // weights for its own workgroups (the floor once tiles spread over the chip;
  // at B = 256 <= 0.5 % of a Res2Net 1x1's bytes, at the TDNN's B = 64 the
  // k = 3 layers' 1.5 MB x 8 is a third of them, DESIGN.md "TDNN traffic")
  op.bytes += 8.0 * es * (double)cw.groups * cw.cout * cw.cin * cw.kh * cw.kw;
  B.ops->push_back(op);
}

static void emit_pool(Builder& B, Act x, float* out, const BNW& bn, const BNW* in_bn = nullptr) {
  Op op;
  op.kind = OP_POOL;
  op.type = 2;
  op.vlen = B.vlen; op.vsh = B.vsh;
  op.src = x.p; op.N = x.N; op.H = x.H; op.W = x.W; op.C = x.C;
  op.mean = (const float*)bn.mean->p;
  op.inv = (const float*)bn.inv->p;
  if (in_bn) {
    op.in_mean = (const float*)in_bn->mean->p;
    op.in_inv = (const float*)in_bn->inv->p;
  }
  op.out = out;
  op.bytes = (double)es_of(B.m) * x.N * x.H * x.W * x.C + 4.0 * x.N * x.W * 2 * x.C;
  B.ops->push_back(op);
}

// Attentive statistics pooling (models.py:273-303) in fp32:
//   S = [mean, std] over time              (stats-pool kernel, no BN)
//   Bnw = S W1[C:3C]                        (fp32 1x1 over the N*W rows)
//   H = tanh(x W1[:C] + Bnw)                (fp32 1x1 + bias/tanh kernel)
//   L = H W2 ; softmax over time ; weighted mean/std ; head BN -> pooled
static void emit_att_pool(Builder& B, Act x, float* pooled, Slot free_s) {
  vox_model* m = B.m;
  const int n = x.N, H = x.H, W = x.W, C = x.C, A = m->att_a.cout;
  float* S = (float*)B.base(S_B, (size_t)n * W * 2 * C * 4);
  float* bnw = (float*)B.base(S_PART, (size_t)n * W * A * 4);
  float* hb = (float*)B.base(S_SC, (size_t)n * H * W * A * 4);
  float* lg = (float*)B.base(free_s, (size_t)n * H * W * C * 4);
  {
    Op op;
    op.kind = OP_POOL;
    op.type = 2;
    op.src = x.p; op.N = n; op.H = H; op.W = W; op.C = C;
    op.mean = nullptr; op.inv = nullptr; op.out = S;
    op.bytes = (double)es_of(m) * n * H * W * C + 4.0 * n * W * 2 * C;
    B.ops->push_back(op);
  }
  emit_conv(B, m->att_b, Act{S, 2 * C, n * W, 1, 1, 2 * C}, nullptr, 0, 1, 1, 1, 1, 0, 0, 1, 1, bnw,
            A, 0, nullptr, 0, nullptr, 0, 1 << 30, nullptr, nullptr, F32);
  const float* x32 = (const float*)x.p;
  if (m->dt == BF16) {
    float* xc = (float*)B.base(S_A, (size_t)n * H * W * C * 4);
    Op op;
    op.kind = OP_OTHER;
    op.type = 15;
    op.src = x.p; op.dst = xc; op.count = (int64_t)n * H * W * C;
    op.bytes = 6.0 * op.count;
    B.ops->push_back(op);
    x32 = xc;
  }
  emit_conv(B, m->att_a, Act{x32, C, n, H, W, C}, nullptr, 0, 1, 1, 1, 1, 0, 0, H, W, hb, A, 0,
            nullptr, 0, nullptr, 0, 1 << 30, nullptr, nullptr, F32);
  {
    Op op;
    op.kind = OP_OTHER;
    op.type = 16;
    op.dst = hb; op.src = bnw; op.N = n; op.H = H; op.W = W; op.C = A;
    op.bytes = 8.0 * n * H * W * A;
    B.ops->push_back(op);
  }
  emit_conv(B, m->att_2, Act{hb, A, n, H, W, A}, nullptr, 0, 1, 1, 1, 1, 0, 0, H, W, lg, C, 0,
            nullptr, 0, nullptr, 0, 1 << 30, nullptr, nullptr, F32);
  Op op;
  op.kind = OP_POOL;
  op.type = 17;
  op.src = x.p; op.part = lg; op.N = n; op.H = H; op.W = W; op.C = C;
  op.mean = (const float*)m->head_bn1.mean->p;
  op.inv = (const float*)m->head_bn1.inv->p;
  op.out = pooled;
  op.bytes = (double)es_of(m) * n * H * W * C + 4.0 * n * H * W * C + 4.0 * n * W * 2 * C;
  B.ops->push_back(op);
}

static void emit_head(Builder& B, const float* pooled, int n, float* out) {
  vox_model* m = B.m;
  const ConvW& hw = m->head;
  const int D = hw.cin;
  // split-K over a partition fixed per model (never per batch size n), so an
  // utterance's fp32 partial sums -- and its embedding bits -- do not depend on
  // its batch mates: ~256 K-slices x cout blocks (one 64-row block per slice)
  const int gy = hw.coutp / (16 * hw.wco);
  int S = std::max(1, std::min(64, 256 / std::max(1, gy)));
  int kchunk = (hw.cinp + S - 1) / S;
  kchunk = (kchunk + 15) / 16 * 16;
  S = (hw.cinp + kchunk - 1) / kchunk;
  float* part = (float*)B.base(S_PART, (size_t)S * n * hw.coutp * 4);
  Op op;
  op.kind = OP_HEAD;
  op.type = 0;
  ConvParams& p = op.cp;
  std::memset(&p, 0, sizeof(p));
  p.x = pooled; p.ldx = D;
  p.w = hw.w->p; p.kp = hw.kp;
  p.partial = part;
  p.N = n; p.H = 1; p.W = 1; p.Cin = D; p.Ho = 1; p.Wo = 1; p.Cout = hw.cout; p.coutp = hw.coutp;
  p.kh = 1; p.kw = 1; p.sh = p.sw = p.dh = p.dw = 1;
  p.cinp = hw.cinp; p.kchunk = kchunk; p.flags = EPI_PARTIAL; p.ysplit = 1 << 30;
  p.groups = 1; p.cblocks = gy;
  // 128 pixels per workgroup at large batches: each workgroup re-reads its
  // weight slice once per pixel block (64-pixel blocks read 84 MB of weights
  // for a 21 MB matrix at B = 256); the K partition, and so every utterance's
  // bits, do not depend on it
  op.cl.wco = hw.wco; op.cl.wpx = n >= 128 ? 2 : 1; op.cl.vec = 1; op.cl.splitk = S;
  op.flops = 2.0 * n * D * hw.cout;
  op.bytes = 4.0 * ((double)n * D + (double)D * hw.cout);
  op.cp.fast4 = 0;
  // dtype of the head is always fp32: mark with type 5 (fp32 conv)
  op.type = 5;
  B.ops->push_back(op);
  Op r;
  r.kind = OP_HEAD;
  r.type = 1;
  r.part = part; r.S = S; r.M = n; r.coutp = hw.coutp; r.cout = hw.cout;
  r.flags = EPI_BN2D;
  r.mean = (const float*)hw.mean->p; r.inv = (const float*)hw.inv->p;
  r.out = out; r.ldo = hw.cout;
  r.bytes = 4.0 * ((double)S * n * hw.cout + (double)n * hw.cout);
  B.ops->push_back(r);
}

// H / rowlen: the batch's rows (ragged batches zero each utterance's padded rows)
static const void* emit_input(Builder& B, const float* x, int64_t count, int H = 1, int rowlen = 1) {
  vox_model* m = B.m;
  if (m->dt == F32) return x;
  void* in = B.base(S_IN, (size_t)count * 2);
  Op op;
  op.kind = OP_OTHER;
  op.type = 4;
  op.src = x; op.dst = in; op.count = count;
  op.vlen = B.vlen; op.H = H; op.W = rowlen;
  op.bytes = 6.0 * count;
  B.ops->push_back(op);
  return in;
}

// 1-channel 3x3 stem + BN + ReLU straight from the fp32 features (no cast op)
static void emit_stem(Builder& B, const ConvW& stem, const float* x, int n, int H, int W, void* y) {
  if (stem.wstem && !B.m->no_stem) {
    Op op;
    op.kind = OP_CONV;
    op.type = 11;
    op.src = x; op.dst = y; op.N = n; op.H = H; op.W = W; op.C = stem.cout;
    op.vlen = B.vlen; op.vsh = B.vsh;
    op.part = (const float*)stem.wstem->p;
    op.mean = (const float*)stem.mean->p;
    op.inv = (const float*)stem.inv->p;
    op.flops = 2.0 * n * H * W * 9.0 * stem.cout;
    op.bytes = 4.0 * n * H * W + (double)es_of(B.m) * n * H * W * stem.cout;
    B.ops->push_back(op);
    return;
  }
  Act in{emit_input(B, x, (int64_t)n * H * W, H, W), 1, n, H, W, 1};
  emit_conv(B, stem, in, nullptr, 0, 1, 1, 1, 1, 1, 1, H, W, y, stem.cout, EPI_AFFINE | EPI_RELU);
}

// Row segments per utterance for a row-streamed kernel that runs one workgroup
// per CU (LDS-bound): the count that minimises (workgroup rounds) x (segment
// rows + warm-up rows a segment recomputes), segments of >= min_rows rows.  At
// B = 256 every utterance is one segment (one round); at B = 192 the L1
// bottleneck takes 4 segments (3 rounds of 59 rows) where doubling until the
// grid covers the chip took 2 (2 rounds of 109).
static int row_segments(int n, int rows, int warm, int min_rows, int num_cu) {
  int nseg = 1;
  long best = -1;
  for (int ns = 1; ns <= 16; ++ns) {
    const int sg = (rows + ns - 1) / ns;
    if (ns > 1 && sg < min_rows) break;
    const long wgs = (long)n * ((rows + sg - 1) / sg);
    const long cost = (wgs + num_cu - 1) / num_cu * (sg + warm);
    if (best < 0 || cost < best) {
      best = cost;
      nseg = ns;
    }
  }
  return nseg;
}

static int build_tdnn(Builder& B, const float* x, int n, int t, float* out) {
  vox_model* m = B.m;
  const int F = m->feat_dim;
  const size_t es = es_of(m);
  auto kern = m->spec.getv("kernels");
  auto dil = m->spec.getv("dilations");
  Act a{emit_input(B, x, (int64_t)n * t * F, t, F), F, n, t, 1, F};
  Slot ping[2] = {S_X0, S_X1};
  for (size_t l = 0; l < m->convs.size(); ++l) {
    const ConvW& cw = m->convs[l];
    const int d = dil[l];
    const int ph = ((kern[l] - 1) * d) / 2;  // SAME, stride 1 (Appendix A.2)
    void* y = B.base(ping[l & 1], (size_t)n * t * cw.cout * es);
    emit_conv(B, cw, a, nullptr, 0, 1, 1, d, 1, ph, 0, t, 1, y, cw.cout,
              EPI_PRE_RELU | EPI_AFFINE);
    a = Act{y, cw.cout, n, t, 1, cw.cout};
    B.tap(y, n, t, 1, cw.cout, cw.cout);
  }
  float* pooled = (float*)B.base(S_POOL, (size_t)n * 2 * a.C * 4);
  emit_pool(B, a, pooled, m->head_bn1);
  emit_head(B, pooled, n, out);
  return VOX_OK;
}

static int build_res2net(Builder& B, const float* x, int n, int t, float* out) {
  vox_model* m = B.m;
  const size_t es = es_of(m);
  const int s = m->spec.geti("split");
  auto blocks = m->spec.getv("block_sizes");
  auto strides = m->spec.getv("block_strides");
  auto widths = m->spec.getv("widths");
  int H = t, W = m->feat_dim;
  size_t ci = 0;
  const ConvW& stem = m->convs[ci++];
  Slot cur_s = S_X0, nxt_s = S_X1;
  void* y = B.base(cur_s, (size_t)n * H * W * stem.cout * es);
  emit_stem(B, stem, x, n, H, W, y);  // res2net_model.py:192-203, SAME pad 1
  Act cur{y, stem.cout, n, H, W, stem.cout};
  B.tap(y, n, H, W, stem.cout, stem.cout);
  for (size_t st = 0; st < blocks.size(); ++st) {
    const int w = widths[st];
    const int sw = s * w;
    for (int b = 0; b < blocks[st]; ++b) {
      const int stride = b == 0 ? strides[st] : 1;
      const int Ho = (H + stride - 1) / stride, Wo = (W + stride - 1) / stride;
      if (stride == 1 && m->dt == BF16 && !m->no_bneck && cur.ld == cur.C) {
        // whole bottleneck in one launch (bneck.hip): identity shortcut, or the
        // 1x1 projection of block 0 (stride 1 only)
        const bool proj = b == 0;
        const size_t base = ci + (proj ? 1 : 0);
        const ConvW& c1a = m->convs[base];
        const ConvW& c1c = m->convs[base + s];
        const int C = c1c.cout;
        bool ok = (proj ? cur.C != C : cur.C == C) && bneck_lds(cur.C, C, w, s, W) > 0 &&
                  s - 1 <= 8 && c1a.wpair && c1c.wpair && c1a.cin == cur.C && c1a.cout == sw &&
                  c1c.cin == sw && c1a.mean && c1c.mean;
        for (int j = 0; ok && j < s - 1; ++j)
          ok = m->convs[base + 1 + j].wtc != nullptr &&
               m->convs[base + 1 + j].coutp >= 16 * ((w + 15) / 16);
        if (ok && proj) {
          const ConvW& pr = m->convs[ci];
          ok = pr.wpair && pr.cin == cur.C && pr.cout == C && pr.mean;
        }
        if (ok) {
          BneckParams q{};
          void* yo = B.base(nxt_s, (size_t)n * H * W * C * es);
          q.x = cur.p; q.y = yo; q.N = n; q.H = H; q.W = W;
          // one workgroup per CU (3(s-1) warm-up rows per segment)
          int nseg = row_segments(n, H, 3 * (s - 1), 16, m->num_cu);
          if (m->bneck_nseg > 0) nseg = std::min(m->bneck_nseg, H);
          q.seg = (H + nseg - 1) / nseg;
          q.nseg = (H + q.seg - 1) / q.seg;
          q.wa = c1a.wpair->p; q.ma = (const float*)c1a.mean->p; q.ia = (const float*)c1a.inv->p;
          for (int j = 0; j < s - 1; ++j) {
            const ConvW& br = m->convs[base + 1 + j];
            q.wb[j] = br.wtc->p; q.mb[j] = (const float*)br.mean->p; q.ib[j] = (const float*)br.inv->p;
          }
          q.wc = c1c.wpair->p; q.mc = (const float*)c1c.mean->p; q.ic = (const float*)c1c.inv->p;
          if (proj) {
            const ConvW& pr = m->convs[ci];
            q.wp = pr.wpair->p; q.mp = (const float*)pr.mean->p; q.ip = (const float*)pr.inv->p;
          }
          q.dbg = m->bneck_dbg;
          q.vlen = B.vlen; q.vsh = B.vsh;
          Op op;
          op.kind = OP_CONV;
          op.type = 12;
          op.bq = q;
          op.cin = cur.C; op.C = C; op.cl.wco = w; op.S = s;
          const double px = (double)n * H * W;
          op.flops = 2.0 * px * ((double)cur.C * sw + (s - 1) * 9.0 * w * w + (double)sw * C +
                                 (proj ? (double)cur.C * C : 0.0));
          op.bytes = (double)es * px * (cur.C + C + (proj ? 0 : C));
          B.ops->push_back(op);
          ci = base + s + 1;
          cur = Act{yo, C, n, H, W, C};
          B.tap(yo, n, H, W, C, C);
          std::swap(cur_s, nxt_s);
          continue;
        }
      }
      const void* shortcut = cur.p;
      int ld_sc = cur.ld;
      if (b == 0) {  // projection_shortcut: 1x1 stride s, no pad, + BN (:85-87,125-127)
        const ConvW& pr = m->convs[ci++];
        void* sc = B.base(S_SC, (size_t)n * Ho * Wo * pr.cout * es);
        emit_conv(B, pr, cur, nullptr, 0, stride, stride, 1, 1, 0, 0, Ho, Wo, sc, pr.cout,
                  EPI_AFFINE);
        shortcut = sc;
        ld_sc = pr.cout;
      }
      char* Bc = B.base(S_B, (size_t)n * Ho * Wo * sw * es);
      bool chained = false, pooled = false;
      if (stride == 2 && m->dt == BF16 && !m->no_split_s2 && !m->no_s2_fused &&
          cur.ld == cur.C && s2_fused_lds(cur.C, w, s, W) > 0) {
        // 1x1a + stride-2 branches + pool of the last split in one launch
        // (bneck.hip s2_fused): the full-resolution 1x1a output stays on chip
        const ConvW& c1a = m->convs[ci];
        bool ok = s - 1 <= 8 && c1a.wpair && c1a.mean && c1a.cin == cur.C && c1a.cout == sw;
        for (int j = 0; ok && j < s - 1; ++j)
          ok = m->convs[ci + 1 + j].wtc && m->convs[ci + 1 + j].coutp >= 16 * ((w + 15) / 16);
        if (ok) {
          ChainParams q{};
          q.x = cur.p; q.ldx = cur.ld; q.cin = cur.C;
          q.wa = c1a.wpair->p; q.ma = (const float*)c1a.mean->p; q.ia = (const float*)c1a.inv->p;
          q.b = Bc; q.ldb = sw;
          q.N = n; q.H = H; q.W = W; q.w = w; q.nst = s - 1;
          // (one workgroup per CU; one warm-up step per segment)
          int nseg = row_segments(n, Ho, 1, 8, m->num_cu);
          q.R = (Ho + nseg - 1) / nseg;
          q.nwaves = (Ho + q.R - 1) / q.R;
          for (int j = 0; j < s - 1; ++j) {
            const ConvW& br = m->convs[ci + 1 + j];
            q.wt[j] = br.wtc->p;
            q.mean[j] = (const float*)br.mean->p;
            q.inv[j] = (const float*)br.inv->p;
          }
          q.lds = s2_fused_lds(cur.C, w, s, W);
          q.dbg = m->bneck_dbg;
          q.vlen = B.vlen; q.vsh = B.vsh;
          Op op;
          op.kind = OP_CONV;
          op.type = 22;
          op.ch = q;
          op.flops = 2.0 * n * H * W * (double)cur.C * sw +
                     2.0 * n * Ho * Wo * 9.0 * w * w * (s - 1);
          op.bytes = (double)es * ((double)n * H * W * cur.C + (double)n * Ho * Wo * sw);
          B.ops->push_back(op);
          ci += s;
          chained = pooled = true;
        }
      }
      if (stride == 1 && m->dt == BF16 && !m->no_chain && !m->no_chain_rows &&
          !m->no_chain_fused && cur.ld == cur.C && chain_fused_lds(cur.C, w, s, W) > 0) {
        // 1x1a + row-streamed chain in one launch (bneck.hip chain_fused): only
        // x_s of the 1x1a output reaches HBM
        const ConvW& c1a = m->convs[ci];
        bool ok = s - 1 <= 8 && c1a.wpair && c1a.mean && c1a.cin == cur.C && c1a.cout == sw;
        for (int j = 0; ok && j < s - 1; ++j)
          ok = m->convs[ci + 1 + j].wtc && m->convs[ci + 1 + j].coutp >= 16 * ((w + 15) / 16);
        if (ok) {
          ChainParams q{};
          q.x = cur.p; q.ldx = cur.ld; q.cin = cur.C;
          q.wa = c1a.wpair->p; q.ma = (const float*)c1a.mean->p; q.ia = (const float*)c1a.inv->p;
          q.b = Bc; q.ldb = sw;
          q.N = n; q.H = H; q.W = W; q.w = w; q.nst = s - 1;
          // (one workgroup per CU; the stage lags recompute 2(s-1) rows per segment)
          int nseg = row_segments(n, H, 2 * (s - 1), 16, m->num_cu);
          q.R = (H + nseg - 1) / nseg;
          q.nwaves = (H + q.R - 1) / q.R;
          for (int j = 0; j < s - 1; ++j) {
            const ConvW& br = m->convs[ci + 1 + j];
            q.wt[j] = br.wtc->p;
            q.mean[j] = (const float*)br.mean->p;
            q.inv[j] = (const float*)br.inv->p;
          }
          q.lds = chain_fused_lds(cur.C, w, s, W);
          q.dbg = m->bneck_dbg;
          q.vlen = B.vlen; q.vsh = B.vsh;
          Op op;
          op.kind = OP_CONV;
          op.type = 24;
          op.ch = q;
          op.flops = 2.0 * n * H * W * ((double)cur.C * sw + 9.0 * w * w * (s - 1));
          op.bytes = (double)es * n * H * W * ((double)cur.C + sw);
          B.ops->push_back(op);
          ci += s;
          chained = true;
        }
      }
      const ConvW& c1a = m->convs[chained ? 0 : ci++];
      char* A = chained ? nullptr : B.base(S_A, (size_t)n * H * W * sw * es);
      if (chained) {
        // (s2_fused above)
      } else if (stride == 1) {
        // x_{s-1} passes straight through: write it into the concat buffer
        emit_conv(B, c1a, cur, nullptr, 0, 1, 1, 1, 1, 0, 0, H, W, A, sw, EPI_AFFINE | EPI_RELU,
                  nullptr, 0, Bc ? Bc + (size_t)(s - 1) * w * es : nullptr, sw, (s - 1) * w);
      } else {
        emit_conv(B, c1a, cur, nullptr, 0, 1, 1, 1, 1, 0, 0, H, W, A, sw, EPI_AFFINE | EPI_RELU);
      }
      if (!chained && stride == 1 && m->dt == BF16 && !m->no_chain && !m->no_chain_rows &&
          chain_rows_lds(w, s, W) > 0) {
        // row-streamed chain (bneck.hip): no halo recompute
        bool ok = s - 1 <= 8;
        for (int j = 0; ok && j < s - 1; ++j)
          ok = m->convs[ci + j].wtc && m->convs[ci + j].coutp >= 16 * ((w + 15) / 16);
        if (ok) {
          ChainParams q{};
          q.a = A; q.lda = sw; q.b = Bc; q.ldb = sw;
          q.N = n; q.H = H; q.W = W; q.w = w; q.nst = s - 1;
          // (one workgroup per CU; the stage lags recompute 2(s-1) rows per segment)
          int nseg = row_segments(n, H, 2 * (s - 1), 16, m->num_cu);
          q.R = (H + nseg - 1) / nseg;           // rows per segment
          q.nwaves = (H + q.R - 1) / q.R;        // segments per utterance
          double fl = 0;
          for (int j = 0; j < s - 1; ++j) {
            const ConvW& br = m->convs[ci + j];
            q.wt[j] = br.wtc->p;
            q.mean[j] = (const float*)br.mean->p;
            q.inv[j] = (const float*)br.inv->p;
            fl += 2.0 * n * H * W * 9.0 * w * w;
          }
          q.lds = chain_rows_lds(w, s, W);
          q.vlen = B.vlen; q.vsh = B.vsh;
          Op op;
          op.kind = OP_CONV;
          op.type = 13;
          op.ch = q;
          op.flops = fl;
          op.bytes = (double)es * n * H * W * w * (2.0 * (s - 1));
          B.ops->push_back(op);
          ci += s - 1;
          chained = true;
        }
      }
      if (!chained && stride == 1 && m->dt == BF16 && !m->no_chain && w % 8 == 0) {
        // fused split chain: all s-1 branches in one launch (kernels.hip split_chain)
        const ConvW& b0 = m->convs[ci];
        ChainParams q{};
        q.a = A; q.lda = sw; q.b = Bc; q.ldb = sw;
        q.N = n; q.H = H; q.W = W; q.w = w; q.nst = s - 1; q.coutp = b0.coutp;
        int au = w / 8;
        if (!(au & 1)) ++au;
        q.astr = au * 16;
        q.kcp = (9 * w + 31) / 32 * 32;
        int wu = q.kcp / 8;
        if (!(wu & 1)) ++wu;
        q.wstr = wu * 16;
        const long fixed = (long)16 * b0.wco * q.wstr + (q.kcp / 8) * 4;
        int R = 0;
        const int nthreads = 64 * 8;
        for (int r = 16; r >= 1; --r) {
          const long buf = (long)(r + 2 * q.nst) * (W + 2) * q.astr;
          // the next input x_{k+1} (r + 2*(nst-1) rows) is prefetched into 8 chunks/thread
          const long xchunks = (long)(r + 2 * (q.nst - 1)) * W * (w / 8);
          if (2 * buf + fixed <= 160 * 1024 && xchunks <= 8L * nthreads) { R = r; break; }
        }
        // register-prefetched weights: the kernel holds enough chunks for w <= 16*wco;
        // keep the widest tile counts (wco 6) out (too many registers)
        bool ok = R > 0 && s - 1 <= 8 && b0.wtc && b0.wco <= 4 && w <= 16 * b0.wco;
        for (int j = 0; ok && j < s - 1; ++j) ok = m->convs[ci + j].wtc != nullptr;
        if (ok) {
          q.R = R;
          q.nwaves = 8;
          q.buf_bytes = (R + 2 * q.nst) * (W + 2) * q.astr;
          q.lds = (int)(2L * q.buf_bytes + fixed);
          double fl = 0;
          for (int j = 0; j < s - 1; ++j) {
            const ConvW& br = m->convs[ci + j];
            q.wt[j] = br.wtc->p;
            q.mean[j] = (const float*)br.mean->p;
            q.inv[j] = (const float*)br.inv->p;
            fl += 2.0 * n * H * W * 9.0 * w * w;
          }
          Op op;
          op.kind = OP_CONV;
          op.type = 10;
          op.ch = q;
          op.cl.wco = b0.wco;
          op.cl.wpx = b0.wco <= 2 ? 4 : 2;  // wco 3 spills at 4
          op.flops = fl;
          op.bytes = (double)es * n * H * W * w * (2.0 * (s - 1));
          B.ops->push_back(op);
          ci += s - 1;
          chained = true;
        }
      }
      if (!chained && stride == 2 && m->dt == BF16 && !m->no_split_s2 && split_s2_lds(w, s, W) > 0) {
        // all stride-2 branches + the last split's avg pool in one launch (bneck.hip)
        bool ok = s - 1 <= 8;
        for (int j = 0; ok && j < s - 1; ++j)
          ok = m->convs[ci + j].wtc && m->convs[ci + j].coutp >= 16 * ((w + 15) / 16);
        if (ok) {
          ChainParams q{};
          q.a = A; q.lda = sw; q.b = Bc; q.ldb = sw;
          q.N = n; q.H = H; q.W = W; q.w = w; q.nst = s - 1;
          // (one workgroup per CU; one warm-up step per segment)
          int nseg = row_segments(n, Ho, 1, 8, m->num_cu);
          q.R = (Ho + nseg - 1) / nseg;
          q.nwaves = (Ho + q.R - 1) / q.R;
          for (int j = 0; j < s - 1; ++j) {
            const ConvW& br = m->convs[ci + j];
            q.wt[j] = br.wtc->p;
            q.mean[j] = (const float*)br.mean->p;
            q.inv[j] = (const float*)br.inv->p;
          }
          q.lds = split_s2_lds(w, s, W);
          q.vlen = B.vlen; q.vsh = B.vsh;
          Op op;
          op.kind = OP_CONV;
          op.type = 14;
          op.ch = q;
          op.flops = 2.0 * n * Ho * Wo * 9.0 * w * w * (s - 1);
          op.bytes = (double)es * ((double)n * H * W * sw + (double)n * Ho * Wo * sw);
          B.ops->push_back(op);
          ci += s - 1;
          chained = pooled = true;
        }
      }
      if (!chained && m->dt == BF16 && !m->no_conv3) {
        // wide branches (w = 96 / 192) on the pipelined 3x3 implicit GEMM
        // (conv3.hip); at stride 1 branch j's epilogue also forms the next
        // branch's input z_{j+1} = x_{j+1} + y_j in place over x_{j+1}
        std::vector<Op> ops3;
        bool ok = true;
        for (int j = 0; ok && j < s - 1; ++j) {
          const ConvW& br = m->convs[ci + j];
          const bool z = stride == 1 && j < s - 2;
          Op op;
          op.kind = OP_CONV;
          op.type = 20;
          ConvParams& p = op.cp;
          p.x = A ? A + (size_t)j * w * es : nullptr; p.ldx = sw;
          p.w = br.wtc ? br.wtc->p : nullptr; p.kp = 9 * br.cin;
          p.y = Bc ? Bc + (size_t)j * w * es : nullptr; p.ldy = sw;
          p.res = (z && A) ? A + (size_t)(j + 1) * w * es : nullptr; p.ldr = sw;
          p.y2 = (void*)p.res; p.ldy2 = sw; p.ysplit = 1 << 30;
          p.mean = br.mean ? (const float*)br.mean->p : nullptr;
          p.inv = br.inv ? (const float*)br.inv->p : nullptr;
          p.N = n; p.H = H; p.W = W; p.Cin = br.cin; p.Ho = Ho; p.Wo = Wo;
          p.Cout = br.cout; p.coutp = br.coutp;
          p.kh = br.kh; p.kw = br.kw; p.sh = p.sw = stride; p.dh = p.dw = 1; p.ph = p.pw = 1;
          p.groups = br.groups; p.flags = EPI_AFFINE | EPI_RELU;
          p.vlen = B.vlen; p.vsh = B.vsh;
          ok = br.wtc && br.mean && br.cin == w && br.cout == w && conv3_pipe_ok(p);
          // stride-1 w = 96: K-split register weights, 32x32 MFMA tiles (conv3k.hip),
          // or one 16-cout tile per wave (conv3r.hip, VOXEMB_NO_CONV3_KS)
          if (ok && !m->no_conv3_ks && conv3_ks_ok(p)) op.type = 30;
          else if (ok && !m->no_conv3_rw && conv3_rw_ok(p)) op.type = 25;
          // w = 192: one utterance band's window staged once, weights streamed (conv3u.hip)
          else if (ok && !m->no_conv3_utt && conv3_utt_ok(p)) op.type = 26;
          // stride 2, w = 96: register weights, 3-row window tiles (conv3s.hip)
          else if (ok && !m->no_conv3_s2r && conv3_s2r_ok(p)) op.type = 28;
          op.flops = 2.0 * n * Ho * Wo * 9.0 * br.cin * br.cout;
          op.bytes = (double)es * ((double)n * H * W * br.cin +
                                   (double)n * Ho * Wo * br.cout * (z ? 3.0 : 1.0));
          ops3.push_back(op);
        }
        if (ok) {
          for (const Op& op : ops3) B.ops->push_back(op);
          ci += s - 1;
          chained = true;
        }
      }
      for (int j = 0; !chained && j < s - 1; ++j) {  // res2net_pad_conv_bn_relu :53-75
        const ConvW& br = m->convs[ci++];
        Act xin{A ? A + (size_t)j * w * es : nullptr, sw, n, H, W, w};
        const void* add = (stride == 1 && j > 0 && Bc) ? Bc + (size_t)(j - 1) * w * es : nullptr;
        void* yb = Bc ? Bc + (size_t)j * w * es : nullptr;
        // stride 1: SAME (pad 1); stride 2: fixed pad 1 + VALID -> same index map
        emit_conv(B, br, xin, add, sw, stride, stride, 1, 1, 1, 1, Ho, Wo, yb, sw,
                  EPI_AFFINE | EPI_RELU);
      }
      if (stride != 1 && !pooled) {  // last split: AvgPool 3x3/2 VALID on the padded tensor (:77)
        Op op;
        op.kind = OP_OTHER;
        op.type = 3;
        op.src = A ? A + (size_t)(s - 1) * w * es : nullptr;
        op.lds = sw; op.N = n; op.H = H; op.W = W; op.C = w;
        op.dst = Bc ? Bc + (size_t)(s - 1) * w * es : nullptr;
        op.ldd = sw; op.Ho = Ho; op.Wo = Wo;
        op.vlen = B.vlen; op.vsh = B.vsh;
        op.bytes = (double)es * ((double)n * H * W * w + (double)n * Ho * Wo * w);
        B.ops->push_back(op);
      }
      const ConvW& c1c = m->convs[ci++];
      void* yo = B.base(nxt_s, (size_t)n * Ho * Wo * c1c.cout * es);
      Act bin{Bc, sw, n, Ho, Wo, sw};
      emit_conv(B, c1c, bin, nullptr, 0, 1, 1, 1, 1, 0, 0, Ho, Wo, yo, c1c.cout,
                EPI_AFFINE | EPI_RES | EPI_RELU, shortcut, ld_sc);  // :98-101
      cur = Act{yo, c1c.cout, n, Ho, Wo, c1c.cout};
      B.tap(yo, n, Ho, Wo, c1c.cout, c1c.cout);
      std::swap(cur_s, nxt_s);
      if (stride == 2) ++B.vsh;   // the next blocks read rows at the halved resolution
      H = Ho;
      W = Wo;
    }
  }
  float* pooled = (float*)B.base(S_POOL, (size_t)n * W * 2 * cur.C * 4);
  if (m->att)
    emit_att_pool(B, cur, pooled, nxt_s);
  else
    emit_pool(B, cur, pooled, m->head_bn1);
  emit_head(B, pooled, n, out);
  return VOX_OK;
}

static int tf_same_beg(int n, int k, int s) {
  const int out = (n + s - 1) / s;
  const int total = std::max((out - 1) * s + k - n, 0);
  return total / 2;
}

static int build_dpn(Builder& B, const float* x, int n, int t, float* out) {
  vox_model* m = B.m;
  const size_t es = es_of(m);
  const int bw0 = m->spec.geti("bw"), kr = m->spec.geti("k_r");
  auto ksec = m->spec.getv("k_sec");
  auto inc_sec = m->spec.getv("inc_sec");
  int H = t, W = m->feat_dim;
  size_t ci = 0, bi = 0;
  const ConvW& stem = m->convs[ci++];
  Slot stage_s[2] = {S_X0, S_X1};
  void* y = B.base(S_SC, (size_t)n * H * W * stem.cout * es);
  emit_stem(B, stem, x, n, H, W, y);  // conv_bn_relu, SAME
  Act cur{y, stem.cout, n, H, W, stem.cout};
  B.tap(y, n, H, W, stem.cout, stem.cout);
  for (size_t st = 0; st < ksec.size(); ++st) {
    const int bw = bw0 << st;
    const int r = kr * bw / bw0;
    const int inc = inc_sec[st];
    const int blocks = ksec[st];
    const int ctot = bw + 2 * inc + blocks * inc;  // final concat width of this stage
    const int stride = st == 0 ? 1 : 2;
    const int Ho = (H + stride - 1) / stride, Wo = (W + stride - 1) / stride;
    char* S = B.base(stage_s[st & 1], (size_t)n * Ho * Wo * ctot * es);
    int dense = 0;
    for (int b = 0; b < blocks; ++b) {
      const int bs = b == 0 ? stride : 1;
      Act inp = cur;  // concat of [res | dense] = channel prefix of the stage buffer
      if (b == 0) {  // projection: BN->ReLU->1x1 stride s -> [res bw | dense 2inc]
        const BNW& pb = m->bns[bi++];
        const ConvW& pc = m->convs[ci++];
        emit_conv(B, pc, inp, nullptr, 0, bs, bs, 1, 1, tf_same_beg(H, 1, bs),
                  tf_same_beg(W, 1, bs), Ho, Wo, S, ctot, 0, nullptr, 0, nullptr, 0, 1 << 30,
                  (const float*)pb.mean->p, (const float*)pb.inv->p);
        dense = 2 * inc;
      } else {
        inp = Act{S, ctot, n, Ho, Wo, bw + dense};
      }
      const int Hi = inp.H, Wi = inp.W;
      const BNW& b1 = m->bns[bi++];
      const ConvW& c1 = m->convs[ci++];
      const BNW& b2 = m->bns[bi++];
      const ConvW& c2 = m->convs[ci++];
      const BNW& b3 = m->bns[bi++];
      const ConvW& c3 = m->convs[ci++];
      // stride-1 block at <= 80 columns and r = 128 (stage 1): 1x1a + grouped 3x3
      // + 1x1c in one row-streamed launch (dpnblk.hip), bit-identical to the
      // three launches below
      // the grouped 3x3 + 1x1c part (and for b > 0 the 1x1a too) as one
      // row-streamed launch (dpnblk.hip)
      const bool rest_ok = bs == 1 && !m->no_dpn_block && m->dt == BF16 && c3.wpair && c2.wgc &&
                           r == 128 && c2.cin <= 16 && c2.cin * c2.groups == r && c3.cin == r &&
                           c3.cout == bw + inc && b2.mean && b3.mean;
      auto block_params = [&](bool from_a, const void* xin) {
        DpnBlockParams dq{};
        dq.from_a = from_a ? 1 : 0;
        dq.x = xin; dq.ldx = from_a ? r : ctot; dq.cin = from_a ? r : inp.C;
        dq.res = S; dq.ldr = ctot;
        if (!from_a) {
          dq.w1 = c1.wpair->p; dq.kp1 = c1.kp;
          dq.m1 = (const float*)b1.mean->p; dq.i1 = (const float*)b1.inv->p;
        }
        dq.wg = c2.wgc->p;
        dq.m2 = (const float*)b2.mean->p; dq.i2 = (const float*)b2.inv->p;
        dq.w3 = c3.wpair->p; dq.kp3 = c3.kp;
        dq.m3 = (const float*)b3.mean->p; dq.i3 = (const float*)b3.inv->p;
        dq.y = S; dq.y2 = S ? S + (size_t)(bw + dense) * es : nullptr; dq.ldy = ctot;
        dq.bw = bw; dq.cout = c3.cout;
        dq.N = n; dq.H = Ho; dq.W = Wo;
        dq.dbg = m->dpn_dbg;
        // one workgroup per CU (118 KB LDS): enough segments to cover the chip,
        // each >= 8 rows (the first and last rows' 3x3 windows reach into the
        // neighbours: their h1 rows are computed twice)
        int nseg = m->dpn_nseg > 0 ? m->dpn_nseg : 1;
        if (m->dpn_nseg <= 0)
          while ((long)n * nseg < m->num_cu && Ho / (2 * nseg) >= 8) nseg *= 2;
        dq.seg = (Ho + nseg - 1) / nseg;
        dq.nseg = (Ho + dq.seg - 1) / dq.seg;
        return dq;
      };
      auto push_block = [&](const DpnBlockParams& dq) {
        Op op;
        op.kind = OP_CONV;
        op.type = 31;
        op.dq = dq;
        const double px = (double)n * Ho * Wo;
        op.flops = 2.0 * px * (9.0 * r * c2.cin + (double)r * c3.cout);
        op.bytes = es * px * ((double)bw + c3.cout + (dq.from_a ? r : inp.C));
        if (!dq.from_a) op.flops += 2.0 * px * c1.cin * r;
        B.ops->push_back(op);
      };
      DpnBlockParams dq{};
      bool fused = false;
      if (b > 0 && rest_ok && c1.wpair && c1.cout == r && c1.cin == inp.C && b1.mean) {
        dq = block_params(false, S);
        fused = dpn_block_ok(dq) != 0;
        if (fused) dq.halo = B.base(S_A, dpn_block_halo_bytes(dq));
      }
      if (fused) {
        push_block(dq);
      } else {
        char* Bb = B.base(S_B, (size_t)n * Ho * Wo * r * es);
        // 1x1a + grouped 3x3 in one row-streamed launch (dpnblk.hip),
        // bit-identical to the two below: the stride-2 projection blocks of
        // stages 2-3 (1x1a at full resolution) and stage 2's stride-1 blocks
        DpnDownParams dd{};
        bool down = false;
        if ((bs == 2 || b > 0) && !m->no_dpn_block && m->dt == BF16 && c1.wpair && c1.cout == r &&
            c1.cin == inp.C && c2.wgc && c2.cin <= 16 && c2.cin * c2.groups == r && b1.mean &&
            b2.mean) {
          dd.x = inp.p; dd.ldx = inp.ld; dd.cin = inp.C;
          dd.w1 = c1.wpair->p; dd.kp1 = c1.kp;
          dd.m1 = (const float*)b1.mean->p; dd.i1 = (const float*)b1.inv->p;
          dd.wg = c2.wgc->p;
          dd.m2 = (const float*)b2.mean->p; dd.i2 = (const float*)b2.inv->p;
          dd.y = Bb; dd.ldy = r; dd.r = r;
          dd.N = n; dd.H = Hi; dd.W = Wi; dd.Ho = Ho; dd.Wo = Wo; dd.stride = bs;
          // one workgroup per CU (~130 KB LDS) per (segment, 128-channel slice)
          int nseg = m->dpn_nseg > 0 ? m->dpn_nseg : 1;
          if (m->dpn_nseg <= 0)
            while ((long)n * nseg * (r / 128) < m->num_cu && Ho / (2 * nseg) >= 8) nseg *= 2;
          dd.seg = (Ho + nseg - 1) / nseg;
          dd.nseg = (Ho + dd.seg - 1) / dd.seg;
          down = dpn_down_ok(dd) != 0;
        }
        if (down) {
          Op op;
          op.kind = OP_CONV;
          op.type = 32;
          op.ddq = dd;
          op.flops = 2.0 * n * ((double)Hi * Wi * c1.cin * r + (double)Ho * Wo * r * 9.0 * c2.cin);
          op.bytes = es * ((double)n * Hi * Wi * inp.C + (double)n * Ho * Wo * r);
          B.ops->push_back(op);
        } else {
          // 1x1a
          char* A = B.base(S_A, (size_t)n * Hi * Wi * r * es);
          emit_conv(B, c1, inp, nullptr, 0, 1, 1, 1, 1, 0, 0, Hi, Wi, A, r, 0, nullptr, 0, nullptr, 0,
                    1 << 30, (const float*)b1.mean->p, (const float*)b1.inv->p);
          DpnBlockParams da = rest_ok ? block_params(true, A) : DpnBlockParams{};
          if (rest_ok && dpn_block_ok(da)) {
            push_block(da);
            dense += inc;
            B.tap(S, n, Ho, Wo, bw + dense, ctot);
            continue;
          }
          // grouped 3x3, stride bs, TF SAME (asymmetric for stride 2)
          GconvParams g{};
          g.x = A; g.ldx = r; g.in_mean = (const float*)b2.mean->p; g.in_inv = (const float*)b2.inv->p;
          g.w = c2.wgc ? c2.wgc->p : nullptr; g.y = Bb; g.ldy = r;
          g.N = n; g.H = Hi; g.W = Wi; g.C = r; g.Ho = Ho; g.Wo = Wo; g.gw = c2.cin;
          g.sh = bs; g.ph = tf_same_beg(Hi, 3, bs); g.pw = tf_same_beg(Wi, 3, bs);
          g.rs_force = m->gconv_rs;
          if (c2.wgc && !m->no_gconv && c2.cin * c2.groups == r && gconv_ok(g)) {
            // row segments: enough workgroups to cover the chip a few times over,
            // each segment >= 4 steps (warm-up window re-read per segment)
            const int rs = gconv_rs(g);
            int nseg = 1;
            while ((long)n * (r / 64) * nseg < m->gconv_wgs && Ho / (2 * nseg) >= 4 * rs) nseg *= 2;
            g.seg = (Ho + nseg - 1) / nseg;
            g.nseg = (Ho + g.seg - 1) / g.seg;
            Op op;
            op.kind = OP_CONV;
            op.type = 19;
            op.gq = g;
            op.flops = 2.0 * n * Ho * Wo * (double)r * 9.0 * c2.cin;
            op.bytes = es * ((double)n * Hi * Wi * r + (double)n * Ho * Wo * r);
            B.ops->push_back(op);
          } else {
            emit_conv(B, c2, Act{A, r, n, Hi, Wi, r}, nullptr, 0, bs, bs, 1, 1, tf_same_beg(Hi, 3, bs),
                      tf_same_beg(Wi, 3, bs), Ho, Wo, Bb, r, 0, nullptr, 0, nullptr, 0, 1 << 30,
                      (const float*)b2.mean->p, (const float*)b2.inv->p);
          }
        }
        // 1x1c -> [res add in place | new dense channels appended]
        emit_conv(B, c3, Act{Bb, r, n, Ho, Wo, r}, nullptr, 0, 1, 1, 1, 1, 0, 0, Ho, Wo, S, ctot,
                  EPI_RES, S, ctot, S ? S + (size_t)(bw + dense) * es : nullptr, ctot, bw,
                  (const float*)b3.mean->p, (const float*)b3.inv->p);
      }
      dense += inc;
      B.tap(S, n, Ho, Wo, bw + dense, ctot);
    }
    cur = Act{S, ctot, n, Ho, Wo, bw + dense};
    H = Ho;
    W = Wo;
  }
  // concat_bn_relu (dpn_model.py:24-29): applied by the pool to every element
  // it reads (the bits of the in-place BN+ReLU pass, without its 2 x 160 MB
  // round trip at B = 64); a separate pass only if the map is not packed
  const BNW& fb = m->bns[bi++];
  float* pooled = (float*)B.base(S_POOL, (size_t)n * W * 2 * cur.C * 4);
  if (cur.ld == cur.C && !m->no_pool_pro) {
    emit_pool(B, cur, pooled, m->head_bn1, &fb);
    emit_head(B, pooled, n, out);
    return VOX_OK;
  }
  {
    Op op;
    op.kind = OP_OTHER;
    op.type = 6;  // in-place BN+ReLU over [n,H,W,C] with ld
    op.dst = (void*)cur.p; op.ldd = cur.ld; op.N = n; op.H = H; op.W = W; op.C = cur.C;
    op.mean = (const float*)fb.mean->p; op.inv = (const float*)fb.inv->p;
    op.bytes = 2.0 * es * n * H * W * cur.C;
    B.ops->push_back(op);
  }
  emit_pool(B, cur, pooled, m->head_bn1);
  emit_head(B, pooled, n, out);
  return VOX_OK;
}

// destroy every cached plan (after the last launch, which may be one of them)
static void drop_cache(vox_model* m) {
  if (m->cache.empty()) return;
  if (m->done) (void)hipEventSynchronize(m->done);
  for (PlanEntry& e : m->cache)
    if (e.exec) (void)hipGraphExecDestroy(e.exec);
  m->plans_dropped += (int64_t)m->cache.size();
  m->cache.clear();
}

// move the current plan into the cache (evicting the least recently used entry)
static void stash_current(vox_model* m) {
  if (m->plan_n < 0 || m->cache_max <= 0) {
    if (m->graph_exec) {
      if (m->done) (void)hipEventSynchronize(m->done);
      (void)hipGraphExecDestroy(m->graph_exec);
      m->graph_exec = nullptr;
    }
    m->plan_n = m->plan_t = -1;
    return;
  }
  if ((int)m->cache.size() >= m->cache_max) {
    size_t lru = 0;
    for (size_t i = 1; i < m->cache.size(); ++i)
      if (m->cache[i].used < m->cache[lru].used) lru = i;
    if (m->cache[lru].exec) {
      if (m->done) (void)hipEventSynchronize(m->done);
      (void)hipGraphExecDestroy(m->cache[lru].exec);
    }
    ++m->plans_dropped;
    m->cache.erase(m->cache.begin() + (long)lru);
  }
  PlanEntry e;
  e.n = m->plan_n; e.t = m->plan_t; e.x = m->plan_x; e.out = m->plan_out; e.rag = m->plan_rag;
  e.plan.swap(m->plan);
  e.taps.swap(m->taps);
  e.exec = m->graph_exec;
  e.uses = m->plan_uses;
  e.used = ++m->clock;
  m->graph_exec = nullptr;
  m->plan_n = m->plan_t = -1;
  m->cache.push_back(std::move(e));
}

// Ops whose kernels honour per-utterance lengths (ragged batches): every
// kernel that reads a row's neighbours masks the rows past the utterance's
// (device_common.h valid_rows); the 1x1 GEMMs and the head are per pixel.
static bool ragged_ok(const Op& op, DType dt) {
  if (dt != BF16) return false;
  switch (op.type) {
    case 11: return op.C == 32;                    // stem_conv1_c32
    case 12: case 13: case 14: case 22: case 24:   // bneck / chain / stride-2 row kernels
    case 20: case 26: case 28: case 30:            // 3x3 branch kernels
    case 1: case 2: case 4:                        // split-K reduce, stats pool, input cast
      return true;
    case 3: return op.C % 8 == 0 && op.lds % 8 == 0 && op.ldd % 8 == 0;   // avgpool3s2_v8
    case 5: return op.kind == OP_HEAD;             // the fp32 head dense
    case 21:                                       // 1x1 (per pixel) or the TDNN's taps
      if (op.cp.kh > 1)                            // GS_TAPS: the tap rows masked (gemm_wide.hip)
        return op.cp.kw == 1 && op.cp.W == 1 && op.cp.wblk && !op.cp.in_mean && !op.cp.res;
      return op.cp.kw == 1 && !op.cp.in_mean;
    case 9: case 18: case 29: case 8:              // 1x1 convs (per pixel)
      return op.cp.kh == 1 && op.cp.kw == 1 && !op.cp.in_mean;
  }
  return false;
}

static int build_plan(vox_model* m, const float* x, int n, int t, float* out, bool rag = false) {
  auto run = [&](bool dry) -> int {
    Builder B{m, dry, &m->plan};
    m->plan.clear();
    m->taps.clear();
    if (rag) {
      if ((m->family != "res2net" && m->family != "tdnn") || m->att)
        return fail(VOX_EINVAL, "per-utterance lengths: res2net (without attentive pooling) and "
                                "tdnn models only");
      B.vlen = (const int*)B.base(S_LEN, (size_t)n * 4);
    }
    if (m->family == "tdnn") return build_tdnn(B, x, n, t, out);
    if (m->family == "res2net") return build_res2net(B, x, n, t, out);
    if (m->family == "dpn") return build_dpn(B, x, n, t, out);
    return fail(VOX_EINVAL, "unknown family");
  };
  // the previous plan's last launch may still be running on a caller's stream:
  // a graph exec (and the kernel arguments HIP keeps with it) and the slots
  // it reads and writes must outlive it.  The current plan moves to the cache
  // (the least recently used entry is destroyed when it is full); building the
  // new plan touches host memory only, so no wait unless something is freed
  stash_current(m);
  int rc = run(true);
  if (rc) return rc;
  // slack: kernels with a K padded to 32 (gemm1x1_ws prologue / taps) read up to
  // 62 B past the last row of their input.  Those bytes meet zero weights, but a
  // NaN/Inf bit pattern times zero is still NaN in the MFMA, so a (re)allocated
  // slot is zeroed once: afterwards every byte of it is zero or a value some
  // kernel wrote (a smaller batch's input ends inside the slot, where the read
  // past it lands on an earlier batch's finite data or on the zeros)
  bool grew = false;
  for (int s = 0; s < S_NSLOTS; ++s) {
    const size_t want = m->slot_need[s] + 4096;
    if (want <= m->slots[s].bytes) continue;
    if (!grew) {   // every cached plan points into the slots; the last launch may use them
      if (m->done) HIPCHK(hipEventSynchronize(m->done));
      drop_cache(m);
    }
    HIPCHK(m->slots[s].ensure(want));
    HIPCHK(hipMemsetAsync(m->slots[s].p, 0, m->slots[s].bytes, m->stream));
    grew = true;
  }
  if (grew) HIPCHK(hipStreamSynchronize(m->stream));
  rc = run(false);
  if (rc) return rc;
  if (rag)
    for (const Op& op : m->plan)
      if (!ragged_ok(op, m->dt)) {
        m->plan.clear();
        m->taps.clear();
        return fail(VOX_EINVAL, "per-utterance lengths: op type " + std::to_string(op.type) +
                                    " of this model's plan does not mask padded rows");
      }
  m->plan_n = n;
  m->plan_t = t;
  m->plan_rag = rag;
  m->plan_x = x;
  m->plan_out = out;
  m->plan_uses = 0;
  ++m->plans_built;
  return VOX_OK;
}

static hipError_t run_op(vox_model* m, const Op& op, hipStream_t s) {
  switch (op.type) {
    case 0: return launch_conv(m->dt, op.cp, op.cl, s);
    case 7: return launch_conv_win(op.cp, op.cl, s);
    case 8: return launch_conv1x1_rr(op.cp, op.cl, s);
    case 9: return launch_gemm1x1(op.cp, s);
    case 18: return launch_gemm_pipe(op.cp, m->num_cu, m->gemm_var, s);
    case 19: return launch_gconv(op.gq, s);
    case 20: return launch_conv3_pipe(op.cp, m->num_cu, s);
    case 21: return launch_gemm_wide(op.cp, m->num_cu, m->gemm_var, s, !m->gemm_ksub1);
    case 10: return launch_split_chain(op.ch, op.cl.wco, op.cl.wpx, s);
    case 12: return launch_bneck(op.bq, op.cin, op.C, op.cl.wco, op.S, s);
    case 13: return launch_chain_rows(op.ch, s);
    case 14: return launch_split_s2(op.ch, s);
    case 22: return launch_s2_fused(op.ch, s);
    case 24: return launch_chain_fused(op.ch, s);
    case 25: return launch_conv3_rw(op.cp, m->num_cu, s);
    case 30: return launch_conv3_ks(op.cp, m->num_cu, s);
    case 31: return launch_dpn_block(op.dq, s);
    case 32: return launch_dpn_down(op.ddq, s);
    case 26: return launch_conv3_utt(op.cp, m->num_cu, s);
    case 27: return launch_conv1x1_smallk(op.cp, s, m->smallk_v1);
    case 29: return launch_conv1x1_nw(op.cp, m->num_cu, s);
    case 28: return launch_conv3_s2r(op.cp, m->num_cu, s);
    case 15: return launch_convert_bf16(op.src, (float*)op.dst, op.count, s);
    case 16: return launch_att_bias_tanh((float*)op.dst, (const float*)op.src, op.N, op.H, op.W, op.C, s);
    case 17:
      return launch_att_pool(m->dt, op.src, op.part, op.N, op.H, op.W, op.C, 1e-5f, op.mean,
                             op.inv, op.out, s);
    case 11:
      return launch_stem(m->dt, (const float*)op.src, op.N, op.H, op.W, op.part, op.C, op.mean,
                         op.inv, op.dst, s, op.vlen);
    case 5: return launch_conv(F32, op.cp, op.cl, s);
    case 1:
      return launch_splitk_reduce(op.part, op.S, op.M, op.coutp, op.cout, op.mean, op.inv,
                                  op.flags, op.out, op.ldo, s);
    case 2:
      return launch_stats_pool(m->dt, op.src, op.N, op.H, op.W, op.C, op.mean, op.inv, op.out, s,
                               op.in_mean, op.in_inv, op.vlen, op.vsh);
    case 3:
      return launch_avgpool3s2(m->dt, op.src, op.lds, op.N, op.H, op.W, op.C, op.dst, op.ldd, op.Ho,
                               op.Wo, s, op.vlen, op.vsh);
    case 4: return launch_convert_f32(m->dt, (const float*)op.src, op.dst, op.count, s, op.vlen,
                                      op.H, op.W);
    case 6:
      return launch_bnrelu_inplace(m->dt, op.dst, op.ldd, (int64_t)op.N * op.H * op.W, op.C,
                                   op.mean, op.inv, s);
  }
  return hipErrorInvalidValue;
}

static int check_shape(vox_model* m, int n, int t, int f) {
  if (n <= 0 || t <= 0) return fail(VOX_EINVAL, "empty batch");
  if (f != m->feat_dim)
    return fail(VOX_EINVAL, "feature dim " + std::to_string(f) + " != model " +
                                std::to_string(m->feat_dim));
  return VOX_OK;
}

static int ensure_plan(vox_model* m, const float* d_x, int n, int t, float* d_out, bool rag = false) {
  if (m->plan_n == n && m->plan_t == t && m->plan_x == d_x && m->plan_out == d_out &&
      m->plan_rag == rag) {
    ++m->plan_hits;   // the current plan again (consecutive batches of one shape)
    return VOX_OK;
  }
  for (PlanEntry& e : m->cache) {
    if (e.n != n || e.t != t || e.x != d_x || e.out != d_out || e.rag != rag) continue;
    // swap the resident plan in; the current one takes its cache entry
    std::swap(e.n, m->plan_n);
    std::swap(e.t, m->plan_t);
    std::swap(e.rag, m->plan_rag);
    std::swap(e.x, m->plan_x);
    std::swap(e.out, m->plan_out);
    e.plan.swap(m->plan);
    e.taps.swap(m->taps);
    std::swap(e.exec, m->graph_exec);
    std::swap(e.uses, m->plan_uses);
    e.used = ++m->clock;
    if (e.n < 0) {   // there was no current plan
      if (e.exec) (void)hipGraphExecDestroy(e.exec);
      m->cache.erase(m->cache.begin() + (&e - m->cache.data()));
    }
    ++m->plan_hits;
    return VOX_OK;
  }
  return build_plan(m, d_x, n, t, d_out, rag);
}

// ------------------------------------------------------------------ C-ABI
extern "C" int vox_load_blob(const void* blob, size_t nbytes, int device, int precision,
                             vox_model** out) {
  if (!blob || !out) return fail(VOX_EINVAL, "null argument");
  if (precision != VOX_FP32 && precision != VOX_BF16) return fail(VOX_EINVAL, "bad precision");
  Spec spec;
  std::vector<HostTensor> ts;
  int rc = parse_blob((const uint8_t*)blob, nbytes, spec, ts);
  if (rc) return rc;
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(VOX_EINVAL, "bad device index");
  HIPCHK(hipSetDevice(device));
  std::unique_ptr<vox_model> m(new vox_model());
  m->device = device;
  {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
        ncu > 0)
      m->num_cu = ncu;
  }
  m->dt = precision == VOX_BF16 ? BF16 : F32;
  m->spec = spec;
  m->family = spec.get("family");
  m->feat_dim = spec.geti("feat_dim");
  m->expand_dim = spec.geti("expand_dim", 3);
  if (!spec.get("bn_eps_4d").empty()) m->eps4 = std::strtof(spec.get("bn_eps_4d").c_str(), nullptr);
  if (!spec.get("bn_eps_2d").empty()) m->eps2 = std::strtof(spec.get("bn_eps_2d").c_str(), nullptr);
  if (const char* e = std::getenv("VOXEMB_NO_GRAPH")) m->use_graph = std::atoi(e) == 0;
  if (const char* e = std::getenv("VOXEMB_PLAN_CACHE")) m->cache_max = std::max(0, std::atoi(e));
  if (const char* e = std::getenv("VOXEMB_GRAPH_AFTER")) m->graph_after = std::max(0, std::atoi(e));
  for (const PlanEnv& pe : kPlanEnv)
    if (const char* e = std::getenv(pe.name)) m.get()->*pe.field = std::atoi(e);
#ifndef VOX_DIAG
  // diagnostic variants skip work (wrong results) and are compiled only into
  // the VOX_DIAG build (libvoxemb_diag.so, build_native.py --diag)
  if (m->bneck_dbg || m->dpn_dbg || (m->gemm_var != 0 && m->gemm_var != 1 && m->gemm_var != -1) ||
      std::getenv("VOXEMB_CONV3_RW_DBG"))
    return fail(VOX_EINVAL, "diagnostic switches (VOXEMB_BNECK_DBG / VOXEMB_DPN_DBG / VOXEMB_GEMM_VAR / "
                            "VOXEMB_CONV3_RW_DBG) need the VOX_DIAG build (libvoxemb_diag.so)");
#endif
  if ((rc = load_weights(m.get(), ts))) return rc;
  HIPCHK(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));
  HIPCHK(hipEventCreateWithFlags(&m->done, hipEventDisableTiming));
  *out = m.release();
  return VOX_OK;
}

extern "C" int vox_load(const char* path, int device, int precision, vox_model** out) {
  if (!path) return fail(VOX_EINVAL, "null path");
  std::ifstream f(path, std::ios::binary);
  if (!f) return fail(VOX_EIO, std::string("cannot open ") + path);
  std::vector<char> raw((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  return vox_load_blob(raw.data(), raw.size(), device, precision, out);
}

extern "C" void vox_free(vox_model* m) {
  if (!m) return;
  (void)hipSetDevice(m->device);
  if (m->stream) {
    (void)hipStreamSynchronize(m->stream);
    (void)hipStreamDestroy(m->stream);
  }
  (void)hipDeviceSynchronize();   // replays launched on callers' streams
  if (m->graph_exec) (void)hipGraphExecDestroy(m->graph_exec);
  for (PlanEntry& e : m->cache)
    if (e.exec) (void)hipGraphExecDestroy(e.exec);
  if (m->done) (void)hipEventDestroy(m->done);
  delete m;
}

extern "C" int vox_plan_stats(const vox_model* m, int64_t* built, int64_t* hits, int64_t* dropped,
                              int* resident) {
  if (!m) return fail(VOX_EINVAL, "null handle");
  if (built) *built = m->plans_built;
  if (hits) *hits = m->plan_hits;
  if (dropped) *dropped = m->plans_dropped;
  if (resident) *resident = (int)m->cache.size() + (m->plan_n >= 0 ? 1 : 0);
  return VOX_OK;
}

extern "C" int vox_dim(const vox_model* m) { return m ? m->out_dim : VOX_EINVAL; }
extern "C" int vox_feat_dim(const vox_model* m) { return m ? m->feat_dim : VOX_EINVAL; }
extern "C" int vox_expand_dim(const vox_model* m) { return m ? m->expand_dim : VOX_EINVAL; }
extern "C" int vox_precision(const vox_model* m) {
  return m ? (m->dt == BF16 ? VOX_BF16 : VOX_FP32) : VOX_EINVAL;
}

// d_lens (device int32 [n], each in [1, t]) or null: a ragged batch -- utterance
// i holds d_lens[i] frames padded to t; its embedding equals the unpadded run's
static int embed_device(vox_model* m, const float* d_x, int n, int t, int f, const int* d_lens,
                        float* d_out, void* stream) {
  if (!m || !d_x || !d_out) return fail(VOX_EINVAL, "null argument");
  int rc = check_shape(m, n, t, f);
  if (rc) return rc;
  HIPCHK(hipSetDevice(m->device));
  if ((rc = ensure_plan(m, d_x, n, t, d_out, d_lens != nullptr))) return rc;
  hipStream_t s = stream ? (hipStream_t)stream : m->stream;
  if (m->use_graph && !m->graph_exec && m->plan_uses >= m->graph_after) {
    // capture on the handle's own stream (the caller's may be the legacy null
    // stream, which cannot be captured); the exec then launches on any stream
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamBeginCapture(m->stream, hipStreamCaptureModeThreadLocal);
    if (e == hipSuccess) {
      for (const Op& op : m->plan)
        if ((e = run_op(m, op, m->stream)) != hipSuccess) break;
      hipError_t e2 = hipStreamEndCapture(m->stream, &g);
      if (e == hipSuccess) e = e2;
    }
    if (e == hipSuccess) e = hipGraphInstantiate(&m->graph_exec, g, nullptr, nullptr, 0);
    if (g) (void)hipGraphDestroy(g);
    if (e != hipSuccess) {   // launch eagerly from now on (same kernels)
      (void)hipGetLastError();
      m->graph_exec = nullptr;
      m->use_graph = false;
    }
  }
  // calls on different streams share the slots: order after the previous launch
  HIPCHK(hipStreamWaitEvent(s, m->done, 0));
  // this call's frame counts into the slot the plan's kernels read (stream-ordered)
  if (d_lens) HIPCHK(hipMemcpyAsync(m->slots[S_LEN].p, d_lens, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
  if (m->use_graph && m->graph_exec) {
    HIPCHK(hipGraphLaunch(m->graph_exec, s));
  } else {
    for (const Op& op : m->plan) HIPCHK(run_op(m, op, s));
  }
  HIPCHK(hipEventRecord(m->done, s));
  ++m->plan_uses;
  return VOX_OK;
}

extern "C" int vox_embed_device(vox_model* m, const float* d_x, int n, int t, int f, float* d_out,
                                void* stream) {
  return embed_device(m, d_x, n, t, f, nullptr, d_out, stream);
}

extern "C" int vox_embed_device_lens(vox_model* m, const float* d_x, int n, int t, int f,
                                     const int* d_lens, float* d_out, void* stream) {
  if (!d_lens) return fail(VOX_EINVAL, "null lengths");
  return embed_device(m, d_x, n, t, f, d_lens, d_out, stream);
}

extern "C" int vox_embed_lens(vox_model* m, const float* x, int n, int t, int f, const int* lens,
                              float* out) {
  if (!m || !x || !lens || !out) return fail(VOX_EINVAL, "null argument");
  int rc = check_shape(m, n, t, f);
  if (rc) return rc;
  for (int i = 0; i < n; ++i)
    if (lens[i] < 1 || lens[i] > t)
      return fail(VOX_EINVAL, "length " + std::to_string(lens[i]) + " of utterance " +
                                  std::to_string(i) + " outside [1, " + std::to_string(t) + "]");
  HIPCHK(hipSetDevice(m->device));
  const size_t in_b = (size_t)n * t * f * 4, out_b = (size_t)n * m->out_dim * 4;
  HIPCHK(m->stage_in.ensure(in_b));
  HIPCHK(m->stage_out.ensure(out_b));
  HIPCHK(m->stage_len.ensure((size_t)n * 4));
  HIPCHK(hipMemcpyAsync(m->stage_in.p, x, in_b, hipMemcpyHostToDevice, m->stream));
  HIPCHK(hipMemcpyAsync(m->stage_len.p, lens, (size_t)n * 4, hipMemcpyHostToDevice, m->stream));
  rc = embed_device(m, (const float*)m->stage_in.p, n, t, f, (const int*)m->stage_len.p,
                    (float*)m->stage_out.p, m->stream);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(out, m->stage_out.p, out_b, hipMemcpyDeviceToHost, m->stream));
  HIPCHK(hipStreamSynchronize(m->stream));
  return VOX_OK;
}

extern "C" int vox_embed(vox_model* m, const float* x, int n, int t, int f, float* out) {
  if (!m || !x || !out) return fail(VOX_EINVAL, "null argument");
  int rc = check_shape(m, n, t, f);
  if (rc) return rc;
  HIPCHK(hipSetDevice(m->device));
  const size_t in_b = (size_t)n * t * f * 4, out_b = (size_t)n * m->out_dim * 4;
  HIPCHK(m->stage_in.ensure(in_b));
  HIPCHK(m->stage_out.ensure(out_b));
  HIPCHK(hipMemcpyAsync(m->stage_in.p, x, in_b, hipMemcpyHostToDevice, m->stream));
  rc = vox_embed_device(m, (const float*)m->stage_in.p, n, t, f, (float*)m->stage_out.p, m->stream);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(out, m->stage_out.p, out_b, hipMemcpyDeviceToHost, m->stream));
  HIPCHK(hipStreamSynchronize(m->stream));
  return VOX_OK;
}

extern "C" int vox_embed_utt(vox_model* m, const float* x, int t, int f, float* out) {
  if (!m || !x || !out) return fail(VOX_EINVAL, "null argument");
  const int max_frames = 1000;
  if (t < 25)  // tf_extract.py:102 -> 0 chunks -> ZeroDivisionError at :111
    return fail(VOX_ESHORT, "utterance shorter than 25 frames (reference: ZeroDivisionError)");
  const int nchunks = 1 + (t - 25) / max_frames;
  const int D = m->out_dim;
  std::vector<float> acc(D, 0.f), e(D);
  int total = 0;
  for (int i = 0; i < nchunks; ++i) {
    const int len = (i + 1) * max_frames <= t ? max_frames : t - i * max_frames;
    int rc = vox_embed(m, x + (size_t)i * max_frames * f, 1, len, f, e.data());
    if (rc) return rc;
    for (int d = 0; d < D; ++d) acc[d] += e[d] * (float)len;  // target_value * input_length
    total += len;
  }
  for (int d = 0; d < D; ++d) out[d] = acc[d] / (float)total;
  return VOX_OK;
}

extern "C" int vox_profile(vox_model* m, const float* d_x, int n, int t, int f, int reps,
                           float* op_ms, double* op_flops, double* op_bytes, int* op_kind,
                           int max_ops, void* stream) {
  if (!m || !d_x) return fail(VOX_EINVAL, "null argument");
  int rc = check_shape(m, n, t, f);
  if (rc) return rc;
  HIPCHK(hipSetDevice(m->device));
  HIPCHK(m->stage_out.ensure((size_t)n * m->out_dim * 4));
  float* d_out = (float*)m->stage_out.p;
  if ((rc = ensure_plan(m, d_x, n, t, d_out))) return rc;
  hipStream_t s = stream ? (hipStream_t)stream : m->stream;
  const int nops = (int)m->plan.size();
  std::vector<hipEvent_t> ev(nops + 1);
  for (auto& e : ev) HIPCHK(hipEventCreate(&e));
  std::vector<double> tot(nops, 0.0);
  // the slots are shared with vox_embed_device launches on other streams:
  // order after the previous one, and make the next one wait for this run
  HIPCHK(hipStreamWaitEvent(s, m->done, 0));
  for (int r = 0; r < std::max(1, reps); ++r) {
    HIPCHK(hipEventRecord(ev[0], s));
    for (int i = 0; i < nops; ++i) {
      HIPCHK(run_op(m, m->plan[i], s));
      HIPCHK(hipEventRecord(ev[i + 1], s));
    }
    HIPCHK(hipEventSynchronize(ev[nops]));
    for (int i = 0; i < nops; ++i) {
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
      tot[i] += ms;
    }
  }
  HIPCHK(hipEventRecord(m->done, s));
  for (auto& e : ev) (void)hipEventDestroy(e);
  for (int i = 0; i < nops && i < max_ops; ++i) {
    if (op_ms) op_ms[i] = (float)(tot[i] / std::max(1, reps));
    if (op_flops) op_flops[i] = m->plan[i].flops;
    if (op_bytes) op_bytes[i] = m->plan[i].bytes;
    if (op_kind) {
      // kind | kernel-variant tag (wco, wpx, vec, fp32) so callers can group
      // launches by template instantiation, as rocprof names them
      const Op& o = m->plan[i];
      int tag = o.kind;
      if (o.type == 7)
        tag |= (o.cl.wco << 4) | (o.cl.wpx << 8) | (1 << 15);
      else if (o.type == 9)
        tag |= (1 << 21);
      else if (o.type == 18)
        tag |= (1 << 27);
      else if (o.type == 10)
        tag |= (o.cl.wco << 4) | (o.cl.wpx << 8) | (1 << 22);
      else if (o.type == 11)
        tag |= (1 << 23);
      else if (o.type == 27)
        tag |= (1 << 23) | (1 << 19);
      else if (o.type == 29)
        tag |= (1 << 21) | (1 << 19);
      else if (o.type == 12)
        tag |= (1 << 24);
      else if (o.type == 13)
        tag |= (1 << 25);
      else if (o.type == 14)
        tag |= (1 << 26);
      else if (o.type == 19)
        tag |= (1 << 28);
      else if (o.type == 20)
        tag |= (1 << 29);
      else if (o.type == 21)   // bit 17: launched as gemm1x1_ws (the default, gemm_wide.hip)
        tag |= (1 << 30) | ((m->gemm_var == 0 || m->gemm_var == 1) ? (1 << 17) : 0);
      else if (o.type == 22)
        tag |= (1 << 26) | (1 << 19);
      else if (o.type == 24)
        tag |= (1 << 25) | (1 << 19);
      else if (o.type == 25)
        tag |= (1 << 29) | (1 << 18);
      else if (o.type == 26)
        tag |= (1 << 29) | (1 << 18) | (1 << 17);
      else if (o.type == 28)
        tag |= (1 << 29) | (1 << 18) | (1 << 19);
      else if (o.type == 30)
        tag |= (1 << 29) | (1 << 18) | (1 << 16);
      else if (o.type == 31)
        tag |= (1 << 28) | (1 << 19);
      else if (o.type == 32)
        tag |= (1 << 28) | (1 << 18);
      else if (o.type == 8)
        tag |= (o.cl.wco << 4) | (o.cl.wpx << 8) | (((o.cp.cinp + 31) / 32) << 16) | (1 << 20);
      else if (o.type == 0 || o.type == 5)
        tag |= (o.cl.wco << 4) | (o.cl.wpx << 8) | (o.cl.vec << 12) |
               ((o.type == 5 || m->dt == F32) ? 1 << 13 : 0) | (1 << 14);
      op_kind[i] = tag;
    }
  }
  return nops;
}

// diagnostics: dpn_block_rows clock stamps (8 waves x 256 steps x 8 u64), see dpnblk.hip
extern "C" int vox_debug_dpn_trace(void* dst, size_t bytes) {
  if (!dst) return fail(VOX_EINVAL, "null argument");
  HIPCHK(dpn_trace_read(dst, bytes));
  return VOX_OK;
}

// diagnostics: bneck_fused clock stamps (8 waves x 512 steps x 4 u64), see bneck.hip
extern "C" int vox_debug_bneck_trace(void* dst, size_t bytes) {
  if (!dst) return fail(VOX_EINVAL, "null argument");
  HIPCHK(bneck_trace_read(dst, bytes));
  return VOX_OK;
}

// diagnostics: conv3x3_ks clock stamps (12 waves x 16 tiles x 8 u64), see conv3k.hip
extern "C" int vox_debug_ks_trace(void* dst, size_t bytes) {
  if (!dst) return fail(VOX_EINVAL, "null argument");
  HIPCHK(ks_trace_read(dst, bytes));
  return VOX_OK;
}

extern "C" int vox_plan_describe(vox_model* m, const float* d_x, int n, int t, int f, char* buf,
                                 size_t cap) {
  if (!m || !d_x) return fail(VOX_EINVAL, "null argument");
  int rc = check_shape(m, n, t, f);
  if (rc) return rc;
  HIPCHK(hipSetDevice(m->device));
  HIPCHK(m->stage_out.ensure((size_t)n * m->out_dim * 4));
  if ((rc = ensure_plan(m, d_x, n, t, (float*)m->stage_out.p))) return rc;
  std::string out;
  static const char* tn[] = {"igemm", "reduce", "pool", "avgpool", "convert", "igemm32", "bnrelu",
                             "win", "rr", "gemm", "chain", "stem", "bneck", "chainrows", "splits2",
                             "cvt16", "atttanh", "attpool", "gemmpipe", "gconv", "conv3pipe",
                             "gemmwide", "s2fused", "-", "chainfused", "conv3rw", "conv3utt",
                             "smallk", "conv3s2r", "nw", "conv3ks", "dpnblock", "dpndown"};
  for (const Op& o : m->plan) {
    char line[256];
    const ConvParams& p = o.cp;
    if (o.type == 0 || o.type == 5 || o.type == 7 || o.type == 8 || o.type == 9 || o.type == 18 ||
        o.type == 20 || o.type == 21 || o.type == 25 || o.type == 26 ||
        o.type == 27 || o.type == 28 || o.type == 29 || o.type == 30)
      std::snprintf(line, sizeof(line),
                    "%s wco=%d wpx=%d s=%d N=%d H=%d W=%d Cin=%d Ho=%d Wo=%d Cout=%d k=%dx%d st=%d "
                    "g=%d flags=%d x2=%d pro=%d flops=%.4g bytes=%.4g\n",
                    tn[o.type], o.cl.wco, o.cl.wpx, o.cl.splitk, p.N, p.H, p.W, p.Cin, p.Ho, p.Wo,
                    p.Cout, p.kh, p.kw, p.sh, p.groups, p.flags, p.x2 ? 1 : 0, p.in_mean ? 1 : 0,
                    o.flops, o.bytes);
    else if (o.type == 12)
      std::snprintf(line, sizeof(line), "bneck N=%d H=%d W=%d Cin=%d C=%d w=%d split=%d seg=%d nseg=%d flops=%.4g bytes=%.4g\n",
                    o.bq.N, o.bq.H, o.bq.W, o.cin, o.C, o.cl.wco, o.S, o.bq.seg, o.bq.nseg, o.flops,
                    o.bytes);
    else if (o.type == 32)
      std::snprintf(line, sizeof(line), "dpndown N=%d H=%d W=%d Cin=%d r=%d Ho=%d Wo=%d st=%d seg=%d nseg=%d flops=%.4g bytes=%.4g\n",
                    o.ddq.N, o.ddq.H, o.ddq.W, o.ddq.cin, o.ddq.r, o.ddq.Ho, o.ddq.Wo, o.ddq.stride,
                    o.ddq.seg, o.ddq.nseg, o.flops, o.bytes);
    else if (o.type == 31)
      std::snprintf(line, sizeof(line), "dpnblock N=%d H=%d W=%d Cin=%d Cout=%d bw=%d from_a=%d seg=%d nseg=%d flops=%.4g bytes=%.4g\n",
                    o.dq.N, o.dq.H, o.dq.W, o.dq.cin, o.dq.cout, o.dq.bw, o.dq.from_a, o.dq.seg, o.dq.nseg,
                    o.flops, o.bytes);
    else if (o.type == 19)
      std::snprintf(line, sizeof(line), "gconv N=%d H=%d W=%d C=%d gw=%d Ho=%d Wo=%d st=%d rs=%d seg=%d nseg=%d flops=%.4g bytes=%.4g\n",
                    o.gq.N, o.gq.H, o.gq.W, o.gq.C, o.gq.gw, o.gq.Ho, o.gq.Wo, o.gq.sh,
                    gconv_rs(o.gq), o.gq.seg, o.gq.nseg, o.flops, o.bytes);
    else if (o.type == 22 || o.type == 24)
      std::snprintf(line, sizeof(line), "%s N=%d H=%d W=%d Cin=%d w=%d nst=%d seg=%d nseg=%d lds=%d flops=%.4g bytes=%.4g\n",
                    tn[o.type], o.ch.N, o.ch.H, o.ch.W, o.ch.cin, o.ch.w, o.ch.nst, o.ch.R,
                    o.ch.nwaves, o.ch.lds, o.flops, o.bytes);
    else if (o.type == 14)
      std::snprintf(line, sizeof(line), "splits2 N=%d H=%d W=%d w=%d nst=%d seg=%d nseg=%d lds=%d flops=%.4g bytes=%.4g\n",
                    o.ch.N, o.ch.H, o.ch.W, o.ch.w, o.ch.nst, o.ch.R, o.ch.nwaves, o.ch.lds,
                    o.flops, o.bytes);
    else if (o.type == 13)
      std::snprintf(line, sizeof(line), "chainrows N=%d H=%d W=%d w=%d nst=%d seg=%d nseg=%d lds=%d flops=%.4g bytes=%.4g\n",
                    o.ch.N, o.ch.H, o.ch.W, o.ch.w, o.ch.nst, o.ch.R, o.ch.nwaves, o.ch.lds,
                    o.flops, o.bytes);
    else if (o.type == 10)
      std::snprintf(line, sizeof(line), "chain wco=%d wpx=%d N=%d H=%d W=%d w=%d nst=%d R=%d lds=%d flops=%.4g bytes=%.4g\n",
                    o.cl.wco, o.cl.wpx, o.ch.N, o.ch.H, o.ch.W, o.ch.w, o.ch.nst, o.ch.R, o.ch.lds,
                    o.flops, o.bytes);
    else if (o.type == 2)
      std::snprintf(line, sizeof(line), "pool N=%d H=%d W=%d C=%d pro=%d bytes=%.4g\n", o.N, o.H,
                    o.W, o.C, o.in_mean ? 1 : 0, o.bytes);
    else
      std::snprintf(line, sizeof(line), "%s N=%d H=%d W=%d C=%d bytes=%.4g\n", tn[o.type], o.N,
                    o.H, o.W, o.C, o.bytes);
    if (o.type == 21 && std::strlen(line) > 0) {   // + the tile (couts x pixels) it launches with
      line[std::strlen(line) - 1] = 0;
      char t[64];
      std::snprintf(t, sizeof(t), " bn=%d bm=%d\n", gemm_wide_bn(p), gemm_wide_bm(p, m->num_cu));
      std::strncat(line, t, sizeof(line) - std::strlen(line) - 1);
    }
    out += line;
  }
  if (buf && cap > 0) {
    std::strncpy(buf, out.c_str(), cap - 1);
    buf[cap - 1] = 0;
  }
  return (int)out.size() + 1;
}

// ---- layer-by-layer parity support (tests/test_bf16_oracle.py) -------------
extern "C" int vox_debug_taps(vox_model* m, const float* d_x, int n, int t, int f, float* d_out,
                              vox_tap* taps, int max_taps, int* n_ops) {
  if (!m || !d_x || !d_out) return fail(VOX_EINVAL, "null argument");
  int rc = check_shape(m, n, t, f);
  if (rc) return rc;
  HIPCHK(hipSetDevice(m->device));
  if ((rc = ensure_plan(m, d_x, n, t, d_out))) return rc;
  const int nt = (int)m->taps.size();
  if (n_ops) *n_ops = (int)m->plan.size();
  for (int i = 0; i < nt && i < max_taps && taps; ++i) {
    const Tap& a = m->taps[i];
    taps[i].op_end = a.op_end;
    taps[i].n = a.n; taps[i].h = a.h; taps[i].w = a.w; taps[i].c = a.c; taps[i].ld = a.ld;
    taps[i].dtype = m->dt == BF16 ? VOX_BF16 : VOX_FP32;
    taps[i].data = a.p;
  }
  return nt;
}

extern "C" int vox_debug_run_ops(vox_model* m, int op_begin, int op_end, void* stream) {
  if (!m) return fail(VOX_EINVAL, "null argument");
  const int nops = (int)m->plan.size();
  if (op_begin < 0 || op_end > nops || op_begin > op_end)
    return fail(VOX_EINVAL, "op range outside the plan");
  HIPCHK(hipSetDevice(m->device));
  hipStream_t s = stream ? (hipStream_t)stream : m->stream;
  HIPCHK(hipStreamWaitEvent(s, m->done, 0));
  for (int i = op_begin; i < op_end; ++i) HIPCHK(run_op(m, m->plan[i], s));
  HIPCHK(hipEventRecord(m->done, s));
  HIPCHK(hipStreamSynchronize(s));
  return VOX_OK;
}

extern "C" int64_t vox_debug_struct_size(int which) {
  return which == 0 ? (int64_t)sizeof(BneckParams) : which == 1 ? (int64_t)sizeof(GconvParams) : -1;
}

extern "C" int vox_debug_read(void* dst, const void* d_src, size_t bytes) {
  if (!dst || !d_src) return fail(VOX_EINVAL, "null argument");
  HIPCHK(hipMemcpy(dst, d_src, bytes, hipMemcpyDeviceToHost));
  return VOX_OK;
}

extern "C" int vox_stats_pool_device(const void* d_x, int dtype, int n, int h, int w, int c,
                                     const float* d_mean, const float* d_inv, float* d_out,
                                     void* stream) {
  if (!d_x || !d_out || n <= 0 || h <= 0 || w <= 0 || c <= 0)
    return fail(VOX_EINVAL, "bad stats-pool arguments");
  if (dtype != VOX_FP32 && dtype != VOX_BF16) return fail(VOX_EINVAL, "bad dtype");
  HIPCHK(launch_stats_pool(dtype == VOX_BF16 ? BF16 : F32, d_x, n, h, w, c, d_mean, d_inv, d_out,
                           (hipStream_t)stream));
  return VOX_OK;
}

// ORACLE-SIDE CPU BASELINE (test / measurement infrastructure only) -- an
// optimised fp32 C++/OpenMP restatement of the reference TF1 forward
// (tensorflow/tf_extract.py:94-111's `sess.run` on the CPU): the stand-in for
// the TF1 CPU path SURVEY.md §8(d) times beside the GPU ("CPU baseline").
//
// Only bench.py's cpu_baseline leg and tests/ load it (oracle/ rules); the
// product path never does.  Same weight blob (VOXEMB01) and the same graph as
// oracle/models_ref.py's fp32 mode, which it must match to 1e-4
// (tests/test_cpu_baseline.py):
//   TDNN    tensorflow/models/tdnn_model.py:24-30,128-161
//   Res2Net tensorflow/models/res2net_model.py:26-136,185-243 (+ attentive
//           pooling models.py:273-303)
//   DPN     tensorflow/models/dpn_model.py:24-171
//   head    models.py:262-269,306-309
//
// Convolutions are NHWC implicit GEMMs: out[p][co] = sum_{tap,ci} x[pix(p,tap)][ci]
// * w[tap][ci][co], with the HWIO weights re-packed per (group, 16-wide cout
// block) as [K][16]; register tiles of 12 pixels x 32 couts (AVX-512, picked
// at run time when the host has it) or 6 x 16 (AVX2 + FMA, the -march=x86-64-v3
// baseline); OpenMP over (pixel block, cout block); BN / ReLU / residual /
// the next split's addend fused into the conv epilogue.  The 4-D BNs are
// applied as (x - mean) * (1 / sqrt(var + eps)) (TF's fused kernel), the 2-D
// head BNs as x * inv + (-mean * inv) (tf.nn.batch_normalization, bn2d);
// everything in float32.
// Measured in this build container (8 Sapphire Rapids cores): res2net50 80x200
// 15.7 utt/s = 350 GFLOP/s (AVX-512), 9.3 utt/s (AVX2); the numpy oracle ~6.6.
#include <immintrin.h>
#include <omp.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

namespace {

thread_local std::string g_err;
int fail(const std::string& m) {
  g_err = m;
  return -1;
}

struct Tensor {
  std::string name;
  std::vector<int> shape;
  std::vector<float> data;
};

struct Spec {
  std::map<std::string, std::string> kv;
  std::string get(const std::string& k) const {
    auto it = kv.find(k);
    return it == kv.end() ? std::string() : it->second;
  }
  int geti(const std::string& k, int d = -1) const {
    auto s = get(k);
    return s.empty() ? d : std::atoi(s.c_str());
  }
  std::vector<int> getv(const std::string& k) const {
    std::vector<int> v;
    std::stringstream ss(get(k));
    std::string it;
    while (std::getline(ss, it, ','))
      if (!it.empty()) v.push_back(std::atoi(it.c_str()));
    return v;
  }
};

// ---------------------------------------------------------------- tensors
struct Act {  // NHWC view: element (n,h,w,c) at p[((n*H+h)*W+w)*ld + c]
  float* p;
  int N, H, W, C, ld;
};

struct Conv {
  int kh = 1, kw = 1, cig = 0, cout = 0, groups = 1;  // cout = total
  int cog = 0, nb = 0, K = 0;                          // per group
  std::vector<float> pk;  // [groups][nb][K][16] packed, zero padded
};

struct BN {
  std::vector<float> mean, inv;
  std::vector<float> nmi;  // -mean * inv: the 2-D head's non-fused form (bn2d)
};

// tf.nn.batch_normalization, what TF1 runs for the 2-D head BNs
// (tf.compat.v1.layers fuses 4-D inputs only): x * inv + (-mean * inv), a Mul
// and an Add, two roundings -- the volatile keeps gcc from contracting them
// to an FMA under -march=x86-64-v3
static inline float bn2d(float x, float inv, float nmi) {
  volatile float t = x * inv;
  return t + nmi;
}

Conv make_conv(const Tensor& t, int groups) {
  Conv c;
  c.kh = t.shape[0];
  c.kw = t.shape[1];
  c.cig = t.shape[2];
  c.cout = t.shape[3];
  c.groups = groups;
  c.cog = c.cout / groups;
  c.nb = (c.cog + 15) / 16;
  c.K = c.kh * c.kw * c.cig;
  c.pk.assign((size_t)groups * c.nb * c.K * 16, 0.f);
  for (int g = 0; g < groups; ++g)
    for (int b = 0; b < c.nb; ++b)
      for (int k = 0; k < c.K; ++k)
        for (int j = 0; j < 16; ++j) {
          const int co = b * 16 + j;
          if (co >= c.cog) continue;
          // HWIO flattened: k = (ky*kw + kx)*cig + ci
          c.pk[(((size_t)g * c.nb + b) * c.K + k) * 16 + j] =
              t.data[(size_t)k * c.cout + g * c.cog + co];
        }
  return c;
}

BN make_bn(const Tensor& m, const Tensor& v, float eps) {
  BN b;
  b.mean = m.data;
  b.inv.resize(v.data.size());
  for (size_t i = 0; i < v.data.size(); ++i) b.inv[i] = 1.0f / std::sqrt(v.data[i] + eps);
  return b;
}

// Epilogue applied to each conv output element, in TF's order:
//   [ReLU] -> [BN (x - mean) * inv] -> [+ residual] -> [ReLU], then optionally
//   z = out + addend to a second buffer (the next Res2Net split's input).
struct Epi {
  bool pre_relu = false, relu = false;
  const struct BN* bn = nullptr;
  const float* res = nullptr;
  int ldr = 0;
  const float* add = nullptr;  // z = y + add[p*lda + c]
  int lda = 0;
  float* z = nullptr;
  int ldz = 0;
};

// AVX-512 tile: 12 pixels x 32 couts (two packed 16-blocks), accumulators as
// named registers (an accumulator array was kept in memory by the compiler)
#define VOX_R12(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11)
__attribute__((target("avx512f,avx512vl,avx512dq,avx512bw"))) static void conv_unit_512_12x2(
    const float* const* xr, int taps, int cig, const float* W, size_t bstride, float (*out)[32]) {
#define DECL(i) __m512 a##i##0 = _mm512_setzero_ps(), a##i##1 = _mm512_setzero_ps();
  VOX_R12(DECL)
#undef DECL
  for (int t = 0; t < taps; ++t) {
    const float* Wt = W + (size_t)t * cig * 16;
#define PTR(i) const float* x##i = xr[t * 12 + i];
    VOX_R12(PTR)
#undef PTR
    for (int ci = 0; ci < cig; ++ci) {
      const __m512 w0 = _mm512_loadu_ps(Wt + ci * 16), w1 = _mm512_loadu_ps(Wt + bstride + ci * 16);
#define FMA(i)                                        \
  {                                                   \
    const __m512 b = _mm512_set1_ps(x##i[ci]);        \
    a##i##0 = _mm512_fmadd_ps(b, w0, a##i##0);        \
    a##i##1 = _mm512_fmadd_ps(b, w1, a##i##1);        \
  }
      VOX_R12(FMA)
#undef FMA
    }
  }
#define ST(i) _mm512_storeu_ps(out[i], a##i##0); _mm512_storeu_ps(out[i] + 16, a##i##1);
  VOX_R12(ST)
#undef ST
}

__attribute__((target("avx512f,avx512vl,avx512dq,avx512bw"))) static void conv_unit_512_12x1(
    const float* const* xr, int taps, int cig, const float* W, size_t, float (*out)[32]) {
#define DECL(i) __m512 a##i##0 = _mm512_setzero_ps();
  VOX_R12(DECL)
#undef DECL
  for (int t = 0; t < taps; ++t) {
    const float* Wt = W + (size_t)t * cig * 16;
#define PTR(i) const float* x##i = xr[t * 12 + i];
    VOX_R12(PTR)
#undef PTR
    for (int ci = 0; ci < cig; ++ci) {
      const __m512 w0 = _mm512_loadu_ps(Wt + ci * 16);
#define FMA(i) a##i##0 = _mm512_fmadd_ps(_mm512_set1_ps(x##i[ci]), w0, a##i##0);
      VOX_R12(FMA)
#undef FMA
    }
  }
#define ST(i) _mm512_storeu_ps(out[i], a##i##0);
  VOX_R12(ST)
#undef ST
}

// AVX2 tile: 6 pixels x 16 couts (two 8-wide vectors), named accumulators
#define VOX_R6(X) X(0) X(1) X(2) X(3) X(4) X(5)
static void conv_unit_256_6x1(const float* const* xr, int taps, int cig, const float* W,
                              float (*out)[16]) {
#define DECL(i) __m256 a##i##0 = _mm256_setzero_ps(), a##i##1 = _mm256_setzero_ps();
  VOX_R6(DECL)
#undef DECL
  for (int t = 0; t < taps; ++t) {
    const float* Wt = W + (size_t)t * cig * 16;
#define PTR(i) const float* x##i = xr[t * 6 + i];
    VOX_R6(PTR)
#undef PTR
    for (int ci = 0; ci < cig; ++ci) {
      const __m256 w0 = _mm256_loadu_ps(Wt + ci * 16), w1 = _mm256_loadu_ps(Wt + ci * 16 + 8);
#define FMA(i)                                        \
  {                                                   \
    const __m256 b = _mm256_broadcast_ss(x##i + ci);  \
    a##i##0 = _mm256_fmadd_ps(b, w0, a##i##0);        \
    a##i##1 = _mm256_fmadd_ps(b, w1, a##i##1);        \
  }
      VOX_R6(FMA)
#undef FMA
    }
  }
#define ST(i) _mm256_storeu_ps(out[i], a##i##0); _mm256_storeu_ps(out[i] + 8, a##i##1);
  VOX_R6(ST)
#undef ST
}

// VOXCPU_NO_AVX512=1 forces the AVX2 kernel (A/B)
static const bool g_avx512 = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl") &&
                             __builtin_cpu_supports("avx512dq") && __builtin_cpu_supports("avx512bw") &&
                             !std::getenv("VOXCPU_NO_AVX512");
static double g_conv_s = 0;

// conv2d: out[n,ho,wo,co] = sum x[n, ho*s - pt + ky*d, wo*s - pl + kx*d, ci] w
// (zero outside), then the epilogue.  Optional BN-ReLU prologue on the input
// (DPN bn_relu_conv).
void conv2d(const Conv& c, const Act& x, int sh, int dh, int dw, int pt, int pl, Act y,
            const BN* pro = nullptr, const Epi& epi = Epi()) {
  const double t0 = omp_get_wtime();
  struct Acc { double t0; ~Acc() { g_conv_s += omp_get_wtime() - t0; } } acc_{t0};
  const int Ho = y.H, Wo = y.W;
  const long M = (long)x.N * Ho * Wo;
  const bool wide = g_avx512;
  const int MR = wide ? 12 : 6;        // pixels per unit
  const int NBU = wide ? 2 : 1;        // 16-cout blocks per unit
  const long nmb = (M + MR - 1) / MR;
  const int taps = c.kh * c.kw;
  // BN-ReLU prologue: materialise relu(bn(x)) once (DPN bn_relu_conv)
  std::vector<float> tmp;
  Act xin = x;
  if (pro) {
    tmp.resize((size_t)x.N * x.H * x.W * x.C);
    const long P = (long)x.N * x.H * x.W;
#pragma omp parallel for schedule(static)
    for (long p = 0; p < P; ++p)
      for (int ch = 0; ch < x.C; ++ch) {
        const float v = (x.p[p * x.ld + ch] - pro->mean[ch]) * pro->inv[ch];
        tmp[p * x.C + ch] = v > 0.f ? v : 0.f;
      }
    xin = Act{tmp.data(), x.N, x.H, x.W, x.C, x.C};
  }
  std::vector<float> zero(std::max(c.cig, 1) + 16, 0.f);
  const int nbu = (c.nb + NBU - 1) / NBU;
  const long units = nmb * c.groups * nbu;
#pragma omp parallel for schedule(static)
  for (long u = 0; u < units; ++u) {
    const long mb = u / (c.groups * nbu);
    const int gb = (int)(u - mb * c.groups * nbu);
    const int g = gb / nbu, b0 = (gb - (gb / nbu) * nbu) * NBU;
    const int nbh = std::min(NBU, c.nb - b0);   // blocks in this unit
    const float* W = c.pk.data() + (((size_t)g * c.nb + b0) * c.K) * 16;
    const size_t bstride = (size_t)c.K * 16;
    int pn[12], ph[12], pw[12];
    bool pv[12];
    for (int i = 0; i < MR; ++i) {
      const long p = mb * MR + i;
      pv[i] = p < M;
      const long q = pv[i] ? p : 0;
      pn[i] = (int)(q / ((long)Ho * Wo));
      const int r = (int)(q - (long)pn[i] * Ho * Wo);
      ph[i] = r / Wo;
      pw[i] = r - ph[i] * Wo;
    }
    const float* xr[9 * 12 * 8 > 0 ? 2048 : 1];
    std::vector<const float*> xrv;
    const float** X = xr;
    if (taps * MR > 2048) {
      xrv.resize((size_t)taps * MR);
      X = xrv.data();
    }
    for (int t = 0; t < taps; ++t) {
      const int ky = t / c.kw, kx = t - (t / c.kw) * c.kw;
      for (int i = 0; i < MR; ++i) {
        const int hi = ph[i] * sh - pt + ky * dh, wi = pw[i] * sh - pl + kx * dw;
        const bool ok = pv[i] && hi >= 0 && hi < xin.H && wi >= 0 && wi < xin.W;
        X[t * MR + i] = ok ? xin.p + (((size_t)pn[i] * xin.H + hi) * xin.W + wi) * xin.ld + g * c.cig
                           : zero.data();
      }
    }
    float o[12][32];
    if (wide) {
      if (nbh == 2)
        conv_unit_512_12x2(X, taps, c.cig, W, bstride, o);
      else
        conv_unit_512_12x1(X, taps, c.cig, W, bstride, o);
    } else {
      conv_unit_256_6x1(X, taps, c.cig, W, reinterpret_cast<float(*)[16]>(&o[0][0]));
    }
    const int rowlen = wide ? 32 : 16;
    const float* ob = &o[0][0];
    for (int i = 0; i < MR; ++i) {
      if (!pv[i]) continue;
      const long p = mb * MR + i;
      const int cb = g * c.cog + b0 * 16;
      float* dst = y.p + (size_t)p * y.ld + cb;
      const int n = std::min(nbh * 16, c.cog - b0 * 16);
      for (int j = 0; j < n; ++j) {
        float v = ob[i * rowlen + j];
        const int ch = cb + j;
        if (epi.pre_relu) v = v > 0.f ? v : 0.f;
        if (epi.bn) v = (v - epi.bn->mean[ch]) * epi.bn->inv[ch];
        if (epi.res) v = v + epi.res[(size_t)p * epi.ldr + ch];
        if (epi.relu) v = v > 0.f ? v : 0.f;
        dst[j] = v;
        if (epi.z) epi.z[(size_t)p * epi.ldz + ch] = epi.add[(size_t)p * epi.lda + ch] + v;
      }
    }
  }
}

// TF SAME padding (before) for one dim
int same_beg(int n, int k, int s, int d = 1) {
  const int keff = (k - 1) * d + 1, out = (n + s - 1) / s;
  const int tot = std::max((out - 1) * s + keff - n, 0);
  return tot / 2;
}

void bn_apply(Act y, const BN& b, bool relu, const Act* res = nullptr, bool pre_relu = false) {
  const long P = (long)y.N * y.H * y.W;
#pragma omp parallel for schedule(static)
  for (long p = 0; p < P; ++p) {
    float* r = y.p + p * y.ld;
    const float* s = res ? res->p + p * res->ld : nullptr;
    for (int c = 0; c < y.C; ++c) {
      float v = r[c];
      if (pre_relu) v = v > 0.f ? v : 0.f;
      v = (v - b.mean[c]) * b.inv[c];
      if (s) v = v + s[c];
      if (relu) v = v > 0.f ? v : 0.f;
      r[c] = v;
    }
  }
}

struct Buf {
  std::vector<float>& v;
  Act act(int N, int H, int W, int C) {
    if (v.size() < (size_t)N * H * W * C) v.resize((size_t)N * H * W * C);
    return Act{v.data(), N, H, W, C, C};
  }
};

}  // namespace

struct voxcpu_model {
  Spec spec;
  std::string family;
  int feat_dim = 0, out_dim = 0;
  float eps4 = 1.001e-5f, eps2 = 1e-5f;
  std::vector<Conv> convs;
  std::vector<BN> bns;
  // head
  BN hb1, hb2;
  std::vector<float> dense;  // [D][out]
  int pooled = 0;
  // attentive pooling [1,1,3C,A], [1,1,A,C]
  bool att = false;
  std::vector<float> k1, k2;
  int att_a = 0;
  // workspace, kept across calls (fresh allocations fault in GBs of pages per call)
  std::vector<float> ws[12];
};

namespace {

struct Cur {
  const std::vector<Tensor>& t;
  size_t i = 0;
  const Tensor* next() { return i < t.size() ? &t[i++] : nullptr; }
};

int load_weights(voxcpu_model* m, const std::vector<Tensor>& ts) {
  Cur c{ts};
  auto conv_bn = [&](int groups = 1) -> bool {
    const Tensor* k = c.next();
    const Tensor* bm = c.next();
    const Tensor* bv = c.next();
    if (!k || !bm || !bv) return false;
    m->convs.push_back(make_conv(*k, groups));
    m->bns.push_back(make_bn(*bm, *bv, m->eps4));
    return true;
  };
  if (m->family == "tdnn") {
    for (size_t l = 0; l < m->spec.getv("filters").size(); ++l)
      if (!conv_bn()) return fail("blob exhausted");
  } else if (m->family == "res2net") {
    const int s = m->spec.geti("split");
    auto blocks = m->spec.getv("block_sizes");
    if (!conv_bn()) return fail("blob exhausted");
    for (size_t st = 0; st < blocks.size(); ++st)
      for (int b = 0; b < blocks[st]; ++b) {
        if (b == 0 && !conv_bn()) return fail("blob exhausted");
        if (!conv_bn()) return fail("blob exhausted");
        const Tensor* k = c.next();
        if (!k) return fail("blob exhausted");
        const int w = k->shape[2];
        for (int j = 0; j < s - 1; ++j) {  // the split kernel's column slices
          Tensor kj;
          kj.shape = {3, 3, w, w};
          kj.data.resize((size_t)9 * w * w);
          for (int kk = 0; kk < 9 * w; ++kk)
            for (int co = 0; co < w; ++co)
              kj.data[(size_t)kk * w + co] = k->data[(size_t)kk * k->shape[3] + j * w + co];
          m->convs.push_back(make_conv(kj, 1));
          const Tensor* bm = c.next();
          const Tensor* bv = c.next();
          if (!bm || !bv) return fail("blob exhausted");
          m->bns.push_back(make_bn(*bm, *bv, m->eps4));
        }
        if (!conv_bn()) return fail("blob exhausted");
      }
    if (m->spec.get("pool") == "att") {
      const Tensor* k1 = c.next();
      const Tensor* k2 = c.next();
      if (!k1 || !k2) return fail("blob exhausted");
      m->k1 = k1->data;
      m->k2 = k2->data;
      m->att_a = k1->shape[3];
      m->att = true;
    }
  } else if (m->family == "dpn") {
    const int G = m->spec.geti("cardinality");
    if (!conv_bn()) return fail("blob exhausted");
    auto ks = m->spec.getv("k_sec");
    for (size_t st = 0; st < ks.size(); ++st)
      for (int b = 0; b < ks[st]; ++b)
        for (int j = 0; j < (b == 0 ? 4 : 3); ++j) {
          const Tensor* bm = c.next();
          const Tensor* bv = c.next();
          const Tensor* k = c.next();
          if (!bm || !bv || !k) return fail("blob exhausted");
          m->bns.push_back(make_bn(*bm, *bv, m->eps4));
          m->convs.push_back(make_conv(*k, k->shape[0] == 3 ? G : 1));
        }
    const Tensor* fm = c.next();
    const Tensor* fv = c.next();
    if (!fm || !fv) return fail("blob exhausted");
    m->bns.push_back(make_bn(*fm, *fv, m->eps4));
  } else {
    return fail("unknown family " + m->family);
  }
  const Tensor* h1m = c.next();
  const Tensor* h1v = c.next();
  const Tensor* dk = c.next();
  const Tensor* h2m = c.next();
  const Tensor* h2v = c.next();
  if (!h1m || !h1v || !dk || !h2m || !h2v) return fail("blob exhausted (head)");
  m->hb1 = make_bn(*h1m, *h1v, m->eps2);
  m->hb2 = make_bn(*h2m, *h2v, m->eps2);
  for (BN* b : {&m->hb1, &m->hb2}) {
    b->nmi.resize(b->mean.size());
    for (size_t i = 0; i < b->mean.size(); ++i) b->nmi[i] = -b->mean[i] * b->inv[i];
  }
  m->dense = dk->data;
  m->pooled = dk->shape[0];
  m->out_dim = dk->shape[1];
  if (c.i != ts.size()) return fail("blob has trailing tensors");
  return 0;
}

// stats pooling (models.py:262-269): two-pass moments over H, std =
// sqrt(var + 1e-5), NHWC flatten (w*2C + {c, C+c}) -> pooled [N][W*2C]
void stats_pool(const Act& x, float* out) {
  const int N = x.N, H = x.H, W = x.W, C = x.C;
#pragma omp parallel for collapse(2) schedule(static)
  for (int n = 0; n < N; ++n)
    for (int w = 0; w < W; ++w) {
      float* o = out + ((size_t)n * W + w) * 2 * C;
      for (int c = 0; c < C; ++c) {
        float s = 0.f;
        for (int h = 0; h < H; ++h) s += x.p[(((size_t)n * H + h) * W + w) * x.ld + c];
        const float mu = s / (float)H;
        float q = 0.f;
        for (int h = 0; h < H; ++h) {
          const float d = x.p[(((size_t)n * H + h) * W + w) * x.ld + c] - mu;
          q += d * d;
        }
        o[c] = mu;
        o[C + c] = std::sqrt(q / (float)H + 1e-5f);
      }
    }
}

// attentive statistics pooling (models.py:273-303)
void att_pool(const voxcpu_model* m, const Act& x, float* out) {
  const int N = x.N, H = x.H, W = x.W, C = x.C, A = m->att_a;
  std::vector<float> st((size_t)N * W * 2 * C);
  stats_pool(x, st.data());
#pragma omp parallel for collapse(2) schedule(dynamic)
  for (int n = 0; n < N; ++n)
    for (int w = 0; w < W; ++w) {
      const float* ms = st.data() + ((size_t)n * W + w) * 2 * C;
      std::vector<float> bias(A, 0.f), hcol(A), lg((size_t)H * C);
      for (int j = 0; j < 2 * C; ++j)
        for (int a = 0; a < A; ++a) bias[a] += ms[j] * m->k1[(size_t)(C + j) * A + a];
      for (int h = 0; h < H; ++h) {
        const float* xr = x.p + (((size_t)n * H + h) * W + w) * x.ld;
        for (int a = 0; a < A; ++a) hcol[a] = 0.f;
        for (int c = 0; c < C; ++c)
          for (int a = 0; a < A; ++a) hcol[a] += xr[c] * m->k1[(size_t)c * A + a];
        for (int a = 0; a < A; ++a) hcol[a] = std::tanh(hcol[a] + bias[a]);
        for (int c = 0; c < C; ++c) {
          float s = 0.f;
          for (int a = 0; a < A; ++a) s += hcol[a] * m->k2[(size_t)a * C + c];
          lg[(size_t)h * C + c] = s;
        }
      }
      float* o = out + ((size_t)n * W + w) * 2 * C;
      for (int c = 0; c < C; ++c) {
        float mx = -INFINITY;
        for (int h = 0; h < H; ++h) mx = std::max(mx, lg[(size_t)h * C + c]);
        float den = 0.f;
        for (int h = 0; h < H; ++h) den += std::exp(lg[(size_t)h * C + c] - mx);
        float wm = 0.f, wss = 0.f;
        for (int h = 0; h < H; ++h) {
          const float wt = std::exp(lg[(size_t)h * C + c] - mx) / den;
          const float v = x.p[(((size_t)n * H + h) * W + w) * x.ld + c];
          wm += v * wt;
          wss += v * v * wt;
        }
        o[c] = wm;
        o[C + c] = std::sqrt(wss - wm * wm + 1e-5f);
      }
    }
}

void head(const voxcpu_model* m, const float* pooled, int n, float* out) {
  const int D = m->pooled, O = m->out_dim;
#pragma omp parallel for schedule(static)
  for (int i = 0; i < n; ++i) {
    std::vector<float> z(D);
    for (int d = 0; d < D; ++d) z[d] = bn2d(pooled[(size_t)i * D + d], m->hb1.inv[d], m->hb1.nmi[d]);
    std::vector<float> acc(O, 0.f);
    for (int d = 0; d < D; ++d) {
      const float a = z[d];
      const float* wr = m->dense.data() + (size_t)d * O;
      for (int o = 0; o < O; ++o) acc[o] += a * wr[o];
    }
    for (int o = 0; o < O; ++o) out[(size_t)i * O + o] = bn2d(acc[o], m->hb2.inv[o], m->hb2.nmi[o]);
  }
}

void pool_head(const voxcpu_model* m, const Act& x, float* out) {
  std::vector<float> pooled((size_t)x.N * x.W * 2 * x.C);
  if (m->att)
    att_pool(m, x, pooled.data());
  else
    stats_pool(x, pooled.data());
  head(m, pooled.data(), x.N, out);
}

int forward_tdnn(voxcpu_model* m, const float* feats, int n, int t, float* out) {
  auto ker = m->spec.getv("kernels"), dil = m->spec.getv("dilations");
  Act x{const_cast<float*>(feats), n, t, 1, m->feat_dim, m->feat_dim};
  Buf b[2] = {{m->ws[0]}, {m->ws[1]}};
  for (size_t l = 0; l < m->convs.size(); ++l) {
    const Conv& c = m->convs[l];
    Act y = b[l & 1].act(n, t, 1, c.cout);
    Epi e;
    e.pre_relu = true;   // conv -> ReLU -> BN
    e.bn = &m->bns[l];
    conv2d(c, x, 1, dil[l], 1, same_beg(t, ker[l], 1, dil[l]), 0, y, nullptr, e);
    x = y;
  }
  pool_head(m, x, out);
  return 0;
}

int forward_res2net(voxcpu_model* m, const float* feats, int n, int t, float* out) {
  const int s = m->spec.geti("split");
  auto blocks = m->spec.getv("block_sizes"), strides = m->spec.getv("block_strides"),
       widths = m->spec.getv("widths");
  int H = t, W = m->feat_dim;
  size_t ci = 0, bi = 0;
  Buf xb[2] = {{m->ws[0]}, {m->ws[1]}}, sc{m->ws[2]}, ab{m->ws[3]}, cat{m->ws[4]},
      zb[2] = {{m->ws[5]}, {m->ws[6]}};
  Act in{const_cast<float*>(feats), n, H, W, 1, 1};
  Act x = xb[0].act(n, H, W, m->convs[0].cout);
  auto bnrelu = [&](const BN* b, bool relu) {
    Epi e;
    e.bn = b;
    e.relu = relu;
    return e;
  };
  conv2d(m->convs[ci++], in, 1, 1, 1, 1, 1, x, nullptr, bnrelu(&m->bns[bi++], true));
  int cur = 0;
  for (size_t st = 0; st < blocks.size(); ++st) {
    const int w = widths[st], sw = s * w;
    for (int b = 0; b < blocks[st]; ++b) {
      const int stride = b == 0 ? strides[st] : 1;
      const int Ho = (H + stride - 1) / stride, Wo = (W + stride - 1) / stride;
      Act shortcut = x;
      if (b == 0) {  // projection: 1x1 stride s (fixed pad 0) + BN
        const Conv& pc = m->convs[ci++];
        shortcut = sc.act(n, Ho, Wo, pc.cout);
        conv2d(pc, x, stride, 1, 1, 0, 0, shortcut, nullptr, bnrelu(&m->bns[bi++], false));
      }
      const Conv& ca = m->convs[ci++];
      Act a = ab.act(n, H, W, sw);
      conv2d(ca, x, 1, 1, 1, 0, 0, a, nullptr, bnrelu(&m->bns[bi++], true));
      Act cc = cat.act(n, Ho, Wo, sw);
      for (int j = 0; j < s - 1; ++j) {
        const Conv& cb = m->convs[ci++];
        Act xin{a.p + j * w, n, H, W, w, sw};
        Act yo{cc.p + j * w, n, Ho, Wo, w, sw};
        if (stride == 1 && j > 0) xin = Act{zb[j & 1].v.data(), n, H, W, w, w};  // z_j
        Epi e = bnrelu(&m->bns[bi++], true);
        if (stride == 1 && j + 1 < s - 1) {  // the epilogue also forms z_{j+1} = x_{j+1} + y_j
          Act z = zb[(j + 1) & 1].act(n, H, W, w);
          e.z = z.p;
          e.ldz = w;
          e.add = a.p + (j + 1) * w;
          e.lda = sw;
        }
        // stride 1: SAME (pad 1); stride 2: fixed pad (1,1) + VALID -> same index map
        conv2d(cb, xin, stride, 1, 1, 1, 1, yo, nullptr, e);
      }
      // last split: passthrough, or AvgPool 3x3/2 VALID on the zero-padded input (divisor 9)
      {
        const long P = (long)n * Ho * Wo;
#pragma omp parallel for schedule(static)
        for (long p = 0; p < P; ++p) {
          const int nn = (int)(p / ((long)Ho * Wo)), r = (int)(p - (long)nn * Ho * Wo);
          const int ho = r / Wo, wo = r - (r / Wo) * Wo;
          float* dst = cc.p + p * sw + (s - 1) * w;
          if (stride == 1) {
            std::memcpy(dst, a.p + p * sw + (s - 1) * w, sizeof(float) * w);
            continue;
          }
          for (int c = 0; c < w; ++c) {
            float acc = 0.f;
            for (int ky = 0; ky < 3; ++ky)
              for (int kx = 0; kx < 3; ++kx) {
                const int hi = 2 * ho - 1 + ky, wi = 2 * wo - 1 + kx;
                if (hi >= 0 && hi < H && wi >= 0 && wi < W)
                  acc += a.p[(((size_t)nn * H + hi) * W + wi) * sw + (s - 1) * w + c];
              }
            dst[c] = acc / 9.0f;
          }
        }
      }
      const Conv& cc1 = m->convs[ci++];
      Act y = xb[cur ^ 1].act(n, Ho, Wo, cc1.cout);
      Epi e = bnrelu(&m->bns[bi++], true);  // BN, + shortcut, ReLU
      e.res = shortcut.p;
      e.ldr = shortcut.ld;
      conv2d(cc1, cc, 1, 1, 1, 0, 0, y, nullptr, e);
      x = y;
      cur ^= 1;
      H = Ho;
      W = Wo;
    }
  }
  pool_head(m, x, out);
  return 0;
}

int forward_dpn(voxcpu_model* m, const float* feats, int n, int t, float* out) {
  const int bw0 = m->spec.geti("bw"), kr = m->spec.geti("k_r");
  auto ksec = m->spec.getv("k_sec"), inc_sec = m->spec.getv("inc_sec");
  int H = t, W = m->feat_dim;
  size_t ci = 0, bi = 0;
  Buf stem{m->ws[0]}, stage[2] = {{m->ws[1]}, {m->ws[2]}}, ab{m->ws[3]}, bb{m->ws[4]}, cb{m->ws[5]};
  Act in{const_cast<float*>(feats), n, H, W, 1, 1};
  Act x = stem.act(n, H, W, m->convs[0].cout);
  Epi se;
  se.bn = &m->bns[bi++];
  se.relu = true;
  conv2d(m->convs[ci++], in, 1, 1, 1, 1, 1, x, nullptr, se);
  for (size_t st = 0; st < ksec.size(); ++st) {
    const int bw = bw0 << st, r = kr * bw / bw0, inc = inc_sec[st], blocks = ksec[st];
    const int ctot = bw + 2 * inc + blocks * inc;
    const int stride = st == 0 ? 1 : 2;
    const int Ho = (H + stride - 1) / stride, Wo = (W + stride - 1) / stride;
    Act S = stage[st & 1].act(n, Ho, Wo, ctot);
    int dense = 0;
    for (int b = 0; b < blocks; ++b) {
      const int bs = b == 0 ? stride : 1;
      Act inp = x;
      if (b == 0) {  // BN-ReLU -> 1x1 stride s (TF SAME) -> [res bw | dense 2 inc]
        const BN& pb = m->bns[bi++];
        const Conv& pc = m->convs[ci++];
        Act dst{S.p, n, Ho, Wo, pc.cout, ctot};
        conv2d(pc, inp, bs, 1, 1, same_beg(H, 1, bs), same_beg(W, 1, bs), dst, &pb);
        dense = 2 * inc;
      } else {
        inp = Act{S.p, n, Ho, Wo, bw + dense, ctot};
      }
      const int Hi = inp.H, Wi = inp.W;
      const BN& b1 = m->bns[bi++];
      const Conv& c1 = m->convs[ci++];
      Act A = ab.act(n, Hi, Wi, r);
      conv2d(c1, inp, 1, 1, 1, 0, 0, A, &b1);
      const BN& b2 = m->bns[bi++];
      const Conv& c2 = m->convs[ci++];
      Act Bq = bb.act(n, Ho, Wo, r);
      conv2d(c2, A, bs, 1, 1, same_beg(Hi, 3, bs), same_beg(Wi, 3, bs), Bq, &b2);
      const BN& b3 = m->bns[bi++];
      const Conv& c3 = m->convs[ci++];
      Act Cq = cb.act(n, Ho, Wo, c3.cout);
      conv2d(c3, Bq, 1, 1, 1, 0, 0, Cq, &b3);
      // residual add in place + dense channels appended (dual_path_block :80-87)
      const long P = (long)n * Ho * Wo;
#pragma omp parallel for schedule(static)
      for (long p = 0; p < P; ++p) {
        float* s = S.p + p * ctot;
        const float* c = Cq.p + p * c3.cout;
        for (int k = 0; k < bw; ++k) s[k] = s[k] + c[k];
        for (int k = bw; k < c3.cout; ++k) s[dense + k] = c[k];
      }
      dense += inc;
    }
    x = Act{S.p, n, Ho, Wo, bw + dense, ctot};
    H = Ho;
    W = Wo;
  }
  bn_apply(x, m->bns[bi++], true);  // concat_bn_relu
  pool_head(m, x, out);
  return 0;
}

}  // namespace

extern "C" {

const char* voxcpu_last_error(void) { return g_err.c_str(); }

int voxcpu_load(const void* blob, size_t nbytes, voxcpu_model** out) {
  const uint8_t* raw = (const uint8_t*)blob;
  if (!blob || !out || nbytes < 16 || std::memcmp(raw, "VOXEMB01", 8) != 0)
    return fail("not a VOXEMB01 blob");
  uint64_t hlen;
  std::memcpy(&hlen, raw + 8, 8);
  if (16 + hlen > nbytes) return fail("truncated header");
  std::stringstream ss(std::string((const char*)raw + 16, hlen));
  const size_t data_start = (16 + hlen + 63) / 64 * 64;
  std::unique_ptr<voxcpu_model> m(new voxcpu_model());
  std::vector<Tensor> ts;
  std::string line;
  int ntensors = -1;
  while (std::getline(ss, line)) {
    if (line.empty()) continue;
    if (ntensors < 0) {
      const size_t eq = line.find('=');
      if (eq == std::string::npos) return fail("bad header line");
      const std::string k = line.substr(0, eq), v = line.substr(eq + 1);
      if (k == "tensors")
        ntensors = std::atoi(v.c_str());
      else
        m->spec.kv[k] = v;
      continue;
    }
    std::vector<std::string> f;
    std::stringstream ls(line);
    std::string it;
    while (std::getline(ls, it, '|')) f.push_back(it);
    if (f.size() != 5) return fail("bad tensor line");
    Tensor t;
    t.name = f[0];
    std::stringstream ds(f[2]);
    size_t numel = 1;
    while (std::getline(ds, it, ',')) {
      t.shape.push_back(std::atoi(it.c_str()));
      numel *= t.shape.back();
    }
    const size_t off = std::strtoull(f[3].c_str(), nullptr, 10), nb = std::strtoull(f[4].c_str(), nullptr, 10);
    if (nb != numel * 4 || data_start + off + nb > nbytes) return fail("tensor out of range");
    t.data.resize(numel);
    std::memcpy(t.data.data(), raw + data_start + off, nb);
    ts.push_back(std::move(t));
  }
  if ((int)ts.size() != ntensors) return fail("tensor count mismatch");
  m->family = m->spec.get("family");
  m->feat_dim = m->spec.geti("feat_dim");
  if (!m->spec.get("bn_eps_4d").empty()) m->eps4 = std::strtof(m->spec.get("bn_eps_4d").c_str(), nullptr);
  if (!m->spec.get("bn_eps_2d").empty()) m->eps2 = std::strtof(m->spec.get("bn_eps_2d").c_str(), nullptr);
  if (load_weights(m.get(), ts)) return -1;
  *out = m.release();
  return 0;
}

int voxcpu_dim(const voxcpu_model* m) { return m ? m->out_dim : -1; }

// x: [n, t, feat_dim] float32; out: [n, dim].  threads <= 0: OpenMP default.
int voxcpu_embed(voxcpu_model* m, const float* x, int n, int t, int f, float* out, int threads) {
  if (!m || !x || !out || n <= 0 || t <= 0) return fail("bad arguments");
  if (f != m->feat_dim) return fail("feature dim mismatch");
  if (threads > 0) omp_set_num_threads(threads);
  if (m->family == "tdnn") return forward_tdnn(m, x, n, t, out);
  if (m->family == "res2net") return forward_res2net(m, x, n, t, out);
  if (m->family == "dpn") return forward_dpn(m, x, n, t, out);
  return fail("unknown family");
}

int voxcpu_max_threads(void) { return omp_get_max_threads(); }
double voxcpu_conv_seconds(void) { return g_conv_s; }

void voxcpu_free(voxcpu_model* m) { delete m; }

}  // extern "C"

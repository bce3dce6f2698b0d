// Host-side Kaldi table I/O and sliding CMN -- the parts of the reference's
// read/write path that live in Kaldi binaries or kaldi_io.py:
//   * apply-cmvn-sliding --norm-vars=false --center=true --cmn-window=300
//     (tensorflow/tf_extract.py:63), restated from Kaldi's
//     SlidingWindowCmnInternal: double-precision running sums, window
//     [t-w/2, t-w/2+w) shifted to stay inside [0,T), output = x - sum/n.
//   * binary matrix reader "\0B" + FM / DM / CM (kaldi_io.py:420-454), with
//     CM decoded exactly as kaldi_io._read_compressed_mat (kaldi_io.py:471-504,
//     float32 arithmetic in the same operation order: vox_read_mat), or with
//     Kaldi C++'s CompressedMatrix arithmetic (vox_read_mat_kaldi: the values
//     `apply-cmvn-sliding` sees when it reads the `copy-feats --compress` arks
//     of prepare_data.sh:69).
//   * FV record writer (kaldi_io.write_vec_flt, kaldi_io.py:304-334).
// Compiled with -ffp-contract=off so no multiply-add is fused.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

#include "../../include/voxemb.h"

int vox_set_error(int code, const char* msg);  // api.cpp (shared thread-local message)
static int kfail(int code, const char* msg) { return vox_set_error(code, msg); }

// The recursion over t in [0, t1) (the running sums always start at t = 0, so
// every output row has the same bits as the whole-utterance pass); rows
// t >= t0 are written to out[(t - t0) * F].
// (cloned for AVX2 with a run-time pick: the loops are element-wise over F,
// nothing is reassociated or contracted, so every clone gives the same bits)
__attribute__((target_clones("avx2", "default")))
static void sliding_cmn_kernel(const float* in, int T, int F, int cmn_window, int center, int t0,
                               int t1, float* out, double* sum) {
  const int min_window = 100;  // Kaldi default (only used when center == false)
  for (int f = 0; f < F; ++f) sum[f] = 0.0;
  int last_start = -1, last_end = -1;
  for (int t = 0; t < t1; ++t) {
    int ws, we;
    if (center) {
      ws = t - cmn_window / 2;
      we = ws + cmn_window;
    } else {
      ws = t - cmn_window;
      we = t + 1;
    }
    if (ws < 0) {
      we -= ws;
      ws = 0;
    }
    if (!center && we < min_window) we = min_window;
    if (we > T) {
      ws -= (we - T);
      we = T;
      if (ws < 0) ws = 0;
    }
    if (last_start == -1) {
      for (int r = ws; r < we; ++r)
        for (int f = 0; f < F; ++f) sum[f] += (double)in[(size_t)r * F + f];
    } else {
      if (ws > last_start)
        for (int f = 0; f < F; ++f) sum[f] -= (double)in[(size_t)last_start * F + f];
      if (we > last_end)
        for (int f = 0; f < F; ++f) sum[f] += (double)in[(size_t)last_end * F + f];
    }
    const int n = we - ws;
    last_start = ws;
    last_end = we;
    const double alpha = -1.0 / n;
    if (t < t0) continue;
    for (int f = 0; f < F; ++f)
      out[(size_t)(t - t0) * F + f] = (float)((double)in[(size_t)t * F + f] + alpha * sum[f]);
  }
}

static void sliding_cmn_rows(const float* in, int T, int F, int cmn_window, int center, int t0,
                             int t1, float* out) {
  thread_local std::vector<double> sum;
  sum.resize(F);
  sliding_cmn_kernel(in, T, F, cmn_window, center, t0, t1, out, sum.data());
}

extern "C" int vox_sliding_cmn(const float* in, int T, int F, int cmn_window, int center,
                               float* out) {
  if (!in || !out || T <= 0 || F <= 0 || cmn_window <= 0) return kfail(VOX_EINVAL, "bad cmn args");
  sliding_cmn_rows(in, T, F, cmn_window, center, 0, T, out);
  return VOX_OK;
}

// ---------------------------------------------------------------- matrices
namespace {
struct Reader {
  const uint8_t* p;
  size_t n, i = 0;
  bool take(void* dst, size_t k) {
    if (k > n - i) return false;   // i <= n always; no wraparound for huge k
    if (k == 0) return true;       // dst may be null for an empty matrix
    std::memcpy(dst, p + i, k);
    i += k;
    return true;
  }
};

// Parse the header; on success sets rows/cols/kind and leaves r at the payload.
int parse_header(Reader& r, int* rows, int* cols, int* kind /*0 FM 1 DM 2 CM 3 CM2*/) {
  char b[2];
  if (!r.take(b, 2)) return kfail(VOX_EIO, "truncated matrix");
  if (b[0] != '\0' || b[1] != 'B') return kfail(VOX_EIO, "not a binary Kaldi matrix (ascii unsupported)");
  char h[3];
  if (!r.take(h, 3)) return kfail(VOX_EIO, "truncated matrix header");
  if (h[0] == 'C' && h[1] == 'M') {
    if (h[2] != ' ' && h[2] != '2') return kfail(VOX_EIO, "CM3 compressed format is not supported");
    if (h[2] == '2') {   // Kaldi WriteToken ends a token with a space: "CM2 "
      char sp;
      if (!r.take(&sp, 1) || sp != ' ') return kfail(VOX_EIO, "malformed CM2 token");
    }
    float mn, range;
    int32_t nr, nc;
    if (!r.take(&mn, 4) || !r.take(&range, 4) || !r.take(&nr, 4) || !r.take(&nc, 4))
      return kfail(VOX_EIO, "truncated CM header");
    if (nr < 0 || nc < 0) return kfail(VOX_EIO, "negative matrix dims");
    *rows = nr;
    *cols = nc;
    *kind = h[2] == '2' ? 3 : 2;
    return VOX_OK;
  }
  if (h[0] == 'F' && h[1] == 'M' && h[2] == ' ') *kind = 0;
  else if (h[0] == 'D' && h[1] == 'M' && h[2] == ' ') *kind = 1;
  else return kfail(VOX_EIO, "unknown matrix header");
  int8_t s1, s2;
  int32_t nr, nc;
  if (!r.take(&s1, 1) || !r.take(&nr, 4) || !r.take(&s2, 1) || !r.take(&nc, 4))
    return kfail(VOX_EIO, "truncated matrix dims");
  if (nr < 0 || nc < 0) return kfail(VOX_EIO, "negative matrix dims");
  *rows = nr;
  *cols = nc;
  return VOX_OK;
}

// cm_kaldi = 0: kaldi_io._read_compressed_mat's float32 order (kaldi_io.py:471-504);
// cm_kaldi = 1: Kaldi C++ CompressedMatrix (compressed-matrix.cc, what
// `apply-cmvn-sliding` decodes in the reference pipeline, tf_extract.py:63):
//   Uint16ToFloat = min + range * 1.52590218966964e-05f * v       (float, left to right)
//   CharToFloat   = p + (q - p) * v * (1/64.0 | 1/128.0 | 1/63.0)  (double constants:
//                   the float product (q - p) * v is promoted, the sum rounded once)
int parse_payload(Reader& r, int kind, int rows, int cols, float* out, int cm_kaldi = 0) {
  const size_t n = (size_t)rows * cols;
  if (kind == 0) {
    if (!r.take(out, n * 4)) return kfail(VOX_EIO, "truncated FM payload");
    return VOX_OK;
  }
  if (kind == 1) {
    std::vector<double> d(n);
    if (!r.take(d.data(), n * 8)) return kfail(VOX_EIO, "truncated DM payload");
    for (size_t i = 0; i < n; ++i) out[i] = (float)d[i];
    return VOX_OK;
  }
  // CM / CM2: re-read the global header fields that precede the payload
  float mn, range;
  std::memcpy(&mn, r.p + r.i - 16, 4);
  std::memcpy(&range, r.p + r.i - 12, 4);
  if (kind == 3) {
    // CM2 (kTwoByte, Kaldi CopyToMat): min + v * float(range * (1 / 65535.0)),
    // uint16 row-major; kaldi_io has no CM2 reader (kaldi_io.py:477 asserts "CM ")
    if (!cm_kaldi) return kfail(VOX_EIO, "CM2 is not readable by kaldi_io (use cm=\"kaldi\")");
    std::vector<uint16_t> q(n);
    if (!r.take(q.data(), n * 2)) return kfail(VOX_EIO, "truncated CM2 payload");
    const float inc = (float)((double)range * (1.0 / 65535.0));
    for (size_t i = 0; i < n; ++i) out[i] = mn + (float)q[i] * inc;
    return VOX_OK;
  }
  // column headers and bytes are decoded in place (no copy of the payload)
  const size_t nch = (size_t)cols * 8;
  if (nch > r.n - r.i) return kfail(VOX_EIO, "truncated CM column headers");
  const uint8_t* ch = r.p + r.i;
  r.i += nch;
  if (n > r.n - r.i) return kfail(VOX_EIO, "truncated CM payload");
  const uint8_t* data = r.p + r.i;
  r.i += n;
  const float c = 1.52590218966964e-05f;
  // Each column maps its 256 byte codes through 4 percentiles, so the decode
  // is a per-column table of the 256 values (each computed by the formula
  // below, so the same bits) and the payload pass is a lookup, written row by
  // row: 256 * cols formula evaluations instead of rows * cols branchy ones.
  thread_local std::vector<float> lut;
  lut.resize((size_t)cols * 256);
  for (int col = 0; col < cols; ++col) {
    float p[4];
    for (int k = 0; k < 4; ++k) {
      uint16_t hv;
      std::memcpy(&hv, ch + ((size_t)col * 4 + k) * 2, 2);
      const float u = (float)hv;
      if (cm_kaldi) {
        p[k] = mn + (range * c) * u;
      } else {
        // kaldi_io: uint16 * float32(range) * float32(1/65535) + float32(min), float32 ops
        float v = u * range;
        v = v * c;
        p[k] = v + mn;
      }
    }
    float* L = &lut[(size_t)col * 256];
    if (cm_kaldi) {
      // the three segments as branch-free loops (v <= 64, <= 192, above)
      for (int v = 0; v <= 64; ++v)
        L[v] = (float)((double)p[0] + (double)((p[1] - p[0]) * (float)v) * (1 / 64.0));
      for (int v = 65; v <= 192; ++v)
        L[v] = (float)((double)p[1] + (double)((p[2] - p[1]) * (float)(v - 64)) * (1 / 128.0));
      for (int v = 193; v < 256; ++v)
        L[v] = (float)((double)p[2] + (double)((p[3] - p[2]) * (float)(v - 192)) * (1 / 63.0));
      continue;
    }
    const float s0 = (p[1] - p[0]) / 64.0f;
    const float s1 = (p[2] - p[1]) / 128.0f;
    const float s2 = (p[3] - p[2]) / 63.0f;
    for (int v = 0; v <= 64; ++v) L[v] = p[0] + s0 * (float)v;
    for (int v = 65; v <= 192; ++v) L[v] = p[1] + s1 * (float)(v - 64);
    for (int v = 193; v < 256; ++v) L[v] = p[2] + s2 * (float)(v - 192);
  }
  // payload is column-major (rows bytes per column); out is row-major
  for (int row = 0; row < rows; ++row) {
    float* o = out + (size_t)row * cols;
    const uint8_t* d = data + row;
    for (int col = 0; col < cols; ++col) o[col] = lut[(size_t)col * 256 + d[(size_t)col * rows]];
  }
  return VOX_OK;
}

int read_file_at(const char* path, int64_t offset, std::vector<uint8_t>& buf) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return kfail(VOX_EIO, "cannot open matrix file");
  if (std::fseek(f, 0, SEEK_END) != 0) {
    std::fclose(f);
    return kfail(VOX_EIO, "seek failed");
  }
  const long size = std::ftell(f);
  if (offset < 0 || offset > size) {
    std::fclose(f);
    return kfail(VOX_EIO, "offset beyond end of file");
  }
  // read the header first to size the payload
  std::fseek(f, (long)offset, SEEK_SET);
  const size_t head = std::min<size_t>(64, (size_t)(size - offset));
  buf.resize(head);
  if (std::fread(buf.data(), 1, head, f) != head) {
    std::fclose(f);
    return kfail(VOX_EIO, "short read");
  }
  Reader r{buf.data(), buf.size()};
  int rows, cols, kind;
  int rc = parse_header(r, &rows, &cols, &kind);
  if (rc) {
    std::fclose(f);
    return rc;
  }
  size_t total = r.i;
  if (kind == 0) total += (size_t)rows * cols * 4;
  else if (kind == 1) total += (size_t)rows * cols * 8;
  else if (kind == 3) total += (size_t)rows * cols * 2;
  else total += (size_t)cols * 8 + (size_t)rows * cols;
  if ((size_t)offset + total > (size_t)size) {
    std::fclose(f);
    return kfail(VOX_EIO, "matrix extends beyond end of file");
  }
  buf.resize(total);
  std::fseek(f, (long)offset, SEEK_SET);
  const size_t got = std::fread(buf.data(), 1, total, f);
  std::fclose(f);
  if (got != total) return kfail(VOX_EIO, "short read");
  return VOX_OK;
}
}  // namespace

extern "C" int vox_parse_mat_shape(const uint8_t* buf, size_t nbytes, int* rows, int* cols) {
  if (!buf || !rows || !cols) return kfail(VOX_EINVAL, "null argument");
  Reader r{buf, nbytes};
  int kind;
  return parse_header(r, rows, cols, &kind);
}

static int parse_mat(const uint8_t* buf, size_t nbytes, float* out, int rows, int cols,
                     size_t* consumed, int cm_kaldi) {
  if (!buf || (!out && rows * cols > 0)) return kfail(VOX_EINVAL, "null argument");
  Reader r{buf, nbytes};
  int nr, nc, kind;
  int rc = parse_header(r, &nr, &nc, &kind);
  if (rc) return rc;
  if (nr != rows || nc != cols) return kfail(VOX_EINVAL, "matrix shape mismatch");
  rc = parse_payload(r, kind, nr, nc, out, cm_kaldi);
  if (rc) return rc;
  if (consumed) *consumed = r.i;
  return VOX_OK;
}

extern "C" int vox_parse_mat(const uint8_t* buf, size_t nbytes, float* out, int rows, int cols,
                             size_t* consumed) {
  return parse_mat(buf, nbytes, out, rows, cols, consumed, 0);
}

extern "C" int vox_parse_mat_kaldi(const uint8_t* buf, size_t nbytes, float* out, int rows,
                                   int cols, size_t* consumed) {
  return parse_mat(buf, nbytes, out, rows, cols, consumed, 1);
}

extern "C" int vox_mat_shape(const char* path, int64_t offset, int* rows, int* cols) {
  if (!path || !rows || !cols) return kfail(VOX_EINVAL, "null argument");
  std::vector<uint8_t> buf;
  int rc = read_file_at(path, offset, buf);
  if (rc) return rc;
  return vox_parse_mat_shape(buf.data(), buf.size(), rows, cols);
}

static int read_mat(const char* path, int64_t offset, float* out, int rows, int cols,
                    int cm_kaldi) {
  if (!path) return kfail(VOX_EINVAL, "null argument");
  std::vector<uint8_t> buf;
  int rc = read_file_at(path, offset, buf);
  if (rc) return rc;
  return parse_mat(buf.data(), buf.size(), out, rows, cols, nullptr, cm_kaldi);
}

extern "C" int vox_read_mat(const char* path, int64_t offset, float* out, int rows, int cols) {
  return read_mat(path, offset, out, rows, cols, 0);
}

extern "C" int vox_read_mat_kaldi(const char* path, int64_t offset, float* out, int rows,
                                  int cols) {
  return read_mat(path, offset, out, rows, cols, 1);
}

extern "C" int64_t vox_format_vec_flt(const char* key, const float* v, int dim, uint8_t* buf,
                                      size_t cap, int64_t* data_offset) {
  if (!key || dim < 0 || (!v && dim > 0)) return kfail(VOX_EINVAL, "bad arguments");
  const size_t klen = std::strlen(key);
  if (klen == 0 || std::strchr(key, ' ')) return kfail(VOX_EINVAL, "key must be non-empty without spaces");
  const size_t need = klen + 1 + 2 + 3 + 1 + 4 + (size_t)dim * 4;
  if (data_offset) *data_offset = (int64_t)klen + 1;
  if (!buf || cap < need) return (int64_t)need;
  uint8_t* q = buf;
  std::memcpy(q, key, klen);
  q += klen;
  *q++ = ' ';
  *q++ = '\0';
  *q++ = 'B';
  std::memcpy(q, "FV ", 3);
  q += 3;
  *q++ = 4;
  const uint32_t d = (uint32_t)dim;
  std::memcpy(q, &d, 4);
  q += 4;
  std::memcpy(q, v, (size_t)dim * 4);
  return (int64_t)need;
}

// ------------------------------------------------------ batched chunk reader
// The reader side of tf_extract.py (get_batch in its own process feeding a
// Queue(32), :85-90; features through the apply-cmvn-sliding pipe, :63),
// for a whole batch of equal-length chunks at once on `threads` workers.
namespace {
struct FirstError {
  std::atomic<int> code{0};
  std::string msg;
  std::atomic_flag taken = ATOMIC_FLAG_INIT;
  void set(int c, const char* m) {
    if (!taken.test_and_set()) {
      msg = m;
      code.store(c);
    }
  }
};

// body(i) for i < n on up to `threads` workers (the caller is one of them).
// The workers are persistent: each calling thread (an extraction lane, the
// main thread) owns a pool that grows to the largest `threads` it asked for
// and is joined when that thread exits, so the workers' thread_local decode
// buffers stay mapped across calls (a fresh thread per call re-faulted them
// every batch, which cost more than the decode itself).  Nothing escapes to
// the extern "C" callers: an exception in a body (e.g. std::bad_alloc) stops
// the loop and is returned as VOX_EIO, and a worker that cannot be started
// leaves its share to the ones that did (down to the calling thread alone).
class WorkerPool {
 public:
  ~WorkerPool() {
    {
      std::lock_guard<std::mutex> l(m_);
      stop_ = true;
    }
    go_.notify_all();
    for (auto& t : th_) t.join();
  }
  // runs job() on the caller and on min(want, size) - 1 workers; returns when all are done
  void run(int want, const std::function<void()>& job) {
    grow(want - 1);
    std::unique_lock<std::mutex> l(m_);
    job_ = &job;
    active_ = std::min<int>(want - 1, (int)th_.size());
    helpers_ = active_;
    ++gen_;
    l.unlock();
    go_.notify_all();
    job();
    l.lock();
    done_.wait(l, [&] { return active_ == 0; });
    job_ = nullptr;
  }

 private:
  void grow(int k) {
    try {
      while ((int)th_.size() < k) {
        const int idx = (int)th_.size();
        th_.emplace_back([this, idx] { loop(idx); });
      }
    } catch (...) {
      // std::system_error / bad_alloc: run with the workers already started
    }
  }
  void loop(int idx) {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> l(m_);
    for (;;) {
      go_.wait(l, [&] { return stop_ || (gen_ != seen && idx < helpers_); });
      if (stop_) return;
      seen = gen_;
      const std::function<void()>* j = job_;
      l.unlock();
      (*j)();
      l.lock();
      if (--active_ == 0) done_.notify_one();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable go_, done_;
  const std::function<void()>* job_ = nullptr;
  uint64_t gen_ = 0;
  int active_ = 0, helpers_ = 0;
  bool stop_ = false;
};

// The calling thread's pool.  A forked child (Python multiprocessing's default
// start method) inherits the object but none of its worker threads, and would
// wait for them forever: a pool made in another process is abandoned (leaked --
// its threads cannot be joined here) and a new one started.
struct PoolHolder {
  WorkerPool* p = nullptr;
  pid_t pid = 0;
  ~PoolHolder() {
    if (p && pid == getpid()) delete p;
  }
  WorkerPool& get() {
    const pid_t me = getpid();
    if (!p || pid != me) {
      p = new WorkerPool();
      pid = me;
    }
    return *p;
  }
};

template <typename F>
int parallel_for(int n, int threads, F&& body) noexcept {
  threads = std::max(1, std::min(threads, n));
  std::atomic<int> next{0};
  std::atomic<bool> threw{false};
  auto work = [&]() noexcept {
    try {
      for (int i; (i = next.fetch_add(1)) < n;) body(i);
    } catch (...) {
      threw.store(true);
      next.store(n);
    }
  };
  if (threads == 1) {
    work();
  } else {
    try {
      static thread_local PoolHolder pool;
      const std::function<void()> job = work;
      pool.get().run(threads, job);
    } catch (...) {
      work();   // no pool (allocation failed): the calling thread alone
    }
  }
  if (threw.load()) {
    try {
      return kfail(VOX_EIO, "host worker failed (out of memory?)");
    } catch (...) {
      return VOX_EIO;
    }
  }
  return VOX_OK;
}

// header only (no payload read): rows / cols of the matrix at path:offset
int read_shape_at(const char* path, int64_t offset, int* rows, int* cols, int* kind = nullptr) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return kfail(VOX_EIO, "cannot open matrix file");
  uint8_t head[64];
  size_t got = 0;
  if (offset >= 0 && std::fseek(f, (long)offset, SEEK_SET) == 0) got = std::fread(head, 1, sizeof(head), f);
  std::fclose(f);
  if (got == 0) return kfail(VOX_EIO, "offset beyond end of file");
  Reader r{head, got};
  int k;
  const int rc = parse_header(r, rows, cols, &k);
  if (kind) *kind = k;
  return rc;
}
}  // namespace

extern "C" int vox_mat_kinds(const char* const* paths, const int64_t* offsets, int n, int* kinds,
                             int threads) {
  if (n < 0 || (n > 0 && (!paths || !offsets || !kinds))) return kfail(VOX_EINVAL, "null argument");
  FirstError err;
  const int prc = parallel_for(n, threads, [&](int i) {
    if (err.code.load()) return;
    int r, c;
    const int rc = paths[i] ? read_shape_at(paths[i], offsets[i], &r, &c, &kinds[i])
                            : kfail(VOX_EINVAL, "null path");
    if (rc) err.set(rc, (std::string(paths[i] ? paths[i] : "?") + ": " + vox_last_error()).c_str());
  });
  if (err.code.load()) return kfail(err.code.load(), err.msg.c_str());
  return prc;
}

// The CM payloads (what follows each "\0B" "CM " header token) of n matrices
// into buf: payload i at buf + blob_off[i], blob_off[i+1] - blob_off[i] =
// 16 + 8 cols + rows cols bytes.  Nothing is decoded: the device does that
// (vox_cm_chunks_device).  A matrix that is not "CM " with those dimensions
// (rows > 8) is VOX_EINVAL, so the caller can fall back to the host reader.
extern "C" int vox_read_cm_payloads(const char* const* paths, const int64_t* offsets, int n,
                                    const int64_t* blob_off, int cols, uint8_t* buf, int threads) {
  if (n < 0 || cols <= 0 || (n > 0 && (!paths || !offsets || !blob_off || !buf)))
    return kfail(VOX_EINVAL, "null argument");
  FirstError err;
  const int prc = parallel_for(n, threads, [&](int i) {
    if (err.code.load()) return;
    auto bad = [&](int rc) {
      err.set(rc, (std::string(paths[i] ? paths[i] : "?") + ": " + vox_last_error()).c_str());
    };
    const int64_t size = blob_off[i + 1] - blob_off[i];
    const int64_t rows = (size - 16 - 8 * (int64_t)cols) / cols;
    if (!paths[i] || size <= 16 + 8 * (int64_t)cols || rows <= 8 || rows > (1 << 30) ||
        16 + 8 * (int64_t)cols + rows * cols != size)
      return bad(kfail(VOX_EINVAL, "bad CM payload size"));
    FILE* f = std::fopen(paths[i], "rb");
    if (!f) return bad(kfail(VOX_EIO, "cannot open matrix file"));
    uint8_t tok[5];
    uint8_t* dst = buf + blob_off[i];
    const bool ok = offsets[i] >= 0 && std::fseek(f, (long)offsets[i], SEEK_SET) == 0 &&
                    std::fread(tok, 1, 5, f) == 5 && std::fread(dst, 1, (size_t)size, f) == (size_t)size;
    std::fclose(f);
    if (!ok) return bad(kfail(VOX_EIO, "short read"));
    if (std::memcmp(tok, "\0BCM ", 5) != 0) return bad(kfail(VOX_EINVAL, "not a CM matrix"));
    int32_t hr, hc;
    std::memcpy(&hr, dst + 8, 4);
    std::memcpy(&hc, dst + 12, 4);
    if (hr != rows || hc != cols) return bad(kfail(VOX_EINVAL, "CM header dimensions differ"));
  });
  if (err.code.load()) return kfail(err.code.load(), err.msg.c_str());
  return prc;
}

extern "C" int vox_mat_shapes(const char* const* paths, const int64_t* offsets, int n, int* rows,
                              int* cols, int threads) {
  if (n < 0 || (n > 0 && (!paths || !offsets || !rows || !cols))) return kfail(VOX_EINVAL, "null argument");
  FirstError err;
  const int prc = parallel_for(n, threads, [&](int i) {
    if (err.code.load()) return;
    const int rc = paths[i] ? read_shape_at(paths[i], offsets[i], &rows[i], &cols[i])
                            : kfail(VOX_EINVAL, "null path");
    if (rc) err.set(rc, (std::string(paths[i] ? paths[i] : "?") + ": " + vox_last_error()).c_str());
  });
  if (err.code.load()) return kfail(err.code.load(), err.msg.c_str());
  return prc;
}

// chunk i (lens ? lens[i] : len rows) at out + i * stride * f; rows past a
// chunk's own length up to stride are left as they are (ragged batches).
// The chunks of one utterance in a call (a long utterance's 1000-frame
// chunks sort next to each other) are read, decoded and CMN'd once, by one
// worker: the recursion runs to the last chunk's end and every chunk is a
// slice of it (the same bits as one pass per chunk, sliding_cmn_rows).
static int read_chunks(const char* const* paths, const int64_t* offsets, const int* r0,
                       const int* T, const int* c0, const int* start, const int* lens, int n, int f,
                       int len, int stride, int cmn_window, float* out, int threads) {
  if (n < 0 || f <= 0 || stride <= 0 || (!lens && (len <= 0 || len > stride)) ||
      (n > 0 && (!paths || !offsets || !r0 || !T || !c0 || !start || !out)))
    return kfail(VOX_EINVAL, "bad arguments");
  std::vector<int> order, gbeg;
  try {
    order.resize(n);
    for (int i = 0; i < n; ++i) order[i] = i;
    auto same = [&](int a, int b) {
      return offsets[a] == offsets[b] && r0[a] == r0[b] && T[a] == T[b] && c0[a] == c0[b] &&
             (paths[a] == paths[b] || (paths[a] && paths[b] && !std::strcmp(paths[a], paths[b])));
    };
    // group equal utterances (stable: a group keeps its chunks' order)
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
      if (offsets[a] != offsets[b]) return offsets[a] < offsets[b];
      const int c = std::strcmp(paths[a] ? paths[a] : "", paths[b] ? paths[b] : "");
      if (c) return c < 0;
      if (r0[a] != r0[b]) return r0[a] < r0[b];
      if (T[a] != T[b]) return T[a] < T[b];
      return c0[a] < c0[b];
    });
    for (int k = 0; k < n; ++k)
      if (k == 0 || !same(order[k - 1], order[k])) gbeg.push_back(k);
    gbeg.push_back(n);
  } catch (...) {
    return kfail(VOX_ENOMEM, "host allocation failed");
  }
  FirstError err;
  const int ngroups = (int)gbeg.size() - 1;
  const int prc = parallel_for(ngroups, threads, [&](int gi) {
    if (err.code.load()) return;
    const int first = order[gbeg[gi]];
    auto bad = [&](int rc) {
      err.set(rc, (std::string(paths[first] ? paths[first] : "?") + ": " + vox_last_error()).c_str());
    };
    // the group's rows [lo, hi) of the (ranged) utterance
    int lo = 1 << 30, hi = 0;
    for (int k = gbeg[gi]; k < gbeg[gi + 1]; ++k) {
      const int i = order[k];
      const int clen = lens ? lens[i] : len;
      if (clen <= 0 || clen > stride) return bad(kfail(VOX_EINVAL, "chunk length outside [1, stride]"));
      if (!paths[i] || T[i] <= 0 || r0[i] < 0 || c0[i] < 0 || start[i] < 0 || start[i] + clen > T[i])
        return bad(kfail(VOX_EINVAL, "chunk outside its utterance"));
      lo = std::min(lo, start[i]);
      hi = std::max(hi, start[i] + clen);
    }
    thread_local std::vector<uint8_t> buf;
    thread_local std::vector<float> mat, utt, cm;
    int rc = read_file_at(paths[first], offsets[first], buf);
    if (rc) return bad(rc);
    Reader r{buf.data(), buf.size()};
    int rows, cols, kind;
    if ((rc = parse_header(r, &rows, &cols, &kind))) return bad(rc);
    if (r0[first] + T[first] > rows || c0[first] + f > cols)
      return bad(kfail(VOX_EINVAL, "range outside the matrix"));
    mat.resize((size_t)rows * cols);
    // Kaldi's CompressedMatrix arithmetic: what apply-cmvn-sliding decodes (tf_extract.py:63)
    if ((rc = parse_payload(r, kind, rows, cols, mat.data(), 1))) return bad(rc);
    const float* u = mat.data();
    if (r0[first] != 0 || T[first] != rows || c0[first] != 0 || f != cols) {   // the rxfile's [range]
      utt.resize((size_t)T[first] * f);
      for (int t = 0; t < T[first]; ++t)
        std::memcpy(&utt[(size_t)t * f], &mat[(size_t)(r0[first] + t) * cols + c0[first]], (size_t)f * 4);
      u = utt.data();
    }
    const float* rowsrc = u + (size_t)lo * f;   // row lo of the (CMN'd) utterance
    if (cmn_window > 0) {
      cm.resize((size_t)(hi - lo) * f);
      sliding_cmn_rows(u, T[first], f, cmn_window, 1, lo, hi, cm.data());
      rowsrc = cm.data();
    }
    for (int k = gbeg[gi]; k < gbeg[gi + 1]; ++k) {
      const int i = order[k];
      const int clen = lens ? lens[i] : len;
      std::memcpy(out + (size_t)i * stride * f, rowsrc + (size_t)(start[i] - lo) * f,
                  (size_t)clen * f * 4);
    }
  });
  if (err.code.load()) return kfail(err.code.load(), err.msg.c_str());
  return prc;
}

extern "C" int vox_read_chunks(const char* const* paths, const int64_t* offsets, const int* r0,
                               const int* T, const int* c0, const int* start, int n, int f,
                               int len, int cmn_window, float* out, int threads) {
  return read_chunks(paths, offsets, r0, T, c0, start, nullptr, n, f, len, len, cmn_window, out,
                     threads);
}

extern "C" int vox_read_chunks_ragged(const char* const* paths, const int64_t* offsets,
                                      const int* r0, const int* T, const int* c0, const int* start,
                                      const int* lens, int n, int f, int stride, int cmn_window,
                                      float* out, int threads) {
  if (n > 0 && !lens) return kfail(VOX_EINVAL, "null lengths");
  return read_chunks(paths, offsets, r0, T, c0, start, lens, n, f, 0, stride, cmn_window, out,
                     threads);
}

// Host sanitizer driver for csrc/kaldi_host.cpp (the reader
// parses untrusted ark/scp bytes, restating kaldi_io.py:437-504).  Built with
// -fsanitize=address,undefined by tests/test_host_sanitizers.py and run on the
// golden arks (tests/golden) plus deterministic mutations of them (bit flips,
// truncations, forged dimensions), the sliding CMN on edge shapes, and the FV
// record formatter with short buffers.  Any out-of-bounds access, overflow or
// UB aborts the process; the printed checksums pin the valid-input results.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <random>
#include <vector>

#include "../../include/voxemb.h"

int vox_set_error(int code, const char*) { return code; }   // api.cpp's, minus the message
extern "C" const char* vox_last_error(void) { return ""; }

static std::vector<uint8_t> slurp(const char* path) {
  std::ifstream f(path, std::ios::binary);
  return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

// walk an ark of matrices: key SP "\0B" ...; returns matrices parsed, or -1
static int walk(const std::vector<uint8_t>& b, double* checksum, int kaldi) {
  size_t pos = 0;
  int count = 0;
  while (pos < b.size()) {
    size_t sp = pos;
    while (sp < b.size() && b[sp] != ' ') ++sp;
    if (sp >= b.size()) return count ? count : -1;
    pos = sp + 1;
    int rows = 0, cols = 0;
    if (vox_parse_mat_shape(b.data() + pos, b.size() - pos, &rows, &cols) != VOX_OK) return -1;
    if ((int64_t)rows * cols > (int64_t)1 << 26) return -1;   // driver's allocation cap
    std::vector<float> m((size_t)rows * cols + 1);
    size_t used = 0;
    const int rc = kaldi ? vox_parse_mat_kaldi(b.data() + pos, b.size() - pos, m.data(), rows, cols, &used)
                         : vox_parse_mat(b.data() + pos, b.size() - pos, m.data(), rows, cols, &used);
    if (rc != VOX_OK || used == 0) return -1;
    for (size_t i = 0; i < (size_t)rows * cols; ++i)
      if (std::isfinite(m[i])) *checksum += m[i];
    pos += used;
    ++count;
  }
  return count;
}

int main(int argc, char** argv) {
  std::mt19937 rng(12345);
  for (int a = 1; a < argc; ++a) {
    const std::vector<uint8_t> b = slurp(argv[a]);
    for (int kaldi = 0; kaldi < 2; ++kaldi) {
      double cs = 0;
      const int n = walk(b, &cs, kaldi);
      std::printf("%s kaldi=%d matrices=%d checksum=%.6e\n", argv[a], kaldi, n, cs);
    }
    // mutations: every outcome is fine except a sanitizer report
    for (int it = 0; it < 4000; ++it) {
      std::vector<uint8_t> m = b;
      const int kind = it % 4;
      if (kind == 0 && !m.empty()) {                    // bit flips
        for (int k = 0; k < 4; ++k) m[rng() % m.size()] ^= (uint8_t)(1u << (rng() % 8));
      } else if (kind == 1) {                           // truncation
        m.resize(m.empty() ? 0 : rng() % m.size());
      } else if (kind == 2 && m.size() > 32) {          // forged 32-bit field
        const size_t at = rng() % (m.size() - 4);
        const int32_t v[] = {-1, 0, 1, 0x7fffffff, (int32_t)0x80000000, 65536, 3};
        std::memcpy(&m[at], &v[rng() % 7], 4);
      } else if (!m.empty()) {                          // random tail
        for (size_t k = rng() % m.size(); k < m.size(); ++k) m[k] = (uint8_t)rng();
      }
      double cs = 0;
      (void)walk(m, &cs, it & 1);
    }
  }
  // forged dimensions in every header field of the first matrix of each file
  for (int a = 1; a < argc; ++a) {
    const std::vector<uint8_t> b = slurp(argv[a]);
    size_t sp = 0;
    while (sp < b.size() && b[sp] != ' ') ++sp;
    for (size_t at = sp + 1; at + 4 <= b.size() && at < sp + 24; ++at) {
      for (int32_t v : {-1, -7, (int32_t)0x80000000, 0x7fffffff, 0x40000000, 0}) {
        std::vector<uint8_t> m = b;
        std::memcpy(&m[at], &v, 4);
        int rows = 0, cols = 0;
        const uint8_t* q = m.data() + sp + 1;
        const size_t nb = m.size() - sp - 1;
        if (vox_parse_mat_shape(q, nb, &rows, &cols) != VOX_OK) continue;
        if (rows < 0 || cols < 0) return 4;   // a negative shape must never be accepted
        if ((int64_t)rows * cols > (int64_t)1 << 26) continue;
        std::vector<float> o((size_t)rows * cols + 1);
        size_t used = 0;
        (void)vox_parse_mat(q, nb, o.data(), rows, cols, &used);
        (void)vox_parse_mat_kaldi(q, nb, o.data(), rows, cols, &used);
      }
    }
  }
  // file-path readers at every offset of each file (and one past the end)
  for (int a = 1; a < argc; ++a) {
    const std::vector<uint8_t> b = slurp(argv[a]);
    for (int64_t off = 0; off <= (int64_t)b.size() + 1; ++off) {
      int rows = 0, cols = 0;
      if (vox_mat_shape(argv[a], off, &rows, &cols) != VOX_OK) continue;
      if ((int64_t)rows * cols > (int64_t)1 << 26) continue;
      std::vector<float> m((size_t)rows * cols + 1);
      (void)vox_read_mat(argv[a], off, m.data(), rows, cols);
      (void)vox_read_mat_kaldi(argv[a], off, m.data(), rows, cols);
    }
  }
  // batched readers (vox_mat_shapes / vox_read_chunks, 3 host threads): every
  // matrix each file holds, whole and as [range] chunks, against the
  // single-matrix reader + whole-utterance CMN bit for bit; then forged ranges
  for (int a = 1; a < argc; ++a) {
    const std::vector<uint8_t> b = slurp(argv[a]);
    std::vector<int64_t> offs;
    for (int64_t off = 0; off < (int64_t)b.size(); ++off) {
      int rows = 0, cols = 0;
      if (b[off] == '\0' && vox_mat_shape(argv[a], off, &rows, &cols) == VOX_OK && rows > 0 &&
          cols > 0 && (int64_t)rows * cols <= (int64_t)1 << 22 && (off == 0 || b[off - 1] == ' '))
        offs.push_back(off);
    }
    const int n = (int)offs.size();
    if (!n) continue;
    std::vector<const char*> paths(n, argv[a]);
    std::vector<int> rows(n), cols(n);
    if (vox_mat_shapes(paths.data(), offs.data(), n, rows.data(), cols.data(), 3) != VOX_OK) return 5;
    for (int i = 0; i < n; ++i) {
      const int T = rows[i], F = cols[i];
      std::vector<float> m((size_t)T * F), c((size_t)T * F);
      if (vox_read_mat_kaldi(argv[a], offs[i], m.data(), T, F) != VOX_OK) return 5;
      if (vox_sliding_cmn(m.data(), T, F, 300, 1, c.data()) != VOX_OK) return 5;
      for (int len : {T, (T + 1) / 2, 1}) {
        const int start = T - len, r0 = 0, c0 = 0;
        std::vector<float> o((size_t)len * F);
        for (int cmn = 0; cmn < 2; ++cmn) {
          if (vox_read_chunks(&paths[i], &offs[i], &r0, &T, &c0, &start, 1, F, len, cmn ? 300 : 0,
                              o.data(), 3) != VOX_OK)
            return 5;
          const float* ref = (cmn ? c.data() : m.data()) + (size_t)start * F;
          if (std::memcmp(o.data(), ref, o.size() * 4) != 0) return 6;
        }
      }
    }
    // forged ranges / starts: rejected or in bounds, never a sanitizer report
    for (int it = 0; it < 200; ++it) {
      const int i = (int)(rng() % n);
      const int r0 = (int)(rng() % (rows[i] + 2)) - 1, T = (int)(rng() % (rows[i] + 2));
      const int c0 = (int)(rng() % 3) - 1, st = (int)(rng() % (rows[i] + 2)) - 1;
      const int len = 1 + (int)(rng() % (rows[i] + 1));
      std::vector<float> o((size_t)len * cols[i] + 1);
      (void)vox_read_chunks(&paths[i], &offs[i], &r0, &T, &c0, &st, 1, cols[i], len, 300, o.data(), 2);
    }
  }
  // sliding CMN on edge shapes (T = 1, window > T, odd windows, centre off)
  for (int T : {1, 2, 25, 151, 300, 301, 777}) {
    for (int win : {1, 3, 300, 1000}) {
      for (int center = 0; center < 2; ++center) {
        std::vector<float> in((size_t)T * 3), out((size_t)T * 3);
        for (auto& v : in) v = (float)((int)(rng() % 2001) - 1000) / 100.f;
        if (vox_sliding_cmn(in.data(), T, 3, win, center, out.data()) != VOX_OK) return 2;
      }
    }
  }
  // FV records into short and exact buffers
  const float v[5] = {1.f, -2.f, 3.5f, 0.f, 1e-30f};
  for (size_t cap = 0; cap < 64; ++cap) {
    std::vector<uint8_t> buf(cap + 1);
    int64_t off = 0;
    const int64_t need = vox_format_vec_flt("utt-1", v, 5, buf.data(), cap, &off);
    if (need <= 0) return 3;
  }
  std::printf("ok\n");
  return 0;
}

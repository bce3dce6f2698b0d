// Host-side AddressSanitizer / UBSan run of the native reader (kaldi_host.cpp is
// host-only code): the golden FM / CM arks walked record by record, every
// record parsed whole and from every truncated prefix (each must fail cleanly),
// batched shape reads and ragged chunk reads through the worker pool and on the
// calling thread, with valid and invalid chunk tables.  Build + run:
//   bash tools/asan/run.sh
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/voxemb.h"

// api.cpp's error slot, for the reader alone
static thread_local std::string g_err;
int vox_set_error(int code, const char* msg) {
  g_err = msg ? msg : "";
  return code;
}
extern "C" const char* vox_last_error(void) { return g_err.c_str(); }

static std::vector<uint8_t> slurp(const char* path) {
  std::vector<uint8_t> b;
  FILE* f = std::fopen(path, "rb");
  if (!f) return b;
  std::fseek(f, 0, SEEK_END);
  b.resize((size_t)std::ftell(f));
  std::fseek(f, 0, SEEK_SET);
  if (std::fread(b.data(), 1, b.size(), f) != b.size()) b.clear();
  std::fclose(f);
  return b;
}

int main(int argc, char** argv) {
  int fails = 0;
  std::mt19937 rng(7);
  for (int a = 1; a < argc; ++a) {
    const char* path = argv[a];
    std::vector<uint8_t> ark = slurp(path);
    if (ark.empty()) { std::printf("cannot read %s\n", path); return 2; }
    // records: "key " then a binary matrix
    std::vector<int64_t> offs;
    std::vector<int> R, C;
    size_t i = 0;
    while (i < ark.size()) {
      while (i < ark.size() && ark[i] != ' ') ++i;
      ++i;
      int r, c;
      if (vox_parse_mat_shape(ark.data() + i, ark.size() - i, &r, &c)) { ++fails; break; }
      std::vector<float> m((size_t)r * c + 1);
      size_t used = 0;
      if (vox_parse_mat_kaldi(ark.data() + i, ark.size() - i, m.data(), r, c, &used)) { ++fails; break; }
      // every truncated prefix fails cleanly
      for (size_t cut = 0; cut < used; cut += 1 + used / 97)
        if (vox_parse_mat_kaldi(ark.data() + i, cut, m.data(), r, c, nullptr) == 0) ++fails;
      offs.push_back((int64_t)i);
      R.push_back(r);
      C.push_back(c);
      i += used;
    }
    const int n = (int)offs.size();
    std::vector<const char*> paths(n, path);
    std::vector<int> rows(n), cols(n);
    for (int th : {1, 4})
      if (vox_mat_shapes(paths.data(), offs.data(), n, rows.data(), cols.data(), th) || rows != R) ++fails;
    // ragged chunk reads: random chunks of random utterances
    // chunk reads over the records of the first record's width
    const int F = C.empty() ? 0 : C[0];
    std::vector<int> pick;
    for (int u = 0; u < n; ++u)
      if (C[u] == F) pick.push_back(u);
    if (F == 0) continue;
    for (int rep = 0; rep < 200; ++rep) {
      const int nb = 1 + (int)(rng() % 9), stride = 64;
      std::vector<const char*> p(nb, path);
      std::vector<int64_t> o(nb);
      std::vector<int> r0(nb, 0), T(nb), c0(nb, 0), st(nb), ln(nb);
      for (int k = 0; k < nb; ++k) {
        const int u = pick[rng() % pick.size()];
        o[k] = offs[u];
        T[k] = R[u];
        ln[k] = 1 + (int)(rng() % std::min(stride, T[k]));
        st[k] = (int)(rng() % (T[k] - ln[k] + 1));
      }
      const bool bad = rep % 5 == 4;
      if (bad) {   // one invalid chunk: past the end, or a length outside [1, stride]
        const int k = (int)(rng() % nb);
        if (rep % 10 == 4) st[k] = T[k] - ln[k] + 1; else ln[k] = (rep % 20 == 9) ? 0 : stride + 1;
      }
      std::vector<float> out((size_t)nb * stride * F, 0.f);
      for (int th : {1, 4}) {
        const int rc = vox_read_chunks_ragged(p.data(), o.data(), r0.data(), T.data(), c0.data(),
                                              st.data(), ln.data(), nb, F, stride, 300, out.data(), th);
        if ((rc != 0) != bad) ++fails;
      }
    }
    std::printf("%s: %d records, chunk reads over %zu of width %d\n", path, n, pick.size(), F);
  }
  std::printf("%s (%d failures)\n", fails ? "FAILED" : "ok", fails);
  return fails ? 1 : 0;
}

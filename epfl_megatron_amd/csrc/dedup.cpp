// Near-duplicate detection for corpus cleaning (tools/openwebtext).
//
// The reference (tools/openwebtext/find_duplicates.py) fingerprints documents
// with the third-party `lsh` package (MinHash over character 5-grams, murmur3
// with 100 seeds, 10 LSH bands) driven from a 40-process Python pool, and
// computes Jaccard similarities of Python sets of shingles.  Here both are
// native: fingerprints are computed by a std::thread pool with the GIL
// released, band keys are 64-bit hashes of each band's minhash rows, and the
// Jaccard of two documents is computed on sorted 64-bit shingle hashes.
//
// Shingles are windows of `char_ngram` Unicode code points (texts arrive as
// UTF-8 and are decoded here), taken at offsets 0 .. len-ngram-1 exactly as the
// reference's `range(0, len(text) - char_ngram)` (the last window is skipped).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#ifdef EMA_EMBEDDED
#include <pybind11/embed.h>
#endif
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace {

std::vector<uint32_t> decode_utf8(const std::string& s) {
  std::vector<uint32_t> cps;
  cps.reserve(s.size());
  for (size_t i = 0; i < s.size();) {
    unsigned char c = s[i];
    int n = c < 0x80 ? 1 : (c >> 5) == 0x6 ? 2 : (c >> 4) == 0xE ? 3 : (c >> 3) == 0x1E ? 4 : 1;
    uint32_t cp = n == 1 ? c : c & (0x7F >> n);
    for (int k = 1; k < n && i + k < s.size(); ++k) cp = (cp << 6) | (s[i + k] & 0x3F);
    cps.push_back(cp);
    i += n;
  }
  return cps;
}

inline uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
  x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27; x *= 0x94d049bb133111ebULL;
  return x ^ (x >> 31);
}

// 64-bit hashes of every shingle window (FNV-1a over code points, then mixed).
std::vector<uint64_t> shingle_hashes(const std::string& text, int ngram) {
  auto cps = decode_utf8(text);
  std::vector<uint64_t> out;
  if ((int64_t)cps.size() <= ngram) return out;
  out.reserve(cps.size() - ngram);
  for (size_t h = 0; h + ngram < cps.size(); ++h) {
    uint64_t v = 1469598103934665603ULL;
    for (int k = 0; k < ngram; ++k) { v ^= cps[h + k]; v *= 1099511628211ULL; }
    out.push_back(mix64(v));
  }
  return out;
}

inline uint32_t seeded32(uint64_t shingle, uint64_t seed) {
  return (uint32_t)(mix64(shingle ^ mix64(seed + 0x9e3779b97f4a7c15ULL)) >> 32);
}

template <typename F>
void parallel_for(int64_t n, int threads, F fn) {
  threads = std::max(1, std::min<int>(threads, (int)std::max<int64_t>(1, n)));
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([=] { for (int64_t i = t; i < n; i += threads) fn(i); });
  for (auto& th : pool) th.join();
}

// [n_docs, n_seeds] uint32 MinHash signatures.  Empty documents get all-ones.
py::array_t<uint32_t> minhash(const std::vector<std::string>& texts,
                              py::array_t<int64_t, py::array::c_style> seeds, int char_ngram,
                              int threads) {
  const int64_t n = texts.size(), k = seeds.size();
  py::array_t<uint32_t> out({n, k});
  uint32_t* o = out.mutable_data();
  const int64_t* sd = seeds.data();
  {
    py::gil_scoped_release nogil;
    parallel_for(n, threads, [&](int64_t i) {
      auto sh = shingle_hashes(texts[i], char_ngram);
      std::sort(sh.begin(), sh.end());
      sh.erase(std::unique(sh.begin(), sh.end()), sh.end());
      for (int64_t j = 0; j < k; ++j) {
        uint32_t m = 0xFFFFFFFFu;
        for (uint64_t s : sh) m = std::min(m, seeded32(s, (uint64_t)sd[j]));
        o[i * k + j] = m;
      }
    });
  }
  return out;
}

// [n_docs, n_bands] uint64 band keys: hash of (band id, the band's minhash rows).
py::array_t<uint64_t> band_keys(py::array_t<uint32_t, py::array::c_style> sig, int num_bands) {
  const int64_t n = sig.shape(0), k = sig.shape(1);
  if (num_bands <= 0 || k % num_bands) throw std::invalid_argument("num_seeds % num_bands != 0");
  const int64_t rows = k / num_bands;
  py::array_t<uint64_t> out({n, (int64_t)num_bands});
  auto s = sig.unchecked<2>();
  auto o = out.mutable_unchecked<2>();
  for (int64_t i = 0; i < n; ++i)
    for (int b = 0; b < num_bands; ++b) {
      uint64_t v = mix64((uint64_t)b + 1);
      for (int64_t r = 0; r < rows; ++r) v = mix64(v ^ s(i, b * rows + r));
      o(i, b) = v;
    }
  return out;
}

// Jaccard of the shingle sets of two texts: mode 0 union, 1 min, 2 max.
double jaccard(const std::string& a, const std::string& b, int char_ngram, int mode) {
  auto x = shingle_hashes(a, char_ngram), y = shingle_hashes(b, char_ngram);
  for (auto* v : {&x, &y}) {
    std::sort(v->begin(), v->end());
    v->erase(std::unique(v->begin(), v->end()), v->end());
  }
  if (x.empty() || y.empty()) return 0.0;
  size_t i = 0, j = 0, inter = 0;
  while (i < x.size() && j < y.size()) {
    if (x[i] == y[j]) { ++inter; ++i; ++j; }
    else if (x[i] < y[j]) ++i;
    else ++j;
  }
  double denom = mode == 1 ? std::min(x.size(), y.size())
               : mode == 2 ? std::max(x.size(), y.size())
                           : x.size() + y.size() - inter;
  return inter / denom;
}

}  // namespace

// EMA_EMBEDDED: linked into the host-sanitizer harness (csrc/sanitize_main.cpp)
#ifdef EMA_EMBEDDED
PYBIND11_EMBEDDED_MODULE(_dedup, m) {
#else
PYBIND11_MODULE(_dedup, m) {
#endif
  m.doc() = "MinHash / LSH / shingle-Jaccard kernels for corpus de-duplication";
  m.def("minhash", &minhash, py::arg("texts"), py::arg("seeds"), py::arg("char_ngram") = 5,
        py::arg("threads") = 8);
  m.def("band_keys", &band_keys, py::arg("signatures"), py::arg("num_bands"));
  m.def("jaccard", &jaccard, py::arg("a"), py::arg("b"), py::arg("char_ngram") = 5,
        py::arg("mode") = 0);
}

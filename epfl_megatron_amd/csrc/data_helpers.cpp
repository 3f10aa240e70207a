// CPU dataset index builders (pybind11 module epfl_megatron_amd.data._helpers).
//
// Same algorithms and output arrays as the reference (megatron/data/helpers.cpp)
// so cached *_indexmap_*.npy files stay interchangeable:
//   sample_index  : int32 [num_samples + 1, 2] = (position in doc_idx, token offset),
//                   windows of seq_length + 1 tokens overlapping by one token;
//   blend_indices : greedy "largest deficit" interleave of several datasets;
//   sentence_pair_mapping : BERT/T5 samples (first sentence, end sentence,
//                   target length), shuffled with mt19937_64(seed + 1);
//   block_mapping : ICT evidence blocks (first sentence, end sentence, doc, block id).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#ifdef EMA_EMBEDDED
#include <pybind11/embed.h>
#endif

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <iostream>
#include <limits>
#include <random>
#include <stdexcept>
#include <vector>

namespace py = pybind11;

namespace {

py::array_t<int32_t> sample_index(py::array_t<int32_t, py::array::c_style | py::array::forcecast> sizes,
                                  py::array_t<int32_t, py::array::c_style | py::array::forcecast> doc_idx,
                                  int32_t seq_length, int32_t num_epochs, int64_t tokens_per_epoch) {
  if (seq_length <= 1 || num_epochs <= 0 || tokens_per_epoch <= 1)
    throw std::invalid_argument("invalid sample index arguments");
  const int32_t* sz = sizes.data();
  const int32_t* di = doc_idx.data();
  const int64_t n_doc_idx = doc_idx.shape(0);
  const int64_t num_samples = (num_epochs * tokens_per_epoch - 1) / seq_length;
  py::array_t<int32_t> out({num_samples + 1, (int64_t)2});
  int32_t* o = out.mutable_data();
  int64_t pos = 0;     // index into doc_idx
  int32_t offset = 0;  // token offset inside doc_idx[pos]
  o[0] = 0;
  o[1] = 0;
  for (int64_t s = 1; s <= num_samples; ++s) {
    int32_t need = seq_length + 1;
    while (need > 0) {
      if (pos >= n_doc_idx) throw std::out_of_range("doc_idx exhausted while building samples");
      const int32_t avail = sz[di[pos]] - offset;
      if (avail >= need) {
        // the window ends inside this document; the last token is shared with
        // the next sample (hence the -1)
        offset += need - 1;
        need = 0;
      } else {
        need -= avail;
        ++pos;
        offset = 0;
      }
    }
    o[2 * s] = (int32_t)pos;
    o[2 * s + 1] = offset;
  }
  return out;
}

py::tuple blend_indices(py::array_t<double, py::array::c_style | py::array::forcecast> weights,
                        int64_t size, bool verbose) {
  const int64_t n = weights.shape(0);
  if (n <= 0 || n > 255) throw std::invalid_argument("1..255 datasets supported");
  const double* w = weights.data();
  py::array_t<uint8_t> which(size);
  py::array_t<int64_t> within(size);
  uint8_t* pw = which.mutable_data();
  int64_t* pi = within.mutable_data();
  std::vector<int64_t> taken(n, 0);
  for (int64_t i = 0; i < size; ++i) {
    const double t = std::max((double)i, 1.0);
    int64_t best = 0;
    double best_err = w[0] * t - (double)taken[0];
    for (int64_t d = 1; d < n; ++d) {
      const double err = w[d] * t - (double)taken[d];
      if (err > best_err) {
        best_err = err;
        best = d;
      }
    }
    pw[i] = (uint8_t)best;
    pi[i] = taken[best]++;
  }
  if (verbose) {
    std::cout << " > sample ratios:" << std::endl;
    for (int64_t d = 0; d < n; ++d)
      std::cout << "   dataset " << d << ", input: " << w[d]
                << ", achieved: " << (double)taken[d] / (double)size << std::endl;
  }
  return py::make_tuple(which, within);
}

// Sample assembly: for every requested sample id s, copy the token window
// [sample_idx[s], sample_idx[s+1]] (inclusive end) out of the mapped corpus
// into row r of an int64 [n, seq_length + 1] batch, walking doc_idx across
// document boundaries.  Replaces the reference's per-sample Python loop of
// np.concatenate (megatron/data/gpt_dataset.py:243-269); releases the GIL so
// DataLoader worker threads scale.
template <typename T>
void stitch_impl(const T* tok, const int64_t* ptr, const int32_t* sz, const int32_t* di,
                 int64_t n_di, const int32_t* si, int64_t n_si, const int64_t* samples,
                 int64_t n, int64_t L, int64_t* out) {
  for (int64_t r = 0; r < n; ++r) {
    const int64_t s = samples[r];
    if (s < 0 || s + 1 >= n_si) throw std::out_of_range("sample id out of range");
    int64_t d = si[2 * s], off = si[2 * s + 1];
    const int64_t d_end = si[2 * s + 2], off_end = si[2 * s + 3];
    int64_t* o = out + r * L;
    int64_t w = 0;
    while (true) {
      if (d >= n_di) throw std::out_of_range("doc_idx position out of range");
      const int64_t item = di[d];
      const T* src = tok + ptr[item] / (int64_t)sizeof(T);
      const int64_t stop = (d == d_end) ? off_end + 1 : (int64_t)sz[item];
      const int64_t cnt = stop - off;
      if (cnt < 0 || w + cnt > L) throw std::length_error("sample window does not match seq_length");
      for (int64_t i = 0; i < cnt; ++i) o[w + i] = (int64_t)src[off + i];
      w += cnt;
      if (d == d_end) break;
      ++d;
      off = 0;
    }
    if (w != L) throw std::length_error("sample shorter than seq_length + 1");
  }
}

py::array_t<int64_t> stitch_samples(py::array tokens,
                                    py::array_t<int64_t, py::array::c_style | py::array::forcecast> pointers,
                                    py::array_t<int32_t, py::array::c_style | py::array::forcecast> sizes,
                                    py::array_t<int32_t, py::array::c_style | py::array::forcecast> doc_idx,
                                    py::array_t<int32_t, py::array::c_style | py::array::forcecast> sample_idx,
                                    py::array_t<int64_t, py::array::c_style | py::array::forcecast> samples,
                                    int64_t seq_length) {
  const int64_t n = samples.size(), L = seq_length + 1;
  py::array_t<int64_t> out({n, L});
  int64_t* o = out.mutable_data();
  const int64_t* p = pointers.data();
  const int32_t* sz = sizes.data();
  const int32_t* di = doc_idx.data();
  const int32_t* si = sample_idx.data();
  const int64_t* sm = samples.data();
  const int64_t n_di = doc_idx.size(), n_si = sample_idx.size() / 2;
  const char kind = tokens.dtype().kind();
  const ssize_t isz = tokens.itemsize();
  const void* t = tokens.data();
  py::gil_scoped_release nogil;
  if (kind == 'u' && isz == 2) stitch_impl((const uint16_t*)t, p, sz, di, n_di, si, n_si, sm, n, L, o);
  else if (kind == 'u' && isz == 1) stitch_impl((const uint8_t*)t, p, sz, di, n_di, si, n_si, sm, n, L, o);
  else if (kind == 'i' && isz == 4) stitch_impl((const int32_t*)t, p, sz, di, n_di, si, n_si, sm, n, L, o);
  else if (kind == 'i' && isz == 8) stitch_impl((const int64_t*)t, p, sz, di, n_di, si, n_si, sm, n, L, o);
  else if (kind == 'i' && isz == 2) stitch_impl((const int16_t*)t, p, sz, di, n_di, si, n_si, sm, n, L, o);
  else throw std::invalid_argument("unsupported token dtype");
  return out;
}

// ---- sentence-level samples (BERT / T5 / ICT) ------------------------------
// Reference: megatron/data/helpers.cpp build_mapping_impl :188-392 and
// build_blocks_mapping_impl :454-656.  One pass that appends to a vector (the
// reference counts in a first pass and fills in a second; with the same RNG
// consumption the arrays are identical), then a Fisher-Yates shuffle driven
// by mt19937_64(seed + 1) exactly as the reference so cached maps interchange.
constexpr int32_t kLongSentence = 512;

int32_t target_len(int32_t short_ratio, int32_t max_len, std::mt19937& gen) {
  if (short_ratio == 0) return max_len;
  const auto r = gen();
  if (r % (uint64_t)short_ratio == 0) return (int32_t)(2 + r % (uint64_t)(max_len - 1));
  return max_len;
}

bool has_long_sentence(const int32_t* sizes, int64_t first, int64_t last) {
  for (int64_t i = first; i < last; ++i)
    if (sizes[i] > kLongSentence) return true;
  return false;
}

template <typename Idx>
py::array shuffled(std::vector<uint64_t>& rows, int cols, int32_t seed) {
  const int64_t n = (int64_t)rows.size() / cols;
  std::mt19937_64 gen((uint64_t)(seed + 1));
  for (int64_t i = n - 1; i > 0; --i) {
    const int64_t j = (int64_t)(gen() % (uint64_t)(i + 1));
    for (int c = 0; c < cols; ++c) std::swap(rows[i * cols + c], rows[j * cols + c]);
  }
  py::array_t<Idx> out({n, (int64_t)cols});
  Idx* o = out.mutable_data();
  for (int64_t k = 0; k < n * cols; ++k) o[k] = (Idx)rows[k];
  return out;
}

py::array sentence_pair_mapping(py::array_t<int64_t, py::array::c_style | py::array::forcecast> docs,
                                py::array_t<int32_t, py::array::c_style | py::array::forcecast> sizes,
                                int32_t num_epochs, uint64_t max_num_samples,
                                int32_t max_seq_length, double short_seq_prob, int32_t seed,
                                bool verbose, int32_t min_num_sent) {
  if (num_epochs <= 0 || max_seq_length <= 1 || short_seq_prob < 0.0 || short_seq_prob > 1.0 ||
      seed <= 0)
    throw std::invalid_argument("invalid mapping arguments");
  const int64_t* d = docs.data();
  const int32_t* sz = sizes.data();
  const int64_t ndocs = docs.shape(0) - 1;
  const int32_t short_ratio = short_seq_prob > 0 ? (int32_t)std::round(1.0 / short_seq_prob) : 0;
  std::mt19937 gen((uint32_t)seed);
  std::vector<uint64_t> rows;
  uint64_t n = 0, empty = 0, one = 0, longd = 0;
  for (int32_t epoch = 0; epoch < num_epochs && n < max_num_samples; ++epoch) {
    for (int64_t doc = 0; doc < ndocs; ++doc) {
      const int64_t first = d[doc], last = d[doc + 1];
      int64_t remain = last - first;
      if (epoch == 0) {
        empty += remain == 0;
        one += remain == 1;
      }
      const bool lng = remain > 1 && has_long_sentence(sz, first, last);
      if (epoch == 0) longd += lng;
      if (remain < min_num_sent || lng) continue;
      int64_t start = first;
      int32_t len = 0, nsent = 0;
      int32_t target = target_len(short_ratio, max_seq_length, gen);
      for (int64_t s = first; s < last; ++s) {
        len += sz[s];
        ++nsent;
        --remain;
        if ((len >= target && remain > 1 && nsent >= min_num_sent) || remain == 0) {
          rows.push_back((uint64_t)start);
          rows.push_back((uint64_t)(s + 1));
          rows.push_back((uint64_t)target);
          ++n;
          start = s + 1;
          target = target_len(short_ratio, max_seq_length, gen);
          len = 0;
          nsent = 0;
        }
      }
    }
  }
  if (verbose)
    std::cout << "    sentence-pair mapping: " << n << " samples (" << empty << " empty, " << one
              << " one-sentence, " << longd << " long-sentence documents)" << std::endl;
  if (sizes.size() > (py::ssize_t)std::numeric_limits<uint32_t>::max())
    return shuffled<uint64_t>(rows, 3, seed);
  return shuffled<uint32_t>(rows, 3, seed);
}

py::array block_mapping(py::array_t<int64_t, py::array::c_style | py::array::forcecast> docs,
                        py::array_t<int32_t, py::array::c_style | py::array::forcecast> sizes,
                        py::array_t<int32_t, py::array::c_style | py::array::forcecast> title_sizes,
                        int32_t num_epochs, uint64_t max_num_samples, int32_t max_seq_length,
                        int32_t seed, bool verbose, bool use_one_sent_blocks) {
  if (num_epochs <= 0 || max_seq_length <= 1 || seed <= 0)
    throw std::invalid_argument("invalid block mapping arguments");
  const int64_t* d = docs.data();
  const int32_t* sz = sizes.data();
  const int32_t* tz = title_sizes.data();
  const int64_t ndocs = docs.shape(0) - 1;
  if (title_sizes.shape(0) < ndocs) throw std::invalid_argument("title sizes shorter than docs");
  const int32_t min_sent = use_one_sent_blocks ? 1 : 2;
  std::vector<uint64_t> rows;
  uint64_t n = 0;
  for (int32_t epoch = 0; epoch < num_epochs && n < max_num_samples; ++epoch) {
    int64_t block_id = 0;
    for (int64_t doc = 0; doc < ndocs; ++doc) {
      const int64_t first = d[doc], last = d[doc + 1];
      const int32_t target = max_seq_length - tz[doc];
      int64_t remain = last - first;
      if (remain < min_sent || has_long_sentence(sz, first, last)) continue;
      int64_t start = first;
      int32_t len = 0, nsent = 0;
      for (int64_t s = first; s < last; ++s) {
        len += sz[s];
        ++nsent;
        --remain;
        if ((len >= target && remain >= min_sent && nsent >= min_sent) || remain == 0) {
          rows.push_back((uint64_t)start);
          rows.push_back((uint64_t)(s + 1));
          rows.push_back((uint64_t)doc);
          rows.push_back((uint64_t)block_id);
          ++n;
          ++block_id;
          start = s + 1;
          len = 0;
          nsent = 0;
        }
      }
    }
  }
  if (verbose) std::cout << "    block mapping: " << n << " blocks" << std::endl;
  if (sizes.size() > (py::ssize_t)std::numeric_limits<uint32_t>::max())
    return shuffled<uint64_t>(rows, 4, seed);
  return shuffled<uint32_t>(rows, 4, seed);
}

}  // namespace

// EMA_EMBEDDED: linked into the host-sanitizer harness (csrc/sanitize_main.cpp)
#ifdef EMA_EMBEDDED
PYBIND11_EMBEDDED_MODULE(_helpers, m) {
#else
PYBIND11_MODULE(_helpers, m) {
#endif
  m.doc() = "dataset index builders";
  m.def("sample_index", &sample_index);
  m.def("blend_indices", &blend_indices);
  m.def("stitch_samples", &stitch_samples);
  m.def("sentence_pair_mapping", &sentence_pair_mapping);
  m.def("block_mapping", &block_mapping);
}

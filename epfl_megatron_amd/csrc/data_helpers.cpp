// CPU dataset index builders (pybind11 module epfl_megatron_amd.data._helpers).
//
// Same algorithms and output arrays as the reference (megatron/data/helpers.cpp)
// so cached *_indexmap_*.npy files stay interchangeable:
//   sample_index  : int32 [num_samples + 1, 2] = (position in doc_idx, token offset),
//                   windows of seq_length + 1 tokens overlapping by one token;
//   blend_indices : greedy "largest deficit" interleave of several datasets.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <cstdint>
#include <iostream>
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

}  // namespace

PYBIND11_MODULE(_helpers, m) {
  m.doc() = "dataset index builders";
  m.def("sample_index", &sample_index);
  m.def("blend_indices", &blend_indices);
}

// smx_pybind.cc — the search surface of the reference's pybind module in C++
// (pybind11 over the C ABI of include/scann_mi355x.h).
//
// Reference: scann/scann_ops/cc/python/scann_pybind.cc:24-54 binds
// research_scann::ScannNumpy (scann/scann_ops/cc/scann_npy.{h,cc});
// ScannNumpy::Search / SearchBatched (scann_npy.cc:213-271) check the query
// rank, release the GIL around the search, map a failed Status to
// RuntimeError("Error during search: ...") (RuntimeErrorIfNotOk,
// scann_npy.cc:41-47) and return (indices, distances) numpy arrays laid out
// by ReshapeNNResult / ReshapeBatchedNNResult (scann.h:162-180: ids and
// distances, padded with 0 / NaN, distances x -1 for dot-product indexes).
//
// ScannNumpyCore is that class for the MI355X path: it owns one smx_index
// (uploaded from an smx_index_desc whose arrays the Python side built by
// training or by loading the reference's assets, scann_amd/scann_pybind.py)
// and holds the config defaults ScannInterface resolves -1 arguments against
// (scann.cc:384-430).  Index construction (training, asset parsing) stays in
// Python; everything a search call does on the host is here.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>

#include "../../include/scann_mi355x.h"

namespace py = pybind11;

namespace {

template <typename T>
using np_row_major_arr = py::array_t<T, py::array::c_style | py::array::forcecast>;

void RuntimeErrorIfNotOk(const char* prefix, int status) {
  if (status != SMX_OK) throw std::runtime_error(std::string(prefix) + smx_last_error());
}

class ScannNumpyCore {
 public:
  // desc_address: the address of a filled smx_index_desc (its arrays must
  // stay alive for the duration of this call only: smx_index_create copies
  // them to the device).
  ScannNumpyCore(uintptr_t desc_address, int device, int num_neighbors, int reorder_num_neighbors,
                 int leaves_to_search, bool has_reordering, bool dot_product)
      : num_neighbors_(num_neighbors),
        reorder_num_neighbors_(reorder_num_neighbors),
        leaves_to_search_(leaves_to_search),
        has_reordering_(has_reordering),
        multiplier_(dot_product ? -1.0f : 1.0f) {
    if (desc_address == 0) throw std::invalid_argument("null index description");
    const auto* desc = reinterpret_cast<const smx_index_desc*>(desc_address);
    RuntimeErrorIfNotOk("Failed to create the index: ", smx_index_create(desc, device, &h_));
    int32_t dim = 0, nl = 0, shift = 0;
    uint32_t n = 0;
    RuntimeErrorIfNotOk("Failed to create the index: ", smx_index_info(h_, &dim, &nl, &n, &shift));
    dim_ = dim;
    size_ = n;
  }
  ~ScannNumpyCore() {
    if (h_) smx_index_destroy(h_);
  }
  ScannNumpyCore(const ScannNumpyCore&) = delete;
  ScannNumpyCore& operator=(const ScannNumpyCore&) = delete;

  // ScannNumpy::Search (scann_npy.cc:213-232): one query through the
  // single-query numerics (smx_search).
  std::pair<py::array_t<uint32_t>, py::array_t<float>> Search(const np_row_major_arr<float>& query,
                                                              int final_nn, int pre_reorder_nn,
                                                              int leaves) {
    if (query.ndim() != 1) throw std::invalid_argument("Query must be one-dimensional");
    const smx_search_params p = Resolve(final_nn, pre_reorder_nn, leaves);
    py::array_t<uint32_t> idx(p.final_nn);
    py::array_t<float> dist(p.final_nn);
    int32_t count = 0;
    int rc;
    {
      py::gil_scoped_release release;
      rc = smx_search(h_, query.data(), int32_t(query.size()), &p, idx.mutable_data(),
                      dist.mutable_data(), &count);
    }
    RuntimeErrorIfNotOk("Error during search: ", rc);
    // ReshapeNNResult: exactly the results found, distances x multiplier
    py::array_t<uint32_t> out_idx(count);
    py::array_t<float> out_dist(count);
    for (int32_t i = 0; i < count; ++i) {
      out_idx.mutable_data()[i] = idx.data()[i];
      out_dist.mutable_data()[i] = dist.data()[i] * multiplier_;
    }
    return {out_idx, out_dist};
  }

  // ScannNumpy::SearchBatched (scann_npy.cc:234-271).  `parallel` and
  // `batch_size` select the reference's CPU thread split
  // (SearchBatchedParallel); the device batch is one pipeline either way,
  // with identical results.
  std::pair<py::array_t<uint32_t>, py::array_t<float>> SearchBatched(
      const np_row_major_arr<float>& queries, int final_nn, int pre_reorder_nn, int leaves,
      bool parallel, int batch_size) {
    (void)parallel;
    (void)batch_size;
    if (queries.ndim() != 2)
      throw std::invalid_argument("Queries must be in two-dimensional array");
    const smx_search_params p = Resolve(final_nn, pre_reorder_nn, leaves);
    const py::ssize_t nq = queries.shape(0);
    py::array_t<uint32_t> idx({nq, py::ssize_t(p.final_nn)});
    py::array_t<float> dist({nq, py::ssize_t(p.final_nn)});
    int rc;
    {
      py::gil_scoped_release release;
      rc = smx_search_batched(h_, queries.data(), int32_t(nq), int32_t(queries.shape(1)), &p,
                              idx.mutable_data(), dist.mutable_data(), nullptr);
      if (rc == SMX_OK && multiplier_ != 1.0f) {
        float* d = dist.mutable_data();
        for (py::ssize_t i = 0; i < nq * p.final_nn; ++i) d[i] *= multiplier_;   // NaN pads stay NaN
      }
    }
    RuntimeErrorIfNotOk("Error during search: ", rc);
    return {idx, dist};
  }

  size_t Size() const { return size_; }
  int Dim() const { return dim_; }

 private:
  // ScannInterface::GetSearchParameters[Batched] (scann.cc:384-430): a
  // non-positive argument takes the config's default; without reordering
  // pre_reorder_nn is final_nn.
  smx_search_params Resolve(int final_nn, int pre_reorder_nn, int leaves) const {
    smx_search_params p;
    p.final_nn = final_nn > 0 ? final_nn : num_neighbors_;
    p.pre_reorder_nn = has_reordering_ ? (pre_reorder_nn > 0 ? pre_reorder_nn : reorder_num_neighbors_)
                                       : p.final_nn;
    p.leaves_to_search = leaves > 0 ? leaves : leaves_to_search_;
    p.reorder = has_reordering_ ? 1 : 0;
    return p;
  }

  smx_index* h_ = nullptr;
  int num_neighbors_, reorder_num_neighbors_, leaves_to_search_;
  bool has_reordering_;
  float multiplier_;
  int dim_ = 0;
  size_t size_ = 0;
};

}  // namespace

PYBIND11_MODULE(_smx_pybind, m) {
  m.doc() = "pybind11 search surface of ScannNumpy over the MI355X C ABI";
  py::class_<ScannNumpyCore>(m, "ScannNumpyCore")
      .def(py::init<uintptr_t, int, int, int, int, bool, bool>(), py::arg("desc_address"),
           py::arg("device"), py::arg("num_neighbors"), py::arg("reorder_num_neighbors"),
           py::arg("leaves_to_search"), py::arg("has_reordering"), py::arg("dot_product"))
      .def("search", &ScannNumpyCore::Search, py::arg("query"), py::arg("final_nn") = -1,
           py::arg("pre_reorder_nn") = -1, py::arg("leaves") = -1)
      .def("search_batched", &ScannNumpyCore::SearchBatched, py::arg("queries"),
           py::arg("final_nn") = -1, py::arg("pre_reorder_nn") = -1, py::arg("leaves") = -1,
           py::arg("parallel") = false, py::arg("batch_size") = 256)
      .def("size", &ScannNumpyCore::Size)
      .def("dim", &ScannNumpyCore::Dim);
}

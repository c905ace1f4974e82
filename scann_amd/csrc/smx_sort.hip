// smx_sort.hip — the index build's grouping of members by leaf on the device
// (the reference's datapoints_by_token: members of each leaf in ascending
// datapoint id, kmeans_tree_partitioner.cc:477-620, 532-535; with SOAR every
// datapoint appears in its primary and its spilled leaf).
//
// (leaf, id) pairs are packed into 64-bit keys leaf << 32 | id and sorted by
// rocPRIM's device radix sort over the significant bits only; the leaf
// offsets are the first positions of each leaf in the sorted keys (one
// thread per key, no atomics), and the gather of the members' residuals
// (x[row] - center[leaf], float32) follows the sorted order.
#include <hip/hip_runtime.h>

#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>

#include <cstdint>

#include "smx_internal.h"

namespace smx {
namespace {

__global__ void __launch_bounds__(256) pack_keys_kernel(const int32_t* __restrict__ labels,
                                                        const uint32_t* __restrict__ ids,
                                                        int64_t m, uint64_t* __restrict__ keys) {
  const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= m) return;
  keys[i] = (uint64_t(uint32_t(labels[i])) << 32) | ids[i];
}

// offsets[l] = the first sorted position with leaf >= l; offsets[k] = m.
__global__ void __launch_bounds__(256) leaf_offsets_kernel(const uint64_t* __restrict__ keys,
                                                           int64_t m, int k,
                                                           uint64_t* __restrict__ offsets,
                                                           uint32_t* __restrict__ members,
                                                           int32_t* __restrict__ member_leaf) {
  const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i > m) return;
  const int64_t leaf = i < m ? int64_t(keys[i] >> 32) : int64_t(k);
  const int64_t prev = i > 0 ? int64_t(keys[i - 1] >> 32) : -1;
  for (int64_t l = prev + 1; l <= leaf && l <= k; ++l) offsets[l] = uint64_t(i);
  if (i < m) {
    members[i] = uint32_t(keys[i]);
    member_leaf[i] = int32_t(leaf);
  }
}

__global__ void __launch_bounds__(256) gather_residuals_kernel(
    const float* __restrict__ x, int d, const uint32_t* __restrict__ rows,
    const int32_t* __restrict__ leaf, const float* __restrict__ centers, int64_t m,
    int64_t row_base, float* __restrict__ out) {
  const int64_t e = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (e >= m * d) return;
  const int64_t i = e / d;
  const int j = int(e - i * d);
  const float v = x[(int64_t(rows[i]) - row_base) * d + j];
  out[e] = centers ? __fsub_rn(v, centers[int64_t(leaf[i]) * d + j]) : v;
}

}  // namespace

hipError_t GroupByLeaf(const int32_t* labels, const uint32_t* ids, int64_t m, int k, void* temp,
                       size_t* temp_bytes, uint64_t* keys, uint64_t* offsets, uint32_t* members,
                       int32_t* member_leaf, hipStream_t s) {
  // keys [2 m] (input half, sorted half); temp: rocPRIM's scratch
  int bits = 1;
  while ((int64_t(1) << bits) < int64_t(k)) ++bits;
  const unsigned end_bit = 32u + unsigned(bits);
  if (!temp) {
    return rocprim::radix_sort_keys(nullptr, *temp_bytes, keys, keys + m, size_t(m), 0u, end_bit,
                                    s);
  }
  if (m > 0) {
    hipLaunchKernelGGL(pack_keys_kernel, dim3(unsigned((m + 255) / 256)), dim3(256), 0, s, labels,
                       ids, m, keys);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = rocprim::radix_sort_keys(temp, *temp_bytes, keys, keys + m, size_t(m), 0u, end_bit, s);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(leaf_offsets_kernel, dim3(unsigned((m + 1 + 255) / 256)), dim3(256), 0, s,
                     keys + m, m, k, offsets, members, member_leaf);
  return hipGetLastError();
}

hipError_t LaunchGatherResiduals(const float* x, int d, const uint32_t* rows, const int32_t* leaf,
                                 const float* centers, int64_t m, int64_t row_base, float* out,
                                 hipStream_t s) {
  if (m <= 0) return hipSuccess;
  const int64_t total = m * d;
  hipLaunchKernelGGL(gather_residuals_kernel, dim3(unsigned((total + 255) / 256)), dim3(256), 0,
                     s, x, d, rows, leaf, centers, m, row_base, out);
  return hipGetLastError();
}

}  // namespace smx

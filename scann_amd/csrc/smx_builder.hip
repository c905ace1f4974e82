// smx_builder.hip — index-build kernels for gfx950: the nearest center of
// every row (the assignment step of k-means training and of the datapoint
// partitioning) and the SOAR secondary assignment.
//
// Reference:
//   k-means assignment: GmmUtils::KMeansImpl's nearest-center step
//     (scann/utils/gmm_utils.cc:539-1318; squared L2 to every center,
//     ties to the lowest center index);
//   SOAR: KMeansTreePartitioner's spilled assignment
//     (scann/partitioning/kmeans_tree_partitioner.cc:926-997): with r = x -
//     c_primary, loss_j = ||x - c_j||^2 + lambda * <r, x - c_j>^2 / ||r||^2,
//     the primary center excluded.
//
// One 256-thread block takes 64 rows and sweeps all centers in tiles of 64:
// rows and centers staged through LDS 32 dimensions at a time (coalesced
// row-major loads, stored dimension-major), each thread a 4 x 4 micro-tile
// of dot products as an explicit fma chain; the running best (loss, index)
// per row stays in registers across the center tiles, and the 16 threads
// sharing a row reduce lexicographically at the end.  The per-center
// ||c||^2 and the SOAR per-row scalars (||x||^2, ||r||^2, <r, x>) are
// accumulated in the same sweep.  Build-time work: the roofline is the f32
// VALU (2 flops per fma per row-center pair per dimension).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "smx_internal.h"

namespace smx {
namespace {

constexpr int kNcRows = 64, kNcCtr = 64, kNcDim = 32, kNcPad = 4;

template <bool SOAR>
__global__ void __launch_bounds__(256) nearest_centers_kernel(
    const float* __restrict__ x, int64_t n, int d, const float* __restrict__ c, int k,
    const int32_t* __restrict__ primary, float lambda, int32_t* __restrict__ out,
    float* __restrict__ out_loss) {
  __shared__ __align__(16) float xs[kNcDim][kNcRows + kNcPad];   // [dim][row]
  __shared__ __align__(16) float cs[kNcDim][kNcCtr + kNcPad];    // [dim][center]
  __shared__ __align__(16) float rs[SOAR ? kNcDim : 1][kNcRows + kNcPad];
  __shared__ int32_t s_prim[kNcRows];
  __shared__ float s_bv[kNcRows][17];
  __shared__ int32_t s_bi[kNcRows][17];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int64_t r0 = int64_t(blockIdx.x) * kNcRows;
  if (SOAR && tid < kNcRows) s_prim[tid] = r0 + tid < n ? primary[r0 + tid] : 0;
  float best[4];
  int32_t bidx[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    best[i] = __int_as_float(0x7f800000);   // +inf
    bidx[i] = -1;
  }
  for (int c0 = 0; c0 < k; c0 += kNcCtr) {
    float acc[4][4], accr[4][4], cn[4];
    float xx[4], rr[4], rx[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      cn[i] = xx[i] = rr[i] = rx[i] = 0.0f;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = accr[i][j] = 0.0f;
    }
    for (int d0 = 0; d0 < d; d0 += kNcDim) {
      __syncthreads();   // the previous chunk's tiles are consumed
#pragma unroll
      for (int m = 0; m < kNcRows * kNcDim / 256; ++m) {
        const int e = tid + 256 * m, rr_ = e / kNcDim, dd = e % kNcDim;
        const int64_t row = r0 + rr_;
        const bool ok = row < n && d0 + dd < d;
        const float xv = ok ? x[row * d + d0 + dd] : 0.0f;
        xs[dd][rr_] = xv;
        if (SOAR) rs[dd][rr_] = ok ? __fsub_rn(xv, c[int64_t(s_prim[rr_]) * d + d0 + dd]) : 0.0f;
        const int cj = c0 + rr_;
        cs[dd][rr_] = (cj < k && d0 + dd < d) ? c[int64_t(cj) * d + d0 + dd] : 0.0f;
      }
      __syncthreads();
#pragma unroll 8
      for (int dd = 0; dd < kNcDim; ++dd) {
        const float4 xv = *reinterpret_cast<const float4*>(&xs[dd][ty * 4]);
        const float4 cv = *reinterpret_cast<const float4*>(&cs[dd][tx * 4]);
        const float xa[4] = {xv.x, xv.y, xv.z, xv.w}, ca[4] = {cv.x, cv.y, cv.z, cv.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) cn[j] = __fmaf_rn(ca[j], ca[j], cn[j]);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __fmaf_rn(xa[i], ca[j], acc[i][j]);
        if (SOAR) {
          const float4 rv = *reinterpret_cast<const float4*>(&rs[dd][ty * 4]);
          const float ra[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            xx[i] = __fmaf_rn(xa[i], xa[i], xx[i]);
            rr[i] = __fmaf_rn(ra[i], ra[i], rr[i]);
            rx[i] = __fmaf_rn(ra[i], xa[i], rx[i]);
#pragma unroll
            for (int j = 0; j < 4; ++j) accr[i][j] = __fmaf_rn(ra[i], ca[j], accr[i][j]);
          }
        }
      }
    }
    // centers are visited in increasing index order within a thread, so a
    // strict < keeps the lowest index of equal losses
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int cj = c0 + tx * 4 + j;
      if (cj >= k) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float loss;
        if (SOAR) {
          if (cj == s_prim[ty * 4 + i]) continue;
          // ||x - c||^2 = ||x||^2 - 2<x, c> + ||c||^2; <r, x - c> = <r, x> - <r, c>
          const float d2 = __fadd_rn(__fsub_rn(xx[i], __fmul_rn(2.0f, acc[i][j])), cn[j]);
          const float proj = __fsub_rn(rx[i], accr[i][j]);
          const float rn = fmaxf(rr[i], 1e-30f);
          loss = __fadd_rn(d2, __fdiv_rn(__fmul_rn(lambda, __fmul_rn(proj, proj)), rn));
        } else {
          // argmin ||x - c||^2 = argmin ||c||^2 - 2<x, c>
          loss = __fsub_rn(cn[j], __fmul_rn(2.0f, acc[i][j]));
        }
        if (loss < best[i]) {
          best[i] = loss;
          bidx[i] = cj;
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    s_bv[ty * 4 + i][tx] = best[i];
    s_bi[ty * 4 + i][tx] = bidx[i];
  }
  __syncthreads();
  if (tid < kNcRows && r0 + tid < n) {
    float bv = s_bv[tid][0];
    int32_t bi = s_bi[tid][0];
    for (int t = 1; t < 16; ++t) {
      const float v = s_bv[tid][t];
      const int32_t i = s_bi[tid][t];
      if (i >= 0 && (bi < 0 || v < bv || (v == bv && i < bi))) {
        bv = v;
        bi = i;
      }
    }
    out[r0 + tid] = bi;
    if (out_loss) out_loss[r0 + tid] = bv;
  }
}

}  // namespace

hipError_t LaunchNearestCenters(const float* x, int64_t n, int d, const float* centers, int k,
                                const int32_t* primary, float lambda, int32_t* out,
                                float* out_loss, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const unsigned blocks = unsigned((n + kNcRows - 1) / kNcRows);
  if (primary)
    hipLaunchKernelGGL(nearest_centers_kernel<true>, dim3(blocks), dim3(256), 0, s, x, n, d,
                       centers, k, primary, lambda, out, out_loss);
  else
    hipLaunchKernelGGL(nearest_centers_kernel<false>, dim3(blocks), dim3(256), 0, s, x, n, d,
                       centers, k, primary, lambda, out, out_loss);
  return hipGetLastError();
}

}  // namespace smx

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

#include <algorithm>
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


// ---------------------------------------------------------------------------
// Nearest codebook center per (row, block): the plain AH encoding
// (asymmetric_hashing_impl.cc IndexDatapoint's nearest-center search over the
// 16 centers of each block; squared L2 summed over the block's coordinates in
// order, the last block zero-padded; ties to the lowest center).  One thread
// per (row, block).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) block_encode_kernel(const float* __restrict__ r, int64_t n,
                                                           int dim, const float* __restrict__ cb,
                                                           int nb, int dpb,
                                                           uint8_t* __restrict__ out) {
  const int64_t e = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (e >= n * nb) return;
  const int64_t row = e / nb;
  const int b = int(e - row * nb);
  float best = 0.0f;
  int bi = 0;
  for (int c = 0; c < 16; ++c) {
    float d = 0.0f;
    for (int i = 0; i < dpb; ++i) {
      const int j = b * dpb + i;
      const float v = __fsub_rn(j < dim ? r[row * dim + j] : 0.0f, cb[(b * 16 + c) * dpb + i]);
      d = __fadd_rn(d, __fmul_rn(v, v));
    }
    if (c == 0 || d < best) {
      best = d;
      bi = c;
    }
  }
  out[e] = uint8_t(bi);
}

// ---------------------------------------------------------------------------
// k-means center update (GmmUtils' mean step, gmm_utils.cc:539-1318) as exact
// fixed-point sums: every value enters as llrint(x * scale) (scale = 2^e
// chosen by the caller so that no sum can overflow), so the 64-bit integer
// atomics give the same sums in any order -- the center update is
// deterministic, run to run.  One thread per (row, coordinate).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) kmeans_accumulate_kernel(
    const float* __restrict__ x, int64_t n, int d, const int32_t* __restrict__ label, int k,
    double scale, unsigned long long* __restrict__ sums, uint32_t* __restrict__ counts) {
  const int64_t e = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (e >= n * d) return;
  const int64_t row = e / d;
  const int j = int(e - row * d);
  const int l = label[row];
  if (l < 0 || l >= k) return;
  const long long v = llrint(double(x[e]) * scale);
  atomicAdd(&sums[int64_t(l) * d + j], (unsigned long long)v);
  if (j == 0) atomicAdd(&counts[l], 1u);
}

// centers[c] = sums[c] / scale / count[c] for every non-empty center (empty
// ones keep their value: the caller reseeds them)
__global__ void __launch_bounds__(256) kmeans_finalize_kernel(
    const unsigned long long* __restrict__ sums, const uint32_t* __restrict__ counts, int k, int d,
    double scale, float* __restrict__ centers) {
  const int64_t e = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (e >= int64_t(k) * d) return;
  const uint32_t cnt = counts[e / d];
  if (cnt == 0) return;
  const double mean = __ddiv_rn(__ddiv_rn(double((long long)sums[e]), scale), double(cnt));
  centers[e] = float(mean);
}

// The codebook's k-means mean step for all blocks at once: sums[(b*16 +
// code) * dpb + i] += r[row][b*dpb + i] (fixed point), counts[b*16 + code]++.
// The block's partial sums are kept in LDS (ds_add_u64) and flushed with one
// global atomic per entry; shapes whose sums exceed 64 KB of LDS add to the
// global sums directly (codebook_accumulate_global_kernel).  256 threads,
// each a run of rows.
__global__ void __launch_bounds__(256) codebook_accumulate_global_kernel(
    const float* __restrict__ r, int64_t n, int dim, const uint8_t* __restrict__ codes, int nb,
    int dpb, double scale, unsigned long long* __restrict__ sums, uint32_t* __restrict__ counts) {
  const int64_t e = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (e >= n * nb) return;
  const int64_t row = e / nb;
  const int b = int(e - row * nb);
  const int c = codes[e];
  for (int i = 0; i < dpb; ++i) {
    const int j = b * dpb + i;
    const float v = j < dim ? r[row * dim + j] : 0.0f;
    atomicAdd(&sums[(b * 16 + c) * dpb + i], (unsigned long long)llrint(double(v) * scale));
  }
  atomicAdd(&counts[b * 16 + c], 1u);
}

__global__ void __launch_bounds__(256) codebook_accumulate_kernel(
    const float* __restrict__ r, int64_t n, int dim, const uint8_t* __restrict__ codes, int nb,
    int dpb, double scale, unsigned long long* __restrict__ sums, uint32_t* __restrict__ counts) {
  extern __shared__ unsigned long long cb_lds[];
  const int ne = nb * 16 * dpb, nc = nb * 16;
  uint32_t* lcnt = reinterpret_cast<uint32_t*>(cb_lds + ne);
  for (int i = threadIdx.x; i < ne; i += 256) cb_lds[i] = 0ull;
  for (int i = threadIdx.x; i < nc; i += 256) lcnt[i] = 0u;
  __syncthreads();
  const int64_t total = n * nb;
  for (int64_t e = int64_t(blockIdx.x) * 256 + threadIdx.x; e < total;
       e += int64_t(gridDim.x) * 256) {
    const int64_t row = e / nb;
    const int b = int(e - row * nb);
    const int c = codes[e];
    for (int i = 0; i < dpb; ++i) {
      const int j = b * dpb + i;
      const float v = j < dim ? r[row * dim + j] : 0.0f;
      atomicAdd(&cb_lds[(b * 16 + c) * dpb + i], (unsigned long long)llrint(double(v) * scale));
    }
    atomicAdd(&lcnt[b * 16 + c], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < ne; i += 256)
    if (cb_lds[i]) atomicAdd(&sums[i], cb_lds[i]);
  for (int i = threadIdx.x; i < nc; i += 256)
    if (lcnt[i]) atomicAdd(&counts[i], lcnt[i]);
}

// ---------------------------------------------------------------------------
// Anisotropic (AVQ) noise-shaped encoding: IndexDatapointNoiseShaped
// (asymmetric_hashing_impl.cc:434-503) with ComputeResidualStats (:283-343),
// InitializeToMinResidualNorm and OptimizeSingleSubspace (:366-404), in
// double precision with every rounding explicit, bit for bit the oracle's
// orc_avq_encode (oracle/scann_oracle.cc).  One row per 16 lanes (lane c =
// center c of the block being optimised), 4 rows per 64-thread block; the
// row's residual and original coordinates (zero-padded to nb * dpb) staged
// in LDS; the per-(block, center) residual norm and parallel component are
// recomputed where needed (the same operations give the same doubles).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void AvqStats(const float* rs, const float* xs, const float* cb, int b,
                                         int c, int dpb, double inv_norm, double& a, double& p) {
  a = 0.0;
  p = 0.0;
  for (int i = 0; i < dpb; ++i) {
    const int j = b * dpb + i;
    const double rc = __dsub_rn(double(rs[j]), double(cb[(b * 16 + c) * dpb + i]));
    a = __dadd_rn(a, __dmul_rn(rc, rc));
    p = __dadd_rn(p, __dmul_rn(__dmul_rn(rc, double(xs[j])), inv_norm));
  }
}

__global__ void __launch_bounds__(64) avq_encode_kernel(const float* __restrict__ resid,
                                                        const float* __restrict__ orig, int64_t n,
                                                        int dim, const float* __restrict__ cb,
                                                        int nb, int dpb, double threshold,
                                                        uint8_t* __restrict__ out) {
  extern __shared__ __align__(16) unsigned char avq_lds[];
  const int lane = threadIdx.x, g = lane >> 4, c = lane & 15, base = g * 16;
  const int nbd = nb * dpb;
  // per row: rs[nbd], xs[nbd] (float); curv[nb] (double); code[nb]; ord[nb] (u16)
  float* rs = reinterpret_cast<float*>(avq_lds) + size_t(g) * 2 * nbd;
  float* xs = rs + nbd;
  const size_t fbytes = (size_t(4) * 2 * nbd * 4 + 15) & ~size_t(15);
  double* curv = reinterpret_cast<double*>(avq_lds + fbytes) + size_t(g) * nb;
  uint16_t* ord = reinterpret_cast<uint16_t*>(avq_lds + fbytes + size_t(4) * nb * 8) + size_t(g) * nb;
  uint8_t* code =
      reinterpret_cast<uint8_t*>(avq_lds + fbytes + size_t(4) * nb * 8 + size_t(4) * nb * 2) +
      size_t(g) * nb;
  const int64_t row = int64_t(blockIdx.x) * 4 + g;
  const bool live = row < n;   // (uniform per 16-lane group)
  for (int j = c; j < nbd; j += 16) {
    rs[j] = live && j < dim ? resid[row * dim + j] : 0.0f;
    xs[j] = live && j < dim ? orig[row * dim + j] : 0.0f;
  }
  __syncthreads();
  if (!live) return;   // no barrier follows (one wave per block)
  // ||x||^2 in coordinate order (lane 0 of the group), then the cost multiplier
  double sqn = 0.0;
  if (c == 0)
    for (int j = 0; j < nbd; ++j) sqn = __dadd_rn(sqn, __dmul_rn(double(xs[j]), double(xs[j])));
  sqn = __shfl(sqn, base);
  const double inv_norm = __ddiv_rn(1.0, __dsqrt_rn(sqn));
  const double t2 = __dmul_rn(threshold, threshold);
  const double eta = __ddiv_rn(__ddiv_rn(t2, sqn),
                               __ddiv_rn(__dsub_rn(1.0, __ddiv_rn(t2, sqn)),
                                         __dsub_rn(double(dim), 1.0)));
  // InitializeToMinResidualNorm: each block's first-minimum residual norm
  // (a NaN at center 0 keeps center 0, as the sequential scan does); P = the
  // sum of the chosen parallel components in block order
  double P = 0.0;
  for (int b = 0; b < nb; ++b) {
    double a, p;
    AvqStats(rs, xs, cb, b, c, dpb, inv_norm, a, p);
    double bv = a;
    int bc = c;
    const bool nan0 = __shfl(a, base) != __shfl(a, base);
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {   // min of (value, index), NaN never wins
      const double ov = __shfl_xor(bv, off, 16);
      const int oc = __shfl_xor(bc, off, 16);
      const bool take = (ov < bv) || (ov == bv && oc < bc) || (bv != bv && ov == ov);
      if (take) {
        bv = ov;
        bc = oc;
      }
    }
    if (nan0 || bv != bv) bc = 0;
    const double pb = __shfl(p, base + bc);
    const double ab = __shfl(a, base + bc);
    if (c == 0) {
      code[b] = uint8_t(bc);
      curv[b] = ab;
      P = __dadd_rn(P, pb);
    }
  }
  P = __shfl(P, base);
  // (one wave per block: LDS accesses execute in order; the fence keeps the
  // compiler from caching another lane's LDS words in registers)
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  // blocks by their residual norm, largest first, ties in block order
  for (int b = c; b < nb; b += 16) {
    const double v = curv[b];
    int rank = 0;
    for (int o = 0; o < nb; ++o) rank += (curv[o] > v) || (curv[o] == v && o < b);
    ord[rank] = uint16_t(b);
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  bool changed = true;
  for (int round = 0; changed && round < 10; ++round) {
    changed = false;
    for (int i = 0; i < nb; ++i) {
      const int b = ord[i];
      const int cur = code[b];
      double a, p;
      AvqStats(rs, xs, cb, b, c, dpb, inv_norm, a, p);
      const double old_rn = __shfl(a, base + cur), old_par = __shfl(p, base + cur);
      const double new_p = __dadd_rn(__dsub_rn(P, old_par), p);
      const double pnd = __dsub_rn(__dmul_rn(new_p, new_p), __dmul_rn(P, P));
      const double rnd = __dsub_rn(a, old_rn);
      const double perp = __dsub_rn(rnd, pnd);
      const double cost = __dadd_rn(__dmul_rn(eta, pnd), perp);
      const bool cand = c != cur && !(pnd > 0.0) && cost < 0.0;
      double bv = cand ? cost : 0.0;
      int bc = cand ? c : 16;
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) {
        const double ov = __shfl_xor(bv, off, 16);
        const int oc = __shfl_xor(bc, off, 16);
        if (oc < 16 && (bc == 16 || ov < bv || (ov == bv && oc < bc))) {
          bv = ov;
          bc = oc;
        }
      }
      if (bc < 16) {   // (uniform in the group)
        P = __shfl(new_p, base + bc);
        if (c == 0) code[b] = uint8_t(bc);
        changed = true;
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
  }
  for (int b = c; b < nb; b += 16) out[row * nb + b] = code[b];
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


hipError_t LaunchBlockEncode(const float* r, int64_t n, int dim, const float* cb, int nb, int dpb,
                             uint8_t* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t total = n * nb;
  hipLaunchKernelGGL(block_encode_kernel, dim3(unsigned((total + 255) / 256)), dim3(256), 0, s, r,
                     n, dim, cb, nb, dpb, out);
  return hipGetLastError();
}

hipError_t LaunchKmeansAccumulate(const float* x, int64_t n, int d, const int32_t* label, int k,
                                  double scale, unsigned long long* sums, uint32_t* counts,
                                  hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t total = n * d;
  hipLaunchKernelGGL(kmeans_accumulate_kernel, dim3(unsigned((total + 255) / 256)), dim3(256), 0,
                     s, x, n, d, label, k, scale, sums, counts);
  return hipGetLastError();
}

hipError_t LaunchKmeansFinalize(const unsigned long long* sums, const uint32_t* counts, int k,
                                int d, double scale, float* centers, hipStream_t s) {
  const int64_t total = int64_t(k) * d;
  hipLaunchKernelGGL(kmeans_finalize_kernel, dim3(unsigned((total + 255) / 256)), dim3(256), 0, s,
                     sums, counts, k, d, scale, centers);
  return hipGetLastError();
}

size_t CodebookAccumulateLds(int nb, int dpb) {
  return size_t(nb) * 16 * dpb * 8 + size_t(nb) * 16 * 4;
}

hipError_t LaunchCodebookAccumulate(const float* r, int64_t n, int dim, const uint8_t* codes,
                                    int nb, int dpb, double scale, unsigned long long* sums,
                                    uint32_t* counts, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t total = n * nb;
  if (CodebookAccumulateLds(nb, dpb) > 65536) {
    hipLaunchKernelGGL(codebook_accumulate_global_kernel, dim3(unsigned((total + 255) / 256)),
                       dim3(256), 0, s, r, n, dim, codes, nb, dpb, scale, sums, counts);
    return hipGetLastError();
  }
  const unsigned grid = unsigned(std::min<int64_t>(2048, (total + 255) / 256));
  hipLaunchKernelGGL(codebook_accumulate_kernel, dim3(grid), dim3(256),
                     CodebookAccumulateLds(nb, dpb), s, r, n, dim, codes, nb, dpb, scale, sums,
                     counts);
  return hipGetLastError();
}

size_t AvqEncodeLds(int nb, int dpb) {
  const size_t f = (size_t(4) * 2 * nb * dpb * 4 + 15) & ~size_t(15);
  return f + size_t(4) * nb * (8 + 2 + 1);
}

hipError_t LaunchAvqEncode(const float* resid, const float* orig, int64_t n, int dim,
                           const float* cb, int nb, int dpb, double threshold, uint8_t* out,
                           hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(avq_encode_kernel, dim3(unsigned((n + 3) / 4)), dim3(64), AvqEncodeLds(nb, dpb),
                     s, resid, orig, n, dim, cb, nb, dpb, threshold, out);
  return hipGetLastError();
}

}  // namespace smx

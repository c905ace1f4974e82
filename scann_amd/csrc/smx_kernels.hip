// smx_kernels.hip — HIP kernels (gfx950 / CDNA4) of the tree-AH LUT16 query
// path.  Every float operation whose rounding the reference fixes is spelled
// with an explicit round-to-nearest intrinsic; the library is also built with
// -ffp-contract=off.
//
//   partition_scores_kernel query tokenization on MFMA f32 32x32x2: the exact
//                           fma chain of the transposed many-to-many path
//                           (many_to_many_impl.inc:522-560)
//   topl_select_kernel      exact top-L by (distance, leaf) per query
//                           (kmeans_tree_partitioner.cc:703-728)
//   lut_build_kernel        raw float LUT + uint8 fixed point
//                           (asymmetric_hashing_impl.cc:505-645)
//   pairs_* kernels         InvertCentersToSearch on the GPU
//                           (tree_ah_hybrid_residual.cc:610-622)
//   lut16_scan_kernel<K>    THE hot loop (lut16_avx2.inc:403-526): LUT16 sums
//                           on MFMA i32_32x32x32_i8 (one-hot codes x int8 LUT),
//                           fused distance + threshold + candidate emission
//   seed/tighten/final      exact top-k by the reference's total order
//                           (fast_top_neighbors.h:175-228), SOAR dedupe
//                           (internal/utils.cc:135-162), exact reorder
//                           (one_to_many_symmetric.h:373-503) and SortAndDrop
//                           (single_machine_base.cc:872-901)
#include <hip/hip_runtime.h>

#include <climits>
#include <stdint.h>

#include <algorithm>

#include "smx_internal.h"

namespace smx {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// sqrtf(FLT_EPSILON) as the reference computes it on the host
// (asymmetric_hashing_impl.cc:575): 3.4526698e-04f.
__device__ __forceinline__ float SqrtFltEps() { return __uint_as_float(0x39b504f3u); }

// Order-preserving map float -> uint32 (total order of the reference's
// comparator for non-NaN values; -0 canonicalised to +0 first).
__device__ __forceinline__ uint32_t OrderedBits(float f) {
  f = __fadd_rn(f, 0.0f);
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float FromOrdered(uint32_t o) {
  const uint32_t u = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
  return __uint_as_float(u);
}

__device__ __forceinline__ uint32_t NextPow2(uint32_t x) {
  return x <= 1 ? 1u : 1u << (32 - __clz(x - 1));
}

// Block-wide bitonic sort (ascending) of n (power of two) keys in LDS.
__device__ void BitonicSort(uint64_t* keys, uint32_t n) {
  for (uint32_t k = 2; k <= n; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t ixj = i ^ j;
        if (ixj > i) {
          const uint64_t a = keys[i], b = keys[ixj];
          const bool up = (i & k) == 0;
          if ((a > b) == up) {
            keys[i] = b;
            keys[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
}


// Exact k smallest of n keys (u64, LDS) into out[0..m) sorted ascending,
// m = min(k, n).  Keys are binned linearly on their high word between its
// min and max; the keys in bins up to the one holding the k-th are compacted
// and sorted (usually a few hundred), everything else is discarded.  Falls
// back to sorting all n keys when one bin holds too many (massive ties).
// scratch: kSelBins u32 + 256 u32.  All threads of the block must call.
constexpr uint32_t kSelBins = 2048;

__device__ uint32_t SelectSmallest(uint64_t* keys, uint32_t n, uint32_t k, uint64_t* out,
                                   uint32_t out_cap, uint32_t* hist, uint32_t* scan_buf) {
  __shared__ uint32_t s_lo[8], s_hi[8], s_bin, s_cnt;
  const uint32_t m = min(n, k);
  if (m == 0) return 0;
  uint32_t lo = 0xFFFFFFFFu, hi = 0;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t v = uint32_t(keys[i] >> 32);
    lo = min(lo, v);
    hi = max(hi, v);
  }
  for (int off = 32; off > 0; off >>= 1) {
    lo = min(lo, __shfl_xor(lo, off));
    hi = max(hi, __shfl_xor(hi, off));
  }
  const int wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) { s_lo[wid] = lo; s_hi[wid] = hi; }
  for (uint32_t b = threadIdx.x; b < kSelBins; b += blockDim.x) hist[b] = 0;
  if (threadIdx.x == 0) { s_bin = kSelBins - 1; s_cnt = 0; }
  __syncthreads();
  lo = s_lo[0];
  hi = s_hi[0];
  for (int w = 1; w < nw; ++w) { lo = min(lo, s_lo[w]); hi = max(hi, s_hi[w]); }
  const uint64_t span = uint64_t(hi - lo) + 1;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t v = uint32_t(keys[i] >> 32);
    atomicAdd(&hist[uint32_t((uint64_t(v - lo) * kSelBins) / span)], 1u);
  }
  __syncthreads();
  const uint32_t per = kSelBins / blockDim.x;
  uint32_t local = 0;
  for (uint32_t u = 0; u < per; ++u) local += hist[threadIdx.x * per + u];
  scan_buf[threadIdx.x] = local;
  __syncthreads();
  for (uint32_t off = 1; off < blockDim.x; off <<= 1) {
    const uint32_t v = threadIdx.x >= off ? scan_buf[threadIdx.x - off] : 0u;
    __syncthreads();
    scan_buf[threadIdx.x] += v;
    __syncthreads();
  }
  const uint32_t before = threadIdx.x ? scan_buf[threadIdx.x - 1] : 0u;
  if (before < m && before + local >= m) {
    uint32_t cum = before;
    for (uint32_t u = 0; u < per; ++u) {
      cum += hist[threadIdx.x * per + u];
      if (cum >= m) { s_bin = threadIdx.x * per + u; break; }
    }
  }
  __syncthreads();
  const uint32_t bsel = s_bin;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    const uint64_t key = keys[i];
    const uint32_t b = uint32_t((uint64_t(uint32_t(key >> 32) - lo) * kSelBins) / span);
    if (b <= bsel) {
      const uint32_t p = atomicAdd(&s_cnt, 1u);
      if (p < out_cap) out[p] = key;
    }
  }
  __syncthreads();
  const uint32_t c = s_cnt;
  if (c <= out_cap) {
    const uint32_t np2 = NextPow2(c);
    for (uint32_t i = c + threadIdx.x; i < np2; i += blockDim.x) out[i] = ~0ull;
    __syncthreads();
    BitonicSort(out, np2);
  } else {  // too many keys share the boundary bin: sort everything
    const uint32_t np2 = NextPow2(n);
    for (uint32_t i = n + threadIdx.x; i < np2; i += blockDim.x) keys[i] = ~0ull;
    __syncthreads();
    BitonicSort(keys, np2);
    for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) out[i] = keys[i];
    __syncthreads();
  }
  return m;
}

// ---------------------------------------------------------------------------
// Query tokenization on the f32 MFMA.  v_mfma_f32_32x32x2_f32 computes
// D = fma(a_k1, b_k1, fma(a_k0, b_k0, C)) with one rounding per step, so
// feeding A = -q, B = c (or 2c) two dims per instruction, d ascending,
// reproduces the reference's transposed many-to-many chain
// acc <- fma(-q_d, c_d, acc) bit for bit (many_to_many_impl.inc:544-556).
// One wave = 32 queries x 32 centers.  Odd dims pad with (-0) * (+0), which
// leaves every accumulator (zeros included) unchanged.
// ---------------------------------------------------------------------------
typedef float v16f __attribute__((ext_vector_type(16)));

// A 256-thread block computes 64 queries x 64 centers (wave w: query half
// w & 1, center half w >> 1); the operands are staged in LDS 32 dims at a time
// with coalesced row loads (-q and c or 2c, zero-padded past dim), so every
// MFMA reads its two floats per lane from LDS instead of a strided global row.
constexpr int kPartTile = 64, kPartChunk = 32;

__global__ void __launch_bounds__(256) partition_scores_kernel(
    const float* __restrict__ queries, int nq, int dim, const float* __restrict__ centers,
    const float* __restrict__ cnorm, int nl, int metric, float* __restrict__ scores) {
  __shared__ float qs[kPartTile][kPartChunk + 1];
  __shared__ float cs[kPartTile][kPartChunk + 1];
  __shared__ float qn[kPartTile];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, k = lane >> 5;
  const int qt = blockIdx.x * kPartTile, ct = blockIdx.y * kPartTile;
  const int qw = (wave & 1) * 32, cw = (wave >> 1) * 32;   // this wave's sub-tile
  const int q0 = qt + qw, c0 = ct + cw;
  const int cb = min(c0 + r, nl - 1);     // B column (center) of this lane
  v16f acc;
  if (metric == 1) {
    if (tid < kPartTile) {
      double s = 0.0;
      const float* qq = queries + size_t(min(qt + tid, nq - 1)) * dim;
      for (int d = 0; d < dim; ++d) s += double(qq[d]) * double(qq[d]);
      qn[tid] = float(s);
    }
    __syncthreads();
    // C layout: col = lane & 31 (center), row = (i&3) + 8*(i>>2) + 4*(lane>>5)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = (i & 3) + 8 * (i >> 2) + 4 * k;
      acc[i] = __fadd_rn(cnorm[cb], qn[qw + row]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
  }
  const float cscale = metric == 1 ? 2.0f : 1.0f;
  for (int d0 = 0; d0 < dim; d0 += kPartChunk) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < (kPartTile * kPartChunk) / 256; ++i) {
      const int e = tid + i * 256;
      const int row = e / kPartChunk, col = e % kPartChunk, d = d0 + col;
      const float* qrow = queries + size_t(min(qt + row, nq - 1)) * dim;
      const float* crow = centers + size_t(min(ct + row, nl - 1)) * dim;
      qs[row][col] = d < dim ? -qrow[d] : -0.0f;
      cs[row][col] = d < dim ? __fmul_rn(crow[d], cscale) : 0.0f;
    }
    __syncthreads();
    const int steps = min(kPartChunk, ((dim - d0) + 1) & ~1);
    for (int s = 0; s < steps; s += 2)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(qs[qw + r][s + k], cs[cw + r][s + k], acc, 0, 0,
                                                 0);
  }
  const int col = c0 + r;
  if (col < nl) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = q0 + (i & 3) + 8 * (i >> 2) + 4 * k;
      if (row < nq) scores[size_t(row) * nl + col] = acc[i];
    }
  }
}

// Exact top-L per query by (score, center index) from the score matrix.
__global__ void __launch_bounds__(256) topl_select_kernel(const float* __restrict__ scores, int nl,
                                                          int L, uint32_t kcap,
                                                          int32_t* __restrict__ out_leaf,
                                                          float* __restrict__ out_dist) {
  extern __shared__ uint64_t lds64[];
  uint64_t* keys = lds64;
  uint64_t* sel = keys + kcap;
  const uint32_t selcap = max(2048u, 2 * NextPow2(uint32_t(L)));
  uint32_t* hist = reinterpret_cast<uint32_t*>(sel + selcap);
  uint32_t* scan_buf = hist + kSelBins;
  const int qi = blockIdx.x;
  for (int c = threadIdx.x; c < nl; c += blockDim.x)
    keys[c] = (uint64_t(OrderedBits(scores[size_t(qi) * nl + c])) << 32) | uint32_t(c);
  __syncthreads();
  const uint32_t m = SelectSmallest(keys, uint32_t(nl), uint32_t(L), sel, selcap, hist, scan_buf);
  for (int i = threadIdx.x; i < L; i += blockDim.x) {
    const bool has = uint32_t(i) < m;
    out_leaf[size_t(qi) * L + i] = has ? int32_t(sel[i] & 0xFFFFFFFFu) : -1;
    out_dist[size_t(qi) * L + i] = has ? FromOrdered(uint32_t(sel[i] >> 32)) : __int_as_float(0x7fc00000);
  }
}

// Above this many leaves the score row is selected from global memory.
constexpr int kLdsSelectLeaves = 16384;

// Exact top-L per query when the score row does not fit in LDS (more than
// kLdsSelectLeaves leaves, e.g. Deep1B's 50000): four 8-bit radix passes over
// the row in global memory (L2-resident, nl*4 bytes) find the ordered bits T
// of the L-th smallest score and how many of the L are ties at T; the keys
// below T plus the lowest-index ties (the reference's (distance, index)
// order) are compacted into LDS and bitonic-sorted.  Same output as
// topl_select_kernel.  LDS: lcap = NextPow2(min(L, nl)) u64 keys.
__global__ void __launch_bounds__(256) topl_select_global_kernel(const float* __restrict__ scores,
                                                                 int nl, int L, uint32_t lcap,
                                                                 int32_t* __restrict__ out_leaf,
                                                                 float* __restrict__ out_dist) {
  extern __shared__ uint64_t lds64[];
  uint64_t* sel = lds64;
  __shared__ uint32_t hist[256];
  __shared__ uint32_t s_prefix, s_need, s_eq, s_cnt, s_tie;
  __shared__ uint32_t s_wave[4];
  const int qi = blockIdx.x;
  const float* row = scores + size_t(qi) * nl;
  const uint32_t m = min(uint32_t(L), uint32_t(nl));
  if (threadIdx.x == 0) { s_prefix = 0; s_need = m; s_cnt = 0; s_tie = 0; }
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    hist[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t prefix = s_prefix;
    for (int c = threadIdx.x; c < nl; c += blockDim.x) {
      const uint32_t v = OrderedBits(row[c]);
      if (pass == 0 || (v >> (shift + 8)) == (prefix >> (shift + 8)))
        atomicAdd(&hist[(v >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 64) {   // wave 0: inclusive scan of 4 bins per lane
      const int lane = threadIdx.x;
      const uint32_t h0 = hist[4 * lane], h1 = hist[4 * lane + 1], h2 = hist[4 * lane + 2],
                     h3 = hist[4 * lane + 3];
      uint32_t incl = h0 + h1 + h2 + h3;
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = __shfl_up(incl, off);
        if (lane >= off) incl += t;
      }
      const uint32_t excl = incl - (h0 + h1 + h2 + h3);
      const uint32_t need = s_need;
      if (excl < need && incl >= need) {
        uint32_t cum = excl, b = 4 * lane;
        const uint32_t h[4] = {h0, h1, h2, h3};
        int u = 0;
        while (cum + h[u] < need) { cum += h[u]; ++u; }
        b += u;
        s_prefix = prefix | (b << shift);
        s_need = need - cum;   // rank of the L-th key among the keys in bin b
        s_eq = h[u];
      }
    }
    __syncthreads();
  }
  const uint32_t T = s_prefix, need = s_need, eq = s_eq;   // need ties at T of eq
  const bool all_ties = need == eq;
  for (int c = threadIdx.x; c < nl; c += blockDim.x) {
    const uint32_t v = OrderedBits(row[c]);
    if (v < T || (all_ties && v == T)) sel[atomicAdd(&s_cnt, 1u)] = (uint64_t(v) << 32) | uint32_t(c);
  }
  if (!all_ties) {   // only the `need` lowest-index ties: ordered chunk scan
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int base = 0; base < nl; base += blockDim.x) {
      const int c = base + threadIdx.x;
      const bool is_eq = c < nl && OrderedBits(row[c]) == T;
      const uint64_t bal = __ballot(is_eq);
      if (lane == 0) s_wave[wid] = uint32_t(__popcll(bal));
      __syncthreads();
      uint32_t before = s_tie;
      for (int w = 0; w < wid; ++w) before += s_wave[w];
      before += uint32_t(__popcll(bal & ((1ull << lane) - 1ull)));
      if (is_eq && before < need) sel[atomicAdd(&s_cnt, 1u)] = (uint64_t(T) << 32) | uint32_t(c);
      __syncthreads();
      if (threadIdx.x == 0) s_tie += s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
      __syncthreads();
      if (s_tie >= need) break;
    }
  }
  __syncthreads();
  for (uint32_t i = m + threadIdx.x; i < lcap; i += blockDim.x) sel[i] = ~0ull;
  __syncthreads();
  BitonicSort(sel, lcap);
  for (int i = threadIdx.x; i < L; i += blockDim.x) {
    const bool has = uint32_t(i) < m;
    out_leaf[size_t(qi) * L + i] = has ? int32_t(sel[i] & 0xFFFFFFFFu) : -1;
    out_dist[size_t(qi) * L + i] = has ? FromOrdered(uint32_t(sel[i] >> 32)) : __int_as_float(0x7fc00000);
  }
}

// ---------------------------------------------------------------------------
// LUT build: raw[b][c] = -(fl(q0*c0) + fl(q1*c1)) (dot) or
// fl(t0*t0) + fl(t1*t1), t = q - c (squared L2); multiplier
// 127 / max(sqrt(FLT_EPSILON), max|raw|); int8 = round(raw * m) (the uint8
// table minus its bias 128); inv = (float)(1.0/(double)m) for residual
// indexes (lut16_avx2.inc:427-430), 1.0f/m otherwise (querying.h:450-454).
// LUT rows are padded to 2*K blocks with zeros.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) lut_build_kernel(
    const float* __restrict__ queries, int dim, const float* __restrict__ codebook,
    int nb, int dpb, int padded_blocks, int metric, int residual,
    int8_t* __restrict__ lut, float* __restrict__ mult, float* __restrict__ inv,
    uint8_t* __restrict__ lut_u8, LutInit init) {
  __shared__ float raw[kMaxBlocks * 16];
  __shared__ float red[256];
  {
    // the search's per-call state, reset here instead of by separate memset
    // nodes: counters and candidate counts to 0, thresholds to "open"
    const uint32_t gt = blockIdx.x * blockDim.x + threadIdx.x, gs = gridDim.x * blockDim.x;
    for (uint32_t i = gt; i < init.n_counters; i += gs) init.counters[i] = 0u;
    for (uint32_t i = gt; i < init.n_cand; i += gs) init.cand_count[i] = 0u;
    for (uint32_t i = gt; i < init.n_tau; i += gs) init.tau[i] = kNoThreshold;
  }
  const int qi = blockIdx.x;
  const float* q = queries + size_t(qi) * dim;
  const int nent = nb * 16;
  const int last = dim - dpb * (nb - 1);
  float local_max = 0.0f;
  for (int e = threadIdx.x; e < nent; e += blockDim.x) {
    const int b = e >> 4, c = e & 15;
    const int nd = (b == nb - 1) ? last : dpb;
    const float* qb = q + size_t(b) * dpb;
    const float* cb = codebook + (size_t(b) * 16 + c) * dpb;
    float v;
    if (metric == 0) {
      float s = __fmul_rn(qb[0], cb[0]);
      for (int i = 1; i < nd; ++i) s = __fadd_rn(s, __fmul_rn(qb[i], cb[i]));
      v = -s;
    } else {
      float t = __fsub_rn(qb[0], cb[0]);
      float s = __fmul_rn(t, t);
      for (int i = 1; i < nd; ++i) {
        const float u = __fsub_rn(qb[i], cb[i]);
        s = __fadd_rn(s, __fmul_rn(u, u));
      }
      v = s;
    }
    raw[e] = v;
    local_max = fmaxf(local_max, fabsf(v));
  }
  red[threadIdx.x] = local_max;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  const float m = __fdiv_rn(127.0f, fmaxf(SqrtFltEps(), red[0]));
  const int tot = padded_blocks * 16;
  for (int e = threadIdx.x; e < tot; e += blockDim.x) {
    int8_t v8 = 0;
    if (e < nent) {
      const float r = roundf(__fmul_rn(raw[e], m));
      v8 = int8_t(int(r));
      if (lut_u8) lut_u8[size_t(qi) * nent + e] = uint8_t(int(r) + 128);
    }
    lut[size_t(qi) * tot + e] = v8;
  }
  if (threadIdx.x == 0) {
    mult[qi] = m;
    inv[qi] = residual ? float(1.0 / double(m)) : __fdiv_rn(1.0f, m);
  }
}

// Work items split a leaf's 32-datapoint tiles into chunks of at most
// chunk_tiles so that no single wave (or block) owns a whole large leaf.
__device__ __forceinline__ uint32_t LeafChunks(uint32_t n, uint32_t chunk_tiles) {
  const uint32_t tiles = (n + 31u) / 32u;
  return tiles == 0 ? 1u : (tiles + chunk_tiles - 1) / chunk_tiles;
}

// ---------------------------------------------------------------------------
// Invert (query -> leaves) into (leaf -> queries) and cut every leaf's query
// list into 32-query work items, listed largest leaf first (longest items
// dequeued first).
// ---------------------------------------------------------------------------
// Block-local counting: every block histograms kPairsPerBlock pairs in LDS and
// publishes one count per (block, leaf) -- no contended global atomics.
constexpr int kPairsPerBlock = 4096;
constexpr int kLeafRange = 16384;   // leaves per LDS counter range (64 KiB)

__global__ void __launch_bounds__(256) pairs_count_kernel(const int32_t* __restrict__ topl_leaf,
                                                          int n, int nl,
                                                          uint32_t* __restrict__ block_cnt,
                                                          uint32_t* __restrict__ cnt) {
  extern __shared__ uint32_t hist[];
  // blockIdx.y selects a range of kLeafRange leaves (indexes whose per-leaf
  // counters exceed LDS, e.g. 50000 leaves)
  const int l0 = blockIdx.y * kLeafRange, nr = min(kLeafRange, nl - l0);
  for (int l = threadIdx.x; l < nr; l += blockDim.x) hist[l] = 0;
  __syncthreads();
  const int beg = blockIdx.x * kPairsPerBlock, end = min(n, beg + kPairsPerBlock);
  for (int i = beg + threadIdx.x; i < end; i += blockDim.x) {
    const int leaf = topl_leaf[i] - l0;
    if (leaf >= 0 && leaf < nr) atomicAdd(&hist[leaf], 1u);
  }
  __syncthreads();
  uint32_t* bc = block_cnt + size_t(blockIdx.x) * nl + l0;
  for (int l = threadIdx.x; l < nr; l += blockDim.x) {
    const uint32_t c = hist[l];
    bc[l] = c;
    if (c) atomicAdd(&cnt[l0 + l], c);
  }
}

// Exclusive prefix over blocks for every leaf: block b's first slot in leaf l.
__global__ void pairs_block_offsets_kernel(uint32_t* __restrict__ block_cnt, int nblocks, int nl) {
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= nl) return;
  uint32_t run = 0;
  for (int b = 0; b < nblocks; ++b) {
    const uint32_t c = block_cnt[size_t(b) * nl + l];
    block_cnt[size_t(b) * nl + l] = run;
    run += c;
  }
}

__global__ void __launch_bounds__(1024) pairs_scan_kernel(const uint32_t* __restrict__ cnt,
                                                          const uint32_t* __restrict__ order,
                                                          const uint32_t* __restrict__ leaf_size,
                                                          int nl, int nb, uint32_t chunk_tiles,
                                                          uint32_t qpi,
                                                          uint32_t* __restrict__ pair_off,
                                                          uint32_t* __restrict__ tile_prefix,
                                                          uint32_t* __restrict__ totals,
                                                          unsigned long long* __restrict__ code_bytes,
                                                          uint2* __restrict__ work,
                                                          uint32_t* __restrict__ block_cnt,
                                                          int fused_blocks) {
  // small trees: the per-leaf exclusive prefix over the counting blocks
  // (pairs_block_offsets_kernel) is done here, 8 loads in flight per step
  for (int l = threadIdx.x; l < nl && fused_blocks > 0; l += blockDim.x) {
    uint32_t run = 0;
    for (int b0 = 0; b0 < fused_blocks; b0 += 8) {
      uint32_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = b0 + u < fused_blocks ? block_cnt[size_t(b0 + u) * nl + l] : 0u;
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (b0 + u < fused_blocks) {
          block_cnt[size_t(b0 + u) * nl + l] = run;
          run += v[u];
        }
    }
  }
  __shared__ uint32_t s_pairs[1024];
  __shared__ uint32_t s_tiles[1024];
  __shared__ unsigned long long s_bytes[1024];
  const int per = (nl + blockDim.x - 1) / blockDim.x;
  const int beg = threadIdx.x * per;
  const int end = min(nl, beg + per);
  uint32_t sp = 0, st = 0, sit = 0;
  unsigned long long sb = 0;
  for (int p = beg; p < end; ++p) {
    const uint32_t leaf = order[p];
    const uint32_t c = cnt[leaf];
    sp += c;
    st += ((c + qpi - 1) / qpi) * LeafChunks(leaf_size[leaf], chunk_tiles);
    sit += ((c + kQueriesPerTile - 1) / kQueriesPerTile) * ((leaf_size[leaf] + 31u) / 32u);
    // algorithmic code bytes: 16 * B * ceil(n / 32) per (query, leaf) pair
    sb += 16ull * nb * ((leaf_size[leaf] + 31u) / 32u) * c;
  }
  s_pairs[threadIdx.x] = sp;
  s_tiles[threadIdx.x] = st;
  s_bytes[threadIdx.x] = sb;
  __syncthreads();
  for (int off = int(blockDim.x) / 2; off > 0; off >>= 1) {
    if (int(threadIdx.x) < off) s_bytes[threadIdx.x] += s_bytes[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) code_bytes[0] = s_bytes[0];
  __syncthreads();
  s_tiles[threadIdx.x] = sit;   // reuse: item-tiles (MFMA tile count) reduction
  __syncthreads();
  for (int off = int(blockDim.x) / 2; off > 0; off >>= 1) {
    if (int(threadIdx.x) < off) s_tiles[threadIdx.x] += s_tiles[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) totals[2] = s_tiles[0];
  __syncthreads();
  s_tiles[threadIdx.x] = st;
  for (int off = 1; off < int(blockDim.x); off <<= 1) {
    uint32_t a = 0, b = 0;
    if (int(threadIdx.x) >= off) {
      a = s_pairs[threadIdx.x - off];
      b = s_tiles[threadIdx.x - off];
    }
    __syncthreads();
    s_pairs[threadIdx.x] += a;
    s_tiles[threadIdx.x] += b;
    __syncthreads();
  }
  uint32_t rp = threadIdx.x ? s_pairs[threadIdx.x - 1] : 0;
  uint32_t rt = threadIdx.x ? s_tiles[threadIdx.x - 1] : 0;
  for (int p = beg; p < end; ++p) {
    const uint32_t leaf = order[p];
    const uint32_t c = cnt[leaf];
    pair_off[leaf] = rp;
    tile_prefix[p] = rt;
    rp += c;
    // this leaf's work items: (leaf, query tile << 16 | dp chunk)
    const uint32_t chunks = LeafChunks(leaf_size[leaf], chunk_tiles);
    const uint32_t items = ((c + qpi - 1) / qpi) * chunks;
    for (uint32_t u = 0; u < items; ++u)
      work[rt + u] = make_uint2(leaf, ((u / chunks) << 16) | (u % chunks));
    rt += items;
  }
  if (threadIdx.x == blockDim.x - 1) {
    tile_prefix[nl] = s_tiles[blockDim.x - 1];
    totals[0] = s_pairs[blockDim.x - 1];
    totals[1] = s_tiles[blockDim.x - 1];
  }
}

__global__ void __launch_bounds__(256) pairs_scatter_kernel(
    const int32_t* __restrict__ topl_leaf, const float* __restrict__ topl_dist, int n, int L, int nl,
    const uint32_t* __restrict__ pair_off, const uint32_t* __restrict__ block_off,
    uint32_t* __restrict__ pair_q, float* __restrict__ pair_bias) {
  extern __shared__ uint32_t fill[];
  const int l0 = blockIdx.y * kLeafRange, nr = min(kLeafRange, nl - l0);
  for (int l = threadIdx.x; l < nr; l += blockDim.x) fill[l] = 0;
  __syncthreads();
  const uint32_t* bo = block_off + size_t(blockIdx.x) * nl;
  const int beg = blockIdx.x * kPairsPerBlock, end = min(n, beg + kPairsPerBlock);
  for (int i = beg + threadIdx.x; i < end; i += blockDim.x) {
    const int leaf = topl_leaf[i];
    if (leaf < l0 || leaf >= l0 + nr) continue;
    const uint32_t pos = pair_off[leaf] + bo[leaf] + atomicAdd(&fill[leaf - l0], 1u);
    pair_q[pos] = uint32_t(i / L);
    pair_bias[pos] = topl_dist[i];
  }
}

// ---------------------------------------------------------------------------
// LUT16 scan on MFMA.
//
// A 256-thread block owns a work item = (leaf, 32 queries of that leaf, a
// chunk of the leaf's 32-datapoint tiles).  For every tile it computes the
// 32x32 matrix of LUT16 sums
//     S[dp][q] = sum_b int8LUT_q[b][code(dp, b)]
// as K = ceil(B/2) MFMA i32_32x32x32_i8 steps: A = one-hot codes (row = dp,
// 16 bytes per lane-half = one block's 16 centers), B = the queries' int8
// LUT rows (staged in LDS once per item).  The i32 sums are exact
// (|S| <= 127*B).  Lane (c, h) of the accumulator holds 16 datapoints of
// query c; a datapoint can only pass when S <= amax_c (the largest sum whose
// distance can pass the query's threshold: d is monotone in S), and only
// those are converted:
//     d = fl(fl(float(S) * inv_q) + bias_{q,leaf})
// and emitted as (ordered(d) << 32 | tie) when that key <= the threshold key.
// ---------------------------------------------------------------------------
// 16-byte one-hot of nibble t (byte t = 1): 1 << 8(t mod 8) in the 64-bit
// half selected by bit 3.  `sh` = 8 * t (bits 3..6), so the 64-bit shift
// uses sh & 63 and bit 6 of sh picks the half.
__device__ __forceinline__ v4i OneHot16(uint32_t sh) {
  const uint64_t x = 1ull << (sh & 63u);
  const uint32_t lo = uint32_t(x), hi = uint32_t(x >> 32);
  const uint32_t m = 0u - ((sh >> 6) & 1u);  // all ones when t >= 8
  v4i r;
  r[0] = int(lo & ~m);
  r[1] = int(hi & ~m);
  r[2] = int(lo & m);
  r[3] = int(hi & m);
  return r;
}

__device__ __forceinline__ float DistOf(int s, float inv, float bias) {
  return __fadd_rn(__fmul_rn(float(s), inv), bias);
}

// Largest sum in [lo, hi] whose distance is <= td (lo - 1 if none).
__device__ int SumLimit(float td, float inv, float bias, int lo, int hi) {
  if (!(DistOf(lo, inv, bias) <= td)) return lo - 1;
  if (DistOf(hi, inv, bias) <= td) return hi;
  while (hi - lo > 1) {
    const int mid = lo + ((hi - lo) >> 1);
    if (DistOf(mid, inv, bias) <= td) lo = mid; else hi = mid;
  }
  return lo;
}

template <int K>
__device__ __forceinline__ v16i TileSums(const uint32_t* codes, const v4i* frag) {
  v16i acc = {0};
#pragma unroll
  for (int s = 0; s < K; ++s) {
    const int sh = (s & 7) * 4;
    const uint32_t w = codes[s >> 3];
    const uint32_t e8 = sh >= 3 ? ((w >> (sh - 3)) & 0x78u) : ((w << 3) & 0x78u);
    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(OneHot16(e8), frag[s], acc, 0, 0, 0);
  }
  return acc;
}

template <int K>
__device__ __forceinline__ void LoadCodes(const uint8_t* p, uint32_t* codes) {
  constexpr int NW = ((((K + 1) / 2) + 3) / 4);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(p);
  if constexpr (NW == 4) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    codes[0] = v.x; codes[1] = v.y; codes[2] = v.z; codes[3] = v.w;
  } else if constexpr (NW == 2) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    codes[0] = v.x; codes[1] = v.y;
  } else {
#pragma unroll
    for (int i = 0; i < NW; ++i) codes[i] = w[i];
  }
}

// ---------------------------------------------------------------------------
// Per-query threshold from the query's first `seed` leaves (one block per
// query).  Every datapoint there is scored with the int8 LUT in LDS; the
// exact k'-th smallest of those distances bounds the final k'-th from above
// (the main pass rescans those leaves and every stored key is a genuine
// candidate), so the threshold key admits every datapoint at that distance.
// The seed datapoints are numbered across the seed leaves (a wave prefix sum
// of their sizes), thread t scores numbers t, t+256, ... into registers (at
// most kSeedCap per query: a subset's k'-th is still a bound), and rounds of
// a 256-bin histogram over the order-preserving bits narrow down to the
// exact k'-th value.
// ---------------------------------------------------------------------------
constexpr int kSeedPerThread = 32;
constexpr uint32_t kSeedCap = 256u * kSeedPerThread;
constexpr int kSeedMaxLeaves = 64;   // one wave of leaf slots

// Inclusive block scan of one value per thread (256 threads).
__device__ __forceinline__ uint32_t BlockInclusiveScan256(uint32_t v, uint32_t* wsum) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t t = uint32_t(__shfl_up(int(v), off));
    if (lane >= off) v += t;
  }
  if (lane == 63) wsum[wid] = v;
  __syncthreads();
  for (int w = 0; w < wid; ++w) v += wsum[w];
  return v;
}

template <int K>
__global__ void __launch_bounds__(256) seed_tau_kernel(SeedArgs a) {
  constexpr int NW = ((((K + 1) / 2) + 3) / 4);
  constexpr int W = 4 * NW;
  constexpr int U = 4;   // datapoints whose code loads are in flight together
  __shared__ int8_t lut[2 * K * 16];
  __shared__ uint32_t hist[256];
  __shared__ uint32_t s_start[kSeedMaxLeaves + 1];
  __shared__ uint64_t s_tile0[kSeedMaxLeaves];
  __shared__ float s_bias[kSeedMaxLeaves];
  __shared__ uint32_t wsum[4], s_lo[4], s_hi[4], s_bin, s_below;
  const int qi = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int e = tid; e < 2 * K * 16; e += 256) lut[e] = a.lut[size_t(qi) * 2 * K * 16 + e];
  const float inv = a.inv[qi];
  const int nseed = min(a.seed, min(a.L, kSeedMaxLeaves));
  if (wid == 0) {
    // seed leaves and the exclusive prefix of their sizes (lanes >= nseed add 0)
    const int leaf = lane < nseed ? a.topl_leaf[size_t(qi) * a.L + lane] : -1;
    const uint32_t sz = leaf >= 0 ? a.leaf_size[leaf] : 0u;
    uint32_t inc = sz;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t t = uint32_t(__shfl_up(int(inc), off));
      if (lane >= off) inc += t;
    }
    s_start[lane] = inc - sz;
    s_tile0[lane] = leaf >= 0 ? a.tile_off[leaf] : 0ull;
    s_bias[lane] = (leaf >= 0 && a.residual) ? a.topl_dist[size_t(qi) * a.L + lane] : 0.0f;
    if (lane == 63) s_start[kSeedMaxLeaves] = inc;
  }
  __syncthreads();
  const uint32_t total = min(s_start[kSeedMaxLeaves], kSeedCap);
  const uint32_t kk = uint32_t(a.kk);
  if (kk == 0 || total < kk) return;   // no bound: the threshold stays open

  uint32_t vals[kSeedPerThread];
  int r = 0;   // seed leaf of this thread's current number (numbers only grow)
#pragma unroll
  for (int i0 = 0; i0 < kSeedPerThread; i0 += U) {
    if (uint32_t(i0) * 256u < total) {   // block-uniform
      uint32_t c0[U][NW], c1[U][NW];
      int ru[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t g = min(uint32_t(tid) + 256u * uint32_t(i0 + u), total - 1);
        while (g >= s_start[r + 1]) ++r;
        ru[u] = r;
        const uint32_t dp = g - s_start[r];
        const uint8_t* t0 = a.tiles + ((s_tile0[r] + (dp >> 5)) * 64 + (dp & 31)) * W;
        LoadCodes<K>(t0, c0[u]);
        LoadCodes<K>(t0 + 32 * W, c1[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        int acc = 0;
#pragma unroll
        for (int s = 0; s < K; ++s) {
          const uint32_t n0 = (c0[u][s >> 3] >> ((s & 7) * 4)) & 15u;
          const uint32_t n1 = (c1[u][s >> 3] >> ((s & 7) * 4)) & 15u;
          acc += int(lut[(2 * s) * 16 + n0]) + int(lut[(2 * s + 1) * 16 + n1]);
        }
        const uint32_t g = uint32_t(tid) + 256u * uint32_t(i0 + u);
        vals[i0 + u] = g < total ? OrderedBits(DistOf(acc, inv, s_bias[ru[u]])) : 0xFFFFFFFFu;
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) vals[i0 + u] = 0xFFFFFFFFu;   // no datapoint
    }
  }
  // range of the values, then histogram rounds down to the kk-th value
  uint32_t lo = 0xFFFFFFFFu, hi = 0;
#pragma unroll
  for (int i = 0; i < kSeedPerThread; ++i)
    if (vals[i] != 0xFFFFFFFFu) {
      lo = min(lo, vals[i]);
      hi = max(hi, vals[i]);
    }
  for (int off = 32; off > 0; off >>= 1) {
    lo = min(lo, uint32_t(__shfl_xor(int(lo), off)));
    hi = max(hi, uint32_t(__shfl_xor(int(hi), off)));
  }
  if (lane == 0) { s_lo[wid] = lo; s_hi[wid] = hi; }
  __syncthreads();
  lo = min(min(s_lo[0], s_lo[1]), min(s_lo[2], s_lo[3]));
  hi = max(max(s_hi[0], s_hi[1]), max(s_hi[2], s_hi[3]));
  uint32_t below = 0;   // values smaller than lo
  while (lo < hi) {     // block-uniform; each round shrinks [lo, hi] 256-fold
    const uint64_t span = uint64_t(hi - lo) + 1;
    hist[tid] = 0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kSeedPerThread; ++i) {
      const uint32_t v = vals[i];
      if (v >= lo && v <= hi) atomicAdd(&hist[uint32_t((uint64_t(v - lo) * 256u) / span)], 1u);
    }
    __syncthreads();
    const uint32_t hv = hist[tid];
    const uint32_t inc = BlockInclusiveScan256(hv, wsum);
    if (below + inc - hv < kk && below + inc >= kk) {
      s_bin = uint32_t(tid);
      s_below = below + inc - hv;
    }
    __syncthreads();
    const uint32_t b = s_bin;
    below = s_below;
    // values of bin b: [lo + ceil(b*span/256), lo + ceil((b+1)*span/256) - 1]
    const uint32_t blo = lo + uint32_t((uint64_t(b) * span + 255u) / 256u);
    const uint32_t bhi = lo + uint32_t((uint64_t(b + 1) * span + 255u) / 256u) - 1u;
    lo = blo;
    hi = bhi;
    __syncthreads();   // hist, wsum and s_bin are rewritten by the next round
  }
  if (tid == 0) {
    const uint64_t t = (uint64_t(hi) << 32) | 0xFFFFFFFFull;
    if (t < a.tau_key[qi]) a.tau_key[qi] = t;
  }
}


// K MFMAs of one tile.  The one-hot A fragments come from a 16-entry LDS
// table (oh_tab[t] = 16 bytes with byte t = 1): per MFMA one nibble
// extraction and two ds_read_b128, both conflict-free (the table spans the 64
// banks exactly; a step's B rows are 1 KiB contiguous per wave).  Both are
// read R steps ahead of their MFMA, and a full scheduling barrier closes each
// step so the compiler cannot collapse the ring.
constexpr int kRing = 4;
template <int K, int Q, int R = kRing>
__device__ __forceinline__ v16i TileMfma(const uint32_t* codes, const v4i* lut, int off,
                                         const v4i* oh_tab) {
  asm volatile("" : "+v"(off));
  v4i b[R], o[R];
#pragma unroll
  for (int p = 0; p < R; ++p)
    if (p < K) {
      b[p] = lut[2 * p * Q + off];
      o[p] = oh_tab[(codes[p >> 3] >> ((p & 7) * 4)) & 15u];
    }
  v16i acc = v16i{0};
#pragma unroll
  for (int s = 0; s < K; ++s) {
    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(o[s % R], b[s % R], acc, 0, 0, 0);
    if (s + R < K) {
      const int t = s + R;
      b[s % R] = lut[2 * t * Q + off];
      o[s % R] = oh_tab[(codes[t >> 3] >> ((t & 7) * 4)) & 15u];
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  return acc;
}

// ---------------------------------------------------------------------------
// The scan kernel.  Persistent blocks claim items from a work counter
// (largest leaves first).  Per item: the 32 queries' parameters and LUT rows
// go to LDS ([row][query] x 16 B), the 4 waves take the chunk's tiles
// round-robin (code tile j+4 prefetched while tile j computes).  The
// threshold epilogue is split in two: in the tile loop a lane whose 16-sum
// minimum passes only appends its sums (packed int16) and a tag to its wave's
// LDS hit list; drain() runs the per-element test, the key and the exact
// threshold compare lane-parallel over the hits, once per item (or when the
// list fills), and stages survivors per query in LDS: one global atomic per
// query per item.
// ABL = 4: timing ablation without the epilogue (results invalid).
// ---------------------------------------------------------------------------
constexpr int kHitsPerWave = 64;   // >= 64: a tile may add a hit per lane right after a drain
constexpr int kQStageHits = 16;

template <int K, int ABL = 0>
__global__ void __launch_bounds__(256, (K <= 25 ? 4 : 3)) lut16_scan_kernel(ScanArgs a) {
  constexpr int NW = ((((K + 1) / 2) + 3) / 4);
  constexpr int W = 4 * NW;
  constexpr int Q = 32, NWV = 4, NT = 256, HW = kHitsPerWave, S = kQStageHits;
  constexpr int ROWS = 2 * K * Q, PER = (ROWS + NT - 1) / NT;
  __shared__ v4i lut_s[ROWS];
  __shared__ uint4 hsum[NWV][HW][2];     // 16 sums as int16 pairs
  __shared__ uint32_t hmeta[NWV][HW];    // tile << 6 | lane
  __shared__ uint64_t qstage[Q * S];
  __shared__ uint32_t qcnt[Q], q_slot[Q], q_id[Q];
  __shared__ float q_bias[Q], q_inv[Q];
  __shared__ int q_amax[Q];
  __shared__ uint64_t q_T[Q];
  __shared__ uint32_t s_w;
  __shared__ v4i oh_tab[16];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int c = lane & 31;
  const int h = lane >> 5;
  if (tid < 16) {
    v4i t = {0, 0, 0, 0};
    t[tid >> 2] = int(1u << (8 * (tid & 3)));
    oh_tab[tid] = t;
  }
  const uint32_t total = a.tile_prefix[a.nl];
  const int smin = -128 * a.nb, smax = 128 * a.nb;
  for (;;) {
    if (tid == 0) s_w = atomicAdd(a.work_counter, 1u);
    if (tid < Q) qcnt[tid] = 0;
    __syncthreads();
    const uint32_t w = s_w;
    if (w >= total) break;
    const uint2 item = a.work[w];
    const int leaf = int(item.x);
    const uint32_t t = item.y >> 16;
    const uint32_t chunk = item.y & 0xFFFFu;
    const uint32_t pbeg = a.pair_off[leaf] + t * uint32_t(Q);
    const int nvalid = int(min(uint32_t(Q), a.pair_off[leaf] + a.leaf_count[leaf] - pbeg));
    // this thread's query slot is fixed (NT is a multiple of Q): one id load
    const uint32_t qid = a.pair_q[pbeg + uint32_t(c < nvalid ? c : 0)];
    if (tid < Q) {
      const bool v = tid < nvalid;
      const float bias = a.residual ? a.pair_bias[pbeg + uint32_t(v ? tid : 0)] : 0.0f;
      const float inv = a.inv[qid];
      const uint64_t T = a.tau_key[qid];
      q_id[tid] = qid;
      q_bias[tid] = bias;
      q_inv[tid] = inv;
      q_T[tid] = T;
      q_amax[tid] = !v ? smin - 1
                  : (T == kNoThreshold) ? smax
                  : SumLimit(FromOrdered(uint32_t(T >> 32)), inv, bias, smin, smax);
    }
    {
      // LUT rows of the 32 queries into LDS ([row][query] x 16 B); the loads
      // are unconditional (clamped row) so they are all in flight together
      const v4i* src = reinterpret_cast<const v4i*>(a.lut) + size_t(qid) * 2 * K;
      v4i stg[PER];
#pragma unroll
      for (int i = 0; i < PER; ++i) stg[i] = src[min(tid + i * NT, ROWS - 1) / Q];
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int e = tid + i * NT;
        if (e < ROWS) lut_s[e] = stg[i];
      }
    }
    __syncthreads();
    const int amax = q_amax[c];
    const uint32_t n = a.leaf_size[leaf];
    const uint32_t ntile_leaf = (n + kDpPerTile - 1) / kDpPerTile;
    const uint32_t j0 = chunk * a.chunk_tiles;
    const uint32_t jend = min(ntile_leaf, j0 + a.chunk_tiles);
    const uint8_t* tb = a.tiles + a.tile_off[leaf] * 64ull * W + size_t(lane) * W;
    const uint64_t moff = a.member_off[leaf];
    uint32_t whits = 0;   // wave-uniform

    // lane k of the wave takes hit k: per-element test, key, exact
    // threshold compare, append to the query's LDS stage
    auto drain = [&]() {
      if (uint32_t(lane) < whits) {
        const uint32_t meta = hmeta[wave][lane];
        const uint32_t jj = meta >> 6;
        const int cc = int(meta & 31u), hh = int((meta >> 5) & 1u);
        const uint4 s0 = hsum[wave][lane][0], s1 = hsum[wave][lane][1];
        const uint32_t sw[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        const int am = q_amax[cc];
        const float iv = q_inv[cc], bs = q_bias[cc];
        const uint64_t TT = q_T[cc];
        const uint32_t qq = q_id[cc];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int sum = int(int16_t(uint16_t(sw[i >> 1] >> (16 * (i & 1)))));
          if (sum <= am) {
            const uint32_t dp = jj * kDpPerTile + (i & 3) + 8 * (i >> 2) + 4 * hh;
            const float d = DistOf(sum, iv, bs);
            const uint32_t tie = a.shift > 0 ? ((uint32_t(leaf) << a.shift) | dp)
                                             : a.members[moff + dp];
            const uint64_t key = (uint64_t(OrderedBits(d)) << 32) | tie;
            if (key <= TT) {
              const uint32_t p = atomicAdd(&qcnt[cc], 1u);
              if (p < uint32_t(S)) {
                qstage[cc * S + p] = key;
              } else {  // stage full: straight to the global list
                const uint32_t gs = atomicAdd(&a.cand_count[qq], 1u);
                if (gs < a.cap) a.cand[size_t(qq) * a.cap + gs] = key;
              }
            }
          }
        }
      }
    };

    auto body = [&](const uint32_t (&codes)[NW], uint32_t j) {
      v16i acc = TileMfma<K, Q>(codes, lut_s, h * Q + c, oh_tab);
      if (ABL & 4) {
        int x = acc[0];
#pragma unroll
        for (int i = 1; i < 16; ++i) x ^= acc[i];
        if (x == 0x7fffffff) a.cand_count[0] = x;
        return;
      }
      const uint32_t rows_left = n - j * kDpPerTile;
      if (rows_left < uint32_t(kDpPerTile)) {  // last tile of the leaf
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const uint32_t row = (i & 3) + 8 * (i >> 2) + 4 * h;
          if (row >= rows_left) acc[i] = 0x7FFF;
        }
      }
      int m = min(min(acc[0], acc[1]), acc[2]);
#pragma unroll
      for (int i = 3; i < 15; i += 2) m = min(min(m, acc[i]), acc[i + 1]);
      m = min(m, acc[15]);
      const bool hit = m <= amax;
      const uint64_t hb = __builtin_amdgcn_ballot_w64(hit);
      if (hb) {
        const uint32_t nh = uint32_t(__popcll(hb));
        if (whits + nh > uint32_t(HW)) {
          drain();
          whits = 0;
        }
        if (hit) {
          const uint32_t slot =
              whits + __builtin_amdgcn_mbcnt_hi(uint32_t(hb >> 32),
                                                __builtin_amdgcn_mbcnt_lo(uint32_t(hb), 0u));
          uint32_t pk[8];
#pragma unroll
          for (int k = 0; k < 8; ++k)
            pk[k] = (uint32_t(acc[2 * k]) & 0xFFFFu) | (uint32_t(acc[2 * k + 1]) << 16);
          hsum[wave][slot][0] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
          hsum[wave][slot][1] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
          hmeta[wave][slot] = (j << 6) | uint32_t(lane);
        }
        whits += nh;
      }
    };

    // tiles j, j+4, ... of the chunk; the prefetch of tile j+4 is
    // unconditional (clamped to the chunk's last tile) so no exec branch
    // sits around the load and the wait before the next tile is counted
    uint32_t j = j0 + wave;
    if (j < jend) {
      uint32_t codes[NW], next[NW];
      const uint32_t jl = jend - 1;
      LoadCodes<K>(tb + size_t(j) * 64 * W, codes);
      for (; j < jend; j += NWV) {
        LoadCodes<K>(tb + size_t(min(j + NWV, jl)) * 64 * W, next);
        body(codes, j);
#pragma unroll
        for (int i = 0; i < NW; ++i) codes[i] = next[i];
      }
    }
    drain();
    __syncthreads();
    // one global atomic per query slot with survivors, then the copy
    if (tid < Q) {
      const uint32_t m = min(qcnt[tid], uint32_t(S));
      q_slot[tid] = m ? atomicAdd(&a.cand_count[q_id[tid]], m) : 0u;
    }
    __syncthreads();
    for (int e = tid; e < Q * S; e += NT) {
      const int qs = e / S, u = e - qs * S;
      if (uint32_t(u) < min(qcnt[qs], uint32_t(S))) {
        const uint32_t slot = q_slot[qs] + u;
        if (slot < a.cap) a.cand[size_t(q_id[qs]) * a.cap + slot] = qstage[e];
      }
    }
    __syncthreads();
  }
}

// One-query variant for the stage entry point: raw sums of one leaf.
template <int K>
__global__ void __launch_bounds__(64) leaf_scores_kernel(const uint8_t* __restrict__ tiles,
                                                         uint64_t tile0, uint32_t n,
                                                         const int8_t* __restrict__ lut,
                                                         int32_t* __restrict__ out) {
  constexpr int NW = ((((K + 1) / 2) + 3) / 4);
  constexpr int W = 4 * NW;
  const int lane = threadIdx.x & 63;
  const int c = lane & 31;
  const int h = lane >> 5;
  v4i frag[K];
  const v4i* lrow = reinterpret_cast<const v4i*>(lut);
#pragma unroll
  for (int s = 0; s < K; ++s) frag[s] = lrow[2 * s + h];
  const uint32_t ntile = (n + 31) / 32;
  for (uint32_t j = 0; j < ntile; ++j) {
    uint32_t codes[NW];
    LoadCodes<K>(tiles + (tile0 + j) * 64ull * W + size_t(lane) * W, codes);
    const v16i acc = TileSums<K>(codes, frag);
    if (c == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t dp = j * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (dp < n) out[dp] = acc[i];
      }
    }
  }
}

// Overflow recovery: the k'-th smallest stored key is a valid (tighter)
// threshold because every stored key is a genuine candidate.
__global__ void __launch_bounds__(256) tighten_kernel(const uint64_t* __restrict__ cand,
                                                      const uint32_t* __restrict__ cand_count,
                                                      uint32_t cap, int kk,
                                                      uint64_t* __restrict__ tau_key) {
  extern __shared__ uint64_t keys[];
  const int qi = blockIdx.x;
  if (cand_count[qi] <= cap || kk <= 0) return;
  const uint32_t np2 = NextPow2(cap);
  for (uint32_t i = threadIdx.x; i < np2; i += blockDim.x)
    keys[i] = i < cap ? cand[size_t(qi) * cap + i] : ~0ull;
  __syncthreads();
  BitonicSort(keys, np2);
  if (threadIdx.x == 0 && keys[kk - 1] < tau_key[qi]) tau_key[qi] = keys[kk - 1];
}

// Exact reorder distance (A.8): 8 fused accumulators over dims 0..8m-1,
// folded (l, l+4), a 4-wide and a 2-wide (lanes 2,3) tail, then
// (s0+s2)+(s1+s3) and a fused scalar tail.
__device__ float ExactDistance(const float* __restrict__ q, const float* __restrict__ x,
                               int dim, int metric) {
  auto term = [metric](float acc, float a, float b) {
    if (metric == 0) return __fmaf_rn(-a, b, acc);
    const float t = __fsub_rn(a, b);
    return __fmaf_rn(t, t, acc);
  };
  float a8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int j = 0;
  for (; j + 8 <= dim; j += 8) {
#pragma unroll
    for (int l = 0; l < 8; ++l) a8[l] = term(a8[l], q[j + l], x[j + l]);
  }
  float s[4];
#pragma unroll
  for (int l = 0; l < 4; ++l) s[l] = __fadd_rn(a8[l + 4], a8[l]);
  if (j + 4 <= dim) {
#pragma unroll
    for (int l = 0; l < 4; ++l) s[l] = term(s[l], q[j + l], x[j + l]);
    j += 4;
  }
  if (j + 2 <= dim) {
    s[2] = term(s[2], q[j], x[j]);
    s[3] = term(s[3], q[j + 1], x[j + 1]);
    j += 2;
  }
  float r = __fadd_rn(__fadd_rn(s[0], s[2]), __fadd_rn(s[1], s[3]));
  if (j < dim) r = term(r, q[j], x[j]);
  return r;
}

// ---------------------------------------------------------------------------
// Final selection per query: exact k' best by (distance, tie id) among the
// candidates, tie -> global id, SOAR de-duplication, exact reorder, and the
// (distance, id) sort of SortAndDropResults.
// LDS: keys[cap_pow2] u64 | q[dim] f32 | gid/dist scratch.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) final_select_kernel(SelectArgs a) {
  extern __shared__ uint64_t lds[];
  const int qi = a.qlist ? int(a.qlist[blockIdx.x]) : int(blockIdx.x);
  const uint32_t raw_n = a.cand_count[qi];

  const uint32_t n = min(raw_n, a.cap);
  // LDS: keys[kcap] | sel[selcap] | aux[kkp2] | q[dim] | gid[kk] | dist[kk] | hist | scan
  const uint32_t kcap = NextPow2(a.cap);
  const uint32_t kkp2 = NextPow2(uint32_t(a.kk));
  const uint32_t selcap = max(2048u, 2 * kkp2);
  uint64_t* keys = lds;
  uint64_t* sel = lds + kcap;
  uint64_t* aux = sel + selcap;
  float* q = reinterpret_cast<float*>(aux + kkp2);
  uint32_t* gid = reinterpret_cast<uint32_t*>(q + a.dim);
  float* dist = reinterpret_cast<float*>(gid + a.kk);
  uint32_t* hist = reinterpret_cast<uint32_t*>(dist + a.kk);
  uint32_t* scan_buf = hist + kSelBins;
  __shared__ uint32_t s_m;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) keys[i] = a.cand[size_t(qi) * a.cap + i];
  if (a.reorder)
    for (int d = threadIdx.x; d < a.dim; d += blockDim.x) q[d] = a.queries[size_t(qi) * a.dim + d];
  __syncthreads();
  uint32_t m = SelectSmallest(keys, n, uint32_t(a.kk), sel, selcap, hist, scan_buf);
  __syncthreads();
  keys = sel;  // the m smallest, sorted
  // tie -> global id
  for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) {
    const uint64_t k = keys[i];
    uint32_t tie = uint32_t(k & 0xFFFFFFFFu);
    if (a.shift > 0) {
      const uint32_t leaf = tie >> a.shift;
      const uint32_t local = tie & ((1u << a.shift) - 1u);
      tie = a.members[a.member_off[leaf] + local];
    }
    gid[i] = tie;
    dist[i] = FromOrdered(uint32_t(k >> 32));
  }
  __syncthreads();
  if (a.shard_out) {   // shard mode (rare fallback path): local top-k' entries
    ShardEntry* so = a.shard_out + size_t(qi) * a.kk;
    for (uint32_t i = threadIdx.x; i < uint32_t(a.kk); i += blockDim.x) {
      ShardEntry e;
      e.key = ~0ull;
      e.id = 0u;
      e.exact = 0.0f;
      if (i < m) {
        uint64_t key = keys[i];
        const float* x = a.dataset ? a.dataset + size_t(gid[i]) * a.dim : nullptr;
        if (a.shift > 0) {
          const uint32_t tie = uint32_t(key & 0xFFFFFFFFu);
          const uint32_t leaf = tie >> a.shift;
          const uint32_t local = tie & ((1u << a.shift) - 1u);
          if (a.member_rows) x = a.member_rows + (a.member_off[leaf] + local) * uint64_t(a.dim);
          if (a.row_base)
            key = (key & 0xFFFFFFFF00000000ull) | ((leaf << a.shift) | (local + a.row_base[leaf]));
        }
        e.key = key;
        e.id = gid[i];
        e.exact = a.reorder ? ExactDistance(q, x, a.dim, a.metric) : dist[i];
      }
      so[i] = e;
    }
    return;
  }
  if (!a.disjoint) {
    // Group duplicates by id: sort (gid << 32 | rank).
    const uint32_t mp2 = NextPow2(m);
    for (uint32_t i = threadIdx.x; i < mp2; i += blockDim.x)
      keys[i] = i < m ? ((uint64_t(gid[i]) << 32) | i) : ~0ull;
    __syncthreads();
    BitonicSort(keys, mp2);
    // For each run start: averaged distance 0.5a + 0.5b (two copies at most).
    // (ordered(d) << 32 | gid) for run starts, MAX for the rest.
    for (uint32_t i = threadIdx.x; i < mp2; i += blockDim.x) {
      uint64_t out = ~0ull;
      if (i < m) {
        const uint32_t g = uint32_t(keys[i] >> 32);
        const bool start = (i == 0) || uint32_t(keys[i - 1] >> 32) != g;
        if (start) {
          float d = dist[uint32_t(keys[i] & 0xFFFFFFFFu)];
          if (i + 1 < m && uint32_t(keys[i + 1] >> 32) == g) {
            const float d2 = dist[uint32_t(keys[i + 1] & 0xFFFFFFFFu)];
            d = __fadd_rn(__fmul_rn(0.5f, d), __fmul_rn(0.5f, d2));
          }
          out = (uint64_t(OrderedBits(d)) << 32) | g;
        }
      }
      aux[i] = out;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < mp2; i += blockDim.x) keys[i] = aux[i];
    __syncthreads();
    BitonicSort(keys, mp2);
    if (threadIdx.x == 0) {
      uint32_t u = 0;
      while (u < m && keys[u] != ~0ull) ++u;
      s_m = min(u, uint32_t(a.pre_nn));
    }
    __syncthreads();
    m = s_m;
    for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) {
      gid[i] = uint32_t(keys[i] & 0xFFFFFFFFu);
      dist[i] = FromOrdered(uint32_t(keys[i] >> 32));
    }
    __syncthreads();
  }
  if (a.reorder && !a.pre_only) {
    for (uint32_t i = threadIdx.x; i < m; i += blockDim.x)
      dist[i] = ExactDistance(q, a.dataset + size_t(gid[i]) * a.dim, a.dim, a.metric);
    __syncthreads();
  }
  // Sort by (distance, global id) and keep the output width.
  const uint32_t mp2 = NextPow2(m);
  for (uint32_t i = threadIdx.x; i < mp2; i += blockDim.x)
    keys[i] = i < m ? ((uint64_t(OrderedBits(dist[i])) << 32) | gid[i]) : ~0ull;
  __syncthreads();
  BitonicSort(keys, mp2);
  const uint32_t keep = min(m, uint32_t(a.out_width));
  for (int i = threadIdx.x; i < a.out_width; i += blockDim.x) {
    const bool has = uint32_t(i) < keep;
    a.out_idx[size_t(qi) * a.out_width + i] = has ? uint32_t(keys[i] & 0xFFFFFFFFu) : 0u;
    a.out_dist[size_t(qi) * a.out_width + i] =
        has ? FromOrdered(uint32_t(keys[i] >> 32)) : __int_as_float(0x7fc00000);
  }
  if (threadIdx.x == 0 && a.out_count) a.out_count[qi] = int32_t(keep);
}

// ---------------------------------------------------------------------------
// Final selection, default path: one 256-thread block per query and at most
// kSelMax keys ever held in LDS.  A linear histogram of the distance word
// (refined up to 6 times, straight from the global candidate list) bounds the
// k'-th key; the <= kSelMax keys under that bound are ordered by a counting
// rank (keys are unique, so each thread's rank is its slot; one barrier
// instead of a bitonic network).  Then tie -> global id, SOAR
// de-duplication, the exact reorder with 8 lanes per candidate (the A.8
// order of ExactDistance) and the final (distance, id) rank.  Queries whose
// boundary distance value alone holds more than kSelMax keys are appended to
// a.fallback and re-run by final_select_kernel.
// ---------------------------------------------------------------------------
constexpr int kSelMax = 256;
constexpr int kFsBins = 256;

// Exact distances of m candidates (rows + rowid[i] * dim) into dist[], 8
// lanes per candidate: lane l of a group owns accumulator l of the A.8 layout
// (dims l, l+8, ...) and the folds follow ExactDistance exactly.  256
// threads; ends with a barrier.
__device__ void ExactDistances8(const SelectArgs& a, const float* rows, const uint32_t* rowid,
                                uint32_t m, float* dist, int qi) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int l = tid & 7, gb = lane & ~7;
  const float* q = a.queries + size_t(qi) * a.dim;
  const int dim = a.dim, j8 = dim & ~7;
  const bool l2 = a.metric != 0;
  auto term = [l2](float acc, float x, float y) {
    if (!l2) return __fmaf_rn(-x, y, acc);
    const float t = __fsub_rn(x, y);
    return __fmaf_rn(t, t, acc);
  };
  for (uint32_t base = 0; base < m; base += 32) {
    const uint32_t i = base + uint32_t(tid >> 3);
    const bool act = i < m;
    const float* x = rows + size_t(rowid[act ? i : 0]) * dim;
    float acc = 0.0f;
    for (int j = 0; j < j8; j += 8) acc = term(acc, q[j + l], x[j + l]);
    const float hi4 = __shfl(acc, gb + ((l + 4) & 7));
    float sv = __fadd_rn(hi4, acc);   // lanes l < 4: s[l]
    int j = j8;
    if (j + 4 <= dim) {
      if (l < 4) sv = term(sv, q[j + l], x[j + l]);
      j += 4;
    }
    if (j + 2 <= dim) {
      if (l == 2 || l == 3) sv = term(sv, q[j + l - 2], x[j + l - 2]);
      j += 2;
    }
    const float s1 = __shfl(sv, gb + 1), s2 = __shfl(sv, gb + 2), s3 = __shfl(sv, gb + 3);
    float r = __fadd_rn(__fadd_rn(sv, s2), __fadd_rn(s1, s3));
    if (j < dim) r = term(r, q[j], x[j]);
    __syncthreads();   // every read of rowid/dist for this pass is done
    if (l == 0 && act) dist[i] = r;
  }
  __syncthreads();
}

__global__ void __launch_bounds__(256) final_select_rank_kernel(SelectArgs a) {
  __shared__ uint64_t sel[kSelMax], out[kSelMax];
  __shared__ uint32_t hist[kFsBins], wsum[4], gid[kSelMax], rowid[kSelMax];
  __shared__ float dist[kSelMax];
  __shared__ uint32_t s_lo[4], s_hi[4], s_b, s_cle, s_cbef, s_c;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int qi = blockIdx.x;
  const uint32_t raw_n = a.cand_count[qi];
  if (tid == 0) s_c = 0;
  const uint32_t n = min(raw_n, a.cap);
  const uint32_t k = uint32_t(a.kk);
  const uint64_t* ck = a.cand + size_t(qi) * a.cap;
  if (n <= uint32_t(kSelMax)) {
    if (uint32_t(tid) < n) sel[tid] = ck[tid];
    __syncthreads();
  } else {
    uint32_t lo = 0xFFFFFFFFu, hi = 0;
    for (uint32_t i = tid; i < n; i += 256) {
      const uint32_t v = uint32_t(ck[i] >> 32);
      lo = min(lo, v);
      hi = max(hi, v);
    }
    for (int off = 32; off > 0; off >>= 1) {
      lo = min(lo, uint32_t(__shfl_xor(int(lo), off)));
      hi = max(hi, uint32_t(__shfl_xor(int(hi), off)));
    }
    if (lane == 0) { s_lo[wid] = lo; s_hi[wid] = hi; }
    __syncthreads();
    lo = min(min(s_lo[0], s_lo[1]), min(s_lo[2], s_lo[3]));
    hi = max(max(s_hi[0], s_hi[1]), max(s_hi[2], s_hi[3]));
    uint32_t below = 0, lim = 0;
    bool ok = false;
    for (int it = 0; it < 6; ++it) {
      const uint64_t span = uint64_t(hi - lo) + 1;
      hist[tid] = 0;
      __syncthreads();
      for (uint32_t i = tid; i < n; i += 256) {
        const uint32_t v = uint32_t(ck[i] >> 32);
        if (v >= lo && v <= hi) atomicAdd(&hist[uint32_t((uint64_t(v - lo) * kFsBins) / span)], 1u);
      }
      __syncthreads();
      const uint32_t hv = hist[tid];
      const uint32_t inc = BlockInclusiveScan256(hv, wsum);
      if (below + inc - hv < k && below + inc >= k) {
        s_b = uint32_t(tid);
        s_cle = below + inc;
        s_cbef = below + inc - hv;
      }
      __syncthreads();
      const uint32_t b = s_b, cle = s_cle, cbef = s_cbef;
      // values of bin b: [lo + ceil(b*span/256), lo + ceil((b+1)*span/256) - 1]
      const uint32_t blo = lo + uint32_t((uint64_t(b) * span + kFsBins - 1) / kFsBins);
      const uint32_t bhi = lo + uint32_t((uint64_t(b + 1) * span + kFsBins - 1) / kFsBins) - 1;
      __syncthreads();   // s_b/wsum are rewritten by the next round
      if (cle <= uint32_t(kSelMax)) {
        lim = bhi;
        ok = true;
        break;
      }
      if (bhi == blo) break;   // one distance value holds too many keys
      below = cbef;
      lo = blo;
      hi = bhi;
    }
    if (!ok) {   // block-uniform
      if (tid == 0) a.fallback[atomicAdd(&a.overflow[9], 1u)] = uint32_t(qi);
      return;
    }
    for (uint32_t i = tid; i < n; i += 256) {
      const uint64_t key = ck[i];
      if (uint32_t(key >> 32) <= lim) sel[atomicAdd(&s_c, 1u)] = key;
    }
    __syncthreads();
  }
  const uint32_t c = n <= uint32_t(kSelMax) ? n : s_c;
  // counting rank: keys are unique, so rank = number of smaller keys
  if (uint32_t(tid) < c) {
    const uint64_t key = sel[tid];
    uint32_t r = 0;
    for (uint32_t j = 0; j < c; ++j) r += sel[j] < key ? 1u : 0u;
    out[r] = key;
  }
  __syncthreads();
  uint32_t m = min(c, k);
  // exact-reorder rows: dataset[global id], or in a shard with its own rows,
  // member_rows[member slot]
  const float* rows = a.member_rows ? a.member_rows : a.dataset;
  if (uint32_t(tid) < m) {
    const uint64_t key = out[tid];
    uint32_t tie = uint32_t(key & 0xFFFFFFFFu);
    uint32_t rid = tie;
    if (a.shift > 0) {
      const uint32_t leaf = tie >> a.shift;
      const uint32_t local = tie & ((1u << a.shift) - 1u);
      const uint64_t slot = a.member_off[leaf] + local;
      tie = a.members[slot];
      rid = a.member_rows ? uint32_t(slot) : tie;
      if (a.shard_out && a.row_base)   // whole-index tie for the merge
        out[tid] = (key & 0xFFFFFFFF00000000ull) |
                   ((leaf << a.shift) | (local + a.row_base[leaf]));
    }
    gid[tid] = tie;
    rowid[tid] = rid;
    dist[tid] = FromOrdered(uint32_t(key >> 32));
  }
  __syncthreads();
  if (a.shard_out) {
    // local top-k' with exact distances of this shard's rows; de-duplication
    // and the final order happen in the merge
    if (a.reorder) ExactDistances8(a, rows, rowid, m, dist, qi);
    ShardEntry* so = a.shard_out + size_t(qi) * a.kk;
    for (int i = tid; i < a.kk; i += 256) {
      ShardEntry e;
      e.key = uint32_t(i) < m ? out[i] : ~0ull;
      e.id = uint32_t(i) < m ? gid[i] : 0u;
      e.exact = uint32_t(i) < m ? dist[i] : 0.0f;
      so[i] = e;
    }
    return;
  }
  if (!a.disjoint) {
    // group duplicate ids: rank (gid << 32 | slot); run starts keep the
    // averaged distance 0.5a + 0.5b (two copies at most), the rest drop out
    if (uint32_t(tid) < m) {
      const uint64_t key = (uint64_t(gid[tid]) << 32) | uint32_t(tid);
      uint32_t r = 0;
      for (uint32_t j = 0; j < m; ++j) r += ((uint64_t(gid[j]) << 32) | j) < key ? 1u : 0u;
      sel[r] = key;
    }
    __syncthreads();
    uint64_t o = ~0ull;
    if (uint32_t(tid) < m) {
      const uint32_t g = uint32_t(sel[tid] >> 32);
      if (tid == 0 || uint32_t(sel[tid - 1] >> 32) != g) {
        float d = dist[uint32_t(sel[tid] & 0xFFFFFFFFu)];
        if (uint32_t(tid) + 1 < m && uint32_t(sel[tid + 1] >> 32) == g) {
          const float d2 = dist[uint32_t(sel[tid + 1] & 0xFFFFFFFFu)];
          d = __fadd_rn(__fmul_rn(0.5f, d), __fmul_rn(0.5f, d2));
        }
        o = (uint64_t(OrderedBits(d)) << 32) | g;
        hist[tid] = rowid[uint32_t(sel[tid] & 0xFFFFFFFFu)];   // the run's row
      }
    }
    out[tid] = o;
    if (tid == 0) s_c = 0;
    __syncthreads();
    if (o != ~0ull) {
      uint32_t r = 0;
      for (uint32_t j = 0; j < m; ++j) r += out[j] < o ? 1u : 0u;
      atomicAdd(&s_c, 1u);
      if (r < uint32_t(a.pre_nn)) {
        gid[r] = uint32_t(o & 0xFFFFFFFFu);
        dist[r] = FromOrdered(uint32_t(o >> 32));
        rowid[r] = hist[tid];
      }
    }
    __syncthreads();
    m = min(s_c, uint32_t(a.pre_nn));
  }
  if (a.reorder && !a.pre_only) ExactDistances8(a, rows, rowid, m, dist, qi);
  // final (distance, global id) rank; keep the output width
  const uint32_t keep = min(m, uint32_t(a.out_width));
  if (uint32_t(tid) < m) {
    const uint64_t key = (uint64_t(OrderedBits(dist[tid])) << 32) | gid[tid];
    uint32_t r = 0;
    for (uint32_t j = 0; j < m; ++j) r += ((uint64_t(OrderedBits(dist[j])) << 32) | gid[j]) < key;
    if (r < keep) {
      a.out_idx[size_t(qi) * a.out_width + r] = uint32_t(key & 0xFFFFFFFFu);
      a.out_dist[size_t(qi) * a.out_width + r] = FromOrdered(uint32_t(key >> 32));
    }
  }
  for (int i = int(keep) + tid; i < a.out_width; i += 256) {
    a.out_idx[size_t(qi) * a.out_width + i] = 0u;
    a.out_dist[size_t(qi) * a.out_width + i] = __int_as_float(0x7fc00000);
  }
  if (tid == 0 && a.out_count) a.out_count[qi] = int32_t(keep);
}

// ---------------------------------------------------------------------------
// Merge of range-split shards.  Per query: the world lists
// (each sorted by key, UINT64_MAX-padded) are loaded into LDS; an entry's
// global rank is its position in its list plus, in every other list, the
// number of smaller keys (binary search; keys are unique across shards since
// ties are whole-index rows).  The kk smallest then go through the SOAR
// de-duplication of final_select (averaged approximate distance of a
// datapoint's two copies) and the final (distance, id) order, with the exact
// distances the owning shards computed.
// ---------------------------------------------------------------------------
constexpr int kMergeMaxEntries = 2048;

__global__ void __launch_bounds__(256) merge_shards_kernel(MergeArgs a) {
  __shared__ uint64_t lk[kMergeMaxEntries];
  __shared__ uint64_t sel[kSelMax], outk[kSelMax];
  __shared__ uint32_t sid[kSelMax], gid[kSelMax];
  __shared__ float sex[kSelMax], dist[kSelMax], ex[kSelMax];
  __shared__ uint32_t cnt[64], s_c;
  const int tid = threadIdx.x;
  const int qi = blockIdx.x;
  const int W = a.world, kk = a.kk;
  auto entry = [&](int w, int j) -> const ShardEntry& {
    return a.entries[(size_t(w) * a.nq + qi) * kk + j];
  };
  for (int e = tid; e < W * kk; e += 256) lk[e] = entry(e / kk, e % kk).key;
  if (tid == 0) s_c = 0;
  __syncthreads();
  if (tid < W) {   // valid entries: the padding sorts last
    int lo = 0, hi = kk;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (lk[tid * kk + mid] != ~0ull) lo = mid + 1; else hi = mid;
    }
    cnt[tid] = uint32_t(lo);
  }
  __syncthreads();
  for (int e = tid; e < W * kk; e += 256) {
    const int w = e / kk, j = e % kk;
    if (uint32_t(j) >= cnt[w]) continue;
    const uint64_t key = lk[e];
    uint32_t r = uint32_t(j);
    for (int v = 0; v < W && r < uint32_t(kk); ++v) {
      if (v == w) continue;
      int lo = 0, hi = int(cnt[v]);
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (lk[v * kk + mid] < key) lo = mid + 1; else hi = mid;
      }
      r += uint32_t(lo);
    }
    if (r < uint32_t(kk)) {
      const ShardEntry& se = entry(w, j);
      sel[r] = key;
      sid[r] = se.id;
      sex[r] = se.exact;
    }
  }
  uint32_t total = 0;
  for (int w = 0; w < W; ++w) total += cnt[w];
  uint32_t m = min(total, uint32_t(kk));
  __syncthreads();
  if (uint32_t(tid) < m) {
    gid[tid] = sid[tid];
    dist[tid] = FromOrdered(uint32_t(sel[tid] >> 32));
    ex[tid] = sex[tid];
  }
  __syncthreads();
  if (!a.disjoint) {
    if (uint32_t(tid) < m) {
      const uint64_t key = (uint64_t(gid[tid]) << 32) | uint32_t(tid);
      uint32_t r = 0;
      for (uint32_t j = 0; j < m; ++j) r += ((uint64_t(gid[j]) << 32) | j) < key ? 1u : 0u;
      sel[r] = key;
    }
    __syncthreads();
    uint64_t o = ~0ull;
    float oex = 0.0f;
    if (uint32_t(tid) < m) {
      const uint32_t g = uint32_t(sel[tid] >> 32);
      if (tid == 0 || uint32_t(sel[tid - 1] >> 32) != g) {
        const uint32_t s0 = uint32_t(sel[tid] & 0xFFFFFFFFu);
        float d = dist[s0];
        if (uint32_t(tid) + 1 < m && uint32_t(sel[tid + 1] >> 32) == g) {
          const float d2 = dist[uint32_t(sel[tid + 1] & 0xFFFFFFFFu)];
          d = __fadd_rn(__fmul_rn(0.5f, d), __fmul_rn(0.5f, d2));
        }
        o = (uint64_t(OrderedBits(d)) << 32) | g;
        oex = ex[s0];
      }
    }
    outk[tid] = o;
    __syncthreads();
    if (o != ~0ull) {
      uint32_t r = 0;
      for (uint32_t j = 0; j < m; ++j) r += outk[j] < o ? 1u : 0u;
      atomicAdd(&s_c, 1u);
      if (r < uint32_t(a.pre_nn)) {
        gid[r] = uint32_t(o & 0xFFFFFFFFu);
        dist[r] = FromOrdered(uint32_t(o >> 32));
        ex[r] = oex;
      }
    }
    __syncthreads();
    m = min(s_c, uint32_t(a.pre_nn));
  }
  const uint32_t keep = min(m, uint32_t(a.out_width));
  if (uint32_t(tid) < m) {
    const float d = a.reorder ? ex[tid] : dist[tid];
    const uint64_t key = (uint64_t(OrderedBits(d)) << 32) | gid[tid];
    uint32_t r = 0;
    for (uint32_t j = 0; j < m; ++j)
      r += ((uint64_t(OrderedBits(a.reorder ? ex[j] : dist[j])) << 32) | gid[j]) < key;
    if (r < keep) {
      a.out_idx[size_t(qi) * a.out_width + r] = gid[tid];
      a.out_dist[size_t(qi) * a.out_width + r] = FromOrdered(uint32_t(key >> 32));
    }
  }
  for (int i = int(keep) + tid; i < a.out_width; i += 256) {
    a.out_idx[size_t(qi) * a.out_width + i] = 0u;
    a.out_dist[size_t(qi) * a.out_width + i] = __int_as_float(0x7fc00000);
  }
  if (tid == 0 && a.out_count) a.out_count[qi] = int32_t(keep);
}

// Candidate-list statistics for the host loop (one block; no same-address
// atomics from every query's block): [0] any list over capacity, [1] the
// largest such count, [2] the largest count, [8] the sum of counts.
__global__ void __launch_bounds__(1024) cand_stats_kernel(const uint32_t* __restrict__ cand_count,
                                                          int nq, uint32_t cap,
                                                          uint32_t* __restrict__ stats) {
  __shared__ uint32_t s_over[16], s_max[16], s_sum[16];
  uint32_t over = 0, mx = 0, sum = 0;
  for (int i = threadIdx.x; i < nq; i += blockDim.x) {
    const uint32_t v = cand_count[i];
    if (v > cap) over = max(over, v);
    mx = max(mx, v);
    sum += v;
  }
  for (int off = 32; off > 0; off >>= 1) {
    over = max(over, uint32_t(__shfl_xor(int(over), off)));
    mx = max(mx, uint32_t(__shfl_xor(int(mx), off)));
    sum += uint32_t(__shfl_xor(int(sum), off));
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { s_over[wid] = over; s_max[wid] = mx; s_sum[wid] = sum; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < int(blockDim.x >> 6); ++w) {
      over = max(over, s_over[w]);
      mx = max(mx, s_max[w]);
      sum += s_sum[w];
    }
    stats[0] = over ? 1u : 0u;
    stats[1] = over;
    stats[2] = mx;
    stats[8] = sum;
  }
}

__global__ void exact_distances_kernel(const float* __restrict__ queries, const float* __restrict__ dataset,
                                       int dim, int metric, const uint32_t* __restrict__ ids,
                                       int k, float* __restrict__ out) {
  const int qi = blockIdx.x;
  for (int i = threadIdx.x; i < k; i += blockDim.x) {
    const uint32_t g = ids[size_t(qi) * k + i];
    out[size_t(qi) * k + i] = ExactDistance(queries + size_t(qi) * dim, dataset + size_t(g) * dim, dim, metric);
  }
}

__global__ void fill64_kernel(uint64_t* p, uint64_t v, size_t n) {
  const size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

}  // namespace

// ---------------------------------------------------------------------------
// Launchers.
// ---------------------------------------------------------------------------
hipError_t LaunchPartitionTopL(const DeviceIndex& ix, const float* queries, int nq, int L,
                               int32_t* out_leaf, float* out_dist, float* scores, hipStream_t s) {
  if (nq == 0) return hipSuccess;
  uint32_t kcap = 1;
  while (kcap < uint32_t(ix.nl)) kcap <<= 1;
  uint32_t lp2 = 1;
  while (lp2 < uint32_t(L)) lp2 <<= 1;
  const uint32_t selcap = std::max<uint32_t>(2048u, 2 * lp2);
  const size_t lds = size_t(kcap) * 8 + size_t(selcap) * 8 + (kSelBins + 256) * 4;
  hipLaunchKernelGGL(partition_scores_kernel,
                     dim3((nq + kPartTile - 1) / kPartTile, (ix.nl + kPartTile - 1) / kPartTile),
                     dim3(256), 0, s, queries, nq, ix.dim, ix.centers, ix.cnorm, ix.nl, ix.metric,
                     scores);
  if (ix.nl <= kLdsSelectLeaves && lds <= 160 * 1024) {
    hipLaunchKernelGGL(topl_select_kernel, dim3(nq), dim3(256), lds, s, scores, ix.nl, L, kcap,
                       out_leaf, out_dist);
  } else {
    uint32_t lcap = 1;
    while (lcap < uint32_t(std::min(L, ix.nl))) lcap <<= 1;
    if (size_t(lcap) * 8 > 128 * 1024) return hipErrorInvalidValue;   // L > 16384
    hipLaunchKernelGGL(topl_select_global_kernel, dim3(nq), dim3(256), size_t(lcap) * 8, s, scores,
                       ix.nl, L, lcap, out_leaf, out_dist);
  }
  return hipGetLastError();
}

hipError_t LaunchLutBuild(const DeviceIndex& ix, const float* queries, int nq, int8_t* lut,
                          float* mult, float* inv, uint8_t* lut_u8, hipStream_t s,
                          const LutInit* init) {
  if (nq == 0) return hipSuccess;
  const LutInit none{};
  hipLaunchKernelGGL(lut_build_kernel, dim3(nq), dim3(256), 0, s, queries, ix.dim, ix.codebook,
                     ix.nb, ix.dpb, 2 * ix.ksteps, ix.metric, ix.residual, lut, mult, inv, lut_u8,
                     init ? *init : none);
  return hipGetLastError();
}

hipError_t LaunchPairs(const DeviceIndex& ix, const uint32_t* order, const int32_t* topl_leaf,
                       const float* topl_dist,
                       int nq, int L, uint32_t* cnt, uint32_t* block_cnt, uint32_t* pair_off,
                       uint32_t* tile_prefix, uint32_t* pair_q, float* pair_bias, uint2* work,
                       uint32_t* totals, unsigned long long* code_bytes, uint32_t chunk_tiles,
                       uint32_t queries_per_item, hipStream_t s) {
  const int n = nq * L;
  const int nblocks = (n + kPairsPerBlock - 1) / kPairsPerBlock;
  const int ranges = (ix.nl + kLeafRange - 1) / kLeafRange;
  const size_t lds = size_t(std::min(ix.nl, kLeafRange)) * 4;
  if (n > 0)
    hipLaunchKernelGGL(pairs_count_kernel, dim3(nblocks, ranges), dim3(256), lds, s, topl_leaf, n,
                       ix.nl, block_cnt, cnt);
  // up to 4096 leaves the block offsets ride in the one-block scan kernel
  const int fused = (n > 0 && ix.nl <= 4096) ? nblocks : 0;
  hipLaunchKernelGGL(pairs_scan_kernel, dim3(1), dim3(1024), 0, s, cnt, order,
                     ix.leaf_size, ix.nl, ix.nb, chunk_tiles, queries_per_item, pair_off,
                     tile_prefix, totals, code_bytes, work, block_cnt, fused);
  if (n > 0) {
    if (!fused)
      hipLaunchKernelGGL(pairs_block_offsets_kernel, dim3((ix.nl + 255) / 256), dim3(256), 0, s,
                         block_cnt, nblocks, ix.nl);
    hipLaunchKernelGGL(pairs_scatter_kernel, dim3(nblocks, ranges), dim3(256), lds, s, topl_leaf,
                       topl_dist, n, L, ix.nl, pair_off, block_cnt, pair_q, pair_bias);
  }
  return hipGetLastError();
}

#define SMX_SCAN_CASE(KV)                                                          \
  case KV:                                                                         \
    if (variant == 4)                                                              \
      hipLaunchKernelGGL((lut16_scan_kernel<KV, 4>), dim3(grid), dim3(256), 0, s, a); \
    else                                                                           \
      hipLaunchKernelGGL((lut16_scan_kernel<KV, 0>), dim3(grid), dim3(256), 0, s, a); \
    break;

hipError_t LaunchScan(const DeviceIndex& ix, const ScanArgs& a, int grid, int variant,
                      hipStream_t s) {
  switch (ix.ksteps) {
    SMX_SCAN_CASE(4)
    SMX_SCAN_CASE(8)
    SMX_SCAN_CASE(12)
    SMX_SCAN_CASE(16)
    SMX_SCAN_CASE(20)
    SMX_SCAN_CASE(24)
    SMX_SCAN_CASE(25)
    SMX_SCAN_CASE(28)
    SMX_SCAN_CASE(32)
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

#define SMX_LEAF_CASE(KV)                                                                  \
  case KV:                                                                                 \
    hipLaunchKernelGGL(leaf_scores_kernel<KV>, dim3(1), dim3(64), 0, s, ix.tiles, tile0, n, \
                       lut, out);                                                          \
    break;

hipError_t LaunchLeafScores(const DeviceIndex& ix, int leaf, const int8_t* lut, int32_t* out,
                            hipStream_t s) {
  uint64_t tile0 = 0;
  uint32_t n = 0;
  hipError_t e = hipMemcpyAsync(&tile0, ix.tile_off + leaf, 8, hipMemcpyDeviceToHost, s);
  if (e != hipSuccess) return e;
  e = hipMemcpyAsync(&n, ix.leaf_size + leaf, 4, hipMemcpyDeviceToHost, s);
  if (e != hipSuccess) return e;
  e = hipStreamSynchronize(s);
  if (e != hipSuccess) return e;
  if (n == 0) return hipSuccess;
  switch (ix.ksteps) {
    SMX_LEAF_CASE(4)
    SMX_LEAF_CASE(8)
    SMX_LEAF_CASE(12)
    SMX_LEAF_CASE(16)
    SMX_LEAF_CASE(20)
    SMX_LEAF_CASE(24)
    SMX_LEAF_CASE(25)
    SMX_LEAF_CASE(28)
    SMX_LEAF_CASE(32)
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

#define SMX_SEED_CASE(KV)                                                        \
  case KV:                                                                       \
    hipLaunchKernelGGL(seed_tau_kernel<KV>, dim3(nq), dim3(256), 0, s, a);       \
    break;

hipError_t LaunchSeed(const DeviceIndex& ix, const SeedArgs& a, int nq, hipStream_t s) {
  if (nq == 0 || a.seed <= 0) return hipSuccess;
  switch (ix.ksteps) {
    SMX_SEED_CASE(4)
    SMX_SEED_CASE(8)
    SMX_SEED_CASE(12)
    SMX_SEED_CASE(16)
    SMX_SEED_CASE(20)
    SMX_SEED_CASE(24)
    SMX_SEED_CASE(25)
    SMX_SEED_CASE(28)
    SMX_SEED_CASE(32)
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t LaunchTighten(const uint64_t* cand, const uint32_t* cand_count, uint32_t cap, int nq,
                         int kk, uint64_t* tau_key, hipStream_t s) {
  if (nq == 0) return hipSuccess;
  uint32_t np2 = 1;
  while (np2 < cap) np2 <<= 1;
  const size_t lds = size_t(np2) * 8;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(tighten_kernel, dim3(nq), dim3(256), lds, s, cand, cand_count, cap, kk,
                     tau_key);
  return hipGetLastError();
}

hipError_t LaunchMergeShards(const MergeArgs& a, hipStream_t s) {
  if (a.nq == 0) return hipSuccess;
  if (a.world < 1 || a.world > 64 || a.kk > kSelMax || a.world * a.kk > kMergeMaxEntries)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(merge_shards_kernel, dim3(a.nq), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t LaunchFinalSelect(const SelectArgs& a, int nq, hipStream_t s) {
  if (nq == 0) return hipSuccess;
  if (!a.qlist)
    hipLaunchKernelGGL(cand_stats_kernel, dim3(1), dim3(1024), 0, s, a.cand_count, nq, a.cap,
                       a.overflow);
  uint32_t kkp2 = 1;
  while (kkp2 < uint32_t(a.kk)) kkp2 <<= 1;
  if (!a.qlist && a.fallback && a.kk <= kSelMax) {   // (shard mode too)
    hipLaunchKernelGGL(final_select_rank_kernel, dim3(nq), dim3(256), 0, s, a);
    return hipGetLastError();
  }
  uint32_t kcap = 1;
  while (kcap < a.cap) kcap <<= 1;
  const uint32_t selcap = std::max<uint32_t>(2048u, 2 * kkp2);
  const size_t lds = size_t(kcap) * 8 + size_t(selcap) * 8 + size_t(kkp2) * 8 +
                     size_t(a.dim) * 4 + size_t(a.kk) * 8 + (kSelBins + 256) * 4;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(final_select_kernel, dim3(nq), dim3(256), lds, s, a);
  return hipGetLastError();
}

hipError_t LaunchExactDistances(const DeviceIndex& ix, const float* queries, int nq,
                                const uint32_t* ids, int k, float* out, hipStream_t s) {
  if (nq == 0 || k == 0) return hipSuccess;
  hipLaunchKernelGGL(exact_distances_kernel, dim3(nq), dim3(128), 0, s, queries, ix.dataset,
                     ix.dim, ix.metric, ids, k, out);
  return hipGetLastError();
}

hipError_t LaunchFill64(uint64_t* p, uint64_t v, size_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(fill64_kernel, dim3((n + 255) / 256), dim3(256), 0, s, p, v, n);
  return hipGetLastError();
}

}  // namespace smx

// smx_kernels.hip — HIP kernels (gfx950 / CDNA4) of the tree-AH LUT16 query
// path.  Every float operation whose rounding the reference fixes is spelled
// with an explicit round-to-nearest intrinsic; the library is also built with
// -ffp-contract=off.
//
//   partition_scores_kernel query tokenization on MFMA f32 32x32x2: the exact
//                           fma chain of the transposed many-to-many path
//                           (many_to_many_impl.inc:522-560); resets the
//                           search's per-call state
//   topl_select_kernel      exact top-L by (distance, leaf) per query
//                           (kmeans_tree_partitioner.cc:703-728), each pair's
//                           rank in its leaf's list, then the query's raw
//                           float LUT + uint8 fixed point
//                           (asymmetric_hashing_impl.cc:505-645)
//   worklist_kernel         InvertCentersToSearch on the GPU
//                           (tree_ah_hybrid_residual.cc:610-622): list
//                           offsets and the scan's work items
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
#include <cstdlib>
#include <type_traits>

#include "smx_internal.h"

namespace smx {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
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

// Diagnostic build only (-DSMX_PHASE_STAMPS, tools/phase_stamps.py): the
// 100 MHz clock at phase boundaries of the front-end and select kernels,
// [kernel][query][8].  Compiled out of the product library.
#ifdef SMX_PHASE_STAMPS
__device__ unsigned long long* g_phase_stamps;
#define SMX_PHASE(kid, qi, ph)                                                             \
  do {                                                                                     \
    if (g_phase_stamps && (threadIdx.x & 63) == 0 && (qi) < kPhaseQueries)                 \
      g_phase_stamps[((size_t(kid) * kPhaseQueries) + (qi)) * 8 + (ph)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define SMX_PHASE(kid, qi, ph) \
  do {                         \
  } while (0)
#endif

// Debug build only (-DSMX_DEBUG_CHECKS): SMX_GUARD(v, bound, tag) stmt; runs
// stmt only when v < bound and otherwise counts and prints the violation
// (the host turns a non-zero count into SMX_INTERNAL after the call);
// SMX_CHECK(v, bound, tag) only counts.  Both vanish from the product library.
#ifdef SMX_DEBUG_CHECKS
__device__ unsigned int g_check_failures;
__device__ __noinline__ bool SmxCheckFailed(const char* tag, int line, unsigned long long v,
                                            unsigned long long bound) {
  if (atomicAdd(&g_check_failures, 1u) < 32u)
    printf("SMX_CHECK %s (line %d): value %llu bound %llu, block %u thread %u\n", tag, line, v,
           bound, blockIdx.x, threadIdx.x);
  return false;
}
#define SMX_LT(v, b, tag) \
  (((unsigned long long)(v) < (unsigned long long)(b)) || \
   SmxCheckFailed(tag, __LINE__, (unsigned long long)(v), (unsigned long long)(b)))
#define SMX_GUARD(v, b, tag) if (SMX_LT(v, b, tag))
#define SMX_CHECK(v, b, tag) ((void)SMX_LT(v, b, tag))
#else
#define SMX_GUARD(v, b, tag)
#define SMX_CHECK(v, b, tag) ((void)0)
#endif

__device__ __forceinline__ uint32_t NextPow2(uint32_t x) {
  return x <= 1 ? 1u : 1u << (32 - __clz(x - 1));
}

// LDS hand-off between the lanes of ONE wave (the scan's workgroups are a
// single wave): a wave's DS instructions execute in issue order, so all that
// is needed is that the compiler keeps them in program order and that the
// wave's outstanding LDS operations are complete.  Unlike __syncthreads()
// this does not wait for the wave's global loads (the code-tile and next-item
// prefetches stay in flight).
__device__ __forceinline__ void WaveLdsSync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

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

// Number of keys[0..n) below key (LDS, all lanes read the same words:
// broadcasts), two keys per step and eight steps in flight.
__device__ __forceinline__ uint32_t CountLess(const uint64_t* keys, uint32_t n, uint64_t key) {
  uint32_t r = 0, j = 0;
#pragma unroll 8
  for (; j + 1 < n; j += 2) {
    const uint64_t k0 = keys[j], k1 = keys[j + 1];
    r += (k0 < key ? 1u : 0u) + (k1 < key ? 1u : 0u);
  }
  if (j < n) r += keys[j] < key ? 1u : 0u;
  return r;
}

// Stable rank of keys[i] == key among keys[0..n): the keys below it plus
// the equal keys at lower positions.  Distinct keys rank as CountLess; equal
// keys (the two copies of a SOAR-spilled datapoint in an index without the
// global top-N tie, whose keys coincide) get consecutive ranks.
__device__ __forceinline__ uint32_t RankStable(const uint64_t* keys, uint32_t n, uint64_t key,
                                               uint32_t i) {
  uint32_t r = 0;
  for (uint32_t j = 0; j < i; ++j) r += keys[j] <= key ? 1u : 0u;
  return r + CountLess(keys + i + 1, n - i - 1, key);
}

// Block-wide bitonic sort (ascending) of n (power of two) keys in LDS.
__device__ void BitonicSort(uint64_t* keys, uint32_t n) {
  // every thread a compare-exchange pair per step (pair p -> the index with a
  // zero inserted at bit log2(j), and its partner i | j): no idle half
  const uint32_t half = n >> 1;
  for (uint32_t k = 2; k <= n; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t p = threadIdx.x; p < half; p += blockDim.x) {
        const uint32_t i = ((p & ~(j - 1u)) << 1) | (p & (j - 1u));
        const uint32_t ixj = i | j;
        const uint64_t a = keys[i], b = keys[ixj];
        const bool up = (i & k) == 0;
        if ((a > b) == up) {
          keys[i] = b;
          keys[ixj] = a;
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

// Orders the m smallest of the n unique keys keys[0..n) (u64 in LDS, high
// words in [?, hi]) into res[0..m) ascending, in O(n): NBINS linear bins of
// the high word between the keys' minimum and hi; the keys of the bins up to
// the one holding the m-th are scattered to tmp in bin order (a counting
// sort) and each is then ranked among the keys of its own bin.  res may alias
// keys (keys are not read after the scatter).  Returns false, with res
// unwritten, when those keys exceed tmp_cap or a bin holds more than
// kBinRankMax of them (near-ties): the caller orders the keys another way.
// 256 threads; all call; block-uniform result.
constexpr uint32_t kBinRankMax = 256;

template <uint32_t NBINS>
__device__ bool OrderSmallestByBins(const uint64_t* keys, uint32_t n, uint32_t m, uint32_t hi,
                                    uint64_t* tmp, uint32_t tmp_cap, uint64_t* res) {
  static_assert(NBINS % 256 == 0, "bins per thread");
  __shared__ uint32_t hist[NBINS], wsum[4], s_min, s_bsel, s_c, s_maxbin;
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  if (tid == 0) { s_min = 0xFFFFFFFFu; s_bsel = NBINS - 1; s_c = n; s_maxbin = 0; }
  for (uint32_t b = tid; b < NBINS; b += 256) hist[b] = 0;
  uint32_t lo = 0xFFFFFFFFu;
  for (uint32_t i = tid; i < n; i += 256) lo = min(lo, uint32_t(keys[i] >> 32));
  for (int off = 32; off > 0; off >>= 1) lo = min(lo, uint32_t(__shfl_xor(int(lo), off)));
  __syncthreads();
  if (lane == 0) atomicMin(&s_min, lo);
  __syncthreads();
  lo = s_min;
  // bin(v) = ((v - lo) * scale) >> 32 < NBINS, monotone; (v - lo) < span keeps
  // the product below 2^(32 + log2 NBINS)
  const uint64_t span = uint64_t(hi - lo) + 1;
  const uint64_t scale = ((uint64_t(NBINS) << 32) - 1) / span;
  auto bin_of = [&](uint64_t key) {
    return uint32_t((uint64_t(uint32_t(key >> 32) - lo) * scale) >> 32);
  };
  for (uint32_t i = tid; i < n; i += 256) atomicAdd(&hist[bin_of(keys[i])], 1u);
  __syncthreads();
  constexpr uint32_t per = NBINS / 256;
  uint32_t h[per], local = 0;
#pragma unroll
  for (uint32_t u = 0; u < per; ++u) {
    h[u] = hist[tid * per + u];
    local += h[u];
  }
  const uint32_t incl = BlockInclusiveScan256(local, wsum);
  uint32_t run = incl - local, mx = 0;
  const bool owner = run < m && incl >= m;
#pragma unroll
  for (uint32_t u = 0; u < per; ++u) {   // bins -> exclusive offsets, in place
    hist[tid * per + u] = run;
    if (owner && run < m && run + h[u] >= m) { s_bsel = tid * per + u; s_c = run + h[u]; }
    run += h[u];
  }
  __syncthreads();
  const uint32_t bsel = s_bsel, c = s_c;
#pragma unroll
  for (uint32_t u = 0; u < per; ++u)
    if (tid * per + u <= bsel) mx = max(mx, h[u]);
  for (int off = 32; off > 0; off >>= 1) mx = max(mx, uint32_t(__shfl_xor(int(mx), off)));
  if (lane == 0) atomicMax(&s_maxbin, mx);
  __syncthreads();
  if (c > tmp_cap || s_maxbin > kBinRankMax) return false;   // (block-uniform)
  for (uint32_t i = tid; i < n; i += 256) {   // counting-sort scatter by bin
    const uint64_t key = keys[i];
    const uint32_t b = bin_of(key);
    if (b <= bsel) tmp[atomicAdd(&hist[b], 1u)] = key;
  }
  __syncthreads();   // hist[b] = end of bin b = start of bin b + 1
  for (uint32_t p = tid; p < c; p += 256) {
    const uint64_t key = tmp[p];
    const uint32_t b = bin_of(key);
    const uint32_t s0 = b ? hist[b - 1] : 0u, e0 = hist[b];
    uint32_t r = s0;
    for (uint32_t q = s0; q < e0; ++q) r += tmp[q] < key ? 1u : 0u;   // keys are unique
    if (r < m) res[r] = key;
  }
  __syncthreads();
  return true;
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
// w & 1, center half w >> 1); the operands are staged in LDS CHUNK dims at a
// time with coalesced row loads (-q and c or 2c, zero-padded past dim), so
// every MFMA reads its two floats per lane from LDS instead of a strided
// global row.  CHUNK = kPartFullDim (dim <= 128: glove, SIFT, Deep): the
// whole tile in one round of loads, and the squared query norms from the
// staged tile -- one load latency per block instead of one per 32 dims plus
// a serial norm loop over global memory (at 256 blocks, one wave per SIMD,
// nothing else hides them).
constexpr int kPartTile = 64, kPartChunk = 32, kPartFullDim = 128;
#ifndef SMX_PART_BLOCKS
#define SMX_PART_BLOCKS 1024
#endif
constexpr int kPartBlocks = SMX_PART_BLOCKS;   // grid size above which a block takes several center tiles

template <int CHUNK>
__global__ void __launch_bounds__(256) partition_scores_kernel(
    const float* __restrict__ queries, int nq, int dim, const float* __restrict__ centers,
    const float* __restrict__ cnorm, int nl, int metric, float* __restrict__ scores,
    StateInit init, int ctiles) {
  constexpr bool kFull = CHUNK == kPartFullDim;   // dim <= CHUNK: one staging round
  {
    // the search's per-call state (no separate memset nodes); nothing in this
    // launch reads it, the top-L launch that follows does
    const uint32_t gt = (blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x;
    const uint32_t gs = gridDim.x * gridDim.y * blockDim.x;
    for (uint32_t i = gt; i < init.n_counters; i += gs) init.counters[size_t(i) * kCounterStride] = 0u;
    for (uint32_t i = gt; i < init.n_stats; i += gs) init.stats[i] = 0u;
    for (uint32_t i = gt; i < init.n_cand; i += gs) init.cand_count[size_t(i) * kCounterStride] = 0u;
    for (uint32_t i = gt; i < init.n_tau; i += gs) init.tau[i] = kNoThreshold;
  }
  __shared__ float qs[kPartTile][CHUNK + 1];
  __shared__ float cs[kPartTile][CHUNK + 1];
  __shared__ float qn[kPartTile];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, k = lane >> 5;
  const int qt = blockIdx.x * kPartTile, ct = blockIdx.y * kPartTile;
  const int qw = (wave & 1) * 32, cw = (wave >> 1) * 32;   // this wave's sub-tile
  const int q0 = qt + qw, c0 = ct + cw;
  const int cb = min(c0 + r, nl - 1);     // B column (center) of this lane
  // the squared query norm in double, dims ascending (exact squares)
  auto init_acc = [&](v16f& acc) {
    if (metric == 1) {
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
  };
  v16f acc;
  if (!kFull) {
    if (metric == 1) {
      if (tid < kPartTile) {
        double s = 0.0;
        const float* qq = queries + size_t(min(qt + tid, nq - 1)) * dim;
        for (int d = 0; d < dim; ++d) s += double(qq[d]) * double(qq[d]);
        qn[tid] = float(s);
      }
      __syncthreads();
    }
    init_acc(acc);
  }
  const float cscale = metric == 1 ? 2.0f : 1.0f;
  if constexpr (kFull) {
    // row tid / 4, dims tid % 4 + 4 j: one buffer offset per operand and
    // immediate offsets (64 loads with 64-bit addresses needed all 256
    // VGPRs); the resources end at the tile's last row, so a read past it
    // returns 0, and dims past dim (the next row's) are masked below.  (Rows
    // by 128-byte runs, tid % 32 + 32 j, measured 8.7 us against 8.0 at
    // glove's 100 dims, 12.6 against 13.1 at SIFT's 128.)
    // A block takes `ctiles` consecutive center tiles with its query tile
    // staged once; the next center tile's loads are in flight (registers)
    // while the MFMAs of the current one run (many leaves: 782 center tiles
    // at configs[4]'s 50000).
    constexpr int kPer = kPartFullDim / 4;
    const int row = tid >> 2, sub = tid & 3;
    const uint32_t qrows = uint32_t(min(kPartTile, nq - qt));
    const auto qrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(queries + size_t(qt) * dim), 0, int(qrows * uint32_t(dim) * 4u), 0x00020000);
    const int off = (row * dim + sub) * 4;
    const int ct_first = blockIdx.y * ctiles * kPartTile;
    const int ct_end = min(nl, ct_first + ctiles * kPartTile);
    float cv[kPer];
    auto load_c = [&](int ct) {
      const uint32_t crows = uint32_t(min(kPartTile, nl - ct));
      const auto crs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(centers + size_t(ct) * dim), 0, int(crows * uint32_t(dim) * 4u), 0x00020000);
#pragma unroll
      for (int j = 0; j < kPer; ++j)
        cv[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(crs, off + 16 * j, 0, 0));
    };
    {
      float qv[kPer];
#pragma unroll
      for (int j = 0; j < kPer; ++j)
        qv[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(qrs, off + 16 * j, 0, 0));
      load_c(ct_first);
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const int d = sub + 4 * j;
        qs[row][d] = d < dim ? -qv[j] : -0.0f;
      }
    }
    for (int cti = ct_first; cti < ct_end; cti += kPartTile) {
      if (cti != ct_first) __syncthreads();   // the previous tile's operand reads are done
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const int d = sub + 4 * j;
        cs[row][d] = d < dim ? __fmul_rn(cv[j], cscale) : 0.0f;
      }
      __syncthreads();
      if (cti + kPartTile < ct_end) load_c(cti + kPartTile);   // in flight beside the MFMAs
      if (metric == 1 && cti == ct_first) {
        if (tid < kPartTile) {   // (-q)^2 = q^2; the zero padding adds +0
          double s = 0.0;
          for (int d0 = 0; d0 < dim; d0 += 16) {
            float x[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) x[u] = qs[tid][d0 + u];
#pragma unroll
            for (int u = 0; u < 16; ++u) s += double(x[u]) * double(x[u]);
          }
          qn[tid] = float(s);
        }
        __syncthreads();
      }
      const int c0t = cti + cw;
      const int cbt = min(c0t + r, nl - 1);
      if (metric == 1) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int rw = (i & 3) + 8 * (i >> 2) + 4 * k;
          acc[i] = __fadd_rn(cnorm[cbt], qn[qw + rw]);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
      }
      // (steps by 16 dims: the zero padding up to 128 leaves acc unchanged, and
      // the operand reads of 8 MFMAs go out together)
      const int steps = (dim + 15) & ~15;
      for (int s = 0; s < steps; s += 16) {
        float av[8], bv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          av[u] = qs[qw + r][s + 2 * u + k];
          bv[u] = cs[cw + r][s + 2 * u + k];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u], acc, 0, 0, 0);
      }
      const int colt = c0t + r;
      if (colt < nl) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int rw = q0 + (i & 3) + 8 * (i >> 2) + 4 * k;
          if (rw < nq) scores[size_t(rw) * nl + colt] = acc[i];
        }
      }
    }
    return;
  }
  for (int d0 = 0; !kFull && d0 < dim; d0 += CHUNK) {
    __syncthreads();
    // all loads of the chunk in flight together: clamped indices, the
    // padding applied after (a guarded load waits on its own)
    constexpr int kPer = (kPartTile * CHUNK) / 256;
    float qv[kPer], cv[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + i * 256;
      const int row = e / CHUNK, col = e % CHUNK, d = min(d0 + col, dim - 1);
      qv[i] = queries[size_t(min(qt + row, nq - 1)) * dim + d];
      cv[i] = centers[size_t(min(ct + row, nl - 1)) * dim + d];
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + i * 256;
      const int row = e / CHUNK, col = e % CHUNK, d = d0 + col;
      qs[row][col] = d < dim ? -qv[i] : -0.0f;
      cs[row][col] = d < dim ? __fmul_rn(cv[i], cscale) : 0.0f;
    }
    __syncthreads();
    const int steps = min(CHUNK, ((dim - d0) + 1) & ~1);
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

// ---------------------------------------------------------------------------
// LUT build: raw[b][c] = -(fl(q0*c0) + fl(q1*c1)) (dot) or
// fl(t0*t0) + fl(t1*t1), t = q - c (squared L2); multiplier
// 127 / max(sqrt(FLT_EPSILON), max|raw|); int8 = round(raw * m) (the uint8
// table minus its bias 128); inv = (float)(1.0/(double)m) for residual
// indexes (lut16_avx2.inc:427-430), 1.0f/m otherwise (querying.h:450-454).
// LUT rows are padded to LutRows(K) blocks with zeros.
// ---------------------------------------------------------------------------
struct LutParams {
  const float* queries;
  int dim;
  const float* codebook;
  int nb, dpb, padded_blocks, metric, residual;
  int8_t* lut;
  float* mult;
  float* inv;
  uint8_t* lut_u8;   // optional biased uint8 copy (stage entry point)
};

// The LUT of query qi by one 256-thread block (all threads must call), four
// entries per thread.  Dimension i of a thread's entries is loaded for all of
// them at once (clamped indices, no guarded loads: a guarded load waits on its
// own), then accumulated in the reference's order.
__device__ void BuildLut(int qi, const LutParams& p) {
  __shared__ float red[16];
  constexpr int kPer = (kMaxBlocks * 16) / 256;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  // the table's entries belong to the first 256 threads; a larger block's
  // other threads only take part in the reduction's barrier
  const bool act = t < 256;
  const float* q = p.queries + size_t(qi) * p.dim;
  const int nb = p.nb, dpb = p.dpb;
  const int nent = nb * 16;
  const int last = p.dim - dpb * (nb - 1);
  float raw[kPer];
  for (int i = 0; act && i < dpb; ++i) {
    float qv[kPer], cv[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int e = min(t + 256 * u, nent - 1);
      const int b = e >> 4, c = e & 15;
      qv[u] = q[min(b * dpb + i, p.dim - 1)];
      cv[u] = p.codebook[(size_t(b) * 16 + c) * dpb + i];
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int b = min(t + 256 * u, nent - 1) >> 4;
      const int nd = (b == nb - 1) ? last : dpb;
      float v;
      if (p.metric == 0) {
        v = __fmul_rn(qv[u], cv[u]);
      } else {
        const float w = __fsub_rn(qv[u], cv[u]);
        v = __fmul_rn(w, w);
      }
      if (i == 0) raw[u] = v;
      else if (i < nd) raw[u] = __fadd_rn(raw[u], v);
    }
  }
  float local_max = 0.0f;
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int e = t + 256 * u;
    float v = 0.0f;
    if (act && e < nent) v = p.metric == 0 ? -raw[u] : raw[u];
    raw[u] = v;
    local_max = fmaxf(local_max, fabsf(v));
  }
  for (int off = 32; off > 0; off >>= 1) local_max = fmaxf(local_max, __shfl_xor(local_max, off));
  if (lane == 0) red[wid] = local_max;
  __syncthreads();
  local_max = red[0];
  for (int w = 1; w < int(blockDim.x >> 6); ++w) local_max = fmaxf(local_max, red[w]);
  const float m = __fdiv_rn(127.0f, fmaxf(SqrtFltEps(), local_max));
  const int tot = p.padded_blocks * 16;
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int e = t + 256 * u;
    if (act && e < tot) {
      int8_t v8 = 0;
      if (e < nent) {
        const float r = roundf(__fmul_rn(raw[u], m));
        v8 = int8_t(int(r));
        if (p.lut_u8) p.lut_u8[size_t(qi) * nent + e] = uint8_t(int(r) + 128);
      }
      p.lut[size_t(qi) * tot + e] = v8;
    }
  }
  if (t == 0) {
    p.mult[qi] = m;
    p.inv[qi] = p.residual ? float(1.0 / double(m)) : __fdiv_rn(1.0f, m);
  }
}

__global__ void __launch_bounds__(256) lut_build_kernel(LutParams p) { BuildLut(blockIdx.x, p); }

// Exact top-L per query by (score, center index) from the score matrix.
// The front end's per-query tail, shared by both top-L kernels: the
// selected pairs' ranks in their leaves' lists, then the query's LUT.
struct TopLTail {
  uint32_t* leaf_count;   // or NULL
  uint32_t* leaf_pair;    // [nl][slot_stride]: pair p at slot rank of its leaf
  uint32_t slot_stride;
  LutParams lut;          // lut.lut NULL: no LUT
  int lut_split;   // topl_block_kernel: the LUTs by their own blocks [nq, 2 nq)
};

__device__ void TopLFinish(int qi, int L, uint32_t m, const uint64_t* sel, int32_t* out_leaf,
                           float* out_dist, const TopLTail& tail) {
  // eight pairs per thread per round, their count atomics all in flight
  // before the first returned rank is stored (one round trip per round, not
  // per pair: L = 2000 is eight of them)
  constexpr int U = 8;
  for (int i0 = threadIdx.x; i0 < L; i0 += U * blockDim.x) {
    uint32_t rk[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * int(blockDim.x);
      if (i >= L) break;
      const bool has = uint32_t(i) < m;
      const int32_t leaf = has ? int32_t(sel[i] & 0xFFFFFFFFu) : -1;
      out_leaf[size_t(qi) * L + i] = leaf;
      out_dist[size_t(qi) * L + i] = has ? FromOrdered(uint32_t(sel[i] >> 32)) : __int_as_float(0x7fc00000);
      if (tail.leaf_count && has) rk[u] = atomicAdd(&tail.leaf_count[size_t(leaf) * kCounterStride], 1u);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * int(blockDim.x);
      if (i >= L) break;
      if (tail.leaf_count && uint32_t(i) < m)
        tail.leaf_pair[size_t(sel[i] & 0xFFFFFFFFu) * tail.slot_stride + rk[u]] =
            uint32_t(qi) * uint32_t(L) + uint32_t(i);
    }
  }
  if (tail.lut.lut) {
    __syncthreads();
    BuildLut(qi, tail.lut);
  }
}

// Exact top-L by (score, center index) with one NT-thread block per query,
// the row in registers (VPT scores per thread, nl <= NT * VPT; a block per
// query, not a wave: 1000 queries must fill 1024 SIMDs several waves deep;
// NT = 1024 up to 1.6 * 10^4 leaves when L > 256 rules the sampled kernel out;
// above kSampleTopLMinLeaves leaves, topl_sample_kernel).  Linear 256-bin histograms of the
// ordered score bits between the boundary set's [LO, HI] (radix digits of
// nearby floats would all hit one bin) narrow down to the bin holding the
// L-th score until at most 256 keys are left.  The boundary set is always a
// value range, so a score's state needs no register: below LO = taken,
// inside [LO, HI] = boundary, above HI = out.  Every taken key and the
// boundary keys are compacted in LDS and ordered by a counting rank over
// (score, leaf) (keys are unique), of which the first L are kept.  Then the
// pairs' ranks in their leaves' lists and the query's LUT (TopLFinish's
// tail).
constexpr int kWaveTopL = 512;         // L limit of the register top-L kernel
constexpr int kBlockTopCand = 1024;    // compacted keys one block orders
constexpr uint32_t kTopNarrow = 256;   // histogram rounds until this many keys
// above this many compacted keys (<= 256) the block rank instead of the
// counting rank (as final_select_rank_kernel's kBlockRankMin)
constexpr uint32_t kBlockRankMinTopL = 128;

__device__ uint32_t BlockRank256(uint64_t key, uint64_t* sbuf);

template <int VPT, int NT>
__device__ __forceinline__ void TopLBlock(const float* __restrict__ scores, int nl, int L,
                                          int32_t* __restrict__ out_leaf,
                                          float* __restrict__ out_dist, const TopLTail& tail) {
  constexpr int NWV = NT / 64;
  __shared__ uint32_t hist[256];
  __shared__ uint64_t sel[kBlockTopCand];
  __shared__ uint64_t srt[kWaveTopL];
  __shared__ uint32_t s_lo[NWV], s_hi[NWV], s_wave[NWV], s_bin, s_cum, s_hb, s_cnt, s_cnt2;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int qi = blockIdx.x;
  SMX_PHASE(0, qi, 0);
  const float* row = scores + size_t(qi) * nl;
  const uint64_t lanes_below = (1ull << lane) - 1ull;
  // every load issued before the first use (clamped index, no guarded load)
  uint32_t v[VPT];
#pragma unroll
  for (int u = 0; u < VPT; ++u) v[u] = __float_as_uint(row[min(tid + NT * u, nl - 1)]);
#pragma unroll
  for (int u = 0; u < VPT; ++u) v[u] = OrderedBits(__uint_as_float(v[u]));
  auto valid = [&](int u) { return tid + NT * u < nl; };
  if (tid == 0) { s_cnt = 0; s_cnt2 = 0; }
  // block-wide min / max of the boundary keys in [lo, hi] with bin `b` under
  // (lo, scale) (b < 0: every key in [lo, hi])
  auto minmax = [&](uint32_t lo, uint32_t hi, uint64_t scale, int b, uint32_t& mn, uint32_t& mx) {
    mn = 0xFFFFFFFFu;
    mx = 0;
#pragma unroll
    for (int u = 0; u < VPT; ++u)
      if (valid(u) && v[u] >= lo && v[u] <= hi &&
          (b < 0 || int((uint64_t(v[u] - lo) * scale) >> 32) == b)) {
        mn = min(mn, v[u]);
        mx = max(mx, v[u]);
      }
    for (int off = 32; off > 0; off >>= 1) {
      mn = min(mn, uint32_t(__shfl_xor(int(mn), off)));
      mx = max(mx, uint32_t(__shfl_xor(int(mx), off)));
    }
    if (lane == 0) { s_lo[wid] = mn; s_hi[wid] = mx; }
    __syncthreads();
    mn = s_lo[0];
    mx = s_hi[0];
#pragma unroll
    for (int w = 1; w < NWV; ++w) {
      mn = min(mn, s_lo[w]);
      mx = max(mx, s_hi[w]);
    }
    __syncthreads();   // s_lo / s_hi are rewritten by the next call
  };
  SMX_PHASE(0, qi, 1);
  const uint32_t m = min(uint32_t(L), uint32_t(nl));
  uint32_t below = 0, incnt = uint32_t(nl);
  uint32_t LO = 0, HI = 0xFFFFFFFFu;
  minmax(LO, HI, 0, -1, LO, HI);
  for (int round = 0; round < 8 && m > 0 && below + incnt > kTopNarrow && LO < HI; ++round) {
    // bin = floor((v - LO) * scale / 2^32), scale = floor(255.99 * 2^32 / span):
    // monotone in v, 0 at LO, <= 255 at HI (no division per value)
    const uint64_t scale = ((uint64_t(255) << 32) + 0xFFFFFFFFull) / (uint64_t(HI - LO));
    for (int i = tid; i < 256; i += NT) hist[i] = 0;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < VPT; ++u)
      if (valid(u) && v[u] >= LO && v[u] <= HI)
        atomicAdd(&hist[uint32_t((uint64_t(v[u] - LO) * scale) >> 32)], 1u);
    __syncthreads();
    if (wid == 0) {   // wave 0: inclusive scan of 4 bins per lane, the bin of the m-th key
      const uint32_t h0 = hist[4 * lane], h1 = hist[4 * lane + 1], h2 = hist[4 * lane + 2],
                     h3 = hist[4 * lane + 3];
      uint32_t incl = h0 + h1 + h2 + h3;
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = uint32_t(__shfl_up(int(incl), off));
        if (lane >= off) incl += t;
      }
      const uint32_t excl = incl - (h0 + h1 + h2 + h3);
      const uint32_t need = m - below;
      if (excl < need && incl >= need) {
        const uint32_t h[4] = {h0, h1, h2, h3};
        uint32_t cum = excl;
        int u = 0;
        while (cum + h[u] < need) { cum += h[u]; ++u; }
        s_bin = uint32_t(4 * lane + u);
        s_cum = cum;
        s_hb = h[u];
      }
    }
    __syncthreads();
    const int bsel = int(s_bin);
    below += s_cum;
    incnt = s_hb;
    minmax(LO, HI, scale, bsel, LO, HI);   // the selected bin's value range
  }
  SMX_PHASE(0, qi, 2);
  // the taken keys and the boundary keys, in LDS (one LDS atomic per wave)
#pragma unroll
  for (int u = 0; u < VPT; ++u) {
    const bool in = valid(u) && v[u] <= HI;
    const uint64_t bal = __ballot(in);
    uint32_t base = 0;
    if (lane == 0 && bal) base = atomicAdd(&s_cnt, uint32_t(__popcll(bal)));
    base = uint32_t(__shfl(int(base), 0));
    if (in) {
      const uint32_t pos = base + uint32_t(__popcll(bal & lanes_below));
      if (pos < uint32_t(kBlockTopCand)) sel[pos] = (uint64_t(v[u]) << 32) | uint32_t(tid + NT * u);
    }
  }
  __syncthreads();
  const uint32_t cnt = s_cnt;
  if (NT == 256 && cnt <= 256u && cnt > kBlockRankMinTopL) {
    // one key per thread, ranked by BlockRank256 (wave bitonic sorts and
    // binary searches of the other waves' runs; padding keys sort last)
    const uint64_t key = uint32_t(tid) < cnt ? sel[tid] : ((~0ull << 16) | uint32_t(tid));
    __syncthreads();   // sel is the rank's scratch
    const uint32_t r = BlockRank256(key, sel);
    if (uint32_t(tid) < cnt && r < m) srt[r] = key;
  } else if (cnt <= uint32_t(kBlockTopCand)) {
    // counting rank over (score, leaf), keys unique; keep the first m
    for (uint32_t i = tid; i < cnt; i += NT) {
      const uint64_t key = sel[i];
      const uint32_t r = CountLess(sel, cnt, key);
      if (r < m) srt[r] = key;
    }
  } else {
    // more than kBlockTopCand keys on one boundary value (LO == HI, e.g. an
    // all-equal row): the keys below it by rank, then the lowest-index ties
    // in index order (index c = tid + NT u: u-major, then thread order)
    const uint32_t T = LO;
    __syncthreads();   // every thread has read s_cnt; sel is rewritten
#pragma unroll
    for (int u = 0; u < VPT; ++u) {
      const bool in = valid(u) && v[u] < T;
      const uint64_t bal = __ballot(in);
      uint32_t base = 0;
      if (lane == 0 && bal) base = atomicAdd(&s_cnt2, uint32_t(__popcll(bal)));
      base = uint32_t(__shfl(int(base), 0));
      if (in) sel[base + uint32_t(__popcll(bal & lanes_below))] = (uint64_t(v[u]) << 32) | uint32_t(tid + NT * u);
    }
    __syncthreads();
    const uint32_t c2 = s_cnt2;   // == below < m
    for (uint32_t i = tid; i < c2; i += NT) {
      const uint64_t key = sel[i];
      srt[CountLess(sel, c2, key)] = key;
    }
    uint32_t ties = 0;
#pragma unroll
    for (int u = 0; u < VPT; ++u) {
      const bool te = valid(u) && v[u] == T;
      const uint64_t bal = __ballot(te);
      if (lane == 0) s_wave[wid] = uint32_t(__popcll(bal));
      __syncthreads();
      uint32_t before = ties + uint32_t(__popcll(bal & lanes_below));
      for (int w = 0; w < wid; ++w) before += s_wave[w];
      if (te && c2 + before < m) srt[c2 + before] = (uint64_t(T) << 32) | uint32_t(tid + NT * u);
      for (int w = 0; w < NWV; ++w) ties += s_wave[w];
      __syncthreads();   // s_wave is rewritten by the next u
    }
  }
  __syncthreads();
  SMX_PHASE(0, qi, 3);
  for (int i = tid; i < L; i += NT) {
    const bool has = uint32_t(i) < m;
    const int32_t leaf = has ? int32_t(srt[i] & 0xFFFFFFFFu) : -1;
    out_leaf[size_t(qi) * L + i] = leaf;
    out_dist[size_t(qi) * L + i] = has ? FromOrdered(uint32_t(srt[i] >> 32)) : __int_as_float(0x7fc00000);
    if (tail.leaf_count && has) {
      const uint32_t rk = atomicAdd(&tail.leaf_count[size_t(leaf) * kCounterStride], 1u);
      tail.leaf_pair[size_t(leaf) * tail.slot_stride + rk] = uint32_t(qi) * uint32_t(L) + uint32_t(i);
    }
  }
  SMX_PHASE(0, qi, 4);
  if (tail.lut.lut && !tail.lut_split) BuildLut(qi, tail.lut);
  SMX_PHASE(0, qi, 5);
}

template <int VPT, int NT>
__global__ void __launch_bounds__(NT) topl_block_kernel(const float* __restrict__ scores, int nl,
                                                        int L, int32_t* __restrict__ out_leaf,
                                                        float* __restrict__ out_dist, TopLTail tail) {
  // (split: the query LUTs, which need no score, by blocks beside the
  // selections instead of after each one)
  if (tail.lut_split && blockIdx.x >= gridDim.x / 2) {
    BuildLut(int(blockIdx.x - gridDim.x / 2), tail.lut);
    return;
  }
  TopLBlock<VPT, NT>(scores, nl, L, out_leaf, out_dist, tail);
}

__global__ void __launch_bounds__(256) topl_select_kernel(const float* __restrict__ scores, int nl,
                                                          int L, uint32_t kcap,
                                                          int32_t* __restrict__ out_leaf,
                                                          float* __restrict__ out_dist,
                                                          TopLTail tail) {
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
  TopLFinish(qi, L, m, sel, out_leaf, out_dist, tail);
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
__device__ void TopLGlobalSelect(const float* __restrict__ scores, int nl, int L, uint32_t lcap,
                                 uint64_t* sel, int32_t* __restrict__ out_leaf,
                                 float* __restrict__ out_dist, const TopLTail& tail) {
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
  TopLFinish(qi, L, m, sel, out_leaf, out_dist, tail);
}

__global__ void __launch_bounds__(256) topl_select_global_kernel(const float* __restrict__ scores,
                                                                 int nl, int L, uint32_t lcap,
                                                                 int32_t* __restrict__ out_leaf,
                                                                 float* __restrict__ out_dist,
                                                                 TopLTail tail) {
  extern __shared__ uint64_t lds64[];
  TopLGlobalSelect(scores, nl, L, lcap, lds64, out_leaf, out_dist, tail);
}

// The values of histogram bin b (bin = floor((v - lo) scale / 2^32)) as the
// new [lo, hi]: v - lo in [ceil(b 2^32 / scale), ceil((b + 1) 2^32 / scale) - 1]
// (64-bit: the upper end passes 2^32 when hi - lo is near 2^32).
__device__ __forceinline__ void BinRange(uint32_t b, uint64_t scale, uint32_t& lo, uint32_t& hi) {
  const uint64_t blo = uint64_t(lo) + ((uint64_t(b) << 32) + scale - 1) / scale;
  const uint64_t bhi = uint64_t(lo) + ((uint64_t(b + 1) << 32) + scale - 1) / scale - 1u;
  lo = uint32_t(blo);
  hi = uint32_t(min(bhi, uint64_t(hi)));
}

// Exact top-L for many leaves (configs[4]: 50000) by a sampled threshold:
// the k-th smallest of 2048 sampled scores (k = 1.5 L * 2048 / nl + 16,
// found exactly by histogram rounds over 8 values per thread) is a value T at
// or below which ~1.5 L + nl / 128 keys lie; one pass over the row compacts
// every key with score <= T into LDS, and -- when at least L and at most cap
// of them arrived (the L smallest keys are then all among them: at least L
// keys have score <= T) -- a histogram select keeps the ~L smallest, a
// counting sort by bin orders them, and the first L are the result.  Otherwise the radix select from
// global memory (TopLGlobalSelect) runs instead; the result is the same
// exact top-L either way.  No per-thread row in registers (the
// register kernel spilled 56 VGPRs at 52 scores per thread).
constexpr int kSampleVals = 8;          // samples per thread (2048 per query)
constexpr uint32_t kSampleCap = 16384;   // most LDS keys (128 KB)
constexpr int kSampleTopLMinLeaves = 4096;   // the sampled top-L above this many leaves

__device__ uint32_t BlockKthOfSamples(const uint32_t (&v)[kSampleVals], uint32_t kk) {
  __shared__ uint32_t hist[256], wsum[4], s_lo[4], s_hi[4], s_bin, s_below;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint32_t lo = 0xFFFFFFFFu, hi = 0;
#pragma unroll
  for (int i = 0; i < kSampleVals; ++i) {
    lo = min(lo, v[i]);
    hi = max(hi, v[i]);
  }
  for (int off = 32; off > 0; off >>= 1) {
    lo = min(lo, uint32_t(__shfl_xor(int(lo), off)));
    hi = max(hi, uint32_t(__shfl_xor(int(hi), off)));
  }
  if (lane == 0) { s_lo[wid] = lo; s_hi[wid] = hi; }
  __syncthreads();
  lo = min(min(s_lo[0], s_lo[1]), min(s_lo[2], s_lo[3]));
  hi = max(max(s_hi[0], s_hi[1]), max(s_hi[2], s_hi[3]));
  uint32_t below = 0;
  while (lo < hi) {   // block-uniform; each round shrinks [lo, hi] ~256-fold
    const uint64_t scale = ((uint64_t(255) << 32) + 0xFFFFFFFFull) / uint64_t(hi - lo);
    hist[tid] = 0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kSampleVals; ++i)
      if (v[i] >= lo && v[i] <= hi) atomicAdd(&hist[uint32_t((uint64_t(v[i] - lo) * scale) >> 32)], 1u);
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
    BinRange(b, scale, lo, hi);
    __syncthreads();   // hist, wsum and s_bin are rewritten by the next round
  }
  return hi;
}

__global__ void __launch_bounds__(256) topl_sample_kernel(const float* __restrict__ scores, int nl,
                                                          int L, uint32_t lcap, uint32_t cap,
                                                          int32_t* __restrict__ out_leaf,
                                                          float* __restrict__ out_dist,
                                                          TopLTail tail) {
  extern __shared__ uint64_t lds64[];
  uint64_t* sel = lds64;   // [max(cap, lcap)]
  __shared__ uint32_t s_cnt;
  const int tid = threadIdx.x, lane = tid & 63;
  const int qi = blockIdx.x;
  SMX_PHASE(0, qi, 0);
  const float* row = scores + size_t(qi) * nl;
  const uint32_t m = min(uint32_t(L), uint32_t(nl));
  constexpr uint32_t kSamples = 256u * kSampleVals;
  // the samples: 64 runs of 32 consecutive scores (one 128-byte line each)
  // at evenly spaced offsets -- a strided sample would touch every line of
  // the row; leaf order carries no score order, and a skewed sample only
  // costs the fallback, never exactness
  uint32_t v[kSampleVals];
#pragma unroll
  for (int i = 0; i < kSampleVals; ++i) {
    const uint32_t j = uint32_t(tid) + 256u * uint32_t(i);
    const uint32_t run = ((uint64_t(j >> 5) * uint32_t(nl)) / (kSamples / 32u)) & ~31u;
    v[i] = OrderedBits(row[run + (j & 31u)]);
  }
  const uint32_t kk = min(kSamples, uint32_t((uint64_t(3 * m) * kSamples) / (2u * uint32_t(nl))) + 16u);
  SMX_PHASE(0, qi, 1);
  uint32_t T = 0;   // the threshold, set below once the first chunk's loads are issued
  // One sweep of the row, 16 scores per thread per chunk with the next chunk's
  // loads in flight; a wave reserves its chunk's slots with one LDS atomic
  // (per-lane counts up to 16 prefix-summed over five ballots).
  constexpr int kPass = 16;
  constexpr int kChunk = 256 * kPass;
  const uint64_t below = (1ull << lane) - 1ull;
  auto load = [&](uint32_t (&x)[kPass], int c0) {
    // clamped, unconditional loads (a guarded load becomes a branch with its
    // own vmcnt(0) wait); take() masks the positions past nl
#pragma unroll
    for (int i = 0; i < kPass; ++i) x[i] = OrderedBits(row[min(c0 + 256 * i + tid, nl - 1)]);
  };
  auto take = [&](const uint32_t (&x)[kPass], int c0) {
    uint32_t mask = 0;
#pragma unroll
    for (int i = 0; i < kPass; ++i)
      if (c0 + 256 * i + tid < nl && x[i] <= T) mask |= 1u << i;
    const uint32_t n_in = uint32_t(__popc(mask));
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int b = 0; b < 5; ++b) {
      const uint64_t bb = __ballot((n_in >> b) & 1u);
      pre += uint32_t(__popcll(bb & below)) << b;
      tot += uint32_t(__popcll(bb)) << b;
    }
    if (tot == 0) return;   // (wave-uniform)
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&s_cnt, tot);
    uint32_t pos = uint32_t(__shfl(int(base), 0)) + pre;
#pragma unroll
    for (int i = 0; i < kPass; ++i)
      if ((mask >> i) & 1u) {
        if (pos < cap) sel[pos] = (uint64_t(x[i]) << 32) | uint32_t(c0 + 256 * i + tid);
        ++pos;
      }
  };
  uint32_t xa[kPass], xb[kPass];
  load(xa, 0);   // (independent of T: in flight during the threshold rounds)
  T = BlockKthOfSamples(v, kk);
  SMX_PHASE(0, qi, 2);
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  for (int c0 = 0; c0 < nl; c0 += 2 * kChunk) {
    if (c0 + kChunk < nl) load(xb, c0 + kChunk);
    take(xa, c0);
    if (c0 + kChunk >= nl) break;
    if (c0 + 2 * kChunk < nl) load(xa, c0 + 2 * kChunk);
    take(xb, c0 + kChunk);
  }
  __syncthreads();
  SMX_PHASE(0, qi, 3);
  const uint32_t cnt = s_cnt;
  if (cnt < m || cnt > cap) {   // (block-uniform) the sample missed: exact radix select
    __syncthreads();
    TopLGlobalSelect(scores, nl, L, lcap, sel, out_leaf, out_dist, tail);
    return;
  }
  // Exact select and order inside LDS (OrderSmallestByBins: the ~L smallest
  // counting-sorted by bin after the compacted keys, ranked inside their
  // bins, written back over the keys); near-ties or no room after the keys:
  // a bitonic sort of all cnt keys in place (cap is a power of two)
  if (!OrderSmallestByBins<kSelBins>(sel, cnt, m, T, sel + cnt, cap - cnt, sel)) {
    const uint32_t np2 = NextPow2(cnt);
    for (uint32_t i = cnt + tid; i < np2; i += 256) sel[i] = ~0ull;
    __syncthreads();
    BitonicSort(sel, np2);
  }
  const uint64_t* res = sel;
  SMX_PHASE(0, qi, 4);
  TopLFinish(qi, L, m, res, out_leaf, out_dist, tail);
  SMX_PHASE(0, qi, 5);
}

constexpr int kGroups = kWorkGroups;   // XCD groups of the work list

// Work items split a leaf's 32-datapoint tiles into LeafChunks equal chunks
// of at most chunk_tiles tiles (37 tiles at 32 -> 19 + 18, not 32 + 5), so
// that no single wave owns a whole large leaf and no item is a short tail.
__device__ __forceinline__ uint32_t LeafChunks(uint32_t n, uint32_t chunk_tiles) {
  const uint32_t tiles = (n + 31u) / 32u;
  return tiles == 0 ? 1u : (tiles + chunk_tiles - 1) / chunk_tiles;
}
// Tiles [begin, end) of chunk `chunk` of a leaf of n datapoints.
__device__ __forceinline__ uint2 ChunkTiles(uint32_t n, uint32_t chunk_tiles, uint32_t chunk) {
  const uint32_t tiles = (n + 31u) / 32u;
  const uint32_t chunks = tiles == 0 ? 1u : (tiles + chunk_tiles - 1) / chunk_tiles;
  return make_uint2((tiles * chunk) / chunks, (tiles * (chunk + 1)) / chunks);
}

// ---------------------------------------------------------------------------
// Invert (query -> leaves) into (leaf -> queries): InvertCentersToSearch
// (tree_ah_hybrid_residual.cc:610-622).  The top-L kernel gives every
// (query, leaf) pair its rank inside the leaf's list (an atomic on the leaf's
// count) and stores the pair at that slot of the leaf (leaf_pair[leaf *
// stride + rank], stride = the call's query count); the work list turns the
// counts into the scan's work items, each with its query tile's slots; the
// seed kernel writes each pair's record once its query's threshold is
// known.  The order of the queries inside a leaf's list is therefore not the
// query order; nothing depends on it (every result is an exact top-k under a
// total order).
//
// Work items = (leaf, query tile, chunk of <= chunk_tiles tiles), listed
// largest leaf first, cut into 8 XCD groups of consecutive leaves with equal
// MFMA work (exclusive work prefix x 8 / total work), so that all items of a
// leaf share a group.  A leaf's c queries fill c / 32 query tiles of 32
// slots; a remainder of at most 16 queries takes one 16-slot tile (the
// v_smfmac_i32_16x16x128_i8 path: half the MFMA work), a larger one a
// 32-slot tile.  A work unit is a 16-slot tile: a 32-slot item's tiles weigh
// 2 units, a 16-slot item's 1; the shares cut the units, and a tile belongs
// to the share that holds its first unit.
// ---------------------------------------------------------------------------
// 32-slot and 16-slot query tiles of a leaf with c queries (narrow 0:
// 32-slot tiles only; kNarrowOnly: 16-slot tiles only).  (Round 4's mixed
// mode -- a remainder of <= 16 queries in one 16-slot tile, scanned by a
// kernel carrying both paths -- lost to one of these at every density
// measured and was removed: DESIGN.md section 3.)
__device__ __forceinline__ uint2 LeafQueryTiles(uint32_t c, uint32_t narrow) {
  if (narrow == kNarrowOnly) return make_uint2(0u, (c + kNarrowSlots - 1u) / kNarrowSlots);
  return make_uint2((c + kQueriesPerTile - 1u) / kQueriesPerTile, 0u);
}
// Per leaf: its items and units.  Every item also weighs kItemCost units
// ahead of its first tile (its setup: the B fragments, the segment record, the
// claim), so that shares of many small items take fewer tiles: the workgroups'
// ends correlated with their segment counts (0.46, scan stamps).  Same-box
// A/B of 0 / 2 / 4 / 6 / 10 (profiles/r06/ab/item_cost/): 4 took the scan
// alone 66.8 -> 66.2 us (glove), 58.5 -> 57.1 us (SIFT), configs[4] even.
#ifndef SMX_ITEM_COST
#define SMX_ITEM_COST 4
#endif
constexpr uint32_t kItemCost = SMX_ITEM_COST;
__device__ __forceinline__ uint32_t LeafUnits(uint32_t c, uint32_t n, uint32_t chunk_tiles,
                                              uint32_t narrow, uint32_t& items) {
  const uint2 qt = LeafQueryTiles(c, narrow);
  items = (qt.x + qt.y) * LeafChunks(n, chunk_tiles);
  return (2u * qt.x + qt.y) * ((n + 31u) / 32u) + kItemCost * items;
}

// Phase 1 in two multi-block passes over the leaf positions in work order
// (256 positions per block; one single-block pass over 10^4 - 5 * 10^4
// leaves took 0.1 ms of dependent loads): per block the sums of its
// positions' items, units, pairs and code bytes; then every block adds the
// sums of the blocks before it to its own block scan -- each leaf's first
// item (leaf_item0) and first unit (pos_unit0, by position), the 8 groups'
// unit boundaries (gunits[0..8]; gunits[8] = all units) and the totals.
struct WorklistPart {
  unsigned long long items, units, pairs, bytes, tiles16;
};
static_assert(sizeof(WorklistPart) == kWorklistPartWords * 8, "work-list part buffer layout");

__device__ __forceinline__ void PositionWork(const uint32_t* __restrict__ cnt,
                                             const uint32_t* __restrict__ order,
                                             const uint32_t* __restrict__ leaf_size, int nl,
                                             int nb, uint32_t chunk_tiles, uint32_t narrow, int p,
                                             uint32_t& items, uint32_t& units, uint32_t& pairs,
                                             uint64_t& bytes, uint32_t& ntiles16) {
  items = units = pairs = ntiles16 = 0;
  bytes = 0;
  if (p < nl) {
    const uint32_t leaf = order[p];
    const uint32_t c = cnt[size_t(leaf) * kCounterStride], n = leaf_size[leaf];
    units = LeafUnits(c, n, chunk_tiles, narrow, items);
    ntiles16 = LeafQueryTiles(c, narrow).y * ((n + 31u) / 32u);
    pairs = c;
    // algorithmic code bytes: 16 * B * ceil(n / 32) per (query, leaf) pair
    bytes = 16ull * nb * ((n + 31u) / 32u) * c;
  }
}

__global__ void __launch_bounds__(256) worklist_part_kernel(
    const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ order,
    const uint32_t* __restrict__ leaf_size, int nl, int nb, uint32_t chunk_tiles,
    uint32_t narrow, WorklistPart* __restrict__ part) {
  __shared__ unsigned long long red[4][5];
  uint32_t items, units, pairs, t16;
  uint64_t bytes;
  PositionWork(cnt, order, leaf_size, nl, nb, chunk_tiles, narrow,
               int(blockIdx.x * 256 + threadIdx.x), items, units, pairs, bytes, t16);
  unsigned long long v[5] = {items, units, pairs, bytes, t16};
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    for (int off = 32; off > 0; off >>= 1) v[k] += __shfl_xor(v[k], off);
    if (lane == 0) red[wid][k] = v[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    WorklistPart w;
    w.items = red[0][0] + red[1][0] + red[2][0] + red[3][0];
    w.units = red[0][1] + red[1][1] + red[2][1] + red[3][1];
    w.pairs = red[0][2] + red[1][2] + red[2][2] + red[3][2];
    w.bytes = red[0][3] + red[1][3] + red[2][3] + red[3][3];
    w.tiles16 = red[0][4] + red[1][4] + red[2][4] + red[3][4];
    part[blockIdx.x] = w;
  }
}

__global__ void __launch_bounds__(256) worklist_kernel(
    const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ order,
    const uint32_t* __restrict__ leaf_size, int nl, int nb, uint32_t chunk_tiles,
    uint32_t narrow, const WorklistPart* __restrict__ part, uint32_t* __restrict__ leaf_item0,
    uint32_t* __restrict__ pos_unit0, uint32_t* __restrict__ gunits, uint32_t* __restrict__ totals,
    unsigned long long* __restrict__ code_bytes) {
  __shared__ unsigned long long red[4][7];
  __shared__ uint32_t wsum[4], s_units[256];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nblk = int(gridDim.x), blk = int(blockIdx.x);
  // the blocks before this one and all blocks (256 per round)
  unsigned long long bi = 0, bu = 0, ti = 0, tu = 0, tp = 0, tb = 0, tn = 0;
  for (int b = tid; b < nblk; b += 256) {
    const WorklistPart w = part[b];
    if (b < blk) { bi += w.items; bu += w.units; }
    ti += w.items; tu += w.units; tp += w.pairs; tb += w.bytes; tn += w.tiles16;
  }
  unsigned long long v[7] = {bi, bu, ti, tu, tp, tb, tn};
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    for (int off = 32; off > 0; off >>= 1) v[k] += __shfl_xor(v[k], off);
    if (lane == 0) red[wid][k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 7; ++k) v[k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
  const uint32_t total_w = uint32_t(v[3]);
  if (blk == 0 && tid == 0) {
    totals[0] = uint32_t(v[4]);
    totals[1] = uint32_t(v[2]);
    totals[2] = total_w;
    totals[kTotalsTiles16] = uint32_t(v[6]);
    code_bytes[0] = v[5];
  }
  const int p = blk * 256 + tid;
  uint32_t items, units, pairs, t16;
  uint64_t bytes;
  PositionWork(cnt, order, leaf_size, nl, nb, chunk_tiles, narrow, p, items, units, pairs, bytes,
               t16);
  const uint32_t inc_i = BlockInclusiveScan256(items, wsum);
  __syncthreads();   // wsum is reused
  const uint32_t inc_u = BlockInclusiveScan256(units, wsum);
  s_units[tid] = units;
  __syncthreads();
  if (p >= nl) return;
  const uint32_t ex_i = uint32_t(v[0]) + inc_i - items;
  const uint32_t ex_u = uint32_t(v[1]) + inc_u - units;
  leaf_item0[order[p]] = ex_i;
  pos_unit0[p] = ex_u;
  // group boundaries: the first position whose exclusive unit prefix puts it
  // in group g (g = 8 * prefix / total); the groups are contiguous ranges
  const uint64_t wdiv = max(1u, total_w);
  auto group_of = [&](uint32_t excl_w) {
    return int(min<uint64_t>(kGroups - 1, (uint64_t(kGroups) * excl_w) / wdiv));
  };
  const int gp = group_of(ex_u);
  int prev = -1;
  if (p > 0) {
    const uint32_t prev_units = tid > 0 ? s_units[tid - 1] : [&] {
      uint32_t it, un, pa, t1;
      uint64_t by;
      PositionWork(cnt, order, leaf_size, nl, nb, chunk_tiles, narrow, p - 1, it, un, pa, by, t1);
      return un;
    }();
    prev = group_of(ex_u - prev_units);
  }
  for (int gg = prev + 1; gg <= gp; ++gg) gunits[gg] = ex_u;
  if (p == nl - 1) {
    for (int gg = gp + 1; gg <= kGroups; ++gg) gunits[gg] = total_w;
    pos_unit0[nl] = total_w;
  }
}

// The scan workgroups whose share starts in position p's units [ua, ub)
// (leaf size n, c queries, first item item0): workgroup i of group g (i % 8
// == g) takes the units [U0 + span * k / nw, U0 + span * (k + 1) / nw) of
// its group, k = i / 8 of the group's nw; its start {item, first tile,
// units, position}: the first tile whose first unit is in the share (a
// share that begins inside a 32-slot tile starts at the next tile, one unit
// later).  Threads first, first + step, ... of the caller take the k in turn.
__device__ void WaveStarts(const WorklistArgs& w, int p, const uint32_t* gunits, uint32_t item0,
                           uint32_t ua, uint32_t ub, uint32_t n, uint32_t c, uint32_t first,
                           uint32_t step) {
  if (ua >= ub) return;
  const uint32_t chunk_tiles = w.chunk_tiles;
  const uint32_t chunks = LeafChunks(n, chunk_tiles);
  const uint2 qt = LeafQueryTiles(c, w.narrow);
  const uint32_t wdiv = max(1u, gunits[kGroups]);
  const int g = int(min<uint64_t>(kGroups - 1, (uint64_t(kGroups) * ua) / wdiv));
  const uint32_t nw = uint32_t(w.grid - g + kGroups - 1) / kGroups;
  const uint32_t U0 = gunits[g], span = gunits[g + 1] - U0;
  // the first k with U0 + span*k/nw >= ua
  uint32_t k = uint32_t((uint64_t(ua - U0) * nw + span - 1) / span);
  const uint32_t tiles = (n + 31u) / 32u;
  for (k += first;; k += step) {
    if (k >= nw) break;
    const uint32_t us = U0 + uint32_t((uint64_t(span) * k) / nw);
    if (us >= ub) break;
    const uint32_t ue = U0 + uint32_t((uint64_t(span) * (k + 1)) / nw);
    const uint32_t off = us - ua;
    // the query tile, then the item (chunk) holding unit `off`: per item
    // kItemCost units, then its tiles (2 units each in a 32-slot tile, 1 in a
    // 16-slot one)
    const uint32_t per32 = 2u * tiles + kItemCost * chunks;
    uint32_t q, r, wt;
    if (off < per32 * qt.x) {
      q = off / per32;
      r = off - q * per32;
      wt = 2u;
    } else {
      const uint32_t per16 = tiles + kItemCost * chunks, o16 = off - per32 * qt.x;
      q = qt.x + o16 / per16;
      r = o16 - (q - qt.x) * per16;
      wt = 1u;
    }
    uint32_t ch = 0;
    uint2 cr = ChunkTiles(n, chunk_tiles, 0);
    while (r >= kItemCost + wt * (cr.y - cr.x)) {
      r -= kItemCost + wt * (cr.y - cr.x);
      cr = ChunkTiles(n, chunk_tiles, ++ch);
    }
    // the first tile whose first unit is at or after `off`, and the units
    // between them (not the share's)
    uint32_t j, skip;
    if (r <= kItemCost) {
      j = cr.x;
      skip = kItemCost - r;
    } else {
      const uint32_t m = (r - kItemCost + wt - 1u) / wt;
      j = cr.x + m;
      skip = wt * m - (r - kItemCost);
      if (j == cr.y) {   // the next item's first tile (the leaf's next query tile,
        skip += kItemCost;   // or the next leaf's first item)
        if (++ch == chunks) {
          ch = 0;
          ++q;
        }
        j = q < qt.x + qt.y ? ChunkTiles(n, chunk_tiles, ch).x : 0u;
      }
    }
    const uint32_t units = ue - us > skip ? ue - us - skip : 0u;
    SMX_CHECK(item0 + q * chunks + ch, w.bd.items + 1, "wave start item");
    SMX_GUARD(kGroups * k + g, w.bd.grid, "wave start")
    w.wave_start[kGroups * k + g] = make_uint4(item0 + q * chunks + ch, j, units, uint32_t(p));
  }
}

// Phase 2 (64 lanes per leaf position): the leaf's work items (16-slot query
// tiles marked narrow), each with its query tile's leaf slots, and the start
// of every scan wave whose share begins inside this leaf.
// (item0 = the leaf's first item, [ua, ub) = its units, gunits = the 8
// groups' unit boundaries)
__device__ void ItemsCore(const WorklistArgs& w, int p, int lane, const uint32_t* gunits,
                          uint32_t item0, uint32_t ua, uint32_t ub) {
  if (p == 0) {
    // the waves of groups without units get an empty share (the other
    // positions write every other wave's share)
    for (int i = lane; i < w.grid; i += 64) {
      const int g = i & (kGroups - 1);
      if (gunits[g + 1] == gunits[g]) {
        SMX_GUARD(i, w.bd.grid, "empty wave start") w.wave_start[i] = make_uint4(0, 0, 0, 0);
      }
    }
  }
  const uint32_t chunk_tiles = w.chunk_tiles;
  const uint32_t leaf = w.order[p];
  const uint32_t c = w.cnt[size_t(leaf) * kCounterStride], n = w.leaf_size[leaf];
  const uint32_t chunks = LeafChunks(n, chunk_tiles);
  const uint2 qts = LeafQueryTiles(c, w.narrow);
  const uint32_t qt = qts.x + qts.y;
  const uint64_t toff = w.tile_off[leaf], moff = w.member_off[leaf];
  for (uint32_t u = lane; u < qt * chunks; u += 64) {
    const uint2 cr = ChunkTiles(n, chunk_tiles, u % chunks);
    const uint32_t q = u / chunks;
    // the query tile's ranks: 32-slot tiles first, then the 16-slot ones
    const uint32_t r0 = q < qts.x ? q * uint32_t(kQueriesPerTile)
                                  : qts.x * uint32_t(kQueriesPerTile) + (q - qts.x) * uint32_t(kNarrowSlots);
    const uint32_t width = q < qts.x ? uint32_t(kQueriesPerTile) : uint32_t(kNarrowSlots);
    WorkItem it;
    it.leaf = leaf | (q >= qts.x ? kItemNarrow : 0u);
    it.n = n;
    it.j0 = cr.x;
    it.jend = cr.y;
    it.tile_off = toff;
    it.member_off = moff;
    it.slot0 = leaf * w.slot_stride + r0;
    it.nslots = min(width, c - r0);
    SMX_GUARD(item0 + u, w.bd.items, "work item") w.work[item0 + u] = it;
  }
  WaveStarts(w, p, gunits, item0, ua, ub, n, c, uint32_t(lane), 64u);
}

__global__ void __launch_bounds__(64) items_kernel(WorklistArgs w) {
  const int p = int(blockIdx.x);
  ItemsCore(w, p, int(threadIdx.x), w.gunits, w.leaf_item0[w.order[p]], w.pos_unit0[p],
            w.pos_unit0[p + 1]);
}

// The work list without extra launches (nl <= kFusedWorklistLeaves): extra
// blocks of the seed launch, each of which scans ALL positions redundantly
// (16 per thread: two rounds of independent loads, then block scans) and
// builds the items of its own kWlPosPerBlock positions, one wave each.  No
// block waits for another; block 0 also writes the global prefixes (the pair
// scatter reads leaf_item0) and totals.  The seed blocks neither read nor
// write anything these touch.
constexpr int kWlPerThread = kFusedWorklistLeaves / 256;
#ifndef SMX_WL_POS
#define SMX_WL_POS 4
#endif
constexpr int kWlPosPerBlock = SMX_WL_POS;

__device__ void WorklistFusedBlock(const WorklistArgs& w, int b) {
  __shared__ uint32_t wsum[4], s_gunits[kGroups + 1], s_last_un[256];
  __shared__ uint32_t s_ex_i[kWlPosPerBlock], s_ex_u[kWlPosPerBlock + 1];
  __shared__ unsigned long long red[4][3];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // (phase stamps of block 0: start, leaf_item0 written, end)
  if (b == 0) SMX_PHASE(1, kPhaseQueries - 1, 0);
  // per thread ceil(nl / 256) consecutive positions (not kWlPerThread: at
  // glove's 1000 leaves 4 per thread instead of 16 on a quarter of them)
  const int nl = w.nl, per = (nl + 255) / 256, p0 = tid * per;
  const int pb = b * kWlPosPerBlock, pe = min(nl, pb + kWlPosPerBlock);
  uint32_t leafv[kWlPerThread], itv[kWlPerThread], unv[kWlPerThread];
#pragma unroll
  for (int k = 0; k < kWlPerThread; ++k) leafv[k] = k < per && p0 + k < nl ? w.order[p0 + k] : 0u;
  uint32_t ti = 0, tu = 0;
  unsigned long long tp = 0, tb = 0, tn = 0;
#pragma unroll
  for (int k = 0; k < kWlPerThread; ++k) {
    itv[k] = unv[k] = 0;
    if (k < per && p0 + k < nl) {
      const uint32_t leaf = leafv[k];
      const uint32_t c = w.cnt[size_t(leaf) * kCounterStride], n = w.leaf_size[leaf];
      unv[k] = LeafUnits(c, n, w.chunk_tiles, w.narrow, itv[k]);
      tp += c;
      tb += 16ull * w.nb * ((n + 31u) / 32u) * c;   // algorithmic code bytes
      if (w.narrow) tn += LeafQueryTiles(c, w.narrow).y * ((n + 31u) / 32u);
    }
    ti += itv[k];
    tu += unv[k];
  }
  uint32_t last_un = 0;   // the units of this thread's last position
#pragma unroll
  for (int k = 0; k < kWlPerThread; ++k)
    if (k == per - 1) last_un = unv[k];
  s_last_un[tid] = last_un;
  const uint32_t inc_i = BlockInclusiveScan256(ti, wsum);
  __syncthreads();   // wsum is reused
  const uint32_t inc_u = BlockInclusiveScan256(tu, wsum);
  const uint32_t total_w = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  if (b == 0) {
    unsigned long long v[3] = {tp, tb, tn};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      for (int off = 32; off > 0; off >>= 1) v[k] += __shfl_xor(v[k], off);
      if (lane == 0) red[wid][k] = v[k];
    }
  }
  __syncthreads();   // s_last_un, red
  if (b == 0 && tid == 255) {
    w.totals[0] = uint32_t(red[0][0] + red[1][0] + red[2][0] + red[3][0]);
    w.totals[1] = inc_i;   // thread 255's inclusive item prefix = all items
    w.totals[2] = total_w;
    w.totals[kTotalsTiles16] = uint32_t(red[0][2] + red[1][2] + red[2][2] + red[3][2]);
    w.code_bytes[0] = red[0][1] + red[1][1] + red[2][1] + red[3][1];
  }
  const uint64_t wdiv = max(1u, total_w);
  auto group_of = [&](uint32_t excl_w) {
    return int(min<uint64_t>(kGroups - 1, (uint64_t(kGroups) * excl_w) / wdiv));
  };
  uint32_t ei = inc_i - ti, eu = inc_u - tu;
  uint32_t prev_un = tid > 0 ? s_last_un[tid - 1] : 0u;
#pragma unroll
  for (int k = 0; k < kWlPerThread; ++k) {
    const int p = p0 + k;
    if (k < per && p < nl) {
      if (b == 0) {
        w.leaf_item0[leafv[k]] = ei;
        w.pos_unit0[p] = eu;
      }
      if (p >= pb && p < pe) {
        s_ex_i[p - pb] = ei;
        s_ex_u[p - pb] = eu;
      }
      if (p == pe) s_ex_u[pe - pb] = eu;
      const int gp = group_of(eu);
      const int prev = p > 0 ? group_of(eu - prev_un) : -1;
      for (int gg = prev + 1; gg <= gp; ++gg) {
        s_gunits[gg] = eu;
        if (b == 0) w.gunits[gg] = eu;
      }
      if (p == nl - 1) {
        for (int gg = gp + 1; gg <= kGroups; ++gg) {
          s_gunits[gg] = total_w;
          if (b == 0) w.gunits[gg] = total_w;
        }
        if (b == 0) w.pos_unit0[nl] = total_w;
        if (pe == nl && pb < nl) s_ex_u[pe - pb] = total_w;
      }
    }
    ei += itv[k];
    eu += unv[k];
    prev_un = unv[k];
  }
  if (b == 0) SMX_PHASE(1, kPhaseQueries - 1, 1);   // (leaf_item0 written)
  __syncthreads();
  for (int p = pb + wid; p < pe; p += 4)
    ItemsCore(w, p, lane, s_gunits, s_ex_i[p - pb], s_ex_u[p - pb], s_ex_u[p - pb + 1]);
  if (b == 0) SMX_PHASE(1, kPhaseQueries - 1, 2);
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
    const uint32_t by = (codes[s >> 3] >> (8 * ((s >> 1) & 3))) & 0xFFu;
    const uint32_t x = (s & 1) ? CodePairHi(by) : CodePairLo(by);
    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(OneHot16(8u * x), frag[s], acc, 0, 0, 0);
  }
  return acc;
}

// NW code words as one vector value (dword-aligned): a ring slot kept as a
// register tuple, so that the allocator does not split it across a loop
// back edge (a split copies the words -- and waits for their load).
template <int N>
using CodeVec = uint32_t __attribute__((ext_vector_type(N), aligned(4)));

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
#ifndef SMX_SEED_U
#define SMX_SEED_U 2
#endif
constexpr int kSeedPerThread = kSeedKeys / 256;
constexpr uint32_t kSeedCap = 256u * kSeedPerThread;
constexpr int kSeedMaxLeaves = 64;   // one wave of leaf slots
constexpr int kSeedSel = 1024;       // values under the minima bound ranked exactly

// The rank of `key` among the 256 keys the threads of a 256-thread block
// hold (distinct keys).  Each wave sorts its 64 keys in registers (bitonic,
// lane exchanges, no barrier) into sbuf[64 w ..]; a key's rank is its place
// in its wave's order plus, per other wave, the number of that wave's keys
// below it (binary search of the sorted run).  Block-wide (every thread
// calls); sbuf holds 256 keys.
// The value of lane (lane ^ J): DPP quad permutes for J = 1, 2, ds_swizzle
// (bit-mask mode, no LDS access) for J = 4, 8, 16, one ds_bpermute for 32.
template <int J>
__device__ __forceinline__ uint32_t LaneXor(uint32_t v) {
  if constexpr (J == 1)
    return uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0xB1, 0xF, 0xF, false));
  else if constexpr (J == 2)
    return uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x4E, 0xF, 0xF, false));
  else if constexpr (J <= 16)
    return uint32_t(__builtin_amdgcn_ds_swizzle(int(v), 0x1F | (J << 10)));
  else
    return uint32_t(__shfl_xor(int(v), J));
}

template <int K, int J>
__device__ __forceinline__ void BitonicStep(uint64_t& v, int lane) {
  const uint32_t lo = LaneXor<J>(uint32_t(v));
  const uint32_t hi = LaneXor<J>(uint32_t(v >> 32));
  const uint64_t o = (uint64_t(hi) << 32) | lo;
  const bool up = (lane & K) == 0, low = (lane & J) == 0;
  v = (low == up) ? (o < v ? o : v) : (o > v ? o : v);
  if constexpr (J > 1) BitonicStep<K, J / 2>(v, lane);
}

template <int K>
__device__ __forceinline__ void BitonicStages(uint64_t& v, int lane) {
  BitonicStep<K, K / 2>(v, lane);
  if constexpr (K < 64) BitonicStages<K * 2>(v, lane);
}

__device__ uint32_t BlockRank256(uint64_t key, uint64_t* sbuf) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint64_t v = key;
  BitonicStages<2>(v, lane);
  sbuf[threadIdx.x] = v;
  __syncthreads();
  uint32_t r = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const uint64_t* run = sbuf + 64 * w;
    if (w == wid) continue;
    uint32_t b = 0;   // keys of run w below key: the first b with run[b] >= key
#pragma unroll
    for (uint32_t step = 32; step > 0; step >>= 1)
      if (run[b + step - 1] < key) b += step;
    r += b + (run[b] < key ? 1u : 0u);   // b = 63: all 64 below?
  }
  // the key's place in its own wave's sorted run
  const uint64_t* own = sbuf + 64 * wid;
  uint32_t b = 0;
#pragma unroll
  for (uint32_t step = 32; step > 0; step >>= 1)
    if (own[b + step - 1] < key) b += step;
  b += own[b] < key ? 1u : 0u;
  __syncthreads();   // sbuf is rewritten by the next call
  return r + b;
}

// The k-th smallest (1-based, k <= 64) of the 64 lanes' values of one wave:
// the answer's bits from the top, each by one ballot count (bit b is 1 when
// fewer than k values lie at or below the prefix with bit b clear and every
// lower bit set).  No LDS, no barrier; the loop is wave-uniform.
// The bits are searched from the highest one in which the values' range
// [lo, hi] (wave-uniform, the k-th inside it) differs: the ones above are
// the prefix every value shares.
__device__ __forceinline__ uint32_t WaveKth(uint32_t v, uint32_t k, uint32_t lo, uint32_t hi) {
  if (lo == hi) return lo;
  const int top = 31 - __clz(lo ^ hi);
  uint32_t x = lo & ~((top == 31) ? 0xFFFFFFFFu : ((2u << top) - 1u));
  for (int b = top; b >= 0; --b) {
    const uint32_t t = x | ((1u << b) - 1u);
    if (uint32_t(__popcll(__ballot(v <= t))) < k) x |= 1u << b;
  }
  return x;
}

__device__ __forceinline__ uint32_t WaveMin(uint32_t v) {
  for (int off = 32; off > 0; off >>= 1) v = min(v, uint32_t(__shfl_xor(int(v), off)));
  return v;
}
__device__ __forceinline__ uint32_t WaveMax(uint32_t v) {
  for (int off = 32; off > 0; off >>= 1) v = max(v, uint32_t(__shfl_xor(int(v), off)));
  return v;
}

// The threshold key of a query from its seed distances (ordered bits, 16
// per thread of a 256-thread block, 0xFFFFFFFF = none; the caller has
// checked that at least kk values are real): (v << 32 | 0xFFFFFFFF) for v
// the exact kk-th smallest value, which admits every candidate at that
// distance.  Block-wide (every thread calls; the key is returned to all).
// kk <= 256: each wave's ceil(kk/4)-th smallest per-thread minimum (WaveKth)
// -- every wave then holds at least ceil(kk/4) values at or below it, so the
// largest of the four bounds the kk-th value from above -- then the values
// at or below that bound (~1.3-1.6 kk) compacted into LDS by ballot slots and
// the exact kk-th of them found by wave 0 alone (WaveKthN).  Otherwise, or
// when more than kSeedSel values pass the bound, the bits of the kk-th value
// by block-wide ballot counts (one barrier per bit).  (Round 5: counting
// ranks of the 256 minima and of the compacted keys, 7.2 us p50 per block.)
__device__ uint64_t ThresholdOfVals(const uint32_t (&vals)[kSeedPerThread], uint32_t kk) {
  __shared__ uint32_t sval[kSeedSel];
  __shared__ uint32_t s_wb[4], s_wlo[4], s_wc[2][4], s_cnt, s_x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (kk <= 256u) {
    uint32_t vmin = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i < kSeedPerThread; ++i) vmin = min(vmin, vals[i]);
    // the wave's bound: none (MAX) when fewer than k of its minima are real
    const uint32_t k4 = (kk + 3u) >> 2;
    const uint32_t wlo = WaveMin(vmin);
    uint32_t wk = 0xFFFFFFFFu;
    if (uint32_t(__popcll(__ballot(vmin != 0xFFFFFFFFu))) >= k4)
      wk = WaveKth(vmin, k4, wlo, WaveMax(vmin != 0xFFFFFFFFu ? vmin : 0u));
    if (lane == 0) {
      s_wb[wid] = wk;
      s_wlo[wid] = wlo;
    }
    if (tid == 0) s_cnt = 0;
    __syncthreads();
    const uint32_t thi = max(max(s_wb[0], s_wb[1]), max(s_wb[2], s_wb[3]));
    const uint32_t blo = min(min(s_wlo[0], s_wlo[1]), min(s_wlo[2], s_wlo[3]));
    // compaction: the wave's count by ballots, one LDS atomic per wave for
    // its base, then the slots again by ballots (no per-value registers)
    uint32_t n = 0;
#pragma unroll
    for (int i = 0; i < kSeedPerThread; ++i) n += uint32_t(__popcll(__ballot(vals[i] <= thi)));
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&s_cnt, n);
    base = uint32_t(__builtin_amdgcn_readfirstlane(int(base)));
#pragma unroll
    for (int i = 0; i < kSeedPerThread; ++i) {
      const bool in = vals[i] <= thi;
      const uint64_t m = __ballot(in);
      const uint32_t pos = base + __builtin_amdgcn_mbcnt_hi(
                                      uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
      if (in && pos < uint32_t(kSeedSel)) sval[pos] = vals[i];
      base += uint32_t(__popcll(m));
    }
    __syncthreads();
    const uint32_t c = s_cnt;
    if (c <= uint32_t(kSeedSel)) {
      // wave 0: the exact kk-th of the c compacted values, held in registers
      // (4 per lane; above 256 values, 16 per lane), the bits by ballots
      if (wid == 0) {
        // the kk-th lies in [blo, thi] (blo = the smallest value; at least kk
        // values are at or below thi): the bits below their highest
        // differing one
        const int top = blo == thi ? -1 : 31 - __clz(blo ^ thi);
        uint32_t x = top < 0 ? blo : blo & ~((top == 31) ? 0xFFFFFFFFu : ((2u << top) - 1u));
        if (c <= 256u) {
          uint32_t v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t j = uint32_t(lane) + 64u * uint32_t(i);
            v[i] = j < c ? sval[j] : 0xFFFFFFFFu;
          }
          for (int b = top; b >= 0; --b) {
            const uint32_t t = x | ((1u << b) - 1u);
            const uint32_t cnt = uint32_t(__popcll(__ballot(v[0] <= t))) +
                                 uint32_t(__popcll(__ballot(v[1] <= t))) +
                                 uint32_t(__popcll(__ballot(v[2] <= t))) +
                                 uint32_t(__popcll(__ballot(v[3] <= t)));
            if (cnt < kk) x |= 1u << b;
          }
        } else {
          uint32_t v[kSeedSel / 64];
#pragma unroll
          for (int i = 0; i < kSeedSel / 64; ++i) {
            const uint32_t j = uint32_t(lane) + 64u * uint32_t(i);
            v[i] = j < c ? sval[j] : 0xFFFFFFFFu;
          }
          for (int b = top; b >= 0; --b) {
            const uint32_t t = x | ((1u << b) - 1u);
            uint32_t cnt = 0;
#pragma unroll
            for (int i = 0; i < kSeedSel / 64; ++i) cnt += uint32_t(__popcll(__ballot(v[i] <= t)));
            if (cnt < kk) x |= 1u << b;
          }
        }
        if (lane == 0) s_x = x;
      }
      __syncthreads();
      return (uint64_t(s_x) << 32) | 0xFFFFFFFFull;
    }
  }
  // the bits of the kk-th value by block-wide counts (s_wc double-buffered by
  // the bit's parity: a wave rewrites one only after the next barrier, which
  // every wave reaches after reading it)
  uint32_t x = 0;
  for (int b = 31; b >= 0; --b) {
    const uint32_t t = x | ((1u << b) - 1u);
    uint32_t cnt = 0;
#pragma unroll
    for (int i = 0; i < kSeedPerThread; ++i) cnt += uint32_t(__popcll(__ballot(vals[i] <= t)));
    if (lane == 0) s_wc[b & 1][wid] = cnt;
    __syncthreads();
    const uint32_t tot = s_wc[b & 1][0] + s_wc[b & 1][1] + s_wc[b & 1][2] + s_wc[b & 1][3];
    if (tot < kk) x |= 1u << b;
  }
  return (uint64_t(x) << 32) | 0xFFFFFFFFull;
}

// Seed scoring tables: per code byte j of half h two 64-entry byte tables,
// each indexed by six bits of the byte and holding one block's LUT entry
// biased by +128 (EncodeCodePair: bits 0-1 = g0, 2-3 = g1, 4-5 = p0, 6-7 =
// p1 for the blocks x0 = 4j + h = 4 g0 + p0 and x1 = 4j + 2 + h = 4 g1 + p1):
//   lo table, index byte & 0x3F = g0 | g1 << 2 | p0 << 4 -> LUT[x0];
//   hi table, index byte >> 2   = g1 | p0 << 2 | p1 << 4 -> LUT[x1];
// in both, entry i = LUT[4 (i & 3) + ((i >> 4) & 3)].  A table is 16 dwords
// in 16 distinct banks and every lane of one read uses the same table, so
// the reads are conflict-free: 2 LDS cycles per lookup, two lookups per code
// byte.  (Round 5's 256-entry int16 byte-pair tables: one lookup per byte
// but ~2.8-way bank conflicts of the random 16-bit reads -- 5.6 cycles per
// byte; 40% of the seed's LDS-active cycles were conflicts.)
template <int K>
__device__ __forceinline__ uint32_t SeedRowSum(const uint8_t* ntab, const uint32_t* c0,
                                               const uint32_t* c1) {
  constexpr int NB = (K + 1) / 2;
  uint32_t acc = 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t* c = h ? c1 : c0;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const uint32_t w = c[j >> 2];
      const uint32_t lo = (w >> (8 * (j & 3))) & 0x3Fu;
      const uint32_t hi = (w >> (8 * (j & 3) + 2)) & 0x3Fu;
      const uint8_t* t = ntab + ((h * NB + j) * 2) * 64;
      acc += uint32_t(t[lo]) + uint32_t(t[64 + hi]);
    }
  }
  return acc;
}

// The threshold key of query qi from its seed leaves, or kNoThreshold (no
// bound); block-wide (256 threads, all call; the value is returned to all).
// Rows: the seed leaves' rows numbered across the leaves (a prefix sum of
// their sizes), at most a.seed_rows (<= kSeedCap) of them; thread t scores
// numbers t, t + 256, ...: groups of U rows whose code loads are issued one
// group ahead of the scoring.
template <int K>
__device__ uint64_t SeedTau(const SeedArgs& a, int qi) {
  constexpr int NW = ((((K + 1) / 2) + 3) / 4);
  constexpr int W = 4 * NW;
  constexpr int U = SMX_SEED_U;   // rows per group
  constexpr int G = kSeedPerThread / U;
  constexpr int NB = (K + 1) / 2;   // code bytes per half holding steps < K
  static_assert(kSeedPerThread % U == 0, "whole groups");
  __shared__ __align__(16) int8_t lut[2 * K * 16];
  __shared__ __align__(16) uint8_t ntab[2 * NB * 2 * 64];
  __shared__ uint32_t s_start[kSeedMaxLeaves + 1];
  __shared__ uint64_t s_tile0[kSeedMaxLeaves];
  __shared__ float s_bias[kSeedMaxLeaves];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  SMX_PHASE(1, qi, 0);
  if (a.seed <= 0) return kNoThreshold;
  static_assert(2 * K * 16 / 4 <= 256, "one LUT word per thread");
  if (tid < 2 * K * 16 / 4)
    reinterpret_cast<uint32_t*>(lut)[tid] =
        reinterpret_cast<const uint32_t*>(a.lut + size_t(qi) * LutRows(K) * 16)[tid];
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
  SMX_PHASE(1, qi, 1);
  const uint32_t total = min(s_start[kSeedMaxLeaves], min(uint32_t(a.seed_rows), kSeedCap));
  const uint32_t kk = uint32_t(a.kk);
  if (kk == 0 || total < kk) return kNoThreshold;   // no bound: the threshold stays open
  // the tables, one dword (four entries) per store: table tb = (h, j, part),
  // entries i0..i0+3 share (i >> 4) & 3 = p and take LUT[4 k + p], k = 0..3
  for (int d = tid; d < 2 * NB * 2 * 16; d += 256) {
    const int tb = d >> 4, i0 = (d & 15) * 4, p = (i0 >> 4) & 3;
    const int hj = tb >> 1, part = tb & 1, h = hj / NB, j = hj % NB;
    const int s = 2 * j + part;   // MFMA step: LUT row 2 s + h = block 4 j + 2 part + h
    uint32_t word = 0x80808080u;  // zero rows (steps >= K) biased
    if (s < K) {
      const int8_t* row = lut + (2 * s + h) * 16 + p;
      word = (uint32_t(uint8_t(row[0] ^ 0x80))) | (uint32_t(uint8_t(row[4] ^ 0x80)) << 8) |
             (uint32_t(uint8_t(row[8] ^ 0x80)) << 16) | (uint32_t(uint8_t(row[12] ^ 0x80)) << 24);
    }
    reinterpret_cast<uint32_t*>(ntab)[d] = word;
  }
  // the leaf boundaries as uniform values (the common seed of <= 4 leaves;
  // more leaves take the LDS walk)
  const uint32_t st1 = s_start[1], st2 = s_start[2], st3 = s_start[3];
  __syncthreads();

  // row -> its code bytes (both halves) and its leaf
  auto row_ptr = [&](uint32_t g, int& r) -> const uint8_t* {
    if (nseed <= 4) {
      r = (g >= st1 ? 1 : 0) + (g >= st2 ? 1 : 0) + (g >= st3 ? 1 : 0);
      r = min(r, nseed - 1);
    } else {
      while (g >= s_start[r + 1]) ++r;
    }
    const uint32_t dp = g - s_start[r];
    SMX_CHECK(s_tile0[r] + (dp >> 5), a.bd.tiles, "seed tile");
    return a.tiles + ((s_tile0[r] + (dp >> 5)) * 64 + (dp & 31)) * W;
  };
  constexpr uint32_t kBias = 2u * NB * 2u * 128u;   // the tables' +128 per lookup
  uint32_t vals[kSeedPerThread];
  uint32_t cb[2][U][2 * NW];   // code words of two groups (double buffer)
  int rb[2][U];
  int r = 0;   // seed leaf of this thread's current number (numbers only grow)
  auto load = [&](int g0, int buf) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t g = min(uint32_t(tid) + 256u * uint32_t(g0 * U + u), total - 1);
      const uint8_t* t0 = row_ptr(g, r);
      rb[buf][u] = r;
      LoadCodes<K>(t0, cb[buf][u]);
      LoadCodes<K>(t0 + 32 * W, cb[buf][u] + NW);
    }
  };
  load(0, 0);
#pragma unroll
  for (int g0 = 0; g0 < G; ++g0) {
    const int buf = g0 & 1;
    if (uint32_t(g0) * U * 256u < total) {   // block-uniform
      if (g0 + 1 < G && uint32_t(g0 + 1) * U * 256u < total) load(g0 + 1, buf ^ 1);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int acc = int(SeedRowSum<K>(ntab, cb[buf][u], cb[buf][u] + NW)) - int(kBias);
        const uint32_t g = uint32_t(tid) + 256u * uint32_t(g0 * U + u);
        vals[g0 * U + u] =
            g < total ? OrderedBits(DistOf(acc, inv, s_bias[rb[buf][u]])) : 0xFFFFFFFFu;
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) vals[g0 * U + u] = 0xFFFFFFFFu;   // no datapoint
    }
  }
  SMX_PHASE(1, qi, 2);
  const uint64_t T = ThresholdOfVals(vals, kk);
  SMX_PHASE(1, qi, 3);
  return T;
}

// Per query: its threshold key (SeedTau), then every one of its (query,
// leaf) pairs' records -- the query, the pair's bias, the query's
// 1/multiplier and the pair's sum limit: the largest LUT16 sum whose distance
// can pass the threshold (d is monotone in the sum), so the scan's setup needs
// neither the threshold nor a search.  The scan finds a pair through its
// leaf's slot (leaf_pair, written by the top-L kernel with the rank): the
// inversion of InvertCentersToSearch (tree_ah_hybrid_residual.cc:610-622)
// without a scatter launch.  Blocks from nq on build the work list
// (WorklistFusedBlock).  (Work-list blocks first, with the old per-item
// record scatter in the seed blocks behind a release flag from block 0,
// measured slower: block 0 published its prefixes only 48.7 us after its
// start beside the seed blocks -- tools/phase_stamps.py)
template <int K>
__global__ void __launch_bounds__(256, 4) seed_tau_kernel(SeedArgs a, WorklistArgs w, int nq) {
  const int qi = blockIdx.x;
  if (qi >= nq) {   // the fused work-list blocks
    WorklistFusedBlock(w, qi - nq);
    return;
  }
  const uint64_t tau = SeedTau<K>(a, qi);
  if (threadIdx.x == 0) a.tau_key[qi] = tau;
  const float inv = a.inv[qi];
  for (int i = threadIdx.x; i < a.L; i += 256) {
    const size_t p = size_t(qi) * a.L + size_t(i);
    if (a.topl_leaf[p] < 0) continue;
    ItemLane v;
    v.qid = uint32_t(qi);
    v.bias = a.residual ? a.topl_dist[p] : 0.0f;
    v.inv = inv;
    v.amax = tau == kNoThreshold ? 128 * a.nb
                                 : SumLimit(FromOrdered(uint32_t(tau >> 32)), inv, v.bias,
                                            -128 * a.nb, 128 * a.nb);
    SMX_GUARD(p, a.bd.pairs, "pair record") a.pair_rec[p] = v;
  }
}

// One tile: S[dp][q] for 32 datapoints x 32 queries with the item's B
// fragments (LUT rows) held in registers, on the 2:4 structured-sparse MFMA
// (v_smfmac_i32_32x32x64_i8:
// K = 64 at the cycles of the dense K = 32 form, measured by
// tools/smfmac_probe.hip).  A one-hot row is exactly 2:4 sparse -- at most
// one non-zero in every group of 4 centers -- so the sparse instruction
// computes the whole dense product.  Operand layout (tools/smfmac_probe2/3):
// lane (r, hA) of A holds 16 compressed values, j < 8 for B lanes (c, 0) and
// j >= 8 for B lanes (c, 1), two per group of 4, value j selecting B byte
// 16*hA + 4*((j % 8) / 2) + idx_j (idx_j = bits [2j, 2j+2) of the index
// VGPR).  Step s covers blocks 4s + 2*hB + hA: lane (r, hA) needs the
// codes of blocks 4s + hA and 4s + 2 + hA = nibbles 2s and 2s + 1 of its
// stream (code byte s, EncodeCodePair), and B lane (c, hB) the LUT rows
// 4s + 2hB and 4s + 2hB + 1 (32 contiguous bytes).  Per step two
// conflict-free LDS reads (16-entry tables spanning distinct banks; equal
// entries broadcast): the compressed values from the byte's group nibble
// (a 1 at value 2*(x0 >> 2) and 8 + 2*(x1 >> 2)) and the index word from its
// position nibble (x0 & 3 in fields 0..7, x1 & 3 in fields 8..15), each
// address two VALU ops; a 256-entry table of both spent 60% of the LDS
// cycles in bank conflicts.
#ifndef SMX_POS_B64
#define SMX_POS_B64 0
#endif
// SMX_POS_VALU: the index word built by VALU from the code byte instead of
// read from the position table.  Only the index fields of the compressed
// values that are 1 matter (value 2 g0 -> bits [4 g0, 4 g0 + 2) must hold
// p0, value 8 + 2 g1 -> bits [16 + 4 g1, ...) must hold p1; the odd values
// are 0, their fields free): u = (byte >> 4) | (byte >> 6) << 16, times
// 0x1111 (v_mul_u32_u24), puts p0 in the low two bits of nibbles 0-3 and p1
// in those of nibbles 4-7 -- 4 VALU instead of one SDWA op and a ds_read_b32
// (the 2-way bank-conflicting read of the position table).
#ifndef SMX_POS_VALU
#define SMX_POS_VALU 0
#endif
#define SMX_POS_WORD(W, B, OUT)                                                                 \
  do {                                                                                          \
    uint32_t b4_, b6_;                                                                          \
    asm("v_lshrrev_b32_sdwa %0, 4, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD "      \
        "src1_sel:BYTE_" #B "\n\tv_lshrrev_b32_sdwa %1, 6, %2 dst_sel:DWORD "                   \
        "dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_" #B                                \
        : "=&v"(b4_), "=&v"(b6_) : "v"(W));                                                     \
    OUT = int(__umul24((b6_ << 16) | b4_, 0x1111u));                                            \
  } while (0)
template <int K, int R, bool NOLDS = false>
__device__ __forceinline__ v16i TileSmfmac(const uint32_t* codes, const v8i (&b)[K / 2],
                                           const v4i* grp_tab, const int* pos_tab) {
  constexpr int KS = K / 2;
  v4i o[R];
  int ix[R];
  // NOLDS (timing ablation, results invalid): operands straight from the
  // code registers (one VALU each), no LDS table reads in the chain
  auto ld = [&](int slot, int t) {
    if constexpr (NOLDS) {
      const int w = int(codes[t >> 2] >> ((t & 3) * 8));
      o[slot] = v4i{w & 0x00010001, 0, w & 0x01000100, 0};
      ix[slot] = w;
    } else {
      // both table offsets in one SDWA op each: the group table (v4i
      // entries at LDS 0) at 16 * (byte & 0xF) = (byte << 4) truncated to its
      // low byte; the position table (one index word per 16 bytes) at
      // byte & 0xF0 = 16 * (byte >> 4)
      const uint32_t w = codes[t >> 2];
      uint32_t og, op;
#define SMX_SDWA_OFFS(B)                                                                        \
  asm("v_lshlrev_b32_sdwa %0, 4, %2 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD "        \
      "src1_sel:BYTE_" #B "\n\tv_and_b32_sdwa %1, %3, %2 dst_sel:DWORD dst_unused:UNUSED_PAD "   \
      "src0_sel:DWORD src1_sel:BYTE_" #B                                                         \
      : "=&v"(og), "=&v"(op) : "v"(w), "v"(0xF0u))
      switch (t & 3) {
        case 0: SMX_SDWA_OFFS(0); break;
        case 1: SMX_SDWA_OFFS(1); break;
        case 2: SMX_SDWA_OFFS(2); break;
        default: SMX_SDWA_OFFS(3); break;
      }
#undef SMX_SDWA_OFFS
      o[slot] = *reinterpret_cast<const v4i*>(reinterpret_cast<const char*>(grp_tab) + og);
#if SMX_POS_VALU
      switch (t & 3) {
        case 0: SMX_POS_WORD(w, 0, ix[slot]); break;
        case 1: SMX_POS_WORD(w, 1, ix[slot]); break;
        case 2: SMX_POS_WORD(w, 2, ix[slot]); break;
        default: SMX_POS_WORD(w, 3, ix[slot]); break;
      }
      (void)op;
#elif SMX_POS_B64
      // the index word read as the low half of a ds_read_b64: its bank is
      // (a/4) mod 64, so the 16 entries 16 bytes apart sit on 16 distinct
      // bank pairs (a ds_read_b32 banks (a/4) mod 32: entries p and p + 8
      // collide).  The entry's high half is 0 and or-ed in, so that the load
      // is not narrowed to b32.
      const uint2 pw = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(pos_tab) + op);
      ix[slot] = int(pw.x | pw.y);
#else
      ix[slot] = *reinterpret_cast<const int*>(reinterpret_cast<const char*>(pos_tab) + op);
#endif
    }
  };
#pragma unroll
  for (int p = 0; p < R; ++p)
    if (p < KS) ld(p, p);
  // zeroed as 8 x v_mov_b64 (the plain v16i{0} became 16 v_mov_b32 plus a
  // chain of 8 register-shifting v_mov_b64 copies per tile)
  typedef long long v8l __attribute__((ext_vector_type(8)));
  v8l z;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    long long t;
    asm volatile("v_mov_b64 %0, 0" : "=v"(t));
    z[k] = t;
  }
  v16i acc = __builtin_bit_cast(v16i, z);
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    acc = __builtin_amdgcn_smfmac_i32_32x32x64_i8(o[s % R], b[s], acc, ix[s % R], 0, 0);
    if (s + R < KS) ld(s % R, s + R);
  }
  constexpr int kDs = SMX_POS_VALU ? 1 : 2;   // LDS reads per operand step
  __builtin_amdgcn_sched_group_barrier(0x100, kDs * R, 0);
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    // the index word's v_or right before its MFMA (placed early, it waits for
    // the step's LDS reads R steps too soon)
    if (!NOLDS && SMX_POS_B64) __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    if (s == 0) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    if (s + R < KS) __builtin_amdgcn_sched_group_barrier(0x100, kDs, 0);
  }
  return acc;
}

// The tile with a dense first step (K % 4 == 2 with nb <= 2 K - 2: glove's
// 50 blocks): the last sparse step would carry two padding blocks, so
// blocks 4 KS + h (KS = K/2 - 1; nibble x0 of code byte KS) go through one
// v_mfma_i32_32x32x32_i8 with C = 0 -- A lane (r, h) = the one-hot row of its
// block (a 16-entry LDS table), B lane (c, h) = that block's LUT row -- and
// the KS sparse steps accumulate onto it: the same MFMA count, no accumulator
// zeroing, no padded half step.
template <int K, int R>
__device__ __forceinline__ v16i TileSmfmacD(const uint32_t* codes, const v8i (&b)[K / 2 - 1],
                                            const v4i& bd, const v4i* grp_tab, const int* pos_tab,
                                            const v4i* hot_tab) {
  constexpr int KS = K / 2 - 1;
  v4i o[R];
  int ix[R];
  auto ld = [&](int slot, int t) {
    const uint32_t w = codes[t >> 2];
    uint32_t og, op;
#define SMX_SDWA_OFFS(B)                                                                        \
  asm("v_lshlrev_b32_sdwa %0, 4, %2 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD "        \
      "src1_sel:BYTE_" #B "\n\tv_and_b32_sdwa %1, %3, %2 dst_sel:DWORD dst_unused:UNUSED_PAD "   \
      "src0_sel:DWORD src1_sel:BYTE_" #B                                                         \
      : "=&v"(og), "=&v"(op) : "v"(w), "v"(0xF0u))
    switch (t & 3) {
      case 0: SMX_SDWA_OFFS(0); break;
      case 1: SMX_SDWA_OFFS(1); break;
      case 2: SMX_SDWA_OFFS(2); break;
      default: SMX_SDWA_OFFS(3); break;
    }
#undef SMX_SDWA_OFFS
    o[slot] = *reinterpret_cast<const v4i*>(reinterpret_cast<const char*>(grp_tab) + og);
#if SMX_POS_VALU
    switch (t & 3) {
      case 0: SMX_POS_WORD(w, 0, ix[slot]); break;
      case 1: SMX_POS_WORD(w, 1, ix[slot]); break;
      case 2: SMX_POS_WORD(w, 2, ix[slot]); break;
      default: SMX_POS_WORD(w, 3, ix[slot]); break;
    }
    (void)op;
#else
    ix[slot] = *reinterpret_cast<const int*>(reinterpret_cast<const char*>(pos_tab) + op);
#endif
  };
  // the dense step's one-hot row: x0 = ((by & 3) << 2) | ((by >> 4) & 3)
  const uint32_t by = (codes[KS >> 2] >> (8 * (KS & 3))) & 0xFFu;
  const uint32_t x0 = ((by & 3u) << 2) | ((by >> 4) & 3u);
  const v4i hot = hot_tab[x0];
#pragma unroll
  for (int p = 0; p < R; ++p)
    if (p < KS) ld(p, p);
  v16i acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(hot, bd, v16i{}, 0, 0, 0);
#pragma unroll
  for (int st = 0; st < KS; ++st) {
    acc = __builtin_amdgcn_smfmac_i32_32x32x64_i8(o[st % R], b[st], acc, ix[st % R], 0, 0);
    if (st + R < KS) ld(st % R, st + R);
  }
  constexpr int kDs = SMX_POS_VALU ? 1 : 2;
  __builtin_amdgcn_sched_group_barrier(0x100, kDs * R + 1, 0);
  __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // the dense step
  __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // (the next tile's code load)
#pragma unroll
  for (int st = 0; st < KS; ++st) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    if (st + R < KS) __builtin_amdgcn_sched_group_barrier(0x100, kDs, 0);
  }
  return acc;
}

// One tile of a 16-slot item: S[dp][q] for 32 datapoints x 16 queries on
// v_smfmac_i32_16x16x128_i8, two accumulator chains (A: datapoints 0..15, B:
// 16..31) of K16 = ceil(K / 4) steps of 8 AH blocks each.  Operand layout
// (tools/smfmac16_probe.hip): A lane (r, gA = lane / 16) holds row r; its
// compressed values j < 8 pair with B lanes of group 2 (gA & 1), j >= 8 with
// group 2 (gA & 1) + 1, in bytes 16 (gA >> 1) + 4 ((j % 8) / 2) + idx_j of
// those lanes; B lane (n, gB) holds column n, 32 bytes; D lane (n, g) holds
// column n, rows 4 g + e.  So A lane group gA takes the code byte 2 s' +
// (gA & 1) of the 32-slot tile layout's half gA >> 1 -- blocks x0 = 8 s' +
// 4 (gA & 1) + (gA >> 1) and x0 + 2 -- and B lane group gB then needs LUT
// rows 8 s' + 2 gB and 8 s' + 2 gB + 1: the 32 contiguous bytes the 32-slot
// path reads at its step 2 s' + (gB >> 1), half gB & 1.  The code bytes are
// the 32-slot layout's (no second copy of the codes): lane (r, gA) loads the
// 16-byte lane records of rows r and r + 16 of half gA >> 1 (`ca`, `cb`),
// shifted right by 8 (gA & 1) bits, so that step s' reads byte 2 (s' % 2) of
// dword s' / 2.  The same operand tables as the 32-slot path.
template <int K, int R, bool NOLDS = false>
__device__ __forceinline__ void TileSmfmac16(const uint32_t* ca, const uint32_t* cb,
                                             const v8i (&b)[(K + 3) / 4], const v4i* grp_tab,
                                             const int* pos_tab, v4i& acc_a, v4i& acc_b) {
  constexpr int K16 = (K + 3) / 4;
  constexpr int NS = 2 * K16;   // MFMAs: steps x chains, A and B in turn
  v4i o[R];
  int ix[R];
  auto ld = [&](int slot, int t) {
    const int st = t >> 1;
    const uint32_t w = (t & 1) ? cb[st >> 1] : ca[st >> 1];
    if constexpr (NOLDS) {   // (timing ablation, results invalid: as TileSmfmac's)
      const int x = int((st & 1) ? (w >> 16) : w);
      o[slot] = v4i{x & 0x00010001, 0, x & 0x01000100, 0};
      ix[slot] = x;
      return;
    }
    uint32_t og, op;
#define SMX_SDWA_OFFS16(B)                                                                      \
  asm("v_lshlrev_b32_sdwa %0, 4, %2 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD "        \
      "src1_sel:BYTE_" #B "\n\tv_and_b32_sdwa %1, %3, %2 dst_sel:DWORD dst_unused:UNUSED_PAD "   \
      "src0_sel:DWORD src1_sel:BYTE_" #B                                                         \
      : "=&v"(og), "=&v"(op) : "v"(w), "v"(0xF0u))
    if (st & 1) {
      SMX_SDWA_OFFS16(2);
    } else {
      SMX_SDWA_OFFS16(0);
    }
#undef SMX_SDWA_OFFS16
    o[slot] = *reinterpret_cast<const v4i*>(reinterpret_cast<const char*>(grp_tab) + og);
#if SMX_POS_VALU
    if (st & 1)
      SMX_POS_WORD(w, 2, ix[slot]);
    else
      SMX_POS_WORD(w, 0, ix[slot]);
    (void)op;
#else
    ix[slot] = *reinterpret_cast<const int*>(reinterpret_cast<const char*>(pos_tab) + op);
#endif
  };
#pragma unroll
  for (int p = 0; p < R; ++p)
    if (p < NS) ld(p, p);
  long long z0, z1, z2, z3;
  asm volatile("v_mov_b64 %0, 0" : "=v"(z0));
  asm volatile("v_mov_b64 %0, 0" : "=v"(z1));
  asm volatile("v_mov_b64 %0, 0" : "=v"(z2));
  asm volatile("v_mov_b64 %0, 0" : "=v"(z3));
  typedef long long v2l __attribute__((ext_vector_type(2)));
  acc_a = __builtin_bit_cast(v4i, v2l{z0, z1});
  acc_b = __builtin_bit_cast(v4i, v2l{z2, z3});
#pragma unroll
  for (int t = 0; t < NS; ++t) {
    if (t & 1)
      acc_b = __builtin_amdgcn_smfmac_i32_16x16x128_i8(o[t % R], b[t >> 1], acc_b, ix[t % R], 0, 0);
    else
      acc_a = __builtin_amdgcn_smfmac_i32_16x16x128_i8(o[t % R], b[t >> 1], acc_a, ix[t % R], 0, 0);
    if (t + R < NS) ld(t % R, t + R);
  }
  constexpr int kDs = SMX_POS_VALU ? 1 : 2;
  __builtin_amdgcn_sched_group_barrier(0x100, kDs * R, 0);
#pragma unroll
  for (int t = 0; t < NS; ++t) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    if (t + R < NS) __builtin_amdgcn_sched_group_barrier(0x100, kDs, 0);
  }
}

// f(integral_constant<I>), ..., f(integral_constant<D - 1>): the ring slots of
// the 16-slot scan, unrolled (each slot's registers fixed at compile time)
template <int I, int D, class F>
__device__ __forceinline__ void EachSlot(F& f) {
  f(std::integral_constant<int, I>{});
  if constexpr (I + 1 < D) EachSlot<I + 1, D>(f);
}
#ifndef SMX_RING16
#define SMX_RING16 0   // 0: 4 tiles in flight per wave at <= 3 code dwords per lane, else 3
#endif

// ---------------------------------------------------------------------------
// The scan kernel: one workgroup of kScanWaves waves per CU (3 per SIMD), the
// CU's waves sharing a static share of the work and balancing it among
// themselves through LDS atomics (a returning device-scope atomic costs
// microseconds under this load; an LDS atomic ~100 cycles).
//
// Work items (leaf, 32-query tile of that leaf, chunk of tiles) are listed in
// 8 groups of consecutive leaves with equal MFMA work, one per XCD group
// (blockIdx % 8 share an XCD under the observed round-robin placement; speed
// only, never correctness), so a leaf's query tiles run on one XCD and re-read
// the leaf's codes from that XCD's L2.  The worklist kernel cuts each group's
// tiles into equal contiguous shares, one per workgroup (wave_start); a share
// may begin and end inside an item.  Wave 0 lists the share's segments (item,
// tile range) in LDS; each wave claims a segment, loads its B fragments once
// and takes the segment's tiles two at a time from the segment's LDS counter
// (one pair claimed ahead); a wave with no unclaimed segment left joins the
// segment with the most tiles left.  Every wave therefore works until the
// CU's share is done, whatever its tiles' hit rates and setup costs.
//
// Per segment: lane (c, h) takes its query slot's record (query, sum limit,
// bias; written by the seed kernel), loads the int8 LUT rows 2s+h, s < K, of
// query c into K registers (the MFMA B fragments); then for each tile K x MFMA
// i32_32x32x32_i8 with A = one-hot codes (row = datapoint, 16 bytes per
// lane-half = one block's 16 centers) gives S[dp][q] = sum_b LUT_q[b][code(dp,
// b)] exactly (|S| <= 127*B).  A datapoint can only pass when S <= amax_q (the
// largest sum whose distance can pass the query's threshold; d is monotone in
// S); a lane whose 16-sum minimum passes appends its sums (packed int16) and a
// tag to the wave's LDS hit list; drain() runs the per-element test, the
// distance
//     d = fl(fl(float(S) * inv_q) + bias_{q,leaf})
// and the key test (ordered(d) << 32 | tie) <= threshold key lane-parallel
// over the hits, and stages the segment's survivors in LDS: one global atomic
// per query per segment reserves their list slots (issued at the segment's
// end, its result consumed after the next segment's first tile).
// ABL = 4: timing ablation without the epilogue; ABL = 2: with the hit test
// but no hit list; ABL = 16: with hit lists and drains but no copy to the
// candidate lists; ABL = 32: every tile of a segment computed from its first
// tile's codes (cache-hot: the code loads' latency out of the loop); ABL =
// 64: the MFMA operands straight from the code registers, no LDS table reads
// (68: and no epilogue); results invalid for all of them.
// ---------------------------------------------------------------------------

constexpr int kHitsPerWave = 64;   // a tile adds at most one hit per lane
constexpr int kItemKeys = 256;     // survivors one segment stages in LDS
constexpr int kMaxSegs = 512;      // share segments listed per round
constexpr uint32_t kStealMin = 3;  // tiles left for a second wave to join a segment

// Waves per scan workgroup: 3 per SIMD (168 VGPRs) up to K = 26; 2 per SIMD
// above (the K B-fragment registers).
#ifndef SMX_SCAN_WAVES
#define SMX_SCAN_WAVES 12
#endif
template <int K>
constexpr int ScanWaves() { return K <= 26 ? SMX_SCAN_WAVES : 8; }
#ifndef SMX_SCAN_R
#define SMX_SCAN_R 2
#endif
#ifndef SMX_SCAN_R16
#define SMX_SCAN_R16 2
#endif

// Diagnostic stamps (ABL & 8; a separate buffer that nothing else reads):
// per segment {hw_id | worker << 32, xcc_id << 32 | item, realtime, memtime at
// the segment's start, after its setup, after its tiles, after its flush,
// tiles | hit lanes << 16 | survivors << 40}; worker = block * waves + wave.
__device__ __forceinline__ void StampItem(const ScanArgs& a, uint32_t worker, uint32_t item,
                                          uint64_t rt, uint64_t t0, uint64_t t1, uint64_t t2,
                                          uint64_t t3, uint64_t tiles) {
  const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_REG_HW_ID
  const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (15 << 11));  // HW_REG_XCC_ID
  const uint32_t slot = atomicAdd(a.stamp_count, 1u);
  if (slot < a.stamp_cap) {
    unsigned long long* p = a.stamps + size_t(slot) * 8;
    p[0] = hw | (uint64_t(worker) << 32);
    p[1] = (uint64_t(xcc) << 32) | item;
    p[2] = rt;
    p[3] = t0;
    p[4] = t1;
    p[5] = t2;
    p[6] = t3;
    p[7] = tiles;
  }
}

// The query parameters of a segment's 32 slots, in LDS for the drain.
struct QParam {
  uint32_t qid;
  int32_t amax;
  float bias;
  float inv;
};

// A wave's own LDS: hit list, the survivor stage of up to kStageSegs of its
// segments (written to the candidate lists together: list_flush), their
// query ids and per-slot counts.
constexpr int kStageSegs = 4;                // segments one stage holds
constexpr int kStageKeys = 2 * kItemKeys;    // survivors one stage holds
struct ScanWaveLds {
  uint4 hsum[2 * kHitsPerWave][2];   // 16 sums as int16 pairs (the flush's scratch too)
  uint32_t hmeta[2 * kHitsPerWave];  // tile << 6 | lane
  uint64_t kbuf[kStageKeys];
  uint8_t kslot[kStageKeys];         // stage segment << 5 | query slot
  uint32_t s_kn;
  uint32_t qcnt[kStageSegs * 32], qtab[kStageSegs * 32];
  QParam qp[32];
};

// A segment's item descriptor, kept in LDS: a segment's setup reads it from
// there instead of waiting for a global load.
struct SegDesc {
  uint64_t tile_off;
  uint64_t member_off;
  uint32_t n;
  uint32_t leaf;
  uint32_t slot0;    // the item's first leaf slot (a.leaf_pair)
  uint32_t nslots;   // slots [slot0, slot0 + nslots); the other slots are empty
};

// Wave 0 of a scan workgroup: the next segments of the share (item, first
// tile, end tile, descriptor) into the LDS table, 64 items per step (a prefix
// of their tiles), at most kMaxSegs; the share's remainder stays in s_sw /
// s_su.  sj: the share's first tile | kShareFirst until the first step (the
// share starts at that tile's first unit: its item's kItemCost units are the
// share before's).
constexpr uint32_t kShareFirst = 0x80000000u;
__device__ __forceinline__ void ListSegments(const ScanArgs& a, int lane, uint32_t& sj,
                                             uint32_t* s_item, uint32_t* s_end, uint32_t* s_next,
                                             SegDesc* s_desc, uint32_t& s_sw, uint32_t& s_su,
                                             uint32_t& s_nseg, uint32_t& s_claim) {
  uint32_t sw = s_sw, su = s_su, nseg = 0;
  while (su > 0 && nseg + 64 <= uint32_t(kMaxSegs)) {
    const uint32_t idx = sw + uint32_t(lane);
    const WorkItem it = a.work[min(idx, a.num_items - 1)];
    const uint32_t wt = (it.leaf & kItemNarrow) ? 1u : 2u;   // units per tile
    const bool first = lane == 0 && (sj & kShareFirst);
    const uint32_t j0 = first ? (sj & ~kShareFirst) : it.j0;
    const uint32_t ic = first ? 0u : kItemCost;                // the item's own units
    const uint32_t tt = it.jend > j0 ? it.jend - j0 : 0u;      // the item's tiles
    const uint32_t t = min(ic + tt * wt, su);                  // ... in units
    uint32_t incl = t;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = uint32_t(__shfl_up(int(incl), off));
      if (lane >= off) incl += y;
    }
    const uint32_t excl = incl - t;
    const bool used = excl < su;   // a prefix of the lanes, lane 0 always
    // the tiles whose first unit is inside the share
    const uint32_t own = su - excl > ic ? min(tt, (su - excl - ic + wt - 1) / wt) : 0u;
    const bool take = used && own > 0;
    if (take) SMX_CHECK(idx, a.bd.items, "listed item");
    const uint64_t bt = __ballot(take);
    if (take) {
      const uint32_t pos = nseg + uint32_t(__popcll(bt & ((1ull << lane) - 1ull)));
      s_item[pos] = idx;
      s_next[pos] = j0;
      s_end[pos] = j0 + own;
      SegDesc dsc;
      dsc.tile_off = it.tile_off;
      dsc.member_off = it.member_off;
      dsc.n = it.n;
      dsc.leaf = it.leaf;   // (with its kItemNarrow flag)
      dsc.slot0 = it.slot0;
      dsc.nslots = it.nslots;
      s_desc[pos] = dsc;
    }
    const uint32_t nused = uint32_t(__popcll(__ballot(used)));
    const uint32_t last_incl = uint32_t(__shfl(int(incl), int(nused) - 1));
    sw += nused;
    su -= min(su, last_incl);
    nseg += uint32_t(__popcll(bt));
    sj = 0;
  }
  if (lane == 0) {
    s_sw = sw;
    s_su = su;
    s_nseg = nseg;
    s_claim = 0;
  }
}

// The lane id from v_mbcnt, opaque to the compiler (volatile asm), so that it
// is rematerialised at every use instead of occupying a register.
struct LaneId {
  __device__ __forceinline__ operator int() const {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
  }
};
template <int MASK, int SHIFT>
struct LaneField {
  __device__ __forceinline__ operator int() const { return (int(LaneId()) >> SHIFT) & MASK; }
};
// ... or computed once and held in a register
template <int MASK, int SHIFT>
struct LaneVal {
  int v;
  __device__ __forceinline__ LaneVal() : v(int((threadIdx.x & 63u) >> SHIFT) & MASK) {}
  __device__ __forceinline__ operator int() const { return v; }
};

// NRW: 0 = 32-slot items only, kNarrowOnly = 16-slot items only (one path
// compiled into each kernel: fewer registers and less code).
template <int K, int ABL = 0, int NRW = 0, bool DN = false>
__global__ void __launch_bounds__(64 * ScanWaves<K>(), 1) lut16_scan_kernel(ScanArgs a) {
  // DN: the dense-first tile (TileSmfmacD), 32-slot items only
  static_assert(!DN || (K % 4 == 2 && NRW == 0), "dense-first tiles: K % 4 == 2, 32-slot");
  constexpr int NW = ((((K + 1) / 2) + 3) / 4);
  constexpr int W = 4 * NW;
  constexpr int Q = 32, KB = kItemKeys, NWAVES = ScanWaves<K>();
  constexpr int R = SMX_SCAN_R;   // one-hot reads in flight ahead of their MFMA
  static_assert(K % 2 == 0, "the sparse scan takes two code nibbles per step");
  __shared__ ScanWaveLds wl_[NWAVES];
  // the two operand tables in one 512-byte array at LDS 0 (256-aligned, the
  // largest alignment is placed first): group entries [0, 256), position
  // entries at 256 + 16 p, so both offsets fold into the ds_read's immediate
  __shared__ __align__(256) v4i opnd_tab[48];
  v4i* const grp_tab = opnd_tab;
  int* const pos_tab = reinterpret_cast<int*>(opnd_tab + 16);
  v4i* const hot_tab = opnd_tab + 32;   // one-hot rows (the dense-first step)
  __shared__ uint32_t s_item[kMaxSegs], s_end[kMaxSegs], s_next[kMaxSegs];
  __shared__ SegDesc s_desc[kMaxSegs];
  __shared__ uint32_t s_nseg, s_claim, s_sw, s_su;
  // wave-uniform values in scalar registers (the B fragments need the VGPRs)
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // the lane id and its fields recomputed where they are used (two VALU ops)
  // instead of held across the segment loop: held, the allocator spilled them
  // and their reloads waited for the segment-record prefetch (vmcnt is in
  // order)
  // (the 16-slot-only kernel has registers to spare and is issue-bound: there
  // the recomputation measured 4% slower, so it keeps them in registers)
  constexpr bool kRemat = NRW != int(kNarrowOnly);
  const std::conditional_t<kRemat, LaneId, LaneVal<63, 0>> lane;
  const std::conditional_t<kRemat, LaneField<31, 0>, LaneVal<31, 0>> c;
  const std::conditional_t<kRemat, LaneField<1, 5>, LaneVal<1, 5>> h;
  ScanWaveLds& wl = wl_[wv];
  if (threadIdx.x < 16) {   // group nibble g0 | g1 << 2: a 1 at values 2*g0, 8 + 2*g1
    const uint32_t g0 = threadIdx.x & 3u, g1 = threadIdx.x >> 2;
    v4i t = {0, 0, 0, 0};
    t[g0 >> 1] = int(1u << (16 * (g0 & 1u)));
    t[2 + (g1 >> 1)] = int(1u << (16 * (g1 & 1u)));
    grp_tab[threadIdx.x] = t;
    // position nibble p0 | p1 << 2: p0 in index fields 0..7, p1 in 8..15
    pos_tab[4 * threadIdx.x] = int((threadIdx.x & 3u) * 0x5555u | ((threadIdx.x >> 2) * 0x5555u) << 16);
    pos_tab[4 * threadIdx.x + 1] = 0;   // the high half of the ds_read_b64
    v4i hv = {0, 0, 0, 0};
    hv[threadIdx.x >> 2] = int(1u << (8 * (threadIdx.x & 3u)));
    hot_tab[threadIdx.x] = hv;
  }
  const uint32_t worker = blockIdx.x * NWAVES + wv;
  // this workgroup's share: `units` tiles from tile jfirst of item w on
  // (wave 0 lists the segments; only its copy is used)
  const uint4 ws = wv != 0 ? make_uint4(0, 0, 0, 0) : a.wave_start[blockIdx.x];
  if (threadIdx.x == 0) {
    s_sw = ws.x;
    s_su = ws.z;
  }
  uint32_t sj = ws.y | kShareFirst;   // the share's first tile inside its first item
  // The survivors of up to kStageSegs segments stay in the wave's stage and
  // go to the candidate lists together, when the stage is full and once at
  // the end: one list-slot atomic per (segment, query slot) with survivors,
  // then each key at its query's reserved slot + a running count.  (Round 5
  // flushed every segment -- its slot atomics issued behind the next
  // segment's first code loads, the keys stored after that tile -- so with
  // vmcnt in order every later code-load wait also waited for those atomics
  // and stores: the ablations put 7-10 us of the scan there, more at looser
  // seed thresholds, profiles/r06/ab/scan_ablations_rows.txt.)
  uint32_t nst = 0;   // segments in the stage (wave-uniform)
  auto list_flush = [&]() {
    const uint32_t kn = min(__builtin_amdgcn_readfirstlane(wl.s_kn), uint32_t(kStageKeys));
    if ((ABL & 16) == 0 && nst > 0) {   // (16: timing ablation without the lists)
      uint32_t* qbase = reinterpret_cast<uint32_t*>(&wl.hsum[0][0]);   // [kStageSegs * 32]
      uint32_t* qrun = qbase + kStageSegs * 32;
      for (uint32_t e = uint32_t(lane); e < nst * 32u; e += 64) {
        const uint32_t m = wl.qcnt[e];
        uint32_t base = 0;
        if (m) {
          SMX_CHECK(wl.qtab[e], a.bd.nq, "slot query");
          base = atomicAdd(&a.cand_count[size_t(wl.qtab[e]) * kCounterStride], m);
        }
        qbase[e] = base;
        qrun[e] = 0;
      }
      WaveLdsSync();
      for (uint32_t e = uint32_t(lane); e < kn; e += 64) {
        const uint32_t qs = wl.kslot[e];
        const uint32_t sl = qbase[qs] + atomicAdd(&qrun[qs], 1u);
        SMX_GUARD(wl.qtab[qs], a.bd.nq, "list query")
        if (sl < a.cap) a.cand[size_t(wl.qtab[qs]) * a.cap + sl] = wl.kbuf[e];
      }
      WaveLdsSync();
    }
    for (uint32_t e = uint32_t(lane); e < uint32_t(kStageSegs * 32); e += 64) wl.qcnt[e] = 0;
    if (lane == 0) wl.s_kn = 0;
    WaveLdsSync();
    nst = 0;
  };
  for (uint32_t e = uint32_t(lane); e < uint32_t(kStageSegs * 32); e += 64) wl.qcnt[e] = 0;
  if (lane == 0) wl.s_kn = 0;
  // one LDS claim of two tiles of segment `sg` (lane 0; broadcast at use)
  auto claim2 = [&](uint32_t sg) -> uint32_t {
    uint32_t v = 0;
    if (lane == 0) v = atomicAdd(&s_next[sg], 2u);
    return v;
  };

  for (;;) {   // rounds of at most kMaxSegs segments (block-uniform)
    __syncthreads();   // s_sw / s_su / the segment table are free
    if (wv == 0) ListSegments(a, lane, sj, s_item, s_end, s_next, s_desc, s_sw, s_su, s_nseg,
                                 s_claim);
    __syncthreads();
    const uint32_t nseg = s_nseg;
    if (nseg == 0) break;
    // claim-ahead segment (a reservation: joiners may still take its tiles)
    uint32_t sg_next = 0;
    if (lane == 0) sg_next = atomicAdd(&s_claim, 1u);
    // the claimed-ahead segment's item and query ids, loaded during the
    // segment before it: the B-fragment addresses need the query id, so
    // without this a segment's setup is two dependent global latencies
    uint32_t pf_seg = ~0u, pf_item = 0;
    ItemLane pf_rec = {};
    for (;;) {
      uint32_t sg = __builtin_amdgcn_readfirstlane(sg_next);
      if (sg >= nseg) {
        // no unclaimed segment: join the last-claimed one (most tiles left,
        // segments are claimed in order) with >= kStealMin tiles left
        int found = -1;
        for (int base = int(nseg) - 64; found < 0 && base > -64; base -= 64) {
          const int i = base + lane;
          bool ok = false;
          if (i >= 0) {
            const uint32_t e = s_end[i], nx = s_next[i];
            ok = nx < e && e - nx >= kStealMin;
          }
          const uint64_t bal = __ballot(ok);
          if (bal) found = base + 63 - int(__clzll(bal));
        }
        if (found < 0) break;
        sg = uint32_t(__builtin_amdgcn_readfirstlane(found));
      } else if (lane == 0) {
        sg_next = atomicAdd(&s_claim, 1u);   // the next one, claimed ahead
      }
      const uint32_t end = __builtin_amdgcn_readfirstlane(s_end[sg]);
      uint32_t j = __builtin_amdgcn_readfirstlane(claim2(sg));
      if (j >= end) continue;   // (joined too late)
      uint64_t st_rt = 0, st_t0 = 0, st_t1 = 0, st_t2 = 0;
      uint32_t st_hits = 0, st_surv = 0;
      if (ABL & 8) {
        st_rt = __builtin_amdgcn_s_memrealtime();
        st_t0 = __builtin_amdgcn_s_memtime();
      }
      // the slot's lane record {query, bias, 1/multiplier, sum limit}:
      // prefetched during the segment before (the claimed-ahead one), so
      // the B-fragment loads issue at once
      // (slot c of the item: record slot0 + c when c < nslots, else empty)
      // (a 16-slot item: slot lane % 16, the column of the lane's B fragment)
      auto slot_rec = [&](uint32_t sgi) {
        const uint32_t s0 = __builtin_amdgcn_readfirstlane(s_desc[sgi].slot0);
        const uint32_t ns = __builtin_amdgcn_readfirstlane(s_desc[sgi].nslots);
        uint32_t cs = uint32_t(c);
        if constexpr (NRW == int(kNarrowOnly)) cs = uint32_t(lane & 15);
        ItemLane r;
        if (cs < ns) {
          SMX_CHECK(s0 + cs, a.bd.recs, "leaf slot");
          const uint32_t p = a.leaf_pair[s0 + cs];
          SMX_CHECK(p, a.bd.pairs, "slot pair");
          r = a.pair_rec[p];
        } else {
          r.qid = kNoQuery;
          r.bias = 0.0f;
          r.inv = 0.0f;
          r.amax = kNoSum;
        }
        return r;
      };
      uint32_t item;
      ItemLane cl;
      if (sg == pf_seg) {
        item = pf_item;
        cl = pf_rec;
      } else {
        item = __builtin_amdgcn_readfirstlane(s_item[sg]);
        SMX_CHECK(item, a.bd.items, "segment item");
        cl = slot_rec(sg);
      }
      const uint32_t qid = cl.qid;
      // an empty slot (kNoQuery) loads query 0's rows and never passes (amax)
      const uint32_t lq = qid == kNoQuery ? 0u : qid;
      const SegDesc& sd = s_desc[sg];
      const uint64_t toff = (uint64_t(__builtin_amdgcn_readfirstlane(uint32_t(sd.tile_off >> 32))) << 32) |
                            __builtin_amdgcn_readfirstlane(uint32_t(sd.tile_off));
      const uint64_t moff = (uint64_t(__builtin_amdgcn_readfirstlane(uint32_t(sd.member_off >> 32))) << 32) |
                            __builtin_amdgcn_readfirstlane(uint32_t(sd.member_off));
      const uint32_t n = __builtin_amdgcn_readfirstlane(sd.n);
      const uint32_t leaf_w = __builtin_amdgcn_readfirstlane(sd.leaf);
      const int leaf = int(leaf_w & ~kItemNarrow);
      SMX_CHECK(qid == kNoQuery ? 0u : qid, a.bd.nq, "slot record query");
      SMX_CHECK(leaf, a.bd.nl, "segment leaf");
      SMX_CHECK(toff + (n + 31u) / 32u, a.bd.tiles + 1, "segment tiles");
      SMX_CHECK(moff + n, a.bd.members + 1, "segment members");
      // the segment's tiles, on the 32-slot or the 16-slot path (the item's
      // kItemNarrow flag; wave-uniform)
      uint32_t tiles_done = 0;
      // a full stage (kStageSegs segments, or less than one segment's worth
      // of key room) goes to the lists before this segment stages its own
      if (nst == uint32_t(kStageSegs) ||
          __builtin_amdgcn_readfirstlane(wl.s_kn) > uint32_t(kStageKeys - KB))
        list_flush();
      const uint32_t kn_seg = __builtin_amdgcn_readfirstlane(wl.s_kn);
      auto run_seg = [&](auto nr_tag) {
      constexpr bool NR = decltype(nr_tag)::value;
      constexpr int KB_STEPS = NR ? (K + 3) / 4 : K / 2 - (DN ? 1 : 0);   // B fragments (steps)
      // this segment's B fragments and first tile: 32-slot, LUT rows
      // 4s + 2h, 4s + 2h + 1 of query c per sparse step; 16-slot, rows
      // 8s' + 2gB, 8s' + 2gB + 1 of query n = lane % 16 (gB = lane / 16)
      v8i b[KB_STEPS];
      v4i bd = {};   // (DN) the dense step's B fragment
      uint32_t codes[NW] = {}, codes_b[NW] = {};
      // addresses as a wave-uniform base + a 32-bit lane offset (saddr
      // loads: no 64-bit per-lane pointers live across the tile loop); the
      // 16-slot path reads rows r and r + 16 of half (lane / 32) of the tile
      const uint8_t* tseg = a.tiles + toff * 64ull * W;
      const uint32_t lane_off =
          NR ? uint32_t((lane >> 5) * 32 + (lane & 15)) * uint32_t(W) : uint32_t(lane) * uint32_t(W);
      auto tile_ptr = [&](uint32_t t) {
        if (ABL & 32) t = j;   // timing ablation: every tile's codes = the first one's (cache-hot)
        return tseg + size_t(t * uint32_t(64 * W) + lane_off);
      };
      const uint32_t boff = NR ? lq * uint32_t(LutRows(K) * 16) + uint32_t(lane >> 4) * 32u
                               : lq * uint32_t(LutRows(K) * 16) + uint32_t(h) * 32u;
      const uint8_t* lutb = reinterpret_cast<const uint8_t*>(a.lut);
      auto load_b = [&]() {
        // one per-lane address, the steps as immediate offsets
        const v8i* bp = reinterpret_cast<const v8i*>(lutb + size_t(boff));
#pragma unroll
        for (int s2 = 0; s2 < KB_STEPS; ++s2) b[s2] = bp[(NR ? 4 : 2) * s2];
        if constexpr (DN && !NR)   // the dense step's LUT row: block 4 (K/2 - 1) + h
          bd = *reinterpret_cast<const v4i*>(lutb + size_t(lq * uint32_t(LutRows(K) * 16) +
                                                           uint32_t(4 * (K / 2 - 1) + h) * 16u));
      };
      auto load_codes = [&](uint32_t t, uint32_t (&ca)[NW], uint32_t (&cbb)[NW]) {
        LoadCodes<K>(tile_ptr(t), ca);
        if constexpr (NR) LoadCodes<K>(tile_ptr(t) + 16 * W, cbb);
      };
      // (the 16-slot-only kernel loads its tiles in its own ring below)
      constexpr bool DEEP = NR && NRW == int(kNarrowOnly);
      load_b();
      if constexpr (!DEEP) load_codes(j, codes, codes_b);
      // the claimed-ahead segment's item and query ids, for its setup
      {
        const uint32_t sn = __builtin_amdgcn_readfirstlane(sg_next);
        if (sn < nseg) {
          pf_seg = sn;
          pf_item = __builtin_amdgcn_readfirstlane(s_item[sn]);
          SMX_CHECK(pf_item, a.bd.items, "prefetch item");
          pf_rec = slot_rec(sn);
        } else {
          pf_seg = ~0u;
        }
      }

      // the slot's sum limit (written with the record by the pair scatter:
      // the largest LUT16 sum whose distance can pass the query's threshold)
      const int amax = cl.amax;
      if (lane < Q) {   // (16-slot: lanes 16..31 repeat slots 0..15; never counted)
        QParam v;
        v.qid = qid;
        v.amax = amax;
        v.bias = cl.bias;
        v.inv = cl.inv;
        wl.qp[lane] = v;
        wl.qtab[nst * 32u + lane] = qid;
      }
      WaveLdsSync();
      uint32_t whits = 0;   // wave-uniform

      // the hit list, one hit per lane: its EPH sums (packed int16, in
      // registers) against the slot's sum limit give a mask, and each round
      // takes one set bit per lane -- the element's distance, key and a
      // ballot-ranked append to the LDS stage (no returning atomic).  A hit
      // lane has ~1-2 passing elements of its EPH, so a round of 64 hits
      // costs ~2-3 element rounds instead of EPH (round 5 spread the EPH x
      // hits elements over the lanes, every one tested and ranked).
      // sum <= amax implies key <= the threshold key: the scan's thresholds
      // are the seed's (ordered(d_k') << 32 | 0xFFFFFFFF) or none, and d is
      // monotone in the sum
      constexpr uint32_t EPH = NR ? 8u : 16u;
      auto drain = [&]() {
        const uint32_t nh = whits;
        uint32_t kn = __builtin_amdgcn_readfirstlane(wl.s_kn);
        for (uint32_t h0 = 0; h0 < nh; h0 += 64) {
          const uint32_t hidx = h0 + uint32_t(lane);
          uint32_t mask = 0, meta = 0;
          uint32_t sw[EPH / 2];
          QParam pq = {};
          if (hidx < nh) {
            meta = wl.hmeta[hidx];
            const uint4 w0 = wl.hsum[hidx][0];
            sw[0] = w0.x; sw[1] = w0.y; sw[2] = w0.z; sw[3] = w0.w;
            if constexpr (!NR) {
              const uint4 w1 = wl.hsum[hidx][1];
              sw[4] = w1.x; sw[5] = w1.y; sw[6] = w1.z; sw[7] = w1.w;
            }
            pq = wl.qp[NR ? (meta & 15u) : (meta & 31u)];
#pragma unroll
            for (uint32_t i = 0; i < EPH; ++i) {
              const int sum = int(int16_t(uint16_t(sw[i >> 1] >> (16u * (i & 1u)))));
              mask |= (sum <= pq.amax ? 1u : 0u) << i;
            }
          } else {
#pragma unroll
            for (uint32_t i = 0; i < EPH / 2; ++i) sw[i] = 0;
          }
          const int cc = int(NR ? (meta & 15u) : (meta & 31u));
          const uint32_t jj = meta >> 6;
          while (__builtin_amdgcn_ballot_w64(mask != 0u)) {   // wave-uniform rounds
            const bool pass = mask != 0u;
            uint64_t key = 0;
            if (pass) {
              const uint32_t i = uint32_t(__builtin_ctz(mask));
              mask &= mask - 1u;
              uint32_t dp;
              if constexpr (NR)   // lane (n, g): column n, rows 4 g + (i & 3) of chain i >> 2
                dp = jj * kDpPerTile + 16u * (i >> 2) + 4u * ((meta >> 4) & 3u) + (i & 3u);
              else
                dp = jj * kDpPerTile + (i & 3u) + 8u * (i >> 2) + 4u * ((meta >> 5) & 1u);
              uint32_t word = sw[0];
#pragma unroll
              for (uint32_t k = 1; k < EPH / 2; ++k)
                if ((i >> 1) == k) word = sw[k];
              const int sum = int(int16_t(uint16_t(word >> (16u * (i & 1u)))));
              const float d = DistOf(sum, pq.inv, pq.bias);
              const uint32_t tie = a.shift > 0 ? ((uint32_t(leaf) << a.shift) | dp)
                                               : a.members[moff + dp];
              key = (uint64_t(OrderedBits(d)) << 32) | tie;
            }
            const uint64_t bm = __builtin_amdgcn_ballot_w64(pass);
            if (pass) {
              const uint32_t p = kn + __builtin_amdgcn_mbcnt_hi(
                                          uint32_t(bm >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(bm), 0u));
              if (p < uint32_t(kStageKeys)) {
                wl.kbuf[p] = key;
                wl.kslot[p] = uint8_t((nst << 5) | uint32_t(cc));
                atomicAdd(&wl.qcnt[nst * 32u + uint32_t(cc)], 1u);
              } else {  // stage full (rare): straight to the global list
                const uint32_t qq = pq.qid;
                const uint32_t gs = atomicAdd(&a.cand_count[size_t(qq) * kCounterStride], 1u);
                if (gs < a.cap) a.cand[size_t(qq) * a.cap + gs] = key;
              }
            }
            kn += uint32_t(__popcll(bm));
          }
        }
        if (lane == 0) wl.s_kn = kn;
        WaveLdsSync();   // the hit list is rewritten next
      };

      // a hit's lanes append their sums (packed int16) and tag to the list
      auto append_hit = [&](bool hit, uint64_t hb, const uint32_t* pk, uint32_t jt) {
        // whits <= 64 here and a tile adds at most 64: the list (128)
        // always has room, so the sums are dead before any drain
        const uint32_t nh = uint32_t(__popcll(hb));
        if (hit) {
          const uint32_t hs =
              whits + __builtin_amdgcn_mbcnt_hi(uint32_t(hb >> 32),
                                                __builtin_amdgcn_mbcnt_lo(uint32_t(hb), 0u));
          wl.hsum[hs][0] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
          if constexpr (!NR) wl.hsum[hs][1] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
          wl.hmeta[hs] = (jt << 6) | uint32_t(lane);
        }
        whits += nh;
        if (ABL & 8) st_hits += nh;
        // no wait for the writes: a wave's LDS instructions execute in
        // order, so the drain's later reads see them (compiler barrier only)
        asm volatile("" ::: "memory");
      };

      // one tile: the MFMAs, then the hit test
      auto tile = [&](const uint32_t (&cd)[NW], const uint32_t (&cd_b)[NW], uint32_t jt) {
        const uint32_t rows_left = n - jt * kDpPerTile;
        if constexpr (NR) {
          // this lane's byte of each step at byte 2 (s' % 2) of dword s' / 2
          const uint32_t sh = uint32_t((lane >> 4) & 1) * 8u;
          uint32_t sa[NW], sb[NW];
#pragma unroll
          for (int i = 0; i < NW; ++i) {
            sa[i] = cd[i] >> sh;
            sb[i] = cd_b[i] >> sh;
          }
          v4i acc_a, acc_b;
          TileSmfmac16<K, SMX_SCAN_R16, (ABL & 64) != 0>(sa, sb, b, grp_tab, pos_tab, acc_a, acc_b);
          if (ABL & 4) {
            int x = acc_a[0] ^ acc_b[0];
#pragma unroll
            for (int i = 1; i < 4; ++i) x ^= acc_a[i] ^ acc_b[i];
            if (x == 0x7fffffff) a.cand_count[0] = x;
            return;
          }
          if (rows_left < uint32_t(kDpPerTile)) {  // last tile of the leaf
            const int lim = int(rows_left) - 4 * (lane >> 4);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              if (i >= lim) acc_a[i] = 0x7FFF;
              if (16 + i >= lim) acc_b[i] = 0x7FFF;
            }
          }
          const int m = min(min(min(acc_a[0], acc_a[1]), min(acc_a[2], acc_a[3])),
                            min(min(acc_b[0], acc_b[1]), min(acc_b[2], acc_b[3])));
          const bool hit = m <= amax;
          const uint64_t hb = __builtin_amdgcn_ballot_w64(hit);
          if (ABL & 2) {
            if (hb == 0x1234567ull) a.cand_count[0] = 1u;
            return;
          }
          if (hb) {
            uint32_t pk[4];
            pk[0] = __builtin_amdgcn_perm(uint32_t(acc_a[1]), uint32_t(acc_a[0]), 0x05040100u);
            pk[1] = __builtin_amdgcn_perm(uint32_t(acc_a[3]), uint32_t(acc_a[2]), 0x05040100u);
            pk[2] = __builtin_amdgcn_perm(uint32_t(acc_b[1]), uint32_t(acc_b[0]), 0x05040100u);
            pk[3] = __builtin_amdgcn_perm(uint32_t(acc_b[3]), uint32_t(acc_b[2]), 0x05040100u);
            append_hit(hit, hb, pk, jt);
          }
        } else {
          v16i acc;
          if constexpr (DN) acc = TileSmfmacD<K, R>(cd, b, bd, grp_tab, pos_tab, hot_tab);
          else acc = TileSmfmac<K, R, (ABL & 64) != 0>(cd, b, grp_tab, pos_tab);
          if (ABL & 4) {
            int x = acc[0];
#pragma unroll
            for (int i = 1; i < 16; ++i) x ^= acc[i];
            if (x == 0x7fffffff) a.cand_count[0] = x;
            return;
          }
          if (rows_left < uint32_t(kDpPerTile)) {  // last tile of the leaf
            // row (i&3) + 8(i>>2) + 4h >= rows_left, against one per-tile value
            // (16 hoisted row numbers would cost 16 registers for the loop)
            const int lim = int(rows_left) - 4 * h;
#pragma unroll
            for (int i = 0; i < 16; ++i)
              if ((i & 3) + 8 * (i >> 2) >= lim) acc[i] = 0x7FFF;
          }
          int m = min(min(acc[0], acc[1]), acc[2]);
#pragma unroll
          for (int i = 3; i < 15; i += 2) m = min(min(m, acc[i]), acc[i + 1]);
          m = min(m, acc[15]);
          const bool hit = m <= amax;
          const uint64_t hb = __builtin_amdgcn_ballot_w64(hit);
          if (ABL & 2) {   // timing ablation: the hit test without its list
            if (hb == 0x1234567ull) a.cand_count[0] = 1u;
            return;
          }
          if (hb) {
            // the 16 sums as int16 pairs, one v_perm_b32 each (low halves of
            // acc[2k] and acc[2k + 1]; a shift + or was two VALU per pair)
            uint32_t pk[8];
#pragma unroll
            for (int k = 0; k < 8; ++k)
              pk[k] = __builtin_amdgcn_perm(uint32_t(acc[2 * k + 1]), uint32_t(acc[2 * k]),
                                            0x05040100u);
            append_hit(hit, hb, pk, jt);
          }
        }
      };
      // a hit list over half full is drained between tiles with the B
      // fragments dead (reloaded after, from L2): the drain's registers
      // then never compete with them (rare: ~1 hit lane per tile)
      // (the 16-slot-only kernel keeps its B fragments through the drain: a
      // reload there would add loads to one side of the join, and the ring's
      // in-flight code loads would be waited for at the join)
      auto drain_mid = [&]() {
        if (whits > 64u) {
          drain();
          whits = 0;
          if constexpr (!DEEP) load_b();
          // (DEEP: nothing left in flight on this rare path, so that the
          // join keeps the ring's exact load counts -- the drain's stores
          // would otherwise make every later wait on the ring vmcnt(0))
          if constexpr (DEEP) __builtin_amdgcn_s_waitcnt(0);
        }
      };

      if (ABL & 8) st_t1 = __builtin_amdgcn_s_memtime();
      if constexpr (DEEP) {
        // 16-slot tiles only (few queries per leaf: a tile's MFMA work is
        // small against its code load): a ring of D tiles in flight per wave
        // instead of one, the registers freed by the 32-slot path's B
        // fragments.  The tiles come from the same pair claims (the current
        // pair, then the pair claimed ahead); every refill issues its load
        // unconditionally (the last tile again at the end), so the wait for a
        // slot's codes leaves the later slots' loads in flight.
        constexpr int D = SMX_RING16 > 0 ? SMX_RING16 : (NW <= 3 ? 4 : 3);
        uint32_t cur = j, pe = min(j + 2, end), na = end;
        uint32_t na_raw = claim2(sg);
        bool na_known = false;
        auto produce = [&](uint32_t& tn) -> bool {   // the tile after the last produced one
          if (cur + 1 < pe) {
            tn = ++cur;
            return true;
          }
          if (!na_known) {
            na = __builtin_amdgcn_readfirstlane(na_raw);
            na_known = true;
          }
          if (na >= end) return false;
          cur = na;
          pe = min(na + 2, end);
          na_raw = claim2(sg);
          na_known = false;
          tn = cur;
          return true;
        };
        using CV = CodeVec<NW>;
        CV ra[D], rb[D];
        uint32_t tq[D];
        bool ok[D];
        auto load_slot = [&](uint32_t t, CV& x, CV& y) {
          const uint8_t* p = tile_ptr(t);
          x = *reinterpret_cast<const CV*>(p);
          y = *reinterpret_cast<const CV*>(p + 16 * W);
        };
        tq[0] = j;
        ok[0] = true;
        load_slot(j, ra[0], rb[0]);
#pragma unroll
        for (int d = 1; d < D; ++d) {
          ok[d] = ok[d - 1] && produce(tq[d]);
          if (!ok[d]) tq[d] = tq[d - 1];
          load_slot(tq[d], ra[d], rb[d]);
        }
        // one ring slot: its tile (when it holds one), then its refill -- the
        // tile after the last produced one.  The loop leaves only at the
        // bottom, when slot 0 is empty (the slots empty in order): early
        // exits between the slots put the ring's registers through merges
        // that cost exact load counts (every wait became vmcnt(0/1)).
        bool live = true;
        auto step = [&](auto dc) {
          constexpr int d = decltype(dc)::value;
          if (ok[d]) {
            uint32_t xa[NW], xb[NW];
#pragma unroll
            for (int i = 0; i < NW; ++i) {
              xa[i] = ra[d][i];
              xb[i] = rb[d][i];
            }
            tile(xa, xb, tq[d]);
            ++tiles_done;
          }
          const uint32_t prev = tq[(d + D - 1) % D];
          ok[d] = live && produce(tq[d]);
          live = ok[d];
          if (!ok[d]) tq[d] = prev;
          load_slot(tq[d], ra[d], rb[d]);
          drain_mid();
        };
        for (;;) {
          EachSlot<0, D>(step);
          if (!ok[0]) break;
        }
      } else {
        // the tiles this wave takes, a claimed pair at a time with the next
        // pair claimed ahead; two code buffers in turn (the load of the next
        // tile is in flight while this one computes; a rotating copy would
        // force a wait for it at the copy)
        uint32_t pe = min(j + 2, end);        // the current pair [.., pe)
        uint32_t na_raw = claim2(sg);          // the next pair (lane 0)
        bool na_known = false;
        uint32_t na = end;
        auto next_tile = [&](uint32_t t, uint32_t& tn) -> bool {
          if (t + 1 < pe) {
            tn = t + 1;
            return true;
          }
          if (!na_known) {
            na = __builtin_amdgcn_readfirstlane(na_raw);
            na_known = true;
          }
          if (na >= end) return false;
          tn = na;
          return true;
        };
        auto advance = [&](uint32_t t, uint32_t tn) {
          if (!(t + 1 < pe)) {   // moved into the pair claimed ahead: claim another
            pe = min(tn + 2, end);
            na_raw = claim2(sg);
            na_known = false;
          }
        };
        {
          uint32_t cb[NW], cb_b[NW];
          uint32_t t = j, tn = 0;
          for (;;) {
            bool more = next_tile(t, tn);
            // unconditional (the current tile again when none follows): one
            // load per tile on every path, so the wait for this tile's codes
            // leaves the next tile's load in flight (vmcnt(1), not vmcnt(0))
            load_codes(more ? tn : t, cb, cb_b);
            tile(codes, codes_b, t);
            ++tiles_done;
            if (!more) break;
            drain_mid();
            advance(t, tn);
            t = tn;
            more = next_tile(t, tn);
            load_codes(more ? tn : t, codes, codes_b);
            tile(cb, cb_b, t);
            ++tiles_done;
            if (!more) break;
            drain_mid();
            advance(t, tn);
            t = tn;
          }
        }
      }
      if (whits) {
        drain();
        whits = 0;
      }
      };
      static_assert(NRW == 0 || NRW == int(kNarrowOnly), "one tile width per kernel");
      if constexpr (NRW == int(kNarrowOnly)) {
        run_seg(std::true_type{});
      } else {
        run_seg(std::false_type{});
      }
      if (ABL & 8) st_t2 = __builtin_amdgcn_s_memtime();
      if (ABL & 8) {
        uint32_t sv = lane < Q ? wl.qcnt[nst * 32u + uint32_t(lane)] : 0u;
        for (int off = 32; off > 0; off >>= 1) sv += uint32_t(__shfl_xor(int(sv), off));
        st_surv = sv;
      }
      // the segment keeps its stage entry when it staged survivors
      if (__builtin_amdgcn_readfirstlane(wl.s_kn) > kn_seg) ++nst;
      if ((ABL & 8) && lane == 0)
        StampItem(a, worker, item, st_rt, st_t0, st_t1, st_t2, __builtin_amdgcn_s_memtime(),
                  uint64_t(tiles_done) | (uint64_t(st_hits) << 16) | (uint64_t(st_surv) << 40));
    }
  }
  list_flush();
}

// Stage entry point of the threshold select: per set of kSeedKeys ordered
// distance bits (0xFFFFFFFF = none), ThresholdOfVals' key, or kNoThreshold
// when the set holds fewer than kk values (SeedTau's rule).
__global__ void __launch_bounds__(256) kth_keys_kernel(const uint32_t* __restrict__ vals,
                                                       uint32_t kk, uint64_t* __restrict__ out) {
  __shared__ uint32_t s_n;
  const int tid = threadIdx.x;
  if (tid == 0) s_n = 0;
  __syncthreads();
  uint32_t v[kSeedPerThread], n = 0;
#pragma unroll
  for (int k = 0; k < kSeedPerThread; ++k) {
    v[k] = vals[size_t(blockIdx.x) * kSeedKeys + uint32_t(tid) + 256u * uint32_t(k)];
    n += v[k] != 0xFFFFFFFFu ? 1u : 0u;
  }
  atomicAdd(&s_n, n);
  __syncthreads();
  const uint64_t T = (kk > 0 && s_n >= kk) ? ThresholdOfVals(v, kk) : kNoThreshold;
  if (tid == 0) out[blockIdx.x] = T;
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

// ---------------------------------------------------------------------------
// Overflow recovery on the device (no host round trip).  A query whose list
// overflowed (more candidates under its threshold than the list holds) keeps
// the first `cap` arrivals, every one a genuine candidate; their k'-th
// smallest key is then a valid, tighter threshold.  The block rescans the
// query's L leaves with the same sums, distances and keys as the scan
// (VALU, pair tables as SeedTau) and keeps the keys under it; cap >= 2 k'
// makes each further pass drop at least cap - k' keys, so this converges.
// Rare path: grid-stride over the queries, most blocks only read counts.
// ---------------------------------------------------------------------------
// k-th smallest (1-based) of n u64 keys in global memory, block-wide: eight
// 8-bit radix passes over the keys that share the prefix found so far.
__device__ uint64_t KthSmallestKey(const uint64_t* keys, uint32_t n, uint32_t k, uint32_t* hist,
                                   uint32_t* wsum) {
  __shared__ uint64_t s_prefix;
  __shared__ uint32_t s_need;
  const int tid = threadIdx.x;
  if (tid == 0) { s_prefix = 0; s_need = k; }
  for (int pass = 0; pass < 8; ++pass) {
    const int shift = 56 - 8 * pass;
    hist[tid] = 0;
    __syncthreads();
    const uint64_t prefix = s_prefix;
    const uint32_t need = s_need;
    for (uint32_t i = tid; i < n; i += 256) {
      const uint64_t key = keys[i];
      if (pass == 0 || (key >> (shift + 8)) == (prefix >> (shift + 8)))
        atomicAdd(&hist[uint32_t(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    const uint32_t hv = hist[tid];
    const uint32_t inc = BlockInclusiveScan256(hv, wsum);
    __syncthreads();   // every thread has read s_prefix / s_need
    if (inc - hv < need && inc >= need) {
      s_prefix = prefix | (uint64_t(tid) << shift);
      s_need = need - (inc - hv);
    }
    __syncthreads();
  }
  return s_prefix;
}

// Query qi's list after a rescan under the k'-th smallest of its first cap
// stored keys (repeated while it still overflows); returns the new count.
// Block-wide (256 threads); runtime K (a rare path: one VALU pass over the
// query's L leaves per round, pair tables as SeedTau).
__device__ __forceinline__ uint32_t RescanQuery(const RescanArgs& a, int qi, uint32_t n) {
  __shared__ __align__(16) int8_t lut[2 * kMaxBlocks * 16];
  __shared__ int16_t ptab[2 * (kMaxBlocks / 4) * 256];   // NB <= 16
  __shared__ uint32_t hist[256], wsum[4], s_n;
  const int tid = threadIdx.x;
  const int K = a.ksteps, NB = (K + 1) / 2, NW = (NB + 3) / 4, W = 4 * NW;
  if (tid == 0) atomicAdd(&a.stats[10], 1u);
  for (int e = tid; e < 2 * K * 16 / 4; e += 256)
    reinterpret_cast<uint32_t*>(lut)[e] =
        reinterpret_cast<const uint32_t*>(a.lut + size_t(qi) * LutRows(K) * 16)[e];
  __syncthreads();
  for (int i = 0; i < 2 * NB; ++i) {
    const int h = i / NB, j = i % NB, s0 = 2 * j, s1 = 2 * j + 1;
    int v = lut[(2 * s0 + h) * 16 + CodePairLo(uint32_t(tid))];
    if (s1 < K) v += lut[(2 * s1 + h) * 16 + CodePairHi(uint32_t(tid))];
    ptab[i * 256 + tid] = int16_t(v);
  }
  const float inv = a.inv[qi];
  uint64_t* row = a.cand + size_t(qi) * a.cap;
  while (n > a.cap) {   // block-uniform
    const uint64_t T = KthSmallestKey(row, a.cap, uint32_t(a.kk), hist, wsum);
    if (tid == 0) {
      s_n = 0;
      atomicAdd(&a.stats[11], 1u);
      a.tau_key[qi] = T;
    }
    __syncthreads();
    for (int i = 0; i < a.L; ++i) {
      const int32_t leaf = a.topl_leaf[size_t(qi) * a.L + i];
      if (leaf < 0) continue;
      const uint32_t ln = a.leaf_size[leaf];
      const uint64_t t0 = a.tile_off[leaf];
      const uint64_t moff = a.member_off[leaf];
      const float bias = a.residual ? a.topl_dist[size_t(qi) * a.L + i] : 0.0f;
      for (uint32_t dp = tid; dp < ln; dp += 256) {
        const uint32_t* tp = reinterpret_cast<const uint32_t*>(
            a.tiles + ((t0 + (dp >> 5)) * 64 + (dp & 31)) * W);
        uint32_t c0[4] = {0, 0, 0, 0}, c1[4] = {0, 0, 0, 0};
        for (int w = 0; w < NW; ++w) {
          c0[w] = tp[w];
          c1[w] = tp[8 * W + w];   // + 32 lanes * W bytes
        }
        int acc = 0;
        for (int j = 0; j < NB; ++j) {
          const uint32_t b0 = (c0[j >> 2] >> (8 * (j & 3))) & 0xFFu;
          const uint32_t b1 = (c1[j >> 2] >> (8 * (j & 3))) & 0xFFu;
          acc += int(ptab[j * 256 + b0]) + int(ptab[(NB + j) * 256 + b1]);
        }
        const float d = DistOf(acc, inv, bias);
        const uint32_t tie = a.shift > 0 ? ((uint32_t(leaf) << a.shift) | dp) : a.members[moff + dp];
        const uint64_t key = (uint64_t(OrderedBits(d)) << 32) | tie;
        if (key <= T) {
          const uint32_t p = atomicAdd(&s_n, 1u);
          if (p < a.cap) row[p] = key;
        }
      }
    }
    __syncthreads();
    n = s_n;
    __syncthreads();   // every thread has read s_n before the next round resets it
  }
  if (tid == 0) a.cand_count[size_t(qi) * kCounterStride] = n;
  __syncthreads();
  return n;
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

// Partition scores of the single-query path (ScannInterface::Search ->
// KMeansTreeNode, kmeans_tree_node.h:159-163): DenseDistanceOneToMany, whose
// AVX2 kernel (one_to_many_symmetric.h:376-503) accumulates each center in
// the A.8 order of ExactDistance -- not the batched transposed FMA chain of
// partition_scores_kernel, so its biases differ in the last bits.  One
// thread per (query, center); also the per-call state reset.
__global__ void __launch_bounds__(256) partition_scores_a8_kernel(
    const float* __restrict__ queries, int nq, int dim, const float* __restrict__ centers,
    int nl, int metric, float* __restrict__ scores, StateInit init) {
  const uint32_t gt = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t gs = gridDim.x * blockDim.x;
  for (uint32_t i = gt; i < init.n_counters; i += gs) init.counters[size_t(i) * kCounterStride] = 0u;
  for (uint32_t i = gt; i < init.n_stats; i += gs) init.stats[i] = 0u;
  for (uint32_t i = gt; i < init.n_cand; i += gs) init.cand_count[size_t(i) * kCounterStride] = 0u;
  for (uint32_t i = gt; i < init.n_tau; i += gs) init.tau[i] = kNoThreshold;
  const size_t p = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (p >= size_t(nq) * nl) return;
  const int qi = int(p / nl), c = int(p % nl);
  scores[p] = ExactDistance(queries + size_t(qi) * dim, centers + size_t(c) * dim, dim, metric);
}

// ---------------------------------------------------------------------------
// Final selection per query: exact k' best by (distance, tie id) among the
// candidates, tie -> global id, SOAR de-duplication, exact reorder, and the
// (distance, id) sort of SortAndDropResults.
// LDS: keys[cap_pow2] u64 | q[dim] f32 | gid/dist scratch.
// ---------------------------------------------------------------------------
// The float row of a candidate known by its global id: the shard's own copy
// (member_rows[row_of[gid]]; row_of exists for shards at shift 0 and spilled
// shards only) or the dataset's row.
__device__ __forceinline__ const float* RowOfId(const SelectArgs& a, uint32_t gid) {
  if (a.member_rows) {
    const uint32_t slot = a.row_of[gid];
    SMX_CHECK(slot, a.bd.members, "row_of slot");
    return a.member_rows + uint64_t(slot) * uint64_t(a.dim);
  }
  return a.dataset + uint64_t(gid) * uint64_t(a.dim);
}

__device__ void FinalSelectQuery(const SelectArgs& a, int qi) {
  extern __shared__ uint64_t lds[];
  uint32_t raw_n = a.cand_count[size_t(qi) * kCounterStride];
  if (raw_n > a.cap) {   // block-uniform: the list overflowed, rescan on the device
    if (threadIdx.x == 0) {
      a.overflow[0] = 1u;
      atomicMax(&a.overflow[1], raw_n);
    }
    raw_n = RescanQuery(a.rescan, qi, raw_n);
  }

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
        const float* x = nullptr;
        if (a.shift > 0) {
          const uint32_t tie = uint32_t(key & 0xFFFFFFFFu);
          const uint32_t leaf = tie >> a.shift;
          const uint32_t local = tie & ((1u << a.shift) - 1u);
          // the member's own row by its slot (row_of is kept for shift 0 only)
          if (a.member_rows) x = a.member_rows + (a.member_off[leaf] + local) * uint64_t(a.dim);
          if (a.row_base)
            key = (key & 0xFFFFFFFF00000000ull) | ((leaf << a.shift) | (local + a.row_base[leaf]));
        }
        if (a.reorder && !x) x = RowOfId(a, gid[i]);
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
    for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) {
      const float* x;
      if (a.member_rows && a.shift > 0 && a.disjoint) {
        // keys[i] still holds candidate i's packed tie (no dedupe ran): its
        // member slot (a disjoint shard keeps no global-id -> slot table)
        const uint32_t tie = uint32_t(keys[i] & 0xFFFFFFFFu);
        x = a.member_rows +
            (a.member_off[tie >> a.shift] + (tie & ((1u << a.shift) - 1u))) * uint64_t(a.dim);
      } else {
        x = RowOfId(a, gid[i]);
      }
      dist[i] = ExactDistance(q, x, a.dim, a.metric);
    }
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

__global__ void __launch_bounds__(256) final_select_kernel(SelectArgs a) {
  FinalSelectQuery(a, int(blockIdx.x));
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
constexpr uint32_t kBlockRankMin = 160;   // more keys: BlockRank256, fewer: counting rank
constexpr int kFsBins = 256;

// Exact distances of m candidates (rows + rowid[i] * dim) into dist[], 8
// lanes per candidate: lane l of a group owns accumulator l of the A.8 layout
// (dims l, l+8, ...) and the folds follow ExactDistance exactly.  256
// threads; ends with a barrier.
constexpr int kXMax = 16;   // dims per lane held in registers (dim <= 128)
#ifndef SMX_XPASS
#define SMX_XPASS 2
#endif
constexpr int kXPass = SMX_XPASS;   // 32-candidate passes whose rows are in flight together
#ifndef SMX_XPASS_EXACT
#define SMX_XPASS_EXACT 4
#endif
constexpr int kXPassExact = SMX_XPASS_EXACT;   // the same at dims of exactly 12 or 16 steps

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
  // the tails of ExactDistance: 4-wide at j8 (lanes 0..3), 2-wide at j2
  // (lanes 2, 3), scalar at j1
  int j = j8;
  const bool has4 = j + 4 <= dim;
  if (has4) j += 4;
  const int j2 = j;
  const bool has2 = j + 2 <= dim;
  if (has2) j += 2;
  const int j1 = j;
  const bool has1 = j < dim;
  // folds of one candidate's 8 accumulators (lane l holds accumulator l)
  auto finish = [&](float acc, float q4, float x4, float q2, float x2, float q1, float x1) {
    const float hi4 = __shfl(acc, gb + ((l + 4) & 7));
    float sv = __fadd_rn(hi4, acc);   // lanes l < 4: s[l]
    if (has4 && l < 4) sv = term(sv, q4, x4);
    if (has2 && (l == 2 || l == 3)) sv = term(sv, q2, x2);
    const float s1 = __shfl(sv, gb + 1), s2 = __shfl(sv, gb + 2), s3 = __shfl(sv, gb + 3);
    float r = __fadd_rn(__fadd_rn(sv, s2), __fadd_rn(s1, s3));
    if (has1) r = term(r, q1, x1);
    return r;
  };
  const int c4 = min(j8 + (l & 3), dim - 1), c2 = min(j2 + (l & 1), dim - 1), c1 = min(j1, dim - 1);
  // NJ 8-dim steps held in registers, NP 32-candidate passes whose rows are in
  // flight together.  kExact: dim's steps are exactly NJ, so lane l's loads
  // x[l + 8k] stay inside the row and share one address (immediate offsets);
  // otherwise they are clamped and the accumulation stops at j8.
  auto passes = [&](auto nj_c, auto np_c, auto exact_c) {
    constexpr int NJ = decltype(nj_c)::value, NP = decltype(np_c)::value;
    constexpr bool kExact = decltype(exact_c)::value;
    float qv[NJ];
    const float* ql = q + l;
#pragma unroll
    for (int k = 0; k < NJ; ++k) qv[k] = kExact ? ql[8 * k] : q[min(l + 8 * k, dim - 1)];
    const float q4 = q[c4], q2 = q[c2], q1 = q[c1];
    const int nj = j8 >> 3;
    for (uint32_t base = 0; base < m; base += 32 * NP) {
      float xv[NP][NJ], x4[NP], x2[NP], x1[NP];
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const uint32_t i = min(base + 32 * p + uint32_t(tid >> 3), m - 1);
        const float* x = rows + size_t(rowid[i]) * dim;
        const float* xl = x + l;
#pragma unroll
        for (int k = 0; k < NJ; ++k) xv[p][k] = kExact ? xl[8 * k] : x[min(l + 8 * k, dim - 1)];
        x4[p] = x[c4];
        x2[p] = x[c2];
        x1[p] = x[c1];
      }
      float r[NP];
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        float acc = 0.0f;
#pragma unroll
        for (int k = 0; k < NJ; ++k)
          if (kExact || k < nj) acc = term(acc, qv[k], xv[p][k]);
        r[p] = finish(acc, q4, x4[p], q2, x2[p], q1, x1[p]);
      }
      __syncthreads();   // every read of rowid/dist for these passes is done
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const uint32_t i = base + 32 * p + uint32_t(tid >> 3);
        if (l == 0 && i < m) dist[i] = r[p];
      }
    }
  };
  using I12 = std::integral_constant<int, 12>;
  using I16 = std::integral_constant<int, 16>;
  using P2 = std::integral_constant<int, kXPass>;
  using P4 = std::integral_constant<int, kXPassExact>;
  using P3 = std::integral_constant<int, kXPassExact - 1>;
  if (j8 == 96) {
    passes(I12{}, P4{}, std::true_type{});   // dims 96..103 (glove-100, deep-96)
  } else if (j8 == 128) {
    passes(I16{}, P3{}, std::true_type{});   // dims 128..135 (sift-128)
  } else if (dim <= 8 * kXMax) {
    passes(I16{}, P2{}, std::false_type{});
  } else {
    for (uint32_t base = 0; base < m; base += 32) {
      const uint32_t i = base + uint32_t(tid >> 3);
      const bool act = i < m;
      const float* x = rows + size_t(rowid[act ? i : 0]) * dim;
      float acc = 0.0f;
#pragma unroll 8
      for (int jj = 0; jj < j8; jj += 8) acc = term(acc, q[jj + l], x[jj + l]);
      const float r = finish(acc, q[c4], x[c4], q[c2], x[c2], q[c1], x[c1]);
      __syncthreads();   // every read of rowid/dist for this pass is done
      if (l == 0 && act) dist[i] = r;
    }
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
  SMX_PHASE(2, qi, 0);
  uint32_t raw_n = a.cand_count[size_t(qi) * kCounterStride];
  if (raw_n > a.cap) {   // block-uniform: the list overflowed, rescan on the device
    if (threadIdx.x == 0) {
      a.overflow[0] = 1u;
      atomicMax(&a.overflow[1], raw_n);
    }
    raw_n = RescanQuery(a.rescan, qi, raw_n);
  }
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
    if (ok) {
      for (uint32_t i = tid; i < n; i += 256) {
        const uint64_t key = ck[i];
        if (uint32_t(key >> 32) <= lim) sel[atomicAdd(&s_c, 1u)] = key;
      }
    } else {   // block-uniform: > kSelMax keys on one distance value (ties):
      // the k-th key itself by a radix select over the whole keys (unique),
      // then exactly the k keys up to it
      const uint64_t kth = KthSmallestKey(ck, n, k, hist, wsum);
      for (uint32_t i = tid; i < n; i += 256) {
        const uint64_t key = ck[i];
        if (key <= kth) {
          // (equal keys -- SOAR copies without the global top-N tie -- can
          // put one more key than k at kth: it ranks >= k and is dropped)
          const uint32_t pos = atomicAdd(&s_c, 1u);
          if (pos < uint32_t(kSelMax)) sel[pos] = key;
        }
      }
    }
    __syncthreads();
  }
  SMX_PHASE(2, qi, 1);
  const uint32_t c = n <= uint32_t(kSelMax) ? n : min(s_c, uint32_t(kSelMax));
  if ((a.disjoint || a.shift > 0) && c > kBlockRankMin) {
    // distinct keys (packed ids, or global ids without SOAR copies): the
    // wave-sort block rank, empty slots padded above every distance (its
    // fixed cost beats the counting rank's O(c) per key only for larger c:
    // glove's ~100 keys measured 1 us slower)
    const uint64_t key = uint32_t(tid) < c ? sel[tid] : (0xFFFFFFFF00000000ull | uint32_t(tid));
    const uint32_t r = BlockRank256(key, out);   // (out: its scratch until it returns)
    if (uint32_t(tid) < c) out[r] = key;
  } else if (uint32_t(tid) < c) {
    // counting rank (stable: equal keys, the SOAR copies of an index without
    // the global top-N tie, take consecutive ranks)
    const uint64_t key = sel[tid];
    out[RankStable(sel, c, key, uint32_t(tid))] = key;
  }
  __syncthreads();
  SMX_PHASE(2, qi, 2);
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
      SMX_CHECK(leaf, a.bd.nl, "select leaf");
      const uint64_t slot = a.member_off[leaf] + local;
      SMX_CHECK(slot, a.bd.members, "select member");
      tie = a.members[slot];
      rid = a.member_rows ? uint32_t(slot) : tie;
      if (a.shard_out && a.row_base)   // whole-index tie for the merge
        out[tid] = (key & 0xFFFFFFFF00000000ull) |
                   ((leaf << a.shift) | (local + a.row_base[leaf]));
    } else if (a.member_rows) {   // ties by global id (no global top-N): its slot
      rid = a.row_of[tie];
    }
    SMX_CHECK(rid, a.member_rows ? a.bd.members : uint64_t(a.bd.datapoints), "select row");
    gid[tid] = tie;
    rowid[tid] = rid;
    dist[tid] = FromOrdered(uint32_t(key >> 32));
  }
  __syncthreads();
  SMX_PHASE(2, qi, 3);
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
    {   // (gid, slot) keys are distinct: the block rank (m <= kSelMax = 256)
      const uint64_t key = uint32_t(tid) < m ? (uint64_t(gid[tid]) << 32) | uint32_t(tid) : ~0ull - uint32_t(tid);
      const uint32_t r = BlockRank256(key, sel);
      if (uint32_t(tid) < m) sel[r] = key;
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
    {   // the run starts' (distance, id) keys are distinct; the rest padded above
      const uint32_t r =
          BlockRank256(o != ~0ull ? o : (0xFFFFFFFF00000000ull | uint32_t(tid)), out);
      if (o != ~0ull) atomicAdd(&s_c, 1u);
      if (o != ~0ull && r < uint32_t(a.pre_nn)) {
        gid[r] = uint32_t(o & 0xFFFFFFFFu);
        dist[r] = FromOrdered(uint32_t(o >> 32));
        rowid[r] = hist[tid];
      }
    }
    __syncthreads();
    m = min(s_c, uint32_t(a.pre_nn));
  }
  SMX_PHASE(2, qi, 4);
  if (a.reorder && !a.pre_only) ExactDistances8(a, rows, rowid, m, dist, qi);
  SMX_PHASE(2, qi, 5);
  // final (distance, global id) rank; keep the output width
  const uint32_t keep = min(m, uint32_t(a.out_width));
  uint64_t fkey = 0;
  if (uint32_t(tid) < m) {
    fkey = (uint64_t(OrderedBits(dist[tid])) << 32) | gid[tid];
    sel[tid] = fkey;
  }
  __syncthreads();
  // (distance, id) keys are distinct (one entry per id): the block rank for
  // many keys, the counting rank for few
  uint32_t r;
  if (m > kBlockRankMin) {
    __syncthreads();   // sel is the block rank's scratch
    r = BlockRank256(uint32_t(tid) < m ? fkey : (0xFFFFFFFF00000000ull | uint32_t(tid)), sel);
  } else {
    r = uint32_t(tid) < m ? CountLess(sel, m, fkey) : 0u;
  }
  if (uint32_t(tid) < m) {
    const uint64_t key = fkey;
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
  SMX_PHASE(2, qi, 6);
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
      // equal keys in two lists (SOAR copies without the global top-N tie)
      // rank by list: the lower list's copy first
      int lo = 0, hi = int(cnt[v]);
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const uint64_t x = lk[v * kk + mid];
        if (x < key || (v < w && x == key)) lo = mid + 1; else hi = mid;
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
    {   // (gid, slot) keys are distinct: the block rank (m <= kSelMax = 256)
      const uint64_t key = uint32_t(tid) < m ? (uint64_t(gid[tid]) << 32) | uint32_t(tid) : ~0ull - uint32_t(tid);
      const uint32_t r = BlockRank256(key, sel);
      if (uint32_t(tid) < m) sel[r] = key;
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

// ---------------------------------------------------------------------------
// The merge for wide shard lists (k' up to 2048 per shard, world x k' up to
// kMergeWideEntries per launch; a SOAR shard keeps k' = 2 x pre_reorder_nn,
// tree_ah_hybrid_residual.h:263-267).  The same global rank as
// merge_shards_kernel (position in its list + smaller keys of every other
// list, equal keys by list), with dynamic LDS sized by the call.  kPartial:
// block (query, group) merges the group's lists into one list of the k'
// smallest entries (sorted by (key, list); padded with UINT64_MAX), so that
// more lists than one launch holds merge in rounds -- the k' smallest of a
// union are the k' smallest of its parts' k' smallest.  Otherwise the SOAR
// de-duplication (tree_ah_hybrid_residual.cc:779-783: a datapoint's two copies
// averaged 0.5a + 0.5b), the pre_reorder_nn cut by (distance, id) and the
// final (distance, id) order, on bitonic sorts of up to 2048 keys.
// ---------------------------------------------------------------------------
constexpr int kMergeWideEntries = 8192;

size_t MergeWideLds(int lists, int kk) {
  uint32_t kkp2 = 1;
  while (kkp2 < uint32_t(kk)) kkp2 <<= 1;
  return size_t(lists) * size_t(kk) * 8 + size_t(kkp2) * (8 + 8 + 4 * 5);
}

template <bool kPartial>
__global__ void __launch_bounds__(256) merge_shards_wide_kernel(MergeArgs a, int group_lists) {
  extern __shared__ uint64_t mlds[];
  __shared__ uint32_t cnt[64], s_c;
  const int tid = threadIdx.x;
  const int qi = blockIdx.x;
  const int kk = a.kk;
  const int w0 = int(blockIdx.y) * group_lists;
  const int W = min(group_lists, a.world - w0);
  const uint32_t kkp2 = NextPow2(uint32_t(kk));
  uint64_t* lk = mlds;                          // [W * kk] the lists' keys
  uint64_t* sel = lk + size_t(W) * kk;          // [kkp2] the kk smallest, by rank
  uint64_t* aux = sel + kkp2;                   // [kkp2] sort keys
  uint32_t* sid = reinterpret_cast<uint32_t*>(aux + kkp2);
  float* sex = reinterpret_cast<float*>(sid + kkp2);
  uint32_t* gid = reinterpret_cast<uint32_t*>(sex + kkp2);
  float* dist = reinterpret_cast<float*>(gid + kkp2);
  float* ex = dist + kkp2;
  auto entry = [&](int w, int j) -> const ShardEntry& {
    return a.entries[(size_t(w0 + w) * a.nq + qi) * kk + j];
  };
  for (int e = tid; e < W * kk; e += 256) lk[e] = entry(e / kk, e % kk).key;
  if (tid == 0) s_c = 0;
  __syncthreads();
  for (int w = tid; w < W; w += 256) {   // valid entries: the padding sorts last
    int lo = 0, hi = kk;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (lk[w * kk + mid] != ~0ull) lo = mid + 1; else hi = mid;
    }
    cnt[w] = uint32_t(lo);
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
        const uint64_t x = lk[v * kk + mid];
        if (x < key || (v < w && x == key)) lo = mid + 1; else hi = mid;
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
  if constexpr (kPartial) {
    ShardEntry* out = a.out_entries + (size_t(blockIdx.y) * a.nq + qi) * kk;
    for (uint32_t i = tid; i < uint32_t(kk); i += 256) {
      ShardEntry e;
      e.key = i < m ? sel[i] : ~0ull;
      e.id = i < m ? sid[i] : 0u;
      e.exact = i < m ? sex[i] : 0.0f;
      out[i] = e;
    }
  } else {
    for (uint32_t i = tid; i < m; i += 256) {
      gid[i] = sid[i];
      dist[i] = FromOrdered(uint32_t(sel[i] >> 32));
      ex[i] = sex[i];
    }
    __syncthreads();
    if (!a.disjoint) {
      // copies of one datapoint next to each other: sort (gid << 32 | slot)
      const uint32_t mp2 = NextPow2(max(m, 1u));
      for (uint32_t i = tid; i < mp2; i += 256)
        aux[i] = i < m ? ((uint64_t(gid[i]) << 32) | i) : ~0ull;
      __syncthreads();
      BitonicSort(aux, mp2);
      // run starts: (ordered(averaged distance) << 32 | gid), the rest MAX;
      // sex[i] = the exact distance of the run starting at sorted position i
      for (uint32_t i = tid; i < mp2; i += 256) {
        uint64_t o = ~0ull;
        if (i < m) {
          const uint32_t g = uint32_t(aux[i] >> 32);
          if (i == 0 || uint32_t(aux[i - 1] >> 32) != g) {
            const uint32_t s0 = uint32_t(aux[i] & 0xFFFFFFFFu);
            float d = dist[s0];
            if (i + 1 < m && uint32_t(aux[i + 1] >> 32) == g) {
              const float d2 = dist[uint32_t(aux[i + 1] & 0xFFFFFFFFu)];
              d = __fadd_rn(__fmul_rn(0.5f, d), __fmul_rn(0.5f, d2));
            }
            o = (uint64_t(OrderedBits(d)) << 32) | g;
            sex[i] = ex[s0];
            atomicAdd(&s_c, 1u);
          }
        }
        sel[i] = o;
      }
      __syncthreads();
      BitonicSort(sel, mp2);
      const uint32_t mu = min(s_c, uint32_t(a.pre_nn));
      // the kept datapoints by (averaged distance, id); each one's exact
      // distance from its run start (binary search of the gid-sorted runs)
      for (uint32_t r = tid; r < mu; r += 256) {
        const uint32_t g = uint32_t(sel[r] & 0xFFFFFFFFu);
        uint32_t lo = 0, hi = m;
        while (lo < hi) {
          const uint32_t mid = (lo + hi) >> 1;
          if (uint32_t(aux[mid] >> 32) < g) lo = mid + 1; else hi = mid;
        }
        gid[r] = g;
        dist[r] = FromOrdered(uint32_t(sel[r] >> 32));
        ex[r] = sex[lo];
      }
      __syncthreads();
      m = mu;
    }
    // the final (distance, id) order of the kept m
    const uint32_t mp2 = NextPow2(max(m, 1u));
    for (uint32_t i = tid; i < mp2; i += 256)
      aux[i] = i < m ? ((uint64_t(OrderedBits(a.reorder ? ex[i] : dist[i])) << 32) | gid[i]) : ~0ull;
    __syncthreads();
    BitonicSort(aux, mp2);
    const uint32_t keep = min(m, uint32_t(a.out_width));
    for (int i = tid; i < a.out_width; i += 256) {
      const bool has = uint32_t(i) < keep;
      a.out_idx[size_t(qi) * a.out_width + i] = has ? uint32_t(aux[i] & 0xFFFFFFFFu) : 0u;
      a.out_dist[size_t(qi) * a.out_width + i] =
          has ? FromOrdered(uint32_t(aux[i] >> 32)) : __int_as_float(0x7fc00000);
    }
    if (tid == 0 && a.out_count) a.out_count[qi] = int32_t(keep);
  }
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
    const uint32_t v = cand_count[size_t(i) * kCounterStride];
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
    if (over) stats[0] = 1u;
    stats[1] = max(stats[1], over);
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

__global__ void row_of_kernel(const uint32_t* __restrict__ members, uint64_t m,
                              uint32_t* __restrict__ row_of) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < m) row_of[members[i]] = uint32_t(i);
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
                               int32_t* out_leaf, float* out_dist, float* scores, hipStream_t s,
                               const FrontArgs* front) {
  if (nq == 0) return hipSuccess;
  uint32_t kcap = 1;
  while (kcap < uint32_t(ix.nl)) kcap <<= 1;
  uint32_t lp2 = 1;
  while (lp2 < uint32_t(L)) lp2 <<= 1;
  const uint32_t selcap = std::max<uint32_t>(2048u, 2 * lp2);
  const size_t lds = size_t(kcap) * 8 + size_t(selcap) * 8 + (kSelBins + 256) * 4;
  const FrontArgs none{};
  const FrontArgs& f = front ? *front : none;
  TopLTail tail{};
  static const int dbg = [] { const char* e = std::getenv("SMX_DBG_FRONT"); return e ? std::atoi(e) : 0; }();
  tail.leaf_count = (dbg & 1) ? nullptr : f.leaf_count;
  tail.leaf_pair = f.leaf_pair;
  tail.slot_stride = f.slot_stride;
  tail.lut = LutParams{queries, ix.dim, ix.codebook, ix.nb, ix.dpb, LutRows(ix.ksteps), ix.metric,
                       ix.residual, (dbg & 2) ? nullptr : f.lut, f.mult, f.inv, nullptr};
  if (f.one_to_many) {
    const size_t n = size_t(nq) * ix.nl;
    hipLaunchKernelGGL(partition_scores_a8_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, s,
                       queries, nq, ix.dim, ix.centers, ix.nl, ix.metric, scores, f.init);
  } else {
    const int qtiles = (nq + kPartTile - 1) / kPartTile, ctl = (ix.nl + kPartTile - 1) / kPartTile;
    if (ix.dim <= kPartFullDim) {
      // center tiles per block: one up to ~kPartBlocks blocks, then as many
      // as keep the grid near it (two blocks per CU at a time, ~2 rounds)
      const int per = std::max(1, (qtiles * ctl + kPartBlocks - 1) / kPartBlocks);
      const dim3 grid(qtiles, (ctl + per - 1) / per);
      hipLaunchKernelGGL(partition_scores_kernel<kPartFullDim>, grid, dim3(256), 0, s, queries, nq,
                         ix.dim, ix.centers, ix.cnorm, ix.nl, ix.metric, scores, f.init, per);
    } else {
      hipLaunchKernelGGL(partition_scores_kernel<kPartChunk>, dim3(qtiles, ctl), dim3(256), 0, s,
                         queries, nq, ix.dim, ix.centers, ix.cnorm, ix.nl, ix.metric, scores, f.init,
                         1);
    }
  }
  // static LDS of the kernel besides the dynamic key buffers: the LUT build's
  // raw table and reduction (~5 KB) and the selection's words
  constexpr size_t kStaticLds = 6 * 1024;
  static const int lut_split = [] { const char* e = std::getenv("SMX_LUT_SPLIT"); return e ? std::atoi(e) : 1; }();
  if (L <= kWaveTopL && ix.nl <= 256 * 8) {
    tail.lut_split = lut_split && tail.lut.lut ? 1 : 0;
    const dim3 grid(unsigned(nq) * (tail.lut_split ? 2u : 1u));
    if (ix.nl <= 256 * 4)
      hipLaunchKernelGGL((topl_block_kernel<4, 256>), grid, dim3(256), 0, s, scores, ix.nl, L,
                         out_leaf, out_dist, tail);
    else
      hipLaunchKernelGGL((topl_block_kernel<8, 256>), grid, dim3(256), 0, s, scores, ix.nl, L,
                         out_leaf, out_dist, tail);
  } else if (ix.nl > kSampleTopLMinLeaves && L <= 4096) {
    // many leaves (configs[3]'s 10^4, configs[4]'s 5 x 10^4): the sampled
    // threshold, exact (same box A/B at 10^4 leaves, L = 100: partition
    // stage 116 -> 106 us against topl_block_kernel<16, 1024>)
    uint32_t lcap = 1;
    while (lcap < uint32_t(std::min(L, ix.nl))) lcap <<= 1;
    // LDS keys: the compacted keys (expected 1.5 L + 16 nl / 2048, room for
    // 1.3x that) plus the appended select output (~L), a power of two from
    // 2048 up to kSampleCap; more keys take the exact fallback
    const uint64_t m = uint64_t(std::min(L, ix.nl));
    const uint64_t expect = (3ull * m) / 2 + (16ull * uint64_t(ix.nl)) / 2048;
    uint32_t cap = 2048;
    while (cap < kSampleCap && cap < (13 * expect) / 10 + m + m / 16 + 64) cap <<= 1;
    const size_t lds_s = size_t(std::max(cap, lcap)) * 8;
    hipLaunchKernelGGL(topl_sample_kernel, dim3(nq), dim3(256), lds_s, s, scores, ix.nl, L, lcap,
                       cap, out_leaf, out_dist, tail);
  } else if (L <= kWaveTopL && ix.nl <= 1024 * 16) {
    hipLaunchKernelGGL((topl_block_kernel<16, 1024>), dim3(nq), dim3(1024), 0, s, scores, ix.nl,
                       L, out_leaf, out_dist, tail);
  } else if (ix.nl <= kLdsSelectLeaves && lds + kStaticLds <= 160 * 1024) {
    hipLaunchKernelGGL(topl_select_kernel, dim3(nq), dim3(256), lds, s, scores, ix.nl, L, kcap,
                       out_leaf, out_dist, tail);
  } else {
    uint32_t lcap = 1;
    while (lcap < uint32_t(std::min(L, ix.nl))) lcap <<= 1;
    if (size_t(lcap) * 8 > 128 * 1024) return hipErrorInvalidValue;   // L > 16384
    hipLaunchKernelGGL(topl_select_global_kernel, dim3(nq), dim3(256), size_t(lcap) * 8, s, scores,
                       ix.nl, L, lcap, out_leaf, out_dist, tail);
  }
  return hipGetLastError();
}

hipError_t LaunchLutBuild(const DeviceIndex& ix, const float* queries, int nq, int8_t* lut,
                          float* mult, float* inv, uint8_t* lut_u8, hipStream_t s) {
  if (nq == 0) return hipSuccess;
  const LutParams p{queries, ix.dim, ix.codebook, ix.nb, ix.dpb, LutRows(ix.ksteps), ix.metric,
                    ix.residual, lut, mult, inv, lut_u8};
  hipLaunchKernelGGL(lut_build_kernel, dim3(nq), dim3(256), 0, s, p);
  return hipGetLastError();
}

WorklistArgs MakeWorklistArgs(const DeviceIndex& ix, const uint32_t* leaf_count, WorkItem* work,
                              uint32_t* leaf_item0, uint32_t* pos_unit0, uint32_t* gunits,
                              uint32_t slot_stride, uint4* wave_start, int grid, uint32_t* totals,
                              unsigned long long* code_bytes, uint32_t chunk_tiles,
                              uint32_t narrow, const Bounds& bd) {
  WorklistArgs w;
  w.bd = bd;
  w.cnt = leaf_count;
  w.order = ix.leaf_order;
  w.leaf_size = ix.leaf_size;
  w.tile_off = ix.tile_off;
  w.member_off = ix.member_off;
  w.nl = ix.nl;
  w.nb = ix.nb;
  w.chunk_tiles = chunk_tiles;
  w.grid = grid;
  w.narrow = narrow;
  w.leaf_item0 = leaf_item0;
  w.pos_unit0 = pos_unit0;
  w.gunits = gunits;
  w.totals = totals;
  w.code_bytes = code_bytes;
  w.work = work;
  w.slot_stride = slot_stride;
  w.wave_start = wave_start;
  return w;
}

hipError_t LaunchWorklist(const DeviceIndex& ix, const uint32_t* leaf_count, WorkItem* work,
                          uint32_t* leaf_item0, uint32_t* pos_unit0, uint32_t* gunits,
                          uint32_t slot_stride, uint4* wave_start, int grid, uint32_t* totals,
                          unsigned long long* code_bytes, uint32_t chunk_tiles, uint32_t narrow,
                          unsigned long long* part, const Bounds& bd, hipStream_t s) {
  const int nblk = (ix.nl + 255) / 256;   // (worklist_kernel loops over any count)
  WorklistPart* wp = reinterpret_cast<WorklistPart*>(part);
  hipLaunchKernelGGL(worklist_part_kernel, dim3(nblk), dim3(256), 0, s, leaf_count, ix.leaf_order,
                     ix.leaf_size, ix.nl, ix.nb, chunk_tiles, narrow, wp);
  hipLaunchKernelGGL(worklist_kernel, dim3(nblk), dim3(256), 0, s, leaf_count, ix.leaf_order,
                     ix.leaf_size, ix.nl, ix.nb, chunk_tiles, narrow, wp, leaf_item0, pos_unit0,
                     gunits, totals, code_bytes);
  const WorklistArgs w = MakeWorklistArgs(ix, leaf_count, work, leaf_item0, pos_unit0, gunits,
                                          slot_stride, wave_start, grid, totals, code_bytes,
                                          chunk_tiles, narrow, bd);
  hipLaunchKernelGGL(items_kernel, dim3(ix.nl), dim3(64), 0, s, w);
  return hipGetLastError();
}

// The product library compiles the scan only; the timing ablations (2, 4,
// 16: results invalid) and the per-segment stamps (8) exist in the
// diagnostic build (-DSMX_SCAN_DIAGNOSTICS, tools/tune.py / scan_stamps.py).
// The 32-slot scan of K = KV: the dense-first tile where the blocks fit it
// (KV % 4 == 2, nb <= 2 KV - 2: glove's 50 blocks at KV = 26; SMX_DENSE_FIRST=0
// for the all-sparse tile).
// A scan launch, timed by the dispatch itself when events are given
// (hipExtLaunchKernelGGL records them in the kernel's own dispatch packet:
// the kernel's execution, as rocprofv3's kernel trace measures it, without
// the command processor's time between separate event packets and the
// dispatch -- 3-5 us on the profiled stage timings of round 5).
template <class F>
void ScanDispatch(F kernel, int grid, int threads, hipStream_t s, const ScanArgs& a,
                  hipEvent_t e0, hipEvent_t e1) {
  if (e0 && e1)
    hipExtLaunchKernelGGL(kernel, dim3(grid), dim3(threads), 0, s, e0, e1, 0, a);
  else
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(threads), 0, s, a);
}

template <int KV>
void LaunchWide(const DeviceIndex& ix, const ScanArgs& a, int grid, hipStream_t s, hipEvent_t e0,
                hipEvent_t e1) {
  if constexpr (KV % 4 == 2) {
    if (ix.dense_first && ix.nb <= 2 * KV - 2) {
      ScanDispatch(lut16_scan_kernel<KV, 0, 0, true>, grid, 64 * ScanWaves<KV>(), s, a, e0, e1);
      return;
    }
  }
  ScanDispatch(lut16_scan_kernel<KV, 0>, grid, 64 * ScanWaves<KV>(), s, a, e0, e1);
}

#ifdef SMX_SCAN_DIAGNOSTICS
#define SMX_SCAN_VARIANT(KV, V)                                                            \
  if (narrow == kNarrowOnly)                                                               \
    ScanDispatch(lut16_scan_kernel<KV, V, int(kNarrowOnly)>, grid, 64 * ScanWaves<KV>(), s, \
                 a, e0, e1);                                                               \
  else                                                                                     \
    ScanDispatch(lut16_scan_kernel<KV, V>, grid, 64 * ScanWaves<KV>(), s, a, e0, e1);
#define SMX_SCAN_CASE(KV)                                                                  \
  case KV:                                                                                 \
    if (variant == 16) {                                                                   \
      SMX_SCAN_VARIANT(KV, 16)                                                             \
    } else if (variant == 2) {                                                             \
      SMX_SCAN_VARIANT(KV, 2)                                                              \
    } else if (variant == 4) {                                                             \
      SMX_SCAN_VARIANT(KV, 4)                                                              \
    } else if (variant == 8) {                                                             \
      SMX_SCAN_VARIANT(KV, 8)                                                              \
    } else if (variant == 32) {                                                            \
      SMX_SCAN_VARIANT(KV, 32)                                                             \
    } else if (variant == 64) {                                                            \
      SMX_SCAN_VARIANT(KV, 64)                                                             \
    } else if (variant == 68) {                                                            \
      SMX_SCAN_VARIANT(KV, 68)                                                             \
    } else if (narrow == kNarrowOnly) {                                                    \
      SMX_SCAN_VARIANT(KV, 0)                                                              \
    } else {                                                                               \
      LaunchWide<KV>(ix, a, grid, s, e0, e1);                                              \
    }                                                                                      \
    break;
#else
#define SMX_SCAN_CASE(KV)                                                                  \
  case KV:                                                                                 \
    if (variant != 0) return hipErrorInvalidValue;                                         \
    if (narrow == kNarrowOnly)                                                             \
      ScanDispatch(lut16_scan_kernel<KV, 0, int(kNarrowOnly)>, grid, 64 * ScanWaves<KV>(), s, \
                   a, e0, e1);                                                             \
    else                                                                                   \
      LaunchWide<KV>(ix, a, grid, s, e0, e1);                                              \
    break;
#endif

hipError_t LaunchScan(const DeviceIndex& ix, const ScanArgs& a, int grid, int variant,
                      hipStream_t s, uint32_t narrow, hipEvent_t e0, hipEvent_t e1) {
  switch (ix.ksteps) {
    SMX_SCAN_CASE(4)
    SMX_SCAN_CASE(8)
    SMX_SCAN_CASE(12)
    SMX_SCAN_CASE(16)
    SMX_SCAN_CASE(20)
    SMX_SCAN_CASE(24)
    SMX_SCAN_CASE(26)
    SMX_SCAN_CASE(28)
    SMX_SCAN_CASE(32)
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

#define SMX_OCC_CASE(KV)                                                                 \
  case KV:                                                                               \
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(                                 \
        blocks, reinterpret_cast<const void*>(&lut16_scan_kernel<KV, 0>), 64 * ScanWaves<KV>(), 0);

hipError_t ScanBlocksPerCU(const DeviceIndex& ix, int* blocks) {
  *blocks = 0;
  switch (ix.ksteps) {
    SMX_OCC_CASE(4)
    SMX_OCC_CASE(8)
    SMX_OCC_CASE(12)
    SMX_OCC_CASE(16)
    SMX_OCC_CASE(20)
    SMX_OCC_CASE(24)
    SMX_OCC_CASE(26)
    SMX_OCC_CASE(28)
    SMX_OCC_CASE(32)
    default:
      return hipErrorInvalidValue;
  }
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
    SMX_LEAF_CASE(26)
    SMX_LEAF_CASE(28)
    SMX_LEAF_CASE(32)
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

#define SMX_SEED_CASE(KV)                                                                   \
  case KV:                                                                                  \
    if (e0 && e1)                                                                           \
      hipExtLaunchKernelGGL(seed_tau_kernel<KV>, dim3(nq + nwl), dim3(256), 0, s, e0, e1, 0, a, \
                            wl ? *wl : WorklistArgs{}, nq);                                 \
    else                                                                                    \
      hipLaunchKernelGGL(seed_tau_kernel<KV>, dim3(nq + nwl), dim3(256), 0, s, a,            \
                         wl ? *wl : WorklistArgs{}, nq);                                    \
    break;

hipError_t LaunchSeed(const DeviceIndex& ix, const SeedArgs& a, int nq, hipStream_t s,
                      const WorklistArgs* wl, hipEvent_t e0, hipEvent_t e1) {
  if (wl && wl->nl > kFusedWorklistLeaves) return hipErrorInvalidValue;
  const int nwl = wl ? (wl->nl + kWlPosPerBlock - 1) / kWlPosPerBlock : 0;
  if (nq + nwl == 0) return hipSuccess;
  switch (ix.ksteps) {
    SMX_SEED_CASE(4)
    SMX_SEED_CASE(8)
    SMX_SEED_CASE(12)
    SMX_SEED_CASE(16)
    SMX_SEED_CASE(20)
    SMX_SEED_CASE(24)
    SMX_SEED_CASE(26)
    SMX_SEED_CASE(28)
    SMX_SEED_CASE(32)
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t LaunchKthKeys(const uint32_t* vals, int sets, int kk, uint64_t* out, hipStream_t s) {
  if (sets <= 0) return hipSuccess;
  hipLaunchKernelGGL(kth_keys_kernel, dim3(sets), dim3(256), 0, s, vals, uint32_t(kk), out);
  return hipGetLastError();
}

int MergeGroupLists(int kk) { return std::max(1, kMergeWideEntries / std::max(kk, 1)); }

hipError_t LaunchMergeShards(const MergeArgs& a, hipStream_t s) {
  if (a.nq == 0) return hipSuccess;
  if (a.world < 1 || a.world > 64 || a.kk < 1 || a.kk > 2048) return hipErrorInvalidValue;
  if (a.kk <= kSelMax && a.world * a.kk <= kMergeMaxEntries) {
    hipLaunchKernelGGL(merge_shards_kernel, dim3(a.nq), dim3(256), 0, s, a);
    return hipGetLastError();
  }
  // wide lists: rounds of partial merges (groups of MergeGroupLists lists,
  // ping-ponging through a.scratch[0/1]) down to one launch's worth
  MergeArgs m = a;
  const int gl = MergeGroupLists(a.kk);
  int round = 0;
  while (m.world > gl) {
    const int groups = (m.world + gl - 1) / gl;
    MergeArgs p = m;
    p.out_entries = a.scratch[round & 1];
    if (!p.out_entries) return hipErrorInvalidValue;
    hipLaunchKernelGGL(merge_shards_wide_kernel<true>, dim3(a.nq, groups), dim3(256),
                       MergeWideLds(gl, a.kk), s, p, gl);
    m.entries = p.out_entries;
    m.world = groups;
    ++round;
  }
  hipLaunchKernelGGL(merge_shards_wide_kernel<false>, dim3(a.nq, 1), dim3(256),
                     MergeWideLds(m.world, a.kk), s, m, m.world);
  return hipGetLastError();
}

size_t MergeScratchEntries(int world, int nq, int kk) {
  if (kk <= kSelMax && world * kk <= kMergeMaxEntries) return 0;
  const int gl = MergeGroupLists(kk);
  if (world <= gl) return 0;
  const int groups = (world + gl - 1) / gl;   // the first round's output is the largest
  return size_t(groups) * size_t(nq) * size_t(kk);
}

bool FinalSelectFits(const SelectArgs& a) {
  if (a.kk <= kSelMax) return true;   // the rank kernel: fixed LDS
  uint32_t kkp2 = 1;
  while (kkp2 < uint32_t(a.kk)) kkp2 <<= 1;
  uint32_t kcap = 1;
  while (kcap < a.cap) kcap <<= 1;
  const uint32_t selcap = std::max<uint32_t>(2048u, 2 * kkp2);
  const size_t lds = size_t(kcap) * 8 + size_t(selcap) * 8 + size_t(kkp2) * 8 +
                     size_t(a.dim) * 4 + size_t(a.kk) * 8 + (kSelBins + 256) * 4;
  // the kernel's static LDS (the inlined overflow rescan's tables and the
  // selection words) counts against the same 160 KiB
  static const size_t static_lds = [] {
    hipFuncAttributes fa{};
    return hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&final_select_kernel)) ==
                   hipSuccess
               ? size_t(fa.sharedSizeBytes)
               : size_t(32 * 1024);
  }();
  return lds + static_lds <= 160 * 1024;
}

hipError_t LaunchFinalSelect(const SelectArgs& a, int nq, hipStream_t s, hipEvent_t e0,
                             hipEvent_t e1) {
  if (nq == 0) return hipSuccess;
  if (!FinalSelectFits(a)) return hipErrorInvalidValue;
  // the overflow flag is raised by the select kernels themselves; the
  // candidate-count statistics only for profiled calls
  if (a.stats)
    hipLaunchKernelGGL(cand_stats_kernel, dim3(1), dim3(1024), 0, s, a.cand_count, nq, a.cap,
                       a.overflow);
  uint32_t kkp2 = 1;
  while (kkp2 < uint32_t(a.kk)) kkp2 <<= 1;
  uint32_t kcap = 1;
  while (kcap < a.cap) kcap <<= 1;
  const uint32_t selcap = std::max<uint32_t>(2048u, 2 * kkp2);
  if (a.kk <= kSelMax) {   // (shard mode too; the list is read from global memory)
    if (e0 && e1)
      hipExtLaunchKernelGGL(final_select_rank_kernel, dim3(nq), dim3(256), 0, s, e0, e1, 0, a);
    else
      hipLaunchKernelGGL(final_select_rank_kernel, dim3(nq), dim3(256), 0, s, a);
    return hipGetLastError();
  }
  const size_t lds = size_t(kcap) * 8 + size_t(selcap) * 8 + size_t(kkp2) * 8 +
                     size_t(a.dim) * 4 + size_t(a.kk) * 8 + (kSelBins + 256) * 4;
  if (e0 && e1)
    hipExtLaunchKernelGGL(final_select_kernel, dim3(nq), dim3(256), lds, s, e0, e1, 0, a);
  else
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

hipError_t SetPhaseStamps(unsigned long long* p) {
#ifdef SMX_PHASE_STAMPS
  return hipMemcpyToSymbol(HIP_SYMBOL(g_phase_stamps), &p, sizeof(p));
#else
  (void)p;
  return hipSuccess;
#endif
}

hipError_t TakeCheckFailures(unsigned int* out) {
#ifdef SMX_DEBUG_CHECKS
  unsigned int zero = 0;
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_check_failures), sizeof(unsigned int));
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_check_failures), &zero, sizeof(zero));
  return e;
#else
  *out = 0;
  return hipSuccess;
#endif
}

hipError_t LaunchRowOf(const uint32_t* members, uint64_t m, uint32_t* row_of, hipStream_t s) {
  if (m == 0) return hipSuccess;
  hipLaunchKernelGGL(row_of_kernel, dim3(unsigned((m + 255) / 256)), dim3(256), 0, s, members, m,
                     row_of);
  return hipGetLastError();
}

hipError_t LaunchFill64(uint64_t* p, uint64_t v, size_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(fill64_kernel, dim3((n + 255) / 256), dim3(256), 0, s, p, v, n);
  return hipGetLastError();
}

}  // namespace smx

// lut16_avx2_port.cc — AVX2 port of the reference's batched tree-AH query
// path, used ONLY as bench.py's cpu_baseline ("kind": "port").
//
// TEST INFRASTRUCTURE (see scann_oracle.h).  Semantics equal
// orc_search(..., ORC_MODE_EMULATE, ...) exactly; the difference is the
// execution strategy, which mirrors the reference:
//   * SearchBatchedParallel chunking over a thread pool (scann.cc:478-501);
//   * per chunk: partition top-L, per-query LUTs, queries inverted by leaf,
//     leaves visited in leaf_tokens_by_norm_ order, batches of <=3 queries
//     per LUT16 call (tree_ah_hybrid_residual.cc:631-786);
//   * the LUT16 inner loop as pshufb lookups over the reference packed layout
//     with 16-bit accumulation (lut16_avx2.inc:55-124, 403-526).
// Partition scoring and LUT construction reuse the scalar restatement's
// numerics (same translation unit family, compiled -ffp-contract=off).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <numeric>
#include <thread>
#include <unordered_map>
#include <vector>

#include "scann_oracle.h"

#if defined(__AVX2__)
#include <immintrin.h>

namespace {

// 32 exact int16 accumulators for one 32-datapoint group of the reference
// packed layout (16*nb bytes) and one LUT (u8 [nb][16]).
inline void Lut16Group(const uint8_t* group, int nb, const uint8_t* lut,
                       int16_t out[32]) {
  const __m256i low4 = _mm256_set1_epi8(0x0F);
  const __m256i lowbyte = _mm256_set1_epi16(0x00FF);
  __m256i e0 = _mm256_setzero_si256(), o0 = e0, e1 = e0, o1 = e0;
  int b = 0;
  for (; b + 2 <= nb; b += 2) {
    const __m256i codes = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(group + b * 16));
    const __m256i lo = _mm256_and_si256(codes, low4);
    const __m256i hi = _mm256_and_si256(_mm256_srli_epi16(codes, 4), low4);
    const __m256i tbl = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(lut + b * 16));
    const __m256i r0 = _mm256_shuffle_epi8(tbl, lo);
    const __m256i r1 = _mm256_shuffle_epi8(tbl, hi);
    e0 = _mm256_add_epi16(e0, _mm256_and_si256(r0, lowbyte));
    o0 = _mm256_add_epi16(o0, _mm256_srli_epi16(r0, 8));
    e1 = _mm256_add_epi16(e1, _mm256_and_si256(r1, lowbyte));
    o1 = _mm256_add_epi16(o1, _mm256_srli_epi16(r1, 8));
  }
  // Fold the two 128-bit lanes (blocks b and b+1 of each pair).
  __m128i E0 = _mm_add_epi16(_mm256_castsi256_si128(e0), _mm256_extracti128_si256(e0, 1));
  __m128i O0 = _mm_add_epi16(_mm256_castsi256_si128(o0), _mm256_extracti128_si256(o0, 1));
  __m128i E1 = _mm_add_epi16(_mm256_castsi256_si128(e1), _mm256_extracti128_si256(e1, 1));
  __m128i O1 = _mm_add_epi16(_mm256_castsi256_si128(o1), _mm256_extracti128_si256(o1, 1));
  __m128i d0 = _mm_unpacklo_epi16(E0, O0);  // dps 0..7
  __m128i d1 = _mm_unpackhi_epi16(E0, O0);  // dps 8..15
  __m128i d2 = _mm_unpacklo_epi16(E1, O1);  // dps 16..23
  __m128i d3 = _mm_unpackhi_epi16(E1, O1);  // dps 24..31
  if (b < nb) {  // odd trailing block (lut16_avx2.inc:102-116)
    const __m128i codes = _mm_loadu_si128(reinterpret_cast<const __m128i*>(group + b * 16));
    const __m128i l4 = _mm_set1_epi8(0x0F);
    const __m128i lo = _mm_and_si128(codes, l4);
    const __m128i hi = _mm_and_si128(_mm_srli_epi16(codes, 4), l4);
    const __m128i tbl = _mm_loadu_si128(reinterpret_cast<const __m128i*>(lut + b * 16));
    const __m128i v0 = _mm_shuffle_epi8(tbl, lo);
    const __m128i v1 = _mm_shuffle_epi8(tbl, hi);
    const __m128i z = _mm_setzero_si128();
    d0 = _mm_add_epi16(d0, _mm_unpacklo_epi8(v0, z));
    d1 = _mm_add_epi16(d1, _mm_unpackhi_epi8(v0, z));
    d2 = _mm_add_epi16(d2, _mm_unpacklo_epi8(v1, z));
    d3 = _mm_add_epi16(d3, _mm_unpackhi_epi8(v1, z));
  }
  const __m128i bias = _mm_set1_epi16(int16_t(nb * 128));
  _mm_storeu_si128(reinterpret_cast<__m128i*>(out + 0), _mm_sub_epi16(d0, bias));
  _mm_storeu_si128(reinterpret_cast<__m128i*>(out + 8), _mm_sub_epi16(d1, bias));
  _mm_storeu_si128(reinterpret_cast<__m128i*>(out + 16), _mm_sub_epi16(d2, bias));
  _mm_storeu_si128(reinterpret_cast<__m128i*>(out + 24), _mm_sub_epi16(d3, bias));
}

// The reference's bottom loop for <= 3 queries sharing one 32-datapoint
// group (Avx2LUT16BottomLoop + PostprocessAccumulatorPair / CombineAvxLanes,
// lut16_avx2.inc:17-124): the group's code nibbles are extracted once per
// block pair and looked up in every query's LUT; each pshufb result is
// accumulated as u16 with its odd byte tagging along (the even sums are
// recovered as acc - (odd << 8)), so a block pair costs one load, two
// shuffles, two shifts and four adds per query.  Prefetch as the reference's
// kSmart strategy (PrefetchDispatcher, :177-198): `pf` (the next partition's
// bytes, NTA) when the driver passes one, else the current stream 768 bytes
// ahead (kPrefetchBytesAhead, lut16_args.h:28).
inline __m256i CombineLanes(__m256i a, __m256i b) {
  return _mm256_add_epi16(_mm256_permute2x128_si256(a, b, 0x30),
                          _mm256_permute2x128_si256(a, b, 0x21));
}

inline __m256i PostprocessPair(__m256i even_tag, __m256i odd) {
  const __m256i even = _mm256_sub_epi16(even_tag, _mm256_slli_epi16(odd, 8));
  return CombineLanes(_mm256_unpacklo_epi16(even, odd), _mm256_unpackhi_epi16(even, odd));
}

template <int NQ>
inline void Lut16GroupN(const uint8_t* group, int nb, const uint8_t* const* luts,
                        int16_t (*out)[32], const uint8_t* pf) {
  const __m256i low4 = _mm256_set1_epi8(0x0F);
  __m256i acc[NQ][4];
  const uint8_t* lp[NQ];
#pragma GCC unroll 3
  for (int j = 0; j < NQ; ++j) {
#pragma GCC unroll 4
    for (int a = 0; a < 4; ++a) acc[j][a] = _mm256_setzero_si256();
    lp[j] = luts[j];
  }
  const uint8_t* data = group;
  for (int it = nb / 2; it != 0; --it) {
    if (pf) {
      _mm_prefetch(reinterpret_cast<const char*>(pf), _MM_HINT_NTA);
      pf += 32;
    } else {
      _mm_prefetch(reinterpret_cast<const char*>(data + 768), _MM_HINT_T0);
    }
    const __m256i codes = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(data));
    data += 32;
    const __m256i m0 = _mm256_and_si256(codes, low4);
    const __m256i m1 = _mm256_and_si256(_mm256_srli_epi16(codes, 4), low4);
#pragma GCC unroll 3
    for (int j = 0; j < NQ; ++j) {
      const __m256i dict = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(lp[j]));
      lp[j] += 32;
      const __m256i r0 = _mm256_shuffle_epi8(dict, m0);
      const __m256i r1 = _mm256_shuffle_epi8(dict, m1);
      acc[j][0] = _mm256_add_epi16(acc[j][0], r0);
      acc[j][1] = _mm256_add_epi16(acc[j][1], _mm256_srli_epi16(r0, 8));
      acc[j][2] = _mm256_add_epi16(acc[j][2], r1);
      acc[j][3] = _mm256_add_epi16(acc[j][3], _mm256_srli_epi16(r1, 8));
    }
  }
  __m256i res[NQ][2];
#pragma GCC unroll 3
  for (int j = 0; j < NQ; ++j) {
    res[j][0] = PostprocessPair(acc[j][0], acc[j][1]);   // datapoints 0..15
    res[j][1] = PostprocessPair(acc[j][2], acc[j][3]);   // datapoints 16..31
  }
  if (nb & 1) {   // the odd trailing block (SSE, :102-116)
    const __m128i l4 = _mm_set1_epi8(0x0F);
    const __m128i codes = _mm_loadu_si128(reinterpret_cast<const __m128i*>(data));
    const __m128i m0 = _mm_and_si128(codes, l4);
    const __m128i m1 = _mm_and_si128(_mm_srli_epi16(codes, 4), l4);
#pragma GCC unroll 3
    for (int j = 0; j < NQ; ++j) {
      const __m128i dict = _mm_loadu_si128(reinterpret_cast<const __m128i*>(lp[j]));
      res[j][0] = _mm256_add_epi16(res[j][0], _mm256_cvtepu8_epi16(_mm_shuffle_epi8(dict, m0)));
      res[j][1] = _mm256_add_epi16(res[j][1], _mm256_cvtepu8_epi16(_mm_shuffle_epi8(dict, m1)));
    }
  }
  const __m256i bias = _mm256_set1_epi16(int16_t(nb * 128));
#pragma GCC unroll 3
  for (int j = 0; j < NQ; ++j) {
    _mm256_storeu_si256(reinterpret_cast<__m256i*>(out[j]), _mm256_sub_epi16(res[j][0], bias));
    _mm256_storeu_si256(reinterpret_cast<__m256i*>(out[j] + 16), _mm256_sub_epi16(res[j][1], bias));
  }
}

void Lut16Batch(const uint8_t* group, int nb, const uint8_t* const* luts, int nq,
                int16_t (*out)[32], const uint8_t* pf) {
  switch (nq) {
    case 1: Lut16GroupN<1>(group, nb, luts, out, pf); break;
    case 2: Lut16GroupN<2>(group, nb, luts, out, pf); break;
    default: Lut16GroupN<3>(group, nb, luts, out, pf); break;
  }
}

inline uint32_t PushMask(const int16_t acc[32], int16_t thr) {
  const __m256i t = _mm256_set1_epi16(thr);
  const __m256i a0 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(acc));
  const __m256i a1 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(acc + 16));
  const __m256i c0 = _mm256_cmpgt_epi16(t, a0);
  const __m256i c1 = _mm256_cmpgt_epi16(t, a1);
  const __m256i packed = _mm256_permute4x64_epi64(_mm256_packs_epi16(c0, c1), 0xD8);
  return uint32_t(_mm256_movemask_epi8(packed));
}

// Partition scores with the centers transposed, eight per vector: per
// center the chain acc <- fma(-q_d, c_d, acc) over d ascending (dot) or from
// ||c||^2 + ||q||^2 with 2 c_d (squared L2) -- fnmadd is that single-rounding
// fma, so every score equals PartitionScoresOne's bit for bit.
void PartitionScoresT(const float* q, int dim, const float* ct, int nlp, int nl, int metric,
                      const float* cnorms, float qnorm, float* out) {
  for (int c = 0; c < nlp; c += 8) {
    __m256 acc;
    if (metric == ORC_METRIC_DOT) {
      acc = _mm256_setzero_ps();
    } else {
      alignas(32) float init[8];
      for (int i = 0; i < 8; ++i) init[i] = c + i < nl ? cnorms[c + i] + qnorm : 0.0f;
      acc = _mm256_load_ps(init);
    }
    for (int d = 0; d < dim; ++d) {
      const __m256 qd = _mm256_set1_ps(q[d]);
      __m256 cd = _mm256_loadu_ps(ct + size_t(d) * nlp + c);
      if (metric != ORC_METRIC_DOT) cd = _mm256_mul_ps(cd, _mm256_set1_ps(2.0f));
      acc = _mm256_fnmadd_ps(qd, cd, acc);
    }
    alignas(32) float r[8];
    _mm256_store_ps(r, acc);
    for (int i = 0; i < 8 && c + i < nl; ++i) out[c + i] = r[i];
  }
}

}  // namespace
#endif  // __AVX2__

// Driver shared with the scalar restatement (defined in scann_oracle.cc so it
// reuses the same partition / LUT / FastTopNeighbors code).
namespace orc_port {
using GroupFn = void (*)(const uint8_t*, int, const uint8_t*, int16_t*);
using MaskFn = uint32_t (*)(const int16_t*, int16_t);
using PartFn = void (*)(const float*, int, const float*, int, int, int, const float*, float,
                        float*);
using BatchFn = void (*)(const uint8_t*, int, const uint8_t* const*, int, int16_t (*)[32],
                         const uint8_t*);
void* Prepare(const orc_index* ix);
void Release(void* p);
int Run(void* prepared, const float* queries, int nq, int leaves, int pre_nn,
        int final_nn, int do_reorder, int nthreads, uint32_t* out_idx,
        float* out_dist, int32_t* out_count, GroupFn group_fn, MaskFn mask_fn,
        PartFn part_fn, double* phase_s, BatchFn batch_fn);
}  // namespace orc_port

extern "C" {
void* orc_avx2_prepare(const orc_index* idx) { return orc_port::Prepare(idx); }
void orc_avx2_release(void* p) { orc_port::Release(p); }
// batch_shared: 1 = the reference's bottom loop (codes shared by the <= 3
// queries of a batch, tag-along accumulation, kSmart prefetch); 0 = one
// group pass per query (the round-2 port, kept for comparison).
int orc_search_avx2(void* prepared, const float* queries, int32_t nq,
                    int32_t leaves, int32_t pre_nn, int32_t final_nn,
                    int32_t do_reorder, int32_t nthreads, uint32_t* out_idx,
                    float* out_dist, int32_t* out_count, double* phase_s,
                    int32_t batch_shared) {
#if defined(__AVX2__)
  return orc_port::Run(prepared, queries, nq, leaves, pre_nn, final_nn,
                       do_reorder, nthreads, out_idx, out_dist, out_count,
                       &Lut16Group, &PushMask, &PartitionScoresT, phase_s,
                       batch_shared ? &Lut16Batch : nullptr);
#else
  (void)prepared; (void)queries; (void)nq; (void)leaves; (void)pre_nn;
  (void)final_nn; (void)do_reorder; (void)nthreads; (void)out_idx;
  (void)out_dist; (void)out_count; (void)phase_s; (void)batch_shared;
  return -2;
#endif
}
}  // extern "C"

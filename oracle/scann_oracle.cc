// scann_oracle.cc — CPU restatement of ScaNN's LUT16 / tree-AH query path.
//
// TEST INFRASTRUCTURE ONLY (see scann_oracle.h).  Compiled with
// -ffp-contract=off so that every float operation written below rounds
// exactly once, in the order written; fused multiply-adds are spelled
// std::fma where the reference fuses them.
//
// Reference anchors (relative to the reference root):
//   partition numerics     many_to_many_impl.inc:236-257, 522-560
//   top-L selection        kmeans_tree_partitioner.cc:703-728
//   raw LUT                asymmetric_hashing_impl.cc:505-569,
//                          one_to_many_symmetric.h:691-799, 983-1025
//   fixed point            asymmetric_hashing_impl.cc:571-645
//   packed layout          asymmetric_hashing_impl.cc:690-737
//   LUT16 scan + top-N     lut16_avx2.inc:403-526
//   FastTopNeighbors       fast_top_neighbors.h:90-355,
//                          fast_top_neighbors_impl.inc:1-391,
//                          fast_top_neighbors.cc:96-150, hwy-compact.cc:41-66
//   driver                 tree_ah_hybrid_residual.cc:631-786
//   SOAR dedupe            tree_x_hybrid/internal/utils.cc:135-162
//   reorder                one_to_many_symmetric.h:373-503, reordering_helper.cc:257-283
//   sort & drop            single_machine_base.cc:570-587, 872-901,
//                          util_functions.cc:69-81, util_functions.h:109-126
#include "scann_oracle.h"

#include <algorithm>
#include <ctime>
#include <mutex>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <numeric>
#include <thread>
#include <unordered_map>
#include <utility>
#include <vector>

namespace orc {

constexpr float kInf = std::numeric_limits<float>::infinity();

// ---------------------------------------------------------------------------
// Partition scoring (A.10).  Dot: acc <- fma(-q_d, c_d, acc) from 0 in dim
// order (many_to_many_impl.inc:544-556 with FusedMultiplySubtract).
// Squared L2: the database side keeps 2*c_d and ||c||^2 computed as
// -(chain acc <- fma(-c_d, c_d, acc)) (:236-257); the query norm is
// SquaredL2Norm(q) accumulated in double then stored as float (:422-426);
// the accumulator starts at ||c||^2 + ||q||^2 (:531-538).
// ---------------------------------------------------------------------------
static float DotChain(const float* q, const float* c, int dim) {
  float acc = 0.0f;
  for (int d = 0; d < dim; ++d) acc = std::fma(-q[d], c[d], acc);
  return acc;
}

static float CenterSqNorm(const float* c, int dim) {
  float acc = 0.0f;
  for (int d = 0; d < dim; ++d) acc = std::fma(-c[d], c[d], acc);
  return acc * -1.0f;
}

static float QuerySqNorm(const float* q, int dim) {
  double acc = 0.0;
  for (int d = 0; d < dim; ++d) {
    const double x = q[d];
    acc += x * x;
  }
  return static_cast<float>(acc);
}

static float SqL2Chain(const float* q, float qnorm, const float* c,
                       float cnorm, int dim) {
  float acc = cnorm + qnorm;
  for (int d = 0; d < dim; ++d) acc = std::fma(-q[d], c[d] * 2.0f, acc);
  return acc;
}

static void PartitionScoresOne(const float* q, int dim, const float* centers,
                               int nl, int metric,
                               const std::vector<float>& cnorms, float* out) {
  if (metric == ORC_METRIC_DOT) {
    for (int c = 0; c < nl; ++c) out[c] = DotChain(q, centers + size_t(c) * dim, dim);
  } else {
    const float qn = QuerySqNorm(q, dim);
    for (int c = 0; c < nl; ++c)
      out[c] = SqL2Chain(q, qn, centers + size_t(c) * dim, cnorms[c], dim);
  }
}

static std::vector<float> CenterNorms(const float* centers, int nl, int dim) {
  std::vector<float> n(nl);
  for (int c = 0; c < nl; ++c) n[c] = CenterSqNorm(centers + size_t(c) * dim, dim);
  return n;
}

// Exact top-L by (score, center index): FastTopNeighbors' final GC keeps an
// exact prefix of that order (fast_top_neighbors.cc:96-105 CompIV).
static void TopL(const float* scores, int nl, int L, std::vector<int>* leaf,
                 std::vector<float>* score) {
  L = std::min(L, nl);
  std::vector<int> ord(nl);
  std::iota(ord.begin(), ord.end(), 0);
  auto less = [&](int a, int b) {
    if (scores[a] != scores[b]) return scores[a] < scores[b];
    return a < b;
  };
  std::partial_sort(ord.begin(), ord.begin() + L, ord.end(), less);
  leaf->assign(ord.begin(), ord.begin() + L);
  score->resize(L);
  for (int i = 0; i < L; ++i) (*score)[i] = scores[(*leaf)[i]];
}

// ---------------------------------------------------------------------------
// LUT creation (A.2, A.3).
// Raw entry for dot with a 2-dim block: -fl(fl(q0*c0) + fl(q1*c1)); 1-dim:
// -fl(q0*c0).  Both the 4-lane Highway path (NegMulAdd from zero, ReduceSum;
// one_to_many_symmetric.h:741-776) used for centers 0..14 and the SSE4
// VectorVector path (dot_product_sse4.cc:278-295) used for center 15 yield
// this value.  Squared L2: fl(fl(t0*t0) + fl(t1*t1)), t_i = fl(q_i - c_i).
// Blocks wider than 2 dims: products summed left to right (parity unpinned;
// no configuration of BASELINE.json uses them).
// ---------------------------------------------------------------------------
static inline int BlockDims(int b, int nb, int dpb, int dim) {
  return (b == nb - 1) ? dim - dpb * (nb - 1) : dpb;
}

static float RawEntry(const float* q, const float* c, int nd, int metric) {
  if (metric == ORC_METRIC_DOT) {
    float s = q[0] * c[0];
    for (int i = 1; i < nd; ++i) {
      const float p = q[i] * c[i];
      s = s + p;
    }
    return -s;
  }
  float t = q[0] - c[0];
  float s = t * t;
  for (int i = 1; i < nd; ++i) {
    const float u = q[i] - c[i];
    const float p = u * u;
    s = s + p;
  }
  return s;
}

struct Lut {
  std::vector<uint8_t> u8;  // [B][16]
  float mult = 0.0f;
};

static int CreateLut(const float* q, int dim, const float* codebook, int nb,
                     int dpb, int metric, float* raw_out, Lut* lut) {
  if (dpb <= 0 || nb <= 0) return -1;
  if (dim - dpb * (nb - 1) <= 0 || dim - dpb * (nb - 1) > dpb) return -1;
  std::vector<float> raw(size_t(nb) * 16);
  for (int b = 0; b < nb; ++b) {
    const int nd = BlockDims(b, nb, dpb, dim);
    const float* qb = q + size_t(b) * dpb;
    for (int c = 0; c < 16; ++c) {
      const float* cb = codebook + (size_t(b) * 16 + c) * dpb;
      raw[size_t(b) * 16 + c] = RawEntry(qb, cb, nd, metric);
    }
  }
  // ComputeMultiplierByQuantile with quantile 1 (hash.proto:87 default):
  // 127 / max(sqrt(FLT_EPSILON), max|LUT|), float division.
  float max_abs = 0.0f;
  for (float v : raw) max_abs = std::max(max_abs, std::fabs(v));
  const float floor_v = std::sqrt(std::numeric_limits<float>::epsilon());
  const float m = 127.0f / std::max(floor_v, max_abs);
  lut->mult = m;
  lut->u8.resize(raw.size());
  for (size_t i = 0; i < raw.size(); ++i) {
    const float scaled = raw[i] * m;
    const float r = std::round(scaled) + 128.0f;  // ROUND (scann_builder.py:312-314)
    lut->u8[i] = static_cast<uint8_t>(r);
  }
  if (raw_out) std::copy(raw.begin(), raw.end(), raw_out);
  return 0;
}

// Exact integer accumulation Sum_b (u8[b][code] - 128).  The reference does
// this modulo 2^16 with lane tricks (lut16_avx2.inc:30-38, 64-123); the
// value is exact for num_blocks <= 256 (CanUseInt16Accumulator, :663-668).
static inline int32_t Accumulate(const uint8_t* codes, int nb,
                                 const uint8_t* lut) {
  int32_t acc = 0;
  for (int b = 0; b < nb; ++b) acc += int32_t(lut[b * 16 + codes[b]]) - 128;
  return acc;
}

// ---------------------------------------------------------------------------
// FastTopNeighbors<DistT, uint32_t> replay (A.6) for DistT = float (the
// global top-N of both pipelines) and int16_t (pipeline B's per-leaf top-N,
// querying.h:403-462).  Storage mirrors the reference's sizes so that reads
// of stale slots beyond sz (UseMasksToFindNewMedian) see the same kind of
// data; initial contents are zero here (uninitialised in the reference:
// unpinnable).
// ---------------------------------------------------------------------------
static inline uint32_t FinalMask32(size_t n) {
  const size_t r = n % 32;
  return r ? (1u << r) - 1 : 0xFFFFFFFFu;
}
static inline int Ctz(uint32_t x) { return __builtin_ctz(x); }
static inline int Popc(uint32_t x) { return __builtin_popcount(x); }

// MaxOrInfinity / DecrementThreshold (fast_top_neighbors_impl.inc:243-251).
template <typename V> struct DistTraits;
template <> struct DistTraits<float> {
  static float Max() { return kInf; }
  static float Decrement(float t) { return std::nextafter(t, -kInf); }
};
template <> struct DistTraits<int16_t> {
  static int16_t Max() { return std::numeric_limits<int16_t>::max(); }
  static int16_t Decrement(int16_t t) { return static_cast<int16_t>(t - 1); }
};

template <typename V>
static inline bool CompIV(uint32_t ia, uint32_t ib, V va, V vb) {
  if (va == vb || va != va || vb != vb) return ia < ib;  // equal or unordered
  return va < vb;
}
template <typename V>
static inline void ZipSwap(size_t a, size_t b, uint32_t* ind, V* val) {
  std::swap(ind[a], ind[b]);
  std::swap(val[a], val[b]);
}
template <typename V>
static inline V Median3(V v0, V v1, V v2) {
  const V big = std::max(v0, v1);
  const V sml = std::min(v0, v1);
  return std::max(sml, std::min(big, v2));
}

// CalculateSwapMasks (fast_top_neighbors_impl.inc:1-24).
template <typename V>
static size_t SwapMasks(bool eq, const V* val, uint32_t* masks, size_t nm,
                        uint32_t final_mask, V thr) {
  size_t kept = 0;
  for (size_t j = 0; j < nm; ++j) {
    uint32_t m = 0;
    for (int l = 0; l < 32; ++l) {
      const V v = val[32 * j + l];
      const bool bit = eq ? (v == thr) : (v < thr);
      m |= uint32_t(bit) << l;
    }
    kept += Popc(m);
    masks[j] = m;
  }
  uint32_t& last = masks[nm - 1];
  kept -= Popc(last);
  last &= final_mask;
  kept += Popc(last);
  return kept;
}

// UseMasksToPartition (:44-93).
template <typename V>
static size_t PartitionByMasks(uint32_t* ind, V* val, const uint32_t* masks,
                               size_t nm) {
  size_t i1 = 0, i2 = nm - 1;
  uint32_t m1 = ~masks[i1];
  uint32_t m2 = masks[i2];
  if (nm > 1) {
    for (;;) {
      while (m1 && m2) {
        const int o1 = Ctz(m1), o2 = Ctz(m2);
        m1 &= m1 - 1;
        m2 &= m2 - 1;
        ZipSwap(i1 * 32 + o1, i2 * 32 + o2, ind, val);
      }
      if (!m1) {
        ++i1;
        if (i1 == i2) break;
        m1 = ~masks[i1];
      }
      if (!m2) {
        --i2;
        if (i1 == i2) {
          m2 = ~m1;
          break;
        }
        m2 = masks[i2];
      }
    }
  }
  size_t w = i2 * 32;
  while (m2) {
    const int o = Ctz(m2);
    m2 &= m2 - 1;
    ZipSwap(w++, i2 * 32 + o, ind, val);
  }
  return w;
}

// UseMasksToCompact for <uint32_t, float> on AVX2 = HwyCompact
// (hwy-compact.cc:41-66): for every 8-lane slice, Compress (selected lanes
// first, then the unselected ones in order: CompressIsPartition for 32-bit
// lanes) stored unaligned at the write cursor.  Order preserving for the
// kept elements.
static size_t CompactByMasks(uint32_t* ind, float* val, uint32_t* masks,
                             size_t nm) {
  size_t w = 0;
  for (size_t j = 0; j < nm; ++j) {
    for (int i = 0; i < 32; i += 8) {
      const size_t r = j * 32 + i;
      const uint32_t bits = (masks[j] >> i) & 0xFFu;
      uint32_t ti[8];
      float tv[8];
      int n = 0;
      for (int l = 0; l < 8; ++l)
        if (bits >> l & 1) { ti[n] = ind[r + l]; tv[n] = val[r + l]; ++n; }
      const int nsel = n;
      for (int l = 0; l < 8; ++l)
        if (!(bits >> l & 1)) { ti[n] = ind[r + l]; tv[n] = val[r + l]; ++n; }
      for (int l = 0; l < 8; ++l) { ind[w + l] = ti[l]; val[w + l] = tv[l]; }
      w += nsel;
    }
  }
  return w;
}

// UseMasksToCompact for every other type (fast_top_neighbors_impl.inc:
// 189-202): UseMaskToCompact for one mask (:96-108), otherwise
// UseMasksToCompactDoublePorted (:110-187) -- the first two 32-lane chunks
// are copied behind the last one, then chunks 2, 3, ... are drained two
// streams at a time (one element of the later chunk, then one of the
// earlier), which does NOT preserve the kept elements' order.
template <typename V>
static size_t CompactByMasks(uint32_t* ind, V* val, uint32_t* masks, size_t nm) {
  size_t w = 0;
  if (nm == 1) {
    uint32_t m = masks[0];
    while (m) {
      const int o = Ctz(m);
      m &= m - 1;
      ind[w] = ind[o];
      val[w] = val[o];
      ++w;
    }
    return w;
  }
  std::copy(val, val + 64, val + nm * 32);
  std::copy(ind, ind + 64, ind + nm * 32);
  masks[nm] = masks[0];
  masks[nm + 1] = masks[1];
  const size_t end = nm + 2;
  uint32_t m1 = masks[2], m2 = masks[3];
  size_t b1 = 2 * 32, b2 = 3 * 32, mp = 3;
  for (;;) {
    if (!m1 || !m2) {
      bool cooldown = false;
      do {
        if (!m1) {
          m1 = m2;
          b1 = b2;
        }
        if (++mp >= end) {
          cooldown = true;
          break;
        }
        m2 = masks[mp];
        b2 += 32;
      } while (!m1 || !m2);
      if (cooldown) break;
    }
    const int o2 = Ctz(m2), o1 = Ctz(m1);
    ind[w] = ind[b2 + o2];
    val[w] = val[b2 + o2];
    ++w;
    ind[w] = ind[b1 + o1];
    val[w] = val[b1 + o1];
    ++w;
    m2 &= m2 - 1;
    m1 &= m1 - 1;
  }
  while (m1) {
    const int o1 = Ctz(m1);
    m1 &= m1 - 1;
    ind[w] = ind[b1 + o1];
    val[w] = val[b1 + o1];
    ++w;
  }
  return w;
}

static size_t SelectByMasks(uint32_t* to, const uint32_t* from,
                            const uint32_t* masks, size_t nm) {
  size_t w = 0;
  for (size_t j = 0; j < nm; ++j) {
    uint32_t m = masks[j];
    while (m) {
      const int o = Ctz(m);
      m &= m - 1;
      to[w++] = from[32 * j + o];
    }
  }
  return w;
}

template <typename V>
static V NewMedian(const V* val, const uint32_t* lt, const uint32_t* eq,
                   size_t nm) {
  size_t n = 0;
  V v[3] = {0, 0, 0};
  for (size_t j = 0; j < nm; ++j) {
    uint32_t m = ~(lt[j] + eq[j]);
    while (m) {
      const int o = Ctz(m);
      m &= m - 1;
      v[n++] = val[j * 32 + o];
      if (n == 3) return Median3(v[0], v[1], v[2]);
    }
  }
  return v[0];
}

// ApproxNthElementImpl (fast_top_neighbors_impl.inc:253-391).
template <typename V>
static size_t ApproxNth(size_t keep_min, size_t keep_max, size_t sz,
                        uint32_t* ind, V* val, uint32_t* masks) {
  V thr = 0;
  size_t already = 0;
  bool skip = false;
  for (;;) {
    if (!skip) {
      if (sz <= 3) {
        // SelectionSort (fast_top_neighbors.cc:122-141)
        auto cos = [&](size_t a, size_t b) {
          if (!CompIV(ind[a], ind[b], val[a], val[b])) ZipSwap(a, b, ind, val);
        };
        if (sz == 3) { cos(0, 1); cos(1, 2); }
        if (sz >= 2) cos(0, 1);
        val[keep_min] = val[keep_min - 1];
        ind[keep_min] = ind[keep_min - 1];
        return already + keep_min;
      }
      thr = Median3(val[0], val[sz / 2], val[sz - 1]);
    }
    skip = false;
    const uint32_t fm = FinalMask32(sz);
    const size_t nm = (sz + 31) / 32;
    size_t n_kept = SwapMasks(false, val, masks, nm, fm, thr);
    const bool need_eq = n_kept < keep_min;
    uint32_t* scratch = ind + 32 * nm + 64;
    if (need_eq) {
      const size_t n_needed = keep_min - n_kept;
      uint32_t* eqm = masks + nm;
      const size_t n_found = SwapMasks(true, val, eqm, nm, fm, thr);
      if (n_found < n_needed) {
        if (n_kept < sz * 3 / 4) {
          thr = NewMedian(val, masks, eqm, nm);
          skip = true;
        } else {
          PartitionByMasks(ind, val, masks, nm);
          already += n_kept;
          keep_min -= n_kept;
          keep_max -= n_kept;
          sz -= n_kept;
          ind += n_kept;
          val += n_kept;
        }
        continue;
      }
      const size_t ns = SelectByMasks(scratch, ind, eqm, nm);
      if (n_found > n_needed) {
        std::nth_element(scratch, scratch + n_needed - 1, scratch + ns);
        std::sort(scratch, scratch + n_needed);
      }
    }
    sz = CompactByMasks(ind, val, masks, nm);
    if (n_kept > keep_max) continue;
    uint32_t tiebreak = std::numeric_limits<uint32_t>::max();
    if (need_eq) {
      const size_t n_needed = keep_min - n_kept;
      std::copy(scratch, scratch + n_needed, ind + n_kept);
      std::fill(val + n_kept, val + n_kept + n_needed, thr);
      n_kept = keep_min;
      tiebreak = scratch[n_needed - 1];
    } else {
      thr = DistTraits<V>::Decrement(thr);
    }
    val[n_kept] = thr;
    ind[n_kept] = tiebreak;
    return already + n_kept;
  }
}

template <typename V>
class FastTopNT {
 public:
  // Init (fast_top_neighbors.h:90-120).  A finite epsilon limits the
  // no-realloc size to 128 results; beyond it the reference grows the
  // arrays by doubling (ReallocateForPureEnn, :505-530) without collecting,
  // so the first GC happens at the same push as with the final capacity,
  // which is allocated here at once.
  explicit FastTopNT(size_t k, V eps = DistTraits<V>::Max()) : k_(k), eps_(eps) {
    cap_ = (k == 0) ? 32 : ((2 * k + 31) / 32) * 32;
    ind_.assign(2 * cap_ + 96, 0);
    val_.assign(cap_ + 96, V(0));
    masks_.assign(2 * cap_ / 32 + 2, 0);
  }
  V epsilon() const { return eps_; }
  size_t size() const { return sz_; }
  // PushNoEpsilonCheck: returns true when the buffer is full (GC needed).
  bool Push(uint32_t i, V d) {
    ind_[sz_] = i;
    val_[sz_] = d;
    ++sz_;
    return sz_ == cap_;
  }
  void GarbageCollectApprox() {
    ++num_gc_;
    Gc(k_, (k_ + cap_) / 2 - 1);
  }
  // FinishUnsorted (fast_top_neighbors.h:176-183): GC(k, k), storage order.
  void Finish(std::vector<std::pair<uint32_t, V>>* out) {
    Gc(k_, k_);
    out->resize(sz_);
    for (size_t i = 0; i < sz_; ++i) (*out)[i] = {ind_[i], val_[i]};
  }
  int num_gc() const { return num_gc_; }

 private:
  // GarbageCollect (fast_top_neighbors.h:530-547).
  void Gc(size_t keep_min, size_t keep_max) {
    if (keep_min == 0) {
      sz_ = 0;
      return;
    }
    if (sz_ <= keep_max) return;
    sz_ = ApproxNth(keep_min, keep_max, sz_, ind_.data(), val_.data(),
                    masks_.data());
    eps_ = val_[sz_];
  }
  size_t k_, cap_, sz_ = 0;
  V eps_;
  int num_gc_ = 0;
  std::vector<uint32_t> ind_;
  std::vector<V> val_;
  std::vector<uint32_t> masks_;
};
using FastTopN = FastTopNT<float>;

// GetInt16Threshold over (epsilon - bias) * mult (lut16_avx2.inc:397-401,
// 432-438, 515-519): float min against 32767 then C++ truncation.  Values
// below -32768 are UB in the reference and clamp here.
static inline int32_t Int16Threshold(float eps, float bias, float mult) {
  const float t = (eps - bias) * mult;
  const float c = std::min(t, 32767.0f);
  if (!(c > -32768.0f)) return -32768;
  return static_cast<int16_t>(c);
}

// ---------------------------------------------------------------------------
// Exact reorder distance (A.8): the AVX2 one-to-many accumulator layout.
// ---------------------------------------------------------------------------
static float ExactDistance(const float* q, const float* x, int dim, int metric) {
  const bool dot = metric == ORC_METRIC_DOT;
  auto term = [dot](float acc, float a, float b) {
    if (dot) return std::fma(-a, b, acc);
    const float t = a - b;
    return std::fma(t, t, acc);
  };
  float a8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int j = 0;
  for (; j + 8 <= dim; j += 8)
    for (int l = 0; l < 8; ++l) a8[l] = term(a8[l], q[j + l], x[j + l]);
  float s[4];
  for (int l = 0; l < 4; ++l) s[l] = a8[l + 4] + a8[l];
  if (j + 4 <= dim) {
    for (int l = 0; l < 4; ++l) s[l] = term(s[l], q[j + l], x[j + l]);
    j += 4;
  }
  if (j + 2 <= dim) {
    s[2] = term(s[2], q[j], x[j]);
    s[3] = term(s[3], q[j + 1], x[j + 1]);
    j += 2;
  }
  const float lo = s[0] + s[2];
  const float hi = s[1] + s[3];
  float r = lo + hi;
  // Scalar tail AccTerm (acc - a*b / acc + t*t) contracted to one FMA by the
  // reference's compiler at default -ffp-contract (documented choice).
  if (j < dim) r = term(r, q[j], x[j]);
  return r;
}

// ---------------------------------------------------------------------------
// Search driver.
// ---------------------------------------------------------------------------
struct Cand {
  uint32_t tie;  // packed (leaf << shift | local) or global id
  float d;
  uint64_t slot = 0;   // member index (ideal mode: the shard reorder's row)
};
static inline bool CandLess(const Cand& a, const Cand& b) {
  if (a.d != b.d) return a.d < b.d;
  return a.tie < b.tie;
}
using NN = std::vector<std::pair<uint32_t, float>>;
static inline bool NNLess(const std::pair<uint32_t, float>& a,
                          const std::pair<uint32_t, float>& b) {
  if (a.second != b.second) return a.second < b.second;
  return a.first < b.first;
}

static int Log2Ceil(uint32_t n) {
  int f = 31 - __builtin_clz(n);
  return ((n & (n - 1)) == 0) ? f : f + 1;
}

struct IndexView {
  const orc_index* ix;
  int shift;            // global top-N shift; 0 = per-leaf path
  bool disjoint;
  // a range-split shard (is_shard, smx_index_desc's tail): leaf l's rows are
  // rows [row_base[l], row_base[l] + n) of the whole index's leaf, so the
  // packed tie is leaf << shift | (row_base[l] + local); NULL otherwise
  const uint32_t* row_base = nullptr;
  // the shard's own float rows per member (reorder source), or NULL
  const float* member_rows = nullptr;
  std::vector<float> cnorms;
  std::vector<int> leaf_rank_by_norm;  // position in leaf_tokens_by_norm_
};

static int GlobalShift(const orc_index* ix) {
  if (!ix->residual || ix->num_leaves <= 1) return 0;
  uint64_t maxsz = 0;
  for (int l = 0; l < ix->num_leaves; ++l)
    maxsz = std::max<uint64_t>(maxsz, ix->leaf_offsets[l + 1] - ix->leaf_offsets[l]);
  const int inner = 32 - Log2Ceil(uint32_t(ix->num_leaves));
  return (maxsz <= (1ull << inner)) ? inner : 0;
}

static void BuildView(const orc_index* ix, IndexView* v) {
  v->ix = ix;
  v->shift = ix->is_shard ? ix->global_topn_shift : GlobalShift(ix);
  const uint64_t nmem = ix->leaf_offsets[ix->num_leaves];
  v->disjoint = ix->is_shard ? !ix->global_spilled : (nmem == ix->num_datapoints);
  v->row_base = ix->is_shard ? ix->leaf_row_base : nullptr;
  v->member_rows = ix->is_shard ? ix->member_rows : nullptr;
  if (v->disjoint && !ix->is_shard) {
    std::vector<uint8_t> seen(ix->num_datapoints, 0);
    for (uint64_t i = 0; i < nmem; ++i) {
      const uint32_t g = ix->leaf_members[i];
      if (g >= ix->num_datapoints || seen[g]) { v->disjoint = false; break; }
      seen[g] = 1;
    }
  }
  v->cnorms = CenterNorms(ix->centers, ix->num_leaves, ix->dim);
  // leaf_tokens_by_norm_: descending squared center norm
  // (tree_ah_hybrid_residual.cc:121-143); equal norms by ascending leaf id.
  std::vector<int> perm(ix->num_leaves);
  std::iota(perm.begin(), perm.end(), 0);
  std::vector<double> nrm(ix->num_leaves);
  for (int l = 0; l < ix->num_leaves; ++l) {
    double s = 0;
    const float* c = ix->centers + size_t(l) * ix->dim;
    for (int d = 0; d < ix->dim; ++d) s += double(c[d]) * c[d];
    nrm[l] = s;
  }
  std::stable_sort(perm.begin(), perm.end(),
                   [&](int a, int b) { return nrm[a] > nrm[b]; });
  v->leaf_rank_by_norm.assign(ix->num_leaves, 0);
  for (int r = 0; r < ix->num_leaves; ++r) v->leaf_rank_by_norm[perm[r]] = r;
}

// DeduplicateDatabaseSpilledResults (internal/utils.cc:135-162):
// duplicates averaged 0.5a+0.5b, then the final_size best by (dist, id).
static void DedupeSpilled(NN* r, size_t final_size) {
  std::unordered_map<uint32_t, size_t> pos;
  NN out;
  out.reserve(r->size());
  for (const auto& p : *r) {
    auto it = pos.find(p.first);
    if (it == pos.end()) {
      pos.emplace(p.first, out.size());
      out.push_back(p);
    } else {
      float& d = out[it->second].second;
      d = 0.5f * d + 0.5f * p.second;
    }
  }
  if (out.size() > final_size) {
    std::nth_element(out.begin(), out.begin() + (final_size - 1), out.end(), NNLess);
    out.resize(final_size);
  }
  *r = std::move(out);
}

static int32_t SpillK(const IndexView& v, int32_t k) {
  if (v.disjoint) return k;
  const double r = double(k) * double(v.ix->spilling_overretrieve_factor);
  if (r > double(std::numeric_limits<int32_t>::max())) return std::numeric_limits<int32_t>::max();
  return static_cast<int32_t>(r);
}

// Pipeline B's per-leaf int16 epsilon: ComputePossiblyFixedPointMaxDistance
// (asymmetric_hashing_impl.h:207-219) of the global epsilon, then
// min(., int16 max - 1) + 1 (querying.h:413-423), narrowed to int16 by the
// FastTopNeighbors<int16_t> constructor.
static int32_t FixedPointMaxDistance(float eps, float mult) {
  constexpr int32_t kI32Max = std::numeric_limits<int32_t>::max();
  if (eps == kInf) return kI32Max;
  const float x = eps * mult;
  if (x >= static_cast<float>(kI32Max)) return kI32Max;
  const float f = std::floor(x);
  return f < -2147483648.0f ? std::numeric_limits<int32_t>::min() : static_cast<int32_t>(f);
}

static int16_t LeafInt16Epsilon(float eps, float mult) {
  const int32_t e =
      std::min<int32_t>(FixedPointMaxDistance(eps, mult), std::numeric_limits<int16_t>::max() - 1) + 1;
  return static_cast<int16_t>(e);
}

// One leaf of pipeline B through GetTopInt16DistancesImpl with one query
// (lut16_avx2.inc:308-389): FastTopNeighbors<int16_t>(k, eps16) over the raw
// sums, pushing iff sum < threshold, the threshold re-read after every GC;
// FinishUnsorted's contents (storage order) into `local` as (leaf-local
// index, int16 sum).
static void LeafInt16TopN(const orc_index* ix, int leaf, const Lut& lut, size_t k, int16_t eps16,
                          std::vector<std::pair<uint32_t, int16_t>>* local) {
  const int nb = ix->num_blocks;
  const uint64_t beg = ix->leaf_offsets[leaf];
  const uint32_t n = uint32_t(ix->leaf_offsets[leaf + 1] - beg);
  local->clear();
  if (n == 0 || k == 0) return;
  FastTopNT<int16_t> lt(k, eps16);
  int32_t thr = lt.epsilon();
  int32_t acc[32];
  const uint32_t groups = (n + 31) / 32;
  for (uint32_t g = 0; g < groups; ++g) {
    const int lanes = (g == groups - 1) ? int(n - 32 * g) : 32;
    for (int l = 0; l < lanes; ++l)
      acc[l] = Accumulate(ix->member_codes + (beg + 32 * g + l) * nb, nb, lut.u8.data());
    auto push_mask = [&]() {
      uint32_t pm = 0;
      for (int l = 0; l < lanes; ++l) pm |= uint32_t(acc[l] < thr) << l;
      return pm;
    };
    uint32_t pm = push_mask();
    while (pm) {
      const int l = Ctz(pm);
      pm &= pm - 1;
      if (lt.Push(32 * g + l, static_cast<int16_t>(acc[l]))) {
        lt.GarbageCollectApprox();
        thr = lt.epsilon();
        pm &= push_mask();
      }
    }
  }
  lt.Finish(local);
}

// TopNeighbors<float> (top_n_amortized_constant.h:34-140): elements kept
// unsorted up to 2 * limit, then partitioned to the exact best `limit` under
// (distance, index) with approx_bottom = the limit-th; while fewer than
// `limit` are held, approx_bottom tracks the worst pushed.
class TopNeighborsF {
 public:
  explicit TopNeighborsF(size_t limit) : limit_(limit) {}
  void Push(uint32_t i, float d) {
    const std::pair<uint32_t, float> e{i, d};
    if (el_.size() < limit_) {
      if (el_.empty() || NNLess(bottom_, e)) bottom_ = e;
      el_.push_back(e);
    } else if (NNLess(e, bottom_)) {
      el_.push_back(e);
      if (el_.size() >= 2 * limit_) Partition();
    }
  }
  bool Full() const { return el_.size() >= limit_; }
  float ApproxBottomDistance() const { return bottom_.second; }
  void TakeUnsorted(NN* out) {
    if (el_.size() > limit_) Partition();
    *out = std::move(el_);
    el_.clear();
  }

 private:
  void Partition() {
    std::nth_element(el_.begin(), el_.begin() + (limit_ - 1), el_.end(), NNLess);
    el_.resize(limit_);
    bottom_ = el_.back();
  }
  size_t limit_;
  std::vector<std::pair<uint32_t, float>> el_;
  std::pair<uint32_t, float> bottom_{0, 0.0f};
};

// Pipeline B emulate mode (A.9): the replay of one query through
// TreeXHybridSMMD::FindNeighborsPreTokenizedBatchedOptimizedImpl
// (tree_x_hybrid_smmd.cc:718-790), the path the reference takes whenever
// nq * leaves_to_search >= num_leaves (:660-667).  Leaves are visited in
// ascending leaf id (InvertQueryTokens, :690-704).  Per leaf: the leaf
// parameters take the global top-N's epsilon at visit time
// (CreateParamsSubsetForLeaf, batching.h:96-116); the leaf's AH searcher
// keeps a FastTopNeighbors<int16_t>(k', eps16) over the raw int16 sums,
// pushing iff sum < threshold and re-reading the threshold after every GC
// (GetTopInt16DistancesImpl, lut16_avx2.inc:308-389); FinishUnsorted's
// contents, scaled by the float reciprocal 1.0f / mult (querying.h:446-455),
// are pushed in storage order into the global FastTopNeighbors<float> iff
// d <= epsilon (SingleMachineSearcherBase::FindNeighborsBatchedImpl,
// single_machine_base.cc:759-808), local ids mapped to global ids.
// The generic per-query path (nq * L < num_leaves) is PipelineBGeneric.
static void PipelineBEmulate(const IndexView& v, const std::vector<int>& leaves,
                             const Lut& lut, float inv, int32_t kk, NN* out) {
  const orc_index* ix = v.ix;
  std::vector<int> ord(leaves);
  std::sort(ord.begin(), ord.end());
  const size_t k = size_t(std::max(kk, 0));
  FastTopN top(k);  // pre_reordering_epsilon = +inf
  std::vector<std::pair<uint32_t, int16_t>> local;
  for (int leaf : ord) {
    const uint64_t beg = ix->leaf_offsets[leaf];
    LeafInt16TopN(ix, leaf, lut, k, LeafInt16Epsilon(top.epsilon(), lut.mult), &local);
    float eps = top.epsilon();
    for (const auto& e : local) {
      const float d = static_cast<float>(e.second) * inv;
      if (d <= eps && top.Push(ix->leaf_members[beg + e.first], d)) {
        top.GarbageCollectApprox();
        eps = top.epsilon();
      }
    }
  }
  top.Finish(out);
}

// Pipeline B emulate mode, the generic per-query path the reference takes
// when nq * leaves_to_search < num_leaves
// (TreeXHybridSMMD::FindNeighborsPreTokenizedBatchedGenericImpl,
// tree_x_hybrid_smmd.cc:669-691 -> FindNeighborsPreTokenizedImpl, :875-1028):
// the query's tokens in top-L order (sequential ParallelFor without a pool);
// per leaf the leaf searcher's single-query LUT16 path
// (FindApproximateNeighborsForceLUT16, querying.h:711-734): no results when
// the fixed-point max distance of the forwarded epsilon is below int16 min,
// else FindApproxNeighborsFastTopNeighbors<1> (:402-459) -- the per-leaf int16
// FastTopNeighbors -- with the results scaled by 1.0f / mult; every result,
// mapped to its global id, pushed into one TopNeighbors<float>(k'); once it
// is full the next leaf's epsilon is its approx_bottom (:1004-1010).
// A single token (:926-949) is the leaf searcher's own search with
// pre_reordering_num_neighbors -- no spilling multiplier, no dedupe -- its
// results remapped to global ids.
static void PipelineBGeneric(const IndexView& v, const std::vector<int>& leaves,
                             const Lut& lut, float inv, int32_t kk, int32_t pre_nn, NN* out) {
  const orc_index* ix = v.ix;
  out->clear();
  if (leaves.size() == 1) {
    const int leaf = leaves[0];
    const size_t k1 = size_t(std::max(pre_nn, 0));
    if (k1 == 0) return;
    std::vector<std::pair<uint32_t, int16_t>> local;
    LeafInt16TopN(ix, leaf, lut, k1, LeafInt16Epsilon(kInf, lut.mult), &local);
    const uint64_t beg = ix->leaf_offsets[leaf];
    for (const auto& e : local)
      out->push_back({ix->leaf_members[beg + e.first], static_cast<float>(e.second) * inv});
    return;
  }
  const size_t k = size_t(std::max(kk, 0));
  if (k == 0 || leaves.empty()) return;
  TopNeighborsF top(k);
  float eps = kInf;  // pre_reordering_epsilon
  std::vector<std::pair<uint32_t, int16_t>> local;
  for (int leaf : leaves) {
    if (FixedPointMaxDistance(eps, lut.mult) < std::numeric_limits<int16_t>::min()) {
      local.clear();
    } else {
      LeafInt16TopN(ix, leaf, lut, k, LeafInt16Epsilon(eps, lut.mult), &local);
    }
    const uint64_t beg = ix->leaf_offsets[leaf];
    for (const auto& e : local)
      top.Push(ix->leaf_members[beg + e.first], static_cast<float>(e.second) * inv);
    if (top.Full()) eps = top.ApproxBottomDistance();
  }
  top.TakeUnsorted(out);
}

// One query's pre-reorder candidates (global ids), unsorted.  `generic`:
// pipeline B's emulate mode takes the per-query path (PipelineBGeneric).
// slots (ideal mode, may be NULL): global id -> member index of the kept
// candidates, for a shard's reorder from its own member rows.
static void QueryPreReorder(const IndexView& v, const float* q, int L,
                            int pre_nn, int mode, bool generic, std::vector<float>* scratch,
                            NN* out, std::unordered_map<uint32_t, uint64_t>* slots = nullptr) {
  const orc_index* ix = v.ix;
  const int nl = ix->num_leaves, nb = ix->num_blocks, dim = ix->dim;
  scratch->resize(nl);
  if (mode & ORC_PARTITION_ONE_TO_MANY) {
    for (int c = 0; c < nl; ++c)
      (*scratch)[c] = ExactDistance(q, ix->centers + size_t(c) * dim, dim, ix->metric);
  } else {
    PartitionScoresOne(q, dim, ix->centers, nl, ix->metric, v.cnorms, scratch->data());
  }
  mode &= 3;
  std::vector<int> leaves;
  std::vector<float> biases;
  TopL(scratch->data(), nl, L, &leaves, &biases);

  Lut lut;
  CreateLut(q, dim, ix->codebook, nb, ix->dims_per_block, ix->metric, nullptr, &lut);
  const bool residual = ix->residual != 0;
  // Pipeline A: inv = (float)(1.0 / (double)mult) (lut16_avx2.inc:427-430).
  // Pipeline B: inv = 1.0f / mult in float (querying.h:450-454).
  const float inv = residual ? static_cast<float>(1.0 / static_cast<double>(lut.mult))
                             : 1.0f / lut.mult;
  const int32_t kk = SpillK(v, pre_nn);
  const int shift = v.shift;

  if (mode == ORC_MODE_EMULATE && residual && shift > 0) {
    // Sequential replay: leaves in leaf_tokens_by_norm_ order, dps in order,
    // int16 truncated prefilter against the running epsilon.
    std::vector<int> ord(leaves.size());
    std::iota(ord.begin(), ord.end(), 0);
    std::sort(ord.begin(), ord.end(), [&](int a, int b) {
      return v.leaf_rank_by_norm[leaves[a]] < v.leaf_rank_by_norm[leaves[b]];
    });
    FastTopN top(kk);
    int32_t acc[32];
    for (int oi : ord) {
      const int leaf = leaves[oi];
      const float bias = biases[oi];
      const uint64_t beg = ix->leaf_offsets[leaf];
      const uint32_t n = uint32_t(ix->leaf_offsets[leaf + 1] - beg);
      if (n == 0) continue;
      int32_t thr = Int16Threshold(top.epsilon(), bias, lut.mult);
      const uint32_t groups = (n + 31) / 32;
      const uint32_t first = uint32_t(leaf) << shift;
      for (uint32_t g = 0; g < groups; ++g) {
        for (int l = 0; l < 32; ++l) {
          uint32_t m = g * 32 + l;
          if (m >= n) m = n - 1;  // packed tail repeats the last datapoint
          acc[l] = Accumulate(ix->member_codes + (beg + m) * nb, nb, lut.u8.data());
        }
        auto push_mask = [&]() {
          uint32_t pm = 0;
          for (int l = 0; l < 32; ++l) pm |= uint32_t(acc[l] < thr) << l;
          return pm;
        };
        uint32_t pm = push_mask();
        if (!pm) continue;
        if (g == groups - 1) pm &= FinalMask32(n);
        while (pm) {
          const int l = Ctz(pm);
          pm &= pm - 1;
          const float p = static_cast<float>(acc[l]) * inv;
          const float d = p + bias;
          if (top.Push(first + g * 32 + l, d)) {
            top.GarbageCollectApprox();
            thr = Int16Threshold(top.epsilon(), bias, lut.mult);
            pm &= push_mask();
          }
        }
      }
    }
    NN res;
    top.Finish(&res);
    for (auto& p : res) {
      const uint32_t leaf = p.first >> shift;
      const uint32_t local = p.first & ((1u << shift) - 1);
      p.first = ix->leaf_members[ix->leaf_offsets[leaf] + local];
    }
    *out = std::move(res);
  } else if (mode == ORC_MODE_EMULATE && !residual && generic) {
    PipelineBGeneric(v, leaves, lut, inv, kk, pre_nn, out);
  } else if (mode == ORC_MODE_EMULATE && !residual) {
    PipelineBEmulate(v, leaves, lut, inv, kk, out);
  } else {
    // Ideal: exact top-k' by (distance, tie id) over every scanned point.
    std::vector<Cand> cands;
    for (size_t li = 0; li < leaves.size(); ++li) {
      const int leaf = leaves[li];
      const float bias = residual ? biases[li] : 0.0f;
      const uint64_t beg = ix->leaf_offsets[leaf];
      const uint32_t n = uint32_t(ix->leaf_offsets[leaf + 1] - beg);
      // a shard's rows keep the whole index's row numbers in the tie
      const uint32_t rb = v.row_base ? v.row_base[leaf] : 0u;
      for (uint32_t i = 0; i < n; ++i) {
        const int32_t a = Accumulate(ix->member_codes + (beg + i) * nb, nb, lut.u8.data());
        const float p = static_cast<float>(a) * inv;
        const float d = residual ? p + bias : p;
        const uint32_t tie = shift > 0 ? ((uint32_t(leaf) << shift) | (rb + i))
                                       : ix->leaf_members[beg + i];
        cands.push_back({tie, d, beg + i});
      }
    }
    const size_t keep = std::min<size_t>(size_t(std::max(kk, 0)), cands.size());
    std::partial_sort(cands.begin(), cands.begin() + keep, cands.end(), CandLess);
    out->resize(keep);
    for (size_t i = 0; i < keep; ++i) {
      const uint32_t g = ix->leaf_members[cands[i].slot];
      if (slots) slots->emplace(g, cands[i].slot);   // (a SOAR id's copies: the same row)
      (*out)[i] = {g, cands[i].d};
    }
  }
  if (!v.disjoint && pre_nn > 0) DedupeSpilled(out, size_t(pre_nn));
}

static void RemovePastLimitAndSort(NN* r, size_t limit) {
  if (limit == 0) { r->clear(); return; }
  if (r->size() > limit) {
    std::nth_element(r->begin(), r->begin() + (limit - 1), r->end(), NNLess);
    r->resize(limit);
  }
  std::sort(r->begin(), r->end(), NNLess);
}

template <typename F>
static void ParallelFor(int n, int nthreads, F f) {
  nthreads = std::max(1, std::min(nthreads, n));
  if (nthreads == 1) {
    for (int i = 0; i < n; ++i) f(i);
    return;
  }
  std::atomic<int> next{0};
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([&]() {
      for (int i; (i = next.fetch_add(1)) < n;) f(i);
    });
  for (auto& t : th) t.join();
}

static int SearchImpl(const orc_index* ix, const float* queries, int nq,
                      int leaves, int pre_nn, int final_nn, int do_reorder,
                      int mode, int nthreads, bool pre_only, uint32_t* out_idx,
                      float* out_dist, int32_t* out_count) {
  if (!ix || nq < 0 || leaves <= 0 || final_nn < 0) return -1;
  IndexView v;
  BuildView(ix, &v);
  const bool reorder = do_reorder && (ix->dataset != nullptr || v.member_rows != nullptr);
  // a shard reorders from its members' own rows (ideal mode only)
  if (reorder && !ix->dataset && (mode & 3) != ORC_MODE_IDEAL) return -2;
  // scann.cc:406-430: without reordering pre_nn = final_nn.
  const int pnn = reorder ? pre_nn : final_nn;
  const int width = pre_only ? pnn : final_nn;
  // tree_x_hybrid_smmd.cc:660-667: the generic per-query path when the
  // batch's tokens number fewer than the leaves
  const bool generic =
      uint64_t(nq) * uint64_t(std::min(leaves, ix->num_leaves)) < uint64_t(ix->num_leaves);
  ParallelFor(nq, nthreads, [&](int qi) {
    std::vector<float> scratch;
    const float* q = queries + size_t(qi) * ix->dim;
    NN r;
    std::unordered_map<uint32_t, uint64_t> slots;
    const bool by_member = reorder && !ix->dataset;
    QueryPreReorder(v, q, leaves, pnn, mode, generic, &scratch, &r, by_member ? &slots : nullptr);
    if (pre_only) {
      std::sort(r.begin(), r.end(), NNLess);
    } else {
      if (reorder)
        for (auto& p : r) {
          const float* row = by_member ? v.member_rows + size_t(slots.at(p.first)) * ix->dim
                                       : ix->dataset + size_t(p.first) * ix->dim;
          p.second = ExactDistance(q, row, ix->dim, ix->metric);
        }
      RemovePastLimitAndSort(&r, reorder ? size_t(final_nn) : r.size());
      if (!reorder && r.size() > size_t(final_nn)) r.resize(final_nn);
    }
    out_count[qi] = int32_t(r.size());
    for (int j = 0; j < width; ++j) {
      const bool has = size_t(j) < r.size();
      out_idx[size_t(qi) * width + j] = has ? r[j].first : 0;
      out_dist[size_t(qi) * width + j] =
          has ? r[j].second : std::numeric_limits<float>::quiet_NaN();
    }
  });
  return 0;
}

}  // namespace orc

extern "C" {

void orc_partition_scores(const float* queries, int32_t nq, int32_t dim,
                          const float* centers, int32_t num_leaves,
                          int32_t metric, float* out) {
  const auto cn = orc::CenterNorms(centers, num_leaves, dim);
  for (int q = 0; q < nq; ++q)
    orc::PartitionScoresOne(queries + size_t(q) * dim, dim, centers, num_leaves,
                            metric, cn, out + size_t(q) * num_leaves);
}

void orc_partition_topl(const float* queries, int32_t nq, int32_t dim,
                        const float* centers, int32_t num_leaves,
                        int32_t metric, int32_t L, int32_t* out_leaf,
                        float* out_score) {
  const auto cn = orc::CenterNorms(centers, num_leaves, dim);
  std::vector<float> s(num_leaves);
  const int Lc = std::min(L, num_leaves);
  for (int q = 0; q < nq; ++q) {
    orc::PartitionScoresOne(queries + size_t(q) * dim, dim, centers, num_leaves,
                            metric, cn, s.data());
    std::vector<int> lf;
    std::vector<float> sc;
    orc::TopL(s.data(), num_leaves, Lc, &lf, &sc);
    for (int i = 0; i < Lc; ++i) {
      out_leaf[size_t(q) * L + i] = lf[i];
      out_score[size_t(q) * L + i] = sc[i];
    }
  }
}

int orc_create_lut(const float* query, int32_t dim, const float* codebook,
                   int32_t num_blocks, int32_t dims_per_block, int32_t metric,
                   float* raw_out, uint8_t* lut_out, float* mult_out) {
  orc::Lut lut;
  if (orc::CreateLut(query, dim, codebook, num_blocks, dims_per_block, metric,
                     raw_out, &lut) != 0)
    return -1;
  std::copy(lut.u8.begin(), lut.u8.end(), lut_out);
  *mult_out = lut.mult;
  return 0;
}

void orc_pack_codes(const uint8_t* codes, uint32_t n, int32_t nb, uint8_t* out) {
  if (n == 0) return;
  const uint32_t groups = (n + 31) / 32;
  for (uint32_t g = 0; g < groups; ++g) {
    uint8_t* dst = out + size_t(g) * 16 * nb;
    for (int b = 0; b < nb; ++b)
      for (int m = 0; m < 16; ++m) {
        uint32_t lo = g * 32 + m, hi = g * 32 + m + 16;
        lo = std::min(lo, n - 1);
        hi = std::min(hi, n - 1);
        dst[b * 16 + m] = uint8_t(codes[size_t(hi) * nb + b] * 16 + codes[size_t(lo) * nb + b]);
      }
  }
}

void orc_lut16_accumulate(const uint8_t* packed, uint32_t n, int32_t nb,
                          const uint8_t* lut, int32_t* out) {
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t g = i / 32, lane = i % 32;
    const uint8_t* src = packed + size_t(g) * 16 * nb;
    int32_t acc = 0;
    for (int b = 0; b < nb; ++b) {
      const uint8_t byte = src[b * 16 + (lane & 15)];
      const uint8_t code = lane < 16 ? (byte & 15) : (byte >> 4);
      acc += int32_t(lut[b * 16 + code]) - 128;
    }
    out[i] = acc;
  }
}

int32_t orc_global_topn_shift(const orc_index* idx) { return orc::GlobalShift(idx); }

int orc_search(const orc_index* idx, const float* queries, int32_t nq,
               int32_t leaves, int32_t pre_nn, int32_t final_nn,
               int32_t do_reorder, int32_t mode, int32_t nthreads,
               uint32_t* out_idx, float* out_dist, int32_t* out_count) {
  return orc::SearchImpl(idx, queries, nq, leaves, pre_nn, final_nn, do_reorder,
                         mode, nthreads, false, out_idx, out_dist, out_count);
}

int orc_search_pre_reorder(const orc_index* idx, const float* queries,
                           int32_t nq, int32_t leaves, int32_t pre_nn,
                           int32_t mode, int32_t nthreads, uint32_t* out_idx,
                           float* out_dist, int32_t* out_count) {
  return orc::SearchImpl(idx, queries, nq, leaves, pre_nn, pre_nn, 1, mode,
                         nthreads, true, out_idx, out_dist, out_count);
}

float orc_exact_distance(const float* q, const float* x, int32_t dim,
                         int32_t metric) {
  return orc::ExactDistance(q, x, dim, metric);
}

int32_t orc_fast_topn_replay(const uint32_t* idx, const float* dist, int32_t n,
                             int32_t k, uint32_t* out_idx, float* out_dist,
                             int32_t* out_num_gc) {
  // PushBlockToFastTopNeighbors scalar loop (fast_top_neighbors.h:430-438):
  // push iff dist < epsilon.
  orc::FastTopN top{size_t(k)};
  for (int32_t i = 0; i < n; ++i) {
    if (dist[i] < top.epsilon()) {
      if (top.Push(idx[i], dist[i])) top.GarbageCollectApprox();
    }
  }
  orc::NN r;
  top.Finish(&r);
  std::sort(r.begin(), r.end(), orc::NNLess);
  for (size_t i = 0; i < r.size(); ++i) {
    out_idx[i] = r[i].first;
    out_dist[i] = r[i].second;
  }
  if (out_num_gc) *out_num_gc = top.num_gc();
  return int32_t(r.size());
}

int32_t orc_fast_topn_replay_i16(const uint32_t* idx, const int16_t* dist, int32_t n,
                                 int32_t k, int16_t epsilon, uint32_t* out_idx,
                                 int16_t* out_dist, int32_t* out_num_gc) {
  // GetTopInt16DistancesImpl's push loop (lut16_avx2.inc:352-375) on one
  // FastTopNeighbors<int16_t>(k, epsilon): push iff dist < epsilon, the
  // threshold re-read after every GC; FinishUnsorted's storage order out.
  orc::FastTopNT<int16_t> top(size_t(k), epsilon);
  for (int32_t i = 0; i < n; ++i) {
    if (dist[i] < top.epsilon()) {
      if (top.Push(idx[i], dist[i])) top.GarbageCollectApprox();
    }
  }
  std::vector<std::pair<uint32_t, int16_t>> r;
  top.Finish(&r);
  for (size_t i = 0; i < r.size(); ++i) {
    out_idx[i] = r[i].first;
    out_dist[i] = r[i].second;
  }
  if (out_num_gc) *out_num_gc = top.num_gc();
  return int32_t(r.size());
}

// AVQ noise-shaped encoding of n rows: IndexDatapointNoiseShaped
// (asymmetric_hashing_impl.cc:434-503) with ComputeResidualStats (:300-343,
// ComputeResidualStatsForCluster :283-298), ComputeParallelCostMultiplier
// (:268-274), InitializeToMinResidualNorm (:345-358) and
// OptimizeSingleSubspace (:372-404), one row at a time.  Blocks are chunks of
// dims_per_block coordinates, the last one zero-padded.  ||x||^2 of the cost
// multiplier is accumulated in coordinate order like the chunked norm (the
// reference's SquaredL2Norm order is its SIMD target's).  Blocks with equal
// residual norms keep block order in the visiting sort.
void orc_avq_encode(const float* residuals, const float* originals, int32_t n, int32_t dim,
                    const float* codebook, int32_t nb, int32_t dpb, double threshold,
                    uint8_t* out) {
  const int nc = 16;
  for (int32_t row = 0; row < n; ++row) {
    const float* r = residuals + size_t(row) * dim;
    const float* x = originals + size_t(row) * dim;
    auto coord = [&](const float* v, int b, int i) -> double {
      const int d = b * dpb + i;
      return d < dim ? static_cast<double>(v[d]) : 0.0;
    };
    double chunked_norm = 0.0;
    for (int b = 0; b < nb; ++b)
      for (int i = 0; i < dpb; ++i) chunked_norm += coord(x, b, i) * coord(x, b, i);
    const double sq_norm = chunked_norm;
    chunked_norm = std::sqrt(chunked_norm);
    const double inv_norm = 1.0 / chunked_norm;
    std::vector<double> rn(size_t(nb) * nc), par(size_t(nb) * nc);
    for (int b = 0; b < nb; ++b)
      for (int c = 0; c < nc; ++c) {
        double a = 0.0, p = 0.0;
        for (int i = 0; i < dpb; ++i) {
          const double rc = coord(r, b, i) - static_cast<double>(codebook[(size_t(b) * nc + c) * dpb + i]);
          a += rc * rc;
          p += rc * coord(x, b, i) * inv_norm;
        }
        rn[size_t(b) * nc + c] = a;
        par[size_t(b) * nc + c] = p;
      }
    const double t2 = threshold * threshold;
    const double eta = (t2 / sq_norm) / ((1.0 - t2 / sq_norm) / (double(dim) - 1.0));
    std::vector<int> code(nb);
    for (int b = 0; b < nb; ++b) {
      int best = 0;
      for (int c = 1; c < nc; ++c)
        if (rn[size_t(b) * nc + c] < rn[size_t(b) * nc + best]) best = c;
      code[b] = best;
    }
    double P = 0.0;
    for (int b = 0; b < nb; ++b) P += par[size_t(b) * nc + code[b]];
    std::vector<int> order(nb);
    for (int b = 0; b < nb; ++b) order[b] = b;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
      return rn[size_t(a) * nc + code[a]] > rn[size_t(b) * nc + code[b]];
    });
    bool changed = true;
    for (int round = 0; changed && round < 10; ++round) {
      changed = false;
      for (int i = 0; i < nb; ++i) {
        const int b = order[i];
        const int cur = code[b];
        const double old_rn = rn[size_t(b) * nc + cur], old_par = par[size_t(b) * nc + cur];
        int new_c = cur;
        double best_cost = 0.0, best_p = P;
        for (int c = 0; c < nc; ++c) {
          if (c == cur) continue;
          const double new_p = P - old_par + par[size_t(b) * nc + c];
          const double pnd = new_p * new_p - P * P;
          if (pnd > 0.0) continue;
          const double rnd = rn[size_t(b) * nc + c] - old_rn;
          const double perp = rnd - pnd;
          const double cost = eta * pnd + perp;
          if (cost < best_cost) {
            new_c = c;
            best_cost = cost;
            best_p = new_p;
          }
        }
        if (new_c != cur) {
          P = best_p;
          code[b] = new_c;
          changed = true;
        }
      }
    }
    for (int b = 0; b < nb; ++b) out[size_t(row) * nb + b] = uint8_t(code[b]);
  }
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Driver for the AVX2 port (lut16_avx2_port.cc): the reference's leaf-major
// batched execution with <=3 queries per LUT16 call.  Per query it performs
// exactly the pushes of the EMULATE branch above, in the same order.
// ---------------------------------------------------------------------------
namespace orc_port {
using GroupFn = void (*)(const uint8_t*, int, const uint8_t*, int16_t*);
// <= 3 queries' accumulators of one group at once (the reference's
// Avx2LUT16BottomLoop): group, blocks, luts, count, out, prefetch pointer
using BatchFn = void (*)(const uint8_t*, int, const uint8_t* const*, int, int16_t (*)[32],
                         const uint8_t*);
using MaskFn = uint32_t (*)(const int16_t*, int16_t);
// Partition scores of one query against the transposed centers ct[dim][nlp]
// (nlp = nl rounded up to 8), the same per-center FMA chain as
// PartitionScoresOne, eight centers per vector (many_to_many_impl.inc:522-560
// runs the reference's chain across centers the same way).
using PartFn = void (*)(const float* q, int dim, const float* ct, int nlp, int nl, int metric,
                        const float* cnorms, float qnorm, float* out);

struct Prepared {
  const orc_index* ix;
  bool pipeline_b = false;                   // non-residual: tree_x_hybrid_smmd
  orc::IndexView view;
  std::vector<std::vector<uint8_t>> packed;  // per leaf, reference layout
  std::vector<int> leaf_order;               // leaf_tokens_by_norm_
  std::vector<float> ct;                     // [dim][nlp] transposed centers
  int nlp = 0;
};

void* Prepare(const orc_index* ix) {
  if (!ix) return nullptr;
  auto* p = new Prepared;
  p->ix = ix;
  p->pipeline_b = !ix->residual;
  orc::BuildView(ix, &p->view);
  if (!p->pipeline_b && p->view.shift == 0) {
    delete p;
    return nullptr;
  }
  const int nl = ix->num_leaves, nb = ix->num_blocks;
  p->packed.resize(nl);
  for (int l = 0; l < nl; ++l) {
    const uint64_t beg = ix->leaf_offsets[l];
    const uint32_t n = uint32_t(ix->leaf_offsets[l + 1] - beg);
    p->packed[l].assign(size_t(nb) * ((n + 31) / 32) * 16, 0);
    orc_pack_codes(ix->member_codes + beg * nb, n, nb, p->packed[l].data());
  }
  // Pipeline A visits leaves in leaf_tokens_by_norm_ order, pipeline B in
  // ascending leaf id (tree_x_hybrid_smmd.cc:761).
  p->leaf_order.resize(nl);
  for (int l = 0; l < nl; ++l)
    p->leaf_order[p->pipeline_b ? l : p->view.leaf_rank_by_norm[l]] = l;
  const int dim = ix->dim;
  p->nlp = (nl + 7) & ~7;
  p->ct.assign(size_t(dim) * p->nlp, 0.0f);
  for (int c = 0; c < nl; ++c)
    for (int d = 0; d < dim; ++d) p->ct[size_t(d) * p->nlp + c] = ix->centers[size_t(c) * dim + d];
  return p;
}

void Release(void* p) { delete static_cast<Prepared*>(p); }

int Run(void* prepared, const float* queries, int nq, int leaves, int pre_nn,
        int final_nn, int do_reorder, int nthreads, uint32_t* out_idx,
        float* out_dist, int32_t* out_count, GroupFn group_fn, MaskFn mask_fn,
        PartFn part_fn, double* phase_s, BatchFn batch_fn) {
  auto* P = static_cast<Prepared*>(prepared);
  if (!P || leaves <= 0 || final_nn < 0 || nq < 0) return -1;
  const orc_index* ix = P->ix;
  const orc::IndexView& v = P->view;
  const int nl = ix->num_leaves, nb = ix->num_blocks, dim = ix->dim;
  const bool reorder = do_reorder && ix->dataset != nullptr;
  const int pnn = reorder ? pre_nn : final_nn;
  const int32_t kk = orc::SpillK(v, pnn);
  const int shift = v.shift;
  nthreads = std::max(1, nthreads);
  // SearchBatchedParallel chunking: min(max(1, ceil(nq/threads)), 256).
  const int chunk = std::min(std::max(1, (nq + nthreads - 1) / nthreads), 256);
  const int nchunks = (nq + chunk - 1) / chunk;
  // CPU seconds per phase: [0] partition + top-L + LUT, [1] the leaf
  // scan (LUT16 + FastTopNeighbors), [2] finish + dedupe + reorder
  std::mutex tmu;
  double tsum[3] = {0.0, 0.0, 0.0};
  // per-thread CPU time (not wall time: robust to a CPU quota below the
  // thread count)
  auto cpu_now = []() {
    timespec ts;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
    return double(ts.tv_sec) + 1e-9 * double(ts.tv_nsec);
  };
  orc::ParallelFor(nchunks, nthreads, [&](int ci) {
    const double c0 = cpu_now();
    const int q0 = ci * chunk, nqc = std::min(chunk, nq - q0);
    std::vector<orc::Lut> luts(nqc);
    std::vector<float> invs(nqc);
    std::vector<orc::FastTopN> tops;
    tops.reserve(nqc);
    std::vector<std::vector<std::pair<int, float>>> by_leaf(nl);
    std::vector<float> scratch(nl);
    for (int j = 0; j < nqc; ++j) {
      const float* q = queries + size_t(q0 + j) * dim;
      if (part_fn)
        part_fn(q, dim, P->ct.data(), P->nlp, nl, ix->metric, v.cnorms.data(),
                ix->metric == ORC_METRIC_DOT ? 0.0f : orc::QuerySqNorm(q, dim), scratch.data());
      else
        orc::PartitionScoresOne(q, dim, ix->centers, nl, ix->metric, v.cnorms,
                                scratch.data());
      std::vector<int> lf;
      std::vector<float> sc;
      orc::TopL(scratch.data(), nl, leaves, &lf, &sc);
      for (size_t i = 0; i < lf.size(); ++i) by_leaf[lf[i]].push_back({j, sc[i]});
      orc::CreateLut(q, dim, ix->codebook, nb, ix->dims_per_block, ix->metric,
                     nullptr, &luts[j]);
      invs[j] = P->pipeline_b ? 1.0f / luts[j].mult
                              : static_cast<float>(1.0 / static_cast<double>(luts[j].mult));
      tops.emplace_back(size_t(kk));
    }
    const double c1 = cpu_now();
    int16_t accs[3][32];
    if (P->pipeline_b) {
      // orc::PipelineBEmulate's pushes, leaf-major: per leaf, batches of
      // <= 3 queries share each code group load (searcher.cc:332-416).
      std::vector<orc::FastTopNT<int16_t>> lts;
      std::vector<std::pair<uint32_t, int16_t>> local;
      for (int leaf : P->leaf_order) {
        const auto& ql = by_leaf[leaf];
        const uint64_t beg = ix->leaf_offsets[leaf];
        const uint32_t n = uint32_t(ix->leaf_offsets[leaf + 1] - beg);
        if (ql.empty() || n == 0 || kk <= 0) continue;
        const uint8_t* packed = P->packed[leaf].data();
        const uint32_t groups = (n + 31) / 32;
        const uint32_t fmask = orc::FinalMask32(n);
        for (size_t bs = 0; bs < ql.size();) {
          const size_t left = ql.size() - bs;
          const size_t nbatch = left <= 3 ? left : (left >= 6 ? 3 : left / 2);
          lts.clear();
          int16_t thr[3];
          for (size_t t = 0; t < nbatch; ++t) {
            const int j = ql[bs + t].first;
            lts.emplace_back(size_t(kk), orc::LeafInt16Epsilon(tops[j].epsilon(), luts[j].mult));
            thr[t] = lts[t].epsilon();
          }
          const uint8_t* bl[3];
          for (size_t t = 0; t < nbatch; ++t) bl[t] = luts[ql[bs + t].first].u8.data();
          for (uint32_t g = 0; g < groups; ++g) {
            const uint8_t* grp = packed + size_t(g) * 16 * nb;
            if (batch_fn) batch_fn(grp, nb, bl, int(nbatch), accs, nullptr);
            for (size_t t = 0; t < nbatch; ++t) {
              const int j = ql[bs + t].first;
              int16_t* acc = accs[t];
              if (!batch_fn) group_fn(grp, nb, luts[j].u8.data(), acc);
              uint32_t pm = mask_fn(acc, thr[t]);
              if (!pm) continue;
              if (g == groups - 1) pm &= fmask;
              while (pm) {
                const int l = orc::Ctz(pm);
                pm &= pm - 1;
                if (lts[t].Push(g * 32 + l, acc[l])) {
                  lts[t].GarbageCollectApprox();
                  thr[t] = lts[t].epsilon();
                  pm &= mask_fn(acc, thr[t]);
                }
              }
            }
          }
          for (size_t t = 0; t < nbatch; ++t) {
            const int j = ql[bs + t].first;
            lts[t].Finish(&local);
            float eps = tops[j].epsilon();
            for (const auto& e : local) {
              const float d = static_cast<float>(e.second) * invs[j];
              if (d <= eps && tops[j].Push(ix->leaf_members[beg + e.first], d)) {
                tops[j].GarbageCollectApprox();
                eps = tops[j].epsilon();
              }
            }
          }
          bs += nbatch;
        }
      }
    }
    // the packed bytes of the leaf visited after `leaf` (with queries), for
    // the prefetch of its first groups
    std::vector<int> next_visit(nl, -1);
    {
      int nxt = -1;
      for (int i = nl - 1; i >= 0; --i) {
        const int l = P->leaf_order[i];
        next_visit[l] = nxt;
        if (!by_leaf[l].empty() && ix->leaf_offsets[l + 1] > ix->leaf_offsets[l]) nxt = l;
      }
    }
    auto next_packed = [&](int leaf) -> const uint8_t* {
      const int l = next_visit[leaf];
      return l < 0 ? nullptr : P->packed[l].data();
    };
    for (int leaf : P->leaf_order) {
      if (P->pipeline_b) break;
      const auto& ql = by_leaf[leaf];
      if (ql.empty()) continue;
      const uint32_t n = uint32_t(ix->leaf_offsets[leaf + 1] - ix->leaf_offsets[leaf]);
      if (n == 0) continue;
      const uint8_t* packed = P->packed[leaf].data();
      const uint32_t groups = (n + 31) / 32;
      const uint32_t first = uint32_t(leaf) << shift;
      const uint32_t fmask = orc::FinalMask32(n);
      for (size_t bs = 0; bs < ql.size();) {
        const size_t left = ql.size() - bs;
        const size_t nbatch = left <= 3 ? left : (left >= 6 ? 3 : left / 2);
        int16_t thr[3];
        for (size_t t = 0; t < nbatch; ++t) {
          const auto& e = ql[bs + t];
          thr[t] = int16_t(orc::Int16Threshold(tops[e.first].epsilon(), e.second,
                                               luts[e.first].mult));
        }
        const uint8_t* bl[3];
        for (size_t t = 0; t < nbatch; ++t) bl[t] = luts[ql[bs + t].first].u8.data();
        // kSmart prefetch (ComputeSmartPrefetchIndex, lut16_avx2.inc): the
        // last groups of this leaf prefetch the next visited leaf's first
        // bytes, 768 bytes ahead of the stream
        const uint8_t* next = next_packed(leaf);
        long pf_idx = std::min(0L, long((768 / 16 + nb - 1) / nb) - long(groups));
        for (uint32_t g = 0; g < groups; ++g, ++pf_idx) {
          const uint8_t* grp = packed + size_t(g) * 16 * nb;
          if (batch_fn)
            batch_fn(grp, nb, bl, int(nbatch), accs,
                     (pf_idx >= 0 && next) ? next + size_t(pf_idx) * 16 * nb : nullptr);
          for (size_t t = 0; t < nbatch; ++t) {
            const int j = ql[bs + t].first;
            const float bias = ql[bs + t].second;
            int16_t* acc = accs[t];
            if (!batch_fn) group_fn(grp, nb, luts[j].u8.data(), acc);
            uint32_t pm = mask_fn(acc, thr[t]);
            if (!pm) continue;
            if (g == groups - 1) pm &= fmask;
            while (pm) {
              const int l = orc::Ctz(pm);
              pm &= pm - 1;
              const float p = static_cast<float>(acc[l]) * invs[j];
              const float d = p + bias;
              if (tops[j].Push(first + g * 32 + l, d)) {
                tops[j].GarbageCollectApprox();
                thr[t] = int16_t(orc::Int16Threshold(tops[j].epsilon(), bias, luts[j].mult));
                pm &= mask_fn(acc, thr[t]);
              }
            }
          }
        }
        bs += nbatch;
      }
    }
    const double c2 = cpu_now();
    for (int j = 0; j < nqc; ++j) {
      const int qi = q0 + j;
      const float* q = queries + size_t(qi) * dim;
      orc::NN r;
      tops[j].Finish(&r);
      for (auto& p : r) {
        if (P->pipeline_b) break;  // global ids already
        const uint32_t leaf = p.first >> shift;
        const uint32_t local = p.first & ((1u << shift) - 1);
        p.first = ix->leaf_members[ix->leaf_offsets[leaf] + local];
      }
      if (!v.disjoint && pnn > 0) orc::DedupeSpilled(&r, size_t(pnn));
      if (reorder)
        for (auto& p : r)
          p.second = orc::ExactDistance(q, ix->dataset + size_t(p.first) * dim,
                                        dim, ix->metric);
      orc::RemovePastLimitAndSort(&r, reorder ? size_t(final_nn) : r.size());
      if (!reorder && r.size() > size_t(final_nn)) r.resize(final_nn);
      out_count[qi] = int32_t(r.size());
      for (int t = 0; t < final_nn; ++t) {
        const bool has = size_t(t) < r.size();
        out_idx[size_t(qi) * final_nn + t] = has ? r[t].first : 0;
        out_dist[size_t(qi) * final_nn + t] =
            has ? r[t].second : std::numeric_limits<float>::quiet_NaN();
      }
    }
    const double c3 = cpu_now();
    std::lock_guard<std::mutex> lk(tmu);
    tsum[0] += c1 - c0;
    tsum[1] += c2 - c1;
    tsum[2] += c3 - c2;
  });
  if (phase_s)
    for (int i = 0; i < 3; ++i) phase_s[i] = tsum[i];
  return 0;
}
}  // namespace orc_port

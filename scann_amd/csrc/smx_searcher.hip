// smx_searcher.hip — host side of the MI355X tree-AH searcher: index upload
// into the device layout, the batched search pipeline and the C ABI of
// include/scann_mi355x.h.
//
// Pipeline of one search_batched call (all on one HIP stream):
//   1 partition_topl      query tokenization (top-L leaves + biases)
//   2 lut_build           per-query int8 LUT16 tables, multipliers
//   3 pairs               invert query->leaves into leaf->queries (seed/main)
//   4 seed scan + select  per-query threshold from its first `seed_leaves`
//                         leaves (k'-th best key there)
//   5 main scan           every (leaf, query tile): MFMA LUT16 sums, fused
//                         distance, emission of keys <= threshold
//   6 final select        exact top-k' -> global ids -> SOAR dedupe -> exact
//                         reorder -> (distance, id) sort -> outputs
// A candidate list that overflows its capacity triggers the tightening loop
// (threshold <- k'-th stored key, rescan), which always makes progress.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/scann_mi355x.h"
#include "smx_internal.h"

namespace {

thread_local std::string g_last_error;

int Fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define SMX_HIP(expr)                                                              \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess)                                                          \
      return Fail(_e == hipErrorOutOfMemory ? SMX_OUT_OF_MEMORY : SMX_DEVICE_ERROR, \
                  std::string("HIP error in ") + #expr + ": " + hipGetErrorString(_e)); \
  } while (0)

template <typename T>
int DAlloc(T** p, size_t n) {
  *p = nullptr;
  if (n == 0) return SMX_OK;
  SMX_HIP(hipMalloc(reinterpret_cast<void**>(p), n * sizeof(T)));
  return SMX_OK;
}

template <typename T>
void DFree(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

int Log2Ceil(uint32_t n) {
  int f = 31 - __builtin_clz(n);
  return ((n & (n - 1)) == 0) ? f : f + 1;
}

// K values with a compiled scan kernel; others round up (zero padding).
int EffectiveKSteps(int nb) {
  // even: the sparse scan takes two code nibbles (four blocks) per step
  static const int kList[] = {4, 8, 12, 16, 20, 24, 26, 28, 32};
  const int k = (nb + 1) / 2;
  for (int v : kList)
    if (v >= k) return v;
  return -1;
}

// Per-call counters (one buffer, zeroed by the partition kernel):
//   [0, nl)            pairs per leaf (strided, kCounterStride)
//   [stats, +32)       stats words (SelectArgs::overflow and the work-list totals)
struct CounterLayout {
  uint32_t stats, words;
  explicit CounterLayout(int nl) {
    stats = uint32_t(nl) * smx::kCounterStride;
    words = stats + 32u;
  }
};

struct Workspace {
  // allocated sizes, each the largest of its own quantity over past calls
  // (never a product of per-dimension maxima: nq = 10^4 at L = 20 followed
  // by nq = 10 at L = 2000 keeps 2 * 10^5 pairs, not 2 * 10^7)
  int nq = 0, dim = 0;              // nq: queries of one sub-batch (RunSearch)
  int sq = 0;                       // staged queries / outputs (whole host batch)
  size_t pairs = 0, cand_words = 0, out_words = 0;
  uint64_t gen = 0;                 // bumped on every (re)allocation
  uint32_t max_items = 0;
  uint32_t cap = 0;                 // this call's list capacity = its [nq][cap] stride
  float* queries = nullptr;
  int32_t* topl_leaf = nullptr;
  float* topl_dist = nullptr;
  float* scores = nullptr;          // [nq][nl] partition scores
  int8_t* lut = nullptr;
  float* mult = nullptr;
  float* inv = nullptr;
  uint32_t* counters = nullptr;     // see CounterLayout
  uint32_t* leaf_pair = nullptr;    // [nl][nq] each leaf's pairs by rank (top-L kernel)
  smx::ItemLane* pair_rec = nullptr;   // [nq*L] every pair's record (seed kernel)
  uint32_t* leaf_item0 = nullptr;   // [nl] each leaf's first work item
  smx::WorkItem* work = nullptr;    // [max_items]
  uint4* wave_start = nullptr;      // [grid] each scan wave's static share
  uint32_t* pos_unit0 = nullptr;    // [nl+1] work units before each leaf (work order)
  uint32_t* gunits = nullptr;       // [16] the XCD groups' unit boundaries
  unsigned long long* wl_part = nullptr;   // [kWorklistPartWords * ceil(nl / 256)] block sums
  uint64_t* tau = nullptr;          // [nq]
  uint64_t* cand = nullptr;         // [nq][cap]
  uint32_t* cand_count = nullptr;   // [nq] strided (kCounterStride)
  uint32_t* out_idx = nullptr;
  float* out_dist = nullptr;
  int32_t* out_count = nullptr;
  smx::ShardEntry* merge_scratch[2] = {nullptr, nullptr};   // the wide merge's rounds
  size_t merge_entries = 0;

  void Release() {
    DFree(queries); DFree(topl_leaf); DFree(topl_dist); DFree(scores); DFree(lut); DFree(mult);
    DFree(inv);
    DFree(counters); DFree(leaf_pair); DFree(pair_rec); DFree(leaf_item0); DFree(wave_start);
    DFree(pos_unit0); DFree(gunits); DFree(wl_part);
    DFree(work); DFree(tau); DFree(cand); DFree(cand_count); DFree(out_idx);
    DFree(out_dist);
    DFree(out_count);
    DFree(merge_scratch[0]);
    DFree(merge_scratch[1]);
    merge_entries = 0;
    nq = sq = dim = 0;
    pairs = cand_words = out_words = 0;
    cap = max_items = 0;
  }
};

// One stream's share of a handle: its per-call buffers and what orders
// them.  Calls on different streams use different slots, so batches issued on
// two streams run concurrently on the device (one batch's latency-bound
// front end and select beside the other's scan; see DESIGN.md "Batches in
// flight"); calls on one stream are ordered by that stream.  A slot reused
// from another stream (more streams than kMaxStreamSlots) first waits for
// its previous stream's work.
struct StreamSlot {
  hipStream_t key = nullptr;          // the stream this slot serves
  Workspace ws;
  hipGraphExec_t graph_exec = nullptr;
  uint64_t graph_key[16] = {};
  hipEvent_t done_ev = nullptr;       // cross-stream ordering (recorded at a stream switch)
  hipStream_t last_stream = nullptr;
  hipStream_t side = nullptr;         // the fork/join branch (SMX_SERIAL_WORKLIST=0)
  hipEvent_t fork_ev = nullptr, join_ev = nullptr;
};
constexpr int kMaxStreamSlots = 4;

// The slot's work must have finished (the callers synchronise the device or
// the slot's last stream first): no caller stream is touched here, since the
// caller may already have destroyed it.
void DestroySlot(StreamSlot* sl) {
  if (sl->graph_exec) (void)hipGraphExecDestroy(sl->graph_exec);
  sl->ws.Release();
  if (sl->done_ev) (void)hipEventDestroy(sl->done_ev);
  if (sl->fork_ev) (void)hipEventDestroy(sl->fork_ev);
  if (sl->join_ev) (void)hipEventDestroy(sl->join_ev);
  if (sl->side) (void)hipStreamDestroy(sl->side);
  delete sl;
}

}  // namespace

struct smx_index {
  smx::DeviceIndex ix;
  int device = 0;
  hipStream_t stream = nullptr;
  mutable std::mutex mu;            // one call at a time per handle (smx_get_timings too)
  std::vector<StreamSlot*> slots;   // one per stream the handle has searched on
  uint32_t cap_per_query = 0;      // candidate list capacity; 0 = sized per call (AutoCap)
  int seed_leaves = 4;
  // rows the seed scores per query (SMX_SEED_ROWS): 2048 of at most 4096.
  // The seed's score loop streams its rows' codes from the fabric (98 MB per
  // glove batch at 4096 rows, 6.3 TB/s: PMC, profiles/r06/pmc_seed.txt), so
  // with batches in flight it competes with the other batches' scans; same
  // box (profiles/r06/ab/seed_rows.txt), glove in flight at L = 20 / 100:
  // 14.89 / 9.31 M QPS at 2048 rows against 13.73 / 8.98 M at 4096 (one batch
  // alone: 10.22 / 6.97 against 10.69 / 7.27 M -- the tighter thresholds of
  // 4096 rows shorten the scan: 40.2 -> 33.1 us at L = 20).
  uint32_t seed_rows = 2048;
  uint64_t leaf_slot_budget = 1ull << 26;   // see kLeafSlotBudget
  int scan_variant = 0;            // see smx::LaunchScan
  int fused_worklist_leaves = smx::kFusedWorklistLeaves;   // 0: always the side stream
  uint32_t chunk_tiles = 20;       // tiles per work item (tools/tune.py: 16-20 best at glove)
  // a leaf's remainder of <= 16 queries on the 16-slot scan path
  // (v_smfmac_i32_16x16x128_i8); SMX_NARROW=0 keeps every query tile 32 wide
  bool narrow_tiles = true;
  bool narrow_only = false;        // SMX_NARROW=2: 16-slot tiles only whatever the density
  // above fused_worklist_leaves: the work-list launches on this stream before
  // the seed (true; SMX_SERIAL_WORKLIST=0: on the side stream beside it --
  // same box A/B, configs[3]/[4]: 0.578 vs 0.584 and 1.478 vs 1.495 ms/step)
  bool serial_worklist = true;
  int grid = 0;                    // scan grid: resident one-wave workgroups (occupancy API)
  int cus = 0;                     // compute units of the device
  bool profiling = false;          // mode 1: per-call stage timings (synchronous calls)
  // mode 2: an event pair around every scan launch, no synchronisation
  // (kScanLog pairs, the latest kept; read by smx_get_timings)
  bool scan_log = false;
  std::vector<hipEvent_t> scan_ev;
  uint64_t scan_logged = 0;
  bool use_graph = false;          // SMX_GRAPH=1: replay the pipeline as a hipGraph
  uint64_t ws_generation = 0;
  uint32_t* host_stats = nullptr;  // pinned copy of the stats words
  smx_timings timings{};
  hipEvent_t ev[16] = {};
  // scan variant 8 (diagnostics): per-item stamps, dumped to $SMX_STAMPS
  unsigned long long* stamps = nullptr;
  uint32_t* stamp_count = nullptr;
};

namespace {

constexpr int GraphKeyWords = 16;
constexpr uint64_t kScanLog = 4096;   // profiling mode 2: scan event pairs kept

int UploadIndex(const smx_index_desc* d, smx_index* h) {
  smx::DeviceIndex& ix = h->ix;
  ix.metric = d->metric;
  ix.dim = d->dim;
  ix.nl = d->num_leaves;
  ix.nb = d->num_blocks;
  ix.dpb = d->dims_per_block;
  ix.residual = d->residual ? 1 : 0;
  ix.num_datapoints = d->num_datapoints;
  ix.spill = d->spilling_overretrieve_factor > 0 ? d->spilling_overretrieve_factor : 2.0f;
  ix.ksteps = EffectiveKSteps(ix.nb);
  ix.lane_bytes = smx::LaneBytes(ix.ksteps);
  const int nl = ix.nl, dim = ix.dim, nb = ix.nb, K = ix.ksteps, W = ix.lane_bytes;
  const uint64_t M = d->leaf_offsets[nl];
  ix.num_members = M;

  // Per-leaf sizes, tile offsets, max leaf, disjointness.
  std::vector<uint32_t> size(nl);
  std::vector<uint64_t> toff(nl + 1, 0);
  for (int l = 0; l < nl; ++l) {
    const uint64_t n = d->leaf_offsets[l + 1] - d->leaf_offsets[l];
    size[l] = uint32_t(n);
    ix.max_leaf = std::max<uint32_t>(ix.max_leaf, uint32_t(n));
    toff[l + 1] = toff[l] + (n + 31) / 32;
  }
  ix.num_tiles = toff[nl];
  ix.disjoint = (M == d->num_datapoints);
  if (ix.disjoint) {
    std::vector<uint8_t> seen(d->num_datapoints, 0);
    for (uint64_t i = 0; i < M; ++i) {
      const uint32_t g = d->leaf_members[i];
      if (seen[g]) { ix.disjoint = false; break; }
      seen[g] = 1;
    }
  }
  // Global top-N shift (tree_ah_hybrid_residual.h:234-247).
  ix.shift = 0;
  if (ix.residual && nl > 1) {
    const int inner = 32 - Log2Ceil(uint32_t(nl));
    if (uint64_t(ix.max_leaf) <= (1ull << inner)) ix.shift = inner;
  }
  if (d->is_shard) {
    // a shard keeps the whole index's tie semantics and spill setting
    if (d->global_topn_shift < 0 || d->global_topn_shift > 31)
      return Fail(SMX_INVALID_ARGUMENT, "global_topn_shift out of range");
    if (d->global_topn_shift > 0 && (!ix.residual || nl <= 1))
      return Fail(SMX_INVALID_ARGUMENT, "global top-N shift needs a residual multi-leaf index");
    ix.shift = d->global_topn_shift;
    ix.disjoint = !d->global_spilled;
    if (!d->leaf_row_base) return Fail(SMX_INVALID_ARGUMENT, "a shard needs leaf_row_base");
    for (int l = 0; l < nl; ++l)
      if (ix.shift > 0 && uint64_t(d->leaf_row_base[l]) + size[l] > (1ull << ix.shift))
        return Fail(SMX_INVALID_ARGUMENT, "shard rows exceed the whole index's leaf range");
  }

  // Code tiles: lane l = h*32 + r of tile j of a leaf holds, as nibbles
  // s = 0..K-1 (two per byte, then EncodeCodePair), the codes of datapoint
  // 32j + r for blocks 2s + h.  Missing datapoints / blocks are code 0
  // against a zero LUT row or are masked in the epilogue.
  std::vector<uint8_t> tiles(size_t(ix.num_tiles) * 64 * W, 0);
  for (int l = 0; l < nl; ++l) {
    const uint64_t beg = d->leaf_offsets[l];
    const uint32_t n = size[l];
    for (uint32_t dp = 0; dp < n; ++dp) {
      const uint8_t* code = d->member_codes + (beg + dp) * nb;
      const uint64_t tile = toff[l] + dp / 32;
      const uint32_t r = dp % 32;
      for (int b = 0; b < nb; ++b) {
        const int h = b & 1, s = b >> 1;
        uint8_t* lane = &tiles[(tile * 64 + size_t(h) * 32 + r) * W];
        lane[s >> 1] |= uint8_t((code[b] & 15) << ((s & 1) * 4));
      }
    }
  }
  for (auto& by : tiles) by = uint8_t(smx::EncodeCodePair(by & 15u, by >> 4));
  (void)K;

  // Transposed centers and squared norms (A.10 database side).
  std::vector<float> ct(size_t(dim) * nl);
  std::vector<float> cn(nl);
  for (int l = 0; l < nl; ++l) {
    float acc = 0.0f;
    for (int k = 0; k < dim; ++k) {
      const float v = d->centers[size_t(l) * dim + k];
      ct[size_t(k) * nl + l] = v;
      acc = std::fma(-v, v, acc);
    }
    cn[l] = acc * -1.0f;
  }
  int rc;
  if ((rc = DAlloc(&ix.centers, size_t(nl) * dim)) ||
      (rc = DAlloc(&ix.centers_t, size_t(nl) * dim)) || (rc = DAlloc(&ix.cnorm, nl)) ||
      (rc = DAlloc(&ix.codebook, size_t(nb) * 16 * ix.dpb)) ||
      (rc = DAlloc(&ix.tiles, tiles.size())) || (rc = DAlloc(&ix.tile_off, nl + 1)) ||
      (rc = DAlloc(&ix.leaf_size, nl)) || (rc = DAlloc(&ix.member_off, nl + 1)) ||
      (rc = DAlloc(&ix.members, M)) || (rc = DAlloc(&ix.leaf_order, nl)))
    return rc;
  if (d->dataset && (rc = DAlloc(&ix.dataset, size_t(d->num_datapoints) * dim))) return rc;
  if (d->is_shard) {
    if ((rc = DAlloc(&ix.row_base, nl))) return rc;
    SMX_HIP(hipMemcpy(ix.row_base, d->leaf_row_base, 4 * nl, hipMemcpyHostToDevice));
    if (d->member_rows && M) {
      if ((rc = DAlloc(&ix.member_rows, size_t(M) * dim))) return rc;
      SMX_HIP(hipMemcpy(ix.member_rows, d->member_rows, sizeof(float) * size_t(M) * dim,
                        hipMemcpyHostToDevice));
      // global id -> member slot, for the candidates known by global id only:
      // ties by global id (shift 0), and a spilled shard's candidates after
      // the block select's SOAR dedupe.  A disjoint shard with the global
      // top-N finds every row from its packed tie (no table: 4 GB per rank at
      // the Deep1B shape).  A SOAR id held twice keeps either slot: same row.
      if (ix.shift == 0 || !ix.disjoint) {
        if ((rc = DAlloc(&ix.row_of, size_t(d->num_datapoints)))) return rc;
        SMX_HIP(hipMemset(ix.row_of, 0xFF, sizeof(uint32_t) * size_t(d->num_datapoints)));
      }
    }
  }
  SMX_HIP(hipMemcpy(ix.centers, d->centers, sizeof(float) * nl * dim, hipMemcpyHostToDevice));
  SMX_HIP(hipMemcpy(ix.centers_t, ct.data(), sizeof(float) * nl * dim, hipMemcpyHostToDevice));
  SMX_HIP(hipMemcpy(ix.cnorm, cn.data(), sizeof(float) * nl, hipMemcpyHostToDevice));
  SMX_HIP(hipMemcpy(ix.codebook, d->codebook, sizeof(float) * nb * 16 * ix.dpb, hipMemcpyHostToDevice));
  if (!tiles.empty())
    SMX_HIP(hipMemcpy(ix.tiles, tiles.data(), tiles.size(), hipMemcpyHostToDevice));
  SMX_HIP(hipMemcpy(ix.tile_off, toff.data(), 8 * (nl + 1), hipMemcpyHostToDevice));
  SMX_HIP(hipMemcpy(ix.leaf_size, size.data(), 4 * nl, hipMemcpyHostToDevice));
  SMX_HIP(hipMemcpy(ix.member_off, d->leaf_offsets, 8 * (nl + 1), hipMemcpyHostToDevice));
  if (M) SMX_HIP(hipMemcpy(ix.members, d->leaf_members, 4 * M, hipMemcpyHostToDevice));
  if (ix.row_of) {
    SMX_HIP(smx::LaunchRowOf(ix.members, M, ix.row_of, nullptr));
    SMX_HIP(hipDeviceSynchronize());
  }
  // Work order: the leaves by descending size dealt to the 8 XCD groups in a
  // snake (0..7, 7..0, ...), each group's leaves contiguous and largest
  // first.  The worklist cuts the order into 8 groups of equal MFMA work, so
  // every group gets the same mix of large and small leaves (large leaves
  // carry more queries near them and more threshold hits per tile: groups of
  // consecutive sizes finished up to 20% apart).
  std::vector<uint32_t> by_size(nl);
  for (int l = 0; l < nl; ++l) by_size[l] = uint32_t(l);
  std::stable_sort(by_size.begin(), by_size.end(),
                   [&](uint32_t a, uint32_t b) { return size[a] > size[b]; });
  std::vector<uint32_t> order;
  order.reserve(nl);
  for (int g = 0; g < smx::kWorkGroups; ++g)
    for (int p = 0; p < nl; ++p) {
      const int r = p / smx::kWorkGroups, i = p % smx::kWorkGroups;
      if ((r % 2 == 0 ? i : smx::kWorkGroups - 1 - i) == g) order.push_back(by_size[p]);
    }
  SMX_HIP(hipMemcpy(ix.leaf_order, order.data(), 4 * nl, hipMemcpyHostToDevice));
  if (d->dataset)
    SMX_HIP(hipMemcpy(ix.dataset, d->dataset, sizeof(float) * size_t(d->num_datapoints) * dim,
                      hipMemcpyHostToDevice));
  return SMX_OK;
}

void FreeIndex(smx::DeviceIndex& ix) {
  DFree(ix.centers); DFree(ix.centers_t); DFree(ix.cnorm); DFree(ix.codebook);
  DFree(ix.tiles); DFree(ix.tile_off); DFree(ix.leaf_size); DFree(ix.member_off);
  DFree(ix.members); DFree(ix.leaf_order); DFree(ix.dataset); DFree(ix.row_base);
  DFree(ix.member_rows); DFree(ix.row_of);
}

int ValidateDesc(const smx_index_desc* d) {
  if (!d) return Fail(SMX_INVALID_ARGUMENT, "null index description");
  if (d->metric != SMX_METRIC_DOT && d->metric != SMX_METRIC_SQUARED_L2)
    return Fail(SMX_INVALID_ARGUMENT, "metric must be dot product or squared L2");
  if (d->dim <= 0 || d->num_leaves <= 0 || d->num_blocks <= 0 || d->dims_per_block <= 0)
    return Fail(SMX_INVALID_ARGUMENT, "dim, num_leaves, num_blocks, dims_per_block must be > 0");
  if (d->num_blocks > smx::kMaxBlocks)
    return Fail(SMX_INVALID_ARGUMENT, "LUT16 path supports at most 64 AH blocks");
  const int last = d->dim - d->dims_per_block * (d->num_blocks - 1);
  if (last <= 0 || last > d->dims_per_block)
    return Fail(SMX_INVALID_ARGUMENT, "num_blocks x dims_per_block does not tile dim");
  if (!d->centers || !d->codebook || !d->leaf_offsets)
    return Fail(SMX_INVALID_ARGUMENT, "centers, codebook and leaf_offsets are required");
  if (d->leaf_offsets[0] != 0) return Fail(SMX_INVALID_ARGUMENT, "leaf_offsets[0] must be 0");
  for (int l = 0; l < d->num_leaves; ++l)
    if (d->leaf_offsets[l + 1] < d->leaf_offsets[l])
      return Fail(SMX_INVALID_ARGUMENT, "leaf_offsets must be non-decreasing");
  const uint64_t M = d->leaf_offsets[d->num_leaves];
  if (M && (!d->leaf_members || !d->member_codes))
    return Fail(SMX_INVALID_ARGUMENT, "leaf_members and member_codes are required");
  if (M > 0xFFFFFFFFull) return Fail(SMX_INVALID_ARGUMENT, "too many members for 32-bit ids");
  for (uint64_t i = 0; i < M; ++i) {
    if (d->leaf_members[i] >= d->num_datapoints)
      return Fail(SMX_INVALID_ARGUMENT, "leaf member id out of range");
  }
  for (uint64_t i = 0; i < M * uint64_t(d->num_blocks); ++i)
    if (d->member_codes[i] > 15) return Fail(SMX_INVALID_ARGUMENT, "LUT16 codes must be < 16");
  return SMX_OK;
}

// Candidate list capacity per query when none is set.  The seed threshold
// is the exact k'-th key over `seed` of the query's L leaves, so about
// k' * L / seed candidates pass it; an overflowing list costs its select
// block a rescan of the query's L leaves (VALU), so the list is sized 8x
// that expectation (Deep1B shape, L = 400 of 50000 leaves: 10^4 expected ->
// 2^17), at least 4096.  The rank select (k' <= 256) reads the list from
// global memory; the LDS select of larger k' bounds it to 8192.
uint32_t AutoCap(int L, int kk, int seed) {
  if (seed <= 0 || kk > 256) return 4096;   // 256 = kSelMax of the rank select
  const uint64_t want = 8ull * uint64_t(kk) * uint64_t(L) / uint64_t(seed);
  uint32_t cap = 4096;
  while (cap < want && cap < (1u << 17)) cap <<= 1;
  return cap;
}

// Work items the workspace holds for `pairs` (query, leaf) pairs: one per
// (leaf, query tile, chunk of >= 8 tiles).  A leaf with c queries has at most
// ceil(c / 16) query tiles (the 16-slot-only mode, kNarrowOnly: every tile 16
// wide; the other modes use fewer), so sum_leaf ceil(c / 16) <= pairs / 16 +
// nl; a leaf of n rows has ceil(ceil(n / 32) / chunk_tiles) chunks, at most
// the bound below for any chunk_tiles smx_set_tuning accepts (>= 8).
// (tests/worklist_model.py: max_items, asserted against every built list)
uint32_t MaxItems(const smx::DeviceIndex& ix, size_t pairs) {
  const uint32_t chunks = (uint32_t((ix.max_leaf + 31) / 32) + 7) / 8 + 1;  // chunk >= 8
  return uint32_t((pairs / smx::kNarrowSlots + ix.nl + 1) * chunks);
}

// The slot of stream s: its own, a new one (up to kMaxStreamSlots), or else
// the least recently created one, which then waits for its last stream.
int SlotFor(smx_index* h, hipStream_t s, StreamSlot** out) {
  for (StreamSlot* sl : h->slots)
    if (sl->key == s) {
      *out = sl;
      return SMX_OK;
    }
  StreamSlot* sl = nullptr;
  if (int(h->slots.size()) < kMaxStreamSlots) {
    sl = new StreamSlot;
    if (hipEventCreateWithFlags(&sl->done_ev, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&sl->fork_ev, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&sl->join_ev, hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithFlags(&sl->side, hipStreamNonBlocking) != hipSuccess) {
      DestroySlot(sl);
      return Fail(SMX_DEVICE_ERROR, "stream slot: hipEventCreate / hipStreamCreate failed");
    }
    sl->last_stream = s;
    h->slots.push_back(sl);
  } else {
    sl = h->slots.front();   // rotated to the back: reused in creation order
    h->slots.erase(h->slots.begin());
    h->slots.push_back(sl);
  }
  sl->key = s;
  *out = sl;
  return SMX_OK;
}

// Leaf-slot words (`leaf_pair`, nl x queries) one sub-batch may use: 2^26
// words = 256 MB per stream slot, and nl x queries < 2^32 (32-bit slot
// indices).  At the Deep1B shape (50000 leaves) that is 1342 queries per
// sub-batch; every BASELINE batch of 1000 runs whole.
// (SMX_LEAF_SLOT_BUDGET at creation lowers it: the tests' sub-batch split)
constexpr uint64_t kLeafSlotBudget = 1ull << 26;

int SubBatchQueries(const smx_index* h) {
  const uint64_t q = h->leaf_slot_budget / uint64_t(std::max(h->ix.nl, 1));
  return int(std::max<uint64_t>(1, std::min<uint64_t>(q, 1u << 30)));
}

int EnsureWorkspace(smx_index* h, StreamSlot* sl, int nq, int L, int kk, int width) {
  Workspace& w = sl->ws;
  const smx::DeviceIndex& ix = h->ix;
  // cap >= 2 k': when a list overflows, its k'-th stored key is strictly
  // below the threshold (keys are unique and all <= it), so every
  // tightening pass drops at least cap - k' keys.  The lists of a call are
  // [nq][cap] with this call's own cap (the kernels' stride), inside a
  // buffer that may be larger.
  const uint32_t base = h->cap_per_query ? h->cap_per_query
                                         : AutoCap(L, kk, std::min(h->seed_leaves, L));
  const uint32_t cap = std::max<uint32_t>(base, 2u * uint32_t(kk));
  // per-sub-batch buffers for at most SubBatchQueries queries; the staged
  // queries and outputs (host-buffer entry points) for the whole batch
  const int sq = nq;
  nq = std::min(nq, SubBatchQueries(h));
  const size_t pairs = size_t(nq) * L;
  const size_t cand_words = size_t(nq) * cap, out_words = size_t(sq) * width;
  if (nq <= w.nq && sq <= w.sq && pairs <= w.pairs && cand_words <= w.cand_words &&
      out_words <= w.out_words && ix.dim == w.dim) {
    w.cap = cap;
    return SMX_OK;
  }
  // grow each quantity to cover this call and the earlier ones, so that
  // alternating shapes (leaves_to_search sweeps) settle after one growth
  // (hipFree synchronises the device)
  const int anq = std::max(nq, w.nq), asq = std::max(sq, w.sq);
  const size_t apairs = std::max(pairs, w.pairs);
  const size_t acand = std::max(cand_words, w.cand_words);
  const size_t aout = std::max(out_words, w.out_words);
  w.Release();
  const int nl = ix.nl;
  const uint32_t max_items = MaxItems(ix, apairs);
  int rc;
  if ((rc = DAlloc(&w.queries, size_t(asq) * ix.dim)) || (rc = DAlloc(&w.topl_leaf, apairs)) ||
      (rc = DAlloc(&w.topl_dist, apairs)) || (rc = DAlloc(&w.scores, size_t(anq) * nl)) ||
      (rc = DAlloc(&w.lut, size_t(anq) * smx::LutRows(ix.ksteps) * 16)) || (rc = DAlloc(&w.mult, anq)) ||
      (rc = DAlloc(&w.inv, anq)) || (rc = DAlloc(&w.counters, CounterLayout(nl).words)) ||
      (rc = DAlloc(&w.leaf_pair, size_t(nl) * size_t(anq))) ||
      (rc = DAlloc(&w.pair_rec, apairs)) || (rc = DAlloc(&w.leaf_item0, size_t(nl))) ||
      (rc = DAlloc(&w.wave_start, size_t(std::max(h->grid, 1)))) ||
      (rc = DAlloc(&w.pos_unit0, size_t(nl + 1))) || (rc = DAlloc(&w.gunits, 16)) ||
      (rc = DAlloc(&w.wl_part, size_t(smx::kWorklistPartWords) * ((nl + 255) / 256))) ||
      (rc = DAlloc(&w.work, max_items)) || (rc = DAlloc(&w.tau, anq)) ||
      (rc = DAlloc(&w.cand, acand)) ||
      (rc = DAlloc(&w.cand_count, size_t(anq) * smx::kCounterStride)) ||
      (rc = DAlloc(&w.out_idx, aout)) || (rc = DAlloc(&w.out_dist, aout)) ||
      (rc = DAlloc(&w.out_count, asq))) {
    w.Release();
    return rc;
  }
  w.nq = anq;
  w.sq = asq;
  w.pairs = apairs;
  w.cand_words = acand;
  w.out_words = aout;
  w.dim = ix.dim;
  w.gen = ++h->ws_generation;
  w.cap = cap;
  w.max_items = max_items;
  return SMX_OK;
}

int32_t SpillK(const smx::DeviceIndex& ix, int32_t k) {
  if (ix.disjoint) return k;
  const double r = double(k) * double(ix.spill);
  return r > 2147483647.0 ? 2147483647 : int32_t(r);
}

void Mark(smx_index* h, int i, hipStream_t s) {
  if (h->profiling) (void)hipEventRecord(h->ev[i], s);
}

float Elapsed(smx_index* h, int a, int b) {
  float ms = 0.0f;
  if (hipEventElapsedTime(&ms, h->ev[a], h->ev[b]) != hipSuccess) {
    (void)hipGetLastError();   // an unrecorded pair: not sticky for the next launch check
    return 0.0f;
  }
  return ms;
}

// The search pipeline for one sub-batch (RunSearch below splits a batch).
// queries: device [nq][dim].  pre_only: stop before reorder and output the
// pre-reorder set (width pre_nn).
int RunSearchChunk(smx_index* h, const float* queries, int nq, int L, int pre_nn, int final_nn,
                   bool reorder, bool pre_only, uint32_t* out_idx, float* out_dist,
                   int32_t* out_count, hipStream_t s, smx::ShardEntry* shard_out, bool single) {
  smx::DeviceIndex& ix = h->ix;
  if (nq == 0) return SMX_OK;
  L = std::min(L, ix.nl);
  const int pnn = reorder ? pre_nn : final_nn;
  const int kk = std::max(1, SpillK(ix, pnn));
  const int width = shard_out ? 1 : pre_only ? pnn : final_nn;
  if (uint64_t(ix.nl) * uint64_t(nq) > 0xFFFFFFFFull)
    return Fail(SMX_INTERNAL, "sub-batch above the leaf-slot bound (RunSearch splits batches)");
  StreamSlot* sl = nullptr;
  int rc = SlotFor(h, s, &sl);
  if (rc) return rc;
  if ((rc = EnsureWorkspace(h, sl, nq, L, kk, width))) return rc;
  Workspace& w = sl->ws;
  const int nl = ix.nl;
  const CounterLayout lay(nl);
  uint32_t* cnt = w.counters;
  // stats: [0] overflow flag [1] max overflowing count [2] max count
  //        [3] pairs [4] work items [5] item-tiles (MFMA tiles of the scan)
  //        [6..7] code bytes (u64) [8] survivors summed over queries [9] fallbacks
  //        [10] rescanned queries [11] rescan rounds [12] 16-slot tiles
  uint32_t* stats = w.counters + lay.stats;
  unsigned long long* code_bytes = reinterpret_cast<unsigned long long*>(stats + 6);
  const int seed = std::min(h->seed_leaves, L);

  const int variant = h->scan_variant;
  // 16-slot tiles only (lut16_scan_kernel<K, 0, kNarrowOnly>) where leaves
  // see fewer than 32 queries on average (configs 3/4: ~8 per leaf; glove's
  // recall gate L = 20: 20 per leaf, scan 38.2 -> 33.6 us); 32-slot tiles at
  // glove's L = 100 (100 per leaf) and SIFT's (50 per leaf), where the wide
  // kernel is faster (106 vs 115 us on SIFT).  SMX_NARROW=2 forces 16-slot
  // tiles, SMX_NARROW=0 32-slot tiles (the tests run every mode).
  const uint64_t qpl_x = uint64_t(nq) * uint64_t(L);   // queries per leaf x nl
  uint32_t narrow = 0;
  if (h->narrow_tiles &&
      (h->narrow_only || qpl_x < uint64_t(smx::kNarrowQueriesPerLeaf) * uint64_t(ix.nl)))
    narrow = smx::kNarrowOnly;
  smx::Bounds bd;
  bd.nq = uint32_t(nq);
  bd.items = w.max_items;
  bd.grid = uint32_t(std::max(h->grid, 1));
  bd.nl = uint32_t(nl);
  bd.datapoints = ix.num_datapoints;
  bd.members = ix.num_members;
  bd.tiles = ix.num_tiles;
  bd.recs = uint32_t(nl) * uint32_t(nq);
  bd.pairs = uint32_t(nq) * uint32_t(L);
  smx::SeedArgs sa{};
  sa.bd = bd;
  sa.topl_leaf = w.topl_leaf;
  sa.topl_dist = w.topl_dist;
  sa.pair_rec = w.pair_rec;
  sa.nb = ix.nb;
  sa.lut = w.lut;
  sa.inv = w.inv;
  sa.tiles = ix.tiles;
  sa.tile_off = ix.tile_off;
  sa.leaf_size = ix.leaf_size;
  sa.tau_key = w.tau;
  sa.L = L;
  sa.seed = seed;
  sa.seed_rows = int(std::min<uint32_t>(h->seed_rows, uint32_t(smx::kSeedKeys)));
  sa.kk = kk;
  sa.nl = nl;
  sa.residual = ix.residual;

  smx::ScanArgs a{};
  a.bd = bd;
  a.tiles = ix.tiles;
  a.members = ix.members;
  a.lut = w.lut;
  a.inv = w.inv;
  a.work = w.work;
  a.leaf_pair = w.leaf_pair;
  a.pair_rec = w.pair_rec;
  a.chunk_tiles = h->chunk_tiles;
  a.wave_start = w.wave_start;
  a.num_items = w.max_items;   // bound of the one-ahead descriptor prefetch
  a.tau_key = w.tau;
  a.cand = w.cand;
  a.cand_count = w.cand_count;
  constexpr uint32_t kStampCap = 1u << 16;
  if (variant == 8 && !h->stamps) {
    int rc2;
    if ((rc2 = DAlloc(&h->stamps, size_t(kStampCap) * 8)) || (rc2 = DAlloc(&h->stamp_count, 1)))
      return rc2;
  }
  a.stamps = h->stamps;
  a.stamp_count = h->stamp_count;
  a.stamp_cap = kStampCap;
  if (variant == 8) SMX_HIP(hipMemsetAsync(h->stamp_count, 0, 4, s));
  a.cap = w.cap;
  a.nl = nl;
  a.nb = ix.nb;
  a.shift = ix.shift;

  smx::SelectArgs sel{};
  sel.bd = bd;
  sel.cand = w.cand;
  sel.cand_count = w.cand_count;
  sel.cap = w.cap;
  sel.kk = kk;
  sel.pre_nn = pnn;
  sel.final_nn = final_nn;
  sel.reorder = reorder ? 1 : 0;
  sel.disjoint = ix.disjoint ? 1 : 0;
  sel.pre_only = pre_only ? 1 : 0;
  sel.shift = ix.shift;
  sel.metric = ix.metric;
  sel.dim = ix.dim;
  sel.member_off = ix.member_off;
  sel.members = ix.members;
  sel.dataset = ix.dataset;
  sel.queries = queries;
  sel.out_idx = out_idx;
  sel.out_dist = out_dist;
  sel.out_count = out_count;
  sel.out_width = width;
  sel.overflow = stats;
  sel.stats = h->profiling ? 1 : 0;
  smx::RescanArgs& ra = sel.rescan;
  ra.bd = bd;
  ra.topl_leaf = w.topl_leaf;
  ra.topl_dist = w.topl_dist;
  ra.L = L;
  ra.residual = ix.residual;
  ra.ksteps = ix.ksteps;
  ra.lut = w.lut;
  ra.inv = w.inv;
  ra.tiles = ix.tiles;
  ra.tile_off = ix.tile_off;
  ra.leaf_size = ix.leaf_size;
  ra.members = ix.members;
  ra.member_off = ix.member_off;
  ra.shift = ix.shift;
  ra.cand = w.cand;
  ra.cand_count = w.cand_count;
  ra.tau_key = w.tau;
  ra.cap = w.cap;
  ra.kk = kk;
  ra.stats = stats;
  sel.shard_out = shard_out;
  sel.row_base = ix.row_base;
  sel.member_rows = ix.member_rows;
  sel.row_of = ix.row_of;
  if (!smx::FinalSelectFits(sel))
    return Fail(SMX_INVALID_ARGUMENT,
                "the candidate list capacity, k' and dim exceed the final selection's 160 KiB of "
                "LDS (lower candidates_per_query or pre_reorder_num_neighbors)");

  // First pass: everything up to the stats copy.  Replayed as a captured
  // hipGraph when the call shape, buffers and stream repeat (one launch
  // instead of ~20, no per-kernel host overhead); eager otherwise.
  bool seed_dispatch_ev = false;   // the seed timed by its own dispatch (fused work list)
  auto first_pass = [&]() -> int {
    Mark(h, 0, s);
    // front end: state reset, partition scores, top-L + ranks + LUTs
    smx::FrontArgs f;
    f.init.counters = w.counters;
    f.init.n_counters = uint32_t(nl);   // the pair counters
    f.init.stats = stats;
    f.init.n_stats = 32u;
    f.init.cand_count = w.cand_count;
    f.init.n_cand = uint32_t(nq);
    f.init.tau = w.tau;
    f.init.n_tau = uint32_t(nq);
    f.leaf_count = cnt;
    f.leaf_pair = w.leaf_pair;
    f.slot_stride = uint32_t(nq);
    f.lut = w.lut;
    f.mult = w.mult;
    f.inv = w.inv;
    f.one_to_many = single ? 1 : 0;
    SMX_HIP(smx::LaunchPartitionTopL(ix, queries, nq, L, w.topl_leaf, w.topl_dist, w.scores, s, &f));
    Mark(h, 1, s);
    if (ix.nl <= h->fused_worklist_leaves) {
      // the work list is built by extra blocks of the seed launch (one
      // stream: a fork/join costs 5-10 us per cross-queue edge)
      const smx::WorklistArgs wla = smx::MakeWorklistArgs(
          ix, cnt, w.work, w.leaf_item0, w.pos_unit0, w.gunits, uint32_t(nq), w.wave_start, h->grid,
          stats + 3, code_bytes, h->chunk_tiles, narrow, bd);
      Mark(h, 3, s);
      SMX_HIP(smx::LaunchSeed(ix, sa, nq, s, &wla, h->profiling ? h->ev[8] : nullptr,
                              h->profiling ? h->ev[9] : nullptr));
      Mark(h, 4, s);
      seed_dispatch_ev = h->profiling;
    } else if (h->serial_worklist) {
      // the work-list launches, then the seed, on one stream: beside the
      // seed's blocks (which fill every CU) the side-stream launches are
      // starved until the seed drains
      SMX_HIP(smx::LaunchWorklist(ix, cnt, w.work, w.leaf_item0, w.pos_unit0, w.gunits,
                                  uint32_t(nq), w.wave_start, h->grid, stats + 3, code_bytes,
                                  h->chunk_tiles, narrow, w.wl_part, bd, s));
      Mark(h, 3, s);
      SMX_HIP(smx::LaunchSeed(ix, sa, nq, s));
      Mark(h, 4, s);
    } else {
      // Fork.  Side stream: the work list (and the empty slots' records);
      // this stream: the seed thresholds.  Write sets ("Two
      // streams"): side = leaf_item0, pos_unit0, gunits, work, wave_start,
      // stats[3..7]; seed = tau, pair_rec.  Both only read the
      // front end's outputs, written before the fork; the per-call state
      // reset happens in the partition kernel, before the fork as well.
      // The seed (the longer branch) is captured first, so that a replayed
      // graph keeps it on the launch queue with the kernels before and after
      // it; the shorter work-list branch pays the cross-queue edges.
      SMX_HIP(hipEventRecord(sl->fork_ev, s));
      SMX_HIP(smx::LaunchSeed(ix, sa, nq, s));
      Mark(h, 4, s);
      SMX_HIP(hipStreamWaitEvent(sl->side, sl->fork_ev, 0));
      SMX_HIP(smx::LaunchWorklist(ix, cnt, w.work, w.leaf_item0, w.pos_unit0, w.gunits,
                                  uint32_t(nq), w.wave_start, h->grid, stats + 3, code_bytes,
                                  h->chunk_tiles, narrow, w.wl_part, bd, sl->side));
      Mark(h, 3, sl->side);
      SMX_HIP(hipEventRecord(sl->join_ev, sl->side));
      SMX_HIP(hipStreamWaitEvent(s, sl->join_ev, 0));   // join
    }
    // the scan's timing events go into its own dispatch (hipExtLaunchKernel):
    // its execution alone, as rocprofv3 measures it
    const size_t le = size_t(h->scan_logged % kScanLog) * 2;
    hipEvent_t se0 = nullptr, se1 = nullptr;
    if (h->profiling) {
      se0 = h->ev[5];
      se1 = h->ev[6];
    } else if (h->scan_log) {
      se0 = h->scan_ev[le];
      se1 = h->scan_ev[le + 1];
    }
    SMX_HIP(smx::LaunchScan(ix, a, h->grid, variant, s, narrow, se0, se1));
    if (h->scan_log && !h->profiling) ++h->scan_logged;
    SMX_HIP(smx::LaunchFinalSelect(sel, nq, s, h->profiling ? h->ev[10] : nullptr,
                                   h->profiling ? h->ev[11] : nullptr));
    Mark(h, 7, s);
    return SMX_OK;
  };
#ifdef SMX_PHASE_STAMPS
  // diagnostic build: the stamp buffer is installed once, before the first
  // call's kernels are enqueued and with the device idle.  (The first
  // version installed it after the first call's launches with a null-stream
  // hipMemcpyToSymbol, which does not order against the handle's
  // non-blocking stream: kernels in flight read g_phase_stamps while it was
  // being rewritten -- a torn 64-bit pointer -- and faulted.)
  static unsigned long long* phase_buf = nullptr;
  if (!phase_buf) {
    const size_t words = size_t(3) * smx::kPhaseQueries * 8;
    SMX_HIP(hipDeviceSynchronize());
    SMX_HIP(hipMalloc(&phase_buf, words * 8));
    SMX_HIP(hipMemset(phase_buf, 0, words * 8));
    SMX_HIP(smx::SetPhaseStamps(phase_buf));
    SMX_HIP(hipDeviceSynchronize());
  }
#endif
  // The workspace is shared by every stream: a call on another stream than
  // the last one waits for that one's work (stream-ordered, no host sync).
  // The event is recorded on the last stream only at such a switch (it then
  // covers all of that stream's calls so far): a record per call put a
  // barrier packet between consecutive graph replays (~4 us per call).
  if (sl->last_stream != s) {
    SMX_HIP(hipEventRecord(sl->done_ev, sl->last_stream));
    SMX_HIP(hipStreamWaitEvent(s, sl->done_ev, 0));
    sl->last_stream = s;
  }
  bool ran = false;
  // (profiled calls run eagerly: HIP events recorded inside a captured graph
  // carry no timestamps)
  if (h->use_graph && !h->profiling && !h->scan_log && s) {
    const uint64_t key[GraphKeyWords] = {
        uint64_t(reinterpret_cast<uintptr_t>(queries)), uint64_t(nq), uint64_t(L), uint64_t(pnn),
        uint64_t(final_nn), uint64_t(reorder) | uint64_t(pre_only) << 1 | uint64_t(h->profiling) << 2 |
                                uint64_t(single) << 3,
        uint64_t(reinterpret_cast<uintptr_t>(out_idx)), uint64_t(reinterpret_cast<uintptr_t>(out_dist)),
        uint64_t(reinterpret_cast<uintptr_t>(out_count)), uint64_t(reinterpret_cast<uintptr_t>(shard_out)),
        uint64_t(reinterpret_cast<uintptr_t>(s)), w.gen, uint64_t(w.cap), uint64_t(seed),
        uint64_t(h->chunk_tiles), uint64_t(variant)};
    if (!sl->graph_exec || std::memcmp(key, sl->graph_key, sizeof(key)) != 0) {
      if (sl->graph_exec) (void)hipGraphExecDestroy(sl->graph_exec);
      sl->graph_exec = nullptr;
      if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) == hipSuccess) {
        const int prc = first_pass();
        hipGraph_t g = nullptr;
        const hipError_t e = hipStreamEndCapture(s, &g);
        if (prc == SMX_OK && e == hipSuccess && g &&
            hipGraphInstantiate(&sl->graph_exec, g, nullptr, nullptr, 0) == hipSuccess)
          std::memcpy(sl->graph_key, key, sizeof(key));
        else
          sl->graph_exec = nullptr;   // capture unsupported here: run eagerly
        if (g) (void)hipGraphDestroy(g);
        (void)hipGetLastError();
      }
    }
    if (sl->graph_exec) {
      SMX_HIP(hipGraphLaunch(sl->graph_exec, s));
      ran = true;
    }
  }
  if (!ran && (rc = first_pass())) return rc;
  // No host round trip: overflow and the select's fallback queries are
  // handled on the device, so the call returns with the work enqueued
  // (search_batched_device is stream-ordered; the host-buffer entry points
  // synchronise on their result copies).  Profiled calls read the stats.
  uint32_t st[16] = {};
  if (h->profiling || variant == 8) {
    SMX_HIP(hipMemcpyAsync(h->host_stats, stats, sizeof(st), hipMemcpyDeviceToHost, s));
    SMX_HIP(hipStreamSynchronize(s));
    std::memcpy(st, h->host_stats, sizeof(st));
  }
  if (variant == 8) {
    // diagnostics: the last call's stamps to the file named by $SMX_STAMPS
    const char* path = std::getenv("SMX_STAMPS");
    uint32_t cnt_st = 0;
    SMX_HIP(hipMemcpy(&cnt_st, h->stamp_count, 4, hipMemcpyDeviceToHost));
    cnt_st = std::min(cnt_st, kStampCap);
    std::vector<unsigned long long> buf(size_t(cnt_st) * 8);
    if (cnt_st)
      SMX_HIP(hipMemcpy(buf.data(), h->stamps, buf.size() * 8, hipMemcpyDeviceToHost));
    if (path) {
      if (FILE* f = std::fopen(path, "wb")) {
        std::fwrite(buf.data(), 8, buf.size(), f);
        std::fclose(f);
      }
    }
  }
#ifdef SMX_PHASE_STAMPS
  {
    // diagnostic build: the phase stamps of this call to $SMX_PHASE_FILE
    const size_t words = size_t(3) * smx::kPhaseQueries * 8;
    if (const char* path = std::getenv("SMX_PHASE_FILE")) {
      SMX_HIP(hipStreamSynchronize(s));
      std::vector<unsigned long long> buf(words);
      SMX_HIP(hipMemcpy(buf.data(), phase_buf, words * 8, hipMemcpyDeviceToHost));
      if (FILE* f = std::fopen(path, "wb")) {
        std::fwrite(buf.data(), 8, buf.size(), f);
        std::fclose(f);
      }
    }
  }
#endif
#ifdef SMX_DEBUG_CHECKS
  {
    // debug build: every call is checked for index violations on the device
    SMX_HIP(hipStreamSynchronize(s));
    unsigned int bad = 0;
    SMX_HIP(smx::TakeCheckFailures(&bad));
    if (bad)
      return Fail(SMX_INTERNAL, "debug build: " + std::to_string(bad) +
                                    " device index-check violations (see the kernel printf)");
  }
#endif
  smx_timings& t = h->timings;
  if (h->profiling) {
    // The stream is idle here, so reading the events costs no extra sync.
    // the LUT build runs inside the top-L launch; the inversion (side
    // stream) and the seed overlap, each timed from the fork
    t.partition_ms = Elapsed(h, 0, 1);
    t.lut_ms = 0.0f;
    // the seed, scan and select kernels from events in their own dispatch
    // packets (their execution, as rocprofv3 reports it); partition + top-L
    // and the three-launch work list from event packets around the launches
    t.invert_ms = Elapsed(h, 1, 3);
    t.seed_scan_ms = seed_dispatch_ev ? Elapsed(h, 8, 9) : Elapsed(h, 1, 4);
    t.seed_select_ms = 0.0f;
    t.scan_ms = Elapsed(h, 5, 6);
    t.select_ms = Elapsed(h, 10, 11);
    t.total_ms = Elapsed(h, 0, 7);
  }
  unsigned long long cb;
  std::memcpy(&cb, st + 6, sizeof(cb));
  t.seed_code_bytes = 0.0;
  t.scan_code_bytes = double(cb);
  t.seed_pairs = int32_t(std::min(seed, L)) * nq;
  t.scan_pairs = int32_t(st[3]);
  t.overflow_retries = int32_t(st[11]);   // rescan passes (queries: st[10])
  t.max_candidates = int32_t(st[2]);
  // units = 2 x 32-slot tiles + 16-slot tiles
  t.scan_item_tiles16 = double(st[12]);
  t.scan_item_tiles = (double(st[5]) - double(st[12])) * 0.5;
  t.mean_candidates = float(st[8]) / float(nq);
  t.scan_workgroups = h->grid;
  return SMX_OK;
}

// The search pipeline over a whole batch: sub-batches of SubBatchQueries
// queries run one after another on the stream (the reference's
// search_batched takes any batch size: scann_npy.cc:233-270), each query's
// results at its own offset of the outputs.
int RunSearch(smx_index* h, const float* queries, int nq, int L, int pre_nn, int final_nn,
              bool reorder, bool pre_only, uint32_t* out_idx, float* out_dist,
              int32_t* out_count, hipStream_t s, smx::ShardEntry* shard_out = nullptr,
              bool single = false) {
  const int chunk = SubBatchQueries(h);
  if (nq <= chunk)
    return RunSearchChunk(h, queries, nq, L, pre_nn, final_nn, reorder, pre_only, out_idx,
                          out_dist, out_count, s, shard_out, single);
  const int pnn = reorder ? pre_nn : final_nn;
  const size_t kk = size_t(std::max(1, SpillK(h->ix, pnn)));
  const size_t width = size_t(shard_out ? 1 : pre_only ? pnn : final_nn);
  for (int q0 = 0; q0 < nq; q0 += chunk) {
    const int n = std::min(chunk, nq - q0);
    const int rc = RunSearchChunk(
        h, queries + size_t(q0) * h->ix.dim, n, L, pre_nn, final_nn, reorder, pre_only,
        out_idx ? out_idx + size_t(q0) * width : nullptr,
        out_dist ? out_dist + size_t(q0) * width : nullptr, out_count ? out_count + q0 : nullptr,
        s, shard_out ? shard_out + size_t(q0) * kk : nullptr, single);
    if (rc) return rc;
  }
  return SMX_OK;
}

// Largest k' (kept candidates per query before SOAR dedupe) the final
// select supports: its block kernel holds the candidate list (cap <=
// 8192 keys) plus 2 k' select buffers in LDS (LaunchFinalSelect).
constexpr int kMaxKPrime = 2048;

int CheckSearchArgs(smx_index* h, int nq, int dim, const smx_search_params* p) {
  if (!h) return Fail(SMX_INVALID_ARGUMENT, "null index");
  if (!p) return Fail(SMX_INVALID_ARGUMENT, "null search params");
  if (nq < 0) return Fail(SMX_INVALID_ARGUMENT, "negative batch size");
  if (dim != h->ix.dim)
    return Fail(SMX_INVALID_ARGUMENT, "Query doesn't match dataset dimsensionality");
  if (p->leaves_to_search <= 0) return Fail(SMX_INVALID_ARGUMENT, "leaves_to_search must be > 0");
  if (p->final_nn <= 0) return Fail(SMX_INVALID_ARGUMENT, "final_num_neighbors must be > 0");
  if (p->reorder && p->pre_reorder_nn <= 0)
    return Fail(SMX_INVALID_ARGUMENT, "pre_reorder_num_neighbors must be > 0");
  if (p->reorder && !h->ix.dataset && !h->ix.member_rows)
    return Fail(SMX_FAILED_PRECONDITION, "exact reordering requested but index has no dataset");
  const int pnn = p->reorder ? p->pre_reorder_nn : p->final_nn;
  if (SpillK(h->ix, pnn) > kMaxKPrime)
    return Fail(SMX_INVALID_ARGUMENT,
                "pre-reorder neighbors (x the spilling overretrieve factor) above 2048 are not "
                "supported");
  return SMX_OK;
}

int CheckFinite(const float* q, size_t n) {
  for (size_t i = 0; i < n; ++i)
    if (!std::isfinite(q[i])) return Fail(SMX_INVALID_ARGUMENT, "queries must be finite");
  return SMX_OK;
}

}  // namespace

extern "C" {

const char* smx_last_error(void) { return g_last_error.c_str(); }
const char* smx_version(void) { return "scann_mi355x 0.1 (gfx950)"; }

int smx_index_create(const smx_index_desc* desc, int32_t device, smx_index** out) {
  if (!out) return Fail(SMX_INVALID_ARGUMENT, "null output handle");
  *out = nullptr;
  int rc = ValidateDesc(desc);
  if (rc) return rc;
  if (EffectiveKSteps(desc->num_blocks) < 0)
    return Fail(SMX_INVALID_ARGUMENT, "unsupported number of AH blocks");
  int ndev = 0;
  SMX_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return Fail(SMX_INVALID_ARGUMENT, "no such HIP device");
  SMX_HIP(hipSetDevice(device));
  auto* h = new smx_index;
  h->device = device;
  rc = UploadIndex(desc, h);
  if (rc) {
    FreeIndex(h->ix);
    delete h;
    return rc;
  }
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
    FreeIndex(h->ix);
    delete h;
    return Fail(SMX_DEVICE_ERROR, "hipStreamCreate failed");
  }
  for (auto& e : h->ev) (void)hipEventCreate(&e);
  hipDeviceProp_t prop;
  SMX_HIP(hipGetDeviceProperties(&prop, device));
  {
    int per_cu = 0;
    SMX_HIP(smx::ScanBlocksPerCU(h->ix, &per_cu));
    h->grid = prop.multiProcessorCount * std::max(1, per_cu);
    h->cus = prop.multiProcessorCount;
  }
  if (hipHostMalloc(reinterpret_cast<void**>(&h->host_stats), 32 * sizeof(uint32_t)) != hipSuccess) {
    smx_index_destroy(h);
    return Fail(SMX_OUT_OF_MEMORY, "hipHostMalloc failed");
  }
  if (const char* fw = std::getenv("SMX_FUSED_WORKLIST"))
    h->fused_worklist_leaves = std::min(std::atoi(fw), smx::kFusedWorklistLeaves);
  if (const char* nw = std::getenv("SMX_NARROW")) {
    // 0: 32-slot tiles only; 1: by density (default); 2: 16-slot tiles only
    // whatever the density
    h->narrow_tiles = nw[0] != '0';
    h->narrow_only = nw[0] == '2';
  }
  if (const char* sw = std::getenv("SMX_SERIAL_WORKLIST")) h->serial_worklist = sw[0] != '0';
  // 0: the all-sparse 32-slot tile at K % 4 == 2 (read per handle, so that the
  // tests run both tiles in one process)
  if (const char* df = std::getenv("SMX_DENSE_FIRST")) h->ix.dense_first = df[0] != '0';
  if (const char* lb = std::getenv("SMX_LEAF_SLOT_BUDGET")) {
    const long long v = std::atoll(lb);
    if (v > 0 && uint64_t(v) < kLeafSlotBudget) h->leaf_slot_budget = uint64_t(v);
  }
#ifdef SMX_SCAN_DIAGNOSTICS
  // a timing ablation for a whole process (tools: the shard configurations'
  // bench lines under the timing library; see smx::LaunchScan)
  if (const char* sv = std::getenv("SMX_SCAN_VARIANT")) {
    const int v = std::atoi(sv);
    if (v == 2 || v == 4 || v == 16 || v == 32 || v == 64 || v == 68) h->scan_variant = v;
  }
#endif
  // tuning knobs for A/Bs (the defaults otherwise; smx_set_tuning overrides)
  if (const char* ct = std::getenv("SMX_CHUNK_TILES")) {
    const int v = std::atoi(ct);
    if (v >= 8 && v <= 65535) h->chunk_tiles = uint32_t(v);
  }
  if (const char* sr = std::getenv("SMX_SEED_ROWS")) {
    const int v = std::atoi(sr);
    if (v >= 1 && v <= smx::kSeedKeys) h->seed_rows = uint32_t(v);
  }
  if (const char* sl = std::getenv("SMX_SEED_LEAVES")) {
    const int v = std::atoi(sl);
    if (v >= 0 && v <= 64) h->seed_leaves = v;
  }
  const char* ng = std::getenv("SMX_NO_GRAPH");
  // Eager launches by default: six kernels a call queue back to back on the
  // stream, while consecutive replays of a captured graph left ~13 us
  // between graphs (0.165 vs 0.158 ms/step, bench A/B on one box).
  const char* gr = std::getenv("SMX_GRAPH");
  h->use_graph = gr && gr[0] == '1' && !(ng && ng[0] == '1');

  *out = h;
  return SMX_OK;
}

int smx_index_destroy(smx_index* h) {
  if (!h) return SMX_OK;
  (void)hipSetDevice(h->device);
  // every slot's work, whatever stream it ran on, without naming the callers'
  // streams (they may be gone; smx_release_stream documents the lifetime)
  (void)hipDeviceSynchronize();
  for (StreamSlot* sl : h->slots) DestroySlot(sl);
  h->slots.clear();
  if (h->host_stats) (void)hipHostFree(h->host_stats);
  DFree(h->stamps);
  DFree(h->stamp_count);
  FreeIndex(h->ix);
  for (auto& e : h->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : h->scan_ev)
    if (e) (void)hipEventDestroy(e);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return SMX_OK;
}

int smx_release_stream(smx_index* h, void* stream) {
  if (!h) return Fail(SMX_INVALID_ARGUMENT, "null index");
  std::lock_guard<std::mutex> lock(h->mu);
  SMX_HIP(hipSetDevice(h->device));
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : h->stream;
  for (size_t i = 0; i < h->slots.size(); ++i) {
    StreamSlot* sl = h->slots[i];
    if (sl->last_stream != s && sl->key != s) continue;
    // the slot's work ran on its last stream (and its side stream)
    if (sl->last_stream) SMX_HIP(hipStreamSynchronize(sl->last_stream));
    if (sl->side) SMX_HIP(hipStreamSynchronize(sl->side));
    DestroySlot(sl);
    h->slots.erase(h->slots.begin() + long(i));
    --i;
  }
  return SMX_OK;
}

int smx_index_info(const smx_index* h, int32_t* dim, int32_t* num_leaves,
                   uint32_t* num_datapoints, int32_t* shift) {
  if (!h) return Fail(SMX_INVALID_ARGUMENT, "null index");
  if (dim) *dim = h->ix.dim;
  if (num_leaves) *num_leaves = h->ix.nl;
  if (num_datapoints) *num_datapoints = h->ix.num_datapoints;
  if (shift) *shift = h->ix.shift;
  return SMX_OK;
}

int smx_search_batched_device(smx_index* h, const float* d_queries, int32_t nq, int32_t dim,
                              const smx_search_params* p, uint32_t* d_out_idx,
                              float* d_out_dist, int32_t* d_out_count, void* stream) {
  int rc = CheckSearchArgs(h, nq, dim, p);
  if (rc) return rc;
  std::lock_guard<std::mutex> lock(h->mu);
  SMX_HIP(hipSetDevice(h->device));
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : h->stream;
  return RunSearch(h, d_queries, nq, p->leaves_to_search, p->pre_reorder_nn, p->final_nn,
                   p->reorder != 0, false, d_out_idx, d_out_dist, d_out_count, s);
}

}  // extern "C"

namespace {

// Host-buffer search: queries in, (ids, distances, counts) out, synchronous.
int SearchHost(smx_index* h, const float* queries, int32_t nq, int32_t dim,
               const smx_search_params* p, uint32_t* out_idx, float* out_dist,
               int32_t* out_count, bool single) {
  int rc = CheckSearchArgs(h, nq, dim, p);
  if (rc) return rc;
  if (nq > 0 && (!queries || !out_idx || !out_dist))
    return Fail(SMX_INVALID_ARGUMENT, "null query or output buffer");
  if ((rc = CheckFinite(queries, size_t(nq) * dim))) return rc;
  if (nq == 0) return SMX_OK;
  std::lock_guard<std::mutex> lock(h->mu);
  SMX_HIP(hipSetDevice(h->device));
  hipStream_t s = h->stream;
  const int width = p->final_nn;
  const int pnn = p->reorder ? p->pre_reorder_nn : p->final_nn;
  StreamSlot* sl = nullptr;
  if ((rc = SlotFor(h, s, &sl))) return rc;
  rc = EnsureWorkspace(h, sl, nq, std::min(p->leaves_to_search, h->ix.nl),
                       std::max(1, SpillK(h->ix, pnn)), width);
  if (rc) return rc;
  Workspace& w = sl->ws;
  SMX_HIP(hipMemcpyAsync(w.queries, queries, sizeof(float) * size_t(nq) * dim,
                         hipMemcpyHostToDevice, s));
  rc = RunSearch(h, w.queries, nq, p->leaves_to_search, p->pre_reorder_nn, p->final_nn,
                 p->reorder != 0, false, w.out_idx, w.out_dist, w.out_count, s, nullptr, single);
  if (rc) return rc;
  SMX_HIP(hipMemcpyAsync(out_idx, w.out_idx, sizeof(uint32_t) * size_t(nq) * width,
                         hipMemcpyDeviceToHost, s));
  SMX_HIP(hipMemcpyAsync(out_dist, w.out_dist, sizeof(float) * size_t(nq) * width,
                         hipMemcpyDeviceToHost, s));
  if (out_count)
    SMX_HIP(hipMemcpyAsync(out_count, w.out_count, sizeof(int32_t) * nq, hipMemcpyDeviceToHost, s));
  SMX_HIP(hipStreamSynchronize(s));
  return SMX_OK;
}

}  // namespace

extern "C" {

int smx_nearest_centers(const float* x, int64_t n, int32_t d, const float* centers, int32_t k,
                        const int32_t* primary, float lambda, int32_t* out, float* out_loss,
                        void* stream) {
  if (n < 0 || d <= 0 || k <= 0) return Fail(SMX_INVALID_ARGUMENT, "need n >= 0, d > 0, k > 0");
  if (primary && k < 2) return Fail(SMX_INVALID_ARGUMENT, "SOAR assignment needs k >= 2");
  if (n == 0) return SMX_OK;
  if (!x || !centers || !out) return Fail(SMX_INVALID_ARGUMENT, "null input or output buffer");
  if (!(lambda >= 0.0f)) return Fail(SMX_INVALID_ARGUMENT, "lambda must be >= 0");
  SMX_HIP(smx::LaunchNearestCenters(x, n, d, centers, k, primary, lambda, out, out_loss,
                                    static_cast<hipStream_t>(stream)));
  return SMX_OK;
}

int smx_kth_threshold_keys(const uint32_t* vals, int32_t sets, int32_t kk, uint64_t* out,
                           void* stream) {
  if (sets < 0 || kk < 0) return Fail(SMX_INVALID_ARGUMENT, "need sets >= 0, kk >= 0");
  if (sets == 0) return SMX_OK;
  if (!vals || !out) return Fail(SMX_INVALID_ARGUMENT, "null input or output buffer");
  SMX_HIP(smx::LaunchKthKeys(vals, sets, kk, out, static_cast<hipStream_t>(stream)));
  return SMX_OK;
}

namespace {
int CheckBlocks(int64_t n, int32_t dim, int32_t nb, int32_t dpb) {
  if (n < 0 || dim <= 0 || nb <= 0 || dpb <= 0)
    return Fail(SMX_INVALID_ARGUMENT, "need n >= 0, dim > 0, num_blocks > 0, dims_per_block > 0");
  if (int64_t(nb) * dpb < dim || int64_t(nb - 1) * dpb >= dim)
    return Fail(SMX_INVALID_ARGUMENT, "num_blocks must be ceil(dim / dims_per_block)");
  return SMX_OK;
}
}  // namespace

int smx_block_encode(const float* r, int64_t n, int32_t dim, const float* codebook, int32_t nb,
                     int32_t dpb, uint8_t* out, void* stream) {
  if (int e = CheckBlocks(n, dim, nb, dpb)) return e;
  if (n == 0) return SMX_OK;
  if (!r || !codebook || !out) return Fail(SMX_INVALID_ARGUMENT, "null input or output buffer");
  SMX_HIP(smx::LaunchBlockEncode(r, n, dim, codebook, nb, dpb, out,
                                 static_cast<hipStream_t>(stream)));
  return SMX_OK;
}

int smx_avq_encode(const float* resid, const float* orig, int64_t n, int32_t dim,
                   const float* codebook, int32_t nb, int32_t dpb, double threshold, uint8_t* out,
                   void* stream) {
  if (int e = CheckBlocks(n, dim, nb, dpb)) return e;
  if (n == 0) return SMX_OK;
  if (!resid || !orig || !codebook || !out)
    return Fail(SMX_INVALID_ARGUMENT, "null input or output buffer");
  if (dim < 2) return Fail(SMX_INVALID_ARGUMENT, "noise shaping needs dim >= 2");
  if (!(threshold == threshold)) return Fail(SMX_INVALID_ARGUMENT, "threshold is NaN");
  if (smx::AvqEncodeLds(nb, dpb) > 65536)
    return Fail(SMX_INVALID_ARGUMENT, "num_blocks * dims_per_block too large for the AVQ kernel");
  SMX_HIP(smx::LaunchAvqEncode(resid, orig, n, dim, codebook, nb, dpb, threshold, out,
                               static_cast<hipStream_t>(stream)));
  return SMX_OK;
}

int smx_kmeans_accumulate(const float* x, int64_t n, int32_t d, const int32_t* label, int32_t k,
                          double scale, uint64_t* sums, uint32_t* counts, void* stream) {
  if (n < 0 || d <= 0 || k <= 0 || !(scale > 0.0))
    return Fail(SMX_INVALID_ARGUMENT, "need n >= 0, d > 0, k > 0, scale > 0");
  if (n == 0) return SMX_OK;
  if (!x || !label || !sums || !counts) return Fail(SMX_INVALID_ARGUMENT, "null buffer");
  SMX_HIP(smx::LaunchKmeansAccumulate(x, n, d, label, k, scale,
                                      reinterpret_cast<unsigned long long*>(sums), counts,
                                      static_cast<hipStream_t>(stream)));
  return SMX_OK;
}

int smx_kmeans_finalize(const uint64_t* sums, const uint32_t* counts, int32_t k, int32_t d,
                        double scale, float* centers, void* stream) {
  if (d <= 0 || k <= 0 || !(scale > 0.0))
    return Fail(SMX_INVALID_ARGUMENT, "need d > 0, k > 0, scale > 0");
  if (!sums || !counts || !centers) return Fail(SMX_INVALID_ARGUMENT, "null buffer");
  SMX_HIP(smx::LaunchKmeansFinalize(reinterpret_cast<const unsigned long long*>(sums), counts, k, d,
                                    scale, centers, static_cast<hipStream_t>(stream)));
  return SMX_OK;
}

int smx_codebook_accumulate(const float* r, int64_t n, int32_t dim, const uint8_t* codes,
                            int32_t nb, int32_t dpb, double scale, uint64_t* sums,
                            uint32_t* counts, void* stream) {
  if (int e = CheckBlocks(n, dim, nb, dpb)) return e;
  if (!(scale > 0.0)) return Fail(SMX_INVALID_ARGUMENT, "scale must be > 0");
  if (n == 0) return SMX_OK;
  if (!r || !codes || !sums || !counts) return Fail(SMX_INVALID_ARGUMENT, "null buffer");
  SMX_HIP(smx::LaunchCodebookAccumulate(r, n, dim, codes, nb, dpb, scale,
                                        reinterpret_cast<unsigned long long*>(sums), counts,
                                        static_cast<hipStream_t>(stream)));
  return SMX_OK;
}

int smx_group_by_leaf(const int32_t* labels, const uint32_t* ids, int64_t m, int32_t k,
                      void* temp, size_t* temp_bytes, uint64_t* keys, uint64_t* offsets,
                      uint32_t* members, int32_t* member_leaf, void* stream) {
  if (m < 0 || k <= 0 || !temp_bytes) return Fail(SMX_INVALID_ARGUMENT, "need m >= 0, k > 0");
  if (m > 0xFFFFFFFFll) return Fail(SMX_INVALID_ARGUMENT, "at most 2^32 - 1 members");
  if (temp && (!keys || !offsets || !members || !member_leaf || (m > 0 && (!labels || !ids))))
    return Fail(SMX_INVALID_ARGUMENT, "null buffer");
  SMX_HIP(smx::GroupByLeaf(labels, ids, m, k, temp, temp_bytes, keys, offsets, members,
                           member_leaf, static_cast<hipStream_t>(stream)));
  return SMX_OK;
}

int smx_gather_residuals(const float* x, int32_t d, const uint32_t* rows, const int32_t* leaf,
                         const float* centers, int64_t m, int64_t row_base, float* out,
                         void* stream) {
  if (d <= 0 || m < 0) return Fail(SMX_INVALID_ARGUMENT, "need d > 0, m >= 0");
  if (m == 0) return SMX_OK;
  if (!x || !rows || !out || (centers && !leaf)) return Fail(SMX_INVALID_ARGUMENT, "null buffer");
  SMX_HIP(smx::LaunchGatherResiduals(x, d, rows, leaf, centers, m, row_base, out,
                                     static_cast<hipStream_t>(stream)));
  return SMX_OK;
}

int smx_search_batched(smx_index* h, const float* queries, int32_t nq, int32_t dim,
                       const smx_search_params* p, uint32_t* out_idx, float* out_dist,
                       int32_t* out_count) {
  return SearchHost(h, queries, nq, dim, p, out_idx, out_dist, out_count, false);
}

int smx_search(smx_index* h, const float* query, int32_t dim, const smx_search_params* p,
               uint32_t* out_idx, float* out_dist, int32_t* out_count) {
  return SearchHost(h, query, 1, dim, p, out_idx, out_dist, out_count, true);
}

int smx_shard_width(const smx_index* h, const smx_search_params* p, int32_t* out_k) {
  if (!h || !p || !out_k) return Fail(SMX_INVALID_ARGUMENT, "null argument");
  const int pnn = p->reorder ? p->pre_reorder_nn : p->final_nn;
  if (pnn <= 0) return Fail(SMX_INVALID_ARGUMENT, "neighbor counts must be > 0");
  *out_k = std::max(1, SpillK(h->ix, pnn));
  return SMX_OK;
}

int smx_search_shard_device(smx_index* h, const float* d_queries, int32_t nq, int32_t dim,
                            const smx_search_params* p, smx_shard_entry* d_entries,
                            void* stream) {
  int rc = CheckSearchArgs(h, nq, dim, p);
  if (rc) return rc;
  if (nq > 0 && !d_entries) return Fail(SMX_INVALID_ARGUMENT, "null entries buffer");
  static_assert(sizeof(smx_shard_entry) == sizeof(smx::ShardEntry), "entry layout");
  std::lock_guard<std::mutex> lock(h->mu);
  SMX_HIP(hipSetDevice(h->device));
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : h->stream;
  return RunSearch(h, d_queries, nq, p->leaves_to_search, p->pre_reorder_nn, p->final_nn,
                   p->reorder != 0, false, nullptr, nullptr, nullptr, s,
                   reinterpret_cast<smx::ShardEntry*>(d_entries));
}

int smx_merge_shards_device(smx_index* h, int32_t world, int32_t nq,
                            const smx_search_params* p, const smx_shard_entry* d_entries,
                            uint32_t* d_out_idx, float* d_out_dist, int32_t* d_out_count,
                            void* stream) {
  if (!h || !p) return Fail(SMX_INVALID_ARGUMENT, "null argument");
  if (world < 1 || world > 64) return Fail(SMX_INVALID_ARGUMENT, "world must be in [1, 64]");
  if (nq < 0) return Fail(SMX_INVALID_ARGUMENT, "negative batch size");
  if (p->final_nn <= 0) return Fail(SMX_INVALID_ARGUMENT, "final_num_neighbors must be > 0");
  const int pnn = p->reorder ? p->pre_reorder_nn : p->final_nn;
  if (pnn <= 0) return Fail(SMX_INVALID_ARGUMENT, "neighbor counts must be > 0");
  const int kk = std::max(1, SpillK(h->ix, pnn));
  if (kk > kMaxKPrime)
    return Fail(SMX_INVALID_ARGUMENT, "shard lists above 2048 entries per query are not supported");
  if (nq == 0) return SMX_OK;
  std::lock_guard<std::mutex> lock(h->mu);
  SMX_HIP(hipSetDevice(h->device));
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : h->stream;
  smx::MergeArgs m{};
  // more lists than one launch of the wide merge holds: its round buffers,
  // in this stream's slot (another stream's merge runs concurrently)
  const size_t scratch = smx::MergeScratchEntries(world, nq, kk);
  if (scratch) {
    StreamSlot* sl = nullptr;
    int rc = SlotFor(h, s, &sl);
    if (rc) return rc;
    if (sl->last_stream != s) {   // the slot's earlier work on its other stream
      SMX_HIP(hipEventRecord(sl->done_ev, sl->last_stream));
      SMX_HIP(hipStreamWaitEvent(s, sl->done_ev, 0));
      sl->last_stream = s;
    }
    Workspace& w = sl->ws;
    if (w.merge_entries < scratch) {
      DFree(w.merge_scratch[0]);
      DFree(w.merge_scratch[1]);
      w.merge_entries = 0;
      if ((rc = DAlloc(&w.merge_scratch[0], scratch)) || (rc = DAlloc(&w.merge_scratch[1], scratch)))
        return rc;
      w.merge_entries = scratch;
    }
    m.scratch[0] = w.merge_scratch[0];
    m.scratch[1] = w.merge_scratch[1];
  }
  m.entries = reinterpret_cast<const smx::ShardEntry*>(d_entries);
  m.world = world;
  m.nq = nq;
  m.kk = kk;
  m.pre_nn = pnn;
  m.disjoint = h->ix.disjoint ? 1 : 0;
  m.reorder = p->reorder ? 1 : 0;
  m.out_idx = d_out_idx;
  m.out_dist = d_out_dist;
  m.out_count = d_out_count;
  m.out_width = p->final_nn;
  SMX_HIP(smx::LaunchMergeShards(m, s));
  return SMX_OK;
}

int smx_search_pre_reorder(smx_index* h, const float* queries, int32_t nq, int32_t leaves,
                           int32_t pre_nn, uint32_t* out_idx, float* out_dist,
                           int32_t* out_count) {
  if (!h) return Fail(SMX_INVALID_ARGUMENT, "null index");
  if (nq < 0) return Fail(SMX_INVALID_ARGUMENT, "negative batch size");
  if (nq > 0 && (!queries || !out_idx || !out_dist))
    return Fail(SMX_INVALID_ARGUMENT, "null query or output buffer");
  if (leaves <= 0 || pre_nn <= 0) return Fail(SMX_INVALID_ARGUMENT, "leaves and pre_nn must be > 0");
  if (SpillK(h->ix, pre_nn) > kMaxKPrime)
    return Fail(SMX_INVALID_ARGUMENT, "pre_nn (x the spilling overretrieve factor) above 2048");
  int rc = CheckFinite(queries, size_t(nq) * h->ix.dim);
  if (rc) return rc;
  if (nq == 0) return SMX_OK;
  std::lock_guard<std::mutex> lock(h->mu);
  SMX_HIP(hipSetDevice(h->device));
  hipStream_t s = h->stream;
  StreamSlot* sl = nullptr;
  if ((rc = SlotFor(h, s, &sl))) return rc;
  rc = EnsureWorkspace(h, sl, nq, std::min(leaves, h->ix.nl), std::max(1, SpillK(h->ix, pre_nn)),
                       pre_nn);
  if (rc) return rc;
  Workspace& w = sl->ws;
  SMX_HIP(hipMemcpyAsync(w.queries, queries, sizeof(float) * size_t(nq) * h->ix.dim,
                         hipMemcpyHostToDevice, s));
  rc = RunSearch(h, w.queries, nq, leaves, pre_nn, pre_nn, true, true, w.out_idx, w.out_dist,
                 w.out_count, s);
  if (rc) return rc;
  SMX_HIP(hipMemcpyAsync(out_idx, w.out_idx, sizeof(uint32_t) * size_t(nq) * pre_nn,
                         hipMemcpyDeviceToHost, s));
  SMX_HIP(hipMemcpyAsync(out_dist, w.out_dist, sizeof(float) * size_t(nq) * pre_nn,
                         hipMemcpyDeviceToHost, s));
  if (out_count)
    SMX_HIP(hipMemcpyAsync(out_count, w.out_count, sizeof(int32_t) * nq, hipMemcpyDeviceToHost, s));
  SMX_HIP(hipStreamSynchronize(s));
  return SMX_OK;
}

int smx_partition_topl(smx_index* h, const float* queries, int32_t nq, int32_t L,
                       int32_t* out_leaf, float* out_dist) {
  if (!h) return Fail(SMX_INVALID_ARGUMENT, "null index");
  if (nq < 0 || L <= 0) return Fail(SMX_INVALID_ARGUMENT, "bad nq / L");
  if (nq == 0) return SMX_OK;
  if (!queries || !out_leaf || !out_dist) return Fail(SMX_INVALID_ARGUMENT, "null buffer");
  std::lock_guard<std::mutex> lock(h->mu);
  SMX_HIP(hipSetDevice(h->device));
  hipStream_t s = h->stream;
  float* dq = nullptr;
  int32_t* dl = nullptr;
  float* dd = nullptr;
  float* dsc = nullptr;
  int rc;
  if ((rc = DAlloc(&dq, size_t(nq) * h->ix.dim)) || (rc = DAlloc(&dl, size_t(nq) * L)) ||
      (rc = DAlloc(&dd, size_t(nq) * L)) || (rc = DAlloc(&dsc, size_t(nq) * h->ix.nl))) {
    DFree(dq); DFree(dl); DFree(dd); DFree(dsc);
    return rc;
  }
  hipError_t e = hipMemcpyAsync(dq, queries, sizeof(float) * size_t(nq) * h->ix.dim,
                                hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = smx::LaunchPartitionTopL(h->ix, dq, nq, L, dl, dd, dsc, s);
  if (e == hipSuccess) e = hipMemcpyAsync(out_leaf, dl, 4 * size_t(nq) * L, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemcpyAsync(out_dist, dd, 4 * size_t(nq) * L, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  DFree(dq); DFree(dl); DFree(dd); DFree(dsc);
  if (e != hipSuccess) return Fail(SMX_DEVICE_ERROR, hipGetErrorString(e));
  return SMX_OK;
}

int smx_create_lookup_tables(smx_index* h, const float* queries, int32_t nq, uint8_t* out_lut,
                             float* out_mult) {
  if (!h) return Fail(SMX_INVALID_ARGUMENT, "null index");
  if (nq <= 0) return nq == 0 ? SMX_OK : Fail(SMX_INVALID_ARGUMENT, "bad nq");
  if (!queries || !out_lut || !out_mult) return Fail(SMX_INVALID_ARGUMENT, "null buffer");
  std::lock_guard<std::mutex> lock(h->mu);
  SMX_HIP(hipSetDevice(h->device));
  hipStream_t s = h->stream;
  const smx::DeviceIndex& ix = h->ix;
  float *dq = nullptr, *dm = nullptr, *di = nullptr;
  int8_t* dl = nullptr;
  uint8_t* du = nullptr;
  int rc;
  if ((rc = DAlloc(&dq, size_t(nq) * ix.dim)) || (rc = DAlloc(&dm, nq)) || (rc = DAlloc(&di, nq)) ||
      (rc = DAlloc(&dl, size_t(nq) * smx::LutRows(ix.ksteps) * 16)) || (rc = DAlloc(&du, size_t(nq) * ix.nb * 16))) {
    DFree(dq); DFree(dm); DFree(di); DFree(dl); DFree(du);
    return rc;
  }
  hipError_t e = hipMemcpyAsync(dq, queries, sizeof(float) * size_t(nq) * ix.dim,
                                hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = smx::LaunchLutBuild(ix, dq, nq, dl, dm, di, du, s);
  if (e == hipSuccess) e = hipMemcpyAsync(out_lut, du, size_t(nq) * ix.nb * 16, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemcpyAsync(out_mult, dm, 4 * size_t(nq), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  DFree(dq); DFree(dm); DFree(di); DFree(dl); DFree(du);
  if (e != hipSuccess) return Fail(SMX_DEVICE_ERROR, hipGetErrorString(e));
  return SMX_OK;
}

int smx_exact_distances(smx_index* h, const float* queries, int32_t nq, const uint32_t* ids,
                        int32_t k, float* out_dist) {
  if (!h) return Fail(SMX_INVALID_ARGUMENT, "null index");
  if (!h->ix.dataset) return Fail(SMX_FAILED_PRECONDITION, "index has no dataset");
  if (nq < 0 || k < 0) return Fail(SMX_INVALID_ARGUMENT, "bad sizes");
  for (size_t i = 0; i < size_t(nq) * k; ++i)
    if (ids[i] >= h->ix.num_datapoints) return Fail(SMX_INVALID_ARGUMENT, "id out of range");
  if (nq == 0 || k == 0) return SMX_OK;
  std::lock_guard<std::mutex> lock(h->mu);
  SMX_HIP(hipSetDevice(h->device));
  hipStream_t s = h->stream;
  float *dq = nullptr, *dout = nullptr;
  uint32_t* dids = nullptr;
  int rc;
  if ((rc = DAlloc(&dq, size_t(nq) * h->ix.dim)) || (rc = DAlloc(&dids, size_t(nq) * k)) ||
      (rc = DAlloc(&dout, size_t(nq) * k))) {
    DFree(dq); DFree(dids); DFree(dout);
    return rc;
  }
  hipError_t e = hipMemcpyAsync(dq, queries, sizeof(float) * size_t(nq) * h->ix.dim,
                                hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(dids, ids, 4 * size_t(nq) * k, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = smx::LaunchExactDistances(h->ix, dq, nq, dids, k, dout, s);
  if (e == hipSuccess) e = hipMemcpyAsync(out_dist, dout, 4 * size_t(nq) * k, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  DFree(dq); DFree(dids); DFree(dout);
  if (e != hipSuccess) return Fail(SMX_DEVICE_ERROR, hipGetErrorString(e));
  return SMX_OK;
}

int smx_lut16_leaf_scores(smx_index* h, int32_t leaf, const uint8_t* lut, int32_t* out_scores) {
  if (!h) return Fail(SMX_INVALID_ARGUMENT, "null index");
  if (leaf < 0 || leaf >= h->ix.nl) return Fail(SMX_INVALID_ARGUMENT, "leaf out of range");
  std::lock_guard<std::mutex> lock(h->mu);
  SMX_HIP(hipSetDevice(h->device));
  hipStream_t s = h->stream;
  const smx::DeviceIndex& ix = h->ix;
  const int rows = smx::LutRows(ix.ksteps);
  std::vector<int8_t> l8(size_t(rows) * 16, 0);
  for (int i = 0; i < ix.nb * 16; ++i) l8[i] = int8_t(int(lut[i]) - 128);
  uint64_t n64 = 0;
  SMX_HIP(hipMemcpy(&n64, ix.member_off + leaf + 1, 8, hipMemcpyDeviceToHost));
  uint64_t b64 = 0;
  SMX_HIP(hipMemcpy(&b64, ix.member_off + leaf, 8, hipMemcpyDeviceToHost));
  const size_t n = size_t(n64 - b64);
  int8_t* dl = nullptr;
  int32_t* dout = nullptr;
  int rc;
  if ((rc = DAlloc(&dl, l8.size())) || (rc = DAlloc(&dout, std::max<size_t>(n, 1)))) {
    DFree(dl); DFree(dout);
    return rc;
  }
  hipError_t e = hipMemcpyAsync(dl, l8.data(), l8.size(), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = smx::LaunchLeafScores(ix, leaf, dl, dout, s);
  if (e == hipSuccess && n) e = hipMemcpyAsync(out_scores, dout, 4 * n, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  DFree(dl); DFree(dout);
  if (e != hipSuccess) return Fail(SMX_DEVICE_ERROR, hipGetErrorString(e));
  return SMX_OK;
}

int smx_set_profiling(smx_index* h, int32_t enabled) {
  if (!h) return Fail(SMX_INVALID_ARGUMENT, "null index");
  if (enabled < 0 || enabled > 2) return Fail(SMX_INVALID_ARGUMENT, "profiling mode must be 0, 1 or 2");
  std::lock_guard<std::mutex> lock(h->mu);
  SMX_HIP(hipSetDevice(h->device));
  h->profiling = enabled == 1;
  h->scan_log = enabled == 2;
  if (h->scan_log) {
    if (h->scan_ev.empty()) {
      h->scan_ev.assign(2 * kScanLog, nullptr);
      for (auto& e : h->scan_ev) SMX_HIP(hipEventCreate(&e));
    }
    h->scan_logged = 0;
  }
  return SMX_OK;
}

int smx_get_timings(const smx_index* h, smx_timings* out) {
  if (!h || !out) return Fail(SMX_INVALID_ARGUMENT, "null argument");
  std::lock_guard<std::mutex> lock(h->mu);   // RunSearch re-records the ring events
  *out = h->timings;
  out->scan_launches = 0;
  out->scan_ms_mode2 = 0.0f;
  if (!h->scan_ev.empty() && h->scan_logged) {
    // the latest min(logged, kScanLog) pairs; a pair not yet complete (the
    // caller has not synchronised) is not counted
    const uint64_t n = std::min<uint64_t>(h->scan_logged, kScanLog);
    double sum = 0.0;
    int32_t cnt = 0;
    for (uint64_t i = 0; i < n; ++i) {
      float ms = 0.0f;
      if (hipEventElapsedTime(&ms, h->scan_ev[2 * i], h->scan_ev[2 * i + 1]) == hipSuccess) {
        sum += ms;
        ++cnt;
      }
    }
    (void)hipGetLastError();
    out->scan_launches = cnt;
    out->scan_ms_mode2 = cnt ? float(sum / cnt) : 0.0f;
  }
  return SMX_OK;
}

int smx_set_tuning(smx_index* h, int32_t candidates_per_query, int32_t seed_leaves,
                   int32_t scan_variant, int32_t chunk_tiles) {
  if (!h) return Fail(SMX_INVALID_ARGUMENT, "null index");
#ifdef SMX_SCAN_DIAGNOSTICS
  if (scan_variant != 0 && scan_variant != 2 && scan_variant != 4 && scan_variant != 8 &&
      scan_variant != 16 && scan_variant != 32 && scan_variant != 64 &&
      scan_variant != 68)
    return Fail(SMX_INVALID_ARGUMENT,
                "scan_variant is 0 (scan), 2 / 4 / 16 / 32 / 64 / 68 (timing ablations) or 8 (diagnostic stamps)");
#else
  if (scan_variant != 0)
    return Fail(SMX_INVALID_ARGUMENT,
                "scan_variant must be 0: the ablations and stamps exist only in the diagnostic "
                "build (-DSMX_SCAN_DIAGNOSTICS)");
#endif
  if (chunk_tiles != 0 && (chunk_tiles < 8 || chunk_tiles > 65535))
    return Fail(SMX_INVALID_ARGUMENT, "chunk_tiles must be 0 (default) or in [8, 65535]");
  if (candidates_per_query != 0 && (candidates_per_query < 32 || candidates_per_query > 8192))
    return Fail(SMX_INVALID_ARGUMENT,
                "candidates_per_query must be 0 (sized per call) or in [32, 8192]");
  if (seed_leaves < 0) return Fail(SMX_INVALID_ARGUMENT, "seed_leaves must be >= 0");
  std::lock_guard<std::mutex> lock(h->mu);
  h->cap_per_query = uint32_t(candidates_per_query);
  h->seed_leaves = seed_leaves;
  h->scan_variant = scan_variant;
  if (chunk_tiles) h->chunk_tiles = uint32_t(chunk_tiles);
  return SMX_OK;
}

}  // extern "C"

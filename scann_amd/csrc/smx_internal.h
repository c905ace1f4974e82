// smx_internal.h — device-side index layout, kernel argument blocks and the
// launcher entry points shared by smx_kernels.hip and smx_searcher.hip.
#ifndef SMX_INTERNAL_H_
#define SMX_INTERNAL_H_

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

namespace smx {

// Query-tile width of the LUT16 scan: one MFMA i32_32x32x32_i8 covers 32
// datapoints x 32 queries x 2 AH blocks.
constexpr int kQueriesPerTile = 32;
// A leaf's last query tile with at most this many queries runs on the
// 16-slot path (v_smfmac_i32_16x16x128_i8); its work item is marked in the
// leaf field.
constexpr int kNarrowSlots = 16;
// WorklistArgs::totals[kTotalsTiles16]: the call's 16-slot tiles (stats[12])
constexpr int kTotalsTiles16 = 9;
// Each query's seed threshold ranks at most kSeedKeys seed distances
// (seed_tau_kernel; the threshold select's stage entry point takes sets of
// this size).
#ifndef SMX_SEED_PER_THREAD
#define SMX_SEED_PER_THREAD 16   // seed rows per query / 256 (a build-time knob)
#endif
constexpr int kSeedKeys = 256 * SMX_SEED_PER_THREAD;
constexpr uint32_t kItemNarrow = 1u << 31;
// WorklistArgs::narrow: 0 = 32-slot tiles only, kNarrowOnly = 16-slot tiles only
constexpr uint32_t kNarrowOnly = 2;
// 16-slot tiles (only) are used when a call averages fewer queries per leaf
// (nq * L / num_leaves) than this
constexpr int kNarrowQueriesPerLeaf = 32;
constexpr int kDpPerTile = 32;
constexpr int kMaxBlocks = 64;           // LUT16 blocks supported (K <= 32)
constexpr uint64_t kNoThreshold = ~0ull;
constexpr int kWorkGroups = 8;        // XCD groups of the scan's work list
// Per-leaf list counters and per-query candidate counters take a 128-byte
// line each: device-scope atomics on one line serialize, and 100k returning
// atomics over 1000 packed counters (32 lines) cost ~12 us where one line per
// counter costs ~1 us.  counter(i) = base[i * kCounterStride].
constexpr uint32_t kCounterStride = 32;

// LUT rows (16 int8 entries each) per query: the 2K blocks of the 32-slot
// scan, padded with zero rows to whole 8-block steps of the 16-slot scan
// (K = 26, glove: 52 -> 56).  Row b = AH block b; rows >= num_blocks are 0.
__host__ __device__ constexpr int LutRows(int ksteps) { return 8 * ((ksteps + 3) / 4); }

// Bytes of code data one lane holds per 32-datapoint tile: lane (r, h) keeps
// the nibbles of datapoint r for blocks h, h+2, h+4, ... (K = ceil(B/2)).
inline int LaneBytes(int ksteps) { return 4 * ((((ksteps + 1) / 2) + 3) / 4); }

// Code byte j of a lane holds the nibbles of its blocks x0 = 4j + h and
// x1 = 4j + 2 + h (one sparse MFMA step), encoded for the sparse operand:
// low nibble = the codes' groups of four, (x0 >> 2) | (x1 >> 2) << 2 (which
// compressed A values are 1), high nibble = their positions in the group,
// (x0 & 3) | (x1 & 3) << 2 (the index fields).  Every consumer decodes
// through these (the pair tables are indexed by the encoded byte).
__host__ __device__ inline uint32_t EncodeCodePair(uint32_t x0, uint32_t x1) {
  return ((x0 >> 2) | ((x1 >> 2) << 2)) | (((x0 & 3u) | ((x1 & 3u) << 2)) << 4);
}
__host__ __device__ inline uint32_t CodePairLo(uint32_t by) {   // x0
  return ((by & 3u) << 2) | ((by >> 4) & 3u);
}
__host__ __device__ inline uint32_t CodePairHi(uint32_t by) {   // x1
  return (by & 0xCu) | ((by >> 6) & 3u);
}

// Index resident in HBM (owned by the handle).
struct DeviceIndex {
  int metric = 0, dim = 0, nl = 0, nb = 0, dpb = 0, residual = 0;
  int ksteps = 0;        // ceil(nb / 2)
  int lane_bytes = 0;    // LaneBytes(ksteps)
  int shift = 0;         // global top-N shift, 0 = tie by global id
  // the dense-first 32-slot scan tile where the blocks fit it (LaunchWide);
  // set per handle at creation (SMX_DENSE_FIRST=0: the all-sparse tile)
  bool dense_first = true;
  uint32_t num_datapoints = 0;
  uint64_t num_members = 0;
  uint64_t num_tiles = 0;
  uint32_t max_leaf = 0;
  bool disjoint = true;
  float spill = 2.0f;
  float* centers = nullptr;     // [nl][dim]
  float* centers_t = nullptr;   // [dim][nl]
  float* cnorm = nullptr;       // [nl], squared L2 only
  float* codebook = nullptr;    // [nb][16][dpb]
  uint8_t* tiles = nullptr;     // [num_tiles][64 lanes][lane_bytes]
  uint64_t* tile_off = nullptr; // [nl+1]
  uint32_t* leaf_size = nullptr;// [nl]
  uint64_t* member_off = nullptr; // [nl+1]
  uint32_t* members = nullptr;  // [num_members]
  uint32_t* leaf_order = nullptr; // [nl] leaves by descending size
  float* dataset = nullptr;     // [num_datapoints][dim] or null
  uint32_t* row_base = nullptr; // [nl] shard's first row in each whole leaf, or null
  float* member_rows = nullptr; // [num_members][dim] shard rows for the reorder, or null
  // with member_rows: [num_datapoints] global id -> a member slot holding it
  // (0xFFFFFFFF: not in this shard); the reorder row of a candidate known by
  // its global id (ties by global id, shift 0; the block select's gid space)
  uint32_t* row_of = nullptr;
};

// smx_shard_entry (include/scann_mi355x.h)
struct ShardEntry {
  uint64_t key;
  uint32_t id;
  float exact;
};

// Sizes of the per-call buffers and of the index, for the index checks of
// the debug build (-DSMX_DEBUG_CHECKS: every computed index into them is
// verified before the access, a violation is counted and reported by the
// host as SMX_INTERNAL; the product library compiles the checks out).
struct Bounds {
  uint32_t nq = 0;          // queries of the call
  uint32_t items = 0;       // work items the workspace holds
  uint32_t grid = 0;        // scan workgroups (wave_start entries)
  uint32_t nl = 0;          // leaves
  uint32_t datapoints = 0;  // dataset rows
  uint32_t recs = 0;        // leaf slots (leaf_pair entries: nl x the call's slot stride)
  uint32_t pairs = 0;       // (query, leaf) pairs (pair_rec entries)
  uint64_t members = 0;     // leaf members (members[], member_rows)
  uint64_t tiles = 0;       // code tiles
};

// One work item of the scan: a chunk [j0, jend) of the 32-datapoint tiles of
// a leaf, for one query tile (32 slots, or 16 with kItemNarrow set in `leaf`)
// of that leaf's query list.
struct WorkItem {
  uint32_t leaf;         // | kItemNarrow for a 16-slot query tile
  uint32_t n;            // leaf size (datapoints)
  uint32_t j0, jend;     // tile range
  uint64_t tile_off;     // the leaf's first code tile
  uint64_t member_off;   // the leaf's first member
  uint32_t slot0;        // the query tile's first leaf slot (leaf_pair index)
  uint32_t nslots;       // its filled slots (the rest of the tile is empty)
};

// Per (query, leaf) pair p = query * L + i: the query (kNoQuery for an empty
// slot), the partition distance (residual bias), the query's 1/multiplier
// and the pair's sum limit -- the largest LUT16 sum whose distance can pass
// the query's seed threshold.  One dwordx4, written by the query's seed block
// once its threshold is known; the scan reads a query tile's slots through
// leaf_pair (leaf slot -> pair, written by the top-L kernel with the rank).
struct ItemLane {
  uint32_t qid;
  float bias;
  float inv;
  int32_t amax;   // the pair's sum limit
};
constexpr uint32_t kNoQuery = 0xFFFFFFFFu;     // ItemLane::qid of an empty slot

constexpr int32_t kNoSum = -2147483647 - 1;   // the sum limit of an empty slot

struct ScanArgs {
  const uint8_t* tiles;
  const uint32_t* members;
  const int8_t* lut;          // [nq][2K][16]
  const float* inv;           // [nq]
  const WorkItem* work;       // [work items]
  const uint32_t* leaf_pair;  // [nl][slot stride] leaf slot -> pair
  const ItemLane* pair_rec;   // [nq][L] per-pair records
  uint32_t chunk_tiles;
  const uint4* wave_start;    // [grid] {first item, first tile, tiles, first position}
  uint32_t num_items;
  const uint64_t* tau_key;    // [nq] emission threshold keys
  uint64_t* cand;             // [nq][cap]
  uint32_t* cand_count;       // [nq] strided (kCounterStride)
  unsigned long long* stamps; // diagnostic variant 8 only: [cap][8] per-item stamps
  uint32_t* stamp_count;
  uint32_t stamp_cap;
  uint32_t cap;
  int nl;
  int nb;
  int shift;
  Bounds bd;                  // debug-build index checks
};

struct SeedArgs {
  const int32_t* topl_leaf;   // [nq][L]
  const float* topl_dist;     // [nq][L]
  int nl;
  ItemLane* pair_rec;         // [nq][L] every pair's record, with its sum limit
  const int8_t* lut;          // [nq][2K][16]
  const float* inv;
  const uint8_t* tiles;
  const uint64_t* tile_off;
  const uint32_t* leaf_size;
  uint64_t* tau_key;
  int L;
  int seed;
  int seed_rows;              // rows scored per query (<= kSeedKeys)
  int kk;
  int residual;
  int nb;
  Bounds bd;                  // debug-build index checks
};

// The work list's inputs and outputs (LaunchWorklist / the fused block of
// LaunchSeed).
struct WorklistArgs {
  const uint32_t* cnt;         // per-leaf query counts (kCounterStride apart)
  const uint32_t* order;       // leaf positions in work order
  const uint32_t* leaf_size;
  const uint64_t* tile_off;
  const uint64_t* member_off;
  int nl;
  int nb;
  uint32_t chunk_tiles;
  int grid;                    // scan workgroups
  uint32_t narrow;             // kNarrowOnly: 16-slot query tiles, 0: 32-slot
  uint32_t* leaf_item0;        // [nl]
  uint32_t* pos_unit0;         // [nl + 1]
  uint32_t* gunits;            // [9]
  uint32_t* totals;            // [3] pairs, items, units; [kTotalsTiles16] 16-slot tiles
  unsigned long long* code_bytes;
  WorkItem* work;
  uint32_t slot_stride;        // leaf slots per leaf in leaf_pair (the call's nq)
  uint4* wave_start;           // [grid]
  Bounds bd;                  // debug-build index checks
};
// 64-bit words of one work-list block's sums (WorklistPart: items, units,
// pairs, code bytes, 16-slot tiles).
constexpr int kWorklistPartWords = 5;
// Up to this many leaves the work list is built by one extra block of the
// seed launch (no second stream, no fork/join); above it by three launches.
constexpr int kFusedWorklistLeaves = 4096;

// An overflowed query's rescan (RescanQuery, inside the select kernels):
// the query's leaves, LUT and lists, and the code layout of the index.
struct RescanArgs {
  const int32_t* topl_leaf;   // [nq][L]
  const float* topl_dist;
  int L;
  int residual;
  int ksteps;
  const int8_t* lut;          // [nq][2K][16]
  const float* inv;
  const uint8_t* tiles;
  const uint64_t* tile_off;
  const uint32_t* leaf_size;
  const uint32_t* members;
  const uint64_t* member_off;
  int shift;
  uint64_t* cand;
  uint32_t* cand_count;       // strided
  uint64_t* tau_key;
  uint32_t cap;
  int kk;
  uint32_t* stats;            // [10] queries rescanned [11] rescan rounds
  Bounds bd;                  // debug-build index checks
};

struct SelectArgs {
  const uint64_t* cand;
  uint32_t* cand_count;       // (rewritten by an overflow rescan)
  uint32_t cap;
  int kk;                     // k' kept before dedupe
  int pre_nn;                 // kept after SOAR dedupe
  int final_nn;
  int reorder;
  int disjoint;
  int pre_only;               // output the pre-reorder set (stage entry)
  int shift;
  int metric;
  int dim;
  const uint64_t* member_off;
  const uint32_t* members;
  const float* dataset;
  const float* queries;
  uint32_t* out_idx;
  float* out_dist;
  int32_t* out_count;
  int out_width;
  uint32_t* overflow;         // stats: [0] flag [1] max overflow [2] max count [8] sum
  int stats;                  // also compute [2] and [8] (profiled calls)
  RescanArgs rescan;          // overflowed lists are rescanned in the select kernels
  ShardEntry* shard_out;      // shard mode: [nq][kk] local top-k' entries (or NULL)
  const uint32_t* row_base;   // shard: whole-leaf row of each leaf's first shard row
  const float* member_rows;   // shard: [members][dim] rows for the exact distances
  const uint32_t* row_of;     // shard with member_rows: global id -> member slot
  Bounds bd;                  // debug-build index checks
};

struct MergeArgs {
  const ShardEntry* entries;  // [world][nq][kk], each list sorted by key
  int world;
  int nq;
  int kk;
  int pre_nn;
  int disjoint;
  int reorder;
  uint32_t* out_idx;
  float* out_dist;
  int32_t* out_count;
  int out_width;
  ShardEntry* out_entries;    // partial rounds of the wide merge (set by the launcher)
  ShardEntry* scratch[2];     // the wide merge's round buffers (MergeScratchEntries each)
};

// ---- launchers (smx_kernels.hip) ------------------------------------------
// Per-call state the partition kernel resets on its way (no memset nodes):
// counters to 0, candidate counts to 0, thresholds to "open".
struct StateInit {
  uint32_t* counters = nullptr;     // n_counters strided leaf counters
  uint32_t n_counters = 0;
  uint32_t* stats = nullptr;        // n_stats packed words
  uint32_t n_stats = 0;
  uint32_t* cand_count = nullptr;   // n_cand strided counters
  uint32_t n_cand = 0;
  uint64_t* tau = nullptr;
  uint32_t n_tau = 0;
};
// The search's front end: the state reset, each (query, leaf) pair's rank in
// the leaf's list (atomics on leaf_count) and the query's LUT16 table, all in
// the partition / top-L launches.  NULL members are skipped.
struct FrontArgs {
  StateInit init;
  uint32_t* leaf_count = nullptr;   // [nl] strided (kCounterStride), zeroed by init
  uint32_t* leaf_pair = nullptr;    // [nl][slot_stride]: each pair at its leaf's slot (its rank)
  uint32_t slot_stride = 0;
  int8_t* lut = nullptr;            // [nq][2K][16]
  float* mult = nullptr;            // [nq]
  float* inv = nullptr;             // [nq]
  int one_to_many = 0;              // the single-query partition scores (A.8 order)
};
hipError_t LaunchPartitionTopL(const DeviceIndex& ix, const float* queries, int nq,
                               int L, int32_t* out_leaf, float* out_dist,
                               float* scores /*[nq][nl] scratch*/, hipStream_t s,
                               const FrontArgs* front = nullptr);
hipError_t LaunchLutBuild(const DeviceIndex& ix, const float* queries, int nq,
                          int8_t* lut, float* mult, float* inv, uint8_t* lut_u8,
                          hipStream_t s);
// Leaf lists -> the scan's work items (8 XCD groups of equal MFMA work,
// each item with its query tile's leaf slots), each leaf's first item and
// every scan wave's static share of its group's tiles (three launches).
hipError_t LaunchWorklist(const DeviceIndex& ix, const uint32_t* leaf_count,
                          WorkItem* work /*[max items]*/, uint32_t* leaf_item0 /*[nl]*/,
                          uint32_t* pos_unit0 /*[nl+1]*/, uint32_t* gunits /*[9]*/,
                          uint32_t slot_stride, uint4* wave_start /*[grid]*/,
                          int grid, uint32_t* totals /*[3]*/,
                          unsigned long long* code_bytes /*[1]*/, uint32_t chunk_tiles,
                          uint32_t narrow,
                          unsigned long long* part /*[kWorklistPartWords * ceil(nl / 256)]*/,
                          const Bounds& bd, hipStream_t s);
// variant 0: the LUT16 scan (lut16_scan_kernel; `narrow`: the work list
// holds 16-slot items); 4: the same without its threshold epilogue (timing
// ablation, results invalid; the diagnostic variants take 32-slot items only).
// e0 / e1 (or NULL): timing events recorded by the scan's own dispatch.
hipError_t LaunchScan(const DeviceIndex& ix, const ScanArgs& a, int grid, int variant,
                      hipStream_t s, uint32_t narrow, hipEvent_t e0 = nullptr,
                      hipEvent_t e1 = nullptr);
// Resident scan workgroups per CU (occupancy of the index's instantiation).
hipError_t ScanBlocksPerCU(const DeviceIndex& ix, int* blocks);
// The per-query thresholds (tau_key) from the seed leaves.
WorklistArgs MakeWorklistArgs(const DeviceIndex& ix, const uint32_t* leaf_count, WorkItem* work,
                              uint32_t* leaf_item0, uint32_t* pos_unit0, uint32_t* gunits,
                              uint32_t slot_stride, uint4* wave_start, int grid, uint32_t* totals,
                              unsigned long long* code_bytes, uint32_t chunk_tiles,
                              uint32_t narrow, const Bounds& bd);
// The seed thresholds and every pair's record (one block per query); with
// `wl`, more blocks build the whole work list (ix.nl <= kFusedWorklistLeaves).
// e0 / e1 (or NULL): timing events recorded by the kernel's own dispatch.
hipError_t LaunchSeed(const DeviceIndex& ix, const SeedArgs& a, int nq, hipStream_t s,
                      const WorklistArgs* wl = nullptr, hipEvent_t e0 = nullptr,
                      hipEvent_t e1 = nullptr);
hipError_t LaunchKthKeys(const uint32_t* vals, int sets, int kk, uint64_t* out, hipStream_t s);
// The rank kernel (one block per query, <= kSelMax keys in LDS) for k' <=
// kSelMax, the block kernel otherwise; both rescan overflowed lists first.
hipError_t LaunchFinalSelect(const SelectArgs& a, int nq, hipStream_t s,
                             hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
// Whether the final selection of these arguments fits the CU's 160 KiB LDS
// (static + dynamic; the block kernel for k' > kSelMax holds the whole list).
bool FinalSelectFits(const SelectArgs& a);
// Nearest center per row, or the SOAR secondary center with `primary`
// (smx_builder.hip).
hipError_t LaunchNearestCenters(const float* x, int64_t n, int d, const float* centers, int k,
                                const int32_t* primary, float lambda, int32_t* out,
                                float* out_loss, hipStream_t s);
// Index-build kernels (smx_builder.hip, smx_sort.hip).
hipError_t LaunchBlockEncode(const float* r, int64_t n, int dim, const float* cb, int nb, int dpb,
                             uint8_t* out, hipStream_t s);
hipError_t LaunchKmeansAccumulate(const float* x, int64_t n, int d, const int32_t* label, int k,
                                  double scale, unsigned long long* sums, uint32_t* counts,
                                  hipStream_t s);
hipError_t LaunchKmeansFinalize(const unsigned long long* sums, const uint32_t* counts, int k,
                                int d, double scale, float* centers, hipStream_t s);
size_t CodebookAccumulateLds(int nb, int dpb);
hipError_t LaunchCodebookAccumulate(const float* r, int64_t n, int dim, const uint8_t* codes,
                                    int nb, int dpb, double scale, unsigned long long* sums,
                                    uint32_t* counts, hipStream_t s);
size_t AvqEncodeLds(int nb, int dpb);
hipError_t LaunchAvqEncode(const float* resid, const float* orig, int64_t n, int dim,
                           const float* cb, int nb, int dpb, double threshold, uint8_t* out,
                           hipStream_t s);
// Members grouped by leaf: sort (leaf, id) pairs, then the leaf offsets.
hipError_t GroupByLeaf(const int32_t* labels, const uint32_t* ids, int64_t m, int k, void* temp,
                       size_t* temp_bytes, uint64_t* keys, uint64_t* offsets, uint32_t* members,
                       int32_t* member_leaf, hipStream_t s);
hipError_t LaunchGatherResiduals(const float* x, int d, const uint32_t* rows, const int32_t* leaf,
                                 const float* centers, int64_t m, int64_t row_base, float* out,
                                 hipStream_t s);
hipError_t LaunchMergeShards(const MergeArgs& a, hipStream_t s);
// Entries of each of the wide merge's two round buffers (0: none needed).
size_t MergeScratchEntries(int world, int nq, int kk);
hipError_t LaunchExactDistances(const DeviceIndex& ix, const float* queries, int nq,
                                const uint32_t* ids, int k, float* out, hipStream_t s);
hipError_t LaunchLeafScores(const DeviceIndex& ix, int leaf, const int8_t* lut,
                            int32_t* out, hipStream_t s);
// Diagnostic build only (-DSMX_PHASE_STAMPS): where the phase stamps go
// ([3 kernels][kPhaseQueries][8] u64, or NULL).
constexpr int kPhaseQueries = 4096;
hipError_t SetPhaseStamps(unsigned long long* p);
// Debug build only (-DSMX_DEBUG_CHECKS): index-check violations counted on
// the device since the last call (reset to 0); always 0 in the product build.
hipError_t TakeCheckFailures(unsigned int* out);
hipError_t LaunchFill64(uint64_t* p, uint64_t v, size_t n, hipStream_t s);
// row_of[members[m]] = m for every member slot m (row_of pre-filled).
hipError_t LaunchRowOf(const uint32_t* members, uint64_t m, uint32_t* row_of, hipStream_t s);

}  // namespace smx

#endif  // SMX_INTERNAL_H_

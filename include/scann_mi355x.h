/*
 * scann_mi355x.h — C ABI of the MI355X tree-AH / LUT16 query path.
 *
 * This is the drop-in boundary for the reference's batched search seam
 * (SURVEY.md §8b).  One call replaces, for a whole query batch:
 *   TreeAHHybridResidual::FindNeighborsBatchedImpl
 *       (scann/tree_x_hybrid/tree_ah_hybrid_residual.cc:631-846)
 *   TreeXHybridSMMD::FindNeighborsBatchedImpl for non-residual indexes
 *       (scann/tree_x_hybrid/tree_x_hybrid_smmd.cc:565-669, 718-790)
 *   followed by the exact reorder and SortAndDropResults of
 *   SingleMachineSearcherBase<float>::FindNeighborsBatched
 *       (scann/base/single_machine_base.cc:570-587, 849-901)
 * and is what ScannInterface::SearchBatched (scann/scann_ops/cc/scann.cc:463-475)
 * would call in place of scann_->FindNeighborsBatched.
 *
 * Conventions
 *  - Plain pointers and sizes only.  Host buffers passed in are borrowed and
 *    copied; device buffers are owned by the index handle.
 *  - Every function returns SMX_OK (0) or a negative smx_status; the message
 *    of the last failure on the calling thread is smx_last_error().  Nothing
 *    throws across the ABI (the reference maps Status to RuntimeError at its
 *    pybind layer, scann_npy.cc:41-55; the Python mirror does the same).
 *  - Distances are returned in the reference's internal convention (smaller
 *    is better; -dot for dot product).  The x(-1) of ReshapeBatchedNNResult
 *    (scann/scann_ops/cc/scann.h:162-180) is applied by the caller.
 *  - Calls on one handle may come from several host threads; their host
 *    side is serialised by the handle's mutex (re-entrant per the
 *    reference's const FindNeighbors*Impl, SURVEY.md §8b "Threading"), and
 *    each stream gets its own per-call workspace (up to 4 streams), so work
 *    enqueued on different streams runs concurrently on the device.
 *  - Device code targets gfx950 (MI355X) only.
 */
#ifndef SCANN_MI355X_H_
#define SCANN_MI355X_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum smx_status {
  SMX_OK = 0,
  SMX_INVALID_ARGUMENT = -1,   /* InvalidArgumentError  */
  SMX_FAILED_PRECONDITION = -2,/* FailedPreconditionError */
  SMX_DEVICE_ERROR = -3,       /* HIP runtime failure   */
  SMX_OUT_OF_MEMORY = -4,
  SMX_INTERNAL = -5
} smx_status;

enum { SMX_METRIC_DOT = 0, SMX_METRIC_SQUARED_L2 = 1 };

/* Index description.  Replaces the state TreeAHHybridResidual builds in
 * BuildLeafSearchers (tree_ah_hybrid_residual.cc:325-495) / the assets
 * ScannInterface::LoadArtifacts reads (scann.cc:105-264):
 *   centers        <- the k-means tree leaf centers (serialized_partitioner.pb)
 *   codebook       <- ah_codebook.pb, [num_blocks][16][dims_per_block]
 *   leaf_offsets/leaf_members <- datapoints_by_token_ (ascending ids per leaf)
 *   member_codes   <- hashed_dataset(.npy / _soar.npy), one row per member
 *   dataset        <- dataset.npy (exact reordering), may be NULL
 * A datapoint may be a member of several leaves (SOAR spilling); results are
 * then de-duplicated as in DeduplicateDatabaseSpilledResults
 * (tree_x_hybrid/internal/utils.cc:135-162). */
typedef struct smx_index_desc {
  int32_t metric;           /* SMX_METRIC_*                                   */
  int32_t dim;
  int32_t num_leaves;
  int32_t num_blocks;       /* AH subspaces; LUT16 requires <= 64 here        */
  int32_t dims_per_block;   /* last block covers dim-(num_blocks-1)*dpb dims  */
  int32_t residual;         /* 1: residual tree-AH, global top-N (pipeline A) */
  const float* centers;     /* [num_leaves][dim]                              */
  const float* codebook;    /* [num_blocks][16][dims_per_block]               */
  const uint64_t* leaf_offsets; /* [num_leaves+1]                             */
  const uint32_t* leaf_members; /* [leaf_offsets[num_leaves]]                 */
  const uint8_t* member_codes;  /* [members][num_blocks], values 0..15         */
  uint32_t num_datapoints;
  const float* dataset;     /* [num_datapoints][dim] or NULL                  */
  float spilling_overretrieve_factor; /* tree_ah_hybrid_residual.h:320 (2.0) */
  int32_t reserved;
  /* Range-split shard of a whole index: the shard holds
   * rows [leaf_row_base[l], leaf_row_base[l] + size) of every full leaf l, so
   * that tie keys stay the whole index's (leaf << shift | row).  Zero for a
   * whole index (then nothing below is read). */
  int32_t is_shard;
  int32_t global_topn_shift;      /* the whole index's shift (smx_index_info)  */
  int32_t global_spilled;         /* 1 if the whole index has SOAR duplicates  */
  int32_t reserved2;
  const uint32_t* leaf_row_base;  /* [num_leaves]                              */
  const float* member_rows;       /* [members][dim] rows of this shard for the
                                     exact reorder (global top-N indexes), or
                                     NULL: `dataset` by global id              */
} smx_index_desc;

/* One entry of a shard's local top-k' list: key = ordered approximate
 * distance << 32 | whole-index tie (UINT64_MAX pads an unused entry), the
 * global datapoint id and the exact distance (the approximate one when the
 * search does not reorder). */
typedef struct smx_shard_entry {
  uint64_t key;
  uint32_t id;
  float exact;
} smx_shard_entry;

typedef struct smx_index smx_index;

/* Per-call search parameters.  Mirrors SearchParameters as produced by
 * ScannInterface::GetSearchParametersBatched (scann.cc:406-430):
 * leaves_to_search -> TreeXOptionalParameters::num_partitions_to_search_override,
 * pre_reorder_nn / final_nn -> pre/post_reordering_num_neighbors.
 * All three must be > 0 (defaults are resolved by the caller, as
 * SetUnspecifiedParametersToDefaults does, single_machine_base.cc:120). */
typedef struct smx_search_params {
  int32_t leaves_to_search;
  int32_t pre_reorder_nn;   /* ignored (= final_nn) when reorder is off       */
  int32_t final_nn;
  int32_t reorder;          /* 1: exact reorder with the float dataset        */
} smx_search_params;

/* Stage timings of the last search on a handle (ms; filled only when
 * profiling was enabled with smx_set_profiling(index, 1), which makes every
 * call synchronous).  The seed, scan and select stages are timed by events in
 * the kernels' own dispatch packets (their execution, as rocprofv3 reports
 * it); partition + top-L by HIP events recorded on the stream around the
 * launches.  smx_set_profiling(index, 2) instead records two events
 * around every scan launch of the calls that follow, without synchronising
 * (up to 4096 launches, the latest kept): smx_get_timings then reports
 * their count and mean duration (scan_launches, scan_ms_mode2) once the
 * caller has synchronised the device. */
typedef struct smx_timings {
  float partition_ms;
  float lut_ms;
  float invert_ms;
  float seed_scan_ms;
  float seed_select_ms;
  float scan_ms;            /* main LUT16 scan kernel                        */
  float select_ms;          /* final top-k + SOAR dedupe + reorder + sort    */
  float total_ms;
  double scan_code_bytes;   /* algorithmic bytes of the main scan launch:
                               sum over its (query, leaf) pairs of
                               16 * num_blocks * ceil(leaf_size / 32)        */
  double seed_code_bytes;
  int32_t scan_pairs;       /* (query, leaf) pairs in the main launch        */
  int32_t seed_pairs;
  int32_t overflow_retries; /* candidate-buffer tightening passes            */
  int32_t max_candidates;   /* largest per-query survivor count              */
  double scan_item_tiles;   /* 32-slot tiles of the main scan
                               (x K/2 v_smfmac_i32_32x32x64_i8)              */
  float mean_candidates;    /* survivors per query (last pass)               */
  int32_t scan_workgroups;  /* persistent scan grid (one wave each)          */
  double scan_item_tiles16; /* 16-slot tiles of the main scan
                               (x 2*ceil(K/4) v_smfmac_i32_16x16x128_i8)     */
  int32_t scan_launches;    /* profiling mode 2: scan launches averaged into
                               scan_ms_mode2                                 */
  float scan_ms_mode2;      /* profiling mode 2: mean duration of those scan
                               launches (HIP events on each call's stream,
                               no synchronisation: batches stay in flight)   */
} smx_timings;

/* Index lifecycle (ScannNumpy ctor / destructor; scann_npy.cc:57-77). */
int smx_index_create(const smx_index_desc* desc, int32_t device, smx_index** out);
int smx_index_destroy(smx_index* index);
int smx_index_info(const smx_index* index, int32_t* dim, int32_t* num_leaves,
                   uint32_t* num_datapoints, int32_t* global_topn_shift);

/* Batched search with host buffers (ScannNumpy::SearchBatched,
 * scann_npy.cc:233-270).  queries: [nq][dim] float32 row-major (host).
 * out_idx / out_dist: [nq][final_nn] (host), padded with id 0 / NaN as
 * ReshapeBatchedNNResult does; out_count: [nq] (host, may be NULL). */
int smx_search_batched(smx_index* index, const float* queries, int32_t nq,
                       int32_t dim, const smx_search_params* params,
                       uint32_t* out_idx, float* out_dist, int32_t* out_count);

/* Same with device buffers, enqueued on `stream` (hipStream_t; NULL = the
 * handle's own stream) with no host synchronisation: the results are ready
 * when the stream reaches them (candidate-list overflow is handled on the
 * device).  Calls on different streams run concurrently (one workspace per
 * stream, up to 4; a fifth stream reuses the oldest one after waiting for
 * its work).  d_out_count may be NULL.  A batch of any size is accepted: it
 * runs as sub-batches of at most 2^26 / num_leaves queries (the leaf-slot
 * table's budget, 256 MB per stream), one after another on the stream.
 * A stream passed here (or to the other *_device search calls) must stay
 * valid until smx_release_stream(index, stream) or smx_index_destroy: the
 * handle orders a later call on another stream after it. */
int smx_search_batched_device(smx_index* index, const float* d_queries, int32_t nq,
                              int32_t dim, const smx_search_params* params,
                              uint32_t* d_out_idx, float* d_out_dist,
                              int32_t* d_out_count, void* stream);

/* Waits for the work the handle enqueued on `stream` and frees that stream's
 * workspace (no-op for a stream the handle has not searched on), after which
 * the caller may destroy the stream.  NULL = the handle's own stream. */
int smx_release_stream(smx_index* index, void* stream);

/* Single-query search (ScannNumpy::Search / ScannInterface::Search,
 * scann_npy.cc, scann.cc; TreeAHHybridResidual::FindNeighborsImpl,
 * tree_ah_hybrid_residual.cc:870-978) with host buffers: one query [dim],
 * out_idx / out_dist [final_nn].  Its partition scores follow the
 * single-query path's one-to-many order (kmeans_tree_node.h:159-163 ->
 * one_to_many_symmetric.h:376-503), not the batched transposed chain, so its
 * leaf biases -- and at exact ties its neighbors -- are those of the
 * reference's search(), not of search_batched(). */
int smx_search(smx_index* index, const float* query, int32_t dim,
               const smx_search_params* params, uint32_t* out_idx, float* out_dist,
               int32_t* out_count);

/* ---- range-split shards -------------------------------
 * Each rank searches its shard, producing its exact local top-k' by (approx
 * distance, whole-index tie) with exact distances of its own rows; the
 * ranks' lists are all-gathered (one collective, [world][nq][k'] entries) and
 * merged.  The exact top-k' under a total order is shard-invariant, so the
 * merged result equals the unsharded search. */

/* k' (entries per query) of a shard search with these params. */
int smx_shard_width(const smx_index* index, const smx_search_params* params, int32_t* out_k);

/* This shard's local lists, device buffers on `stream`: d_entries [nq][k']. */
int smx_search_shard_device(smx_index* index, const float* d_queries, int32_t nq, int32_t dim,
                            const smx_search_params* params, smx_shard_entry* d_entries,
                            void* stream);

/* Merge of `world` shards' lists d_entries [world][nq][k'] (any shard's
 * handle; it supplies the spill/dedupe setting): SOAR de-duplication by id,
 * then the (distance, id) order of SortAndDropResults; outputs as
 * smx_search_batched_device. */
int smx_merge_shards_device(smx_index* index, int32_t world, int32_t nq,
                            const smx_search_params* params, const smx_shard_entry* d_entries,
                            uint32_t* d_out_idx, float* d_out_dist, int32_t* d_out_count,
                            void* stream);

/* ---- stage entry points (used by the parity tests; host buffers) ------- */

/* Query tokenization: top-L leaves per query by partition distance, sorted by
 * (distance, leaf id) — KMeansTreePartitioner::TokensForDatapointWithSpillingBatched
 * (scann/partitioning/kmeans_tree_partitioner.cc:643-730) with the transposed
 * many-to-many numerics (many_to_many_impl.inc:522-560).  [nq][L] outputs. */
int smx_partition_topl(smx_index* index, const float* queries, int32_t nq,
                       int32_t L, int32_t* out_leaf, float* out_dist);

/* Per-query LUT16 tables — AsymmetricQueryer::CreateLookupTable
 * (scann/hashes/asymmetric_hashing2/querying.h:284-329) +
 * ConvertLookupToFixedPoint<uint8_t> (asymmetric_hashing_impl.cc:571-645).
 * out_lut: [nq][num_blocks][16] uint8 (biased by 128); out_mult: [nq]. */
int smx_create_lookup_tables(smx_index* index, const float* queries, int32_t nq,
                             uint8_t* out_lut, float* out_mult);

/* Pre-reorder candidates (global ids) — the NNResultsVector
 * FindNeighborsBatchedNoSortNoExactReorder produces, sorted by (distance,
 * id).  k' = pre_nn (x overretrieve factor before SOAR dedupe).
 * Outputs [nq][pre_nn] padded with 0 / NaN. */
int smx_search_pre_reorder(smx_index* index, const float* queries, int32_t nq,
                           int32_t leaves, int32_t pre_nn, uint32_t* out_idx,
                           float* out_dist, int32_t* out_count);

/* Exact distances of given rows (the reorder kernel alone;
 * one_to_many_symmetric.h:373-503).  ids: [nq][k]; out [nq][k]. */
int smx_exact_distances(smx_index* index, const float* queries, int32_t nq,
                        const uint32_t* ids, int32_t k, float* out_dist);

/* Raw LUT16 accumulation on one leaf: Sum_b (lut[b][code]-128) for every
 * member of `leaf` against one uint8 LUT [num_blocks][16] — the integer core
 * of LUT16Avx2::GetTopFloatDistances (lut16_avx2.inc:55-124).  out: [leaf size]. */
int smx_lut16_leaf_scores(smx_index* index, int32_t leaf, const uint8_t* lut,
                          int32_t* out_scores);

/* The seed threshold select on its own (device buffers, enqueued on `stream`):
 * for each of `sets` sets of 4096 order-preserving distance bits (uint32,
 * 0xFFFFFFFF = no value), out[i] = (v << 32) | 0xFFFFFFFF for v the kk-th
 * smallest value of set i, or ~0 when it holds fewer than kk values -- the
 * pruning bound a query's first leaves give its scan, the role of the
 * running top-k threshold of the reference's TopNeighbors
 * (scann/utils/fast_top_neighbors.h) before the scan starts. */
int smx_kth_threshold_keys(const uint32_t* d_vals, int32_t sets, int32_t kk, uint64_t* d_out,
                           void* stream);

/* ---- index build (device buffers, enqueued on `stream`) ----------------- */

/* Nearest center of every row: out[i] = argmin_j ||x_i - c_j||^2 (ties to the
 * lowest j) — the assignment step of k-means training, GmmUtils::KMeansImpl
 * (scann/utils/gmm_utils.cc:539-1318).  With `primary` (one center per row,
 * device int32) the SOAR secondary assignment instead
 * (kmeans_tree_partitioner.cc:926-997): argmin over j != primary_i of
 * ||x_i - c_j||^2 + lambda <r_i, x_i - c_j>^2 / ||r_i||^2, r_i = x_i -
 * c_primary_i.  x: [n][d], centers: [k][d] float32; out: [n] int32;
 * out_loss: [n] float32 (the winning loss; the k-means form omits ||x_i||^2)
 * or NULL. */
int smx_nearest_centers(const float* d_x, int64_t n, int32_t d, const float* d_centers,
                        int32_t k, const int32_t* d_primary, float lambda, int32_t* d_out,
                        float* d_out_loss, void* stream);

/* The rest of the index build on the device (scann_amd/device_builder.py
 * drives them; device buffers, enqueued on `stream`):
 *
 * smx_block_encode: codes[i][b] = the nearest of block b's 16 codebook
 *   centers to rows[i]'s block b (squared L2 over the block's coordinates in
 *   order, the last block zero-padded, ties to the lowest center) -- the AH
 *   encoding of IndexDatapoint (asymmetric_hashing_impl.cc).  rows [n][dim],
 *   codebook [nb][16][dpb] float32, codes [n][nb] uint8.
 * smx_avq_encode: the anisotropic noise-shaped codes of
 *   IndexDatapointNoiseShaped (asymmetric_hashing_impl.cc:434-503) with the
 *   given noise_shaping_threshold: residuals and the datapoints themselves
 *   [n][dim]; double precision, bit for bit the oracle's orc_avq_encode.
 * smx_kmeans_accumulate / smx_kmeans_finalize: the k-means mean step
 *   (gmm_utils.cc:539-1318) as exact fixed-point sums: sums[label][j] +=
 *   llrint(x[i][j] * scale), counts[label]++ (int64 / uint32 device arrays
 *   zeroed by the caller; scale a power of two small enough that no sum
 *   overflows), then centers[c] = sums[c] / scale / counts[c] for every
 *   non-empty c (empty centers keep their values).  Order-independent, so
 *   deterministic run to run.
 * smx_codebook_accumulate: the same mean step for all blocks' 16-center
 *   codebooks at once (asymmetric_hashing_impl.cc:41-198): sums[nb][16][dpb],
 *   counts[nb][16], from rows [n][dim] and their codes [n][nb].
 * smx_group_by_leaf: members by (leaf, id) -- datapoints_by_token
 *   (kmeans_tree_partitioner.cc:477-620) -- from m (label, id) pairs: keys
 *   [2 m] uint64 scratch, offsets [k + 1] uint64, members [m] uint32,
 *   member_leaf [m] int32.  Call first with temp = NULL to get temp_bytes.
 * smx_gather_residuals: out[i] = x[rows[i] - row_base] - centers[leaf[i]]
 *   (float32), or the row itself when centers is NULL. */
int smx_block_encode(const float* d_rows, int64_t n, int32_t dim, const float* d_codebook,
                     int32_t num_blocks, int32_t dims_per_block, uint8_t* d_codes, void* stream);
int smx_avq_encode(const float* d_residuals, const float* d_datapoints, int64_t n, int32_t dim,
                   const float* d_codebook, int32_t num_blocks, int32_t dims_per_block,
                   double threshold, uint8_t* d_codes, void* stream);
int smx_kmeans_accumulate(const float* d_x, int64_t n, int32_t d, const int32_t* d_label,
                          int32_t k, double scale, uint64_t* d_sums, uint32_t* d_counts,
                          void* stream);
int smx_kmeans_finalize(const uint64_t* d_sums, const uint32_t* d_counts, int32_t k, int32_t d,
                        double scale, float* d_centers, void* stream);
int smx_codebook_accumulate(const float* d_rows, int64_t n, int32_t dim, const uint8_t* d_codes,
                            int32_t num_blocks, int32_t dims_per_block, double scale,
                            uint64_t* d_sums, uint32_t* d_counts, void* stream);
int smx_group_by_leaf(const int32_t* d_labels, const uint32_t* d_ids, int64_t m, int32_t k,
                      void* d_temp, size_t* temp_bytes, uint64_t* d_keys, uint64_t* d_offsets,
                      uint32_t* d_members, int32_t* d_member_leaf, void* stream);
int smx_gather_residuals(const float* d_x, int32_t d, const uint32_t* d_rows,
                         const int32_t* d_leaf, const float* d_centers, int64_t m,
                         int64_t row_base, float* d_out, void* stream);

/* ---- diagnostics ---------------------------------------------------------- */
/* 0: off; 1: per-call stage timings (synchronous calls); 2: scan-launch
 * durations of the calls in flight (see smx_timings). */
int smx_set_profiling(smx_index* index, int32_t enabled);
int smx_get_timings(const smx_index* index, smx_timings* out);
/* Tuning knobs: candidate buffer capacity per query (0, the default: sized
 * per call from k', leaves_to_search and the seed leaves), seed leaves used for the
 * per-query threshold, scan kernel variant (must be 0 in this library; the
 * timing ablations 2, 4, 16 -- whose results are invalid -- and the stamps
 * of variant 8 exist only in the diagnostic build, -DSMX_SCAN_DIAGNOSTICS)
 * and tiles per work item (0 keeps the default, 20; at least 8). */
int smx_set_tuning(smx_index* index, int32_t candidates_per_query, int32_t seed_leaves,
                   int32_t scan_variant, int32_t chunk_tiles);

const char* smx_last_error(void);
const char* smx_version(void);

#ifdef __cplusplus
}
#endif
#endif /* SCANN_MI355X_H_ */

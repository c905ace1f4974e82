/*
 * scann_oracle.h — CPU restatement of ScaNN's LUT16 / tree-AH query path.
 *
 * TEST INFRASTRUCTURE, NOT PRODUCT CODE.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load liboracle.so.  The product path
 * (scann_amd/, libscann_mi355x.so) never links or calls anything here.
 *
 * Parity status: the reference (owlwang/scann) cannot be compiled in this
 * image (bazel/abseil/Eigen/Highway absent, plus 20 source
 * defects) and ships no golden vectors for this path, so this restatement is
 * pinned only by the hand-derived known-answer tests in tests/ (see DESIGN.md
 * "Oracle").  Where the reference's float behaviour depends on the build's
 * SIMD target, the choice made here is stated at the function.
 *
 * Every function cites the reference file:line whose semantics it follows
 * (paths relative to the reference root).
 */
#ifndef SCANN_ORACLE_H_
#define SCANN_ORACLE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_METRIC_DOT = 0, ORC_METRIC_SQUARED_L2 = 1 };
enum { ORC_MODE_IDEAL = 0, ORC_MODE_EMULATE = 1 };
/* or'ed into mode: partition scores of the single-query path (ScannInterface::
 * Search -> KMeansTreeNode, kmeans_tree_node.h:159-163: DenseDistanceOneToMany,
 * one_to_many_symmetric.h:376-503, the A.8 accumulator order of ExactDistance)
 * instead of the batched transposed FMA chain. */
enum { ORC_PARTITION_ONE_TO_MANY = 4 };

/* Same field layout as smx_index_desc in include/scann_mi355x.h. */
typedef struct orc_index {
  int32_t metric;            /* ORC_METRIC_* */
  int32_t dim;
  int32_t num_leaves;
  int32_t num_blocks;        /* AH blocks (subspaces)                       */
  int32_t dims_per_block;    /* chunk width; last block may be narrower     */
  int32_t residual;          /* 1: tree-AH residual (pipeline A)            */
  const float* centers;      /* [num_leaves][dim]                           */
  const float* codebook;     /* [num_blocks][16][dims_per_block]            */
  const uint64_t* leaf_offsets; /* [num_leaves+1] into leaf_members         */
  const uint32_t* leaf_members; /* global datapoint id per member           */
  const uint8_t* member_codes;  /* [num_members][num_blocks], 0..15          */
  uint32_t num_datapoints;
  const float* dataset;      /* [num_datapoints][dim] or NULL (no reorder)  */
  float spilling_overretrieve_factor; /* SOAR over-retrieval (default 2)   */
  int32_t pad_;
  /* A range-split shard (the tail of smx_index_desc): with is_shard the
   * whole index's tie shift and spill setting replace the ones this index's
   * own leaves would give (the rows' order inside a leaf is the same). */
  int32_t is_shard;
  int32_t global_topn_shift;
  int32_t global_spilled;
  int32_t reserved2;
  /* ideal mode: leaf l's rows are rows [leaf_row_base[l], +n) of the whole
   * index's leaf (the packed tie, tree_ah_hybrid_residual.h:234-247) */
  const uint32_t* leaf_row_base;
  /* ideal mode with a NULL dataset: the reorder rows per member */
  const float* member_rows;
} orc_index;

/* Partition scores, transposed many-to-many numerics
 * (many_to_many_impl.inc:522-560, A.10).  out[q*num_leaves + c]. */
void orc_partition_scores(const float* queries, int32_t nq, int32_t dim,
                          const float* centers, int32_t num_leaves,
                          int32_t metric, float* out);

/* Exact top-L per query by (score, center index)
 * (kmeans_tree_partitioner.cc:703-728).  Outputs sorted ascending. */
void orc_partition_topl(const float* queries, int32_t nq, int32_t dim,
                        const float* centers, int32_t num_leaves,
                        int32_t metric, int32_t L, int32_t* out_leaf,
                        float* out_score);

/* Raw float LUT + uint8 fixed point for one query
 * (asymmetric_hashing_impl.cc:505-645).  raw_out may be NULL.
 * Returns 0, or -1 for an unsupported block width. */
int orc_create_lut(const float* query, int32_t dim, const float* codebook,
                   int32_t num_blocks, int32_t dims_per_block, int32_t metric,
                   float* raw_out, uint8_t* lut_out, float* mult_out);

/* Reference packed LUT16 layout (asymmetric_hashing_impl.cc:690-737).
 * out size = num_blocks * round_up(n, 32) / 2 bytes. */
void orc_pack_codes(const uint8_t* codes, uint32_t n, int32_t num_blocks,
                    uint8_t* out);

/* Sum_b (lut[b][code] - 128) per datapoint, read from the reference packed
 * layout (lut16_avx2.inc:55-124 semantics, exact in int32). */
void orc_lut16_accumulate(const uint8_t* packed, uint32_t n,
                          int32_t num_blocks, const uint8_t* lut,
                          int32_t* out);

/* Global top-N shift (tree_ah_hybrid_residual.h:234-247). */
int32_t orc_global_topn_shift(const orc_index* idx);

/* Whole search_batched path (single_machine_base.cc:570-587 over
 * tree_ah_hybrid_residual.cc:631-846, or tree_x_hybrid_smmd.cc:718-790 for
 * non-residual indexes).  mode: ORC_MODE_IDEAL (exact top-k by the
 * reference's total order) or ORC_MODE_EMULATE (sequential AVX2 replay with
 * FastTopNeighbors GC: pipeline A's int16 truncated prefilter over the
 * global top-N, or pipeline B's per-leaf int16 FastTopNeighbors merged into
 * the global top-N at leaf-visit time; residual indexes without the global
 * top-N path fall back to IDEAL).
 * final_nn/pre_nn/leaves follow scann.cc:406-430: reorder happens iff
 * idx->dataset != NULL and do_reorder != 0.
 * Outputs [nq][final_nn] (padded with idx 0 / NaN), counts [nq].
 * Distances are in the internal convention (smaller is better). */
int orc_search(const orc_index* idx, const float* queries, int32_t nq,
               int32_t leaves, int32_t pre_nn, int32_t final_nn,
               int32_t do_reorder, int32_t mode, int32_t nthreads,
               uint32_t* out_idx, float* out_dist, int32_t* out_count);

/* Pre-reorder candidate stage only (packed or global ids, see out_is_packed)
 * for stage-level parity: returns per query the k' = pre_nn(*SOAR factor)
 * best (global id, distance) sorted by (distance, tie id). */
int orc_search_pre_reorder(const orc_index* idx, const float* queries,
                           int32_t nq, int32_t leaves, int32_t pre_nn,
                           int32_t mode, int32_t nthreads, uint32_t* out_idx,
                           float* out_dist, int32_t* out_count);

/* Exact reorder distance of one row (one_to_many_symmetric.h:373-503, A.8). */
float orc_exact_distance(const float* q, const float* x, int32_t dim,
                         int32_t metric);

/* FastTopNeighbors replay for unit tests (fast_top_neighbors.h:41-440).
 * Pushes (idx[i], dist[i]) in order with PushBlock semantics and returns the
 * FinishUnsorted set sorted by (dist, idx). */
int32_t orc_fast_topn_replay(const uint32_t* idx, const float* dist,
                             int32_t n, int32_t k, uint32_t* out_idx,
                             float* out_dist, int32_t* out_num_gc);

/* FastTopNeighbors<int16_t> replay (pipeline B's per-leaf top-N,
 * querying.h:403-462): push iff dist < epsilon; FinishUnsorted order out. */
int32_t orc_fast_topn_replay_i16(const uint32_t* idx, const int16_t* dist,
                                 int32_t n, int32_t k, int16_t epsilon,
                                 uint32_t* out_idx, int16_t* out_dist,
                                 int32_t* out_num_gc);

/* AVQ noise-shaped AH encoding (IndexDatapointNoiseShaped,
 * asymmetric_hashing_impl.cc:434-503) of n rows: residuals and the original
 * rows [n][dim], codebook [nb][16][dpb], threshold T; codes [n][nb]. */
void orc_avq_encode(const float* residuals, const float* originals, int32_t n, int32_t dim,
                    const float* codebook, int32_t nb, int32_t dpb, double threshold,
                    uint8_t* out);

/* AVX2 port of the reference's hot loop (lut16_avx2.inc) driving the same
 * emulate-mode pipeline, multithreaded like SearchBatchedParallel
 * (scann.cc:478-501).  Used only as bench.py's cpu_baseline.
 * orc_avx2_prepare packs every leaf into the reference layout once (the
 * reference does this when it builds its leaf searchers, searcher.cc:108-111)
 * and returns NULL for indexes the port does not cover (residual with the
 * global top-N path disabled).  Non-residual indexes run pipeline B's
 * emulate semantics (tree_x_hybrid_smmd.cc:718-790, per-leaf int16
 * FastTopNeighbors), residual ones pipeline A's.  orc_search_avx2 returns -2 if the library was
 * built without AVX2.  Partition scoring runs eight centers per AVX2 vector
 * over transposed centers (the reference's many-to-many order), bit-equal to
 * the scalar chain. */
void* orc_avx2_prepare(const orc_index* idx);
void orc_avx2_release(void* prepared);
int orc_search_avx2(void* prepared, const float* queries, int32_t nq,
                    int32_t leaves, int32_t pre_nn, int32_t final_nn,
                    int32_t do_reorder, int32_t nthreads, uint32_t* out_idx,
                    float* out_dist, int32_t* out_count,
                    double* phase_s /* [3] CPU seconds: front, scan, tail; or NULL */,
                    int32_t batch_shared /* 1: the reference's bottom loop, the <= 3
                                            queries of a batch sharing each group's
                                            code extraction, tag-along accumulation
                                            and kSmart prefetch (lut16_avx2.inc:
                                            17-198); 0: one group pass per query */);

#ifdef __cplusplus
}
#endif
#endif /* SCANN_ORACLE_H_ */

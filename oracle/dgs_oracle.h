/*
 * dgs_oracle.h -- CPU restatement of the CommediaJW/Dist-GNN ("DGS") sampling and
 * feature-gather hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under dist-gnn_amd/ includes, links or calls this
 * code; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, as
 * the checker / CPU baseline.  Every function cites the reference file:line it restates
 * (paths relative to the reference repository root).
 *
 * Parity status (see DESIGN.md "Oracle"):
 *   - The reference is CUDA-only and cannot be built or run here, and its own tests hold
 *     no golden outputs (they print).  The oracle is pinned by (a) the Random123 /
 *     curand Philox4x32-10 known-answer vectors, (b) the std::mt19937_64 known answer,
 *     (c) the hand-derived known answers of the reference tests (tests/test_extract.py,
 *     test_p2p_server.py, test_feature_server.py, sampler invariants), and (d) the
 *     structural invariants of each kernel.  Bit-level parity with a CUDA run of the
 *     reference is therefore "parity unpinned" beyond those KATs.
 *   - Biased sampling WITHOUT replacement: the reference key __powf(u, 1/p) is a CUDA
 *     fast-math approximation that cannot be reproduced bit-for-bit; both this oracle and
 *     the HIP kernels use the deterministic key defined by dgs_ares_key() below (same
 *     A-Res distribution, total order (key desc, edge index asc)).
 *
 * Ids are int64 throughout (the reference's datasets are int64, dataset_preprocess.py:54-58).
 */
#ifndef DGS_ORACLE_H_
#define DGS_ORACLE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- RNG: curand Philox4x32-10 semantics (curand_kernel.h / curand_philox4x32_x.h) ---- */
typedef struct {
  uint32_t ctr[4];
  uint32_t key[2];
  uint32_t output[4];
  uint32_t state; /* index of the next output word, 0..3 */
} oracle_philox_t;

void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
void oracle_curand_init(uint64_t seed, uint64_t subsequence, uint64_t offset, oracle_philox_t *st);
uint32_t oracle_curand(oracle_philox_t *st);
float oracle_curand_uniform(oracle_philox_t *st);
/* j-th (0-based) curand() output of the stream (seed, subsequence, offset 0). */
uint32_t oracle_philox_draw(uint64_t seed, uint64_t subsequence, uint64_t j);

/* ---- launch-seed source: std::mt19937_64 (context/context.h:7-21) ---- */
typedef struct {
  uint64_t mt[312];
  int idx;
} oracle_mt64_t;
void oracle_mt64_seed(oracle_mt64_t *g, uint64_t seed);
uint64_t oracle_mt64_next(oracle_mt64_t *g);

/* ---- A-Res key used for biased sampling without replacement (see header comment) ---- */
float oracle_log2f(float u);
float oracle_ares_key(float u, float p);

/* ---- row-wise sampling (one launch; `launch_seed` = the randn_uint64() of that launch) ----
 * Outputs must hold S*k entries; the return value is nnz.  out_row receives the seed nid
 * of each sampled edge (coo_row), out_col the sampled neighbour (coo_col). */
int64_t oracle_sample_uniform(const int64_t *seeds, int64_t S, const int64_t *indptr,
                              const int64_t *indices, int64_t k, int replace,
                              uint64_t launch_seed, int64_t *out_row, int64_t *out_col);
int64_t oracle_sample_bias(const int64_t *seeds, int64_t S, const int64_t *indptr,
                           const int64_t *indices, const float *probs, int64_t k, int replace,
                           uint64_t launch_seed, int64_t *out_row, int64_t *out_col);

/* ---- unique + relabel (tensor_relabel.cu:82-205) ----
 * unique_out must hold n_map entries; returns the number of unique ids. */
int64_t oracle_relabel(const int64_t *mapping, int64_t n_map, const int64_t *req, int64_t n_req,
                       int64_t *unique_out, int64_t *relabeled_out);

/* ---- multi-hop node-classification sample (sampler.cc:14-62,146-166) ----
 * fan_out[L]; hops run from fan_out[L-1] down to fan_out[0].  Buffers are caller-sized
 * with the bounds of oracle_nc_bounds().  sizes_out[3*h + {0,1,2}] = (S_h, U_h, nnz_h). */
void oracle_nc_bounds(int64_t B, const int64_t *fan_out, int L, int64_t *frontier_cap,
                      int64_t *edge_cap);
void oracle_node_classification_sample(const int64_t *seeds, int64_t B, const int64_t *indptr,
                                       const int64_t *indices, const float *probs,
                                       const int64_t *fan_out, int L, int replace,
                                       const uint64_t *launch_seeds, int64_t **frontiers,
                                       int64_t **rows, int64_t **cols, int64_t *sizes_out);

/* ---- cache extraction (sampling/cuda/utils.cu:12-101) ---- */
void oracle_extract_indptr(const int64_t *nids, int64_t n, const int64_t *indptr,
                           int64_t *sub_indptr);
void oracle_extract_edge_data(const int64_t *nids, int64_t n, const int64_t *indptr,
                              const int64_t *sub_indptr, const void *edge_data, int64_t elsize,
                              void *sub_edge_data);

/* ---- gather (feature_ops.cu:140-210 / 12-73 semantics: out[i,:] = data[nids[i],:]) ---- */
void oracle_index_select(const void *data, int64_t row_bytes, const int64_t *nids, int64_t n,
                         void *out, int nthreads);

/* ---- heat (cache/cuda/preprocess_heat.cu:14-121), sequential accumulation ---- */
void oracle_frontier_heat(const int64_t *seeds, int64_t n, const int64_t *indptr,
                          const int64_t *indices, const float *seeds_heat, int64_t num_picks,
                          int64_t indptr_diff, int64_t num_nodes, float *frontier_heat);
void oracle_frontier_heat_with_bias(const int64_t *seeds, int64_t n, const int64_t *indptr,
                                    const int64_t *indices, const float *probs,
                                    const float *seeds_heat, int64_t num_picks,
                                    int64_t indptr_diff, int64_t num_nodes,
                                    float *frontier_heat);

/* ---- OpenMP variants used as the CPU baseline (same results as the serial ones) ---- */
int64_t oracle_sample_uniform_omp(const int64_t *seeds, int64_t S, const int64_t *indptr,
                                  const int64_t *indices, int64_t k, int replace,
                                  uint64_t launch_seed, int64_t *out_row, int64_t *out_col,
                                  int nthreads);
int64_t oracle_sample_bias_omp(const int64_t *seeds, int64_t S, const int64_t *indptr,
                               const int64_t *indices, const float *probs, int64_t k,
                               int replace, uint64_t launch_seed, int64_t *out_row,
                               int64_t *out_col, int nthreads);
int oracle_max_threads(void);

#ifdef __cplusplus
}
#endif

#endif

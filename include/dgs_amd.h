/*
 * dgs_amd.h -- C ABI of the DGS-AMD sampling / feature-gather library (libdgs_amd.so).
 *
 * This is the drop-in boundary for the hot path of CommediaJW/Dist-GNN: every entry point
 * replaces one binding of the reference's pybind11 module `dgs` (src/pybind.cc:17-77) or
 * the service method behind it.  Signatures use plain pointers and sizes only -- no torch
 * types.  The Python package `dgs` (dist-gnn_amd/python/dgs, a ctypes binding) mirrors the
 * reference module layout on top of these functions; INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - Every function returns 0 on success and -1 on error; dgs_last_error() then returns a
 *    thread-local message.  (The reference calls exit()/abort() on CUDA/NCCL errors,
 *    dgs_headers.h:11-34; DGS-AMD reports instead.)
 *  - `stream` is a hipStream_t (NULL = the legacy default stream, which is what the
 *    reference launches on).  Calls are stream-ordered; calls that must return a size
 *    computed on the device (marked SYNC) synchronise `stream` once.
 *  - Device arrays: pointers usable by the current HIP device (device memory, or host
 *    memory registered with dgs_host_register / allocated pinned).
 *  - Host arrays handed to a service constructor (graph, features) may be pageable: the
 *    library copies what it needs and never registers them (dgs_host_register below).
 *  - Ids and CSR offsets are int64 unless an `*_bytes` argument says otherwise.
 */
#ifndef DGS_AMD_H_
#define DGS_AMD_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const char *dgs_last_error(void);
/* Library build identification (gfx target and version string). */
const char *dgs_version(void);

/* ------------------------------------------------------------------------------------
 * Context: communicator and launch-seed RNG (src/nccl/nccl_context.{h,cc}, src/context)
 * ---------------------------------------------------------------------------------- */
/* replaces nccl::GetUniqueId (nccl_context.cc:13-18; pybind.cc:50). out[16] */
int dgs_get_unique_id(int64_t *out_id16);
/* replaces nccl::SetNCCL / NCCLContext::SetNCCL_ (nccl_context.cc:20-45; pybind.cc:51) */
int dgs_set_nccl(int64_t nranks, const int64_t *unique_id, int64_t n_id, int64_t rank);
/* ADDITIVE: host transport for the setup collectives instead of RCCL -- allgather(send[bytes]
 * -> recv[world*bytes]) and barrier over host memory, supplied by the caller (e.g. over
 * torch.distributed / gloo).  Lets ranks that share one GPU (tests) build P2P caches; the hot
 * path is unchanged (one-sided device loads). */
typedef int (*dgs_host_allgather_fn)(const void *send, int64_t bytes, void *recv, void *ctx);
typedef int (*dgs_host_barrier_fn)(void *ctx);
int dgs_set_host_comm(int64_t nranks, int64_t rank, dgs_host_allgather_fn allgather,
                      dgs_host_barrier_fn barrier, void *ctx);
/* replaces _Test_GetLocalRank / _Test_GetWorldSize (nccl_context.cc:31-32; pybind.cc:72-73).
 * Before dgs_set_nccl they report rank 0 of 1. */
int dgs_get_local_rank(void);
int dgs_get_world_size(void);
/* replaces NCCLContext::Barrier_ (nccl_context.cc:46-50): 1-float all-reduce + sync */
int dgs_barrier(void);
/* replaces NCCLContext::NCCLTensorAllGather_ (nccl_context.cc:52-112), split in the two
 * phases the reference runs: sizes (8 B per rank) then payload via grouped send/recv. */
int dgs_allgather_sizes(int64_t my_size, int64_t *all_sizes /* [world] host */);
int dgs_allgather_bytes(const void *send, int64_t send_bytes, void *const *recv /* [world] */,
                        const int64_t *recv_bytes /* [world] */, void *stream);
/* replaces ctx::randn_uint64 (context/context.h:22-27; pybind.cc:71 _Test_Randn) */
uint64_t dgs_randn_uint64(void);
/* ADDITIVE: n consecutive draws of the same engine under one lock (the seeds one
 * dgs_sampler_sample call would draw, for dgs_sampler_sample_seeded). */
int dgs_randn_uint64_n(int64_t n, uint64_t *out);
/* ADDITIVE (not in the reference): reseed the launch-seed engine (std::mt19937_64) so that
 * sampling is reproducible; the reference seeds it from std::random_device
 * (context/context.h:9-10). */
int dgs_set_random_seed(uint64_t seed);

/* ------------------------------------------------------------------------------------
 * Host memory registration (src/common/pin_memory.cc:7-19; pybind.cc:57-58)
 * ---------------------------------------------------------------------------------- */
/* hipHostRegister (mapped) of [ptr, ptr + bytes) in place, as pin_memory.cc:7-12.  These pins are
 * the only caller memory the library registers: a sampler or feature server over pageable host
 * memory copies what it reads (a device temporary for the cache build, or a library-owned
 * pinned mirror for rows that stay on the host), and one over a pinned
 * range reads it in place, holding a reference on the pin.  Unregister drops this call's
 * reference; the range is unmapped when the last reference goes.  A failed hipHostUnregister is
 * reported by the next dgs_check_async_errors (and gather entry point).  Memory pinned outside
 * this library (hipHostMalloc, torch pin_memory) is refused, as is a range that partly
 * overlaps a pin. */
int dgs_host_register(void *ptr, int64_t bytes);
int dgs_host_unregister(void *ptr);
/* ADDITIVE (diagnostics, tests): the library's live registrations -- base, bytes, references
 * (pins + service views) and pins keyed by the base -- up to `cap` entries (any array may be
 * NULL); *n_out = their number. */
int dgs_host_registrations(int64_t cap, uint64_t *bases, int64_t *bytes, int64_t *refs,
                           int64_t *pins, int64_t *n_out);
/* ADDITIVE (diagnostics, tests): number of live registrations, and the bytes / number of the
 * library's pinned host mirrors (services with rows left on the host). */
int dgs_host_memory_state(int64_t *n_registrations, int64_t *mirror_bytes, int64_t *n_mirrors);
/* ADDITIVE: the ABI revision of this header (DGS_ABI_VERSION).  Round 5 inserted num_rows /
 * label_rows arguments into dgs_index_select, dgs_index_select_device and dgs_loader_gather;
 * a binding checks this at load time instead of passing shifted arguments. */
#define DGS_ABI_VERSION 6
int dgs_abi_version(void);

/* ------------------------------------------------------------------------------------
 * Stateless ops (pybind.cc:53-76)
 * ---------------------------------------------------------------------------------- */
/* replaces feature::cuda::GetFeaturesCUDA (feature_ops.cu:140-210; _CAPI_cuda_index_select):
 * out[i, :] = data[nid[i], :] as a byte copy of row_bytes per row; data has num_rows rows.
 * nid_bytes = 4 | 8.  Range guard (every gather of this header): an id outside [0, num_rows)
 * -- which the reference reads out of bounds -- fills its row from row 0 instead, and the next
 * gather entry point of the process (or dgs_check_async_errors) returns -1 naming the id. */
int dgs_index_select(const void *data, int64_t num_rows, int64_t row_bytes, const void *nid,
                     int nid_bytes, int64_t n, void *out, void *stream);

/* ADDITIVE: dgs_index_select for callers that know data and nid are device memory (no
 * pointer-attribute queries: the per-batch loader path). */
int dgs_index_select_device(const void *data, int64_t num_rows, int64_t row_bytes,
                            const void *nid, int nid_bytes, int64_t n, void *out, void *stream);
/* ADDITIVE: -1 (with the message) when a gather kernel of this process met an id outside its
 * source's rows since the last check; clears the report.  No synchronisation: the report of a
 * kernel still queued appears once it has run. */
int dgs_check_async_errors(void);
/* ADDITIVE: the call tag of the calling thread's last gather launch -- the "gather call #"
 * an out-of-range report names -- so a caller can tell which of its batches reported (0: no
 * gather launched on this thread yet). */
int dgs_last_gather_tag(uint64_t *tag);
/* ADDITIVE: a non-blocking HIP stream owned by the caller (hipStreamCreateWithPriority;
 * priority 0 = default, lower = higher priority), for a loader's batch streams: unlike a
 * framework's pooled streams it is never handed to anyone else. */
int dgs_stream_create(int priority, void **stream_out);
int dgs_stream_destroy(void *stream);
/* ADDITIVE: `consumer` waits (on the device) for the work enqueued on `producer` so far -- an
 * event record + stream wait in one call (DistGNN.dataloading.PrefetchLoader). */
int dgs_stream_wait(void *producer, void *consumer);

/* replaces sampling::cuda::RowWiseSamplingUniformCUDA (rowwise_sampling.cu:143-189) and,
 * when probs != NULL, RowWiseSamplingBiasCUDA (rowwise_sampling_bias.cu:226-288)
 * (_CAPI_cuda_sample_neighbors / _CAPI_cuda_sample_neighbors_bias).  Draws one launch seed
 * from the context RNG.  out_row/out_col capacity: S * num_picks.  SYNC: *nnz_out. */
int dgs_sample_neighbors(const int64_t *seeds, int64_t S, const int64_t *indptr,
                         const int64_t *indices, const float *probs, int64_t num_picks,
                         int replace, int64_t *out_row, int64_t *out_col, int64_t *nnz_out,
                         void *stream);

/* replaces sampling::cuda::TensorRelabelCUDA (tensor_relabel.cu:182-205;
 * _CAPI_cuda_sampled_tensor_relabel).  unique_out capacity: sum(map_sizes).
 * req_out[j] receives the relabeled req[j].  SYNC: *n_unique. */
int dgs_relabel(const int64_t *const *maps, const int64_t *map_sizes, int n_maps,
                const int64_t *const *reqs, const int64_t *req_sizes, int n_reqs,
                int64_t *unique_out, int64_t *n_unique, int64_t *const *req_out, void *stream);

/* replaces sampling::cuda::ExtractIndptr (utils.cu:12-42; _Test_ExtractIndptr) */
int dgs_extract_indptr(const int64_t *nids, int64_t n, const int64_t *indptr,
                       int64_t *sub_indptr /* [n+1] */, void *stream);
/* replaces sampling::cuda::ExtractEdgeData (utils.cu:44-101; _Test_ExtractEdgeData) */
int dgs_extract_edge_data(const int64_t *nids, int64_t n, const int64_t *indptr,
                          const int64_t *sub_indptr, const void *edge_data, int64_t elem_bytes,
                          void *sub_edge_data, void *stream);

/* Test-only (no reference counterpart; a _Test_ op like _Test_ExtractIndptr): for each i < n,
 * key[i] = the A-Res key of draw x[i] under probability p[i] (the definition the biased
 * samplers and the oracle share), key_lower[i] = the provable lower bound the biased hub
 * sampling threshold is built from, and flags[i] bit 0 / bit 1 = the streamed hub filter's /
 * the row filter's "certainly below thr[i]" verdict.  Device arrays; the bits must only be set
 * when key[i] < thr[i] (tests/test_gpu_parity.py::test_bias_filter_bounds_are_sound). */
int dgs_test_bias_bounds(const uint32_t *x, const float *p, const float *thr, int64_t n,
                         float *key, float *key_lower, uint8_t *flags, void *stream);

/* replaces cache::cuda::ComputeFrontierHeat[WithBias] (preprocess_heat.cu:35-56,100-121;
 * _CAPI_compute_frontier_heat[_with_bias]).  probs == NULL selects the unbiased form.
 * frontier_heat[num_nodes] is overwritten. */
int dgs_compute_frontier_heat(const int64_t *seeds, int64_t n_seeds, const int64_t *indptr,
                              const int64_t *indices, const float *probs,
                              const float *seeds_heat, int64_t num_nodes, int64_t num_picks,
                              int64_t indptr_diff, float *frontier_heat, void *stream);
/* ADDITIVE.  The same heat, accumulated deterministically: every message is rounded to a
 * multiple of 2^-36 and summed in int64 (associative, so independent of atomic order), then
 * converted to float.  Differs from the float-atomic form by at most 2^-37 per message. */
int dgs_compute_frontier_heat_fixed(const int64_t *seeds, int64_t n_seeds,
                                    const int64_t *indptr, const int64_t *indices,
                                    const float *probs, const float *seeds_heat,
                                    int64_t num_nodes, int64_t num_picks, int64_t indptr_diff,
                                    float *frontier_heat, void *stream);

/* ------------------------------------------------------------------------------------
 * TensorP2PServer (src/cache/tensor_p2p_cache.{h,cc}; pybind.cc:41-45)
 * ---------------------------------------------------------------------------------- */
typedef struct dgs_p2p_server dgs_p2p_server;
/* Copies `bytes` from `src` (device or registered host) into a block owned by the server,
 * exports it to every rank (collective when world_size > 1). item_bytes = bytes per item. */
int dgs_p2p_server_create(const void *src, int64_t items, int64_t item_bytes,
                          dgs_p2p_server **out);
int dgs_p2p_server_device_ptr(dgs_p2p_server *s, int64_t rank, void **ptr, int64_t *items);
int dgs_p2p_server_destroy(dgs_p2p_server *s); /* collective when world_size > 1 */

/* ------------------------------------------------------------------------------------
 * P2PCacheSampler (src/sampling/sampler.{h,cc}; pybind.cc:21-31)
 * ---------------------------------------------------------------------------------- */
typedef struct dgs_sampler dgs_sampler;
/* indptr[num_nodes+1], indices[num_edges], probs[num_edges] or NULL: host arrays (pageable
 * ones are copied: see dgs_host_register) -- sampler.cc:64-136.  cache_nids: this rank's
 * cached node ids (device or host; an id outside [0, num_nodes) is refused).  Collective when
 * world_size > 1.  Destruction waits for the sampler's calls and the device's queued work. */
int dgs_sampler_create(const int64_t *indptr, const int64_t *indices, const float *probs,
                       int64_t num_nodes, int64_t num_edges, const int64_t *cache_nids,
                       int64_t n_cache, int64_t device_id, dgs_sampler **out);
/* Upper bounds for the per-hop output buffers of dgs_sampler_sample:
 * frontier_cap[h], edge_cap[h] for h = 0..L-1 (hop h uses fan_out[L-1-h]). */
int dgs_sampler_bounds(const dgs_sampler *s, int64_t n_seeds, const int64_t *fan_out, int L,
                       int64_t *frontier_cap, int64_t *edge_cap);
/* replaces P2PCacheSampler::NodeClassifictionSample (sampler.cc:146-166): hop h writes the
 * frontier (unique(seeds_h ++ sampled cols), first-occurrence order) to frontiers[h] and the
 * relabeled COO to rows[h]/cols[h]; sizes_out[3h..3h+2] = (S_h, |frontier_h|, nnz_h).
 * One launch seed per hop comes from the global engine (rowwise_sampling.cu:162).  The host
 * waits once, for the sizes the last kernel publishes; the last relabel pass may still run on
 * `stream` when the call returns.  Calls on different streams run concurrently (each stream
 * has its own sampling context over the shared graph). */
int dgs_sampler_sample(dgs_sampler *s, const int64_t *seeds, int64_t n_seeds,
                       const int64_t *fan_out, int L, int replace, int64_t *const *frontiers,
                       int64_t *const *rows, int64_t *const *cols, int64_t *sizes_out,
                       void *stream);
/* ADDITIVE: dgs_sampler_sample with every hop's outputs packed in one device buffer `out` (per
 * hop h: frontier[fcap_h], rows[ecap_h], cols[ecap_h] back to back, the capacities of
 * dgs_sampler_bounds); `seeds` must be device memory.  What the Python binding's
 * _CAPI_sample_node_classifiction calls: no per-hop pointer arrays to build per call. */
int dgs_sampler_sample_packed(dgs_sampler *s, const int64_t *seeds, int64_t n_seeds,
                              const int64_t *fan_out, int L, int replace, int64_t *out,
                              int64_t *sizes_out, void *stream);
/* ADDITIVE: dgs_sampler_sample in two halves.  _begin enqueues every hop on `stream` and
 * returns without waiting; _end waits for that call's sizes (same `stream`, same L).  At most
 * one call per stream is outstanding.  launch_seeds: the L per-hop launch seeds (hop h uses
 * launch_seeds[h]), or NULL to draw them from the global engine; a pipelined loader draws
 * them with dgs_randn_uint64_n in batch order, so overlapped calls on several streams give
 * exactly the results of sequential dgs_sampler_sample calls.
 * flags: DGS_SAMPLE_HOST_ASYNC -- a library thread (one per stream) issues the launches and
 * _begin returns before they are enqueued; the caller then must not enqueue work on `stream`
 * until _end returns.  The output buffers and seeds must stay alive until _end. */
#define DGS_SAMPLE_HOST_ASYNC 1
#define DGS_SAMPLE_WAIT 2 /* dgs_sampler_sample_begin_after: wait for `wait_for` first */
/* dgs_sampler_sample_begin_after: `wait_for` is a hipEvent_t the caller recorded (e.g. where
 * its seeds were complete); `stream` waits on it first */
#define DGS_SAMPLE_WAIT_EVENT 4
int dgs_sampler_sample_begin(dgs_sampler *s, const int64_t *seeds, int64_t n_seeds,
                             const int64_t *fan_out, int L, int replace,
                             int64_t *const *frontiers, int64_t *const *rows,
                             int64_t *const *cols, const uint64_t *launch_seeds, int flags,
                             void *stream);
int dgs_sampler_sample_end(dgs_sampler *s, int L, int64_t *sizes_out, void *stream);
/* ADDITIVE: the synchronous call (dgs_sampler_sample_packed) in parts, so the caller can use a
 * hop's outputs while later hops run: _packed_begin enqueues every hop with the synchronous
 * call's kernel shapes; _wait_hop returns hop h's (U_h, nnz_h) once its compaction has published
 * them (h < L, the call stays outstanding); dgs_sampler_sample_end ends the call (and reports
 * its errors) as for dgs_sampler_sample_begin.  Same draws and outputs as the one-call form. */
int dgs_sampler_sample_packed_begin(dgs_sampler *s, const int64_t *seeds, int64_t n_seeds,
                                    const int64_t *fan_out, int L, int replace, int64_t *out,
                                    void *stream);
int dgs_sampler_sample_wait_hop(dgs_sampler *s, int L, int h, int64_t *u_nnz /* [2] */,
                                void *stream);
/* ADDITIVE: with DGS_SAMPLE_WAIT in `flags`, `stream` first waits for the work enqueued on
 * `wait_for` so far (any stream, NULL = the null stream); with DGS_SAMPLE_WAIT_EVENT it waits on
 * the event `wait_for`; a non-NULL `wait_for` without either flag is an error (round 3's
 * header waited whenever it was non-NULL); then dgs_sampler_sample_begin with
 * every hop's outputs packed in one device buffer `out`:
 * per hop h, frontier[fcap_h], rows[ecap_h], cols[ecap_h] back to back (the capacities of
 * dgs_sampler_bounds) -- one call per batch for a pipelined loader.  `seeds` must be device
 * memory (no pointer-attribute query); 1 <= L <= 64. */
int dgs_sampler_sample_begin_after(dgs_sampler *s, void *wait_for, const int64_t *seeds,
                                   int64_t n_seeds, const int64_t *fan_out, int L, int replace,
                                   int64_t *out, const uint64_t *launch_seeds, int flags,
                                   void *stream);
/* ADDITIVE (diagnostics): sampling contexts the sampler holds, one per stream that sampled
 * recently.  At most DGS_SAMPLER_MAX_CTX (default 8) are kept: a new stream evicts the least
 * recently used idle one (the reference keeps no per-stream state, sampler.cc:146-166). */
int dgs_sampler_context_count(dgs_sampler *s, int64_t *n);
/* _CAPI_get_local_cache_structure_tensors (sampler.cc:183-195): non-owning device views. */
int dgs_sampler_local_cache(const dgs_sampler *s, const int64_t **sub_indptr, int64_t *n_rows,
                            const int64_t **sub_indices, int64_t *n_edges,
                            const float **sub_probs);
/* _CAPI_get_local_cache_hashmap_tensors (sampler.cc:197-201): the reference's open-addressing
 * cache map (hashmap.cu:15-77) -- key / idx / devid arrays of dir_size = 2 * _UpPower(total cached)
 * ids of `id_bytes` (4 or 8, the cache lists' id type), empty slots -1, every rank's list inserted
 * in the reference's rotation order with its Murmur3 hash and probe sequence, the local list last
 * (a node cached locally keeps its local idx/devid).  Built on the device when asked for (SYNC);
 * the sampler's lookups use its dense node table instead.  As in the reference, the slot a key
 * lands in depends on the order of concurrent inserts; the key set and every lookup do not. */
int dgs_sampler_cache_hashmap_capacity(const dgs_sampler *s, int64_t *dir_size);
int dgs_sampler_cache_hashmap_fill(const dgs_sampler *s, int id_bytes, void *key, void *idx,
                                   void *devid, void *stream);
/* ADDITIVE: the same map compacted -- one (nid, row, device) entry per cached node, in node-id
 * order, local entries taking priority.  Two-step: the count, then a fill of caller buffers
 * (device, int64). */
int dgs_sampler_cache_map_size(const dgs_sampler *s, int64_t *n);
int dgs_sampler_cache_map_fill(const dgs_sampler *s, int64_t *key, int64_t *idx,
                               int64_t *devid, void *stream);
int dgs_sampler_destroy(dgs_sampler *s); /* collective when world_size > 1 */

/* ------------------------------------------------------------------------------------
 * P2PCacheFeatureServer (src/feature/feature_server.cc, feature_sever.h; pybind.cc:33-39)
 * ---------------------------------------------------------------------------------- */
typedef struct dgs_feature_server dgs_feature_server;
/* data: host array [num_rows, row_bytes] (copied when pageable: see dgs_host_register);
 * cache_nids: rows cached in this GPU's HBM (device or host; an id outside [0, num_rows) is
 * refused).  feature_server.cc:10-61.  Destruction waits for the device's queued work. */
int dgs_feature_server_create(const void *data, int64_t num_rows, int64_t row_bytes,
                              const int64_t *cache_nids, int64_t n_cache, int64_t device_id,
                              dgs_feature_server **out);
/* replaces P2PCacheFeatureServer::GetFeatures (feature_server.cc:69-74) and
 * GetFeaturesP2PCacheCUDA (feature_ops.cu:75-138): out[i,:] = X[nids[i],:] from the local
 * cache, a peer's cache (xGMI) or host memory, in one fused lookup+gather kernel. */
int dgs_feature_server_gather(dgs_feature_server *s, const int64_t *nids, int64_t n,
                              void *out, void *stream);
int dgs_feature_server_local_cache(const dgs_feature_server *s, const void **ptr,
                                   int64_t *rows);
/* ADDITIVE: `consumer` waits on a hipEvent_t the caller recorded (hipStreamWaitEvent). */
int dgs_stream_wait_event(void *event, void *consumer);
/* ADDITIVE (PrefetchLoader, one call per batch): `consumer` waits for `producer` (the batch's
 * sample call), then on `consumer` the feature gather of nids[n] into feat_out (fs may be
 * NULL) and, when labels != NULL, label_out[i] = labels[seeds[i]] (label_rows rows of
 * label_row_bytes, int64 seeds; both gathers range-guarded as dgs_index_select).  nids, seeds
 * and every buffer are device memory.  With s != NULL the call on
 * `producer` must have been ended (dgs_sampler_sample_end) and no new one begun: `consumer`
 * waits on the event that call's launches recorded, with no event record here; with s == NULL
 * an event is recorded on `producer` now. */
int dgs_loader_gather(dgs_sampler *s, dgs_feature_server *fs, void *producer, void *consumer,
                      const int64_t *nids, int64_t n, void *feat_out, const void *labels,
                      int64_t label_rows, int64_t label_row_bytes, const int64_t *seeds,
                      int64_t n_seeds, void *label_out);
/* ADDITIVE.  Address layout the gather uses: -1 = per-node address table (general cache
 * placement), w >= 0 = every node cached in the strided layout (node v at row v >> w of GPU
 * v & (2^w - 1); w = 0 is the whole-graph-in-HBM identity), no per-node table read. */
int dgs_feature_server_layout(const dgs_feature_server *s, int *wshift);
int dgs_feature_server_destroy(dgs_feature_server *s);

/* ------------------------------------------------------------------------------------
 * Instrumentation (bench.py).  `mask` selects what is timed: DGS_PROFILE_GATHER = feature-
 * server gather kernels, DGS_PROFILE_SELECT = index_select kernels (both timed by the kernel
 * itself: the first wave of every workgroup stamps s_memrealtime, the 100 MHz device wall
 * clock, at its start and after its last store; a launch's time is its last end - first start,
 * read back from a stamp slab reserved when profiling is switched on), DGS_PROFILE_SAMPLE =
 * whole sample calls (one stream event before the first and one after the last kernel).
 * 0 disables; any nonzero value outside the three bits enables all.  dgs_profile_read()
 * returns the summed milliseconds and counts, then resets them.
 * ---------------------------------------------------------------------------------- */
#define DGS_PROFILE_GATHER 1
#define DGS_PROFILE_SAMPLE 2
#define DGS_PROFILE_SELECT 4
int dgs_profile_enable(int mask);
int dgs_profile_read(double *gather_ms, int64_t *gather_launches, double *sample_ms,
                     int64_t *sample_calls, double *select_ms, int64_t *select_launches);

#ifdef __cplusplus
}
#endif

#endif /* DGS_AMD_H_ */

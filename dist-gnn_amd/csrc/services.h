// services.h -- stateful services behind the C ABI: TensorP2PServer, P2PCacheSampler,
// P2PCacheFeatureServer (reference: src/cache/tensor_p2p_cache.*, src/sampling/sampler.*,
// src/feature/feature_server.cc).
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <exception>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "context.h"
#include "dgs_ops.h"

namespace dgs {

// A device block shared with every rank of the communicator through HIP IPC (one-sided
// peer loads over xGMI).  Construction and destruction are collective when world > 1
// (tensor_p2p_cache.cc:11-118).
class P2PServer {
 public:
  // copies `items * item_bytes` bytes from src (device or host) into an owned block
  P2PServer(const void *src, int64_t items, int64_t item_bytes);
  // adopts an existing hipMalloc'd block
  static P2PServer *adopt(void *block, int64_t items, int64_t item_bytes);
  ~P2PServer();
  void *ptr(int r) const { return ptrs_[r]; }
  void *local() const { return ptrs_[rank_]; }
  int64_t items(int r) const { return items_[r]; }
  int64_t item_bytes() const { return item_bytes_; }
  int world() const { return world_; }
  int rank() const { return rank_; }

 private:
  P2PServer() = default;
  void share();
  std::vector<void *> ptrs_;
  std::vector<int64_t> items_;
  int64_t item_bytes_ = 0;
  int rank_ = 0, world_ = 1;
};

// A caller's host array as a service's kernels read it (sampler CSR and probabilities, feature
// matrix).  Pageable caller memory is never registered (round 6):
//  - keep == false (every row is cached on some GPU: the array only feeds the cache build): a
//    device temporary filled through the library's pinned staging (a pinned mirror when the
//    device lacks room), dropped by release() once the caches are built;
//  - keep == true (rows stay on the host and are read zero-copy while the service lives): a
//    library-owned pinned, mapped mirror (hipHostMalloc) holding a copy.
// Device memory, and host memory pinned by its owner or by dgs_host_register (then a
// reference is held on that pin), are read in place.
struct HostSource {
  void *dev = nullptr;  // device-accessible address of the array (nullptr: empty)
  HostSource() = default;
  HostSource(const HostSource &) = delete;
  HostSource &operator=(const HostSource &) = delete;
  void attach(const void *p, int64_t bytes, bool keep, hipStream_t st);
  // no device read of `dev` may follow (the caller synchronises first)
  void release();
  bool host_resident() const { return mirror_ != nullptr || pin_ != nullptr; }
  ~HostSource() { release(); }

 private:
  const void *pin_ = nullptr;  // a dgs_host_register range holding our reference
  void *dtemp_ = nullptr;      // device temporary (hipMalloc)
  void *mirror_ = nullptr;     // pinned mirror (hipHostMalloc)
  size_t bytes_ = 0;
};

class Sampler {
 public:
  Sampler(const int64_t *indptr, const int64_t *indices, const float *probs, int64_t num_nodes,
          int64_t num_edges, const int64_t *cache_nids, int64_t n_cache, int64_t device_id);
  ~Sampler();
  void bounds(int64_t n_seeds, const int64_t *fan_out, int L, int64_t *fcap,
              int64_t *ecap) const;
  // launch_seeds: L per-hop seeds, or nullptr to draw them from the global engine
  void sample(const int64_t *seeds, int64_t n_seeds, const int64_t *fan_out, int L,
              bool replace, int64_t *const *frontiers, int64_t *const *rows,
              int64_t *const *cols, int64_t *sizes, hipStream_t st,
              const uint64_t *launch_seeds = nullptr);
  // sample() in two halves: enqueue every hop, then wait for the published sizes
  // (host_async: a per-stream library thread issues the launches; the caller must not use
  // the stream before sample_end)
  void sample_begin(const int64_t *seeds, int64_t n_seeds, const int64_t *fan_out, int L,
                    bool replace, int64_t *const *frontiers, int64_t *const *rows,
                    int64_t *const *cols, hipStream_t st, const uint64_t *launch_seeds,
                    bool host_async = false, bool solo = false);
  void sample_end(int L, int64_t *sizes, hipStream_t st);
  // hop h's (U, nnz) of the call outstanding on `st`, once published (the call stays pending)
  void sample_wait_hop(int L, int h, int64_t *u_nnz, hipStream_t st);
  // `consumer` waits for the last call ended on `st`, on the event that call recorded after its
  // launches (no event record on the caller's thread).
  void wait_ended(hipStream_t st, hipStream_t consumer);
  // sampling contexts currently held (one per stream that sampled recently; at most max_ctx)
  size_t num_contexts();
  const int64_t *sub_indptr() const { return (const int64_t *)indptr_srv_->local(); }
  int64_t n_rows() const { return indptr_srv_->items(rank_) - 1; }
  const int64_t *sub_indices() const { return (const int64_t *)indices_srv_->local(); }
  int64_t n_edges() const { return indices_srv_->items(rank_); }
  const float *sub_probs() const {
    return probs_srv_ ? (const float *)probs_srv_->local() : nullptr;
  }
  // the reference's open-addressing cache map (hashmap.cu:15-77): capacity, then a build into
  // caller buffers of that many ids (id_bytes 4 or 8)
  int64_t cache_hashmap_capacity() const;
  void cache_hashmap_fill(int id_bytes, void *key, void *idx, void *devid, hipStream_t st) const;
  int64_t cache_map_size() const;
  void cache_map_fill(int64_t *key, int64_t *idx, int64_t *devid, hipStream_t st) const;

 private:
  void build_cache_rowtab(int64_t *tab, hipStream_t st) const;
  int64_t num_nodes_ = 0, num_edges_ = 0;
  int rank_ = 0, world_ = 1;
  bool bias_ = false;
  HostSource h_indptr_, h_indices_, h_probs_;
  P2PServer *indptr_srv_ = nullptr, *indices_srv_ = nullptr, *probs_srv_ = nullptr;
  P2PServer *nids_srv_ = nullptr;
  DevBuf ntab_;
  RowSrc src_{};
  // Per-stream sampling state: calls on different streams run concurrently over the shared
  // (read-only) graph; calls on one stream take turns on its context.
  struct Job {
    const int64_t *seeds = nullptr;
    int64_t n_seeds = 0;
    int L = 0;
    bool replace = false;
    std::vector<int64_t> fan_out;
    std::vector<int64_t *> fr, rows, cols;
    std::vector<uint64_t> hop_seed;
    bool solo = false;  // a synchronous call (sample()): nothing else of ours runs beside it
  };
  struct Ctx {
    std::mutex mu;
    std::condition_variable cv;
    std::thread launcher;  // started by the first host-asynchronous call
    Job job;
    bool job_ready = false, job_done = true, stop = false;
    std::atomic<bool> job_flag{false};  // job_ready, readable without the lock (launcher spin)
    std::atomic<bool> stop_flag{false};  // stop, likewise
    std::exception_ptr job_err;
    HopScratch ws;
    DevBuf dpair[2];  // direct relabel tables over node ids ((first position, label) pairs),
    bool dirty[2] = {false, false};  // used by alternate hops
    DevBuf sizes;
    HostPinned sizes_host;  // [0] publication sequence, [1..3L] per-hop sizes, [3L+1] bad seed
    int64_t *sizes_host_dev = nullptr;
    uint64_t seq = 0;
    hipStream_t stream = nullptr;
    bool pending = false;  // a call was begun and not yet ended
    int pending_L = 0;
    int64_t pending_seeds = 0;
    hipEvent_t end_ev = nullptr;  // recorded on the stream after each call's launches
    uint64_t last_use = 0;        // ctx_mu_ tick of the last lookup
  };
  // The context of `st`, created on first use.  At most max_ctx_ are kept (DGS_SAMPLER_MAX_CTX,
  // default 8): a new stream evicts the least recently used context that no thread holds and
  // that has no call outstanding, after its last call's kernels have finished (its end event).
  // A caller cycling through fresh streams therefore holds a bounded amount of HBM (each
  // context holds relabel tables of 16 B per node plus scratch); the reference keeps no state
  // between calls (sampler.cc:146-166).
  std::shared_ptr<Ctx> ctx_for(hipStream_t st);
  // the context of `st` if there is one (no creation, no eviction)
  std::shared_ptr<Ctx> ctx_find(hipStream_t st);
  static void retire(Ctx &c);
  void launch(Ctx &c, const Job &j, hipStream_t st);
  void launch_hops(Ctx &c, const Job &j, hipStream_t st);
  void launcher_loop(Ctx &c, int dev);
  std::mutex ctx_mu_;
  std::unordered_map<hipStream_t, std::shared_ptr<Ctx>> ctxs_;
  uint64_t ctx_tick_ = 0;
  size_t max_ctx_ = 8;
};

class FeatureServer {
 public:
  FeatureServer(const void *data, int64_t num_rows, int64_t row_bytes, const int64_t *cache_nids,
                int64_t n_cache, int64_t device_id);
  ~FeatureServer();
  // tail: a label gather fused into the same launch (n > 0 only)
  void gather(const int64_t *nids, int64_t n, void *out, hipStream_t st,
              const LabelTail *tail = nullptr) const;
  const void *local() const { return feat_srv_ ? feat_srv_->local() : nullptr; }
  int64_t local_rows() const { return feat_srv_ ? feat_srv_->items(rank_) : 0; }
  int layout() const { return wshift_; }
  int64_t row_bytes() const { return row_bytes_; }

 private:
  int64_t num_rows_ = 0, row_bytes_ = 0;
  int rank_ = 0, world_ = 1;
  HostSource h_data_;
  P2PServer *feat_srv_ = nullptr;
  void detect_strided(const std::vector<void *> &lists, const std::vector<int64_t> &nbytes,
                      hipStream_t st);
  DevBuf ftab_;
  uintptr_t align_or_ = 0;
  // >= 0: every node is cached in the strided layout of gather_strided (no ftab reads)
  int wshift_ = -1;
  const void *bases_[kMaxDevices] = {};
};

}  // namespace dgs

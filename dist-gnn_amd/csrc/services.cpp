// services.cpp -- TensorP2PServer, P2PCacheSampler, P2PCacheFeatureServer.
#include "services.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace dgs {

// test hook: DGS_TEST_BUILD_FAIL=r makes rank r's service build fail (after its local argument
// checks), to test that the failure is collective
static bool test_build_fail(int rank) {
  static const int r = [] {
    const char *e = std::getenv("DGS_TEST_BUILD_FAIL");
    return e ? std::atoi(e) : -1;
  }();
  return rank == r;
}

// ============================================================== P2PServer
// tensor_p2p_cache.cc:11-118: raw device block, IPC handle all-gather, peer handles opened
// with lazy peer access; the destructor closes them behind a collective barrier.
P2PServer::P2PServer(const void *src, int64_t items, int64_t item_bytes) {
  const int64_t bytes = items * item_bytes;
  void *block = nullptr;
  std::string err;
  try {
    DGS_HIP(hipMalloc(&block, bytes > 0 ? bytes : 1));
    if (bytes > 0) DGS_HIP(hipMemcpy(block, src, bytes, hipMemcpyDefault));
  } catch (const std::exception &e) {
    err = e.what();
  }
  try {
    Comm::get().check_all(err, "TensorP2PServer: copying the block");
    item_bytes_ = item_bytes;
    Comm &c = Comm::get();
    rank_ = c.rank();
    world_ = c.world();
    ptrs_.assign(world_, nullptr);
    ptrs_[rank_] = block;
    items_.assign(world_, items);
    share();
  } catch (...) {
    // (a failed share() has opened no peer handle; every rank raises from the same point)
    if (block) (void)hipFree(block);
    throw;
  }
}

P2PServer *P2PServer::adopt(void *block, int64_t items, int64_t item_bytes) {
  std::unique_ptr<P2PServer> s(new P2PServer());
  s->item_bytes_ = item_bytes;
  Comm &c = Comm::get();
  s->rank_ = c.rank();
  s->world_ = c.world();
  s->ptrs_.assign(s->world_, nullptr);
  s->ptrs_[s->rank_] = block;
  s->items_.assign(s->world_, items);
  s->share();  // on failure the destructor frees the adopted block (collectively)
  return s.release();
}

// The IPC handle exchange carries each rank's export status: a rank whose hipIpcGetMemHandle
// fails still takes part in the all-gather, and then every rank raises naming it (instead of
// the others waiting in the collective for a rank that has left it).
namespace {
struct ShareMsg {
  hipIpcMemHandle_t h;
  int32_t err;  // hipError_t of the export (0: ok)
  int32_t pad;
};
}  // namespace

void P2PServer::share() {
  Comm &c = Comm::get();
  if (world_ <= 1) return;
  items_ = c.allgather_sizes(items_[rank_]);
  ShareMsg m;
  std::memset(&m, 0, sizeof(m));
  m.err = (int32_t)hipIpcGetMemHandle(&m.h, ptrs_[rank_]);
  // test hook: DGS_TEST_IPC_EXPORT_FAIL=r makes rank r report a failed export
  static const int fail_rank = [] {
    const char *e = std::getenv("DGS_TEST_IPC_EXPORT_FAIL");
    return e ? std::atoi(e) : -1;
  }();
  if (rank_ == fail_rank) m.err = (int32_t)hipErrorInvalidValue;
  std::string local;
  if (m.err != hipSuccess) {
    (void)hipGetLastError();
    void *base = nullptr;
    size_t size = 0;
    const hipError_t re = hipMemGetAddressRange(reinterpret_cast<hipDeviceptr_t *>(&base),
                                                &size, ptrs_[rank_]);
    (void)hipGetLastError();
    char buf[256];
    snprintf(buf, sizeof(buf), " (block %p of %lld items x %lld B; allocation %p, %zu B%s)",
             ptrs_[rank_], (long long)items_[rank_], (long long)item_bytes_, base, size,
             re == hipSuccess ? "" : ", range unknown");
    local = buf;
  }
  void *dh = nullptr;
  DGS_HIP(hipMalloc(&dh, sizeof(m)));
  DGS_HIP(hipMemcpy(dh, &m, sizeof(m), hipMemcpyHostToDevice));
  std::vector<int64_t> nbytes;
  std::vector<void *> all = c.allgather_device(dh, sizeof(m), &nbytes);
  DGS_HIP(hipFree(dh));
  c.barrier();
  std::vector<ShareMsg> msgs(world_);
  for (int i = 0; i < world_; ++i) {
    DGS_HIP(hipMemcpy(&msgs[i], all[i], sizeof(ShareMsg), hipMemcpyDeviceToHost));
    DGS_HIP(hipFree(all[i]));
  }
  for (int i = 0; i < world_; ++i) {
    if (msgs[i].err == hipSuccess) continue;
    for (int j = 0; j < world_; ++j) ptrs_[j] = j == rank_ ? ptrs_[j] : nullptr;
    char buf[200];
    snprintf(buf, sizeof(buf), "TensorP2PServer: rank %d could not export its block for IPC: "
             "hipIpcGetMemHandle: %s", i, hipGetErrorString((hipError_t)msgs[i].err));
    DGS_CHECK(false, std::string(buf) + (i == rank_ ? local : std::string()));
  }
  for (int i = 0; i < world_; ++i) {
    if (i == rank_) continue;
    DGS_HIP(hipIpcOpenMemHandle(&ptrs_[i], msgs[i].h, hipIpcMemLazyEnablePeerAccess));
  }
}

P2PServer::~P2PServer() {
  // views of the block (and of the peers' blocks) may still be read by work queued on any
  // stream of this device: it finishes before the mappings go
  (void)hipDeviceSynchronize();
  try {
    if (world_ > 1)
      for (int i = 0; i < world_; ++i)
        if (i != rank_ && ptrs_[i]) (void)hipIpcCloseMemHandle(ptrs_[i]);
    Comm::get().barrier();
  } catch (...) {
  }
  if (!ptrs_.empty() && ptrs_[rank_]) (void)hipFree(ptrs_[rank_]);
}

// Rotation order of hashmap.cu:37-72: remote ranks (local+1, local+2, ...) then local last,
// later writers win -- a node cached on several GPUs is read from the local one if present.
static std::vector<int> rotation(int rank, int world) {
  std::vector<int> order;
  for (int d = 0; d < world; ++d) {
    const int idx = (d + rank) % world;
    if (idx != rank) order.push_back(idx);
  }
  order.push_back(rank);
  return order;
}

static int64_t *device_copy_ids(const int64_t *ids, int64_t n, hipStream_t st) {
  int64_t *d = nullptr;
  DGS_HIP(hipMalloc(&d, sizeof(int64_t) * (size_t)(n > 0 ? n : 1)));
  if (n > 0) DGS_HIP(hipMemcpyAsync(d, ids, sizeof(int64_t) * n, hipMemcpyDefault, st));
  return d;
}

// ============================================================== host sources
void HostSource::attach(const void *p, int64_t bytes, bool keep, hipStream_t st) {
  release();
  if (!p || bytes <= 0) return;
  bool ref = false;
  if (void *v = pinned_view(p, bytes, &ref)) {
    dev = v;
    if (ref) pin_ = p;
    return;
  }
  bytes_ = (size_t)bytes;
  if (!keep) {
    // the build reads it from HBM; half the free memory stays for the caches it builds
    size_t free_b = 0, total_b = 0;
    DGS_HIP(hipMemGetInfo(&free_b, &total_b));
    if (bytes_ <= free_b / 2) {
      DGS_HIP(hipMalloc(&dtemp_, bytes_));
      dev = dtemp_;
      upload_pageable(dtemp_, p, bytes_, st);
      return;
    }
  }
  mirror_ = mirror_alloc(bytes_);
  host_copy(mirror_, p, bytes_);
  DGS_HIP(hipHostGetDevicePointer(&dev, mirror_, 0));
}

void HostSource::release() {
  if (pin_) release_host_view(pin_);
  if (dtemp_) (void)hipFree(dtemp_);
  if (mirror_) mirror_free(mirror_, bytes_);
  pin_ = nullptr;
  dtemp_ = mirror_ = nullptr;
  dev = nullptr;
  bytes_ = 0;
}

// ============================================================== Sampler
Sampler::Sampler(const int64_t *indptr, const int64_t *indices, const float *probs,
                 int64_t num_nodes, int64_t num_edges, const int64_t *cache_nids,
                 int64_t n_cache, int64_t device_id) {
  Comm &c = Comm::get();
  rank_ = c.rank();
  world_ = c.world();
  hipStream_t st = nullptr;
  // The local checks and the cache list's copy, then their outcome made collective (a rank with
  // a bad argument must not leave its peers in the first exchange).
  int64_t *nids = nullptr;
  std::string err;
  try {
    // sampler.cc:72.  Without a communicator every process is an independent replica (the
    // reference would read an uninitialised rank); with the host transport ranks may share a
    // GPU.
    DGS_CHECK(device_id == rank_ || c.host_mode() || !c.initialized(),
              "device_id must equal the communicator rank (sampler.cc:72)");
    DGS_CHECK(num_nodes >= 0 && num_edges >= 0 && n_cache >= 0, "negative sizes");
    // the biased top-k keeps row-local edge indices in 32 bits
    if (num_edges >= INT32_MAX) {
      int64_t prev = indptr[0];
      for (int64_t v = 1; v <= num_nodes; ++v) {
        DGS_CHECK(indptr[v] - prev < INT32_MAX, "a row has 2^31 - 1 or more edges");
        prev = indptr[v];
      }
    }
    // a cached id outside [0, num_nodes) is refused (the reference reads indptr out of bounds,
    // utils.cu:12-42)
    nids = device_copy_ids(cache_nids, n_cache, st);
    DGS_CHECK(count_out_of_range(nids, n_cache, num_nodes, st) == 0,
              "cache_nids: an id is outside [0, num_nodes)");
  } catch (const std::exception &e) {
    err = e.what();
  }
  try {
    c.check_all(err, "P2PCacheSampler: argument checks");
  } catch (...) {
    if (nids) (void)hipFree(nids);
    throw;
  }
  num_nodes_ = num_nodes;
  num_edges_ = num_edges;
  bias_ = probs != nullptr;
  if (const char *e = std::getenv("DGS_SAMPLER_MAX_CTX"))
    max_ctx_ = (size_t)std::max(1, std::atoi(e));

  // this rank's cache list, shared with every rank first: it decides what the build needs
  nids_srv_ = P2PServer::adopt(nids, n_cache, 8);
  // Rows no GPU caches are read from the host while the sampler lives (a pinned mirror of the
  // neighbour ids / probabilities); with none, the host graph only feeds the cache build (a
  // device temporary).  indptr is only read by the build.
  std::vector<const int64_t *> lists(world_);
  std::vector<int64_t> counts(world_);
  for (int d = 0; d < world_; ++d) {
    lists[d] = (const int64_t *)nids_srv_->ptr(d);
    counts[d] = nids_srv_->items(d);
  }
  // this rank's build (host sources, then its cached sub-CSR, sampler.cc:89-110), its outcome
  // made collective before the sub-CSR blocks are exchanged
  int64_t *sub_indptr = nullptr;
  void *sub_indices = nullptr, *sub_probs = nullptr;
  int64_t n_sub = 0;
  bool host_rows = false;
  err.clear();
  try {
    host_rows = count_uncovered(lists.data(), counts.data(), world_, num_nodes, st) > 0;
    DGS_CHECK(!test_build_fail(rank_), "test hook: sampler build failure");
    h_indptr_.attach(indptr, (num_nodes + 1) * 8, /*keep=*/false, st);
    h_indices_.attach(indices, num_edges * 8, host_rows, st);
    if (bias_) h_probs_.attach(probs, num_edges * 4, host_rows, st);
    const int64_t *d_indptr = (const int64_t *)h_indptr_.dev;
    DGS_HIP(hipMalloc(&sub_indptr, sizeof(int64_t) * (size_t)(n_cache + 1)));
    extract_indptr(nids, n_cache, d_indptr, sub_indptr, st);
    DGS_HIP(hipMemcpyAsync(&n_sub, sub_indptr + n_cache, sizeof(int64_t),
                           hipMemcpyDeviceToHost, st));
    DGS_HIP(hipStreamSynchronize(st));
    DGS_HIP(hipMalloc(&sub_indices, sizeof(int64_t) * (size_t)(n_sub > 0 ? n_sub : 1)));
    extract_edge_data(nids, n_cache, d_indptr, sub_indptr, h_indices_.dev, 8, sub_indices, st);
    if (bias_) {
      DGS_HIP(hipMalloc(&sub_probs, sizeof(float) * (size_t)(n_sub > 0 ? n_sub : 1)));
      extract_edge_data(nids, n_cache, d_indptr, sub_indptr, h_probs_.dev, 4, sub_probs, st);
    }
    DGS_HIP(hipStreamSynchronize(st));
  } catch (const std::exception &e) {
    err = e.what();
  }
  try {
    c.check_all(err, "P2PCacheSampler: building the cache");
  } catch (...) {
    (void)hipDeviceSynchronize();
    for (void *p : {(void *)sub_indptr, sub_indices, sub_probs})
      if (p) (void)hipFree(p);
    delete nids_srv_;  // (collective: every rank is on this path)
    nids_srv_ = nullptr;
    throw;
  }
  const int64_t *d_indptr = (const int64_t *)h_indptr_.dev;
  indptr_srv_ = P2PServer::adopt(sub_indptr, n_cache + 1, 8);
  indices_srv_ = P2PServer::adopt(sub_indices, n_sub, 8);
  if (bias_) probs_srv_ = P2PServer::adopt(sub_probs, n_sub, 4);

  // graph shard context: node table (replaces CreateNidsP2PCacheHashMapCUDA, hashmap.cu)
  ntab_.ensure(sizeof(NodeEntry) * (size_t)(num_nodes > 0 ? num_nodes : 1));
  NodeEntry *ntab = ntab_.as<NodeEntry>();
  ntab_init_host(ntab, d_indptr, num_nodes, (const int64_t *)h_indices_.dev, st);
  for (int d : rotation(rank_, world_))
    ntab_assign(ntab, num_nodes, (const int64_t *)nids_srv_->ptr(d),
                (const int64_t *)indptr_srv_->ptr(d), nids_srv_->items(d), d,
                (const int64_t *)indices_srv_->ptr(d), st);
  DGS_HIP(hipStreamSynchronize(st));
  // the table's host pointers name exactly the uncovered rows
  DGS_CHECK((count_loc(ntab, num_nodes, kLocHost, st) > 0) == host_rows,
            "sampler: node table and cache coverage disagree");
  h_indptr_.release();
  if (!host_rows) {
    h_indices_.release();
    h_probs_.release();
  }

  src_.ntab = ntab;
  src_.indptr = nullptr;
  src_.indices = nullptr;
  for (int d = 0; d <= kMaxDevices; ++d) {
    src_.indices_base.p[d] = nullptr;
    src_.probs.p[d] = nullptr;
  }
  for (int d = 0; d < world_; ++d) {
    src_.indices_base.p[d] = indices_srv_->ptr(d);
    src_.probs.p[d] = bias_ ? probs_srv_->ptr(d) : nullptr;
  }
  src_.indices_base.p[kLocHost] = h_indices_.dev;
  src_.probs.p[kLocHost] = bias_ ? h_probs_.dev : nullptr;
  src_.num_nodes = num_nodes;
  src_.num_edges = num_edges;
}

// Stops a context's launcher thread and waits for its last call's kernels (the last relabel pass
// may still run) before its buffers go.  A job the launcher thread has taken is launched to the
// end (join waits for it) and its end event waited on; a job it has not taken is dropped
// unlaunched.  launch() records the end event also when it fails part way, so the event
// always follows every kernel the context enqueued.
void Sampler::retire(Ctx &c) {
  if (c.launcher.joinable()) {
    {
      std::lock_guard<std::mutex> g(c.mu);
      c.stop = true;
      c.stop_flag.store(true, std::memory_order_relaxed);
    }
    c.cv.notify_all();
    c.launcher.join();
  }
  if (c.seq > 0) {
    if (c.end_ev)
      (void)hipEventSynchronize(c.end_ev);
    else
      (void)hipStreamSynchronize(c.stream);
  }
  if (c.end_ev) (void)hipEventDestroy(c.end_ev);
  c.end_ev = nullptr;
}

Sampler::~Sampler() {
  for (auto &kv : ctxs_) retire(*kv.second);
  ctxs_.clear();
  // the graph's device copies may still be read by a call whose context was already retired
  // by a failing caller: nothing of this device runs when they go
  (void)hipDeviceSynchronize();
  delete indptr_srv_;
  delete indices_srv_;
  delete probs_srv_;
  delete nids_srv_;
}

void Sampler::bounds(int64_t n_seeds, const int64_t *fan_out, int L, int64_t *fcap,
                     int64_t *ecap) const {
  // frontier_h <= S_h * (1 + k) and, being unique node ids, <= N (the first hop's seeds may
  // repeat, so its bound keeps S_0 in).
  int64_t s = n_seeds;
  for (int h = 0; h < L; ++h) {
    const int64_t k = fan_out[L - 1 - h];
    DGS_CHECK(k >= 0, "fan_out entries must be non-negative");
    // The relabel tables record positions in cat(seeds, col) as int32 (kTableNoPos = INT32_MAX
    // is the empty mark): every position of the hop must stay below it.
    DGS_CHECK(k == 0 || s <= (int64_t)(INT32_MAX - 1 - s) / k,
              "one hop of this call could hold 2^31 - 1 or more seeds + sampled edges "
              "(relabel positions are 32-bit): split the seed batch");
    const int64_t e = s * k;
    ecap[h] = e;
    s = s + e;
    if (s > num_nodes_ && num_nodes_ > 0) s = std::max<int64_t>(num_nodes_, 1);
    fcap[h] = s;
  }
}

std::shared_ptr<Sampler::Ctx> Sampler::ctx_for(hipStream_t st) {
  std::shared_ptr<Ctx> c, victim;
  {
    std::lock_guard<std::mutex> g(ctx_mu_);
    std::shared_ptr<Ctx> &slot = ctxs_[st];
    if (!slot) {
      slot = std::make_shared<Ctx>();
      slot->stream = st;
    }
    slot->last_use = ++ctx_tick_;
    c = slot;
    if (ctxs_.size() > max_ctx_) {
      auto best = ctxs_.end();
      for (auto it = ctxs_.begin(); it != ctxs_.end(); ++it) {
        if (it->second == c || it->second.use_count() != 1) continue;  // held by a caller
        std::unique_lock<std::mutex> lk(it->second->mu, std::try_to_lock);
        if (!lk.owns_lock() || it->second->pending) continue;  // a call is outstanding
        if (best == ctxs_.end() || it->second->last_use < best->second->last_use) best = it;
      }
      if (best != ctxs_.end()) {
        victim = std::move(best->second);
        ctxs_.erase(best);
      }
    }
  }
  if (victim) retire(*victim);  // no longer reachable: nothing else can hold it
  return c;
}

size_t Sampler::num_contexts() {
  std::lock_guard<std::mutex> g(ctx_mu_);
  return ctxs_.size();
}

// sampler.cc:14-62, 146-166: hops run fan_out[L-1] .. fan_out[0]; seeds <- frontier.
// All hops are enqueued without host synchronisation: hop h+1 reads its seed count from the
// device word the relabel of hop h wrote, grids are sized by the host-side upper bounds, and
// the per-hop sizes are published to pinned host memory by the last kernel.
// DGS_CALL_TRACE=1 (diagnostics): host time of the synchronous call's phases -- entry to the
// last launch enqueued, then to the sizes seen -- averaged and printed to stderr at exit.
namespace {
struct CallTrace {
  std::mutex mu;
  int64_t n = 0;
  double launch_us = 0, wait_us = 0;
  ~CallTrace() {
    if (n)
      fprintf(stderr, "[dgs call trace] %lld synchronous calls: launches %.2f us, wait for sizes "
              "%.2f us (host, per call)\n", (long long)n, launch_us / n, wait_us / n);
  }
};
CallTrace *call_trace() {
  // (printed by the destructor at process exit)
  static std::unique_ptr<CallTrace> t(std::getenv("DGS_CALL_TRACE") ? new CallTrace() : nullptr);
  return t.get();
}
}  // namespace

void Sampler::sample(const int64_t *seeds, int64_t n_seeds, const int64_t *fan_out, int L,
                     bool replace, int64_t *const *frontiers, int64_t *const *rows,
                     int64_t *const *cols, int64_t *sizes, hipStream_t st,
                     const uint64_t *launch_seeds) {
  if (L <= 0) return;
  CallTrace *tr = call_trace();
  const auto t0 = std::chrono::steady_clock::now();
  sample_begin(seeds, n_seeds, fan_out, L, replace, frontiers, rows, cols, st, launch_seeds,
               /*host_async=*/false, /*solo=*/true);
  const auto t1 = std::chrono::steady_clock::now();
  sample_end(L, sizes, st);
  if (tr) {
    const auto t2 = std::chrono::steady_clock::now();
    std::lock_guard<std::mutex> g(tr->mu);
    tr->n += 1;
    tr->launch_us += std::chrono::duration<double, std::micro>(t1 - t0).count();
    tr->wait_us += std::chrono::duration<double, std::micro>(t2 - t1).count();
  }
}

// Per-context device words, at fixed offsets whatever the call's hop count: the diagnostics of
// the call's first out-of-range sampled id ({seq, hop, edge, id, nnz, row}, IdCheck), the
// flag word, then 3 sizes per hop.  The flag word and the sizes are published together.
constexpr int kDbgWords = 8;
constexpr int kFlagWord = kDbgWords;
constexpr int kSizes0 = kFlagWord + 1;

// Enqueues every hop of one call on `st` and returns: the call's sizes are read by
// sample_end.  One call per stream may be outstanding (its context holds the published sizes).
void Sampler::sample_begin(const int64_t *seeds, int64_t n_seeds, const int64_t *fan_out,
                           int L, bool replace, int64_t *const *frontiers,
                           int64_t *const *rows, int64_t *const *cols, hipStream_t st,
                           const uint64_t *launch_seeds, bool host_async, bool solo) {
  DGS_CHECK(L > 0, "sample: empty fan_out");
  for (int h = 0; h < L; ++h) DGS_CHECK(fan_out[h] >= 0, "fan_out entries must be non-negative");
  Job j;
  j.seeds = seeds;
  j.n_seeds = n_seeds;
  j.L = L;
  j.replace = replace;
  j.solo = solo;
  j.fan_out.assign(fan_out, fan_out + L);
  j.fr.assign(frontiers, frontiers + L);
  j.rows.assign(rows, rows + L);
  j.cols.assign(cols, cols + L);
  const std::shared_ptr<Ctx> cp = ctx_for(st);
  Ctx &c = *cp;
  std::unique_lock<std::mutex> lk(c.mu);
  DGS_CHECK(!c.pending, "sample: the previous call on this stream has not been ended");
  // One launch seed per hop (rowwise_sampling.cu:162), drawn together so that concurrent calls
  // on other streams cannot interleave with this call's draws (a rejected call draws none).
  j.hop_seed.resize(L);
  if (launch_seeds)
    std::copy(launch_seeds, launch_seeds + L, j.hop_seed.begin());
  else
    rng().next_n(L, j.hop_seed.data());
  c.pending = true;
  c.pending_L = L;
  c.pending_seeds = n_seeds;
  if (!host_async) {
    try {
      launch(c, j, st);
    } catch (...) {
      c.pending = false;
      throw;
    }
    return;
  }
  // The context's launcher thread issues the launches (about 2.7 us of host time each); the
  // caller's thread is free at once.  sample_end waits for it.
  if (!c.launcher.joinable()) {
    int dev = 0;
    DGS_HIP(hipGetDevice(&dev));
    c.launcher = std::thread([this, &c, dev] { launcher_loop(c, dev); });
  }
  c.job = std::move(j);
  c.job_ready = true;
  c.job_flag.store(true, std::memory_order_release);
  c.job_done = false;
  c.job_err = nullptr;
  c.cv.notify_all();
}

void Sampler::launcher_loop(Ctx &c, int dev) {
  (void)hipSetDevice(dev);
  // Spin up to DGS_LAUNCHER_SPIN_US (default 1000; 0 = off) for the next job before sleeping on
  // the condition variable: a sleeping thread's wake-up delays the batch's first launch (same
  // box: biased pipeline +2 %, arxiv-like loader 35.5 -> 31.9 us/batch, 20 steps +1 %).
  static const int64_t spin_ns = [] {
    const char *e = std::getenv("DGS_LAUNCHER_SPIN_US");
    return (e ? (int64_t)std::atoll(e) : (int64_t)1000) * 1000;
  }();
  // Adaptive: the thread spins only while jobs keep arriving within the window (a loader's
  // batch cadence); once a wait outlasts it, the next waits sleep until a job again comes
  // within the window of the previous one, so an idle sampler holds no core.
  bool spin = spin_ns > 0;
  auto idle_since = std::chrono::steady_clock::now();
  std::unique_lock<std::mutex> lk(c.mu);
  for (;;) {
    if (spin && !c.job_ready && !c.stop) {
      lk.unlock();
      for (uint32_t i = 1; !c.job_flag.load(std::memory_order_acquire); ++i) {
        __builtin_ia32_pause();
        if ((i & 63) == 0 &&
            (c.stop_flag.load(std::memory_order_relaxed) ||
             std::chrono::duration_cast<std::chrono::nanoseconds>(
                 std::chrono::steady_clock::now() - idle_since).count() > spin_ns))
          break;
      }
      lk.lock();
    }
    c.cv.wait(lk, [&] { return c.job_ready || c.stop; });
    if (spin_ns > 0)
      spin = std::chrono::duration_cast<std::chrono::nanoseconds>(
                 std::chrono::steady_clock::now() - idle_since).count() <= spin_ns;
    if (c.stop) return;
    c.job_ready = false;
    c.job_flag.store(false, std::memory_order_relaxed);
    Job j = std::move(c.job);
    lk.unlock();
    std::exception_ptr err;
    try {
      launch(c, j, c.stream);
    } catch (...) {
      err = std::current_exception();
    }
    lk.lock();
    c.job_err = err;
    c.job_done = true;
    c.cv.notify_all();
    idle_since = std::chrono::steady_clock::now();
  }
}

// Enqueues every hop of one call (the caller holds the context: its `pending` flag is set).  The
// context's end event is recorded after the launches, also when a launch fails part way (the
// kernels enqueued before the failure still run: retire() waits for them on this event).
void Sampler::launch(Ctx &c, const Job &j, hipStream_t st) {
  if (!c.end_ev) DGS_HIP(hipEventCreateWithFlags(&c.end_ev, hipEventDisableTiming));
  try {
    launch_hops(c, j, st);
  } catch (...) {
    (void)hipEventRecord(c.end_ev, st);
    throw;
  }
  // recorded here (on the launcher thread when the call is asynchronous), so a consumer of the
  // outputs only needs a stream wait on the caller's thread (ended_event)
  DGS_HIP(hipEventRecord(c.end_ev, st));
}

void Sampler::launch_hops(Ctx &c, const Job &j, hipStream_t st) {
  const int64_t *seeds = j.seeds;
  const int64_t n_seeds = j.n_seeds;
  const int L = j.L;
  const bool replace = j.replace;
  const int64_t *fan_out = j.fan_out.data();
  int64_t *const *frontiers = j.fr.data();
  int64_t *const *rows = j.rows.data();
  int64_t *const *cols = j.cols.data();
  const uint64_t *hop_seed = j.hop_seed.data();
  // Device words (kDbgWords diagnostics, the flag word, 3 sizes per hop; zeroed at allocation).
  // The flag word holds seq when this call saw a seed outside [0, num_nodes) and -seq when one
  // of its sampled ids was outside it (an out-of-range id in the graph's indices, or an internal
  // error): tagged by the call, so it is never reset and never read for another call.
  if (c.sizes.ensure(sizeof(int64_t) * (size_t)(kSizes0 + 3 * L)))
    DGS_HIP(hipMemsetAsync(c.sizes.p, 0, c.sizes.bytes, st));
  // pinned host words: [0] publication sequence, [1] flag, [2 + 3h + i] sizes
  if (c.sizes_host.bytes < sizeof(int64_t) * (size_t)(3 * L + 2)) {
    c.sizes_host.flags = hipHostMallocCoherent | hipHostMallocMapped;
    c.sizes_host.ensure(sizeof(int64_t) * (size_t)(3 * L + 2));
    // every word zeroed: the per-hop markers (host[2 + 3h]) are compared with the call's
    // sequence number, and a recycled pinned block could hold a matching stale value
    std::memset(c.sizes_host.p, 0, c.sizes_host.bytes);
    DGS_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&c.sizes_host_dev),
                                    c.sizes_host.p, 0));
  }
  int64_t *dsz = c.sizes.as<int64_t>();
  int64_t *dsizes = dsz + kSizes0;  // hop h: [3h + 1] unique count, [3h + 2] nnz
  // (the previous call on this stream may still be relabelling: stream order covers it)
  const uint64_t seq = ++c.seq;
  RowSrc src = src_;
  src.bad = dsz + kFlagWord;
  src.bad_tag = (int64_t)seq;
  IdCheck chk;
  chk.bad = dsz + kFlagWord;
  chk.bad_tag = -(int64_t)seq;
  chk.dbg = dsz;
  chk.seq = seq;
  std::vector<int64_t> fcap(L), ecap(L);
  bounds(n_seeds, fan_out, L, fcap.data(), ecap.data());
  const int64_t *cur = seeds;
  Count S{n_seeds, nullptr};
  profile_begin(st, 1);
  // Relabel tables alternate between hops (hop h uses table h & 1): the last pass of hop h's
  // relabel, which empties table h & 1, runs in the same launch as hop h+1's prep, which fills
  // the other one.
  RelabelTail tail{};
  bool have_tail = false;
  for (int h = 0; h < L; ++h) {
    const int64_t k = fan_out[L - 1 - h];
    const uint64_t seed = hop_seed[h];
    const int64_t nnz_cap = ecap[h];
    int64_t *d_nnz = dsizes + 3 * h + 2;
    int64_t *d_uniq = dsizes + 3 * h + 1;
    const int tb = h & 1;
    const Table t = direct_table(c.dpair[tb], num_nodes_, &c.dirty[tb], st);
    c.dirty[tb] = true;
    // rows[h] receives each edge's seed row r from the sampler and is relabelled in place
    sample_hop(src, cur, S, k, replace, bias_, seed, rows[h], cols[h], d_nnz, t, c.ws, st,
               have_tail ? &tail : nullptr, j.solo);
    if (have_tail) c.dirty[tb ^ 1] = false;  // the previous hop's clean-up is enqueued
    // the last hop's scatter publishes the flag word and every size to pinned host memory (no
    // copy, no sync); each hop's count pass range-checks its sampled ids before that, so the
    // call sees its own flag
    // Every hop's scatter publishes its (U, nnz) with the call's sequence number in the hop's
    // S slot (host[2 + 3h], which the host never reads as a size), so a synchronous caller can
    // build hop h's views while later hops run (sample_wait_hop); the last hop's publication
    // then writes the flag word and every size (host[2 + 3h] back to the device word's 0).
    const bool last = h == L - 1;
    const HostSizes pub =
        last ? HostSizes{dsz + kFlagWord, 3 * L + 1, c.sizes_host_dev, seq}
             : HostSizes{dsizes + 3 * h + 1, 2, c.sizes_host_dev + 2 + 3 * h, seq};
    chk.hop = h;
    relabel_hop(cur, S, cols[h], d_nnz, nnz_cap, /*seeds_unique=*/h > 0, t, frontiers[h],
                rows[h], cols[h], d_uniq, c.ws, st, pub, &tail, chk);
    if (last) launch_relabel_tail(tail, st);
    have_tail = !last;
    if (last) c.dirty[tb] = false;
    cur = frontiers[h];
    S = Count{fcap[h], d_uniq};
  }
  profile_end(st, 1);
}

// Lookup only: a missing context is an error (never created, never evicting another).
std::shared_ptr<Sampler::Ctx> Sampler::ctx_find(hipStream_t st) {
  std::lock_guard<std::mutex> g(ctx_mu_);
  auto it = ctxs_.find(st);
  return it == ctxs_.end() ? nullptr : it->second;
}

void Sampler::wait_ended(hipStream_t st, hipStream_t consumer) {
  const std::shared_ptr<Ctx> cp = ctx_find(st);
  DGS_CHECK(cp, "wait_ended: this stream has no sampling context (no call was ended on it, or "
                "its context was evicted: more than DGS_SAMPLER_MAX_CTX streams in use)");
  Ctx &c = *cp;
  std::lock_guard<std::mutex> g(c.mu);
  DGS_CHECK(!c.pending && c.end_ev, "wait_ended: no ended call on this stream");
  DGS_HIP(hipStreamWaitEvent(consumer, c.end_ev, 0));
}

// Waits for the sizes of the call begun on `st` (published by its last scatter kernel): the
// host returns while the last relabel pass still runs (every consumer of the outputs is
// ordered after it on the stream).  A failed kernel shows up through hipStreamQuery.
void Sampler::sample_end(int L, int64_t *sizes, hipStream_t st) {
  const std::shared_ptr<Ctx> cp = ctx_find(st);
  DGS_CHECK(cp, "sample_end: no call outstanding on this stream");
  Ctx &c = *cp;
  std::unique_lock<std::mutex> lk(c.mu);
  DGS_CHECK(c.pending, "sample_end: no call outstanding on this stream");
  DGS_CHECK(L == c.pending_L, "sample_end: hop count differs from the call's");
  c.cv.wait(lk, [&] { return c.job_done; });  // an asynchronous launch has been issued
  c.pending = false;
  if (c.job_err) {
    std::exception_ptr e = c.job_err;
    c.job_err = nullptr;
    std::rethrow_exception(e);
  }
  const int64_t *hsz = c.sizes_host.as<int64_t>();
  const uint64_t seq = c.seq;
  const int64_t n_seeds = c.pending_seeds;
  for (uint64_t spin = 1;; ++spin) {
    if (__atomic_load_n(hsz, __ATOMIC_ACQUIRE) == (int64_t)seq) break;
    if ((spin & 255) == 0) {
      const hipError_t q = hipStreamQuery(st);
      if (q == hipSuccess) {
        DGS_CHECK(__atomic_load_n(hsz, __ATOMIC_ACQUIRE) == (int64_t)seq,
                  "sample: sizes were not published");
        break;
      }
      if (q != hipErrorNotReady) DGS_HIP(q);
    }
    __builtin_ia32_pause();
  }
  // A call with a bad seed fails after it has run (its rows were sampled as empty; the
  // reference reads out of bounds instead).
  const int64_t flag = hsz[1];
  DGS_CHECK(flag != (int64_t)seq, "sample: a seed is outside [0, num_nodes)");
  if (flag == -(int64_t)seq) {
    int64_t d[kDbgWords] = {};
    (void)hipMemcpy(d, c.sizes.as<int64_t>(), sizeof(d), hipMemcpyDeviceToHost);
    DGS_CHECK(false, "sample: a sampled neighbour id was outside [0, num_nodes): the graph's "
                         "indices hold an id out of range, or an internal error (first: hop " +
                         std::to_string(d[1]) + " edge " + std::to_string(d[2]) +
                         " id " + std::to_string(d[3]) + " nnz " + std::to_string(d[4]) +
                         " row " + std::to_string(d[5]) + ")");
  }
  int64_t s = n_seeds;
  for (int h = 0; h < L; ++h) {
    sizes[3 * h + 0] = s;
    sizes[3 * h + 1] = hsz[2 + 3 * h + 1];
    sizes[3 * h + 2] = hsz[2 + 3 * h + 2];
    s = sizes[3 * h + 1];
  }
}

// Waits until hop h (< L - 1) of the call outstanding on `st` has published its sizes (or the
// whole call has), without ending the call; u_nnz = (U_h, nnz_h).
void Sampler::sample_wait_hop(int L, int h, int64_t *u_nnz, hipStream_t st) {
  const std::shared_ptr<Ctx> cp = ctx_find(st);
  DGS_CHECK(cp, "sample_wait_hop: no call outstanding on this stream");
  Ctx &c = *cp;
  std::unique_lock<std::mutex> lk(c.mu);
  DGS_CHECK(c.pending, "sample_wait_hop: no call outstanding on this stream");
  DGS_CHECK(L == c.pending_L && h >= 0 && h < L, "sample_wait_hop: bad hop");
  c.cv.wait(lk, [&] { return c.job_done; });  // an asynchronous launch has been issued
  DGS_CHECK(!c.job_err, "sample_wait_hop: the call's launch failed (sample_end reports it)");
  const int64_t *hsz = c.sizes_host.as<int64_t>();
  const int64_t seq = (int64_t)c.seq;
  for (uint64_t spin = 1;; ++spin) {
    if (__atomic_load_n(hsz + 2 + 3 * h, __ATOMIC_ACQUIRE) == seq ||
        __atomic_load_n(hsz, __ATOMIC_ACQUIRE) == seq)
      break;
    if ((spin & 255) == 0) {
      const hipError_t q = hipStreamQuery(st);
      if (q == hipSuccess) {
        DGS_CHECK(__atomic_load_n(hsz + 2 + 3 * h, __ATOMIC_ACQUIRE) == seq ||
                      __atomic_load_n(hsz, __ATOMIC_ACQUIRE) == seq,
                  "sample: sizes were not published");
        break;
      }
      if (q != hipErrorNotReady) DGS_HIP(q);
    }
    __builtin_ia32_pause();
  }
  u_nnz[0] = hsz[3 + 3 * h];
  u_nnz[1] = hsz[4 + 3 * h];
}

void Sampler::build_cache_rowtab(int64_t *tab, hipStream_t st) const {
  loctab_init_host(tab, num_nodes_, st);
  for (int d : rotation(rank_, world_))
    loctab_assign(tab, num_nodes_, (const int64_t *)nids_srv_->ptr(d), nids_srv_->items(d), d,
                  st);
}

int64_t Sampler::cache_hashmap_capacity() const {
  int64_t total = 0;
  for (int d = 0; d < world_; ++d) total += nids_srv_->items(d);
  return refmap_dir_size(total);
}

void Sampler::cache_hashmap_fill(int id_bytes, void *key, void *idx, void *devid,
                                 hipStream_t st) const {
  std::vector<const int64_t *> lists(world_);
  std::vector<int64_t> counts(world_);
  for (int d = 0; d < world_; ++d) {
    lists[d] = (const int64_t *)nids_srv_->ptr(d);
    counts[d] = nids_srv_->items(d);
  }
  const std::vector<int> order = rotation(rank_, world_);  // remote ranks, then the local one
  refmap_build(lists.data(), counts.data(), order.data(), (int)order.size(), id_bytes,
               cache_hashmap_capacity(), key, idx, devid, st);
}

int64_t Sampler::cache_map_size() const {
  int64_t n = 0;
  for (int d = 0; d < world_; ++d) n += nids_srv_->items(d);
  // upper bound before dedup; the exact count is produced by cache_map_fill's caller query
  int64_t *tab = nullptr;
  hipStream_t st = nullptr;
  DGS_HIP(hipMalloc(&tab, sizeof(int64_t) * (size_t)(num_nodes_ > 0 ? num_nodes_ : 1)));
  build_cache_rowtab(tab, st);
  int64_t *cnt = nullptr;
  DGS_HIP(hipMalloc(&cnt, sizeof(int64_t)));
  cache_map_compact(tab, num_nodes_, nullptr, nullptr, nullptr, cnt, st);
  DGS_HIP(hipMemcpy(&n, cnt, sizeof(int64_t), hipMemcpyDeviceToHost));
  DGS_HIP(hipFree(cnt));
  DGS_HIP(hipFree(tab));
  return n;
}

void Sampler::cache_map_fill(int64_t *key, int64_t *idx, int64_t *devid, hipStream_t st) const {
  int64_t *tab = nullptr, *cnt = nullptr;
  DGS_HIP(hipMalloc(&tab, sizeof(int64_t) * (size_t)(num_nodes_ > 0 ? num_nodes_ : 1)));
  DGS_HIP(hipMalloc(&cnt, sizeof(int64_t)));
  build_cache_rowtab(tab, st);
  cache_map_compact(tab, num_nodes_, key, idx, devid, cnt, st);
  DGS_HIP(hipStreamSynchronize(st));
  DGS_HIP(hipFree(cnt));
  DGS_HIP(hipFree(tab));
}

// ============================================================== FeatureServer
// feature_server.cc:10-61: cache rows = data[cache_nids] in this GPU's HBM, cache lists
// all-gathered with RCCL (NCCLTensorAllGather_), node -> (GPU, row) map with local priority.
FeatureServer::FeatureServer(const void *data, int64_t num_rows, int64_t row_bytes,
                             const int64_t *cache_nids, int64_t n_cache, int64_t device_id) {
  Comm &c = Comm::get();
  rank_ = c.rank();
  world_ = c.world();
  num_rows_ = num_rows;
  row_bytes_ = row_bytes;
  hipStream_t st = nullptr;
  // the local checks, then their outcome made collective (as the sampler's)
  int64_t *nids = nullptr;
  std::string err;
  try {
    DGS_CHECK(device_id == rank_ || c.host_mode() || !c.initialized(),
              "device_id must equal the communicator rank (feature_server.cc:14)");
    nids = device_copy_ids(cache_nids, n_cache, st);
    // a cached id outside [0, num_rows) is refused (the reference's hashmap would take it and
    // its gather read out of bounds, feature_server.cc:10-61)
    DGS_CHECK(count_out_of_range(nids, n_cache, num_rows, st) == 0,
              "cache_nids: an id is outside [0, num_rows)");
  } catch (const std::exception &e) {
    err = e.what();
  }
  try {
    c.check_all(err, "P2PCacheFeatureServer: argument checks");
  } catch (...) {
    if (nids) (void)hipFree(nids);
    throw;
  }
  // every rank's cache list (NCCLTensorAllGather_), first: rows no GPU caches are read from the
  // host while the server lives (a pinned mirror); with none, the host matrix only fills the
  // caches (a device temporary)
  std::vector<int64_t> nbytes(world_, n_cache * 8);
  DGS_CHECK(world_ <= kMaxDevices, "at most 8 GPUs");
  std::vector<void *> lists(world_, nullptr);
  if (world_ > 1) {
    lists = c.allgather_device(nids, n_cache * 8, &nbytes);
  } else {
    lists[0] = nids;
  }
  std::vector<const int64_t *> lp(world_);
  std::vector<int64_t> counts(world_);
  for (int d = 0; d < world_; ++d) {
    lp[d] = (const int64_t *)lists[d];
    counts[d] = nbytes[d] / 8;
  }
  // this rank's cache block, the outcome made collective before the blocks are exchanged
  void *block = nullptr;
  bool host_rows = false;
  std::string berr;
  try {
    host_rows = count_uncovered(lp.data(), counts.data(), world_, num_rows, st) > 0;
    DGS_CHECK(!test_build_fail(rank_), "test hook: feature server build failure");
    h_data_.attach(data, num_rows * row_bytes, host_rows, st);
    DGS_HIP(hipMalloc(&block, (size_t)(n_cache * row_bytes > 0 ? n_cache * row_bytes : 1)));
    gather_plain(h_data_.dev, num_rows, row_bytes, nids, 8, n_cache, block, st);
    DGS_HIP(hipStreamSynchronize(st));
  } catch (const std::exception &e) {
    berr = e.what();
  }
  try {
    c.check_all(berr, "P2PCacheFeatureServer: building the cache");
  } catch (...) {
    (void)hipDeviceSynchronize();
    if (block) (void)hipFree(block);
    (void)hipFree(nids);
    for (int d = 0; d < world_; ++d)
      if (world_ > 1 && lists[d]) (void)hipFree(lists[d]);
    throw;
  }
  feat_srv_ = P2PServer::adopt(block, n_cache, row_bytes);

  ftab_.ensure(sizeof(int64_t) * (size_t)(num_rows > 0 ? num_rows : 1));
  int64_t *ftab = ftab_.as<int64_t>();
  // absolute row addresses: host rows first, then every GPU's cache (local last = priority)
  ftab_init(ftab, num_rows, h_data_.dev, row_bytes, st);
  align_or_ = host_rows ? (uintptr_t)h_data_.dev : 0;
  for (int d : rotation(rank_, world_)) {
    ftab_assign(ftab, num_rows, (const int64_t *)lists[d], nbytes[d] / 8, feat_srv_->ptr(d),
                row_bytes, st);
    align_or_ |= (uintptr_t)feat_srv_->ptr(d);
  }
  DGS_HIP(hipStreamSynchronize(st));
  detect_strided(lists, nbytes, st);
  if (world_ > 1)
    for (void *p : lists) DGS_HIP(hipFree(p));
  DGS_HIP(hipFree(nids));
  if (!host_rows) {
    // every row is cached on some GPU: no entry of the table names the host source
    DGS_CHECK(!h_data_.dev || num_rows * row_bytes == 0 ||
                  count_in_range(ftab, num_rows, h_data_.dev, num_rows * row_bytes, st) == 0,
              "feature server: address table and cache coverage disagree");
    h_data_.release();
  }
}

// Whole graph cached in a computable layout: the local list is arange(N) (local priority makes
// every read local), or GPU d holds arange(d, N, W) for a power-of-two W (the v mod W shard).
void FeatureServer::detect_strided(const std::vector<void *> &lists,
                                   const std::vector<int64_t> &nbytes, hipStream_t st) {
  const int64_t N = num_rows_;
  if (N <= 0) return;
  if (nbytes[rank_] / 8 == N &&
      count_stride_mismatch((const int64_t *)lists[rank_], N, 0, 1, st) == 0) {
    wshift_ = 0;
    for (int d = 0; d < kMaxDevices; ++d) bases_[d] = feat_srv_->ptr(rank_);
    return;
  }
  const int W = world_;
  if (W < 2 || (W & (W - 1)) != 0) return;
  for (int d = 0; d < W; ++d) {
    const int64_t want = N > d ? (N - d + W - 1) / W : 0;
    if (nbytes[d] / 8 != want) return;
    if (count_stride_mismatch((const int64_t *)lists[d], want, d, W, st) != 0) return;
  }
  int sh = 0;
  while ((1 << sh) < W) ++sh;
  for (int d = 0; d < kMaxDevices; ++d) bases_[d] = feat_srv_->ptr(d < W ? d : 0);
  wshift_ = sh;
}

FeatureServer::~FeatureServer() {
  // gathers queued on any stream read the table, the cache blocks and the host view: they
  // finish before those go
  (void)hipDeviceSynchronize();
  delete feat_srv_;
}

void FeatureServer::gather(const int64_t *nids, int64_t n, void *out, hipStream_t st,
                           const LabelTail *tail) const {
  if (wshift_ >= 0)
    gather_strided(bases_, wshift_, num_rows_, row_bytes_, nids, n, out, st, tail);
  else
    gather_table(ftab_.as<int64_t>(), num_rows_, align_or_, row_bytes_, nids, n, out, st, tail);
}

}  // namespace dgs

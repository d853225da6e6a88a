// capi.cpp -- extern "C" boundary (include/dgs_amd.h).  Every entry point maps C++
// exceptions to a -1 return + thread-local message.
#include "../../include/dgs_amd.h"

#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_set>
#include <vector>

#include "services.h"

using namespace dgs;

namespace {
thread_local std::string g_err;

template <typename F>
int guard(F &&f) {
  try {
    f();
    return 0;
  } catch (const std::exception &e) {
    g_err = e.what();
  } catch (...) {
    g_err = "unknown error";
  }
  return -1;
}

hipStream_t S(void *s) { return reinterpret_cast<hipStream_t>(s); }

// The object behind a handle; a null handle (or one whose object is gone) is an error, not a
// crash (the Python binding passes None once an object has been destroyed).
template <typename H>
auto &obj(H *h, const char *what) {
  if (!h || !h->s) throw Error(std::string(what) + ": null handle (destroyed?)");
  return *h->s;
}

// Pointer usable by kernels: device memory or registered/pinned host memory.
template <typename T>
T *dev_ptr(T *p, const char *what) {
  if (!p) return p;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, (const void *)p) != hipSuccess) {
    (void)hipGetLastError();
    throw Error(std::string(what) + " must be a device (CUDA) tensor or pinned host memory");
  }
  if (a.type == hipMemoryTypeHost) {
    void *d = nullptr;
    if (hipHostGetDevicePointer(&d, (void *)p, 0) == hipSuccess && d) return (T *)d;
    (void)hipGetLastError();
    return a.devicePointer ? (T *)a.devicePointer : p;
  }
  if (a.type == hipMemoryTypeUnregistered)
    throw Error(std::string(what) + " must be a device (CUDA) tensor or pinned host memory");
  return p;
}

// Device-memory check for the per-batch entry points, remembered per address: a caching
// allocator hands the same few blocks back batch after batch, so the pointer query runs about
// once per block (a host pointer fails here instead of faulting on the GPU later).  Best effort:
// an address is not forgotten when its memory is freed, so a later allocation at a remembered
// address skips the query (the cache is dropped every 4096 new addresses).
void check_device_cached(const void *p, const char *what) {
  thread_local std::unordered_set<uintptr_t> seen;
  if (!p) throw Error(std::string(what) + " is null");
  if (seen.count((uintptr_t)p)) return;
  if (!is_device_pointer(p)) throw Error(std::string(what) + " must be device memory");
  if (seen.size() >= 4096) seen.clear();
  seen.insert((uintptr_t)p);
}

// Scratch of the standalone ops (dgs_sample_neighbors, dgs_relabel), one per (device, stream):
// calls on different streams or threads never share buffers, calls on one stream are ordered
// by the stream, and the returned lock serialises the host side of calls on one stream.  (The
// reference allocates per call through the caching allocator.)  At most kOpScratchMax entries
// are kept: a caller cycling through short-lived streams evicts the least recently used idle
// entry (its buffers are freed after a device synchronisation, so no launch still uses them).
struct OpScratch {
  std::mutex mu;
  HopScratch ws;
  uint64_t last_use = 0;
};
struct OpScratchLease {
  std::shared_ptr<OpScratch> o;  // keeps an entry evicted meanwhile alive until the call ends
  std::unique_lock<std::mutex> lk;
};
constexpr size_t kOpScratchMax = 16;
OpScratchLease op_scratch(hipStream_t st, HopScratch **ws) {
  static std::mutex m;
  static std::map<std::pair<int, hipStream_t>, std::shared_ptr<OpScratch>> all;
  static uint64_t tick = 0;
  int dev = 0;
  DGS_HIP(hipGetDevice(&dev));
  std::shared_ptr<OpScratch> o, evicted;
  {
    std::lock_guard<std::mutex> g(m);
    std::shared_ptr<OpScratch> &p = all[{dev, st}];
    if (!p) p = std::make_shared<OpScratch>();
    p->last_use = ++tick;
    o = p;
    if (all.size() > kOpScratchMax) {
      // only an entry of the current device: the synchronisation below covers its stream
      auto victim = all.end();
      for (auto it = all.begin(); it != all.end(); ++it)
        if (it->first.first == dev && it->second != o && it->second.use_count() == 1 &&
            (victim == all.end() || it->second->last_use < victim->second->last_use))
          victim = it;
      if (victim != all.end()) {
        evicted = std::move(victim->second);
        all.erase(victim);
      }
    }
  }
  if (evicted) {
    (void)hipDeviceSynchronize();  // its stream may be gone: wait for everything instead
    evicted.reset();
  }
  *ws = &o->ws;
  OpScratchLease lease{o, std::unique_lock<std::mutex>(o->mu)};
  return lease;
}
// `consumer` waits (on the device) for the work enqueued on `producer` so far.  One event per
// calling thread and device: a wait already enqueued keeps the record it saw, so the event can
// be recorded again at once.
void stream_wait_impl(void *producer, void *consumer) {
  thread_local std::vector<hipEvent_t> evs;
  int dev = 0;
  DGS_HIP(hipGetDevice(&dev));
  if ((int)evs.size() <= dev) evs.resize((size_t)dev + 1, nullptr);
  if (!evs[dev]) DGS_HIP(hipEventCreateWithFlags(&evs[dev], hipEventDisableTiming));
  hipEvent_t ev = evs[dev];
  DGS_HIP(hipEventRecord(ev, S(producer)));
  DGS_HIP(hipStreamWaitEvent(S(consumer), ev, 0));
}
}  // namespace

struct dgs_p2p_server {
  P2PServer *s;
};
struct dgs_sampler {
  Sampler *s;
};
struct dgs_feature_server {
  FeatureServer *s;
};

extern "C" {

const char *dgs_last_error(void) { return g_err.c_str(); }

const char *dgs_version(void) { return "dgs_amd 0.1 (gfx950, wave64, HIP)"; }

// ------------------------------------------------------------------ context
int dgs_get_unique_id(int64_t *out_id16) {
  return guard([&] {
    static_assert(sizeof(ncclUniqueId) <= 16 * sizeof(int64_t), "unique id size");
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) throw Error(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    std::memset(out_id16, 0, 16 * sizeof(int64_t));
    std::memcpy(out_id16, &id, sizeof(id));
  });
}

int dgs_set_nccl(int64_t nranks, const int64_t *unique_id, int64_t n_id, int64_t rank) {
  return guard([&] {
    DGS_CHECK(n_id * (int64_t)sizeof(int64_t) >= (int64_t)sizeof(ncclUniqueId),
              "unique id array too short");
    Comm::get().init((int)nranks, unique_id, (int)rank);
  });
}

int dgs_set_host_comm(int64_t nranks, int64_t rank, dgs_host_allgather_fn allgather,
                      dgs_host_barrier_fn barrier, void *ctx) {
  return guard([&] { Comm::get().init_host((int)nranks, (int)rank, allgather, barrier, ctx); });
}

int dgs_get_local_rank(void) { return Comm::get().rank(); }
int dgs_get_world_size(void) { return Comm::get().world(); }

int dgs_barrier(void) {
  return guard([&] { Comm::get().barrier(); });
}

int dgs_allgather_sizes(int64_t my_size, int64_t *all_sizes) {
  return guard([&] {
    std::vector<int64_t> v = Comm::get().allgather_sizes(my_size);
    std::memcpy(all_sizes, v.data(), sizeof(int64_t) * v.size());
  });
}

int dgs_allgather_bytes(const void *send, int64_t send_bytes, void *const *recv,
                        const int64_t *recv_bytes, void *stream) {
  return guard([&] { Comm::get().allgather_bytes(send, send_bytes, recv, recv_bytes, S(stream)); });
}

uint64_t dgs_randn_uint64(void) { return rng().next(); }

int dgs_randn_uint64_n(int64_t n, uint64_t *out) {
  return guard([&] {
    DGS_CHECK(n >= 0 && (n == 0 || out), "randn_uint64_n: bad arguments");
    rng().next_n(n, out);
  });
}

int dgs_set_random_seed(uint64_t seed) {
  rng().set_seed(seed);
  return 0;
}

// ------------------------------------------------------------------ host memory
int dgs_host_register(void *ptr, int64_t bytes) {
  return guard([&] {
    if (!ptr || bytes <= 0) return;
    // through the library's refcounted registry, shared with the services' host views
    host_pin(ptr, bytes);
  });
}

int dgs_host_unregister(void *ptr) {
  return guard([&] {
    if (!ptr) return;
    host_unpin(ptr);
  });
}

int dgs_host_registrations(int64_t cap, uint64_t *bases, int64_t *bytes, int64_t *refs,
                           int64_t *pins, int64_t *n_out) {
  return guard([&] {
    const std::vector<HostRegInfo> v = host_registrations();
    *n_out = (int64_t)v.size();
    for (int64_t i = 0; i < cap && i < (int64_t)v.size(); ++i) {
      if (bases) bases[i] = v[i].base;
      if (bytes) bytes[i] = v[i].bytes;
      if (refs) refs[i] = v[i].refs;
      if (pins) pins[i] = v[i].pins;
    }
  });
}

int dgs_host_memory_state(int64_t *n_registrations, int64_t *mirror_bytes,
                          int64_t *n_mirrors) {
  return guard([&] {
    *n_registrations = (int64_t)host_registrations().size();
    host_mirror_stats(mirror_bytes, n_mirrors);
  });
}

int dgs_abi_version(void) { return DGS_ABI_VERSION; }

// ------------------------------------------------------------------ async errors, streams
int dgs_check_async_errors(void) {
  return guard([&] { check_async_errors(); });
}

int dgs_last_gather_tag(uint64_t *tag) {
  return guard([&] { *tag = async_err_last_tag(); });
}

int dgs_stream_create(int priority, void **out) {
  return guard([&] {
    hipStream_t st = nullptr;
    DGS_HIP(hipStreamCreateWithPriority(&st, hipStreamNonBlocking, priority));
    *out = st;
  });
}

int dgs_stream_destroy(void *stream) {
  return guard([&] {
    DGS_CHECK(stream, "stream_destroy: the null stream is not the library's");
    DGS_HIP(hipStreamDestroy(S(stream)));
  });
}

// ------------------------------------------------------------------ ops
int dgs_index_select(const void *data, int64_t num_rows, int64_t row_bytes, const void *nid,
                     int nid_bytes, int64_t n, void *out, void *stream) {
  return guard([&] {
    check_async_errors();
    gather_plain(dev_ptr(data, "data"), num_rows, row_bytes, dev_ptr(nid, "nid"), nid_bytes, n,
                 out, S(stream));
  });
}

int dgs_index_select_device(const void *data, int64_t num_rows, int64_t row_bytes,
                            const void *nid, int nid_bytes, int64_t n, void *out, void *stream) {
  return guard([&] {
    check_async_errors();
    gather_plain(data, num_rows, row_bytes, nid, nid_bytes, n, out, S(stream));
  });
}

int dgs_stream_wait(void *producer, void *consumer) {
  return guard([&] { stream_wait_impl(producer, consumer); });
}

int dgs_stream_wait_event(void *event, void *consumer) {
  return guard([&] {
    DGS_CHECK(event, "stream_wait_event: null event");
    DGS_HIP(hipStreamWaitEvent(S(consumer), reinterpret_cast<hipEvent_t>(event), 0));
  });
}

int dgs_loader_gather(dgs_sampler *s, dgs_feature_server *fs, void *producer, void *consumer,
                      const int64_t *nids, int64_t n, void *feat_out, const void *labels,
                      int64_t label_rows, int64_t label_row_bytes, const int64_t *seeds,
                      int64_t n_seeds, void *label_out) {
  return guard([&] {
    check_async_errors();
    if (s)
      obj(s, "sampler").wait_ended(S(producer), S(consumer));
    else
      stream_wait_impl(producer, consumer);
    const bool want_labels = labels && n_seeds > 0;
    // 4- and 8-byte label rows ride in the feature gather's launch
    // (a zero-width feature matrix launches no gather: its labels go on their own)
    const bool fuse = want_labels && fs && n > 0 && obj(fs, "feature server").row_bytes() > 0 &&
                      n_seeds < (int64_t(1) << 31) &&
                      (label_row_bytes == 4 || label_row_bytes == 8) &&
                      ((uintptr_t)labels % label_row_bytes) == 0 &&
                      ((uintptr_t)label_out % label_row_bytes) == 0;
    LabelTail lt;
    if (fuse) {
      lt.data = (const char *)labels;
      lt.ids = seeds;
      lt.out = (char *)label_out;
      lt.nrows = (uint64_t)(label_rows > 0 ? label_rows : 0);
      lt.n = (uint32_t)n_seeds;
      lt.row_bytes = (uint32_t)label_row_bytes;
    }
    if (fs && n > 0) obj(fs, "feature server").gather(nids, n, feat_out, S(consumer),
                                                      fuse ? &lt : nullptr);
    if (want_labels && !fuse)
      gather_plain(labels, label_rows, label_row_bytes, seeds, 8, n_seeds, label_out,
                   S(consumer));
  });
}

int dgs_sample_neighbors(const int64_t *seeds, int64_t Sn, const int64_t *indptr,
                         const int64_t *indices, const float *probs, int64_t num_picks,
                         int replace, int64_t *out_row, int64_t *out_col, int64_t *nnz_out,
                         void *stream) {
  return guard([&] {
    hipStream_t st = S(stream);
    RowSrc src{};
    src.ntab = nullptr;
    src.indptr = dev_ptr(indptr, "indptr");
    src.indices = dev_ptr(indices, "indices");
    src.indices_base.p[0] = src.indices;
    src.probs.p[0] = dev_ptr(probs, "probs");
    src.num_nodes = INT64_MAX;  // no node count at this boundary (reference: unchecked)
    seeds = dev_ptr(seeds, "seeds");
    HopScratch *wsp = nullptr;
    const OpScratchLease lk = op_scratch(st, &wsp);
    HopScratch &ws = *wsp;
    // [0] = nnz, then rowpos[S*k]: the stream's op scratch (the library does not use the
    // stream-ordered allocator)
    const int64_t cap = Sn * num_picks;
    ws.op_tmp.ensure(sizeof(int64_t) * (size_t)(cap + 1));
    int64_t *tmp = ws.op_tmp.as<int64_t>();
    const Table no_table{nullptr, nullptr, nullptr, nullptr, 0};
    sample_hop(src, seeds, Count{Sn, nullptr}, num_picks, replace != 0, probs != nullptr,
               rng().next(), tmp + 1, out_col, tmp, no_table, ws, st);
    int64_t nnz = 0;
    DGS_HIP(hipMemcpyAsync(&nnz, tmp, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    DGS_HIP(hipStreamSynchronize(st));
    take_i64(seeds, tmp + 1, nnz, out_row, st);
    *nnz_out = nnz;
  });
}

int dgs_relabel(const int64_t *const *maps, const int64_t *map_sizes, int n_maps,
                const int64_t *const *reqs, const int64_t *req_sizes, int n_reqs,
                int64_t *unique_out, int64_t *n_unique, int64_t *const *req_out, void *stream) {
  return guard([&] {
    hipStream_t st = S(stream);
    int64_t nm = 0, nr = 0;
    for (int i = 0; i < n_maps; ++i) nm += map_sizes[i];
    for (int i = 0; i < n_reqs; ++i) nr += req_sizes[i];
    HopScratch *ws = nullptr;
    const OpScratchLease lk = op_scratch(st, &ws);
    // mapping[nm] | req[nr] | req_out[nr] | count, in the stream's op scratch
    ws->op_tmp.ensure(sizeof(int64_t) * (size_t)(nm + 2 * nr + 1));
    int64_t *buf = ws->op_tmp.as<int64_t>();
    int64_t off = 0;
    for (int i = 0; i < n_maps; ++i) {
      if (map_sizes[i] > 0)
        DGS_HIP(hipMemcpyAsync(buf + off, dev_ptr(maps[i], "mapping tensor"),
                               sizeof(int64_t) * map_sizes[i], hipMemcpyDefault, st));
      off += map_sizes[i];
    }
    for (int i = 0; i < n_reqs; ++i) {
      if (req_sizes[i] > 0)
        DGS_HIP(hipMemcpyAsync(buf + off, dev_ptr(reqs[i], "relabel tensor"),
                               sizeof(int64_t) * req_sizes[i], hipMemcpyDefault, st));
      off += req_sizes[i];
    }
    int64_t *d_cnt = buf + nm + 2 * nr;
    relabel_generic(buf, nm, buf + nm, nr, unique_out, buf + nm + nr, d_cnt, *ws, st);
    off = nm + nr;
    for (int i = 0; i < n_reqs; ++i) {
      if (req_sizes[i] > 0)
        DGS_HIP(hipMemcpyAsync(req_out[i], buf + off, sizeof(int64_t) * req_sizes[i],
                               hipMemcpyDeviceToDevice, st));
      off += req_sizes[i];
    }
    int64_t u = 0;
    DGS_HIP(hipMemcpyAsync(&u, d_cnt, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    DGS_HIP(hipStreamSynchronize(st));
    *n_unique = u;
  });
}

int dgs_extract_indptr(const int64_t *nids, int64_t n, const int64_t *indptr,
                       int64_t *sub_indptr, void *stream) {
  return guard([&] {
    extract_indptr(dev_ptr(nids, "nids"), n, dev_ptr(indptr, "indptr"), sub_indptr, S(stream));
  });
}

int dgs_extract_edge_data(const int64_t *nids, int64_t n, const int64_t *indptr,
                          const int64_t *sub_indptr, const void *edge_data, int64_t elem_bytes,
                          void *sub_edge_data, void *stream) {
  return guard([&] {
    extract_edge_data(dev_ptr(nids, "nids"), n, dev_ptr(indptr, "indptr"),
                      dev_ptr(sub_indptr, "sub_indptr"), dev_ptr(edge_data, "edge_data"),
                      elem_bytes, sub_edge_data, S(stream));
  });
}

int dgs_test_bias_bounds(const uint32_t *x, const float *p, const float *thr, int64_t n,
                         float *key, float *key_lower, uint8_t *flags, void *stream) {
  return guard([&] {
    DGS_CHECK(n >= 0, "negative size");
    if (n == 0) return;
    test_bias_bounds(dev_ptr(x, "x"), dev_ptr(p, "p"), dev_ptr(thr, "thr"), n,
                     dev_ptr(key, "key"), dev_ptr(key_lower, "key_lower"), dev_ptr(flags, "flags"),
                     S(stream));
  });
}

int dgs_compute_frontier_heat(const int64_t *seeds, int64_t n_seeds, const int64_t *indptr,
                              const int64_t *indices, const float *probs,
                              const float *seeds_heat, int64_t num_nodes, int64_t num_picks,
                              int64_t indptr_diff, float *frontier_heat, void *stream) {
  return guard([&] {
    hipStream_t st = S(stream);
    DGS_HIP(hipMemsetAsync(frontier_heat, 0, sizeof(float) * (size_t)num_nodes, st));
    heat(dev_ptr(seeds, "seeds"), n_seeds, dev_ptr(indptr, "indptr"),
         dev_ptr(indices, "indices"), dev_ptr(probs, "probs"), dev_ptr(seeds_heat, "seeds_heat"),
         num_picks, indptr_diff, frontier_heat, num_nodes, nullptr, st);
  });
}

int dgs_compute_frontier_heat_fixed(const int64_t *seeds, int64_t n_seeds,
                                    const int64_t *indptr, const int64_t *indices,
                                    const float *probs, const float *seeds_heat,
                                    int64_t num_nodes, int64_t num_picks, int64_t indptr_diff,
                                    float *frontier_heat, void *stream) {
  return guard([&] {
    hipStream_t st = S(stream);
    // the int64 accumulator lives in the stream's op scratch (stream-asynchronous: calls on one
    // stream are ordered by it, calls on other streams use their own scratch)
    HopScratch *ws = nullptr;
    const OpScratchLease lk = op_scratch(st, &ws);
    ws->op_tmp.ensure(sizeof(uint64_t) * (size_t)(num_nodes > 0 ? num_nodes : 1));
    heat(dev_ptr(seeds, "seeds"), n_seeds, dev_ptr(indptr, "indptr"),
         dev_ptr(indices, "indices"), dev_ptr(probs, "probs"),
         dev_ptr(seeds_heat, "seeds_heat"), num_picks, indptr_diff, frontier_heat, num_nodes,
         ws->op_tmp.as<unsigned long long>(), st);
  });
}

// ------------------------------------------------------------------ TensorP2PServer
int dgs_p2p_server_create(const void *src, int64_t items, int64_t item_bytes,
                          dgs_p2p_server **out) {
  return guard([&] { *out = new dgs_p2p_server{new P2PServer(src, items, item_bytes)}; });
}

int dgs_p2p_server_device_ptr(dgs_p2p_server *s, int64_t rank, void **ptr, int64_t *items) {
  return guard([&] {
    DGS_CHECK(rank >= 0 && rank < obj(s, "p2p server").world(), "rank out of range");
    *ptr = obj(s, "p2p server").ptr((int)rank);
    *items = obj(s, "p2p server").items((int)rank);
  });
}

int dgs_p2p_server_destroy(dgs_p2p_server *s) {
  return guard([&] {
    if (!s) return;
    delete s->s;
    delete s;
  });
}

// ------------------------------------------------------------------ sampler
int dgs_sampler_create(const int64_t *indptr, const int64_t *indices, const float *probs,
                       int64_t num_nodes, int64_t num_edges, const int64_t *cache_nids,
                       int64_t n_cache, int64_t device_id, dgs_sampler **out) {
  return guard([&] {
    *out = new dgs_sampler{
        new Sampler(indptr, indices, probs, num_nodes, num_edges, cache_nids, n_cache, device_id)};
  });
}

int dgs_sampler_bounds(const dgs_sampler *s, int64_t n_seeds, const int64_t *fan_out, int L,
                       int64_t *frontier_cap, int64_t *edge_cap) {
  return guard([&] { obj(s, "sampler").bounds(n_seeds, fan_out, L, frontier_cap, edge_cap); });
}

int dgs_sampler_sample(dgs_sampler *s, const int64_t *seeds, int64_t n_seeds,
                       const int64_t *fan_out, int L, int replace, int64_t *const *frontiers,
                       int64_t *const *rows, int64_t *const *cols, int64_t *sizes_out,
                       void *stream) {
  return guard([&] {
    obj(s, "sampler").sample(dev_ptr(seeds, "seeds"), n_seeds, fan_out, L, replace != 0, frontiers, rows,
                 cols, sizes_out, S(stream));
  });
}

int dgs_sampler_sample_begin(dgs_sampler *s, const int64_t *seeds, int64_t n_seeds,
                             const int64_t *fan_out, int L, int replace,
                             int64_t *const *frontiers, int64_t *const *rows,
                             int64_t *const *cols, const uint64_t *launch_seeds, int flags,
                             void *stream) {
  return guard([&] {
    DGS_CHECK((flags & ~DGS_SAMPLE_HOST_ASYNC) == 0, "sample_begin: unknown flags");
    obj(s, "sampler").sample_begin(dev_ptr(seeds, "seeds"), n_seeds, fan_out, L, replace != 0, frontiers,
                       rows, cols, S(stream), launch_seeds, (flags & DGS_SAMPLE_HOST_ASYNC) != 0);
  });
}

// Per-hop pointers into a packed output buffer (frontier[fcap], rows[ecap], cols[ecap] per hop).
static void packed_ptrs(const Sampler &smp, int64_t n_seeds, const int64_t *fan_out, int L,
                        int64_t *out, int64_t **fr, int64_t **rows, int64_t **cols) {
  int64_t fcap[64], ecap[64];
  smp.bounds(n_seeds, fan_out, L, fcap, ecap);
  int64_t *p = out;
  for (int h = 0; h < L; ++h) {
    fr[h] = p;
    rows[h] = p + fcap[h];
    cols[h] = p + fcap[h] + ecap[h];
    p += fcap[h] + 2 * ecap[h];
  }
}

int dgs_sampler_sample_packed(dgs_sampler *s, const int64_t *seeds, int64_t n_seeds,
                              const int64_t *fan_out, int L, int replace, int64_t *out,
                              int64_t *sizes_out, void *stream) {
  return guard([&] {
    DGS_CHECK(L > 0 && L <= 64, "sample: 1 to 64 hops");
    if (n_seeds > 0) check_device_cached(seeds, "seeds");
    check_device_cached(out, "out");
    int64_t *fr[64], *rows[64], *cols[64];
    packed_ptrs(obj(s, "sampler"), n_seeds, fan_out, L, out, fr, rows, cols);
    obj(s, "sampler").sample(seeds, n_seeds, fan_out, L, replace != 0, fr, rows, cols, sizes_out, S(stream));
  });
}

int dgs_sampler_sample_packed_begin(dgs_sampler *s, const int64_t *seeds, int64_t n_seeds,
                                    const int64_t *fan_out, int L, int replace, int64_t *out,
                                    void *stream) {
  return guard([&] {
    DGS_CHECK(L > 0 && L <= 64, "sample: 1 to 64 hops");
    if (n_seeds > 0) check_device_cached(seeds, "seeds");
    check_device_cached(out, "out");
    int64_t *fr[64], *rows[64], *cols[64];
    packed_ptrs(obj(s, "sampler"), n_seeds, fan_out, L, out, fr, rows, cols);
    // the synchronous call's kernel shapes (solo), launched on the caller's thread
    obj(s, "sampler").sample_begin(seeds, n_seeds, fan_out, L, replace != 0, fr, rows, cols,
                                   S(stream), nullptr, /*host_async=*/false, /*solo=*/true);
  });
}

int dgs_sampler_sample_wait_hop(dgs_sampler *s, int L, int h, int64_t *u_nnz, void *stream) {
  return guard([&] { obj(s, "sampler").sample_wait_hop(L, h, u_nnz, S(stream)); });
}

int dgs_sampler_sample_begin_after(dgs_sampler *s, void *wait_for, const int64_t *seeds,
                                   int64_t n_seeds, const int64_t *fan_out, int L, int replace,
                                   int64_t *out, const uint64_t *launch_seeds, int flags,
                                   void *stream) {
  return guard([&] {
    DGS_CHECK((flags & ~(DGS_SAMPLE_HOST_ASYNC | DGS_SAMPLE_WAIT | DGS_SAMPLE_WAIT_EVENT)) == 0,
              "sample_begin: unknown flags");
    DGS_CHECK(!((flags & DGS_SAMPLE_WAIT) && (flags & DGS_SAMPLE_WAIT_EVENT)),
              "sample_begin: DGS_SAMPLE_WAIT and DGS_SAMPLE_WAIT_EVENT exclude each other");
    DGS_CHECK(!(flags & DGS_SAMPLE_WAIT_EVENT) || wait_for,
              "sample_begin: DGS_SAMPLE_WAIT_EVENT needs an event");
    // a handle without a flag is refused rather than ignored: callers written against the
    // round-3 header (wait when wait_for != NULL) would otherwise silently get no wait
    DGS_CHECK(!wait_for || (flags & (DGS_SAMPLE_WAIT | DGS_SAMPLE_WAIT_EVENT)),
              "sample_begin: wait_for given without DGS_SAMPLE_WAIT or DGS_SAMPLE_WAIT_EVENT");
    DGS_CHECK(L > 0 && L <= 64, "sample_begin: 1 to 64 hops");
    if (n_seeds > 0) check_device_cached(seeds, "seeds");
    check_device_cached(out, "out");
    int64_t *fr[64], *rows[64], *cols[64];
    packed_ptrs(obj(s, "sampler"), n_seeds, fan_out, L, out, fr, rows, cols);
    // DGS_SAMPLE_WAIT, not the handle, says whether to wait: NULL is the null stream (torch's
    // default current stream), a producer like any other.  (Rounds 2-3 tested the handle, so a
    // caller on the default stream got no wait at all -- round 4's root cause of the N = 2
    // corruption: the loader's buffers came from that stream's pool.)
    if (flags & DGS_SAMPLE_WAIT) stream_wait_impl(wait_for, stream);
    // or on an event the caller recorded earlier (where its seeds were complete)
    if (flags & DGS_SAMPLE_WAIT_EVENT)
      DGS_HIP(hipStreamWaitEvent(S(stream), reinterpret_cast<hipEvent_t>(wait_for), 0));
    obj(s, "sampler").sample_begin(seeds, n_seeds, fan_out, L, replace != 0, fr, rows, cols, S(stream),
                       launch_seeds, (flags & DGS_SAMPLE_HOST_ASYNC) != 0);
  });
}

int dgs_sampler_sample_end(dgs_sampler *s, int L, int64_t *sizes_out, void *stream) {
  return guard([&] { obj(s, "sampler").sample_end(L, sizes_out, S(stream)); });
}

int dgs_sampler_context_count(dgs_sampler *s, int64_t *n) {
  return guard([&] { *n = (int64_t)obj(s, "sampler").num_contexts(); });
}

int dgs_sampler_local_cache(const dgs_sampler *s, const int64_t **sub_indptr, int64_t *n_rows,
                            const int64_t **sub_indices, int64_t *n_edges,
                            const float **sub_probs) {
  return guard([&] {
    *sub_indptr = obj(s, "sampler").sub_indptr();
    *n_rows = obj(s, "sampler").n_rows();
    *sub_indices = obj(s, "sampler").sub_indices();
    *n_edges = obj(s, "sampler").n_edges();
    *sub_probs = obj(s, "sampler").sub_probs();
  });
}

int dgs_sampler_cache_hashmap_capacity(const dgs_sampler *s, int64_t *dir_size) {
  return guard([&] { *dir_size = obj(s, "sampler").cache_hashmap_capacity(); });
}

int dgs_sampler_cache_hashmap_fill(const dgs_sampler *s, int id_bytes, void *key, void *idx,
                                   void *devid, void *stream) {
  return guard([&] {
    obj(s, "sampler").cache_hashmap_fill(id_bytes, key, idx, devid, S(stream));
  });
}

int dgs_sampler_cache_map_size(const dgs_sampler *s, int64_t *n) {
  return guard([&] { *n = obj(s, "sampler").cache_map_size(); });
}

int dgs_sampler_cache_map_fill(const dgs_sampler *s, int64_t *key, int64_t *idx,
                               int64_t *devid, void *stream) {
  return guard([&] { obj(s, "sampler").cache_map_fill(key, idx, devid, S(stream)); });
}

int dgs_sampler_destroy(dgs_sampler *s) {
  return guard([&] {
    if (!s) return;
    delete s->s;
    delete s;
  });
}

// ------------------------------------------------------------------ feature server
int dgs_feature_server_create(const void *data, int64_t num_rows, int64_t row_bytes,
                              const int64_t *cache_nids, int64_t n_cache, int64_t device_id,
                              dgs_feature_server **out) {
  return guard([&] {
    *out = new dgs_feature_server{
        new FeatureServer(data, num_rows, row_bytes, cache_nids, n_cache, device_id)};
  });
}

int dgs_feature_server_gather(dgs_feature_server *s, const int64_t *nids, int64_t n, void *out,
                              void *stream) {
  return guard([&] {
    check_async_errors();
    obj(s, "feature server").gather(dev_ptr(nids, "nids"), n, out, S(stream));
  });
}

int dgs_feature_server_local_cache(const dgs_feature_server *s, const void **ptr,
                                   int64_t *rows) {
  return guard([&] {
    *ptr = obj(s, "feature server").local();
    *rows = obj(s, "feature server").local_rows();
  });
}

int dgs_feature_server_layout(const dgs_feature_server *s, int *wshift) {
  return guard([&] { *wshift = obj(s, "feature server").layout(); });
}

int dgs_feature_server_destroy(dgs_feature_server *s) {
  return guard([&] {
    if (!s) return;
    delete s->s;
    delete s;
  });
}

// ------------------------------------------------------------------ profiling
int dgs_profile_enable(int mask) {
  return guard([&] {
    profile_collect();
    // which-index bits: 0 = gather, 1 = sample, 2 = select (dgs_ops.h)
    int m = mask & 7;
    if (mask != 0 && (mask & ~7) != 0) m = 7;
    // DGS_PROF_HUB=1 (diagnostics): the hub kernels' workgroup stamps ride along
    static const bool hub = getenv("DGS_PROF_HUB") != nullptr;
    if (hub && m) m |= 8 | 16;
    profiler().mask = m;
    profiler().on = m != 0;
    if (m & 29) profile_reserve();  // gather, select or hub-kernel stamps
  });
}

int dgs_profile_read(double *gather_ms, int64_t *gather_launches, double *sample_ms,
                     int64_t *sample_calls, double *select_ms, int64_t *select_launches) {
  return guard([&] {
    profile_collect();
    Profiler &p = profiler();
    *gather_ms = p.gather_ms;
    *gather_launches = p.gather_n;
    *sample_ms = p.sample_ms;
    *sample_calls = p.sample_n;
    if (select_ms) *select_ms = p.select_ms;
    if (select_launches) *select_launches = p.select_n;
    p.gather_ms = p.sample_ms = p.select_ms = 0;
    p.gather_n = p.sample_n = p.select_n = 0;
  });
}

}  // extern "C"

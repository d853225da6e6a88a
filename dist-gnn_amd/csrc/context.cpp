// context.cpp -- launch-seed RNG, RCCL communicator, pointer utilities, profiler.
#include "context.h"

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>

#include "dgs_ops.h"

namespace dgs {

RandomEngine &rng() {
  static RandomEngine e;
  return e;
}

// ------------------------------------------------------------------ communicator
#define DGS_NCCL(call)                                                                  \
  do {                                                                                  \
    ncclResult_t r_ = (call);                                                           \
    if (r_ != ncclSuccess)                                                              \
      throw ::dgs::Error(std::string(#call) + " failed: " + ncclGetErrorString(r_));    \
  } while (0)

Comm &Comm::get() {
  static Comm c;
  return c;
}

void Comm::init(int nranks, const void *unique_id, int rank) {
  DGS_CHECK(comm_ == nullptr, "communicator already initialised");
  DGS_CHECK(nranks >= 1 && nranks <= kMaxDevices, "world size must be 1..8 (one node)");
  ncclUniqueId id;
  std::memcpy(&id, unique_id, sizeof(id));
  DGS_NCCL(ncclCommInitRank(&comm_, nranks, id, rank));
  DGS_NCCL(ncclCommUserRank(comm_, &rank_));
  DGS_NCCL(ncclCommCount(comm_, &world_));
  DGS_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  DGS_HIP(hipMalloc(&dbuf_, sizeof(float)));
  DGS_HIP(hipMalloc(&dsizes_, sizeof(int64_t) * (kMaxDevices + 1)));
  // Test switch: the own rank is a peer of the all-gathers like any other (ncclAllGather of the
  // sizes, and a self ncclSend / ncclRecv pair in the payload group), so a one-GPU box runs the
  // grouped send / recv path of NCCLTensorAllGather_ (nccl_context.cc:52-112).
  const char *se = std::getenv("DGS_COMM_SELF_EXCHANGE");
  self_exchange_ = se && se[0] == '1';
}

void Comm::init_host(int nranks, int rank, HostAllgatherFn ag, HostBarrierFn bar, void *ctx) {
  DGS_CHECK(!initialized(), "communicator already initialised");
  DGS_CHECK(nranks >= 1 && nranks <= kMaxDevices && rank >= 0 && rank < nranks,
            "bad host communicator geometry");
  DGS_CHECK(ag && bar, "host communicator needs allgather and barrier callbacks");
  host_ag_ = ag;
  host_bar_ = bar;
  host_ctx_ = ctx;
  world_ = nranks;
  rank_ = rank;
}

void Comm::barrier() {
  if (host_ag_) {
    DGS_CHECK(host_bar_(host_ctx_) == 0, "host barrier failed");
    return;
  }
  if (!comm_) return;
  DGS_NCCL(ncclAllReduce(dbuf_, dbuf_, 1, ncclFloat, ncclSum, comm_, stream_));
  DGS_HIP(hipStreamSynchronize(stream_));
}

std::vector<int64_t> Comm::allgather_sizes(int64_t mine) {
  std::vector<int64_t> out(world_, mine);
  if (world_ == 1 && !(comm_ && self_exchange_)) return out;
  if (host_ag_) {
    DGS_CHECK(host_ag_(&mine, sizeof(int64_t), out.data(), host_ctx_) == 0,
              "host allgather failed");
    return out;
  }
  if (!comm_) return out;
  // device staging (the reference hands a host-registered vector to NCCL,
  // nccl_context.cc:61-77; RCCL gets device buffers here)
  DGS_HIP(hipMemcpyAsync(dsizes_ + kMaxDevices, &mine, sizeof(int64_t), hipMemcpyHostToDevice,
                         stream_));
  DGS_NCCL(ncclAllGather(dsizes_ + kMaxDevices, dsizes_, 1, ncclInt64, comm_, stream_));
  DGS_HIP(hipMemcpyAsync(out.data(), dsizes_, sizeof(int64_t) * world_, hipMemcpyDeviceToHost,
                         stream_));
  DGS_HIP(hipStreamSynchronize(stream_));
  return out;
}

void Comm::check_all(const std::string &err, const char *what) {
  const std::vector<int64_t> bad = allgather_sizes(err.empty() ? 0 : 1);
  std::string ranks;
  for (int r = 0; r < (int)bad.size(); ++r)
    if (bad[r]) ranks += (ranks.empty() ? "" : ", ") + std::to_string(r);
  if (ranks.empty()) return;
  if (bad.size() == 1) throw Error(err);
  throw Error(std::string(what) + " failed on rank(s) " + ranks +
              (err.empty() ? std::string(" (this rank's part succeeded)") : ": " + err));
}

void Comm::allgather_bytes(const void *send, int64_t send_bytes, void *const *recv,
                           const int64_t *recv_bytes, hipStream_t st) {
  const bool self = comm_ && self_exchange_ && !host_ag_;
  if (!self && recv[rank_] != send && send_bytes > 0)
    DGS_HIP(hipMemcpyAsync(recv[rank_], send, send_bytes, hipMemcpyDeviceToDevice, st));
  if (world_ == 1 && !self) return;
  if (host_ag_) {
    int64_t maxb = 1;
    for (int i = 0; i < world_; ++i) maxb = std::max(maxb, recv_bytes[i]);
    std::vector<char> hs(maxb, 0), hr((size_t)maxb * world_, 0);
    DGS_HIP(hipStreamSynchronize(st));
    if (send_bytes > 0) DGS_HIP(hipMemcpy(hs.data(), send, send_bytes, hipMemcpyDefault));
    DGS_CHECK(host_ag_(hs.data(), maxb, hr.data(), host_ctx_) == 0, "host allgather failed");
    for (int i = 0; i < world_; ++i)
      if (i != rank_ && recv_bytes[i] > 0)
        DGS_HIP(hipMemcpy(recv[i], hr.data() + (size_t)maxb * i, recv_bytes[i], hipMemcpyDefault));
    return;
  }
  if (!comm_) return;
  DGS_HIP(hipStreamSynchronize(st));
  // self exchange into a buffer aliasing the payload: received into a temporary first
  void *self_dst = nullptr;
  if (self && send_bytes > 0)
    self_dst = recv[rank_] == send ? nullptr : recv[rank_];
  TmpBuf alias_tmp(self && send_bytes > 0 && !self_dst ? (size_t)send_bytes : 0, stream_);
  if (self && send_bytes > 0 && !self_dst) self_dst = alias_tmp.p;
  DGS_NCCL(ncclGroupStart());
  for (int i = 0; i < world_; ++i) {
    if (i == rank_ && !self) continue;
    DGS_NCCL(ncclSend(send, (size_t)send_bytes, ncclChar, i, comm_, stream_));
    DGS_NCCL(ncclRecv(i == rank_ ? self_dst : recv[i], (size_t)recv_bytes[i], ncclChar, i, comm_,
                      stream_));
  }
  DGS_NCCL(ncclGroupEnd());
  if (self && self_dst == alias_tmp.p && send_bytes > 0)
    DGS_HIP(hipMemcpyAsync(recv[rank_], alias_tmp.p, send_bytes, hipMemcpyDeviceToDevice,
                           stream_));
  DGS_HIP(hipStreamSynchronize(stream_));
}

std::vector<void *> Comm::allgather_device(const void *send, int64_t send_bytes,
                                           std::vector<int64_t> *bytes_out) {
  std::vector<int64_t> sizes = allgather_sizes(send_bytes);
  std::vector<void *> bufs(world_, nullptr);
  for (int i = 0; i < world_; ++i) DGS_HIP(hipMalloc(&bufs[i], sizes[i] > 0 ? sizes[i] : 1));
  allgather_bytes(send, send_bytes, bufs.data(), sizes.data(), stream_);
  DGS_HIP(hipStreamSynchronize(stream_));
  if (bytes_out) *bytes_out = sizes;
  return bufs;
}

// ------------------------------------------------------------------ pointers
bool is_device_pointer(const void *p) {
  if (!p) return false;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged ||
         a.type == hipMemoryTypeUnified;
}

namespace {
// Host ranges this library registered (hipHostRegister), with the number of live references to
// each.  Round 6: only dgs_host_register (_CAPI_tensor_pin_memory) registers caller memory; a
// service over a pinned range holds a reference on it, so unpinning it first does not unmap the
// service's view -- the range is unregistered when the last reference goes.
struct HostReg {
  size_t bytes;
  int refs;
};
std::mutex &host_reg_mu() {
  static std::mutex m;
  return m;
}
std::map<uintptr_t, HostReg> &host_regs() {
  static std::map<uintptr_t, HostReg> m;
  return m;
}
// the registered range holding p (caller holds the lock), or end()
std::map<uintptr_t, HostReg>::iterator host_reg_find(const void *p) {
  auto &m = host_regs();
  const uintptr_t x = (uintptr_t)p;
  auto it = m.upper_bound(x);
  if (it == m.begin()) return m.end();
  --it;
  return x < it->first + it->second.bytes ? it : m.end();
}
// whether a registered range intersects [p, p + n) (caller holds the lock)
bool host_reg_overlaps(uintptr_t p, size_t n) {
  auto &m = host_regs();
  auto it = m.lower_bound(p + n);  // first range starting at or after the end
  if (it == m.begin()) return false;
  --it;                             // the last range starting before the end
  return it->first + it->second.bytes > p;
}
// Pins taken through dgs_host_register, by the pointer the caller passed: an unregister must
// name one of them (it cannot drop a reference a service holds).
std::map<uintptr_t, int> &abi_pins() {
  static std::map<uintptr_t, int> m;
  return m;
}
// The first failed hipHostUnregister since the last check (raised by check_async_errors).  A
// failed unregister leaves HIP's mapping of pages the caller is about to free, and a later
// allocation at the same addresses would be taken for registered memory: it must not pass as a
// stderr line (round 5 printed it, and pytest swallowed it for passing tests).
std::string &host_reg_error() {
  static std::string e;
  return e;
}
void release_locked(const void *p) {
  auto it = host_reg_find(p);
  if (it == host_regs().end()) return;
  if (--it->second.refs == 0) {
    const hipError_t e = hipHostUnregister(reinterpret_cast<void *>(it->first));
    if (e != hipSuccess) {
      (void)hipGetLastError();
      if (host_reg_error().empty()) {
        char buf[160];
        snprintf(buf, sizeof(buf), "hipHostUnregister(%p, %zu bytes) failed: ",
                 reinterpret_cast<void *>(it->first), it->second.bytes);
        host_reg_error() = std::string(buf) + hipGetErrorString(e);
      }
    }
    host_regs().erase(it);
  }
}

std::atomic<int64_t> g_mirror_bytes{0}, g_mirror_count{0};
}  // namespace

void release_host_view(const void *p) {
  std::lock_guard<std::mutex> g(host_reg_mu());
  release_locked(p);
}

void host_pin(void *p, int64_t bytes) {
  DGS_CHECK(p && bytes > 0, "host_register: null pointer or empty range");
  const size_t nb = (size_t)bytes;
  std::lock_guard<std::mutex> g(host_reg_mu());
  auto it = host_reg_find(p);
  if (it != host_regs().end() && (uintptr_t)p + nb <= it->first + it->second.bytes) {
    ++it->second.refs;  // inside a range pinned here already: share it
  } else {
    // A range that only partly lies in a registration cannot be mapped: HIP refuses a second
    // registration of the same pages.
    DGS_CHECK(!host_reg_overlaps((uintptr_t)p, nb),
              "host range overlaps a registration made for a different range of the same "
              "buffer; register (pin) the whole buffer first");
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) == hipSuccess) {
      DGS_CHECK(a.type != hipMemoryTypeHost,
                "host_register: the memory is already pinned outside this library");
      DGS_CHECK(a.type != hipMemoryTypeDevice && a.type != hipMemoryTypeManaged &&
                    a.type != hipMemoryTypeUnified,
                "host_register: device memory");
    } else {
      (void)hipGetLastError();
    }
    // pin_memory.cc:7-12 registers the tensor's own range (cudaHostRegisterDefault); mapped
    // here, so kernels read it through the device pointer
    DGS_HIP(hipHostRegister(p, nb, hipHostRegisterMapped));
    void *d = nullptr;
    const hipError_t e = hipHostGetDevicePointer(&d, p, 0);
    if (e != hipSuccess) {
      (void)hipHostUnregister(p);
      DGS_HIP(e);
    }
    host_regs()[(uintptr_t)p] = HostReg{nb, 1};
  }
  ++abi_pins()[(uintptr_t)p];
}

void host_unpin(void *p) {
  std::lock_guard<std::mutex> g(host_reg_mu());
  auto it = abi_pins().find((uintptr_t)p);
  DGS_CHECK(it != abi_pins().end(),
            "host_unregister: this pointer holds no dgs_host_register pin (pass the pointer "
            "that was registered)");
  if (--it->second == 0) abi_pins().erase(it);
  release_locked(p);
}

void *pinned_view(const void *p, int64_t bytes, bool *pin_ref) {
  if (pin_ref) *pin_ref = false;
  if (!p) return nullptr;
  const size_t nb = (size_t)(bytes > 0 ? bytes : 1);
  {
    std::lock_guard<std::mutex> g(host_reg_mu());
    auto it = host_reg_find(p);
    if (it != host_regs().end() && (uintptr_t)p + nb <= it->first + it->second.bytes) {
      // inside a dgs_host_register pin: read in place, holding a reference on it
      void *d = nullptr;
      DGS_HIP(hipHostGetDevicePointer(&d, reinterpret_cast<void *>(it->first), 0));
      ++it->second.refs;
      if (pin_ref) *pin_ref = true;
      return static_cast<char *>(d) + ((uintptr_t)p - it->first);
    }
    DGS_CHECK(!host_reg_overlaps((uintptr_t)p, nb),
              "host range overlaps a pinned range it does not lie in; pin the whole buffer "
              "first");
  }
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) == hipSuccess) {
    if (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged ||
        a.type == hipMemoryTypeUnified)
      return const_cast<void *>(p);
    if (a.type == hipMemoryTypeHost) {  // pinned by its owner (torch pin_memory, hipHostMalloc)
      void *d = nullptr;
      if (hipHostGetDevicePointer(&d, const_cast<void *>(p), 0) == hipSuccess && d) return d;
      (void)hipGetLastError();
      if (a.devicePointer) return a.devicePointer;
    }
  } else {
    (void)hipGetLastError();
  }
  return nullptr;  // pageable
}

std::vector<HostRegInfo> host_registrations() {
  std::lock_guard<std::mutex> g(host_reg_mu());
  std::vector<HostRegInfo> v;
  for (auto &kv : host_regs()) {
    auto pin = abi_pins().find(kv.first);
    v.push_back(HostRegInfo{kv.first, (int64_t)kv.second.bytes, kv.second.refs,
                            pin == abi_pins().end() ? 0 : pin->second});
  }
  return v;
}

void host_mirror_stats(int64_t *bytes, int64_t *count) {
  *bytes = g_mirror_bytes.load();
  *count = g_mirror_count.load();
}

// ------------------------------------------------------------------ host staging
void host_copy(void *dst, const void *src, size_t bytes) {
  constexpr size_t kPart = size_t(32) << 20;
  if (bytes < 2 * kPart) {
    std::memcpy(dst, src, bytes);
    return;
  }
  // a few threads: one core copies pageable memory at ~10 GB/s, well below the memory system
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const size_t nt = std::min<size_t>({(size_t)16, (size_t)hw, bytes / kPart});
  const size_t per = (bytes / nt + 4095) & ~size_t(4095);
  std::vector<std::thread> th;
  for (size_t t = 1; t < nt; ++t) {
    const size_t lo = t * per;
    if (lo >= bytes) break;
    const size_t n = std::min(per, bytes - lo);
    th.emplace_back([=] { std::memcpy((char *)dst + lo, (const char *)src + lo, n); });
  }
  std::memcpy(dst, src, std::min(per, bytes));
  for (auto &t : th) t.join();
}

namespace {
// Two library-owned pinned staging buffers for uploads of pageable host memory (allocated on
// first use, kept for the process).
constexpr size_t kStageBytes = size_t(128) << 20;
struct Staging {
  std::mutex mu;
  void *buf[2] = {nullptr, nullptr};
  hipEvent_t done[2] = {nullptr, nullptr};
};
Staging &staging() {
  static Staging s;
  return s;
}
}  // namespace

void upload_pageable(void *dst, const void *src, size_t bytes, hipStream_t st) {
  if (bytes == 0) return;
  Staging &S = staging();
  std::lock_guard<std::mutex> g(S.mu);
  for (int i = 0; i < 2; ++i) {
    if (!S.buf[i]) DGS_HIP(hipHostMalloc(&S.buf[i], kStageBytes, hipHostMallocDefault));
    if (!S.done[i]) DGS_HIP(hipEventCreateWithFlags(&S.done[i], hipEventDisableTiming));
  }
  // chunk c: wait until the DMA that last read staging buffer c & 1 is done (this call's, or an
  // earlier call's that ended in an error before its closing synchronisation), fill it on the
  // host, enqueue its copy (the host fills the other buffer while the DMA runs)
  for (size_t off = 0, c = 0; off < bytes; off += kStageBytes, ++c) {
    const int b = (int)(c & 1);
    const size_t n = std::min(kStageBytes, bytes - off);
    DGS_HIP(hipEventSynchronize(S.done[b]));  // (an event never recorded is complete)
    host_copy(S.buf[b], (const char *)src + off, n);
    DGS_HIP(hipMemcpyAsync((char *)dst + off, S.buf[b], n, hipMemcpyHostToDevice, st));
    DGS_HIP(hipEventRecord(S.done[b], st));
  }
  DGS_HIP(hipStreamSynchronize(st));
}

void *mirror_alloc(size_t bytes) {
  void *h = nullptr;
  DGS_HIP(hipHostMalloc(&h, bytes ? bytes : 1, hipHostMallocMapped));
  g_mirror_bytes += (int64_t)bytes;
  g_mirror_count += 1;
  return h;
}

void mirror_free(void *h, size_t bytes) {
  if (!h) return;
  (void)hipHostFree(h);
  g_mirror_bytes -= (int64_t)bytes;
  g_mirror_count -= 1;
}

// ------------------------------------------------------------------ async errors
namespace {
struct AsyncErrWords {
  int64_t *host = nullptr, *dev = nullptr;
  std::atomic<uint64_t> tag{0};
};
AsyncErrWords &async_err() {
  static AsyncErrWords w;
  static std::once_flag once;
  std::call_once(once, [] {
    void *h = nullptr;
    // portable: visible to every device of the process; coherent: a kernel's system-scope
    // store is seen by the host without a synchronisation
    DGS_HIP(hipHostMalloc(&h, sizeof(int64_t) * kAsyncErrWords,
                          hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable));
    std::memset(h, 0, sizeof(int64_t) * kAsyncErrWords);
    void *d = nullptr;
    DGS_HIP(hipHostGetDevicePointer(&d, h, 0));
    w.host = static_cast<int64_t *>(h);
    w.dev = static_cast<int64_t *>(d);
  });
  return w;
}
}  // namespace

int64_t *async_err_dev() { return async_err().dev; }

namespace {
thread_local uint64_t t_last_tag = 0;
}
uint64_t async_err_next_tag() {
  t_last_tag = async_err().tag.fetch_add(1) + 1;
  return t_last_tag;
}
uint64_t async_err_last_tag() { return t_last_tag; }

void check_async_errors() {
  {
    std::lock_guard<std::mutex> g(host_reg_mu());
    if (!host_reg_error().empty()) {
      const std::string e = host_reg_error();
      host_reg_error().clear();
      throw Error("host memory: " + e + " (a registration of this library outlived its "
                  "release; its pages stay mapped)");
    }
  }
  AsyncErrWords &w = async_err();
  const int64_t kind = __atomic_load_n(&w.host[0], __ATOMIC_ACQUIRE);
  if (kind == 0) return;
  const int64_t id = w.host[1], rows = w.host[2], tag = w.host[3];
  __atomic_store_n(&w.host[0], 0, __ATOMIC_RELEASE);
  const char *what = kind == kAsyncErrFeature ? "feature gather (nids)"
                     : kind == kAsyncErrLabel ? "label gather (seeds)"
                                              : "index_select (nid)";
  throw Error("an earlier " + std::string(what) + " call read id " + std::to_string(id) +
              ", outside [0, " + std::to_string(rows) + "); its rows were filled from row 0 " +
              "(gather call #" + std::to_string(tag) + " of this process; the reference reads " +
              "out of bounds here)");
}

// ------------------------------------------------------------------ profiler
// Thread-safe: sampling contexts on several streams may record spans concurrently.
namespace {
struct EvPair {
  hipEvent_t a, b;
  int which;
  hipStream_t st;  // span end matches the open span of the same stream
};
std::mutex &prof_mu() {
  static std::mutex m;
  return m;
}
std::vector<EvPair> &pending() {
  static std::vector<EvPair> v;
  return v;
}
std::vector<hipEvent_t> &pool() {
  static std::vector<hipEvent_t> v;
  return v;
}
hipEvent_t take_event() {
  auto &p = pool();
  if (!p.empty()) {
    hipEvent_t e = p.back();
    p.pop_back();
    return e;
  }
  hipEvent_t e;
  DGS_HIP(hipEventCreate(&e));
  return e;
}

struct StampRec {
  uint64_t *buf;
  int64_t nblocks;
  int which;
  bool own;  // a separate allocation (slab full), returned to the pool at collect
  int extra;  // words per workgroup after the 2 x nblocks stamps (kernel-defined counters)
};
// Workgroup stamps are bump-allocated from one slab reserved when profiling is switched on,
// so a profiled launch inside a timed region never calls hipMalloc.  1 GiB holds 2 x 8 B for
// 64 M workgroups (one-wave gather workgroups: B = 1024 ~5000 gathers, B = 8192 ~2100) before
// falling back.
constexpr int64_t kStampSlabWords = int64_t(128) << 20;
struct StampSlab {
  uint64_t *base = nullptr;
  int64_t used = 0;
};
StampSlab &stamp_slab() {
  static StampSlab s;
  return s;
}
std::vector<StampRec> &stamp_recs() {
  static std::vector<StampRec> v;
  return v;
}
std::vector<std::pair<int64_t, uint64_t *>> &stamp_pool() {
  static std::vector<std::pair<int64_t, uint64_t *>> v;
  return v;
}
void add_measure(int which, double ms) {
  if (which == 0) {
    profiler().gather_ms += ms;
    profiler().gather_n += 1;
  } else if (which == 2) {
    profiler().select_ms += ms;
    profiler().select_n += 1;
  } else if (which >= 3) {
    // hub-kernel stamps: diagnostics only (printed by the detail report)
  } else {
    profiler().sample_ms += ms;
    profiler().sample_n += 1;
  }
}
}  // namespace

Profiler &profiler() {
  static Profiler p;
  return p;
}

KernelEvents profile_kernel(int which) {
  KernelEvents ev;
  if (!profiler().wants(which)) return ev;
  std::lock_guard<std::mutex> g(prof_mu());
  ev.start = take_event();
  ev.stop = take_event();
  pending().push_back(EvPair{ev.start, ev.stop, which, nullptr});
  return ev;
}

uint64_t *profile_stamps(int which, int64_t nblocks, int extra) {
  if (!profiler().wants(which) || nblocks <= 0) return nullptr;
  std::lock_guard<std::mutex> g(prof_mu());
  uint64_t *buf = nullptr;
  const int64_t words = (2 + extra) * nblocks;
  StampSlab &slab = stamp_slab();
  if (slab.base && slab.used + words <= kStampSlabWords) {
    buf = slab.base + slab.used;
    slab.used += words;
    stamp_recs().push_back(StampRec{buf, nblocks, which, false, extra});
    return buf;
  }
  auto &pool = stamp_pool();  // (capacity in words, buffer)
  for (auto it = pool.begin(); it != pool.end(); ++it) {
    if (it->first >= words) {
      buf = it->second;
      pool.erase(it);
      break;
    }
  }
  if (!buf) DGS_HIP(hipMalloc(reinterpret_cast<void **>(&buf), sizeof(uint64_t) * words));
  stamp_recs().push_back(StampRec{buf, nblocks, which, true, extra});
  return buf;
}

void profile_begin(hipStream_t st, int which) {
  if (!profiler().wants(which)) return;
  std::lock_guard<std::mutex> g(prof_mu());
  EvPair ev{take_event(), nullptr, which, st};
  DGS_HIP(hipEventRecord(ev.a, st));
  pending().push_back(ev);
}

void profile_end(hipStream_t st, int which) {
  if (!profiler().wants(which)) return;
  std::lock_guard<std::mutex> g(prof_mu());
  auto &pv = pending();
  for (auto it = pv.rbegin(); it != pv.rend(); ++it) {
    if (it->which == which && it->b == nullptr && it->st == st) {
      it->b = take_event();
      DGS_HIP(hipEventRecord(it->b, st));
      return;
    }
  }
}

void profile_reserve() {
  std::lock_guard<std::mutex> g(prof_mu());
  StampSlab &slab = stamp_slab();
  if (!slab.base)
    DGS_HIP(hipMalloc(reinterpret_cast<void **>(&slab.base), sizeof(uint64_t) * kStampSlabWords));
}

void profile_collect() {
  std::lock_guard<std::mutex> g(prof_mu());
  auto &sr = stamp_recs();
  if (!sr.empty()) {
    DGS_HIP(hipDeviceSynchronize());
    int dev = 0, khz = 0;
    DGS_HIP(hipGetDevice(&dev));
    DGS_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
    std::vector<uint64_t> h;
    // DGS_PROF_DETAIL=1: per measurement, how a launch's span splits into the dispatch spread
    // (first to last workgroup start) and the workgroups' own durations (stderr, diagnostics)
    static const bool detail = getenv("DGS_PROF_DETAIL") != nullptr;
    // For the hub kernels (which 3 / 4, whose workgroups each own a fixed share of the work)
    // also the end spread (first to last workgroup end) and the busy fraction (workgroup time
    // over workgroups x span): a low fraction is time lost to late starts and uneven finishes.
    constexpr int kW = 5;
    double d_span[kW] = {}, d_spread[kW] = {}, d_wg[kW] = {}, d_end[kW] = {}, d_busy[kW] = {};
    int64_t d_n[kW] = {};
    // k_bias_stream's per-workgroup counters (extra == 2: candidate flushes, candidates | row
    // switches << 32): workgroup duration against each, in buckets (the end-spread question)
    constexpr int kB = 6;
    double c_dur[3][kB] = {}, c_n[3][kB] = {};
    auto bucket = [](uint64_t v) { return v < 4 ? (int)v : (v < 8 ? 4 : 5); };
    double cu_dur[7] = {}, cu_n[7] = {}, cu_count = 0, cu_launch = 0;
    for (auto &r : sr) {
      h.resize((size_t)((2 + r.extra) * r.nblocks));
      DGS_HIP(hipMemcpy(h.data(), r.buf, sizeof(uint64_t) * h.size(), hipMemcpyDeviceToHost));
      uint64_t t0 = ~0ull, t1 = 0, s1 = 0, e0 = ~0ull;
      double wg = 0;
      for (int64_t b = 0; b < r.nblocks; ++b) {
        t0 = h[2 * b] < t0 ? h[2 * b] : t0;
        t1 = h[2 * b + 1] > t1 ? h[2 * b + 1] : t1;
        s1 = h[2 * b] > s1 ? h[2 * b] : s1;
        e0 = h[2 * b + 1] < e0 ? h[2 * b + 1] : e0;
        wg += (double)(h[2 * b + 1] - h[2 * b]);
      }
      if (t1 > t0 && khz > 0) {
        add_measure(r.which, (double)(t1 - t0) / (double)khz);
        if (detail && r.which >= 0 && r.which < kW) {
          d_span[r.which] += (double)(t1 - t0) / khz;
          d_spread[r.which] += (double)(s1 - t0) / khz;
          d_wg[r.which] += wg / (double)r.nblocks / khz;
          d_end[r.which] += (double)(t1 - e0) / khz;
          d_busy[r.which] += wg / ((double)r.nblocks * (double)(t1 - t0));
          d_n[r.which] += 1;
        }
      }
      // (launches whose workgroups average over 10 us: the ones with work for every worker)
      if (detail && r.extra == 2 && khz > 0 && wg / (double)r.nblocks > khz / 100.0) {
        // the launch's mean workgroup duration, so buckets compare within launches
        const double mean = wg / (double)r.nblocks;
        // workgroups of this launch per CU (the upper word of the first counter: CU id)
        std::map<uint64_t, int> per_cu;
        for (int64_t b = 0; b < r.nblocks; ++b) per_cu[h[2 * r.nblocks + 2 * b] >> 32] += 1;
        for (int64_t b = 0; b < r.nblocks; ++b) {
          const int share = per_cu[h[2 * r.nblocks + 2 * b] >> 32];
          const int sb = share < 6 ? share : 6;
          cu_dur[sb] += (double)(h[2 * b + 1] - h[2 * b]) / mean;
          cu_n[sb] += 1;
        }
        cu_count += (double)per_cu.size();
        cu_launch += 1;
        for (int64_t b = 0; b < r.nblocks; ++b) {
          const double dur = (double)(h[2 * b + 1] - h[2 * b]) / mean;
          const uint64_t fl = h[2 * r.nblocks + 2 * b] & 0xffffffffu;
          const uint64_t cr = h[2 * r.nblocks + 2 * b + 1];
          const uint64_t v[3] = {fl, (cr & 0xffffffffu) / 64, cr >> 32};
          for (int j = 0; j < 3; ++j) {
            c_dur[j][bucket(v[j])] += dur;
            c_n[j][bucket(v[j])] += 1;
          }
        }
      }
      if (r.own) stamp_pool().push_back({(2 + r.extra) * r.nblocks, r.buf});
    }
    if (detail && cu_launch > 0) {
      fprintf(stderr, "[dgs prof] k_bias_stream: %.1f CUs per launch; workgroups by launch "
              "workgroups on their CU (1..5, 6+): duration / launch mean", cu_count / cu_launch);
      for (int sb = 1; sb < 7; ++sb)
        fprintf(stderr, " %.3f (n %.0f)", cu_n[sb] ? cu_dur[sb] / cu_n[sb] : 0.0, cu_n[sb]);
      fprintf(stderr, "\n");
    }
    static const char *cname[3] = {"candidate flushes", "candidates / 64", "row switches"};
    for (int j = 0; detail && j < 3; ++j) {
      if (c_n[j][0] + c_n[j][1] + c_n[j][2] + c_n[j][3] + c_n[j][4] + c_n[j][5] == 0) continue;
      fprintf(stderr, "[dgs prof] k_bias_stream workgroups by %s (0,1,2,3,4-7,8+): "
              "duration / launch mean", cname[j]);
      for (int bk = 0; bk < kB; ++bk)
        fprintf(stderr, " %.3f (n %.0f)", c_n[j][bk] ? c_dur[j][bk] / c_n[j][bk] : 0.0,
                c_n[j][bk]);
      fprintf(stderr, "\n");
    }
    for (int w = 0; detail && w < kW; ++w)
      if (d_n[w])
        fprintf(stderr,
                "[dgs prof] which=%d launches=%lld avg span %.2f us, dispatch spread %.2f us, "
                "workgroup duration %.2f us, end spread %.2f us, busy %.3f\n",
                w, (long long)d_n[w], 1e3 * d_span[w] / d_n[w], 1e3 * d_spread[w] / d_n[w],
                1e3 * d_wg[w] / d_n[w], 1e3 * d_end[w] / d_n[w], d_busy[w] / d_n[w]);
    sr.clear();
    stamp_slab().used = 0;
  }
  auto &pv = pending();
  for (auto &ev : pv) {
    if (!ev.b) continue;
    DGS_HIP(hipEventSynchronize(ev.b));
    float ms = 0;
    // a span with no launch leaves its events unrecorded: nothing to count
    if (hipEventElapsedTime(&ms, ev.a, ev.b) != hipSuccess) {
      (void)hipGetLastError();
      pool().push_back(ev.a);
      pool().push_back(ev.b);
      continue;
    }
    add_measure(ev.which, ms);
    pool().push_back(ev.a);
    pool().push_back(ev.b);
  }
  pv.clear();
}

}  // namespace dgs

// context.h -- process-global context: launch-seed RNG, RCCL communicator, host-memory
// registration and the kernel profiler.
//
// Reference: src/context/context.{h,cc} (RandomEngine, randn_uint64),
// src/nccl/nccl_context.{h,cc} (NCCLContext singleton), src/common/pin_memory.cc.
#pragma once

#include <rccl/rccl.h>

#include <mutex>
#include <random>
#include <vector>

#include "dgs_common.h"

namespace dgs {

// std::mt19937_64 + full-range uniform_int_distribution == raw engine output (libstdc++),
// seeded from std::random_device like the reference; set_seed() makes runs reproducible.
class RandomEngine {
 public:
  RandomEngine() : gen_(std::random_device()()) {}
  uint64_t next() {
    std::lock_guard<std::mutex> g(mu_);
    return dis_(gen_);
  }
  // n consecutive draws under one lock (a multi-hop call's seeds stay contiguous)
  void next_n(int64_t n, uint64_t *out) {
    std::lock_guard<std::mutex> g(mu_);
    for (int64_t i = 0; i < n; ++i) out[i] = dis_(gen_);
  }
  void set_seed(uint64_t s) {
    std::lock_guard<std::mutex> g(mu_);
    gen_.seed(s);
    dis_.reset();
  }

 private:
  std::mutex mu_;
  std::mt19937_64 gen_;
  std::uniform_int_distribution<uint64_t> dis_{0, 0xFFFFFFFFFFFFFFFFULL};
};
RandomEngine &rng();

// RCCL communicator for the setup collectives (no collective runs in the sampling /
// gather hot loop: remote rows are read one-sided through IPC-mapped peer memory).
// Host transport for the setup collectives (tests, or ranks that share one device):
// allgather(send[bytes] -> recv[world * bytes]) and barrier, both host memory.
typedef int (*HostAllgatherFn)(const void *send, int64_t bytes, void *recv, void *ctx);
typedef int (*HostBarrierFn)(void *ctx);

class Comm {
 public:
  static Comm &get();
  void init(int nranks, const void *unique_id, int rank);
  void init_host(int nranks, int rank, HostAllgatherFn ag, HostBarrierFn bar, void *ctx);
  bool initialized() const { return comm_ != nullptr || host_ag_ != nullptr; }
  bool host_mode() const { return host_ag_ != nullptr; }
  int rank() const { return rank_; }
  int world() const { return world_; }
  void barrier();
  std::vector<int64_t> allgather_sizes(int64_t mine);
  // A setup step's local outcome made collective: `err` is this rank's error ("" = ok).  Every
  // rank takes part; if any rank failed, every rank throws naming the failed ranks (and its own
  // error), so no rank is left waiting in the next collective for one that has left.
  void check_all(const std::string &err, const char *what);
  // grouped ncclSend/ncclRecv of byte payloads (recv[rank_] may alias send)
  void allgather_bytes(const void *send, int64_t send_bytes, void *const *recv,
                       const int64_t *recv_bytes, hipStream_t st);
  // convenience: all-gather a device byte buffer into freshly allocated device buffers
  std::vector<void *> allgather_device(const void *send, int64_t send_bytes,
                                       std::vector<int64_t> *bytes_out);

 private:
  ncclComm_t comm_ = nullptr;
  HostAllgatherFn host_ag_ = nullptr;
  HostBarrierFn host_bar_ = nullptr;
  void *host_ctx_ = nullptr;
  int rank_ = 0, world_ = 1;
  hipStream_t stream_ = nullptr;
  float *dbuf_ = nullptr;
  int64_t *dsizes_ = nullptr;
  bool self_exchange_ = false;  // DGS_COMM_SELF_EXCHANGE=1 at init (tests)
};

// Host memory.  Round 6: the library never registers pageable caller memory for a service
// (DESIGN.md section 3).  What a service reads from the host is either pinned by its owner
// (read in place) or a library-owned copy (a device temporary for the cache build, or a pinned
// mirror for rows that stay on the host); only dgs_host_register registers caller memory.
//
// Device-accessible pointer for `p` when it needs no copy: device memory, host memory pinned by
// its owner, or a range inside a dgs_host_register pin (then *pin_ref = true: the caller holds
// a reference, released with release_host_view(p)).  nullptr for pageable memory.  A range
// that partly overlaps a pin is refused (Error).
void *pinned_view(const void *p, int64_t bytes, bool *pin_ref);
void release_host_view(const void *p);
// dgs_host_register / dgs_host_unregister: a reference on the registration plus a pin keyed by
// `p`; unpinning a pointer that holds no pin is an error.
void host_pin(void *p, int64_t bytes);
void host_unpin(void *p);
struct HostRegInfo {
  uintptr_t base;
  int64_t bytes;
  int refs;  // pins + service views
  int pins;  // dgs_host_register pins keyed by base
};
std::vector<HostRegInfo> host_registrations();
// Library-owned copies of host arrays: a multi-threaded memcpy; an upload of pageable memory to
// device memory through two library-owned pinned staging buffers (HIP's own pageable-copy path
// is not used for the caller's arrays); pinned, mapped mirrors (hipHostMalloc) counted for
// diagnostics (dgs_host_memory_state).
void host_copy(void *dst, const void *src, size_t bytes);
void upload_pageable(void *dst, const void *src, size_t bytes, hipStream_t st);
void *mirror_alloc(size_t bytes);
void mirror_free(void *h, size_t bytes);
void host_mirror_stats(int64_t *bytes, int64_t *count);
bool is_device_pointer(const void *p);

// Out-of-range ids met by the gather kernels (feature server, index_select, the loader's fused
// label rows; the reference reads out of bounds there, feature_ops.cu:38-73,140-171).  The
// kernel reads row 0 in place of the bad row and stores {kind, id, num_rows, tag} into these
// coherent pinned host words with system-scope vector stores; no launch or synchronisation is
// added.  The next gather entry point on the host (or dgs_check_async_errors) raises and clears
// them.  kind: kAsyncErrFeature / kAsyncErrLabel / kAsyncErrSelect.
constexpr int64_t kAsyncErrFeature = 1, kAsyncErrLabel = 2, kAsyncErrSelect = 3;
constexpr int kAsyncErrWords = 4;
int64_t *async_err_dev();  // device-visible address of the words (allocated on first use)
uint64_t async_err_next_tag();  // per-process call counter (the tag a launch reports)
uint64_t async_err_last_tag();  // the tag of this thread's last gather launch (0: none)
// throws (and clears) when a kernel stored an error, or when a pin's hipHostUnregister failed
void check_async_errors();

}  // namespace dgs

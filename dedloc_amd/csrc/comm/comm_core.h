// Torch-free core of the RCCL data plane: the communicator registry and its lifecycle rules
// (SURVEY.md §5.8 failure handling, §5.2 race safety).  csrc/comm/rccl_comm.cpp is the thin
// torch.library adapter over it; tests/native/rccl_core_test.cpp builds this same code against a
// stub rccl.h under AddressSanitizer / UBSan / ThreadSanitizer.
//
// Lifecycle rules:
//   * a handle is a small integer into the registry, never a raw pointer: a stale handle is a
//     clean error;
//   * every RCCL call on one communicator happens under that communicator's own mutex, and the
//     ncclComm_t is cleared under it when the communicator is aborted, so a status poll racing an
//     abort on another thread sees "aborted", never freed memory;
//   * release() never aborts a communicator whose non-blocking bootstrap is still in flight
//     (ncclInProgress before status() has ever reported ncclSuccess: RCCL's init thread still owns
//     it).  Such a communicator is QUARANTINED: it stays in the registry (unusable for transfers),
//     reap() polls it, and it is aborted only once RCCL reports that the bootstrap ended (success
//     or error).  A bootstrap whose other members never arrive stays quarantined until process
//     exit — a few idle sockets, instead of freeing state RCCL's background thread may still touch;
//   * once the bootstrap has completed (``bootstrapped``), ncclInProgress only means a grouped
//     send/recv is still being enqueued (e.g. lazy p2p connection set-up towards a member that
//     died): release() then aborts at once — NCCL allows aborting a non-blocking communicator with
//     operations in progress, and that abort is what cancels the round's kernels, sockets and
//     proxy threads.
#pragma once

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace dlcomm {

struct P2POp {
  void* ptr;
  size_t count;
  ncclDataType_t dtype;
  int peer;
  bool send;
};

struct Comm {
  std::mutex mu;              // serialises every RCCL call on this communicator
  ncclComm_t comm = nullptr;  // nullptr once aborted
  int64_t nranks = 0, rank = 0, device = 0;
  bool quarantined = false;   // guarded by mu
  bool bootstrapped = false;  // guarded by mu: status() has reported ncclSuccess at least once
};

// release() outcomes
constexpr int64_t kAborted = 0;
constexpr int64_t kQuarantined = 1;
constexpr int64_t kUnknownHandle = 2;

class Registry {
 public:
  // ncclCommInitRankConfig (blocking = 0) on `device`; returns the handle, or -1 with *err set.
  int64_t init(const ncclUniqueId& id, int nranks, int rank, int device, std::string* err);
  // ncclCommGetAsyncError: ncclSuccess (0) ready, ncclInProgress (7) busy, else the error.  An
  // unknown or aborted handle reports ncclInvalidArgument.
  int64_t status(int64_t h);
  // ncclGroupStart; all receives then all sends; ncclGroupEnd on `stream`.  Returns the first
  // error or ncclGroupEnd's result (ncclInProgress: poll status()).  A quarantined or aborted
  // communicator reports ncclInvalidUsage and posts nothing.
  int64_t group_p2p(int64_t h, const std::vector<P2POp>& ops, hipStream_t stream);
  // The failure / end-of-life path: abort now (kAborted) unless the bootstrap is still in flight,
  // in which case the communicator is quarantined (kQuarantined) and reap() aborts it later.
  int64_t release(int64_t h);
  // Abort every quarantined communicator whose bootstrap has ended; returns how many remain.
  int64_t reap();
  int64_t live();         // registered, not quarantined
  int64_t quarantined();  // waiting for their bootstrap to end
  bool device_of(int64_t h, int64_t* device, int64_t* nranks);

 private:
  std::shared_ptr<Comm> find(int64_t h);
  void abort_locked(Comm& c);  // c.mu held

  std::mutex mu_;  // guards the map only; never held across an RCCL call
  std::unordered_map<int64_t, std::shared_ptr<Comm>> comms_;
  int64_t next_ = 1;
};

Registry& registry();

}  // namespace dlcomm

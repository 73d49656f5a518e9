// Torch-free core of the RCCL data plane (see comm_core.h for the lifecycle rules).
#include "comm_core.h"

#include <cstring>

namespace dlcomm {

namespace {

struct DeviceGuard {
  int prev = -1;
  bool ok = false;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

}  // namespace

Registry& registry() {
  static Registry* r = new Registry();  // never destroyed: RCCL threads may outlive static teardown
  return *r;
}

std::shared_ptr<Comm> Registry::find(int64_t h) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = comms_.find(h);
  return it == comms_.end() ? nullptr : it->second;
}

int64_t Registry::init(const ncclUniqueId& id, int nranks, int rank, int device, std::string* err) {
  if (nranks < 1 || rank < 0 || rank >= nranks) {
    if (err) *err = "bad rank " + std::to_string(rank) + " of " + std::to_string(nranks);
    return -1;
  }
  DeviceGuard g(device);
  if (!g.ok) {
    if (err) *err = "hipSetDevice(" + std::to_string(device) + ") failed";
    return -1;
  }
  auto c = std::make_shared<Comm>();
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclResult_t rc = ncclCommInitRankConfig(&c->comm, nranks, id, rank, &cfg);
  if (rc != ncclSuccess && rc != ncclInProgress) {
    if (err) *err = std::string("ncclCommInitRankConfig failed: ") + ncclGetErrorString(rc);
    if (c->comm != nullptr) {
      // the init failed synchronously; the communicator may still be half built by RCCL's init
      // thread: keep it quarantined like any in-flight bootstrap rather than aborting it here
      std::lock_guard<std::mutex> lk(mu_);
      c->quarantined = true;
      comms_[next_++] = c;
    }
    return -1;
  }
  std::lock_guard<std::mutex> lk(mu_);
  const int64_t h = next_++;
  comms_[h] = c;
  return h;
}

int64_t Registry::status(int64_t h) {
  auto c = find(h);
  if (!c) return (int64_t)ncclInvalidArgument;
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->comm == nullptr) return (int64_t)ncclInvalidArgument;
  ncclResult_t st = ncclSuccess;
  ncclResult_t rc = ncclCommGetAsyncError(c->comm, &st);
  if (rc == ncclSuccess && st == ncclSuccess) c->bootstrapped = true;
  return rc != ncclSuccess ? (int64_t)rc : (int64_t)st;
}

int64_t Registry::group_p2p(int64_t h, const std::vector<P2POp>& ops, hipStream_t stream) {
  auto c = find(h);
  if (!c) return (int64_t)ncclInvalidArgument;
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->comm == nullptr || c->quarantined) return (int64_t)ncclInvalidUsage;
  for (const auto& op : ops)
    if (op.peer < 0 || op.peer >= c->nranks) return (int64_t)ncclInvalidArgument;
  DeviceGuard g((int)c->device);
  if (!g.ok) return (int64_t)ncclUnhandledCudaError;
  ncclResult_t rc = ncclGroupStart();
  if (rc != ncclSuccess) return (int64_t)rc;
  ncclResult_t first = ncclSuccess;
  // receives first: with all-pairs traffic every rank posts its receives before its sends
  for (int pass = 0; pass < 2; ++pass) {
    for (const auto& op : ops) {
      if (op.send != (pass == 1) || op.count == 0) continue;
      rc = op.send ? ncclSend(op.ptr, op.count, op.dtype, op.peer, c->comm, stream)
                   : ncclRecv(op.ptr, op.count, op.dtype, op.peer, c->comm, stream);
      if (rc != ncclSuccess && rc != ncclInProgress && first == ncclSuccess) first = rc;
    }
  }
  rc = ncclGroupEnd();
  if (first != ncclSuccess) return (int64_t)first;
  return (int64_t)rc;
}

void Registry::abort_locked(Comm& c) {
  if (c.comm == nullptr) return;
  DeviceGuard g((int)c.device);
  (void)ncclCommAbort(c.comm);
  c.comm = nullptr;
}

int64_t Registry::release(int64_t h) {
  auto c = find(h);
  if (!c) return kUnknownHandle;
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->comm != nullptr) {
    ncclResult_t st = ncclSuccess;
    ncclResult_t rc = ncclCommGetAsyncError(c->comm, &st);
    if (rc == ncclSuccess && st == ncclInProgress && !c->bootstrapped) {
      c->quarantined = true;
      return kQuarantined;
    }
  }
  {
    std::lock_guard<std::mutex> lk2(mu_);
    auto it = comms_.find(h);
    if (it != comms_.end() && it->second == c) comms_.erase(it);
  }
  abort_locked(*c);
  return kAborted;
}

int64_t Registry::reap() {
  std::vector<std::pair<int64_t, std::shared_ptr<Comm>>> waiting;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& kv : comms_) waiting.emplace_back(kv.first, kv.second);
  }
  int64_t left = 0;
  for (auto& kv : waiting) {
    Comm& c = *kv.second;
    std::lock_guard<std::mutex> lk(c.mu);
    if (!c.quarantined) continue;
    if (c.comm != nullptr) {
      ncclResult_t st = ncclSuccess;
      ncclResult_t rc = ncclCommGetAsyncError(c.comm, &st);
      if (rc == ncclSuccess && st == ncclInProgress) {
        ++left;
        continue;
      }
    }
    {
      std::lock_guard<std::mutex> lk2(mu_);
      auto it = comms_.find(kv.first);
      if (it != comms_.end() && it->second == kv.second) comms_.erase(it);
    }
    abort_locked(c);
  }
  return left;
}

int64_t Registry::live() {
  std::vector<std::shared_ptr<Comm>> all;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& kv : comms_) all.push_back(kv.second);
  }
  int64_t n = 0;
  for (auto& c : all) {
    std::lock_guard<std::mutex> lk(c->mu);
    n += !c->quarantined;
  }
  return n;
}

int64_t Registry::quarantined() {
  std::vector<std::shared_ptr<Comm>> all;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& kv : comms_) all.push_back(kv.second);
  }
  int64_t n = 0;
  for (auto& c : all) {
    std::lock_guard<std::mutex> lk(c->mu);
    n += c->quarantined;
  }
  return n;
}

bool Registry::device_of(int64_t h, int64_t* device, int64_t* nranks) {
  auto c = find(h);
  if (!c) return false;
  *device = c->device;
  *nranks = c->nranks;
  return true;
}

}  // namespace dlcomm

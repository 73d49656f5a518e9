// Native RCCL data plane for open-membership collaborations.
//
// A collaboration has no fixed world: peers come and go, and every matchmade group (any subset of
// the GPU peers on the node, plus newcomers that were never part of any launch) averages over its
// own communicator.  This file owns those communicators:
//
//   unique_id()                      ncclGetUniqueId; the group's leader publishes the 128 bytes
//                                    through the control-plane DHT (parallel/comm.py)
//   comm_init(uid, n, rank, dev)     ncclCommInitRankConfig with blocking = 0: returns at once, the
//                                    bootstrap runs in RCCL's background thread
//   comm_status(h)                   ncclCommGetAsyncError: 0 ready, 7 (ncclInProgress) still
//                                    connecting, anything else failed
//   group_p2p(h, sends, peers, ...)  ncclGroupStart; one ncclSend / ncclRecv per (tensor, peer);
//                                    ncclGroupEnd on the CURRENT HIP stream: the butterfly's
//                                    all-pairs reduce-scatter and gather-back, and peer state
//                                    transfer.  Non-blocking: the host polls completion against its
//                                    own deadline (Python), so a dead member never hangs a peer
//   comm_abort(h)                    ncclCommAbort: cancels posted operations (a stalled round's
//                                    sends can never be matched by a later round) and frees the
//                                    communicator
//
// Handles are small integers into a registry (never raw pointers): a stale handle after an abort
// is a clean error, not a use-after-free.  The library is resolved against the librccl.so.1 that
// torch itself loaded (same soname, torch's lib dir first on the link line), so one RCCL instance
// serves torch and us.
#include <torch/extension.h>
#include <torch/library.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cstring>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace {

struct Comm {
  ncclComm_t comm = nullptr;
  int64_t nranks = 0, rank = 0, device = 0;
};

std::mutex g_mu;
std::unordered_map<int64_t, std::shared_ptr<Comm>> g_comms;
std::atomic<int64_t> g_next{1};

std::shared_ptr<Comm> lookup(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_comms.find(h);
  TORCH_CHECK(it != g_comms.end(), "dedloc_comm: unknown or aborted communicator handle ", h);
  return it->second;
}

ncclDataType_t nccl_dtype(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kHalf: return ncclFloat16;
    case at::kBFloat16: return ncclBfloat16;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kDouble: return ncclFloat64;
    default: TORCH_CHECK(false, "dedloc_comm: unsupported dtype ", t.scalar_type());
  }
  return ncclUint8;
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    TORCH_CHECK(hipSetDevice(dev) == hipSuccess, "dedloc_comm: hipSetDevice(", dev, ") failed");
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

at::Tensor unique_id() {
  ncclUniqueId id;
  ncclResult_t rc = ncclGetUniqueId(&id);
  TORCH_CHECK(rc == ncclSuccess, "ncclGetUniqueId failed: ", ncclGetErrorString(rc));
  auto out = at::empty({(int64_t)sizeof(id.internal)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(out.data_ptr(), id.internal, sizeof(id.internal));
  return out;
}

int64_t comm_init(const at::Tensor& uid, int64_t nranks, int64_t rank, int64_t device) {
  TORCH_CHECK(uid.scalar_type() == at::kByte && uid.numel() == (int64_t)sizeof(ncclUniqueId) && !uid.is_cuda(),
              "dedloc_comm: uid must be a CPU uint8 tensor of ", sizeof(ncclUniqueId), " bytes");
  TORCH_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "dedloc_comm: bad rank ", rank, " of ", nranks);
  ncclUniqueId id;
  std::memcpy(id.internal, uid.contiguous().data_ptr(), sizeof(id.internal));
  DeviceGuard g((int)device);
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  auto c = std::make_shared<Comm>();
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  ncclResult_t rc = ncclCommInitRankConfig(&c->comm, (int)nranks, id, (int)rank, &cfg);
  if (rc != ncclSuccess && rc != ncclInProgress) {
    if (c->comm != nullptr) (void)ncclCommAbort(c->comm);
    TORCH_CHECK(false, "ncclCommInitRankConfig failed: ", ncclGetErrorString(rc));
  }
  const int64_t h = g_next.fetch_add(1);
  std::lock_guard<std::mutex> lk(g_mu);
  g_comms[h] = c;
  return h;
}

int64_t comm_status(int64_t h) {
  auto c = lookup(h);
  ncclResult_t st = ncclSuccess;
  ncclResult_t rc = ncclCommGetAsyncError(c->comm, &st);
  if (rc != ncclSuccess) return (int64_t)rc;
  return (int64_t)st;
}

int64_t group_p2p(int64_t h, at::TensorList sends, at::IntArrayRef send_peers, at::TensorList recvs,
                  at::IntArrayRef recv_peers) {
  TORCH_CHECK(sends.size() == send_peers.size() && recvs.size() == recv_peers.size(),
              "dedloc_comm: one peer per tensor");
  auto c = lookup(h);
  auto check = [&](const at::Tensor& t, int64_t peer) {
    TORCH_CHECK(t.is_cuda() && t.get_device() == c->device, "dedloc_comm: tensors must live on device ", c->device);
    TORCH_CHECK(t.is_contiguous(), "dedloc_comm: tensors must be contiguous");
    TORCH_CHECK(peer >= 0 && peer < c->nranks, "dedloc_comm: peer ", peer, " outside 0..", c->nranks - 1);
  };
  for (size_t i = 0; i < sends.size(); ++i) check(sends[i], send_peers[i]);
  for (size_t i = 0; i < recvs.size(); ++i) check(recvs[i], recv_peers[i]);
  DeviceGuard g((int)c->device);
  hipStream_t stream = c10::hip::getCurrentHIPStream((int)c->device).stream();
  ncclResult_t rc = ncclGroupStart();
  TORCH_CHECK(rc == ncclSuccess, "ncclGroupStart failed: ", ncclGetErrorString(rc));
  ncclResult_t first = ncclSuccess;
  // receives first: with all-pairs traffic every rank posts its receives before its sends
  for (size_t i = 0; i < recvs.size(); ++i) {
    if (recvs[i].numel() == 0) continue;
    rc = ncclRecv(recvs[i].data_ptr(), (size_t)recvs[i].numel(), nccl_dtype(recvs[i]), (int)recv_peers[i], c->comm,
                  stream);
    if (rc != ncclSuccess && rc != ncclInProgress && first == ncclSuccess) first = rc;
  }
  for (size_t i = 0; i < sends.size(); ++i) {
    if (sends[i].numel() == 0) continue;
    rc = ncclSend(sends[i].data_ptr(), (size_t)sends[i].numel(), nccl_dtype(sends[i]), (int)send_peers[i], c->comm,
                  stream);
    if (rc != ncclSuccess && rc != ncclInProgress && first == ncclSuccess) first = rc;
  }
  rc = ncclGroupEnd();
  if (first != ncclSuccess) return (int64_t)first;
  return (int64_t)rc;  // ncclInProgress: poll comm_status until ready, then the stream holds the transfer
}

void comm_abort(int64_t h) {
  std::shared_ptr<Comm> c;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_comms.find(h);
    if (it == g_comms.end()) return;
    c = it->second;
    g_comms.erase(it);
  }
  DeviceGuard g((int)c->device);
  (void)ncclCommAbort(c->comm);
  c->comm = nullptr;
}

int64_t comm_count() {
  std::lock_guard<std::mutex> lk(g_mu);
  return (int64_t)g_comms.size();
}

std::string error_string(int64_t code) { return ncclGetErrorString((ncclResult_t)code); }

}  // namespace

TORCH_LIBRARY(dedloc_comm, m) {
  m.def("unique_id() -> Tensor", &unique_id);
  m.def("comm_init(Tensor uid, int nranks, int rank, int device) -> int", &comm_init);
  m.def("comm_status(int handle) -> int", &comm_status);
  m.def("group_p2p(int handle, Tensor[] sends, int[] send_peers, Tensor(a!)[] recvs, int[] recv_peers) -> int",
        &group_p2p);
  m.def("comm_abort(int handle) -> ()", &comm_abort);
  m.def("comm_count() -> int", &comm_count);
  m.def("error_string(int code) -> str", &error_string);
}

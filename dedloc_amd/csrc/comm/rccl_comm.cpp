// Native RCCL data plane for open-membership collaborations: the
// torch.library adapter over the communicator registry in comm_core.{h,cpp}.
//
// A collaboration has no fixed world: peers come and go, and every matchmade group (any subset of
// the GPU peers on the node, plus newcomers that were never part of any launch) averages over its
// own communicator.  Operators:
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
//   comm_release(h)                  the failure / end-of-life path: ncclCommAbort (cancels posted
//                                    operations, frees the communicator) — unless the bootstrap is
//                                    still in flight, in which case the communicator is quarantined
//                                    (returns 1) and comm_reap() aborts it once RCCL is done with it
//   comm_reap()                      abort quarantined communicators whose bootstrap has ended;
//                                    returns how many are still waiting
//   comm_count() / comm_quarantined()
//
// The library is resolved against the librccl.so.1 that torch itself loaded (same soname, torch's
// lib dir first on the link line), so one RCCL instance serves torch and us.
#include <torch/extension.h>
#include <torch/library.h>
#include <c10/hip/HIPStream.h>

#include <cstring>

#include "comm_core.h"

namespace {

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
  ncclUniqueId id;
  std::memcpy(id.internal, uid.contiguous().data_ptr(), sizeof(id.internal));
  std::string err;
  const int64_t h = dlcomm::registry().init(id, (int)nranks, (int)rank, (int)device, &err);
  TORCH_CHECK(h >= 0, "dedloc_comm: ", err);
  return h;
}

int64_t comm_status(int64_t h) { return dlcomm::registry().status(h); }

int64_t group_p2p(int64_t h, at::TensorList sends, at::IntArrayRef send_peers, at::TensorList recvs,
                  at::IntArrayRef recv_peers) {
  TORCH_CHECK(sends.size() == send_peers.size() && recvs.size() == recv_peers.size(),
              "dedloc_comm: one peer per tensor");
  int64_t device = 0, nranks = 0;
  TORCH_CHECK(dlcomm::registry().device_of(h, &device, &nranks), "dedloc_comm: unknown or aborted communicator ", h);
  std::vector<dlcomm::P2POp> ops;
  ops.reserve(sends.size() + recvs.size());
  auto add = [&](const at::Tensor& t, int64_t peer, bool send) {
    TORCH_CHECK(t.is_cuda() && t.get_device() == device, "dedloc_comm: tensors must live on device ", device);
    TORCH_CHECK(t.is_contiguous(), "dedloc_comm: tensors must be contiguous");
    TORCH_CHECK(peer >= 0 && peer < nranks, "dedloc_comm: peer ", peer, " outside 0..", nranks - 1);
    ops.push_back({t.data_ptr(), (size_t)t.numel(), nccl_dtype(t), (int)peer, send});
  };
  for (size_t i = 0; i < recvs.size(); ++i) add(recvs[i], recv_peers[i], false);
  for (size_t i = 0; i < sends.size(); ++i) add(sends[i], send_peers[i], true);
  hipStream_t stream = c10::hip::getCurrentHIPStream((int)device).stream();
  return dlcomm::registry().group_p2p(h, ops, stream);
}

int64_t comm_release(int64_t h) { return dlcomm::registry().release(h); }
int64_t comm_reap() { return dlcomm::registry().reap(); }
int64_t comm_count() { return dlcomm::registry().live(); }
int64_t comm_quarantined() { return dlcomm::registry().quarantined(); }
std::string error_string(int64_t code) { return ncclGetErrorString((ncclResult_t)code); }

}  // namespace

TORCH_LIBRARY(dedloc_comm, m) {
  m.def("unique_id() -> Tensor", &unique_id);
  m.def("comm_init(Tensor uid, int nranks, int rank, int device) -> int", &comm_init);
  m.def("comm_status(int handle) -> int", &comm_status);
  m.def("group_p2p(int handle, Tensor[] sends, int[] send_peers, Tensor(a!)[] recvs, int[] recv_peers) -> int",
        &group_p2p);
  m.def("comm_release(int handle) -> int", &comm_release);
  m.def("comm_reap() -> int", &comm_reap);
  m.def("comm_count() -> int", &comm_count);
  m.def("comm_quarantined() -> int", &comm_quarantined);
  m.def("error_string(int code) -> str", &error_string);
}

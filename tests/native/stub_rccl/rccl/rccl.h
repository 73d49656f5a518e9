// Host-only stand-in for the subset of <rccl/rccl.h> that csrc/comm/comm_core.cpp uses, so the
// communicator registry can be built and run under the host sanitizers on a machine with no GPU
// (tests/native/rccl_core_test.cpp implements these functions with a simulated bootstrap).
#pragma once
#include <cstddef>

typedef enum {
  ncclSuccess = 0,
  ncclUnhandledCudaError = 1,
  ncclSystemError = 2,
  ncclInternalError = 3,
  ncclInvalidArgument = 4,
  ncclInvalidUsage = 5,
  ncclRemoteError = 6,
  ncclInProgress = 7,
  ncclNumResults = 8
} ncclResult_t;

typedef enum {
  ncclInt8 = 0, ncclUint8 = 1, ncclInt32 = 2, ncclUint32 = 3, ncclInt64 = 4, ncclUint64 = 5,
  ncclFloat16 = 6, ncclFloat32 = 7, ncclFloat64 = 8, ncclBfloat16 = 9
} ncclDataType_t;

#define NCCL_UNIQUE_ID_BYTES 128
typedef struct { char internal[NCCL_UNIQUE_ID_BYTES]; } ncclUniqueId;
typedef struct ncclComm* ncclComm_t;
typedef struct {
  int blocking;
} ncclConfig_t;
#define NCCL_CONFIG_INITIALIZER {1}

typedef void* hipStream_t;

ncclResult_t ncclGetUniqueId(ncclUniqueId* id);
ncclResult_t ncclCommInitRankConfig(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank, ncclConfig_t* cfg);
ncclResult_t ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* state);
ncclResult_t ncclCommAbort(ncclComm_t comm);
ncclResult_t ncclGroupStart();
ncclResult_t ncclGroupEnd();
ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t s);
ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t s);
const char* ncclGetErrorString(ncclResult_t r);

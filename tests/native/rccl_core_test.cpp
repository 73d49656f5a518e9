// Host sanitizer run of the RCCL data plane's communicator registry (csrc/comm/comm_core.cpp),
// built against the stub headers in tests/native/stub_rccl.
//
// The stub RCCL below simulates what matters for the lifecycle: ncclCommInitRankConfig with
// blocking = 0 starts a background "init thread" that keeps writing into the communicator until
// every rank of its unique id has joined; ncclCommAbort frees the communicator.  Aborting a
// communicator whose init thread is still running is counted as a violation (in real RCCL that is
// the window in which the init thread can touch freed state); any use of a freed communicator is
// caught by AddressSanitizer, and unsynchronised registry access by ThreadSanitizer.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../dedloc_amd/csrc/comm/comm_core.h"

// ------------------------------------------------------------------------------------ stub RCCL
struct ncclComm {
  std::string uid;
  int nranks = 0, rank = 0;
  std::atomic<int> state{ncclInProgress};
  std::atomic<bool> init_running{true};
  std::atomic<bool> abort_flag{false};
  std::atomic<long> touched{0};  // written by the init thread
  long ops = 0;                  // written by send/recv (under the registry's per-communicator lock)
};

namespace {
std::mutex g_mu;
std::map<std::string, int> g_joined;
std::atomic<long> g_uid{0};
std::atomic<int> g_violations{0};
std::atomic<bool> g_give_up{false};
std::atomic<int> g_init_threads{0};
std::atomic<bool> g_enqueue_stalls{false};  // sends stay "being enqueued" (lazy connect to a dead peer)
thread_local int g_group_depth = 0;

int joined(const std::string& uid) {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_joined[uid];
}
}  // namespace

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  std::memset(id->internal, 0, sizeof(id->internal));
  std::snprintf(id->internal, sizeof(id->internal), "uid-%ld", g_uid.fetch_add(1));
  return ncclSuccess;
}

ncclResult_t ncclCommInitRankConfig(ncclComm_t* out, int nranks, ncclUniqueId id, int rank, ncclConfig_t* cfg) {
  if (cfg == nullptr || cfg->blocking != 0) return ncclInvalidUsage;
  auto* c = new ncclComm();
  c->uid = std::string(id.internal);
  c->nranks = nranks;
  c->rank = rank;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    g_joined[c->uid] += 1;
  }
  *out = c;
  g_init_threads.fetch_add(1);
  std::thread([c]() {
    // the bootstrap: wait for every rank (or an abort), touching the communicator all along
    while (joined(c->uid) < c->nranks && !c->abort_flag.load() && !g_give_up.load()) {
      c->touched.fetch_add(1);
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    if (!g_give_up.load()) {
      c->touched.fetch_add(1);
      if (c->abort_flag.load()) {  // ncclCommAbort is waiting for this thread: its last access
        c->state.store((int)ncclRemoteError);
        c->init_running.store(false);
      } else {  // done before the state says so; the state store is the last access (then aborts are legal)
        c->init_running.store(false);
        c->state.store((int)ncclSuccess);
      }
    }
    g_init_threads.fetch_sub(1);
  }).detach();
  return ncclInProgress;
}

ncclResult_t ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* state) {
  *state = (ncclResult_t)comm->state.load();
  return ncclSuccess;
}

ncclResult_t ncclCommAbort(ncclComm_t comm) {
  if (comm->init_running.load()) {
    g_violations.fetch_add(1);  // freeing state RCCL's init thread still owns
    comm->abort_flag.store(true);
    while (comm->init_running.load() && !g_give_up.load()) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  delete comm;
  return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
  ++g_group_depth;
  return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
  if (g_group_depth <= 0) return ncclInvalidUsage;
  --g_group_depth;
  return ncclSuccess;
}

ncclResult_t ncclSend(const void*, size_t, ncclDataType_t, int peer, ncclComm_t comm, hipStream_t) {
  if (g_group_depth <= 0 || peer < 0 || peer >= comm->nranks) return ncclInvalidUsage;
  if (comm->state.load() != ncclSuccess) return ncclInvalidUsage;
  comm->ops += 1;
  if (g_enqueue_stalls.load()) {  // non-blocking group: the enqueue never finishes
    comm->state.store((int)ncclInProgress);
    return ncclInProgress;
  }
  return ncclSuccess;
}

ncclResult_t ncclRecv(void*, size_t, ncclDataType_t, int peer, ncclComm_t comm, hipStream_t) {
  if (g_group_depth <= 0 || peer < 0 || peer >= comm->nranks) return ncclInvalidUsage;
  if (comm->state.load() != ncclSuccess) return ncclInvalidUsage;
  comm->ops += 1;
  return ncclSuccess;
}

const char* ncclGetErrorString(ncclResult_t r) { return r == ncclSuccess ? "no error" : "stub error"; }

static thread_local int g_dev = 0;
hipError_t hipGetDevice(int* dev) {
  *dev = g_dev;
  return hipSuccess;
}
hipError_t hipSetDevice(int dev) {
  if (dev < 0 || dev > 7) return hipErrorInvalidDevice;
  g_dev = dev;
  return hipSuccess;
}

// ------------------------------------------------------------------------------------ the test
#define CHECK(cond)                                                             \
  do {                                                                          \
    if (!(cond)) {                                                              \
      std::fprintf(stderr, "CHECK failed at %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

using dlcomm::registry;

static int64_t make(int nranks, int rank, const ncclUniqueId& id) {
  std::string err;
  int64_t h = registry().init(id, nranks, rank, 0, &err);
  CHECK(h > 0);
  return h;
}

static ncclUniqueId new_id() {
  ncclUniqueId id;
  ncclGetUniqueId(&id);
  return id;
}

static void wait_ready(int64_t h) {
  for (int i = 0; i < 20000; ++i) {
    int64_t st = registry().status(h);
    if (st == ncclSuccess) return;
    CHECK(st == ncclInProgress);
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
  CHECK(false && "bootstrap never finished");
}

int main() {
  int payload[4] = {0, 1, 2, 3};
  // 1. one-rank communicator: ready, grouped send/recv, release aborts it
  {
    int64_t h = make(1, 0, new_id());
    wait_ready(h);
    std::vector<dlcomm::P2POp> ops = {{payload, 4, ncclInt32, 0, false}, {payload, 4, ncclInt32, 0, true}};
    CHECK(registry().group_p2p(h, ops, nullptr) == ncclSuccess);
    std::vector<dlcomm::P2POp> bad = {{payload, 4, ncclInt32, 3, true}};
    CHECK(registry().group_p2p(h, bad, nullptr) == ncclInvalidArgument);
    CHECK(registry().live() == 1);
    CHECK(registry().release(h) == dlcomm::kAborted);
    CHECK(registry().release(h) == dlcomm::kUnknownHandle);  // double release: a clean no-op
    CHECK(registry().status(h) == ncclInvalidArgument);
    CHECK(registry().group_p2p(h, ops, nullptr) == ncclInvalidArgument);
    CHECK(registry().live() == 0);
  }
  // 2. a member that never arrives: quarantined (not aborted) until its bootstrap ends
  {
    ncclUniqueId id = new_id();
    int64_t h0 = make(2, 0, id);
    CHECK(registry().release(h0) == dlcomm::kQuarantined);
    CHECK(registry().quarantined() == 1 && registry().live() == 0);
    std::vector<dlcomm::P2POp> ops = {{payload, 4, ncclInt32, 1, true}};
    CHECK(registry().group_p2p(h0, ops, nullptr) == ncclInvalidUsage);  // never used again
    CHECK(registry().reap() == 1);
    int64_t h1 = make(2, 1, id);  // the late member: the bootstrap completes
    wait_ready(h1);
    for (int i = 0; i < 20000 && registry().reap() != 0; ++i) std::this_thread::sleep_for(std::chrono::microseconds(100));
    CHECK(registry().quarantined() == 0);
    CHECK(registry().release(h1) == dlcomm::kAborted);
    CHECK(registry().live() == 0);
  }
  // 3. a grouped send/recv still being enqueued AFTER the bootstrap completed (lazy
  //    connection set-up towards a member that died): release() aborts at once instead of
  //    quarantining — that abort is what cancels the round's operations
  {
    int64_t h = make(1, 0, new_id());
    wait_ready(h);
    g_enqueue_stalls.store(true);
    std::vector<dlcomm::P2POp> ops = {{payload, 4, ncclInt32, 0, true}};
    CHECK(registry().group_p2p(h, ops, nullptr) == ncclSuccess);
    CHECK(registry().status(h) == ncclInProgress);
    g_enqueue_stalls.store(false);
    const int64_t q0 = registry().quarantined();
    CHECK(registry().release(h) == dlcomm::kAborted);
    CHECK(registry().quarantined() == q0);
    CHECK(registry().status(h) == ncclInvalidArgument);
  }
  // 4. two threads hammering the registry: one creates / uses / releases communicators (some
  //    with a missing member), the other polls, posts, releases and reaps the same handles
  {
    std::mutex hm;
    std::vector<int64_t> handles;
    std::atomic<bool> done{false};
    std::thread creator([&]() {
      std::mt19937 rng(1);
      for (int i = 0; i < 400; ++i) {
        ncclUniqueId id = new_id();
        int n = 1 + (int)(rng() % 2);
        int64_t h = make(n, 0, id);
        {
          std::lock_guard<std::mutex> lk(hm);
          handles.push_back(h);
        }
        if (n == 2 && rng() % 2) make(n, 1, id);  // sometimes the member shows up (its handle leaks: fine)
        if (rng() % 3 == 0) (void)registry().release(h);
      }
      done.store(true);
    });
    std::thread poker([&]() {
      std::mt19937 rng(2);
      int p[2] = {0, 0};
      while (!done.load()) {
        int64_t h = 0;
        {
          std::lock_guard<std::mutex> lk(hm);
          if (!handles.empty()) h = handles[rng() % handles.size()];
        }
        if (h == 0) continue;
        switch (rng() % 4) {
          case 0: (void)registry().status(h); break;
          case 1: {
            std::vector<dlcomm::P2POp> ops = {{p, 2, ncclInt32, 0, true}};
            (void)registry().group_p2p(h, ops, nullptr);
            break;
          }
          case 2: (void)registry().release(h); break;
          default: (void)registry().reap(); break;
        }
      }
    });
    creator.join();
    poker.join();
    for (int64_t h : handles) (void)registry().release(h);
    (void)registry().reap();
  }
  CHECK(g_violations.load() == 0);
  g_give_up.store(true);  // bootstraps that will never complete: let their threads end
  for (int i = 0; i < 2000 && g_init_threads.load() > 0; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(1));
  std::printf("rccl_core_test OK (live %lld, quarantined %lld)\n", (long long)registry().live(),
              (long long)registry().quarantined());
  return 0;
}

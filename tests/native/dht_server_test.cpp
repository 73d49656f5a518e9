// Host-side stress test of the native control-plane server (csrc/runtime/dht_server.cpp), built with
// AddressSanitizer + UndefinedBehaviorSanitizer by tests/test_native_sanitizers.py (SURVEY.md §5.2:
// no GPU sanitizers on this pool, so the C++ runtime is checked on the host).
//
// Concurrent clients exercise STORE / GET (plain + subkeys, expiration ordering), KEYS, STATS and
// JOIN matchmaking (several groups forming at once, a group that fails its minimum size), then the
// server is stopped while idle connections are still open.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

extern "C" {
void* dht_server_start(const char* host, int port);
int dht_server_port(void* h);
void dht_server_stop(void* h);
}

namespace {

std::atomic<int> failures{0};
#define CHECK(cond)                                                       \
  do {                                                                    \
    if (!(cond)) {                                                        \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      failures++;                                                         \
    }                                                                     \
  } while (0)

double now_s() {
  using namespace std::chrono;
  return duration<double>(system_clock::now().time_since_epoch()).count();
}

struct Client {
  int fd = -1;
  explicit Client(int port) {
    fd = ::socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    ::inet_pton(AF_INET, "127.0.0.1", &a.sin_addr);
    if (::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) fd = -1;
  }
  ~Client() {
    if (fd >= 0) ::close(fd);
  }
  std::string call(uint8_t op, const std::string& payload) {
    std::string msg(1, (char)op);
    msg += payload;
    uint32_t n = (uint32_t)msg.size();
    ::send(fd, &n, 4, MSG_NOSIGNAL);
    ::send(fd, msg.data(), msg.size(), MSG_NOSIGNAL);
    uint32_t rn = 0;
    if (::recv(fd, &rn, 4, MSG_WAITALL) != 4) return {};
    std::string out(rn, '\0');
    if (rn && ::recv(fd, &out[0], rn, MSG_WAITALL) != (ssize_t)rn) return {};
    return out;
  }
};

void put_u32(std::string& s, uint32_t v) { s.append(reinterpret_cast<const char*>(&v), 4); }
void put_f64(std::string& s, double v) { s.append(reinterpret_cast<const char*>(&v), 8); }
void put_bytes(std::string& s, const std::string& b) {
  put_u32(s, (uint32_t)b.size());
  s += b;
}

bool store(Client& c, const std::string& key, const std::string* sub, const std::string& val, double exp) {
  std::string p;
  put_bytes(p, key);
  p += (char)(sub ? 1 : 0);
  put_bytes(p, sub ? *sub : std::string());
  put_bytes(p, val);
  put_f64(p, exp);
  std::string r = c.call(2, p);
  return r.size() == 1 && r[0] == 1;
}

// returns kind (0 missing, 1 plain, 2 dict) and the plain value / number of live subkeys
int get(Client& c, const std::string& key, std::string* plain, uint32_t* nsub) {
  std::string p;
  put_bytes(p, key);
  std::string r = c.call(3, p);
  if (r.empty()) return -1;
  const int kind = (uint8_t)r[0];
  if (kind == 1 && plain) {
    uint32_t n;
    std::memcpy(&n, r.data() + 1, 4);
    *plain = r.substr(5, n);
  }
  if (kind == 2 && nsub) std::memcpy(nsub, r.data() + 1, 4);
  return kind;
}

// JOIN -> (ok, group id, member count)
bool join(Client& c, const std::string& gkey, const std::string& peer, uint32_t target, uint32_t min_size,
          uint32_t expected, double window, uint64_t* gid, uint32_t* nmembers) {
  std::string p;
  put_bytes(p, gkey);
  put_bytes(p, peer);
  put_bytes(p, "info-" + peer);
  put_u32(p, target);
  put_u32(p, min_size);
  put_u32(p, expected);
  put_f64(p, window);
  std::string r = c.call(4, p);
  if (r.size() < 13) return false;
  const bool ok = r[0] == 0;  // first byte: 1 = the group failed
  std::memcpy(gid, r.data() + 1, 8);
  std::memcpy(nmembers, r.data() + 9, 4);
  return ok;
}

}  // namespace

int main() {
  void* h = dht_server_start("127.0.0.1", 0);
  if (!h) {
    std::fprintf(stderr, "server did not start\n");
    return 2;
  }
  const int port = dht_server_port(h);

  {  // plain values: newer expiration wins, older is rejected, expired is invisible
    Client c(port);
    const double t = now_s();
    CHECK(store(c, "k", nullptr, "v1", t + 30));
    CHECK(!store(c, "k", nullptr, "old", t + 10));
    CHECK(store(c, "k", nullptr, "v2", t + 60));
    std::string v;
    CHECK(get(c, "k", &v, nullptr) == 1 && v == "v2");
    CHECK(!store(c, "dead", nullptr, "x", t - 1));
    CHECK(get(c, "dead", nullptr, nullptr) == 0);
  }

  {  // concurrent subkey writers on one key
    std::vector<std::thread> ts;
    for (int i = 0; i < 8; ++i)
      ts.emplace_back([port, i] {
        Client c(port);
        for (int j = 0; j < 200; ++j) {
          const std::string sub = "peer" + std::to_string(i);
          CHECK(store(c, "progress", &sub, "step" + std::to_string(j), now_s() + 30 + j * 1e-3));
          uint32_t n = 0;
          CHECK(get(c, "progress", nullptr, &n) == 2);
        }
      });
    for (auto& t : ts) t.join();
    Client c(port);
    uint32_t n = 0;
    CHECK(get(c, "progress", nullptr, &n) == 2 && n == 8);
  }

  {  // matchmaking: 3 groups of 4 form concurrently on distinct keys; all members agree on the id
    std::vector<std::thread> ts;
    std::vector<uint64_t> gids(12);
    std::vector<uint32_t> sizes(12);
    for (int i = 0; i < 12; ++i)
      ts.emplace_back([&, i] {
        Client c(port);
        CHECK(join(c, "avg" + std::to_string(i / 4), "p" + std::to_string(i), 4, 2, 4, 5.0, &gids[i], &sizes[i]));
      });
    for (auto& t : ts) t.join();
    for (int i = 0; i < 12; ++i) {
      CHECK(sizes[i] == 4);
      CHECK(gids[i] == gids[(i / 4) * 4]);
    }
    CHECK(gids[0] != gids[4] && gids[4] != gids[8]);
  }

  {  // a lonely joiner fails its minimum group size when the window closes
    Client c(port);
    uint64_t gid = 0;
    uint32_t n = 0;
    CHECK(!join(c, "lonely", "solo", 8, 2, 0, 0.5, &gid, &n));
  }

  {  // keys + stats + an idle connection left open across stop()
    Client c(port);
    std::string keys_payload;
    put_bytes(keys_payload, "");
    CHECK(!c.call(5, keys_payload).empty());
    CHECK(!c.call(6, "").empty());
  }
  Client idle(port);
  dht_server_stop(h);
  if (failures) {
    std::fprintf(stderr, "%d checks failed\n", failures.load());
    return 1;
  }
  std::printf("dht_server_test OK\n");
  return 0;
}

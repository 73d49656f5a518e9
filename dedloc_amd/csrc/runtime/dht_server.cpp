// dedloc control-plane node: a native key/value + matchmaking server (the runtime piece that
// replaces hivemind's asyncio/gRPC Kademlia node).
//
// Semantics (hivemind 0.9.x DHT, as relied on by the reference):
//   * key -> plain value  or  key -> {subkey -> value}, every entry with an absolute expiration
//     (DHT time = wall clock); a write is accepted only if its expiration is later than the stored
//     one for that key/subkey; expired entries are invisible; values are opaque (msgpack blobs,
//     signed/validated by the Python client's record validators).
//   * JOIN implements matchmaking: peers that want to average under the same group key are
//     gathered into a group that closes when it reaches `target` members, when `expected` live
//     peers have joined, or when the window of the first joiner expires (failing if it is then
//     smaller than `min`).  Every member receives the same ordered member list + group id.
//   * Small groups (Moshpit-style, `target` < `expected`, e.g. SwAV's target_group_size 4 with 8
//     peers): the round gathers every expected peer, then splits them into G = ceil(n / target)
//     groups by rank in peer-id order, alternating between two partitions — contiguous blocks on
//     even rounds of the key, stride-G classes on odd rounds.  Each stride class holds a member
//     of every block (G <= target), so two consecutive rounds of equal-weight peers reproduce the
//     exact global average, and only 2G member sets ever occur (their data-plane communicators
//     are created once).  Closing at the first `target` arrivals instead would let an always-
//     faster subset average only among itself, and the collaboration would split in two.
//
// Transport: TCP, one thread per connection, length-prefixed frames:
//   request  = u32 len | u8 op | payload      response = u32 len | payload
// Exposed through a tiny C ABI (dht_server_start / _port / _stop) loaded by dedloc_amd/dht.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

double now_s() {
  using namespace std::chrono;
  return duration<double>(system_clock::now().time_since_epoch()).count();
}

struct Entry {
  std::string value;
  double expiration = 0;
};

struct Record {
  bool is_dict = false;
  Entry plain;
  std::map<std::string, Entry> sub;
  double max_exp() const {
    if (!is_dict) return plain.expiration;
    double m = 0;
    for (auto& kv : sub) m = std::max(m, kv.second.expiration);
    return m;
  }
};

struct Member {
  std::string peer_id, info;
};

struct Group {
  uint64_t id = 0;
  std::vector<Member> members;
  double deadline = 0;
  uint32_t target = 0, min_size = 2, expected = 0;
  uint64_t round = 0;                 // completed rounds of this group key before this one
  bool closed = false, failed = false;
  // filled at close: member index -> sub-group, and per sub-group its member indices, id, failed
  std::vector<int> part_of;
  std::vector<std::vector<int>> parts;
  std::vector<uint64_t> part_ids;
  std::vector<bool> part_failed;
};

// Close a gathered round: one group of everybody, or the Moshpit split described at the top.
void close_group(Group& gr, uint64_t& next_id) {
  gr.closed = true;
  const int n = (int)gr.members.size();
  gr.part_of.assign(n, 0);
  gr.parts.clear();
  gr.part_ids.clear();
  gr.part_failed.clear();
  const int target = (int)std::max<uint32_t>(1, gr.target);
  if (n <= target) {
    std::vector<int> all(n);
    for (int i = 0; i < n; ++i) all[i] = i;
    gr.parts.push_back(all);
    gr.part_ids.push_back(gr.id);
    gr.part_failed.push_back(n < (int)gr.min_size);
    gr.failed = gr.part_failed[0];
    return;
  }
  std::vector<int> order(n);
  for (int i = 0; i < n; ++i) order[i] = i;
  std::sort(order.begin(), order.end(),
            [&](int a, int b) { return gr.members[a].peer_id < gr.members[b].peer_id; });
  const int G = (n + target - 1) / target;
  const int block = (n + G - 1) / G;
  gr.parts.assign(G, {});
  for (int p = 0; p < n; ++p) {
    const int part = (gr.round & 1) ? p % G : p / block;
    gr.parts[part].push_back(order[p]);
    gr.part_of[order[p]] = part;
  }
  for (int q = 0; q < G; ++q) {
    gr.part_ids.push_back(q == 0 ? gr.id : ++next_id);
    gr.part_failed.push_back((int)gr.parts[q].size() < (int)gr.min_size);
  }
  gr.failed = false;
}

// ------------------------------------------------------------------ wire helpers
struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;
  template <typename T>
  T pod() {
    T v{};
    if (end - p < (ptrdiff_t)sizeof(T)) { ok = false; return v; }
    std::memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  std::string bytes() {
    uint32_t n = pod<uint32_t>();
    if (!ok || end - p < (ptrdiff_t)n) { ok = false; return {}; }
    std::string s(reinterpret_cast<const char*>(p), n);
    p += n;
    return s;
  }
};

struct Writer {
  std::string buf;
  template <typename T>
  void pod(T v) { buf.append(reinterpret_cast<const char*>(&v), sizeof(T)); }
  void bytes(const std::string& s) { pod<uint32_t>((uint32_t)s.size()); buf += s; }
};

bool read_full(int fd, void* dst, size_t n) {
  uint8_t* p = static_cast<uint8_t*>(dst);
  while (n) {
    ssize_t r = ::recv(fd, p, n, 0);
    if (r <= 0) return false;
    p += r;
    n -= (size_t)r;
  }
  return true;
}

bool write_full(int fd, const void* src, size_t n) {
  const uint8_t* p = static_cast<const uint8_t*>(src);
  while (n) {
    ssize_t r = ::send(fd, p, n, MSG_NOSIGNAL);
    if (r <= 0) return false;
    p += r;
    n -= (size_t)r;
  }
  return true;
}

// ------------------------------------------------------------------ server
class Server {
 public:
  enum Op : uint8_t { PING = 1, STORE = 2, GET = 3, JOIN = 4, KEYS = 5, STATS = 6 };

  bool start(const char* host, int port) {
    fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd_ < 0) return false;
    int one = 1;
    ::setsockopt(fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    if (!host || !*host || std::strcmp(host, "*") == 0 || std::strcmp(host, "0.0.0.0") == 0) a.sin_addr.s_addr = INADDR_ANY;
    else if (::inet_pton(AF_INET, host, &a.sin_addr) != 1) return false;
    if (::bind(fd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) return false;
    if (::listen(fd_, 256) != 0) return false;
    socklen_t len = sizeof(a);
    ::getsockname(fd_, reinterpret_cast<sockaddr*>(&a), &len);
    port_ = ntohs(a.sin_port);
    running_ = true;
    acceptor_ = std::thread([this] { accept_loop(); });
    janitor_ = std::thread([this] { janitor_loop(); });
    return true;
  }

  void stop() {
    if (!running_.exchange(false)) return;
    ::shutdown(fd_, SHUT_RDWR);
    ::close(fd_);
    {
      std::lock_guard<std::mutex> g(mu_);
      for (int c : clients_) ::shutdown(c, SHUT_RDWR);
    }
    cv_.notify_all();
    if (acceptor_.joinable()) acceptor_.join();
    if (janitor_.joinable()) janitor_.join();
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait_for(g, std::chrono::seconds(5), [this] { return active_ == 0; });
  }

  int port() const { return port_; }

 private:
  void accept_loop() {
    while (running_) {
      int c = ::accept(fd_, nullptr, nullptr);
      if (c < 0) {
        if (!running_) break;
        continue;
      }
      int one = 1;
      ::setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      {
        std::lock_guard<std::mutex> g(mu_);
        clients_.push_back(c);
        ++active_;
      }
      std::thread([this, c] { serve(c); }).detach();
    }
  }

  void janitor_loop() {
    while (running_) {
      std::this_thread::sleep_for(std::chrono::milliseconds(200));
      std::lock_guard<std::mutex> g(mu_);
      const double t = now_s();
      bool changed = false;
      for (auto it = groups_.begin(); it != groups_.end();) {
        Group& gr = *it->second;
        if (!gr.closed && t >= gr.deadline) {
          close_group(gr, next_group_);
          ++rounds_[it->first];
          changed = true;
        }
        if (gr.closed) it = groups_.erase(it);  // members hold shared_ptrs
        else ++it;
      }
      if (++sweep_ % 25 == 0) {
        for (auto it = store_.begin(); it != store_.end();) {
          Record& r = it->second;
          if (r.is_dict) {
            for (auto s = r.sub.begin(); s != r.sub.end();) s = s->second.expiration < t ? r.sub.erase(s) : std::next(s);
          }
          it = (r.max_exp() < t) ? store_.erase(it) : std::next(it);
        }
      }
      if (changed) cv_.notify_all();
    }
  }

  void serve(int c) {
    std::vector<uint8_t> buf;
    while (running_) {
      uint32_t len;
      if (!read_full(c, &len, 4) || len == 0 || len > (256u << 20)) break;
      buf.resize(len);
      if (!read_full(c, buf.data(), len)) break;
      Reader rd{buf.data() + 1, buf.data() + len};
      Writer w;
      switch (buf[0]) {
        case PING: w.pod<uint8_t>(1); break;
        case STORE: handle_store(rd, w); break;
        case GET: handle_get(rd, w); break;
        case JOIN: handle_join(rd, w); break;
        case KEYS: handle_keys(rd, w); break;
        case STATS: handle_stats(w); break;
        default: rd.ok = false;
      }
      if (!rd.ok) break;
      uint32_t out = (uint32_t)w.buf.size();
      if (!write_full(c, &out, 4) || !write_full(c, w.buf.data(), out)) break;
    }
    ::close(c);
    std::lock_guard<std::mutex> g(mu_);
    for (auto it = clients_.begin(); it != clients_.end(); ++it)
      if (*it == c) { clients_.erase(it); break; }
    --active_;
    done_cv_.notify_all();
  }

  void handle_store(Reader& rd, Writer& w) {
    std::string key = rd.bytes();
    uint8_t has_sub = rd.pod<uint8_t>();
    std::string sub = rd.bytes();
    std::string value = rd.bytes();
    double exp = rd.pod<double>();
    if (!rd.ok) return;
    std::lock_guard<std::mutex> g(mu_);
    const double t = now_s();
    uint8_t accepted = 0;
    if (exp >= t) {
      Record& r = store_[key];
      if (has_sub) {
        if (!r.is_dict) {
          if (r.plain.expiration < exp || r.plain.expiration < t) { r = Record(); r.is_dict = true; }
        }
        if (r.is_dict) {
          auto it = r.sub.find(sub);
          if (it == r.sub.end() || it->second.expiration < exp) {
            r.sub[sub] = Entry{value, exp};
            accepted = 1;
          }
        }
      } else {
        if (r.is_dict ? r.max_exp() < exp : r.plain.expiration < exp) {
          r = Record();
          r.plain = Entry{value, exp};
          accepted = 1;
        }
      }
      ++stores_;
    }
    w.pod<uint8_t>(accepted);
  }

  void handle_get(Reader& rd, Writer& w) {
    std::string key = rd.bytes();
    if (!rd.ok) return;
    std::lock_guard<std::mutex> g(mu_);
    ++gets_;
    const double t = now_s();
    auto it = store_.find(key);
    if (it == store_.end()) { w.pod<uint8_t>(0); return; }
    Record& r = it->second;
    if (!r.is_dict) {
      if (r.plain.expiration < t) { w.pod<uint8_t>(0); return; }
      w.pod<uint8_t>(1);
      w.bytes(r.plain.value);
      w.pod<double>(r.plain.expiration);
      return;
    }
    std::vector<const std::pair<const std::string, Entry>*> live;
    for (auto& kv : r.sub)
      if (kv.second.expiration >= t) live.push_back(&kv);
    if (live.empty()) { w.pod<uint8_t>(0); return; }
    w.pod<uint8_t>(2);
    w.pod<uint32_t>((uint32_t)live.size());
    for (auto* kv : live) {
      w.bytes(kv->first);
      w.bytes(kv->second.value);
      w.pod<double>(kv->second.expiration);
    }
  }

  void handle_join(Reader& rd, Writer& w) {
    std::string gkey = rd.bytes();
    std::string peer = rd.bytes();
    std::string info = rd.bytes();
    uint32_t target = rd.pod<uint32_t>();
    uint32_t min_size = rd.pod<uint32_t>();
    uint32_t expected = rd.pod<uint32_t>();
    double window = rd.pod<double>();
    if (!rd.ok) return;
    std::unique_lock<std::mutex> g(mu_);
    std::shared_ptr<Group> gr;
    auto it = groups_.find(gkey);
    if (it != groups_.end() && !it->second->closed) {
      gr = it->second;
      for (auto& m : gr->members)
        if (m.peer_id == peer) {  // duplicate join (the peer gave up on this round): the round fails
          close_group(*gr, next_group_);
          for (size_t q = 0; q < gr->part_failed.size(); ++q) gr->part_failed[q] = true;
          gr->failed = true;
          ++rounds_[gkey];
          groups_.erase(it);
          cv_.notify_all();
          gr.reset();
          break;
        }
    }
    if (!gr) {
      gr = std::make_shared<Group>();
      gr->id = ++next_group_;
      gr->deadline = now_s() + window;
      gr->target = std::max<uint32_t>(1, target);
      gr->min_size = std::max<uint32_t>(1, min_size);
      gr->expected = expected;
      gr->round = rounds_[gkey];
      groups_[gkey] = gr;
    }
    gr->members.push_back(Member{peer, info});
    const int me = (int)gr->members.size() - 1;
    if (expected > gr->expected) gr->expected = expected;
    const size_t n = gr->members.size();
    // with more expected peers than the target group size the round gathers everybody first
    // (then splits); otherwise it closes at the target size or when the expected peers are in
    const bool split_round = gr->expected > gr->target;
    if ((!split_round && n >= gr->target) || (gr->expected > 0 && n >= gr->expected)) {
      close_group(*gr, next_group_);
      ++rounds_[gkey];
      groups_.erase(gkey);
      cv_.notify_all();
    }
    cv_.wait(g, [&] { return gr->closed || !running_; });
    const bool closed_ok = running_ && gr->closed && me < (int)gr->part_of.size();
    const int part = closed_ok ? gr->part_of[me] : 0;
    const bool failed = !closed_ok || gr->part_failed[part];
    w.pod<uint8_t>(failed ? 1 : 0);
    w.pod<uint64_t>(closed_ok ? gr->part_ids[part] : gr->id);
    if (!closed_ok) {
      w.pod<uint32_t>(0);
      return;
    }
    const std::vector<int>& mine = gr->parts[part];
    w.pod<uint32_t>((uint32_t)mine.size());
    for (int i : mine) {
      w.bytes(gr->members[i].peer_id);
      w.bytes(gr->members[i].info);
    }
  }

  void handle_keys(Reader& rd, Writer& w) {
    std::string prefix = rd.bytes();
    if (!rd.ok) return;
    std::lock_guard<std::mutex> g(mu_);
    std::vector<const std::string*> ks;
    for (auto& kv : store_)
      if (kv.first.compare(0, prefix.size(), prefix) == 0) ks.push_back(&kv.first);
    w.pod<uint32_t>((uint32_t)ks.size());
    for (auto* k : ks) w.bytes(*k);
  }

  void handle_stats(Writer& w) {
    std::lock_guard<std::mutex> g(mu_);
    w.pod<uint64_t>(store_.size());
    w.pod<uint64_t>(stores_);
    w.pod<uint64_t>(gets_);
    w.pod<uint64_t>(next_group_);
  }

  int fd_ = -1, port_ = 0;
  std::atomic<bool> running_{false};
  std::thread acceptor_, janitor_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::map<std::string, Record> store_;
  std::map<std::string, std::shared_ptr<Group>> groups_;
  std::map<std::string, uint64_t> rounds_;  // closed rounds per group key (partition parity)
  std::vector<int> clients_;
  int active_ = 0;
  uint64_t next_group_ = 0, stores_ = 0, gets_ = 0, sweep_ = 0;
};

}  // namespace

extern "C" {
void* dht_server_start(const char* host, int port) {
  auto* s = new Server();
  if (!s->start(host, port)) {
    delete s;
    return nullptr;
  }
  return s;
}
int dht_server_port(void* h) { return h ? static_cast<Server*>(h)->port() : -1; }
void dht_server_stop(void* h) {
  if (!h) return;
  auto* s = static_cast<Server*>(h);
  s->stop();
  // intentionally leaked if connections are still draining; the process is usually exiting
}
}

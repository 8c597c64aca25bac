// Native TCP process group (see proc_group.hpp for the rationale).
#include "stencil/comm/proc_group.hpp"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <set>
#include <thread>

#include "stencil/rt/env.hpp"
#include "stencil/rt/logging.hpp"

namespace stencil {
namespace log {
static std::atomic<int> g_rank{0};
int rank() { return g_rank.load(); }
void set_rank(int r) { g_rank.store(r); }
int runtime_level() {
  static int lvl = int(env::get_int("STENCIL_LOG_LEVEL", 2));
  return lvl;
}
} // namespace log

namespace comm {

static std::string local_hostname() {
  if (env::has("STENCIL_HOSTNAME")) return env::get_str("STENCIL_HOSTNAME", "");
  char buf[256] = {0};
  gethostname(buf, sizeof(buf) - 1);
  return buf;
}

// ---------------------------------------------------------------------------------------------
// ProcGroup common helpers
// ---------------------------------------------------------------------------------------------
double ProcGroup::allreduce_max(double v) {
  std::vector<double> all(size());
  allgather(&v, sizeof(v), all.data());
  return *std::max_element(all.begin(), all.end());
}
double ProcGroup::allreduce_sum(double v) {
  std::vector<double> all(size());
  allgather(&v, sizeof(v), all.data());
  double s = 0;
  for (double x : all) s += x; // rank order: deterministic
  return s;
}
uint64_t ProcGroup::allreduce_sum_u64(uint64_t v) {
  std::vector<uint64_t> all(size());
  allgather(&v, sizeof(v), all.data());
  uint64_t s = 0;
  for (uint64_t x : all) s += x;
  return s;
}
int64_t ProcGroup::allreduce_min_i64(int64_t v) {
  std::vector<int64_t> all(size());
  allgather(&v, sizeof(v), all.data());
  return *std::min_element(all.begin(), all.end());
}
std::vector<int> ProcGroup::colocated_ranks() const {
  std::vector<int> r;
  for (int i = 0; i < size(); ++i)
    if (hostname(i) == hostname(rank())) r.push_back(i);
  return r;
}
int ProcGroup::colocated_rank() const {
  auto r = colocated_ranks();
  return int(std::find(r.begin(), r.end(), rank()) - r.begin());
}
int ProcGroup::num_nodes() const {
  std::set<std::string> s;
  for (int i = 0; i < size(); ++i) s.insert(hostname(i));
  return int(s.size());
}

// ---------------------------------------------------------------------------------------------
// Single-process group
// ---------------------------------------------------------------------------------------------
class SingleGroup : public ProcGroup {
  std::string host_;
  std::map<uint32_t, std::deque<std::vector<char>>> self_;

public:
  SingleGroup() : host_(local_hostname()) {}
  int rank() const override { return 0; }
  int size() const override { return 1; }
  const std::string &hostname(int) const override { return host_; }
  void send(int dst, uint32_t tag, const void *buf, size_t n) override {
    STENCIL_REQUIRE(dst == 0, "single group send to " << dst);
    self_[tag].emplace_back((const char *)buf, (const char *)buf + n);
  }
  bool try_recv(int src, uint32_t tag, void *buf, size_t n) override {
    STENCIL_REQUIRE(src == 0, "single group recv from " << src);
    auto &q = self_[tag];
    if (q.empty()) return false;
    STENCIL_REQUIRE(q.front().size() == n, "message size mismatch " << q.front().size() << " vs " << n);
    std::memcpy(buf, q.front().data(), n);
    q.pop_front();
    return true;
  }
  void recv(int src, uint32_t tag, void *buf, size_t n) override {
    if (!try_recv(src, tag, buf, n)) LOG_FATAL("single group recv would block forever (tag " << tag << ")");
  }
  void barrier() override {}
  std::shared_ptr<ProcGroup> fork(double) override { return std::make_shared<SingleGroup>(); }
  void bcast(void *, size_t, int) override {}
  void allgather(const void *in, size_t n, void *out) override { std::memcpy(out, in, n); }
  void gatherv(const void *in, size_t n, std::vector<std::vector<char>> *out, int) override {
    out->assign(1, std::vector<char>((const char *)in, (const char *)in + n));
  }
};

std::shared_ptr<ProcGroup> make_single_group() { return std::make_shared<SingleGroup>(); }

// ---------------------------------------------------------------------------------------------
// TCP full mesh
// ---------------------------------------------------------------------------------------------
namespace {
struct FrameHeader {
  uint32_t tag;
  uint32_t magic;
  uint64_t len;
};
constexpr uint32_t kMagic = 0x57e9c11u;
constexpr uint32_t kCollBit = 0x80000000u;

void write_all(int fd, const void *buf, size_t n) {
  const char *p = (const char *)buf;
  while (n) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      LOG_FATAL("socket send failed: " << strerror(errno));
    }
    p += w;
    n -= size_t(w);
  }
}
// returns false on orderly EOF before any byte
bool read_all(int fd, void *buf, size_t n) {
  char *p = (char *)buf;
  size_t got = 0;
  while (got < n) {
    ssize_t r = ::recv(fd, p + got, n - got, 0);
    if (r == 0) {
      if (got == 0) return false;
      LOG_FATAL("socket closed mid-message");
    }
    if (r < 0) {
      if (errno == EINTR) continue;
      if (got == 0 && (errno == ECONNRESET || errno == EBADF)) return false;
      LOG_FATAL("socket recv failed: " << strerror(errno));
    }
    got += size_t(r);
  }
  return true;
}
void set_nodelay(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}
int listen_on(const std::string &addr, int port, int *actualPort) {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  STENCIL_REQUIRE(fd >= 0, "socket(): " << strerror(errno));
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons(uint16_t(port));
  sa.sin_addr.s_addr = addr.empty() ? htonl(INADDR_ANY) : inet_addr(addr.c_str());
  if (::bind(fd, (sockaddr *)&sa, sizeof(sa)) != 0) {
    int e = errno;
    ::close(fd);
    LOG_FATAL("bind(" << addr << ":" << port << "): " << strerror(e));
  }
  STENCIL_REQUIRE(::listen(fd, 1024) == 0, "listen(): " << strerror(errno));
  socklen_t len = sizeof(sa);
  getsockname(fd, (sockaddr *)&sa, &len);
  if (actualPort) *actualPort = ntohs(sa.sin_port);
  return fd;
}
std::string resolve(const std::string &host) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res) return host;
  char buf[INET_ADDRSTRLEN];
  inet_ntop(AF_INET, &((sockaddr_in *)res->ai_addr)->sin_addr, buf, sizeof(buf));
  freeaddrinfo(res);
  return buf;
}
int connect_to(const std::string &addr, int port, double timeout_s) {
  const std::string ip = resolve(addr);
  auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  while (true) {
    int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = htons(uint16_t(port));
    sa.sin_addr.s_addr = inet_addr(ip.c_str());
    if (::connect(fd, (sockaddr *)&sa, sizeof(sa)) == 0) {
      set_nodelay(fd);
      return fd;
    }
    ::close(fd);
    if (std::chrono::steady_clock::now() > deadline) LOG_FATAL("connect to " << addr << ":" << port << " timed out");
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}
int accept_one(int lfd, double timeout_s) {
  pollfd p{lfd, POLLIN, 0};
  int rc = ::poll(&p, 1, int(timeout_s * 1000));
  STENCIL_REQUIRE(rc > 0, "accept timed out");
  int fd = ::accept(lfd, nullptr, nullptr);
  STENCIL_REQUIRE(fd >= 0, "accept(): " << strerror(errno));
  set_nodelay(fd);
  return fd;
}
void send_str(int fd, const std::string &s) {
  uint64_t n = s.size();
  write_all(fd, &n, sizeof(n));
  write_all(fd, s.data(), n);
}
std::string recv_str(int fd) {
  uint64_t n = 0;
  STENCIL_REQUIRE(read_all(fd, &n, sizeof(n)), "peer closed during bootstrap");
  std::string s(n, '\0');
  if (n) STENCIL_REQUIRE(read_all(fd, &s[0], n), "peer closed during bootstrap");
  return s;
}
} // namespace

class TcpGroup : public ProcGroup {
  int rank_, size_;
  double timeout_s_;
  std::vector<std::string> hosts_;
  std::string masterIp_; // the rendezvous address this rank reached rank 0 at (fork() reuses it)
  std::vector<int> fds_;
  std::vector<std::unique_ptr<std::mutex>> sendMu_;
  std::vector<std::thread> readers_;

  std::mutex mu_;
  std::condition_variable cv_;
  // mailbox[src][tag] -> queued payloads
  std::vector<std::map<uint32_t, std::deque<std::vector<char>>>> mailbox_;
  std::vector<bool> closed_;
  std::string error_;
  uint32_t collSeq_ = 0;

  void reader(int peer) {
    int fd = fds_[peer];
    while (true) {
      FrameHeader h{};
      bool ok;
      try {
        ok = read_all(fd, &h, sizeof(h));
      } catch (std::exception &e) {
        ok = false;
      }
      if (!ok) break;
      if (h.magic != kMagic) {
        std::lock_guard<std::mutex> lk(mu_);
        error_ = "bad frame from rank " + std::to_string(peer);
        break;
      }
      std::vector<char> payload(h.len);
      bool okp = true;
      try {
        if (h.len) okp = read_all(fd, payload.data(), h.len);
      } catch (std::exception &) {
        okp = false;
      }
      if (!okp) break;
      {
        std::lock_guard<std::mutex> lk(mu_);
        mailbox_[peer][h.tag].push_back(std::move(payload));
      }
      cv_.notify_all();
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      closed_[peer] = true;
    }
    cv_.notify_all();
  }

  uint32_t next_coll_tag() { return kCollBit | (collSeq_++ & 0x7fffffffu); }

  void send_raw(int dst, uint32_t tag, const void *buf, size_t n) {
    if (dst == rank_) {
      {
        std::lock_guard<std::mutex> lk(mu_);
        mailbox_[dst][tag].emplace_back((const char *)buf, (const char *)buf + n);
      }
      cv_.notify_all();
      return;
    }
    FrameHeader h{tag, kMagic, uint64_t(n)};
    std::lock_guard<std::mutex> lk(*sendMu_[dst]);
    write_all(fds_[dst], &h, sizeof(h));
    if (n) write_all(fds_[dst], buf, n);
  }

  std::vector<char> recv_raw(int src, uint32_t tag) {
    bool ok = false;
    std::vector<char> m = recv_raw_for(src, tag, timeout_s_, &ok);
    if (!ok)
      LOG_FATAL("recv from rank " << src << " tag " << std::hex << tag << std::dec << " timed out after " << timeout_s_
                                  << " s");
    return m;
  }

  // *ok = false on timeout (nothing consumed)
  std::vector<char> recv_raw_for(int src, uint32_t tag, double timeout_s, bool *ok) {
    std::unique_lock<std::mutex> lk(mu_);
    auto pred = [&] { return !mailbox_[src][tag].empty() || closed_[src] || !error_.empty(); };
    *ok = cv_.wait_for(lk, std::chrono::duration<double>(timeout_s), pred);
    if (!*ok) return {};
    auto &q = mailbox_[src][tag];
    if (q.empty()) LOG_FATAL("rank " << src << " closed its connection (" << error_ << ")");
    std::vector<char> m = std::move(q.front());
    q.pop_front();
    return m;
  }

public:
  TcpGroup(int rank, int size, const std::string &master, int port, double timeout_s)
      : rank_(rank), size_(size), timeout_s_(std::max(timeout_s, 600.0)), hosts_(size), fds_(size, -1),
        mailbox_(size), closed_(size, false) {
    // the rendezvous waits for every rank to start (a fresh node may take minutes to load torch): at least 600 s;
    // the configured timeout applies from the first barrier on
    const double bootTimeout = timeout_s_;
    log::set_rank(rank);
    for (int i = 0; i < size; ++i) sendMu_.emplace_back(new std::mutex);
    const std::string myHost = local_hostname();

    // every rank listens for its higher-ranked peers
    int myPort = 0;
    int lfd = (rank == 0) ? listen_on("", port, &myPort) : listen_on("", 0, &myPort);

    // rendezvous: table of (listen ip, port, hostname) for every rank, assembled by rank 0
    std::vector<std::string> ips(size), names(size);
    std::vector<int> ports(size);
    if (rank == 0) {
      ips[0] = resolve(master);
      ports[0] = myPort;
      names[0] = myHost;
      std::vector<int> bootFds(size, -1);
      for (int k = 1; k < size; ++k) {
        int fd = accept_one(lfd, bootTimeout);
        int32_t r = -1;
        STENCIL_REQUIRE(read_all(fd, &r, sizeof(r)), "bootstrap peer closed");
        STENCIL_REQUIRE(r > 0 && r < size && bootFds[r] < 0, "bad/duplicate bootstrap rank " << r);
        bootFds[r] = fd;
        ips[r] = recv_str(fd);
        int32_t p = 0;
        STENCIL_REQUIRE(read_all(fd, &p, sizeof(p)), "bootstrap peer closed");
        ports[r] = p;
        names[r] = recv_str(fd);
      }
      for (int r = 1; r < size; ++r) {
        for (int k = 0; k < size; ++k) {
          send_str(bootFds[r], ips[k]);
          int32_t p = ports[k];
          write_all(bootFds[r], &p, sizeof(p));
          send_str(bootFds[r], names[k]);
        }
      }
      // rank 0's bootstrap connections double as its links to every other rank
      for (int r = 1; r < size; ++r) fds_[r] = bootFds[r];
    } else {
      int fd = connect_to(master, port, bootTimeout);
      int32_t r = rank;
      write_all(fd, &r, sizeof(r));
      // our address as seen on the route to the master
      sockaddr_in sa{};
      socklen_t len = sizeof(sa);
      getsockname(fd, (sockaddr *)&sa, &len);
      char buf[INET_ADDRSTRLEN];
      inet_ntop(AF_INET, &sa.sin_addr, buf, sizeof(buf));
      send_str(fd, buf);
      int32_t p = myPort;
      write_all(fd, &p, sizeof(p));
      send_str(fd, myHost);
      for (int k = 0; k < size; ++k) {
        ips[k] = recv_str(fd);
        int32_t pk = 0;
        STENCIL_REQUIRE(read_all(fd, &pk, sizeof(pk)), "bootstrap closed");
        ports[k] = pk;
        names[k] = recv_str(fd);
      }
      fds_[0] = fd;
      // connect to ranks 1..rank-1, accept from rank+1..size-1
      for (int k = 1; k < rank; ++k) {
        int cfd = connect_to(ips[k], ports[k], bootTimeout);
        int32_t me = rank;
        write_all(cfd, &me, sizeof(me));
        fds_[k] = cfd;
      }
      for (int k = rank + 1; k < size; ++k) {
        int afd = accept_one(lfd, bootTimeout);
        int32_t who = -1;
        STENCIL_REQUIRE(read_all(afd, &who, sizeof(who)), "mesh peer closed");
        STENCIL_REQUIRE(who > rank && who < size && fds_[who] < 0, "bad mesh rank " << who);
        fds_[who] = afd;
      }
    }
    ::close(lfd);
    hosts_ = names;
    masterIp_ = master;
    for (int k = 0; k < size; ++k)
      if (k != rank) readers_.emplace_back(&TcpGroup::reader, this, k);
    barrier();
    timeout_s_ = timeout_s;
  }

  ~TcpGroup() override {
    for (int k = 0; k < size_; ++k)
      if (fds_[k] >= 0) ::shutdown(fds_[k], SHUT_RDWR);
    for (auto &t : readers_) t.join();
    for (int k = 0; k < size_; ++k)
      if (fds_[k] >= 0) ::close(fds_[k]);
  }

  int rank() const override { return rank_; }
  int size() const override { return size_; }
  const std::string &hostname(int r) const override { return hosts_.at(size_t(r)); }

  void send(int dst, uint32_t tag, const void *buf, size_t n) override {
    STENCIL_REQUIRE(!(tag & kCollBit), "user tags must not set the top bit");
    send_raw(dst, tag, buf, n);
  }
  void recv(int src, uint32_t tag, void *buf, size_t n) override {
    std::vector<char> m = recv_raw(src, tag);
    STENCIL_REQUIRE(m.size() == n, "recv size mismatch from rank " << src << ": got " << m.size() << " want " << n);
    if (n) std::memcpy(buf, m.data(), n);
  }
  bool try_recv(int src, uint32_t tag, void *buf, size_t n) override {
    std::vector<char> m;
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto &q = mailbox_[src][tag];
      if (q.empty()) return false;
      m = std::move(q.front());
      q.pop_front();
    }
    STENCIL_REQUIRE(m.size() == n, "recv size mismatch from rank " << src);
    if (n) std::memcpy(buf, m.data(), n);
    return true;
  }

  void barrier() override {
    char c = 0;
    std::vector<char> all(size_);
    allgather(&c, 1, all.data());
  }
  bool barrier_for(double timeout_s) override {
    const uint32_t tag = next_coll_tag();
    const char c = 0;
    bool ok = true;
    if (rank_ == 0) {
      for (int k = 1; k < size_ && ok; ++k) (void)recv_raw_for(k, tag, timeout_s, &ok);
      if (ok)
        for (int k = 1; k < size_; ++k) send_raw(k, tag, &c, 1);
    } else {
      send_raw(0, tag, &c, 1);
      (void)recv_raw_for(0, tag, timeout_s, &ok);
    }
    return ok;
  }
  void set_timeout(double timeout_s) override { timeout_s_ = timeout_s; }
  double timeout() const override { return timeout_s_; }
  std::shared_ptr<ProcGroup> fork(double timeout_s) override {
    int32_t port = rank_ == 0 ? find_free_port() : 0;
    bcast(&port, sizeof(port), 0);
    return std::make_shared<TcpGroup>(rank_, size_, masterIp_, port, timeout_s);
  }
  void bcast(void *buf, size_t n, int root) override {
    const uint32_t tag = next_coll_tag();
    if (rank_ == root) {
      for (int k = 0; k < size_; ++k)
        if (k != root) send_raw(k, tag, buf, n);
    } else {
      auto m = recv_raw(root, tag);
      STENCIL_REQUIRE(m.size() == n, "bcast size mismatch");
      std::memcpy(buf, m.data(), n);
    }
  }
  void allgather(const void *in, size_t n, void *out) override {
    const uint32_t tag = next_coll_tag();
    char *o = (char *)out;
    if (rank_ == 0) {
      std::memcpy(o, in, n);
      for (int k = 1; k < size_; ++k) {
        auto m = recv_raw(k, tag);
        STENCIL_REQUIRE(m.size() == n, "allgather size mismatch from rank " << k);
        std::memcpy(o + size_t(k) * n, m.data(), n);
      }
      for (int k = 1; k < size_; ++k) send_raw(k, tag, o, n * size_t(size_));
    } else {
      send_raw(0, tag, in, n);
      auto m = recv_raw(0, tag);
      STENCIL_REQUIRE(m.size() == n * size_t(size_), "allgather result size mismatch");
      std::memcpy(o, m.data(), m.size());
    }
  }
  void gatherv(const void *in, size_t n, std::vector<std::vector<char>> *out, int root) override {
    const uint32_t tag = next_coll_tag();
    if (rank_ == root) {
      out->assign(size_, {});
      for (int k = 0; k < size_; ++k) {
        if (k == root)
          (*out)[k].assign((const char *)in, (const char *)in + n);
        else
          (*out)[k] = recv_raw(k, tag);
      }
    } else {
      send_raw(root, tag, in, n);
    }
  }
};

std::shared_ptr<ProcGroup> make_tcp_group(int rank, int size, const std::string &master_addr, int master_port,
                                          double timeout_s) {
  if (size == 1) return make_single_group();
  return std::make_shared<TcpGroup>(rank, size, master_addr, master_port, timeout_s);
}

static int env_int(const char *a, const char *b, int dflt) {
  return int(env::get_int(a, b ? env::get_int(b, dflt) : dflt));
}

std::shared_ptr<ProcGroup> make_group_from_env() {
  const int size = env_int("STENCIL_WORLD_SIZE", "WORLD_SIZE", 1);
  const int rank = env_int("STENCIL_RANK", "RANK", 0);
  if (size <= 1) return make_single_group();
  const std::string addr = env::get_str("STENCIL_MASTER_ADDR", env::get_str("MASTER_ADDR", "127.0.0.1"));
  int port = env_int("STENCIL_MASTER_PORT", nullptr, -1);
  if (port < 0) port = env_int("MASTER_PORT", nullptr, 29500) + 1; // MASTER_PORT is held by torch's store
  const double timeout = env::get_double("STENCIL_COMM_TIMEOUT", env_wait_timeout(600.0));
  return make_tcp_group(rank, size, addr, port, timeout);
}

static std::mutex g_mu;
static std::shared_ptr<ProcGroup> g_default;

std::shared_ptr<ProcGroup> default_group() {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_default) g_default = make_group_from_env();
  return g_default;
}
void set_default_group(std::shared_ptr<ProcGroup> g) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_default = std::move(g);
  if (g_default) log::set_rank(g_default->rank());
}

int find_free_port() {
  int port = 0;
  int fd = listen_on("", 0, &port);
  ::close(fd);
  return port;
}

} // namespace comm
} // namespace stencil

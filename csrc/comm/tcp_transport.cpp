// Native framed TCP transport with ZeroMQ PUSH/PULL semantics.
//
// Replaces the reference's data/control plane (pyzmq PUSH->PULL, one zmq.Context per
// socket, payloads torch.save'd to results/*.pt on disk and re-read:
// /root/reference/utils/node_worker.py:13-67, :397-410, :476-485; config_sender.py:14-47).
//
//  * Pull: binds a listening socket; an epoll thread accepts any number of Push peers and
//    reassembles frames into an in-memory queue. recv(timeout) pops one message
//    (timeout 0 == zmq.NOBLOCK, -1 == block). No disk staging (fixes SURVEY.md Q5) and no
//    busy-poll: callers block on a condition variable (fixes Q6).
//  * Push: queues messages immediately (like ZMQ, a peer may bind later); a writer thread
//    (re)connects with back-off and drains the queue in order. flush(timeout) waits for
//    delivery to the kernel socket buffer - so a short-lived sender (ConfigSender) no longer
//    has to spin forever to keep its socket alive (Q10).
//  * Frame: 16-byte header {u32 magic 'LSA1', u32 flags, u64 length} + payload.
//  * Fault injection for tests: a Push can drop every Nth message or delay each one.
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr uint32_t kMagic = 0x3141534cu;  // "LSA1"
struct FrameHeader {
  uint32_t magic;
  uint32_t flags;
  uint64_t length;
};
static_assert(sizeof(FrameHeader) == 16, "frame header");

constexpr uint64_t kMaxFrame = 1ull << 36;  // 64 GiB sanity bound

using Clock = std::chrono::steady_clock;

struct Message {
  std::string data;
};

// ----------------------------------------------------------------------------- Pull
struct Conn {
  int fd;
  std::string buf;
};

struct Pull {
  int lfd = -1;
  int efd = -1;
  int wake[2] = {-1, -1};
  int port = 0;
  std::string bound_host;
  std::thread th;
  std::atomic<bool> stop{false};
  std::mutex mu;
  std::condition_variable cv;
  std::deque<Message> q;
  std::map<int, Conn> conns;
  uint64_t received = 0;

  ~Pull() { shutdown(); }

  void shutdown() {
    if (stop.exchange(true)) return;
    if (wake[1] >= 0) {
      char c = 1;
      ssize_t r = ::write(wake[1], &c, 1);
      (void)r;
    }
    if (th.joinable()) th.join();
    for (auto& kv : conns) ::close(kv.first);
    conns.clear();
    if (lfd >= 0) ::close(lfd);
    if (efd >= 0) ::close(efd);
    if (wake[0] >= 0) ::close(wake[0]);
    if (wake[1] >= 0) ::close(wake[1]);
    lfd = efd = wake[0] = wake[1] = -1;
    cv.notify_all();
  }

  void drop(int fd) {
    epoll_ctl(efd, EPOLL_CTL_DEL, fd, nullptr);
    ::close(fd);
    conns.erase(fd);
  }

  void on_readable(int fd) {
    auto it = conns.find(fd);
    if (it == conns.end()) return;
    Conn& c = it->second;
    char tmp[1 << 16];
    for (;;) {
      ssize_t n = ::recv(fd, tmp, sizeof(tmp), 0);
      if (n > 0) {
        c.buf.append(tmp, (size_t)n);
        continue;
      }
      if (n == 0) {  // peer closed
        parse(c);
        drop(fd);
        return;
      }
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      if (errno == EINTR) continue;
      drop(fd);
      return;
    }
    parse(c);
  }

  void parse(Conn& c) {
    size_t off = 0;
    std::vector<Message> ready;
    while (c.buf.size() - off >= sizeof(FrameHeader)) {
      FrameHeader h;
      memcpy(&h, c.buf.data() + off, sizeof(h));
      if (h.magic != kMagic || h.length > kMaxFrame) {  // corrupt stream: discard it
        c.buf.clear();
        return;
      }
      if (c.buf.size() - off - sizeof(h) < h.length) break;
      Message m;
      m.data.assign(c.buf.data() + off + sizeof(h), (size_t)h.length);
      ready.push_back(std::move(m));
      off += sizeof(h) + h.length;
    }
    if (off) c.buf.erase(0, off);
    if (!ready.empty()) {
      std::lock_guard<std::mutex> g(mu);
      for (auto& m : ready) q.push_back(std::move(m));
      received += ready.size();
      cv.notify_all();
    }
  }

  void loop() {
    epoll_event evs[64];
    while (!stop.load()) {
      int n = epoll_wait(efd, evs, 64, 200);
      for (int i = 0; i < n; ++i) {
        int fd = evs[i].data.fd;
        if (fd == wake[0]) return;
        if (fd == lfd) {
          for (;;) {
            int cfd = ::accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
            if (cfd < 0) break;
            int one = 1;
            setsockopt(cfd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
            epoll_event ev{};
            ev.events = EPOLLIN | EPOLLRDHUP;
            ev.data.fd = cfd;
            epoll_ctl(efd, EPOLL_CTL_ADD, cfd, &ev);
            conns[cfd] = Conn{cfd, {}};
          }
        } else {
          on_readable(fd);
        }
      }
    }
  }
};

// ----------------------------------------------------------------------------- Push
struct Push {
  std::string host;
  int port = 0;
  std::atomic<int> fd{-1};  // written by the writer thread, read by lsa_push_connected (TSan)
  std::thread th;
  std::atomic<bool> stop{false};
  std::mutex mu;
  std::condition_variable cv;       // queue non-empty / stop
  std::condition_variable drained;  // queue empty
  std::deque<std::string> q;        // framed messages
  uint64_t sent = 0, enqueued = 0;
  // fault injection (set from the caller's thread while the writer runs)
  std::atomic<int> drop_every{0};
  std::atomic<int> delay_ms{0};
  uint64_t attempt = 0;  // writer thread only

  ~Push() { shutdown(); }

  void shutdown() {
    {
      std::lock_guard<std::mutex> g(mu);
      if (stop.exchange(true)) return;
    }
    cv.notify_all();
    if (th.joinable()) th.join();
    if (fd >= 0) ::close(fd);
    fd = -1;
    drained.notify_all();
  }

  bool try_connect() {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    const std::string p = std::to_string(port);
    if (getaddrinfo(host.c_str(), p.c_str(), &hints, &res) != 0 || !res) return false;
    int s = ::socket(res->ai_family, res->ai_socktype | SOCK_CLOEXEC, res->ai_protocol);
    if (s < 0) {
      freeaddrinfo(res);
      return false;
    }
    int rc = ::connect(s, res->ai_addr, res->ai_addrlen);
    freeaddrinfo(res);
    if (rc != 0) {
      ::close(s);
      return false;
    }
    int one = 1;
    setsockopt(s, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    fd = s;
    return true;
  }

  bool write_all(const std::string& m) {
    size_t off = 0;
    while (off < m.size()) {
      ssize_t n = ::send(fd, m.data() + off, m.size() - off, MSG_NOSIGNAL);
      if (n > 0) {
        off += (size_t)n;
        continue;
      }
      if (n < 0 && errno == EINTR) continue;
      return false;
    }
    return true;
  }

  void loop() {
    int backoff_ms = 5;
    for (;;) {
      std::string msg;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop.load() || !q.empty(); });
        if (stop.load() && q.empty()) return;
        if (stop.load()) return;  // pending messages are abandoned on explicit close
        msg = q.front();
      }
      if (fd < 0 && !try_connect()) {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait_for(lk, std::chrono::milliseconds(backoff_ms), [&] { return stop.load(); });
        backoff_ms = backoff_ms < 200 ? backoff_ms * 2 : 200;
        continue;
      }
      backoff_ms = 5;
      ++attempt;
      const int dly = delay_ms.load(), every = drop_every.load();
      if (dly > 0) std::this_thread::sleep_for(std::chrono::milliseconds(dly));
      const bool dropped = every > 0 && (attempt % (uint64_t)every) == 0;
      if (!dropped && !write_all(msg)) {  // peer went away: reconnect and resend
        ::close(fd);
        fd = -1;
        continue;
      }
      std::lock_guard<std::mutex> g(mu);
      q.pop_front();
      ++sent;
      if (q.empty()) drained.notify_all();
    }
  }
};

bool parse_bind_host(const char* host, in_addr* out) {
  if (!host || !*host || strcmp(host, "*") == 0 || strcmp(host, "0.0.0.0") == 0) {
    out->s_addr = htonl(INADDR_ANY);
    return true;
  }
  if (inet_pton(AF_INET, host, out) == 1) return true;
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  if (getaddrinfo(host, nullptr, &hints, &res) != 0 || !res) return false;
  *out = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
  freeaddrinfo(res);
  return true;
}

}  // namespace

extern "C" {

// Returns a handle or nullptr; *out_port receives the bound port (port 0 = ephemeral).
void* lsa_pull_bind(const char* host, int port, int* out_port) {
  in_addr addr{};
  if (!parse_bind_host(host, &addr)) return nullptr;
  int s = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (s < 0) return nullptr;
  int one = 1;
  setsockopt(s, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_addr = addr;
  sa.sin_port = htons((uint16_t)port);
  if (::bind(s, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) != 0 || ::listen(s, 128) != 0) {
    ::close(s);
    return nullptr;
  }
  socklen_t sl = sizeof(sa);
  getsockname(s, reinterpret_cast<sockaddr*>(&sa), &sl);
  auto* p = new Pull();
  p->lfd = s;
  p->port = ntohs(sa.sin_port);
  p->bound_host = host ? host : "*";
  p->efd = epoll_create1(EPOLL_CLOEXEC);
  if (pipe2(p->wake, O_CLOEXEC | O_NONBLOCK) != 0) {
    delete p;
    return nullptr;
  }
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = s;
  epoll_ctl(p->efd, EPOLL_CTL_ADD, s, &ev);
  ev.data.fd = p->wake[0];
  epoll_ctl(p->efd, EPOLL_CTL_ADD, p->wake[0], &ev);
  p->th = std::thread([p] { p->loop(); });
  if (out_port) *out_port = p->port;
  return p;
}

// Wait up to timeout_ms (0 = poll, <0 = forever) for a message. Returns its size, or -1 on
// timeout, -2 if closed. The message stays at the queue head until lsa_pull_take.
long long lsa_pull_wait(void* h, int timeout_ms) {
  auto* p = static_cast<Pull*>(h);
  std::unique_lock<std::mutex> lk(p->mu);
  auto ready = [&] { return !p->q.empty() || p->stop.load(); };
  if (timeout_ms < 0)
    p->cv.wait(lk, ready);
  else if (timeout_ms > 0)
    p->cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), ready);
  if (!p->q.empty()) return (long long)p->q.front().data.size();
  return p->stop.load() ? -2 : -1;
}

// Copy the head message into buf (capacity cap) and pop it. Returns bytes copied or -1.
long long lsa_pull_take(void* h, void* buf, long long cap) {
  auto* p = static_cast<Pull*>(h);
  std::lock_guard<std::mutex> g(p->mu);
  if (p->q.empty()) return -1;
  Message& m = p->q.front();
  if ((long long)m.data.size() > cap) return -1;
  memcpy(buf, m.data.data(), m.data.size());
  long long n = (long long)m.data.size();
  p->q.pop_front();
  return n;
}

int lsa_pull_port(void* h) { return static_cast<Pull*>(h)->port; }
long long lsa_pull_received(void* h) {
  auto* p = static_cast<Pull*>(h);
  std::lock_guard<std::mutex> g(p->mu);
  return (long long)p->received;
}
void lsa_pull_close(void* h) { delete static_cast<Pull*>(h); }

void* lsa_push_connect(const char* host, int port) {
  auto* p = new Push();
  p->host = host;
  p->port = port;
  p->th = std::thread([p] { p->loop(); });
  return p;
}

int lsa_push_send(void* h, const void* data, long long n) {
  auto* p = static_cast<Push*>(h);
  if (n < 0) return -1;
  FrameHeader hd{kMagic, 0u, (uint64_t)n};
  std::string m;
  m.resize(sizeof(hd) + (size_t)n);
  memcpy(&m[0], &hd, sizeof(hd));
  if (n) memcpy(&m[sizeof(hd)], data, (size_t)n);
  {
    std::lock_guard<std::mutex> g(p->mu);
    if (p->stop.load()) return -2;
    p->q.push_back(std::move(m));
    ++p->enqueued;
  }
  p->cv.notify_all();
  return 0;
}

// Wait until every queued message has been written. Returns 0, or -1 on timeout.
int lsa_push_flush(void* h, int timeout_ms) {
  auto* p = static_cast<Push*>(h);
  std::unique_lock<std::mutex> lk(p->mu);
  auto done = [&] { return p->q.empty() || p->stop.load(); };
  if (timeout_ms < 0) {
    p->drained.wait(lk, done);
    return p->q.empty() ? 0 : -1;
  }
  return p->drained.wait_for(lk, std::chrono::milliseconds(timeout_ms), done) && p->q.empty() ? 0 : -1;
}

long long lsa_push_pending(void* h) {
  auto* p = static_cast<Push*>(h);
  std::lock_guard<std::mutex> g(p->mu);
  return (long long)p->q.size();
}

int lsa_push_connected(void* h) { return static_cast<Push*>(h)->fd >= 0 ? 1 : 0; }

void lsa_push_fault(void* h, int drop_every, int delay_ms) {
  auto* p = static_cast<Push*>(h);
  p->drop_every = drop_every;
  p->delay_ms = delay_ms;
}

void lsa_push_close(void* h) { delete static_cast<Push*>(h); }

}  // extern "C"

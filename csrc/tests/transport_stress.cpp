// Host-side stress test for the TCP transport (csrc/comm/tcp_transport.cpp), built and run
// under AddressSanitizer+UBSan and ThreadSanitizer by tests/test_sanitizers.py (SURVEY.md
// §5.2: the reference has no race detection; its known races are the shared temp files of
// Q5 and unsynchronised re-config). Exercises: many concurrent pushers into one pull, frame
// integrity and per-sender ordering, fault injection (drop every Nth), a push that starts
// before its peer binds (reconnect with back-off), status queries racing the writer thread,
// and tearing a pull down while senders are still writing.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

extern "C" {
void* lsa_pull_bind(const char* host, int port, int* out_port);
long long lsa_pull_wait(void* h, int timeout_ms);
long long lsa_pull_take(void* h, void* buf, long long cap);
long long lsa_pull_received(void* h);
void lsa_pull_close(void* h);
void* lsa_push_connect(const char* host, int port);
int lsa_push_send(void* h, const void* data, long long n);
int lsa_push_flush(void* h, int timeout_ms);
long long lsa_push_pending(void* h);
int lsa_push_connected(void* h);
void lsa_push_fault(void* h, int drop_every, int delay_ms);
void lsa_push_close(void* h);
}

#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(2);                                                       \
    }                                                                     \
  } while (0)

namespace {

std::string payload(int sender, int seq) {
  // deterministic size 0..64 KiB and byte pattern per (sender, seq)
  const size_t n = 8 + (size_t)((sender * 7919 + seq * 104729) % 65536);
  std::string s(n, '\0');
  std::memcpy(&s[0], &sender, 4);
  std::memcpy(&s[4], &seq, 4);
  for (size_t i = 8; i < n; ++i) s[i] = (char)((sender + seq + i) & 0xff);
  return s;
}

bool recv_one(void* pull, std::string& out, int timeout_ms) {
  const long long n = lsa_pull_wait(pull, timeout_ms);
  if (n < 0) return false;
  out.resize((size_t)n);
  return lsa_pull_take(pull, n ? &out[0] : nullptr, n) == n;
}

void concurrent_pushers() {
  int port = 0;
  void* pull = lsa_pull_bind("127.0.0.1", 0, &port);
  CHECK(pull && port > 0);
  constexpr int kSenders = 4, kMsgs = 400;
  std::atomic<bool> stop_poll{false};
  std::vector<void*> pushes(kSenders);
  for (int s = 0; s < kSenders; ++s) pushes[s] = lsa_push_connect("127.0.0.1", port);
  // status queries racing the writer threads
  std::thread poller([&] {
    while (!stop_poll.load()) {
      for (void* p : pushes) {
        (void)lsa_push_connected(p);
        (void)lsa_push_pending(p);
      }
      (void)lsa_pull_received(pull);
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
  });
  std::vector<std::thread> th;
  for (int s = 0; s < kSenders; ++s)
    th.emplace_back([&, s] {
      for (int i = 0; i < kMsgs; ++i) {
        const std::string m = payload(s, i);
        CHECK(lsa_push_send(pushes[s], m.data(), (long long)m.size()) == 0);
      }
      CHECK(lsa_push_flush(pushes[s], 30000) == 0);
    });
  std::vector<int> next(kSenders, 0);
  std::string got;
  for (int k = 0; k < kSenders * kMsgs; ++k) {
    CHECK(recv_one(pull, got, 30000));
    int s, i;
    CHECK(got.size() >= 8);
    std::memcpy(&s, &got[0], 4);
    std::memcpy(&i, &got[4], 4);
    CHECK(s >= 0 && s < kSenders);
    CHECK(i == next[s]);  // per-sender FIFO
    CHECK(got == payload(s, i));
    ++next[s];
  }
  for (auto& t : th) t.join();
  stop_poll = true;
  poller.join();
  for (void* p : pushes) lsa_push_close(p);
  CHECK(lsa_pull_wait(pull, 0) == -1);  // nothing extra
  lsa_pull_close(pull);
}

void fault_injection() {
  int port = 0;
  void* pull = lsa_pull_bind("127.0.0.1", 0, &port);
  void* push = lsa_push_connect("127.0.0.1", port);
  lsa_push_fault(push, 3, 0);  // drop every 3rd message
  for (int i = 0; i < 30; ++i) {
    const std::string m = payload(9, i);
    CHECK(lsa_push_send(push, m.data(), (long long)m.size()) == 0);
  }
  CHECK(lsa_push_flush(push, 30000) == 0);
  std::string got;
  int n = 0;
  while (recv_one(pull, got, 500)) ++n;
  CHECK(n == 20);
  lsa_push_close(push);
  lsa_pull_close(pull);
}

void late_bind() {
  int port = 0;
  void* probe = lsa_pull_bind("127.0.0.1", 0, &port);
  lsa_pull_close(probe);  // the port is free again
  void* push = lsa_push_connect("127.0.0.1", port);
  for (int i = 0; i < 10; ++i) {
    const std::string m = payload(3, i);
    CHECK(lsa_push_send(push, m.data(), (long long)m.size()) == 0);
  }
  std::this_thread::sleep_for(std::chrono::milliseconds(100));
  int port2 = 0;
  void* pull = lsa_pull_bind("127.0.0.1", port, &port2);
  CHECK(pull && port2 == port);
  std::string got;
  for (int i = 0; i < 10; ++i) {
    CHECK(recv_one(pull, got, 30000));
    CHECK(got == payload(3, i));
  }
  lsa_push_close(push);
  lsa_pull_close(pull);
}

void teardown_while_sending() {
  int port = 0;
  void* pull = lsa_pull_bind("127.0.0.1", 0, &port);
  std::vector<void*> pushes;
  for (int s = 0; s < 3; ++s) pushes.push_back(lsa_push_connect("127.0.0.1", port));
  std::atomic<bool> go{true};
  std::vector<std::thread> th;
  for (int s = 0; s < 3; ++s)
    th.emplace_back([&, s] {
      int i = 0;
      while (go.load()) {
        const std::string m = payload(s, i++ % 64);
        if (lsa_push_send(pushes[s], m.data(), (long long)m.size()) != 0) break;
        if (i % 64 == 0) std::this_thread::sleep_for(std::chrono::microseconds(50));
      }
    });
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  lsa_pull_close(pull);  // peers see the connection drop and keep retrying
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  go = false;
  for (auto& t : th) t.join();
  for (void* p : pushes) lsa_push_close(p);
}

}  // namespace

int main() {
  concurrent_pushers();
  fault_injection();
  late_bind();
  teardown_while_sending();
  std::printf("transport stress OK\n");
  return 0;
}

// Host-code sanitizer run (AddressSanitizer + UndefinedBehaviorSanitizer) over the native
// runtime that runs on the CPU: the store (WAL append / replay / compaction), the
// persistence worker (group-commit coalescing), the AMQP codec (fuzzed frames), the host
// broker + native load generator over loopback TCP, the pipelined front end driven by the
// in-process echo engine (echo traffic, connections closed mid-stream), and the sharded
// front end: two ranks stepping in lockstep over the shared-memory exchange.  Built and run by scripts/host_sanitize.sh; any report
// aborts with a non-zero exit (halt_on_error).
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <memory>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../core/broker.hpp"
#include "../core/codec.hpp"
#include "../core/frontend.hpp"
#include "../core/loadgen.hpp"
#include "../core/persist.hpp"
#include "../core/store.hpp"

using namespace cmq;

static void check(bool ok, const char* what) {
  if (!ok) {
    fprintf(stderr, "FAILED: %s\n", what);
    exit(2);
  }
}

static void store_roundtrip(const std::string& dir) {
  {
    Store st;
    st.open(dir, false);
    st.insertQueueMeta("v-_.q", -1, {}, true, 0);
    for (int i = 0; i < 2000; ++i) {
      MsgRow m;
      m.id = 1000 + i; m.tstamp = i; m.header = std::string(10, '\0') + "p"; m.body = std::string(37 + i % 300, 'b');
      m.exchange = "x"; m.routing = "k"; m.durable = true; m.refer = 1;
      if (i & 1) st.insertMessage(std::move(m), 0);
      else st.insertMessage(m, 0);
      st.insertQueueMsg("v-_.q", i, 1000 + i, 40, 0);
      if (i % 3 == 0) { st.insertQueueUnack("v-_.q", i, 1000 + i, 40); st.deleteQueueMsg("v-_.q", i); }
      if (i % 5 == 0) {
        if (i % 3 == 0) st.deleteQueueUnack("v-_.q", 1000 + i); else st.deleteQueueMsg("v-_.q", i);
        st.deleteMessage(1000 + i);
      }
    }
    st.sync();
    st.compact();
    st.close();
  }
  Store st;
  st.open(dir, false);   // replay
  QueueMetaRow meta;
  std::vector<QueueMsgRow> msgs, unacks;
  check(st.selectQueue("v-_.q", &meta, &msgs, &unacks), "queue replayed");
  check(msgs.size() + unacks.size() == 1600, "rows replayed");
  MsgRow r;
  check(st.selectMessage(1001, &r) && r.body.size() == 38, "message replayed");
  st.close();
}

static std::string persist_rec(i64 id, u32 q, u64 pos, const std::string& body) {
  PersistHdr h{};
  h.msg_id = id; h.q = q; h.qpos = pos; h.body_len = (u32)body.size(); h.props_len = 3; h.ex_len = 1; h.rk_len = 1;
  std::string pay = std::string("xk") + "\x10\x00\x02" + body;
  h.size = (u32)(sizeof h + ((pay.size() + 7) & ~size_t(7)));
  std::string out((const char*)&h, sizeof h);
  out += pay;
  out.resize(h.size, '\0');
  return out;
}

static std::string consumed_rec(i64 id, u32 q, u64 pos, u32 kind) {
  ConsumedRec r{};
  r.msg_id = id; r.q = q; r.qpos = pos; r.kind = kind;
  return std::string((const char*)&r, sizeof r);
}

static void persist_worker(const std::string& dir) {
  Store st;
  st.open(dir, false);
  PersistWorker w(&st);
  w.set_queue(0, "v-_.a");
  w.set_queue(1, "v-_.b");
  w.start();
  i64 id = 1;
  std::vector<std::pair<i64, u32>> live;
  for (int step = 0; step < 300; ++step) {
    std::string p, c;
    for (int k = 0; k < 20; ++k, ++id) {
      p += persist_rec(id, (u32)(id & 1), (u64)id, std::string(100 + (id % 50), 'm'));
      live.push_back({id, (u32)(id & 1)});
    }
    // deliver + ack / requeue some of the older ones (some in the same group as their publish)
    for (size_t k = 0; k < live.size() && k < 15; ++k) {
      c += consumed_rec(live[k].first, live[k].second, (u64)live[k].first, 3);
      c += consumed_rec(live[k].first, live[k].second, (u64)live[k].first, (k % 4 == 0) ? 4 : 0);
    }
    live.erase(live.begin(), live.begin() + std::min<size_t>(live.size(), 15));
    w.submit((u64)step + 1, std::move(p), std::move(c));
    if (step % 7 == 0) w.drain();
  }
  w.drain();
  w.set_queue(1, "");   // slot freed: its rows go
  w.stop();
  st.close();
}

static void codec_fuzz() {
  std::mt19937 rng(7);
  int parsed = 0;
  for (int it = 0; it < 20000; ++it) {
    std::string b(8 + rng() % 200, '\0');
    for (auto& ch : b) ch = (char)(rng() & 0xff);
    b[0] = 1;
    u32 n = (u32)b.size() - 8;
    b[3] = (char)(n >> 24); b[4] = (char)(n >> 16); b[5] = (char)(n >> 8); b[6] = (char)n;
    b[7] = 0; b[8] = 60; b[9] = 0; b[10] = (char)(10 * (1 + rng() % 12));
    b.back() = (char)0xCE;
    try {
      Method m = decode_method((const u8*)b.data() + 7, n);
      (void)m;
      ++parsed;
    } catch (const std::exception&) {
    }
  }
  fprintf(stderr, "codec fuzz: %d of 20000 random frames decoded\n", parsed);
}

static void broker_and_loadgen(const std::string& dir) {
  BrokerConfig cfg;
  cfg.host = "127.0.0.1";
  cfg.port = 0;
  cfg.heartbeat = 0;
  cfg.data_dir = dir;
  cfg.fsync = false;
  auto bp = std::make_unique<Broker>(cfg);
  Broker& b = *bp;
  b.start();
  for (bool ack : {true, false}) {
    LoadSpec s;
    s.port = b.listen_port();
    s.producers = 2; s.consumers = 2; s.msg_size = 64; s.seconds = 0.7; s.auto_ack = ack; s.prefetch = 200;
    s.queue = ack ? "sq.a" : "sq.m"; s.exchange = ack ? "sx.a" : "sx.m";
    s.persistent = !ack; s.durable = !ack; s.confirm = !ack;
    LoadResult r = run_load(s);
    check(r.error.empty(), "loadgen run");
    check(r.received > 0, "messages received");
    fprintf(stderr, "broker+loadgen %s: sent %llu received %llu\n", ack ? "auto-ack" : "manual/persistent",
            r.sent, r.received);
  }
  b.stop();
}

static void frontend_echo() {
  EchoEngine eng(64, 64, 1 << 20, 1 << 16);
  FrontendCfg cfg;
  cfg.host = "127.0.0.1";
  cfg.port = 0;
  cfg.io_threads = 2;
  cfg.idle_step_ms = 1.0;
  cfg.per_conn_read = 4096;
  // heap objects: std::mutex members are statically initialised (no pthread_mutex_init),
  // so a mutex on stack memory an earlier object's destroyed mutex used looks like that
  // destroyed mutex to ThreadSanitizer
  auto fp = std::make_unique<Frontend>(cfg, (const CmqEngineApi*)eng.c_api());
  Frontend& f = *fp;
  f.start();
  // traffic through the IO threads and the stepper: each client is opened (FE_OPEN),
  // switched to data mode after its first bytes (FE_HOST), then streams a payload larger
  // than a step's per-connection read and reads its echo back; then half the clients close
  // mid-stream while the rest finish (slot reuse, held egress of closed connections)
  const int NC = 6;
  std::vector<int> fds;
  std::vector<u32> ids;
  std::vector<FeEvent> seen;   // events polled but not yet waited for
  auto wait_event = [&](int kind, int64_t conn) -> FeEvent {
    for (int tries = 0; tries < 400; ++tries) {
      for (size_t k = 0; k < seen.size(); ++k)
        if (seen[k].kind == kind && (conn < 0 || seen[k].conn == (u32)conn)) {
          FeEvent e = seen[k];
          seen.erase(seen.begin() + (long)k);
          return e;
        }
      for (FeEvent& e : f.poll_events(25)) seen.push_back(e);
    }
    check(false, "front end event");
    return FeEvent{};
  };
  for (int i = 0; i < NC; ++i) {
    int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)f.port());
    inet_pton(AF_INET, "127.0.0.1", &a.sin_addr);
    check(::connect(fd, (sockaddr*)&a, sizeof a) == 0, "front end connect");
    fds.push_back(fd);
    ids.push_back(wait_event(FE_OPEN, -1).conn);
  }
  std::string payload(20000, '\0');
  for (size_t k = 0; k < payload.size(); ++k) payload[k] = (char)(k * 7 + 3);
  for (int i = 0; i < NC; ++i) {
    check(::send(fds[i], "HI", 2, 0) == 2, "send hello");
    wait_event(FE_HOST, ids[i]);
    (void)f.take(ids[i]);
    f.set_data_mode(ids[i], "");
  }
  for (int i = 0; i < NC; ++i) check(::send(fds[i], payload.data(), payload.size(), 0) == (ssize_t)payload.size(), "send payload");
  for (int i = 0; i < NC; ++i) {
    if (i % 2) { ::close(fds[i]); fds[i] = -1; continue; }   // closed while its echo is in flight
    std::string got;
    timeval tv{5, 0};
    setsockopt(fds[i], SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    char buf[8192];
    while (got.size() < payload.size()) {
      ssize_t n = ::recv(fds[i], buf, sizeof buf, 0);
      if (n <= 0) break;
      got.append(buf, (size_t)n);
    }
    check(got == payload, "front end echo");
  }
  for (int i = 1; i < NC; i += 2) {
    wait_event(FE_CLOSED, ids[i]);
    f.close(ids[i]);
  }
  fprintf(stderr, "front end echo: %d clients, %llu steps\n", NC, (unsigned long long)f.stats().steps);
  f.stop();
  for (int fd : fds)
    if (fd >= 0) ::close(fd);
}

// the sharded front end: two ranks (EchoEngine world 2 + Frontend each) in this process,
// stepping in lockstep over the shared-memory exchange (xchg_host.h): local echo on each
// rank, then bytes after "XR1" shipped from rank 0's connection to rank 1's
static int connect_to(int port) {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  inet_pton(AF_INET, "127.0.0.1", &a.sin_addr);
  check(::connect(fd, (sockaddr*)&a, sizeof a) == 0, "sharded front end connect");
  timeval tv{5, 0};
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  return fd;
}
static bool read_until(int fd, const std::string& token) {
  std::string got;
  char buf[4096];
  while (got.find(token) == std::string::npos) {
    ssize_t n = ::recv(fd, buf, sizeof buf, 0);
    if (n <= 0) return false;
    got.append(buf, (size_t)n);
  }
  return true;
}

static void frontend_sharded(bool async_x) {
  const std::string name = "cmq-sanitize-" + std::to_string(::getpid()) + (async_x ? "-a" : "-s");
  std::unique_ptr<EchoEngine> eng[2];
  for (u32 r = 0; r < 2; ++r) eng[r] = std::make_unique<EchoEngine>(64, 64, 1 << 20, 1 << 16, 2, r);
  {
    std::thread t0([&] { eng[0]->xchg_setup(name, {0, 1}, 2000, async_x); });
    std::thread t1([&] { eng[1]->xchg_setup(name, {0, 1}, 2000, async_x); });
    t0.join();
    t1.join();
  }
  FrontendCfg cfg;
  cfg.host = "127.0.0.1";
  cfg.port = 0;
  cfg.io_threads = 2;
  cfg.idle_step_ms = 1.0;
  cfg.per_conn_read = 4096;
  std::unique_ptr<Frontend> fe[2];
  for (int r = 0; r < 2; ++r) {
    fe[r] = std::make_unique<Frontend>(cfg, (const CmqEngineApi*)eng[r]->c_api());
    fe[r]->start();
  }
  std::atomic<bool> stop{false};
  std::thread ctl[2];
  for (int r = 0; r < 2; ++r)
    ctl[r] = std::thread([&, r] {   // control plane: data mode on open, slot freed on close
      while (!stop.load())
        for (FeEvent& e : fe[r]->poll_events(20)) {
          if (e.kind == FE_OPEN) fe[r]->set_data_mode(e.conn, "");
          else if (e.kind == FE_CLOSED) fe[r]->close(e.conn);
        }
    });
  int c0 = connect_to(fe[0]->port()), c1 = connect_to(fe[1]->port());
  std::this_thread::sleep_for(std::chrono::milliseconds(200));
  check(::send(c0, "hello0", 6, 0) == 6 && read_until(c0, "hello0"), "sharded local echo");
  check(::send(c0, "abcXR1world", 11, 0) == 11, "sharded cross-rank send");
  check(read_until(c0, "abc") && read_until(c1, "world"), "sharded cross-rank delivery");
  std::string big(12000, 'x');
  check(::send(c1, big.data(), big.size(), 0) == (ssize_t)big.size() && read_until(c1, std::string(64, 'x')),
        "sharded echo over steps");
  ::close(c0);
  ::close(c1);
  std::this_thread::sleep_for(std::chrono::milliseconds(100));
  stop = true;
  for (auto& t : ctl) t.join();
  const FeStats s0 = fe[0]->stats();
  {   // both ranks stop together (a rank alone would wait out the exchange timeout)
    std::thread t0([&] { fe[0]->stop(); });
    std::thread t1([&] { fe[1]->stop(); });
    t0.join();
    t1.join();
  }
  fprintf(stderr, "sharded front end (%s exchange): %llu steps, %llu exchanges, imported %llu\n",
          async_x ? "asynchronous" : "synchronous", (unsigned long long)s0.steps, (unsigned long long)s0.xchg_steps,
          (unsigned long long)eng[1]->imported);
}

int main(int argc, char** argv) {
  std::string dir = argc > 1 ? argv[1] : "/tmp/cmq-sanitize";
  ::mkdir(dir.c_str(), 0755);
  store_roundtrip(dir + "/store");
  persist_worker(dir + "/persist");
  codec_fuzz();
  broker_and_loadgen(dir + "/broker");
  frontend_echo();
  frontend_sharded(false);
  frontend_sharded(true);
  fprintf(stderr, "host sanitizer run: ok\n");
  return 0;
}

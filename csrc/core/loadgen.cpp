// Native AMQP load generator: the RabbitMQ PerfTest(Multi) shapes of
// chana-mq-test/perf/publish-consume-spec*.js (producer/consumer counts, minMsgSize,
// auto-ack, channel-prefetch, persistent, time-limit), run against any AMQP 0-9-1 broker.
// Producers stamp a steady-clock send time into the first 8 body bytes; consumers
// histogram publish->deliver latency.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <string>
#include <mutex>
#include <thread>
#include <vector>

#include "codec.hpp"
#include "loadgen.hpp"

namespace cmq {

static i64 mono_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

namespace {

struct Client {
  int fd = -1;
  std::string in;
  size_t pos = 0;
  FrameParser parser;
  u32 frame_max = 131072;
  std::string out;

  bool connect_to(const std::string& host, int port) {
    fd = ::socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    inet_pton(AF_INET, host.c_str(), &a.sin_addr);
    if (::connect(fd, (sockaddr*)&a, sizeof a) < 0) return false;
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    int big = 4 << 20;
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &big, sizeof big);
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &big, sizeof big);
    return true;
  }
  void send_all(const std::string& s) {
    size_t o = 0;
    while (o < s.size()) {
      ssize_t k = ::send(fd, s.data() + o, s.size() - o, MSG_NOSIGNAL);
      if (k <= 0) throw std::runtime_error("loadgen: send failed");
      o += (size_t)k;
    }
  }
  void flush() { if (!out.empty()) { send_all(out); out.clear(); } }
  void method(u16 ch, const Method& m) { append_method_frame(out, ch, m); }
  // read one frame (blocking)
  bool frame(Frame& f, int timeout_ms = 10000) {
    while (!parser.next(in, pos, f)) {
      if (pos > (1u << 20)) { in.erase(0, pos); pos = 0; }
      char buf[1 << 16];
      timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
      setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
      ssize_t k = ::recv(fd, buf, sizeof buf, 0);
      if (k <= 0) return false;
      in.append(buf, (size_t)k);
    }
    return true;
  }
  Method expect(u16 cls, u16 mid) {
    Frame f;
    while (frame(f)) {
      if (f.type != FRAME_METHOD) continue;
      Method m = decode_method((const u8*)f.payload.data(), f.payload.size());
      if (m.cls() == cls && m.mid() == mid) return m;
      if (m.cls() == 10 && m.mid() == 50) throw std::runtime_error("loadgen: connection closed: " + m.s(1));
      if (m.cls() == 20 && m.mid() == 40) throw std::runtime_error("loadgen: channel closed: " + m.s(1));
    }
    throw std::runtime_error("loadgen: timeout waiting for reply");
  }
  void open(const std::string& host, int port, const std::string& vhost) {
    if (!connect_to(host, port)) throw std::runtime_error("loadgen: cannot connect");
    send_all(std::string(PROTOCOL_HEADER, 8));
    expect(10, 10);
    Method so = make_method(10, 11);
    so.args[0].t = {{"product", Value::str("chanamq-loadgen")}};
    so.args[1].s = "PLAIN";
    so.args[2].s = std::string("\0guest\0guest", 12);
    so.args[3].s = "en_US";
    method(0, so);
    flush();
    Method tune = expect(10, 30);
    frame_max = tune.i(1) ? (u32)tune.i(1) : 131072;
    parser.set_frame_max(0);
    Method to = make_method(10, 31);
    to.args[0].i = 2047;
    to.args[1].i = frame_max;
    to.args[2].i = 0;
    method(0, to);
    Method op = make_method(10, 40);
    op.args[0].s = vhost;
    method(0, op);
    flush();
    expect(10, 41);
    Method co = make_method(20, 10);
    method(1, co);
    flush();
    expect(20, 11);
  }
  void close() { if (fd >= 0) { ::close(fd); fd = -1; } }
};

struct Hist {   // log2-spaced microsecond buckets with 8 sub-buckets each
  std::vector<u64> b = std::vector<u64>(64 * 8, 0);
  u64 n = 0;
  void add(double us) {
    if (us < 1) us = 1;
    double l = std::log2(us);
    int e = (int)l;
    int sub = (int)((l - e) * 8);
    size_t i = std::min<size_t>(b.size() - 1, (size_t)(e * 8 + sub));
    ++b[i];
    ++n;
  }
  void merge(const Hist& o) { for (size_t i = 0; i < b.size(); ++i) b[i] += o.b[i]; n += o.n; }
  double q(double p) const {
    if (!n) return 0;
    u64 want = (u64)std::ceil(p * n), acc = 0;
    for (size_t i = 0; i < b.size(); ++i) {
      acc += b[i];
      if (acc >= want) return std::pow(2.0, (double)i / 8.0);
    }
    return 0;
  }
};

}  // namespace

LoadResult run_load(const LoadSpec& s) {
  LoadResult r;
  {   // topology
    Client a;
    a.open(s.host, s.port, s.vhost);
    if (!s.exchange.empty()) {
      Method x = make_method(40, 10);
      x.args[1].s = s.exchange;
      x.args[2].s = s.exchange_type;
      x.args[4].i = s.durable;
      a.method(1, x);
      a.flush();
      a.expect(40, 11);
    }
    for (int qi = 0; qi < std::max(1, s.queues); ++qi) {
      std::string qn = s.queues > 1 ? s.queue + "." + std::to_string(qi) : s.queue;
      Method q = make_method(50, 10);
      q.args[1].s = qn;
      q.args[3].i = s.durable;
      a.method(1, q);
      Method pg = make_method(50, 30);   // start from an empty queue
      pg.args[1].s = qn;
      a.method(1, pg);
      a.flush();
      a.expect(50, 11);
      a.expect(50, 31);
      if (!s.exchange.empty()) {
        Method b = make_method(50, 20);
        b.args[1].s = qn;
        b.args[2].s = s.exchange;
        b.args[3].s = s.exchange_type == "fanout" ? "" : (s.queues > 1 ? s.routing_key + "." + std::to_string(qi) : s.routing_key);
        if (s.exchange_type == "topic" && s.queues > 1) b.args[3].s = s.routing_key + "." + std::to_string(qi) + ".*";
        a.method(1, b);
        a.flush();
        a.expect(50, 21);
      }
    }
    a.close();
  }
  std::atomic<bool> stop{false};
  std::atomic<int> ready{0};
  std::vector<std::thread> th;
  std::vector<u64> sent(s.producers, 0), recv(s.consumers, 0), confirmed(s.producers, 0);
  std::vector<Hist> hists(s.consumers);
  std::string err;
  std::mutex err_mu;
  auto fail = [&](const std::exception& e) { std::lock_guard<std::mutex> g(err_mu); if (err.empty()) err = e.what(); stop = true; };

  for (int ci = 0; ci < s.consumers; ++ci) {
    th.emplace_back([&, ci] {
      try {
        Client c;
        c.open(s.host, s.port, s.vhost);
        Method qos = make_method(60, 10);
        qos.args[1].i = s.prefetch;
        c.method(1, qos);
        c.flush();
        c.expect(60, 11);
        int nq = std::max(1, s.queues);
        std::string qn = s.queues > 1 ? s.queue + "." + std::to_string(ci % nq) : s.queue;
        Method cm = make_method(60, 20);
        cm.args[1].s = qn;
        cm.args[2].s = "lg-" + std::to_string(ci);
        cm.args[4].i = s.auto_ack;
        c.method(1, cm);
        c.flush();
        c.expect(60, 21);
        ++ready;
        Frame f;
        u64 unacked = 0, last_tag = 0;
        bool want_body = false;
        u64 body_left = 0;
        std::string body;
        while (!stop) {
          if (!c.frame(f, 200)) continue;
          if (f.type == FRAME_METHOD) {
            const u8* p = (const u8*)f.payload.data();
            u16 cls = (u16(p[0]) << 8) | p[1], mid = (u16(p[2]) << 8) | p[3];
            if (cls == 60 && mid == 60) {
              Method m = decode_method(p, f.payload.size());
              last_tag = (u64)m.i(1);
              want_body = true;
            }
          } else if (f.type == FRAME_HEADER && want_body) {
            const u8* p = (const u8*)f.payload.data();
            body_left = 0;
            for (int i = 0; i < 8; ++i) body_left = (body_left << 8) | p[4 + i];
            body.clear();
            if (body_left == 0) { want_body = false; ++recv[ci]; ++unacked; }
          } else if (f.type == FRAME_BODY && want_body) {
            if (body.size() < 8) body.append(f.payload, 0, std::min<size_t>(8 - body.size(), f.payload.size()));
            body_left -= f.payload.size();
            if (body_left == 0) {
              want_body = false;
              ++recv[ci];
              ++unacked;
              if (body.size() >= 8) {
                i64 t0;
                memcpy(&t0, body.data(), 8);
                hists[ci].add((mono_ns() - t0) / 1000.0);
              }
            }
          }
          if (!s.auto_ack && unacked && (unacked >= (u64)std::max(1, s.prefetch / 2) || c.pos == c.in.size())) {
            Method ak = make_method(60, 80);
            ak.args[0].i = (i64)last_tag;
            ak.args[1].i = 1;
            c.method(1, ak);
            c.flush();
            unacked = 0;
          }
        }
        c.close();
      } catch (std::exception& e) { fail(e); }
    });
  }
  for (int i = 0; i < 500 && ready < s.consumers && !stop; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(10));
  i64 t_start = mono_ns();
  for (int pi = 0; pi < s.producers; ++pi) {
    th.emplace_back([&, pi] {
      try {
        Client c;
        c.open(s.host, s.port, s.vhost);
        if (s.confirm) {
          c.method(1, make_method(85, 10));
          c.flush();
          c.expect(85, 11);
        }
        std::string props = encode_props_simple(s.persistent ? 2 : 1);
        std::string body(std::max(s.msg_size, 0), 'x');
        int nq = std::max(1, s.queues);
        u64 seq = 0;
        std::string x = s.exchange;
        while (!stop) {
          for (int k = 0; k < 64; ++k) {   // batch 64 publishes per send
            if (body.size() >= 8) { i64 t = mono_ns(); memcpy(&body[0], &t, 8); }
            Method pm = make_method(60, 40);
            pm.args[1].s = x;
            if (x.empty()) pm.args[2].s = s.queues > 1 ? s.queue + "." + std::to_string(seq % nq) : s.queue;
            else if (s.queues > 1) pm.args[2].s = s.routing_key + "." + std::to_string(seq % nq) + (s.exchange_type == "topic" ? ".x" : "");
            else pm.args[2].s = s.routing_key;
            append_method_frame(c.out, 1, pm);
            append_content(c.out, 1, 60, props, body, c.frame_max);
            ++seq;
          }
          c.flush();
          sent[pi] = seq;
          if (s.confirm) {   // keep the confirm stream drained (non-blocking)
            char buf[1 << 16];
            ssize_t k;
            while ((k = ::recv(c.fd, buf, sizeof buf, MSG_DONTWAIT)) > 0) c.in.append(buf, (size_t)k);
            Frame f;
            while (c.parser.next(c.in, c.pos, f)) {
              if (f.type == FRAME_METHOD && f.payload.size() >= 12 && f.payload[1] == 60 && f.payload[3] == 80) {
                const u8* p = (const u8*)f.payload.data() + 4;
                u64 tag = 0;
                for (int i = 0; i < 8; ++i) tag = (tag << 8) | p[i];
                confirmed[pi] = tag;
              }
            }
            if (c.pos > (1u << 20)) { c.in.erase(0, c.pos); c.pos = 0; }
          }
          if (s.rate && seq >= (u64)((mono_ns() - t_start) / 1e9 * s.rate)) std::this_thread::sleep_for(std::chrono::microseconds(200));
        }
        c.close();
      } catch (std::exception& e) { fail(e); }
    });
  }
  std::this_thread::sleep_for(std::chrono::milliseconds((i64)(s.seconds * 1000)));
  u64 s_sent = 0, s_recv = 0;
  for (u64 x : sent) s_sent += x;
  for (u64 x : recv) s_recv += x;
  i64 t_end = mono_ns();
  stop = true;
  for (auto& t : th) t.join();
  Hist all;
  for (auto& h : hists) all.merge(h);
  r.elapsed = (t_end - t_start) / 1e9;
  r.sent = s_sent;
  r.received = s_recv;
  r.p50_us = all.q(0.50);
  r.p95_us = all.q(0.95);
  r.p99_us = all.q(0.99);
  r.error = err;
  return r;
}

}  // namespace cmq

// Native AMQP load generator: the RabbitMQ PerfTest(Multi) shapes of
// chana-mq-test/perf/publish-consume-spec*.js (producer/consumer counts, minMsgSize,
// auto-ack, channel-prefetch, persistent, confirms, time-limit, producer rate), run against
// any AMQP 0-9-1 broker.
//
// Connections are opened blocking (handshake, qos, consume), then driven non-blocking by
// `threads` epoll loops.  Producers send pre-rendered batches of publishes whose bodies
// carry a steady-clock send timestamp in their first 8 bytes (patched in place per batch);
// consumers parse frames in place in one receive buffer and histogram publish->deliver
// latency; manual-ack consumers ack with multiple=true every prefetch/2 deliveries and
// whenever their receive buffer runs dry.  Channel.Flow(active=false) from the broker pauses
// the connection's publishing (and is answered with FlowOk).
#include <arpa/inet.h>
#include <pthread.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
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
  bool frame(Frame& f, int timeout_ms = 10000) {
    timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    while (!parser.next(in, pos, f)) {
      char buf[1 << 16];
      ssize_t k = ::recv(fd, buf, sizeof buf, 0);
      if (k <= 0) return false;
      in.append(buf, (size_t)k);
    }
    return true;
  }
  std::string skipped_;
  Method expect(u16 cls, u16 mid) {
    Frame f;
    std::string& skipped = skipped_;   // (every method skipped on this connection so far)
    while (frame(f)) {
      if (f.type != FRAME_METHOD) continue;
      Method m = decode_method((const u8*)f.payload.data(), f.payload.size());
      if (m.cls() == cls && m.mid() == mid) return m;
      skipped += " " + std::to_string(m.cls()) + "." + std::to_string(m.mid());
      if (m.cls() == 10 && m.mid() == 50) throw std::runtime_error("loadgen: connection closed: " + m.s(1));
      if (m.cls() == 20 && m.mid() == 40) throw std::runtime_error("loadgen: channel closed: " + m.s(1));
    }
    throw std::runtime_error("loadgen: timeout waiting for reply " + std::to_string(cls) + "." + std::to_string(mid) +
                             " (skipped:" + skipped + ")");
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
      if (acc >= want) return std::pow(2.0, (double)(i + 1) / 8.0);   // bucket upper edge
    }
    return 0;
  }
};

u64 rd64(const u8* p) { u64 v = 0; for (int i = 0; i < 8; ++i) v = (v << 8) | p[i]; return v; }
u32 rd32(const u8* p) { return (u32(p[0]) << 24) | (u32(p[1]) << 16) | (u32(p[2]) << 8) | p[3]; }

// one non-blocking AMQP connection after setup
struct Peer {
  Client cl;
  bool producer = false;
  // producer: pre-rendered batch, body-timestamp offsets, pending output
  std::string batch;
  std::vector<size_t> ts_off;
  std::string out;
  size_t out_pos = 0;
  std::atomic<u64> sent{0}, confirmed{0}, nacked{0};
  bool flow = true;
  // any: receive buffer (recv lands in place, frames parsed in place)
  std::vector<char> in = std::vector<char>(4 << 20);
  size_t ilen = 0, pos = 0;
  // consumer
  bool want_body = false;
  u64 body_left = 0, last_tag = 0, unacked = 0;
  std::atomic<u64> recv{0}, redelivered{0}, requeued{0}, flow_off{0};
  u64 acks = 0, first_unacked = 0;
  bool cur_red = false;
  u8 ts[8];
  u32 tsn = 0;
  bool writable = true;
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
  const int nq = std::max(1, s.queues);
  std::vector<std::unique_ptr<Peer>> peers;
  // consumers first: they are attached before any message is published
  for (int ci = 0; ci < s.consumers; ++ci) {
    std::unique_ptr<Peer> p(new Peer());
    p->cl.open(s.host, s.consumer_port ? s.consumer_port : s.port, s.vhost);
    Method qos = make_method(60, 10);
    qos.args[1].i = s.prefetch;
    p->cl.method(1, qos);
    p->cl.flush();
    p->cl.expect(60, 11);
    Method cm = make_method(60, 20);
    cm.args[1].s = s.queues > 1 ? s.queue + "." + std::to_string(ci % nq) : s.queue;
    cm.args[2].s = "lg-" + std::to_string(ci);
    cm.args[4].i = s.auto_ack;
    p->cl.method(1, cm);
    p->cl.flush();
    p->cl.expect(60, 21);
    p->ilen = p->cl.in.size() - p->cl.pos;   // deliveries may already follow ConsumeOk
    memcpy(p->in.data(), p->cl.in.data() + p->cl.pos, p->ilen);
    peers.push_back(std::move(p));
  }
  // producers: batch of K publishes, keys cycling over the queues
  const double rate = s.rate;   // msgs/s per producer (0 = unthrottled)
  int K = 64;
  if (rate > 0) K = std::max(1, std::min(64, (int)(rate * 0.0005)));   // <= 0.5 ms of traffic per batch
  for (int pi = 0; pi < s.producers; ++pi) {
    std::unique_ptr<Peer> p(new Peer());
    p->producer = true;
    p->cl.open(s.host, s.producer_port ? s.producer_port : s.port, s.vhost);
    if (s.confirm) {
      p->cl.method(1, make_method(85, 10));
      p->cl.flush();
      p->cl.expect(85, 11);
    }
    std::string props = encode_props_simple(s.persistent ? 2 : 1);
    std::string body(std::max(s.msg_size, 0), 'x');
    for (int k = 0; k < K; ++k) {
      u64 seq = (u64)pi * 7 + k;
      Method pm = make_method(60, 40);
      pm.args[1].s = s.exchange;
      if (s.exchange.empty()) pm.args[2].s = s.queues > 1 ? s.queue + "." + std::to_string(seq % nq) : s.queue;
      else if (s.queues > 1) pm.args[2].s = s.routing_key + "." + std::to_string(seq % nq) + (s.exchange_type == "topic" ? ".x" : "");
      else pm.args[2].s = s.routing_key;
      append_method_frame(p->batch, 1, pm);
      size_t before = p->batch.size();
      append_content(p->batch, 1, 60, props, body, p->cl.frame_max);
      if (body.size() >= 8) {   // first body frame payload: after the header frame
        size_t hdr = 7 + 12 + props.size() + 1;
        p->ts_off.push_back(before + hdr + 7);
      }
    }
    p->ilen = p->cl.in.size() - p->cl.pos;
    memcpy(p->in.data(), p->cl.in.data() + p->cl.pos, p->ilen);
    peers.push_back(std::move(p));
  }
  for (auto& p : peers) {
    int fl = fcntl(p->cl.fd, F_GETFL);
    fcntl(p->cl.fd, F_SETFL, fl | O_NONBLOCK);
    timeval tv{0, 0};
    setsockopt(p->cl.fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  }
  int nthreads = s.threads > 0 ? s.threads : std::min<int>(8, (int)peers.size());
  nthreads = std::max(1, std::min<int>(nthreads, (int)peers.size()));
  // consumers and producers on separate threads (a thread that can always send would
  // otherwise starve the consumers it also serves)
  const int ncons = s.consumers, nprod = s.producers;
  int tc = 0, tp = 0;
  if (nthreads >= 2 && ncons && nprod) {
    tc = std::max(1, std::min(ncons, s.consumer_threads > 0 ? s.consumer_threads : nthreads / 2));
    tp = std::max(1, std::min(nprod, nthreads - tc));
    nthreads = tc + tp;
  }
  auto thread_of = [&](size_t i) -> int {   // peers: consumers first, then producers
    if (!tc) return (int)(i % nthreads);
    return i < (size_t)ncons ? (int)(i % tc) : tc + (int)((i - ncons) % tp);
  };
  const u64 window = s.confirm ? (u64)std::max(0, s.confirm_window) : 0;
  std::atomic<bool> stop{false};
  std::string err;
  std::mutex err_mu;
  std::vector<Hist> hists(nthreads);
  const i64 t_start = mono_ns();
  const u64 ack_every = (u64)std::max(1, s.prefetch / 2);

  auto worker = [&](int ti) {
    {
      char nm[16];
      snprintf(nm, sizeof nm, "lg-%s%d", (tc && ti >= tc) ? "p" : (tc ? "c" : "x"), ti);
      pthread_setname_np(pthread_self(), nm);
    }
    try {
      int ep = epoll_create1(0);
      std::vector<Peer*> mine;
      for (size_t i = 0; i < peers.size(); ++i) {
        if (thread_of(i) != ti) continue;
        Peer* p = peers[i].get();
        mine.push_back(p);
        epoll_event ev{};
        ev.events = EPOLLIN | EPOLLET | (p->producer ? EPOLLOUT : 0);
        ev.data.ptr = p;
        epoll_ctl(ep, EPOLL_CTL_ADD, p->cl.fd, &ev);
      }
      Hist& h = hists[ti];
      epoll_event evs[256];
      bool any_producer = false;
      for (Peer* p : mine) any_producer |= p->producer;
      auto pump = [&](Peer* p) {   // producer: send until the socket is full or paced out
        while (!stop) {
          if (p->out_pos >= p->out.size()) {
            if (!p->flow) return;   // paused: a started batch is still finished (whole frames)
            const u64 sent = p->sent.load(std::memory_order_relaxed);
            if (rate > 0 && (double)(sent + K) > rate * ((mono_ns() - t_start) * 1e-9)) return;
            if (window && sent + K > window + p->confirmed.load(std::memory_order_relaxed) +
                                         p->nacked.load(std::memory_order_relaxed)) return;   // confirm window full
            p->out = p->batch;
            const i64 t = mono_ns();
            for (size_t o : p->ts_off) memcpy(&p->out[o], &t, 8);
            p->out_pos = 0;
            p->sent.fetch_add((u64)K, std::memory_order_relaxed);
          }
          ssize_t k = ::send(p->cl.fd, p->out.data() + p->out_pos, p->out.size() - p->out_pos, MSG_NOSIGNAL);
          if (k > 0) { p->out_pos += (size_t)k; continue; }
          if (k < 0 && errno == EINTR) continue;
          if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) { p->writable = false; return; }
          throw std::runtime_error("loadgen: producer send failed");
        }
      };
      auto send_small = [&](Peer* p, const std::string& b) {   // acks / FlowOk: tiny, retry until written
        size_t o = 0;
        while (o < b.size() && !stop) {
          ssize_t k = ::send(p->cl.fd, b.data() + o, b.size() - o, MSG_NOSIGNAL);
          if (k > 0) o += (size_t)k;
          else if (k < 0 && (errno == EAGAIN || errno == EINTR)) std::this_thread::yield();
          else throw std::runtime_error("loadgen: send failed");
        }
      };
      auto parse = [&](Peer* p) {
        const u8* b = (const u8*)p->in.data();
        size_t n = p->ilen, pos = p->pos;
        while (n - pos >= 8) {
          u32 size = rd32(b + pos + 3);
          if (n - pos < (size_t)size + 8) break;
          const u8 type = b[pos];
          const u8* pl = b + pos + 7;
          if (b[pos + 7 + size] != 0xCE) throw std::runtime_error("loadgen: bad frame end");
          if (type == FRAME_METHOD && size >= 4) {
            u16 cls = (u16(pl[0]) << 8) | pl[1], mid = (u16(pl[2]) << 8) | pl[3];
            if (cls == 60 && mid == 60) {             // Basic.Deliver
              u32 tl = pl[4];
              p->last_tag = rd64(pl + 5 + tl);
              p->cur_red = pl[5 + tl + 8] & 1;
              if (p->cur_red) p->redelivered.fetch_add(1, std::memory_order_relaxed);
              p->want_body = true;
              p->tsn = 0;
            } else if (cls == 60 && (mid == 80 || mid == 120)) {   // confirm Ack / Nack
              u64 tag = rd64(pl + 4);
              bool multiple = pl[12] & 1;
              u64 before = p->confirmed.load(std::memory_order_relaxed) + p->nacked.load(std::memory_order_relaxed);
              u64 cnt = multiple ? (tag > before ? tag - before : 0) : 1;
              (mid == 80 ? p->confirmed : p->nacked).fetch_add(cnt, std::memory_order_relaxed);
            } else if (cls == 20 && mid == 20) {      // Channel.Flow
              p->flow = pl[4] & 1;
              if (!p->flow && p->producer) p->flow_off.fetch_add(1, std::memory_order_relaxed);
              std::string fo;
              Method m = make_method(20, 21);
              m.args[0].i = p->flow;
              append_method_frame(fo, 1, m);
              if (p->producer && p->out_pos < p->out.size()) {
                p->out += fo;   // after the partly sent batch: frames must not interleave
                p->writable = true;
              } else {
                send_small(p, fo);
              }
            } else if (cls == 10 && mid == 50) {
              throw std::runtime_error("loadgen: connection closed by broker");
            } else if (cls == 20 && mid == 40) {
              throw std::runtime_error("loadgen: channel closed by broker");
            }
          } else if (type == FRAME_HEADER && p->want_body && size >= 12) {
            p->body_left = rd64(pl + 4);
            if (p->body_left == 0) { p->want_body = false; p->recv.fetch_add(1, std::memory_order_relaxed); ++p->unacked; }
          } else if (type == FRAME_BODY && p->want_body) {
            if (p->tsn < 8) {
              u32 take = std::min<u32>(8 - p->tsn, size);
              memcpy(p->ts + p->tsn, pl, take);
              p->tsn += take;
            }
            p->body_left -= std::min<u64>(p->body_left, size);
            if (p->body_left == 0) {
              p->want_body = false;
              p->recv.fetch_add(1, std::memory_order_relaxed);
              ++p->unacked;
              if (p->tsn == 8 && !p->cur_red) {   // latency of first deliveries only
                i64 t0;
                memcpy(&t0, p->ts, 8);
                h.add((mono_ns() - t0) / 1000.0);
              }
            }
          }
          pos += (size_t)size + 8;
        }
        p->pos = pos;
        if (p->pos == p->ilen) {
          p->pos = p->ilen = 0;
        } else if (p->pos > p->in.size() / 2 || p->in.size() - p->ilen < (64u << 10)) {   // compact the tail
          memmove(p->in.data(), p->in.data() + p->pos, p->ilen - p->pos);
          p->ilen -= p->pos;
          p->pos = 0;
          if (p->in.size() - p->ilen < (64u << 10)) p->in.resize(p->in.size() * 2);   // a frame larger than the buffer
        }
      };
      auto ack = [&](Peer* p) {   // everything up to last_tag: Ack, or every nack_every-th time Nack+requeue
        std::string ak;
        const bool nack = s.nack_every > 0 && ++p->acks % (u64)s.nack_every == 0;
        Method m = make_method(60, nack ? 120 : 80);
        m.args[0].i = (i64)p->last_tag;
        m.args[1].i = 1;
        if (nack) {
          m.args[2].i = 1;
          p->requeued.fetch_add(p->unacked, std::memory_order_relaxed);
        }
        append_method_frame(ak, 1, m);
        send_small(p, ak);
        p->unacked = 0;
      };
      auto drain = [&](Peer* p) {
        for (;;) {
          ssize_t k = ::recv(p->cl.fd, p->in.data() + p->ilen, p->in.size() - p->ilen, 0);
          if (k > 0) {
            p->ilen += (size_t)k;
            parse(p);
            if (!p->producer && !s.auto_ack && p->unacked >= ack_every) ack(p);
            continue;
          }
          if (k == 0) throw std::runtime_error("loadgen: broker closed the connection");
          if (errno == EINTR) continue;
          break;
        }
        if (!p->producer && !s.auto_ack && p->unacked) ack(p);   // buffer ran dry: settle what we have
      };
      for (Peer* p : mine) if (p->ilen) parse(p);
      while (!stop) {
        for (Peer* p : mine)
          if (p->producer && p->writable) pump(p);
        int n = epoll_wait(ep, evs, 256, any_producer && rate > 0 ? 0 : 2);
        for (int i = 0; i < n; ++i) {
          Peer* p = (Peer*)evs[i].data.ptr;
          if (evs[i].events & EPOLLOUT) p->writable = true;
          if (evs[i].events & (EPOLLIN | EPOLLHUP | EPOLLERR)) drain(p);
        }
        if (any_producer && rate > 0 && n == 0) std::this_thread::sleep_for(std::chrono::microseconds(50));
      }
      ::close(ep);
      timespec ts;
      clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
      std::lock_guard<std::mutex> g(err_mu);
      (tc && ti >= tc ? r.cpu_producers_s : r.cpu_consumers_s) += ts.tv_sec + ts.tv_nsec * 1e-9;
    } catch (std::exception& e) {
      std::lock_guard<std::mutex> g(err_mu);
      if (err.empty()) err = e.what();
      stop = true;
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) th.emplace_back(worker, t);
  // warm-up excluded from the counts: snapshot after `warmup` seconds
  const double warm = std::max(0.0, s.warmup);
  u64 sent0 = 0, recv0 = 0, conf0 = 0, red0 = 0, rq0 = 0, fl0 = 0;
  if (warm > 0) {
    std::this_thread::sleep_for(std::chrono::milliseconds((i64)(warm * 1000)));
    for (auto& p : peers) {
      sent0 += p->sent; recv0 += p->recv; conf0 += p->confirmed;
      red0 += p->redelivered; rq0 += p->requeued; fl0 += p->flow_off;
    }
  }
  const i64 t_meas = mono_ns();
  std::this_thread::sleep_for(std::chrono::milliseconds((i64)(s.seconds * 1000)));
  u64 s_sent = 0, s_recv = 0, s_conf = 0, s_nack = 0, s_red = 0, s_rq = 0, s_fl = 0;
  for (auto& p : peers) {
    s_sent += p->sent; s_recv += p->recv; s_conf += p->confirmed; s_nack += p->nacked;
    s_red += p->redelivered; s_rq += p->requeued; s_fl += p->flow_off;
  }
  const i64 t_end = mono_ns();
  stop = true;
  for (auto& t : th) t.join();
  Hist all;
  for (auto& h : hists) all.merge(h);
  for (auto& p : peers) p->cl.close();
  r.elapsed = (t_end - t_meas) / 1e9;
  r.sent = s_sent - sent0;
  r.received = s_recv - recv0;
  r.confirmed = s_conf - conf0;
  r.nacked = s_nack;
  r.redelivered = s_red - red0;
  r.requeued = s_rq - rq0;
  r.flow_off = s_fl - fl0;
  r.p50_us = all.q(0.50);
  r.p95_us = all.q(0.95);
  r.p99_us = all.q(0.99);
  r.error = err;
  r.threads = nthreads;
  return r;
}

}  // namespace cmq

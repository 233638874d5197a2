// Native AMQP 0-9-1 broker (see broker.hpp for the reference map).
#include "broker.hpp"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/pkcs12.h>
#include <openssl/ssl.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <random>
#include <sstream>

namespace cmq {

static i64 now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::system_clock::now().time_since_epoch()).count();
}

static const size_t OUT_HIGH = 8u << 20;   // stop delivering to a connection above this
static const size_t OUT_LOW = 1u << 20;

u64 IdGenerator::next() {
  i64 ms = now_ms();
  if (ms < last_ms_) ms = last_ms_;   // clock went back: stay on the last ms (reference throws)
  if (ms == last_ms_) {
    if (++seq_ > 4095) {             // 4096 ids per ms: wait for the next ms (IdGenerator.scala:55-73)
      while ((ms = now_ms()) <= last_ms_) {}
      seq_ = 0;
    }
  } else {
    seq_ = 0;
  }
  last_ms_ = ms;
  return (u64(ms) << 22) | (u64(worker_) << 12) | seq_;
}

// ------------------------------------------------------------------ topic words
static std::vector<std::string> split_words(const std::string& k) {   // Java split("\\.")
  std::vector<std::string> w;
  if (k.empty()) { w.emplace_back(); return w; }
  size_t s = 0;
  while (true) {
    size_t d = k.find('.', s);
    if (d == std::string::npos) { w.push_back(k.substr(s)); break; }
    w.push_back(k.substr(s, d - s));
    s = d + 1;
  }
  while (!w.empty() && w.back().empty()) w.pop_back();
  return w;
}

static bool topic_match(const std::vector<std::string>& pw, const std::vector<std::string>& kw, bool hash) {
  size_t p = 0, k = 0, sp = std::string::npos, sk = 0;
  while (k < kw.size()) {
    if (p < pw.size() && hash && pw[p] == "#") { sp = ++p; sk = k; continue; }
    if (p < pw.size() && (pw[p] == "*" || pw[p] == kw[k])) { ++p; ++k; continue; }
    if (sp != std::string::npos) { k = ++sk; p = sp; continue; }
    return false;
  }
  while (p < pw.size() && hash && pw[p] == "#") ++p;
  return p == pw.size();
}

void Exchange::reindex() {
  direct.clear();
  for (size_t i = 0; i < bindings.size(); ++i) direct[bindings[i].key].push_back(i);
}

static std::string entity_id(const std::string& vhost, const std::string& name) {
  return vhost.empty() ? name : vhost + "-_." + name;    // chana-mq-server/.../package.scala:17-21
}

static std::string table_str(const Value& v) {
  switch (v.tag) {
    case 'S': case 'x': return v.s;
    case 't': return v.i ? "true" : "false";
    case 'd': case 'f': { std::ostringstream o; o << v.d; return o.str(); }
    case 'V': return "";
    default: return std::to_string(v.i);
  }
}
static std::map<std::string, std::string> table_to_map(const Table& t) {
  std::map<std::string, std::string> m;
  for (auto& kv : t) m[kv.first] = table_str(kv.second);
  return m;
}

// ------------------------------------------------------------------ lifecycle
Broker::Broker(const BrokerConfig& cfg) : cfg_(cfg), ids_(cfg.worker_id) {
  store_.open(cfg_.data_dir, cfg_.fsync);
  Vhost* v = vhost(cfg_.default_vhost, true);
  (void)v;
  recover();
}

Broker::~Broker() {
  stop();
  for (auto& kv : conns_) {
    if (kv.second->ssl) SSL_free(kv.second->ssl);
    ::close(kv.first);
  }
  if (ssl_ctx_) SSL_CTX_free(ssl_ctx_);
  store_.close();
}

static int make_listener(const std::string& host, int port, int* bound) {
  int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  inet_pton(AF_INET, host.c_str(), &a.sin_addr);
  if (::bind(fd, (sockaddr*)&a, sizeof a) < 0 || ::listen(fd, 1024) < 0) {
    ::close(fd);
    throw std::runtime_error("cannot listen on " + host + ":" + std::to_string(port));
  }
  socklen_t l = sizeof a;
  getsockname(fd, (sockaddr*)&a, &l);
  *bound = ntohs(a.sin_port);
  return fd;
}

void Broker::setup_tls() {
  SSL_library_init();
  SSL_load_error_strings();
  ssl_ctx_ = SSL_CTX_new(TLS_server_method());
  if (!ssl_ctx_) throw std::runtime_error("SSL_CTX_new failed");
  if (!cfg_.tls_p12.empty()) {
    FILE* f = fopen(cfg_.tls_p12.c_str(), "rb");
    if (!f) throw std::runtime_error("cannot open keystore " + cfg_.tls_p12);
    PKCS12* p12 = d2i_PKCS12_fp(f, nullptr);
    fclose(f);
    EVP_PKEY* pkey = nullptr;
    X509* cert = nullptr;
    if (!p12 || !PKCS12_parse(p12, cfg_.tls_p12_password.c_str(), &pkey, &cert, nullptr))
      throw std::runtime_error("cannot parse PKCS12 keystore");
    SSL_CTX_use_certificate(ssl_ctx_, cert);
    SSL_CTX_use_PrivateKey(ssl_ctx_, pkey);
    X509_free(cert);
    EVP_PKEY_free(pkey);
    PKCS12_free(p12);
  } else {
    if (SSL_CTX_use_certificate_chain_file(ssl_ctx_, cfg_.tls_cert.c_str()) != 1 ||
        SSL_CTX_use_PrivateKey_file(ssl_ctx_, cfg_.tls_key.c_str(), SSL_FILETYPE_PEM) != 1)
      throw std::runtime_error("cannot load TLS certificate/key");
  }
}

void Broker::setup_listeners() {
  epfd_ = epoll_create1(EPOLL_CLOEXEC);
  evfd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = evfd_;
  epoll_ctl(epfd_, EPOLL_CTL_ADD, evfd_, &ev);
  if (cfg_.amqp_enable) {
    lfd_ = make_listener(cfg_.host, cfg_.port, &bound_port_);
    ev.data.fd = lfd_;
    epoll_ctl(epfd_, EPOLL_CTL_ADD, lfd_, &ev);
  }
  if (cfg_.tls_enable) {
    setup_tls();
    tls_lfd_ = make_listener(cfg_.host, cfg_.tls_port, &bound_tls_port_);
    ev.data.fd = tls_lfd_;
    epoll_ctl(epfd_, EPOLL_CTL_ADD, tls_lfd_, &ev);
  }
}

void Broker::start() {
  setup_listeners();
  stop_ = false;
  running_ = true;
  thr_ = std::thread([this] { loop(); });
}

void Broker::stop() {
  if (!running_) return;
  stop_ = true;
  u64 one = 1;
  (void)!::write(evfd_, &one, 8);
  if (thr_.joinable()) thr_.join();
  running_ = false;
  for (int fd : {lfd_, tls_lfd_, evfd_, epfd_})
    if (fd >= 0) ::close(fd);
  lfd_ = tls_lfd_ = evfd_ = epfd_ = -1;
  store_.sync();
}

void Broker::post(std::function<void()> fn) {
  {
    std::lock_guard<std::mutex> g(post_mu_);
    posted_.push_back(std::move(fn));
  }
  u64 one = 1;
  (void)!::write(evfd_, &one, 8);
}

void Broker::drain_posted() {
  std::vector<std::function<void()>> fns;
  {
    std::lock_guard<std::mutex> g(post_mu_);
    fns.swap(posted_);
  }
  for (auto& f : fns) f();
}

template <class T>
static T run_on(Broker* b, std::function<void(std::function<void()>)> poster, std::function<T()> fn) {
  std::mutex m;
  std::condition_variable cv;
  bool done = false;
  T res{};
  poster([&] {
    res = fn();
    std::lock_guard<std::mutex> g(m);
    done = true;
    cv.notify_one();
  });
  std::unique_lock<std::mutex> g(m);
  cv.wait(g, [&] { return done; });
  (void)b;
  return res;
}

bool Broker::create_vhost(const std::string& name) {
  auto f = [this, name]() -> bool {
    Vhost* v = vhost(name, true);
    v->active = true;
    store_.insertVhost(name, true);
    store_.sync();
    return true;
  };
  if (!running_) return f();
  return run_on<bool>(this, [this](std::function<void()> x) { post(std::move(x)); }, f);
}

bool Broker::delete_vhost(const std::string& name) {
  // VhostEntity.Delete does not cascade to exchanges/queues (SURVEY A.Q28): parity
  auto f = [this, name]() -> bool {
    store_.deleteVhost(name);
    store_.sync();
    if (name == cfg_.default_vhost) return true;   // the default vhost always exists
    auto it = vhosts_.find(name);
    if (it != vhosts_.end()) it->second->active = false;
    return true;
  };
  if (!running_) return f();
  return run_on<bool>(this, [this](std::function<void()> x) { post(std::move(x)); }, f);
}

std::string Broker::stats_json() {
  auto f = [this]() -> std::string {
    std::ostringstream o;
    u64 nq = 0, ready = 0, unacked = 0;
    for (auto& v : vhosts_)
      for (auto& q : v.second->queues) { ++nq; ready += q.second->ready.size(); unacked += q.second->unacked; }
    o << "{\"published\":" << stats_.published << ",\"routed\":" << stats_.routed
      << ",\"unroutable\":" << stats_.unroutable << ",\"delivered\":" << stats_.delivered
      << ",\"acked\":" << stats_.acked << ",\"requeued\":" << stats_.requeued << ",\"expired\":" << stats_.expired
      << ",\"returned\":" << stats_.returned << ",\"confirms\":" << stats_.confirms
      << ",\"connections\":" << conns_.size() << ",\"connections_total\":" << stats_.connections
      << ",\"queues\":" << nq << ",\"messages_ready\":" << ready << ",\"messages_unacked\":" << unacked
      << ",\"queued_bytes\":" << queued_bytes_ << ",\"memory_alarm\":" << (mem_alarm_ ? "true" : "false")
      << ",\"bytes_in\":" << stats_.bytes_in << ",\"bytes_out\":" << stats_.bytes_out
      << ",\"store_wal_bytes\":" << store_.walBytes() << "}";
    return o.str();
  };
  if (!running_) return f();
  return run_on<std::string>(this, [this](std::function<void()> x) { post(std::move(x)); }, f);
}

std::string Broker::queues_json() {
  auto f = [this]() -> std::string {
    std::ostringstream o;
    o << "[";
    bool first = true;
    for (auto& v : vhosts_)
      for (auto& q : v.second->queues) {
        if (!first) o << ",";
        first = false;
        o << "{\"vhost\":\"" << v.first << "\",\"name\":\"" << q.first << "\",\"ready\":" << q.second->ready.size()
          << ",\"unacked\":" << q.second->unacked << ",\"consumers\":" << q.second->consumers.size()
          << ",\"durable\":" << (q.second->durable ? "true" : "false") << ",\"published\":" << q.second->published
          << ",\"delivered\":" << q.second->delivered << "}";
      }
    o << "]";
    return o.str();
  };
  if (!running_) return f();
  return run_on<std::string>(this, [this](std::function<void()> x) { post(std::move(x)); }, f);
}

// ------------------------------------------------------------------ event loop
void Broker::loop() {
  std::vector<epoll_event> evs(512);
  while (!stop_) {
    int n = epoll_wait(epfd_, evs.data(), (int)evs.size(), 50);
    for (int i = 0; i < n; ++i) {
      int fd = evs[i].data.fd;
      if (fd == evfd_) {
        u64 x;
        (void)!::read(evfd_, &x, 8);
        drain_posted();
        continue;
      }
      if (fd == lfd_) { accept_all(lfd_, false); continue; }
      if (fd == tls_lfd_) { accept_all(tls_lfd_, true); continue; }
      auto it = conns_.find(fd);
      if (it == conns_.end()) continue;
      Conn* c = it->second.get();
      if (evs[i].events & (EPOLLERR | EPOLLHUP)) c->dead = true;
      if (!c->dead && (evs[i].events & EPOLLIN)) on_readable(c);
      if (!c->dead && (evs[i].events & EPOLLOUT)) on_writable(c);
    }
    // delivery for queues touched by this batch (the reference polls every 1us tick)
    while (!dirty_.empty()) {
      std::set<Queue*> d;
      d.swap(dirty_);
      for (Queue* q : d) deliver(q);
    }
    confirm_flush();
    i64 now = now_ms();
    if (now - last_timer_ >= 100) { timers(now); last_timer_ = now; }
    for (auto& kv : conns_)
      if (kv.second->out.size() > kv.second->out_pos) flush(kv.second.get());
    reap();
  }
}

void Broker::accept_all(int lfd, bool tls) {
  while (true) {
    sockaddr_in a{};
    socklen_t l = sizeof a;
    int fd = ::accept4(lfd, (sockaddr*)&a, &l, SOCK_NONBLOCK | SOCK_CLOEXEC);
    if (fd < 0) return;
    if (cfg_.max_connections && conns_.size() >= cfg_.max_connections) { ::close(fd); continue; }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    auto c = std::make_unique<Conn>();
    c->id = next_conn_id_++;
    c->fd = fd;
    c->last_rx = c->last_tx = now_ms();
    char ip[64];
    inet_ntop(AF_INET, &a.sin_addr, ip, sizeof ip);
    c->peer = std::string(ip) + ":" + std::to_string(ntohs(a.sin_port));
    if (tls) {
      c->ssl = SSL_new(ssl_ctx_);
      SSL_set_fd(c->ssl, fd);
      SSL_set_accept_state(c->ssl);
    }
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = fd;
    epoll_ctl(epfd_, EPOLL_CTL_ADD, fd, &ev);
    conns_[fd] = std::move(c);
    ++stats_.connections;
  }
}

void Broker::on_readable(Conn* c) {
  if (c->blocked) return;
  char buf[65536];
  int budget = 2;    // fairness: at most 128 KB per connection per loop iteration (a publisher
                     // flood must not starve the acks that reopen consumer windows)
  while (budget-- > 0) {
    ssize_t k;
    if (c->ssl) {
      if (!c->tls_handshaken) {
        int r = SSL_do_handshake(c->ssl);
        if (r != 1) {
          int e = SSL_get_error(c->ssl, r);
          if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) return;
          c->dead = true;
          return;
        }
        c->tls_handshaken = true;
      }
      k = SSL_read(c->ssl, buf, sizeof buf);
      if (k <= 0) {
        int e = SSL_get_error(c->ssl, (int)k);
        if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) break;
        c->dead = true;
        break;
      }
    } else {
      k = ::recv(c->fd, buf, sizeof buf, 0);
      if (k == 0) { c->dead = true; break; }
      if (k < 0) {
        if (errno == EAGAIN || errno == EWOULDBLOCK) break;
        c->dead = true;
        break;
      }
    }
    c->in.append(buf, (size_t)k);
    stats_.bytes_in += (u64)k;
    c->last_rx = now_ms();
    if ((size_t)k < sizeof buf) break;
  }
  process_input(c);
}

void Broker::process_input(Conn* c) {
  try {
    if (c->state == CS_HANDSHAKE) {
      if (c->in.size() - c->in_pos < 8) return;
      if (memcmp(c->in.data() + c->in_pos, PROTOCOL_HEADER, 8) != 0) {
        // protocol mismatch: answer with our header and close (the reference keeps the
        // socket open, FrameStage.scala:224-228; AMQP 0-9-1 §4.2.2 says close)
        c->out.append(PROTOCOL_HEADER, 8);
        c->state = CS_CLOSING;
        c->close_deadline = now_ms();
        kick_write(c);
        return;
      }
      c->in_pos += 8;
      Method m = make_method(10, 10);
      m.args[0].i = 0;
      m.args[1].i = 9;
      m.args[2].t = {{"product", Value::str(cfg_.product)},
                     {"version", Value::str(cfg_.version)},
                     {"chana.mq.build", Value::str("1")},
                     {"capabilities", Value::table({{"publisher_confirms", Value::boolean(true)},
                                                    {"exchange_exchange_bindings", Value::boolean(true)},
                                                    {"basic.nack", Value::boolean(true)},
                                                    {"consumer_cancel_notify", Value::boolean(true)},
                                                    {"connection.blocked", Value::boolean(true)}})}};
      m.args[3].s = "PLAIN EXTERNAL";
      m.args[4].s = "en_US";
      send_method(c, 0, m);
      c->state = CS_START_SENT;
    }
    Frame f;
    while (c->state != CS_CLOSED && !c->dead && c->parser.next(c->in, c->in_pos, f)) handle_frame(c, f);
  } catch (AmqpError& e) {
    send_connection_close(c, e.code, e.what(), e.cls, e.mid);
    c->in.clear();
    c->in_pos = 0;
  }
  if (c->in_pos > (1u << 20) || c->in_pos == c->in.size()) {
    c->in.erase(0, c->in_pos);
    c->in_pos = 0;
  }
}

void Broker::kick_write(Conn* c) {
  if (c->want_write) return;
  c->want_write = true;
}

void Broker::flush(Conn* c) {
  while (c->out_pos < c->out.size()) {
    ssize_t k;
    size_t n = c->out.size() - c->out_pos;
    if (c->ssl) {
      if (!c->tls_handshaken) break;
      k = SSL_write(c->ssl, c->out.data() + c->out_pos, (int)std::min<size_t>(n, 1 << 20));
      if (k <= 0) {
        int e = SSL_get_error(c->ssl, (int)k);
        if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) break;
        c->dead = true;
        return;
      }
    } else {
      k = ::send(c->fd, c->out.data() + c->out_pos, n, MSG_NOSIGNAL);
      if (k < 0) {
        if (errno == EAGAIN || errno == EWOULDBLOCK) break;
        c->dead = true;
        return;
      }
    }
    c->out_pos += (size_t)k;
    stats_.bytes_out += (u64)k;
    c->last_tx = now_ms();
  }
  bool pending = c->out_pos < c->out.size();
  if (!pending) {
    bool was_big = c->out.size() > OUT_LOW;
    c->out.clear();
    c->out_pos = 0;
    if (was_big)   // consumers throttled on this connection can take more
      for (auto& chkv : c->channels)
        for (auto& ckv : chkv.second.consumers) mark_dirty(ckv.second->q);
  } else if (c->out_pos > (4u << 20)) {
    c->out.erase(0, c->out_pos);
    c->out_pos = 0;
  }
  epoll_event ev{};
  ev.events = (c->blocked ? 0 : EPOLLIN) | (pending ? EPOLLOUT : 0);
  ev.data.fd = c->fd;
  epoll_ctl(epfd_, EPOLL_CTL_MOD, c->fd, &ev);
  c->want_write = false;
  if (!pending && c->state == CS_CLOSING && c->close_deadline && now_ms() >= c->close_deadline) c->dead = true;
}

void Broker::on_writable(Conn* c) {
  if (c->ssl && !c->tls_handshaken) { on_readable(c); return; }
  flush(c);
}

void Broker::close_conn(Conn* c) {
  for (auto& kv : c->channels) close_channel_state(c, kv.second);
  c->channels.clear();
  std::vector<Queue*> ex(c->exclusive_queues.begin(), c->exclusive_queues.end());
  for (Queue* q : ex) delete_queue(q, false);   // exclusive queues die with their connection
  c->exclusive_queues.clear();
  c->state = CS_CLOSED;
}

void Broker::reap() {
  std::vector<int> dead;
  for (auto& kv : conns_)
    if (kv.second->dead) dead.push_back(kv.first);
  for (int fd : dead) {
    Conn* c = conns_[fd].get();
    if (c->state != CS_CLOSED) close_conn(c);
    epoll_ctl(epfd_, EPOLL_CTL_DEL, fd, nullptr);
    if (c->ssl) SSL_free(c->ssl);
    ::close(fd);
    confirm_conns_.erase(c);
    conns_.erase(fd);
  }
  if (!dead.empty())
    while (!dirty_.empty()) {
      std::set<Queue*> d;
      d.swap(dirty_);
      for (Queue* q : d) deliver(q);
    }
}

void Broker::timers(i64 now) {
  for (auto& kv : conns_) {
    Conn* c = kv.second.get();
    if (c->state == CS_CLOSING && c->close_deadline && now >= c->close_deadline + 2000) c->dead = true;
    if (c->state != CS_OPEN || !c->heartbeat) continue;
    i64 hb = (i64)c->heartbeat * 1000;
    if (now - c->last_tx >= hb) {       // FrameStage.scala:104-107
      c->out.append(HEARTBEAT_FRAME, 8);
      c->last_tx = now;
      kick_write(c);
    }
    if (now - c->last_rx > 2 * hb) c->dead = true;   // missed client heartbeats (SURVEY A.Q36)
  }
  // TTL sweep of queue heads (MessageEntity timers / QueueEntity Pull skip)
  for (auto& v : vhosts_)
    for (auto& q : v.second->queues) expire_head(q.second.get(), now);
}

// ------------------------------------------------------------------ sending
void Broker::send_method(Conn* c, u16 ch, const Method& m) {
  append_method_frame(c->out, ch, m);
  kick_write(c);
}

void Broker::send_connection_close(Conn* c, u16 code, const std::string& text, u16 cls, u16 mid) {
  if (c->state == CS_CLOSING || c->state == CS_CLOSED) return;
  Method m = make_method(10, 50);
  m.args[0].i = code;
  m.args[1].s = text.substr(0, 255);
  m.args[2].i = cls;
  m.args[3].i = mid;
  send_method(c, 0, m);
  for (auto& kv : c->channels) close_channel_state(c, kv.second);
  c->channels.clear();
  c->state = CS_CLOSING;
  c->close_deadline = now_ms();
}

void Broker::send_channel_close(Conn* c, Channel& ch, u16 code, const std::string& text, u16 cls, u16 mid) {
  Method m = make_method(20, 40);
  m.args[0].i = code;
  m.args[1].s = text.substr(0, 255);
  m.args[2].i = cls;
  m.args[3].i = mid;
  send_method(c, ch.id, m);
  close_channel_state(c, ch);
  ch.closing = true;
}

// ------------------------------------------------------------------ frames
void Broker::handle_frame(Conn* c, Frame& f) {
  if (f.type == FRAME_HEARTBEAT) return;
  if (c->state == CS_CLOSING) {
    if (f.ch == 0 && f.type == FRAME_METHOD && f.payload.size() >= 4) {
      Method m = decode_method((const u8*)f.payload.data(), f.payload.size());
      if (m.cls() == 10 && m.mid() == 51) { c->dead = true; return; }
      if (m.cls() == 10 && m.mid() == 50) {
        send_method(c, 0, make_method(10, 51));
        c->close_deadline = now_ms();
      }
    }
    return;
  }
  if (f.ch == 0) {
    if (f.type != FRAME_METHOD) throw AmqpError(UNEXPECTED_FRAME, "content frame on channel 0", true);
    Method m = decode_method((const u8*)f.payload.data(), f.payload.size());
    if (m.cls() != 10) throw AmqpError(COMMAND_INVALID, "non-connection method on channel 0", true, m.cls(), m.mid());
    on_connection(c, m);
    return;
  }
  if (c->state != CS_OPEN) throw AmqpError(CHANNEL_ERROR, "connection not open", true);
  auto it = c->channels.find(f.ch);
  if (it == c->channels.end()) {
    if (f.type == FRAME_METHOD) {
      Method m = decode_method((const u8*)f.payload.data(), f.payload.size());
      if (m.cls() == 20 && m.mid() == 10) { on_channel(c, f.ch, m); return; }
      if (m.cls() == 20 && m.mid() == 41) return;   // late Close-Ok
    }
    throw AmqpError(CHANNEL_ERROR, "channel " + std::to_string(f.ch) + " not open", true);
  }
  Channel& ch = it->second;
  if (ch.closing) {
    if (f.type == FRAME_METHOD) {
      Method m = decode_method((const u8*)f.payload.data(), f.payload.size());
      if (m.cls() == 20 && m.mid() == 41) { c->channels.erase(it); return; }
      if (m.cls() == 20 && m.mid() == 40) { send_method(c, f.ch, make_method(20, 41)); c->channels.erase(it); }
    }
    return;
  }
  try {
    if (f.type == FRAME_METHOD) {
      if (ch.have_method) throw AmqpError(UNEXPECTED_FRAME, "method frame while content pending", true);
      Method m = decode_method((const u8*)f.payload.data(), f.payload.size());
      if (m.spec->content) {
        if (!(m.cls() == 60 && m.mid() == 40))
          throw AmqpError(COMMAND_INVALID, std::string("client may not send ") + m.spec->name, true, m.cls(), m.mid());
        ch.method = std::move(m);
        ch.have_method = true;
        ch.have_header = false;
        return;
      }
      dispatch(c, &ch, m);
    } else if (f.type == FRAME_HEADER) {
      if (!ch.have_method || ch.have_header) throw AmqpError(UNEXPECTED_FRAME, "unexpected content header", true);
      if (f.payload.size() < 14) throw AmqpError(FRAME_ERROR, "short content header", true);
      const u8* p = (const u8*)f.payload.data();
      u64 bs = 0;
      for (int i = 0; i < 8; ++i) bs = (bs << 8) | p[4 + i];
      ch.body_size = bs;
      ch.props.assign(f.payload.data() + 12, f.payload.size() - 12);
      ch.body.clear();
      ch.have_header = true;
      if (bs == 0) {
        ch.have_method = ch.have_header = false;
        on_publish(c, ch, ch.method, std::move(ch.props), std::string());
      } else {
        ch.body.reserve(bs);
      }
    } else if (f.type == FRAME_BODY) {
      if (!ch.have_header) throw AmqpError(UNEXPECTED_FRAME, "unexpected content body", true);
      ch.body += f.payload;
      if (ch.body.size() > ch.body_size) throw AmqpError(FRAME_ERROR, "body larger than declared", true);
      if (ch.body.size() == ch.body_size) {
        ch.have_method = ch.have_header = false;
        on_publish(c, ch, ch.method, std::move(ch.props), std::move(ch.body));
        ch.body = std::string();
      }
    }
  } catch (AmqpError& e) {
    if (e.connection) throw;
    auto it2 = c->channels.find(f.ch);
    if (it2 != c->channels.end() && !it2->second.closing)
      send_channel_close(c, it2->second, e.code, e.what(), e.cls, e.mid);
  }
}

void Broker::dispatch(Conn* c, Channel* ch, Method& m) {
  switch (m.cls()) {
    case 20: on_channel(c, ch->id, m); break;
    case 30: {   // Access.Request: reply OK (reference logs only: SURVEY A.Q12)
      Method r = make_method(30, 11);
      r.args[0].i = 1;
      send_method(c, ch->id, r);
      break;
    }
    case 40: on_exchange(c, *ch, m); break;
    case 50: on_queue(c, *ch, m); break;
    case 60: on_basic(c, *ch, m); break;
    case 85: {
      if (m.mid() != 10) throw AmqpError(COMMAND_INVALID, "bad confirm method", true, 85, m.mid());
      if (ch->tx) throw AmqpError(PRECONDITION_FAILED, "cannot switch from tx to confirm mode", false, 85, 10);
      ch->confirm = true;
      if (!m.b(0)) send_method(c, ch->id, make_method(85, 11));
      break;
    }
    case 90: {
      if (m.mid() == 10) {
        if (ch->confirm) throw AmqpError(PRECONDITION_FAILED, "cannot switch from confirm to tx mode", false, 90, 10);
        ch->tx = true;
        send_method(c, ch->id, make_method(90, 11));
      } else if (m.mid() == 20 || m.mid() == 30) {
        if (!ch->tx) throw AmqpError(PRECONDITION_FAILED, "channel is not transactional", false, 90, m.mid());
        auto pubs = std::move(ch->tx_pubs);
        auto acks = std::move(ch->tx_acks);
        ch->tx_pubs.clear();
        ch->tx_acks.clear();
        if (m.mid() == 20) {   // commit: apply publishes and acks in order
          bool was = ch->tx;
          ch->tx = false;
          for (auto& p : pubs) {
            Method pm = make_method(60, 40);
            pm.args[1].s = p.exchange;
            pm.args[2].s = p.rk;
            pm.args[3].i = p.mandatory;
            pm.args[4].i = p.immediate;
            on_publish(c, *ch, pm, std::move(p.props), std::move(p.body));
          }
          for (auto& a : acks) {
            u16 mid = std::get<0>(a);
            if (mid == 80) ack(c, *ch, std::get<1>(a), std::get<2>(a));
            else reject(c, *ch, std::get<1>(a), std::get<2>(a), std::get<3>(a));
          }
          ch->tx = was;
          store_.sync();
        }
        send_method(c, ch->id, make_method(90, m.mid() + 1));
      } else {
        throw AmqpError(COMMAND_INVALID, "bad tx method", true, 90, m.mid());
      }
      break;
    }
    default:
      throw AmqpError(COMMAND_INVALID, std::string("unexpected method ") + m.spec->name, true, m.cls(), m.mid());
  }
}

// ------------------------------------------------------------------ connection class
void Broker::on_connection(Conn* c, Method& m) {
  switch (m.mid()) {
    case 11: {   // StartOk (SaslMechanism.scala)
      if (c->state != CS_START_SENT) throw AmqpError(COMMAND_INVALID, "unexpected start-ok", true, 10, 11);
      c->client_props = m.t(0);
      const Value* caps = table_get(c->client_props, "capabilities");
      if (caps && caps->tag == 'F' && caps->t) {
        const Value* b = table_get(*caps->t, "connection.blocked");
        c->cap_blocked = b && b->i;
        const Value* cn = table_get(*caps->t, "consumer_cancel_notify");
        c->cap_cancel_notify = cn && cn->i;
      }
      std::string mech = m.s(1);
      if (mech.empty()) throw AmqpError(CONNECTION_FORCED, "no SASL mechanism", true, 10, 11);
      if (mech == "PLAIN") {
        const std::string& r = m.s(2);   // authzid \0 authcid \0 passwd; no password check (parity)
        size_t a = r.find('\0');
        size_t b = a == std::string::npos ? std::string::npos : r.find('\0', a + 1);
        c->user = (a != std::string::npos) ? r.substr(a + 1, b == std::string::npos ? std::string::npos : b - a - 1) : r;
      } else if (mech == "EXTERNAL" || mech == "AMQPLAIN") {
        c->user = "";
      } else {
        throw AmqpError(ACCESS_REFUSED, "unsupported SASL mechanism " + mech, true, 10, 11);
      }
      Method t = make_method(10, 30);
      t.args[0].i = cfg_.channel_max;
      t.args[1].i = cfg_.frame_max;
      t.args[2].i = cfg_.heartbeat;
      send_method(c, 0, t);
      c->state = CS_TUNE_SENT;
      break;
    }
    case 21: break;  // SecureOk: never challenged
    case 31: {   // TuneOk (FrameStage.scala:824-851)
      if (c->state != CS_TUNE_SENT) throw AmqpError(COMMAND_INVALID, "unexpected tune-ok", true, 10, 31);
      u32 fm = (u32)m.i(1);
      if (fm == 0) fm = cfg_.frame_max;
      if (fm > cfg_.frame_max || fm < cfg_.frame_min)
        throw AmqpError(SYNTAX_ERROR, "frame-max " + std::to_string(fm) + " outside negotiated range", true, 10, 31);
      c->frame_max = fm;
      c->parser.set_frame_max(fm);
      u32 cm = (u32)m.i(0);
      c->channel_max = (cm == 0 || cm > 65535) ? 65535 : (u16)cm;
      if (cfg_.channel_max && c->channel_max > cfg_.channel_max) c->channel_max = cfg_.channel_max;
      c->heartbeat = (u16)m.i(2);
      break;
    }
    case 40: {   // Open
      if (c->state != CS_TUNE_SENT) throw AmqpError(COMMAND_INVALID, "unexpected open", true, 10, 40);
      std::string vh = m.s(0);
      if (!vh.empty() && vh[0] == '/') vh = vh.substr(1);
      if (vh.empty()) vh = cfg_.default_vhost;
      Vhost* v = vhost(vh, false);
      if (!v) throw AmqpError(NOT_FOUND, "no vhost '" + vh + "'", true, 10, 40);
      if (!v->active) throw AmqpError(NOT_ALLOWED, "vhost '" + vh + "' is not active", true, 10, 40);
      c->vhost = v;
      c->state = CS_OPEN;
      Method ok = make_method(10, 41);
      ok.args[0].s = "";
      send_method(c, 0, ok);
      break;
    }
    case 50: {   // Close
      send_method(c, 0, make_method(10, 51));
      close_conn(c);
      c->state = CS_CLOSING;
      c->close_deadline = now_ms();
      break;
    }
    case 51: c->dead = true; break;
    case 60: case 61: break;   // Blocked/Unblocked from a client: ignore
    default: throw AmqpError(COMMAND_INVALID, "bad connection method", true, 10, m.mid());
  }
}

// ------------------------------------------------------------------ channel class
void Broker::on_channel(Conn* c, u16 chid, Method& m) {
  switch (m.mid()) {
    case 10: {
      if (c->channels.count(chid)) throw AmqpError(CHANNEL_ERROR, "channel already open", true, 20, 10);
      if (chid > c->channel_max) throw AmqpError(CHANNEL_ERROR, "channel id above channel-max", true, 20, 10);
      Channel& ch = c->channels[chid];
      ch.id = chid;
      ++stats_.channels;
      Method ok = make_method(20, 11);
      ok.args[0].s = std::to_string(chid);
      send_method(c, chid, ok);
      break;
    }
    case 20: {   // Flow from client: pause/resume deliveries
      Channel& ch = c->channels[chid];
      ch.flow_out = m.b(0);
      Method ok = make_method(20, 21);
      ok.args[0].i = ch.flow_out;
      send_method(c, chid, ok);
      if (ch.flow_out)
        for (auto& kv : ch.consumers) mark_dirty(kv.second->q);
      break;
    }
    case 21: c->channels[chid].flow_in = m.b(0); break;
    case 40: {
      Channel& ch = c->channels[chid];
      close_channel_state(c, ch);
      send_method(c, chid, make_method(20, 41));
      c->channels.erase(chid);
      break;
    }
    case 41: c->channels.erase(chid); break;
    default: throw AmqpError(COMMAND_INVALID, "bad channel method", true, 20, m.mid());
  }
}

// ------------------------------------------------------------------ entities
Vhost* Broker::vhost(const std::string& name, bool create) {
  auto it = vhosts_.find(name);
  if (it != vhosts_.end()) return it->second.get();
  if (!create) return nullptr;
  auto v = std::make_unique<Vhost>();
  v->name = name;
  Vhost* p = v.get();
  vhosts_[name] = std::move(v);
  ensure_standard_exchanges(p);
  return p;
}

void Broker::ensure_standard_exchanges(Vhost* v) {
  static const std::pair<const char*, const char*> X[] = {{"", "direct"},           {"amq.direct", "direct"},
                                                         {"amq.fanout", "fanout"}, {"amq.topic", "topic"},
                                                         {"amq.headers", "headers"}, {"amq.match", "headers"}};
  for (auto& x : X) {
    if (v->exchanges.count(x.first)) continue;
    auto e = std::make_unique<Exchange>();
    e->vhost = v->name;
    e->name = x.first;
    e->type = x.second;
    e->durable = true;
    e->id = entity_id(v->name, x.first);
    v->exchanges[x.first] = std::move(e);
  }
}

Exchange* Broker::find_exchange(Vhost* v, const std::string& name) {
  auto it = v->exchanges.find(name);
  return it == v->exchanges.end() ? nullptr : it->second.get();
}

Queue* Broker::find_queue(Vhost* v, const std::string& name) {
  auto it = v->queues.find(name);
  return it == v->queues.end() ? nullptr : it->second.get();
}

static bool is_reserved(const std::string& n) { return n.rfind("amq.", 0) == 0 || n.rfind("amp.", 0) == 0; }

void Broker::persist_exchange(Exchange* x) {
  if (!x->durable || x->name.empty() || x->name.rfind("amq.", 0) == 0) return;
  ExchangeRow r;
  r.tpe = x->type;
  r.durable = x->durable;
  r.autodel = x->auto_delete;
  r.internal = x->internal;
  r.args = table_to_map(x->args);
  store_.insertExchange(x->id, r);
}

void Broker::persist_bind(Exchange* x, const Binding& b) {
  if (!x->durable || !b.q || !b.q->durable) return;
  store_.insertBind(x->id, b.q->id, b.key, table_to_map(b.args));
}

void Broker::persist_queue_meta(Queue* q) {
  if (!q->durable) return;
  std::set<std::string> cons;
  for (Consumer* c : q->consumers)   // AMQConsumer.globalId = "$connId-$chanId-$tag"
    cons.insert(std::to_string(c->conn->id) + "-" + std::to_string(c->ch) + "-" + c->tag);
  // rows with offset > lconsumed are live; requeued messages sit at the front with their
  // original (smallest) offsets, so lconsumed = front offset - 1
  i64 lconsumed = q->ready.empty() ? q->next_offset - 1 : q->ready.front().offset - 1;
  store_.insertQueueMeta(q->id, lconsumed, cons, true, q->ttl);
}

void Broker::on_exchange(Conn* c, Channel& ch, Method& m) {
  Vhost* v = c->vhost;
  switch (m.mid()) {
    case 10: {   // Declare
      const std::string& name = m.s(1);
      const std::string& type = m.s(2);
      bool passive = m.b(3), durable = m.b(4), autodel = m.b(5), internal = m.b(6), nowait = m.b(7);
      Exchange* x = find_exchange(v, name);
      if (passive) {
        if (!x) throw AmqpError(NOT_FOUND, "no exchange '" + name + "' in vhost '" + v->name + "'", false, 40, 10);
      } else if (x) {
        if (x->type != type)
          throw AmqpError(PRECONDITION_FAILED, "inequivalent arg 'type' for exchange '" + name + "'", false, 40, 10);
      } else {
        if (name.empty() || name.rfind("amq.", 0) == 0)
          throw AmqpError(ACCESS_REFUSED, "exchange name '" + name + "' contains reserved prefix 'amq.'", false, 40, 10);
        if (type != "direct" && type != "fanout" && type != "topic" && type != "headers")
          throw AmqpError(COMMAND_INVALID, "unknown exchange type '" + type + "'", true, 40, 10);
        auto e = std::make_unique<Exchange>();
        e->vhost = v->name;
        e->name = name;
        e->type = type;
        e->durable = durable;
        e->auto_delete = autodel;
        e->internal = internal;
        e->args = m.t(8);
        e->id = entity_id(v->name, name);
        x = e.get();
        v->exchanges[name] = std::move(e);
        persist_exchange(x);
      }
      if (!nowait) send_method(c, ch.id, make_method(40, 11));
      break;
    }
    case 20: {   // Delete: remove bindings only (SURVEY A.Q7: the reference force-deletes queues)
      const std::string& name = m.s(1);
      bool if_unused = m.b(2), nowait = m.b(3);
      Exchange* x = find_exchange(v, name);
      if (!x) throw AmqpError(NOT_FOUND, "no exchange '" + name + "'", false, 40, 20);
      if (name.empty() || name.rfind("amq.", 0) == 0)
        throw AmqpError(ACCESS_REFUSED, "cannot delete reserved exchange", false, 40, 20);
      if (if_unused && !x->bindings.empty())
        throw AmqpError(PRECONDITION_FAILED, "exchange '" + name + "' in use", false, 40, 20);
      delete_exchange(x);
      if (!nowait) send_method(c, ch.id, make_method(40, 21));
      break;
    }
    case 30: case 40: {   // exchange-to-exchange Bind / Unbind (RabbitMQ extension)
      Exchange* dst = find_exchange(v, m.s(1));
      Exchange* src = find_exchange(v, m.s(2));
      if (!dst || !src) throw AmqpError(NOT_FOUND, "no such exchange", false, 40, m.mid());
      const std::string& key = m.s(3);
      auto& bs = src->bindings;
      auto it = std::find_if(bs.begin(), bs.end(), [&](const Binding& b) { return b.x == dst && b.key == key; });
      if (m.mid() == 30) {
        if (it == bs.end()) {
          Binding b;
          b.key = key;
          b.x = dst;
          b.words = split_words(key);
          b.args = m.t(5);
          bs.push_back(b);
        }
      } else if (it != bs.end()) {
        bs.erase(it);
      }
      src->reindex();
      if (!m.b(4)) send_method(c, ch.id, make_method(40, m.mid() == 30 ? 31 : 51));
      break;
    }
    default: throw AmqpError(COMMAND_INVALID, "bad exchange method", true, 40, m.mid());
  }
}

void Broker::delete_exchange(Exchange* x) {
  Vhost* v = vhost(x->vhost, false);
  for (auto& kv : v->exchanges) {   // drop e2e bindings pointing at x
    auto& bs = kv.second->bindings;
    size_t before = bs.size();
    bs.erase(std::remove_if(bs.begin(), bs.end(), [&](const Binding& b) { return b.x == x; }), bs.end());
    if (bs.size() != before) kv.second->reindex();
  }
  if (x->durable) store_.deleteExchange(x->id);
  v->exchanges.erase(x->name);
}

void Broker::on_queue(Conn* c, Channel& ch, Method& m) {
  Vhost* v = c->vhost;
  auto check_excl = [&](Queue* q, u16 mid) {
    if (q->exclusive && q->owner != c)
      throw AmqpError(RESOURCE_LOCKED, "queue '" + q->name + "' is exclusive to another connection", false, 50, mid);
  };
  switch (m.mid()) {
    case 10: {   // Declare
      std::string name = m.s(1);
      bool passive = m.b(2), durable = m.b(3), exclusive = m.b(4), autodel = m.b(5), nowait = m.b(6);
      if (name.empty()) {   // server-named queue: "tmp." + uuid (FrameStage.scala:1036-1041)
        static std::mt19937_64 rng(std::random_device{}());
        char b[40];
        snprintf(b, sizeof b, "tmp.%016llx%016llx", (unsigned long long)rng(), (unsigned long long)rng());
        name = b;
      }
      Queue* q = find_queue(v, name);
      if (passive) {
        if (!q) throw AmqpError(NOT_FOUND, "no queue '" + name + "' in vhost '" + v->name + "'", false, 50, 10);
        check_excl(q, 10);
      } else if (q) {
        check_excl(q, 10);
      } else {
        if (is_reserved(name))
          throw AmqpError(ACCESS_REFUSED, "queue name '" + name + "' contains reserved prefix", false, 50, 10);
        auto nq = std::make_unique<Queue>();
        nq->vhost = v->name;
        nq->name = name;
        nq->id = entity_id(v->name, name);
        nq->durable = durable;
        nq->exclusive = exclusive;
        nq->auto_delete = autodel;
        nq->args = m.t(7);
        if (exclusive) { nq->owner = c; c->exclusive_queues.insert(nq.get()); }
        const Value* ttl = table_get(nq->args, "x-message-ttl");   // Int or Long (FrameStage.scala:1047-1051)
        i64 t;
        if (ttl && value_as_int(*ttl, &t) && t >= 0) nq->ttl = t;
        q = nq.get();
        v->queues[name] = std::move(nq);
        persist_queue_meta(q);
      }
      if (!nowait) {
        Method ok = make_method(50, 11);
        ok.args[0].s = name;
        ok.args[1].i = (i64)q->ready.size();
        ok.args[2].i = (i64)q->consumers.size();
        send_method(c, ch.id, ok);
      }
      break;
    }
    case 20: case 50: {   // Bind / Unbind
      const std::string& qn = m.s(1);
      const std::string& xn = m.s(2);
      const std::string& key = m.s(3);
      Queue* q = find_queue(v, qn);
      Exchange* x = find_exchange(v, xn);
      if (!q) throw AmqpError(NOT_FOUND, "no queue '" + qn + "'", false, 50, m.mid());
      if (!x) throw AmqpError(NOT_FOUND, "no exchange '" + xn + "'", false, 50, m.mid());
      if (xn.empty()) throw AmqpError(ACCESS_REFUSED, "operation not permitted on the default exchange", false, 50, m.mid());
      check_excl(q, m.mid());
      auto& bs = x->bindings;
      auto it = std::find_if(bs.begin(), bs.end(), [&](const Binding& b) { return b.q == q && b.key == key; });
      if (m.mid() == 20) {
        if (it == bs.end()) {
          Binding b;
          b.key = key;
          b.q = q;
          b.words = split_words(key);
          b.args = m.t(5);
          bs.push_back(b);
          persist_bind(x, bs.back());
        }
        x->reindex();
        if (!m.b(4)) send_method(c, ch.id, make_method(50, 21));
      } else {
        if (it != bs.end()) {
          if (x->durable && q->durable) store_.deleteBind(x->id, q->id, key);
          bs.erase(it);
        }
        x->reindex();
        if (x->auto_delete && x->bindings.empty()) delete_exchange(x);
        send_method(c, ch.id, make_method(50, 51));
      }
      break;
    }
    case 30: {   // Purge (ready messages only)
      Queue* q = find_queue(v, m.s(1));
      if (!q) throw AmqpError(NOT_FOUND, "no queue '" + m.s(1) + "'", false, 50, 30);
      check_excl(q, 30);
      u64 n = q->ready.size();
      while (!q->ready.empty()) {
        QEntry e = std::move(q->ready.front());
        q->ready.pop_front();
        release(q->name, v, e.m, e.offset, false);
      }
      if (!m.b(2)) {
        Method ok = make_method(50, 31);
        ok.args[0].i = (i64)n;
        send_method(c, ch.id, ok);
      }
      break;
    }
    case 40: {   // Delete (if_unused / if_empty honoured: SURVEY A.Q8)
      Queue* q = find_queue(v, m.s(1));
      u64 n = 0;
      if (q) {
        check_excl(q, 40);
        if (m.b(2) && !q->consumers.empty())
          throw AmqpError(PRECONDITION_FAILED, "queue '" + q->name + "' in use", false, 50, 40);
        if (m.b(3) && !q->ready.empty())
          throw AmqpError(PRECONDITION_FAILED, "queue '" + q->name + "' not empty", false, 50, 40);
        n = q->ready.size();
        delete_queue(q, true);
      }
      if (!m.b(4)) {
        Method ok = make_method(50, 41);
        ok.args[0].i = (i64)n;
        send_method(c, ch.id, ok);
      }
      break;
    }
    default: throw AmqpError(COMMAND_INVALID, "bad queue method", true, 50, m.mid());
  }
}

void Broker::unbind_queue_everywhere(Queue* q) {
  Vhost* v = vhost(q->vhost, false);
  for (auto& kv : v->exchanges) {
    Exchange* x = kv.second.get();
    auto& bs = x->bindings;
    size_t before = bs.size();
    bs.erase(std::remove_if(bs.begin(), bs.end(), [&](const Binding& b) { return b.q == q; }), bs.end());
    if (bs.size() != before) x->reindex();
  }
  if (q->durable) store_.deleteBindsOfQueue(q->id);
}

void Broker::delete_queue(Queue* q, bool notify) {
  Vhost* v = vhost(q->vhost, false);
  // consumers: server-side cancel (Basic.Cancel if the client understands it)
  std::vector<Consumer*> cs = q->consumers;
  for (Consumer* cons : cs) {
    Conn* cc = cons->conn;
    auto it = cc->channels.find(cons->ch);
    if (it == cc->channels.end()) continue;
    std::string tag = cons->tag;
    cancel_consumer(cc, it->second, tag, notify && cc->cap_cancel_notify);
  }
  while (!q->ready.empty()) {
    QEntry e = std::move(q->ready.front());
    q->ready.pop_front();
    release(q->name, v, e.m, e.offset, false);
  }
  unbind_queue_everywhere(q);
  if (q->durable) store_.pendingDeleteQueue(q->id);
  if (q->owner) q->owner->exclusive_queues.erase(q);
  dirty_.erase(q);
  v->queues.erase(q->name);   // unacked deliveries keep their MsgPtr; acks find no queue
}

// ------------------------------------------------------------------ routing
static bool headers_match(const Table& bargs, const Props& pr) {
  std::string mode = "all";
  const Value* xm = table_get(bargs, "x-match");
  if (xm) mode = table_str(*xm);
  int want = 0, hit = 0;
  for (auto& kv : bargs) {
    if (kv.first.rfind("x-", 0) == 0) continue;
    ++want;
    const Value* hv = pr.has_headers ? table_get(pr.headers, kv.first) : nullptr;
    if (hv && (kv.second.tag == 'V' || table_str(*hv) == table_str(kv.second))) ++hit;
  }
  if (mode == "any") return want == 0 || hit > 0;
  return hit == want;
}

void Broker::route(Exchange* x, const std::string& rk, const Props& pr, std::vector<Queue*>& out, int depth) {
  if (depth > 8) return;
  auto add_b = [&](const Binding& b) {
    if (b.q) {
      if (std::find(out.begin(), out.end(), b.q) == out.end()) out.push_back(b.q);
    } else if (b.x && b.x != x) {
      route(b.x, rk, pr, out, depth + 1);
    }
  };
  if (x->name.empty()) {   // default exchange: queue named by the routing key (SURVEY A.Q1 fixed)
    Queue* q = find_queue(vhost(x->vhost, false), rk);
    if (q && std::find(out.begin(), out.end(), q) == out.end()) out.push_back(q);
    return;
  }
  if (x->type == "direct") {
    auto it = x->direct.find(rk);
    if (it != x->direct.end())
      for (size_t i : it->second) add_b(x->bindings[i]);
  } else if (x->type == "fanout") {
    for (auto& b : x->bindings) add_b(b);
  } else if (x->type == "headers") {
    for (auto& b : x->bindings)
      if (headers_match(b.args, pr)) add_b(b);
  } else {
    std::vector<std::string> kw = split_words(rk);
    for (auto& b : x->bindings)
      if (topic_match(b.words, kw, cfg_.hash_wildcard)) add_b(b);
  }
}

// ------------------------------------------------------------------ publish
void Broker::on_publish(Conn* c, Channel& ch, const Method& m, std::string&& props, std::string&& body) {
  if (!ch.flow_in) return;   // publishes on a flow-stopped channel are dropped (FrameStage.scala:351)
  const std::string& xn = m.s(1);
  const std::string& rk = m.s(2);
  bool mandatory = m.b(3), immediate = m.b(4);
  Vhost* v = c->vhost;
  Exchange* x = find_exchange(v, xn);
  if (!x) throw AmqpError(NOT_FOUND, "no exchange '" + xn + "' in vhost '" + v->name + "'", false, 60, 40);
  if (x->internal) throw AmqpError(ACCESS_REFUSED, "cannot publish to internal exchange", false, 60, 40);
  if (body.size() > (size_t)1 << 31) throw AmqpError(CONTENT_TOO_LARGE, "message too large", false, 60, 40);
  Props pr = parse_props(props);
  if (ch.tx) {
    ch.tx_pubs.push_back(PendingPub{xn, rk, mandatory, immediate, std::move(props), std::move(body)});
    return;
  }
  ++stats_.published;
  ++c->published;
  if (ch.confirm) {
    ++ch.pub_seq;
    confirm_conns_.insert(c);
  }
  std::vector<Queue*> qs;
  route(x, rk, pr, qs);
  u16 ret = 0;
  if (qs.empty()) {
    ++stats_.unroutable;
    if (mandatory) ret = NO_ROUTE;
  } else if (immediate) {
    bool any = false;
    for (Queue* q : qs) any |= !q->consumers.empty();
    if (!any) ret = NO_CONSUMERS;   // spec: not enqueued
  }
  if (ret) {
    Method r = make_method(60, 50);
    r.args[0].i = ret;
    r.args[1].s = ret == NO_ROUTE ? "The exchange cannot route the result of a Publish"
                                  : "The exchange cannot deliver to a consumer when the immediate flag is set";
    r.args[2].s = xn;
    r.args[3].s = rk;
    append_method_frame(c->out, ch.id, r);
    append_content(c->out, ch.id, 60, props, body, c->frame_max);
    kick_write(c);
    ++stats_.returned;
    if (ret == NO_CONSUMERS) return;
  }
  if (qs.empty()) return;   // unroutable: freed immediately (SURVEY A.Q30)
  auto msg = std::make_shared<Message>();
  msg->id = ids_.next();
  msg->exchange = xn;
  msg->rk = rk;
  msg->persistent = pr.delivery_mode == 2;
  i64 now = now_ms();
  msg->expire_at = pr.has_expiration ? now + pr.expiration_ms : 0;
  msg->ts_ms = pr.has_timestamp ? (i64)pr.timestamp * 1000 : 0;
  msg->props = std::move(props);
  msg->body = std::move(body);
  ++stats_.routed;
  for (Queue* q : qs) enqueue(q, msg);
  if (mem_alarm_ == false && cfg_.mem_high_watermark && queued_bytes_ > cfg_.mem_high_watermark) check_memory();
}

void Broker::enqueue(Queue* q, const MsgPtr& m, bool redelivered) {
  i64 now = now_ms();
  i64 exp = m->expire_at;
  if (q->ttl > 0) {
    i64 e2 = now + q->ttl;   // effective expiry = min(message, queue) (QueueEntity.scala:290-293)
    exp = exp ? std::min(exp, e2) : e2;
  }
  i64 off = q->next_offset++;
  ++m->refs;
  q->bytes += m->body.size();
  queued_bytes_ += m->body.size();
  ++q->published;
  if (q->durable && m->persistent) {
    if (!m->stored) {
      MsgRow r;
      r.id = (int64_t)m->id;
      r.tstamp = m->ts_ms;
      std::string hdr(10, '\0');   // BasicProperties.writeTo: weight | bodySize | props
      u64 bs = m->body.size();
      for (int i = 0; i < 8; ++i) hdr[2 + i] = (char)(bs >> (56 - 8 * i));
      r.header = hdr + m->props;
      r.body = m->body;
      r.exchange = m->exchange;
      r.routing = m->rk;
      r.durable = true;
      r.refer = m->refs;
      store_.insertMessage(r, m->expire_at ? std::max<i64>(1, m->expire_at - now) : 0);
      m->stored = true;
    } else {
      store_.updateMessageReferCount((int64_t)m->id, m->refs);
    }
    store_.insertQueueMsg(q->id, off, (int64_t)m->id, (int32_t)m->body.size(), exp ? std::max<i64>(1, exp - now) : 0);
  }
  q->ready.push_back(QEntry{m, off, exp, redelivered});
  mark_dirty(q);
}

void Broker::release(const std::string& qname, Vhost* v, const MsgPtr& m, i64 offset, bool was_unacked) {
  --m->refs;
  Queue* q = v ? find_queue(v, qname) : nullptr;
  if (q) q->bytes -= std::min<u64>(q->bytes, m->body.size());
  queued_bytes_ -= std::min<u64>(queued_bytes_, m->body.size());
  if (m->stored) {
    if (m->refs <= 0) store_.deleteMessage((int64_t)m->id);
    else store_.updateMessageReferCount((int64_t)m->id, m->refs);
  }
  if (q && q->durable && m->persistent) {
    if (was_unacked) store_.deleteQueueUnack(q->id, (int64_t)m->id);
    else store_.deleteQueueMsg(q->id, offset);
  }
  if (mem_alarm_ && queued_bytes_ < cfg_.mem_low_watermark) check_memory();
}

void Broker::expire_head(Queue* q, i64 now) {
  Vhost* v = nullptr;
  while (!q->ready.empty() && q->ready.front().expire_at && q->ready.front().expire_at <= now) {
    if (!v) v = vhost(q->vhost, false);
    QEntry e = std::move(q->ready.front());
    q->ready.pop_front();
    ++stats_.expired;
    release(q->name, v, e.m, e.offset, false);
  }
}

// ------------------------------------------------------------------ delivery
bool Broker::consumer_credit(Consumer* c) {
  Conn* cn = c->conn;
  if (cn->state != CS_OPEN || cn->dead) return false;
  auto it = cn->channels.find(c->ch);
  if (it == cn->channels.end()) return false;
  Channel& ch = it->second;
  if (ch.closing || !ch.flow_out) return false;
  if (cn->out.size() - cn->out_pos > OUT_HIGH) return false;
  if (c->no_ack) return true;
  if (ch.prefetch_count) {   // global=false: per consumer; true: per channel (AMQChannel.scala:55-69)
    u32 used = ch.global ? ch.unacked_count : c->unacked;
    if (used >= ch.prefetch_count) return false;
  }
  return true;
}

void Broker::send_deliver(Consumer* c, QEntry& e) {
  Conn* cn = c->conn;
  Channel& ch = cn->channels[c->ch];
  u64 tag = ch.next_tag++;
  Method d = make_method(60, 60);
  d.args[0].s = c->tag;
  d.args[1].i = (i64)tag;
  d.args[2].i = e.redelivered;
  d.args[3].s = e.m->exchange;
  d.args[4].s = e.m->rk;
  append_method_frame(cn->out, ch.id, d);
  append_content(cn->out, ch.id, 60, e.m->props, e.m->body, cn->frame_max);
  kick_write(cn);
  Queue* q = c->q;
  ++q->delivered;
  ++stats_.delivered;
  ++cn->delivered;
  if (c->no_ack) {
    release(q->name, cn->vhost, e.m, e.offset, false);
  } else {
    ch.unacked.emplace(tag, Unacked{e.m, q->name, e.offset, c, c->tag});
    ++ch.unacked_count;
    ++c->unacked;
    ++q->unacked;
    if (q->durable && e.m->persistent) {
      store_.insertQueueUnack(q->id, e.offset, (int64_t)e.m->id, (int32_t)e.m->body.size());
      store_.deleteQueueMsg(q->id, e.offset);
    }
  }
}

void Broker::deliver(Queue* q) {
  expire_head(q, now_ms());
  size_t n = q->consumers.size();
  if (!n) return;
  size_t tried = 0;
  while (!q->ready.empty() && tried < n) {
    n = q->consumers.size();
    if (!n) break;
    Consumer* c = q->consumers[q->rr % n];
    if (consumer_credit(c)) {
      QEntry e = std::move(q->ready.front());
      q->ready.pop_front();
      send_deliver(c, e);
      ++q->rr;   // round-robin (AMQChannel.nextRoundConsumer)
      tried = 0;
    } else {
      ++q->rr;
      ++tried;
    }
  }
}

// ------------------------------------------------------------------ basic class
void Broker::on_basic(Conn* c, Channel& ch, Method& m) {
  Vhost* v = c->vhost;
  switch (m.mid()) {
    case 10: {   // Qos: 0 = unlimited
      ch.prefetch_size = (u32)m.i(0);
      ch.prefetch_count = (u32)m.i(1);
      ch.global = m.b(2);
      send_method(c, ch.id, make_method(60, 11));
      for (auto& kv : ch.consumers) mark_dirty(kv.second->q);
      break;
    }
    case 20: {   // Consume
      const std::string& qn = m.s(1);
      Queue* q = find_queue(v, qn);
      if (!q) throw AmqpError(NOT_FOUND, "no queue '" + qn + "' in vhost '" + v->name + "'", false, 60, 20);
      if (q->exclusive && q->owner != c)
        throw AmqpError(RESOURCE_LOCKED, "queue '" + qn + "' is exclusive", false, 60, 20);
      std::string tag = m.s(2);
      if (tag.empty()) tag = "amq.ctag-" + std::to_string(++ctag_seq_);   // SURVEY A.Q13
      if (ch.consumers.count(tag)) throw AmqpError(NOT_ALLOWED, "consumer tag '" + tag + "' in use", true, 60, 20);
      bool exclusive = m.b(5);
      for (Consumer* o : q->consumers)
        if (o->exclusive) throw AmqpError(ACCESS_REFUSED, "queue has an exclusive consumer", false, 60, 20);
      if (exclusive && !q->consumers.empty())
        throw AmqpError(ACCESS_REFUSED, "cannot obtain exclusive access to queue", false, 60, 20);
      auto cons = std::make_unique<Consumer>();
      cons->tag = tag;
      cons->conn = c;
      cons->ch = ch.id;
      cons->q = q;
      cons->no_ack = m.b(4);
      cons->exclusive = exclusive;
      q->consumers.push_back(cons.get());
      q->had_consumer = true;
      ch.consumers[tag] = std::move(cons);
      persist_queue_meta(q);
      if (!m.b(6)) {
        Method ok = make_method(60, 21);
        ok.args[0].s = tag;
        send_method(c, ch.id, ok);
      }
      mark_dirty(q);
      break;
    }
    case 30: {   // Cancel
      std::string tag = m.s(0);
      cancel_consumer(c, ch, tag, false);
      if (!m.b(1)) {
        Method ok = make_method(60, 31);
        ok.args[0].s = tag;
        send_method(c, ch.id, ok);
      }
      break;
    }
    case 70: {   // Get
      Queue* q = find_queue(v, m.s(1));
      if (!q) throw AmqpError(NOT_FOUND, "no queue '" + m.s(1) + "'", false, 60, 70);
      if (q->exclusive && q->owner != c) throw AmqpError(RESOURCE_LOCKED, "queue is exclusive", false, 60, 70);
      expire_head(q, now_ms());
      if (q->ready.empty()) {
        Method e = make_method(60, 72);
        e.args[0].s = "";
        send_method(c, ch.id, e);
        break;
      }
      QEntry e = std::move(q->ready.front());
      q->ready.pop_front();
      u64 tag = ch.next_tag++;
      Method ok = make_method(60, 71);
      ok.args[0].i = (i64)tag;
      ok.args[1].i = e.redelivered;
      ok.args[2].s = e.m->exchange;
      ok.args[3].s = e.m->rk;
      ok.args[4].i = (i64)q->ready.size();   // real remaining count (SURVEY A.Q15)
      append_method_frame(c->out, ch.id, ok);
      append_content(c->out, ch.id, 60, e.m->props, e.m->body, c->frame_max);
      kick_write(c);
      ++q->delivered;
      ++stats_.delivered;
      if (m.b(2)) {
        release(q->name, v, e.m, e.offset, false);
      } else {   // records the real queue (SURVEY A.Q14)
        ch.unacked.emplace(tag, Unacked{e.m, q->name, e.offset, nullptr, ""});
        ++ch.unacked_count;
        ++q->unacked;
        if (q->durable && e.m->persistent) {
          store_.insertQueueUnack(q->id, e.offset, (int64_t)e.m->id, (int32_t)e.m->body.size());
          store_.deleteQueueMsg(q->id, e.offset);
        }
      }
      break;
    }
    case 80:   // Ack
      if (ch.tx) { ch.tx_acks.emplace_back(80, (u64)m.i(0), m.b(1), false); break; }
      ack(c, ch, (u64)m.i(0), m.b(1));
      break;
    case 90:   // Reject
      if (ch.tx) { ch.tx_acks.emplace_back(90, (u64)m.i(0), false, m.b(1)); break; }
      reject(c, ch, (u64)m.i(0), false, m.b(1));
      break;
    case 120:  // Nack
      if (ch.tx) { ch.tx_acks.emplace_back(120, (u64)m.i(0), m.b(1), m.b(2)); break; }
      reject(c, ch, (u64)m.i(0), m.b(1), m.b(2));
      break;
    case 100: case 110: {   // RecoverAsync / Recover: requeue everything unacked; RecoverOk (A.Q11)
      std::vector<u64> tags;
      for (auto& kv : ch.unacked) tags.push_back(kv.first);
      requeue_unacked(c, ch, tags);
      if (m.mid() == 110) send_method(c, ch.id, make_method(60, 111));
      break;
    }
    default: throw AmqpError(COMMAND_INVALID, std::string("unexpected method ") + m.spec->name, true, 60, m.mid());
  }
}

void Broker::ack(Conn* c, Channel& ch, u64 tag, bool multiple) {
  std::vector<u64> tags;
  if (multiple) {
    auto end = tag == 0 ? ch.unacked.end() : ch.unacked.upper_bound(tag);
    for (auto it = ch.unacked.begin(); it != end; ++it) tags.push_back(it->first);
  } else {
    if (!ch.unacked.count(tag))
      throw AmqpError(PRECONDITION_FAILED, "unknown delivery tag " + std::to_string(tag), false, 60, 80);
    tags.push_back(tag);
  }
  for (u64 t : tags) {
    auto it = ch.unacked.find(t);
    Unacked u = std::move(it->second);
    ch.unacked.erase(it);
    --ch.unacked_count;
    auto ci = ch.consumers.find(u.ctag);
    if (ci != ch.consumers.end() && ci->second->unacked) --ci->second->unacked;
    Queue* q = find_queue(c->vhost, u.qname);
    if (q) {
      --q->unacked;
      ++q->acked;
      mark_dirty(q);
    }
    ++stats_.acked;
    release(u.qname, c->vhost, u.m, u.offset, true);
  }
  if (ch.global)
    for (auto& kv : ch.consumers) mark_dirty(kv.second->q);
}

void Broker::reject(Conn* c, Channel& ch, u64 tag, bool multiple, bool requeue) {
  std::vector<u64> tags;
  if (multiple) {
    auto end = tag == 0 ? ch.unacked.end() : ch.unacked.upper_bound(tag);
    for (auto it = ch.unacked.begin(); it != end; ++it) tags.push_back(it->first);
  } else {
    if (!ch.unacked.count(tag))
      throw AmqpError(PRECONDITION_FAILED, "unknown delivery tag " + std::to_string(tag), false, 60, 90);
    tags.push_back(tag);
  }
  if (requeue) {
    requeue_unacked(c, ch, tags);
    return;
  }
  for (u64 t : tags) {   // drop (no dead-lettering)
    auto it = ch.unacked.find(t);
    Unacked u = std::move(it->second);
    ch.unacked.erase(it);
    --ch.unacked_count;
    auto ci = ch.consumers.find(u.ctag);
    if (ci != ch.consumers.end() && ci->second->unacked) --ci->second->unacked;
    Queue* q = find_queue(c->vhost, u.qname);
    if (q) { --q->unacked; mark_dirty(q); }
    release(u.qname, c->vhost, u.m, u.offset, true);
  }
}

// back to the queue head in original offset order, redelivered (QueueEntity.scala:415-446)
void Broker::requeue_unacked(Conn* c, Channel& ch, std::vector<u64> tags) {
  std::map<Queue*, std::vector<QEntry>> byq;
  for (u64 t : tags) {
    auto it = ch.unacked.find(t);
    if (it == ch.unacked.end()) continue;
    Unacked u = std::move(it->second);
    ch.unacked.erase(it);
    --ch.unacked_count;
    auto ci = ch.consumers.find(u.ctag);
    if (ci != ch.consumers.end() && ci->second->unacked) --ci->second->unacked;   // A.Q32 fixed
    Queue* q = find_queue(c->vhost, u.qname);
    if (!q) { release(u.qname, c->vhost, u.m, u.offset, true); continue; }
    --q->unacked;
    ++stats_.requeued;
    if (q->durable && u.m->persistent) {
      store_.deleteQueueUnack(q->id, (int64_t)u.m->id);
      store_.insertQueueMsg(q->id, u.offset, (int64_t)u.m->id, (int32_t)u.m->body.size(), 0);
    }
    byq[q].push_back(QEntry{u.m, u.offset, u.m->expire_at, true});
  }
  for (auto& kv : byq) {
    auto& v = kv.second;
    std::sort(v.begin(), v.end(), [](const QEntry& a, const QEntry& b) { return a.offset < b.offset; });
    for (auto it = v.rbegin(); it != v.rend(); ++it) kv.first->ready.push_front(std::move(*it));
    persist_queue_meta(kv.first);
    mark_dirty(kv.first);
  }
}

void Broker::cancel_consumer(Conn* c, Channel& ch, const std::string& tag, bool notify) {
  auto it = ch.consumers.find(tag);
  if (it == ch.consumers.end()) return;
  Consumer* cons = it->second.get();
  Queue* q = cons->q;
  auto& v = q->consumers;
  v.erase(std::remove(v.begin(), v.end(), cons), v.end());
  for (auto& kv : ch.unacked)
    if (kv.second.c == cons) kv.second.c = nullptr;
  if (notify) {
    Method m = make_method(60, 30);
    m.args[0].s = tag;
    m.args[1].i = 0;
    send_method(c, ch.id, m);
  }
  ch.consumers.erase(it);
  persist_queue_meta(q);
  if (q->auto_delete && q->had_consumer && q->consumers.empty()) delete_queue(q, false);
}

void Broker::close_channel_state(Conn* c, Channel& ch) {
  std::vector<std::string> tags;
  for (auto& kv : ch.consumers) tags.push_back(kv.first);
  for (auto& t : tags) cancel_consumer(c, ch, t, false);
  std::vector<u64> ut;
  for (auto& kv : ch.unacked) ut.push_back(kv.first);
  requeue_unacked(c, ch, ut);   // unacked deliveries of a closed channel are requeued
  ch.tx_pubs.clear();
  ch.tx_acks.clear();
  ch.have_method = ch.have_header = false;
}

// ------------------------------------------------------------------ confirms / back-pressure
void Broker::confirm_flush() {
  if (confirm_conns_.empty()) return;
  store_.sync();   // confirms for persistent messages only after the durable write
  for (Conn* c : confirm_conns_) {
    for (auto& kv : c->channels) {
      Channel& ch = kv.second;
      if (!ch.confirm || ch.pub_seq <= ch.confirmed || ch.closing) continue;
      Method a = make_method(60, 80);
      a.args[0].i = (i64)ch.pub_seq;
      a.args[1].i = (ch.pub_seq - ch.confirmed) > 1;
      send_method(c, ch.id, a);
      stats_.confirms += ch.pub_seq - ch.confirmed;
      ch.confirmed = ch.pub_seq;
    }
  }
  confirm_conns_.clear();
}

void Broker::check_memory() {
  if (!cfg_.mem_high_watermark) return;
  bool alarm = queued_bytes_ > cfg_.mem_high_watermark ||
               (mem_alarm_ && queued_bytes_ > cfg_.mem_low_watermark);
  if (alarm == mem_alarm_) return;
  mem_alarm_ = alarm;
  for (auto& kv : conns_) {
    Conn* c = kv.second.get();
    if (c->state != CS_OPEN || c->published == 0) continue;   // block publishers only
    if (cfg_.flow_channel) {
      for (auto& chkv : c->channels) {
        Method f = make_method(20, 20);
        f.args[0].i = alarm ? 0 : 1;
        send_method(c, chkv.first, f);
      }
    } else if (c->cap_blocked) {
      if (alarm) {
        Method b = make_method(10, 60);
        b.args[0].s = "low on memory";
        send_method(c, 0, b);
      } else {
        send_method(c, 0, make_method(10, 61));
      }
    }
    c->blocked = alarm;
    epoll_event ev{};
    ev.events = (alarm ? 0 : EPOLLIN) | EPOLLOUT;
    ev.data.fd = c->fd;
    epoll_ctl(epfd_, EPOLL_CTL_MOD, c->fd, &ev);
    if (!alarm && c->in.size() > c->in_pos) process_input(c);
  }
}

// ------------------------------------------------------------------ recovery
void Broker::recover() {
  if (!store_.persistent()) return;
  auto split_id = [](const std::string& id, std::string* vh, std::string* name) {
    size_t p = id.find("-_.");
    if (p == std::string::npos) { *vh = ""; *name = id; }
    else { *vh = id.substr(0, p); *name = id.substr(p + 3); }
  };
  for (auto& vid : store_.vhostIds()) {
    bool active = true;
    store_.selectVhost(vid, &active);
    vhost(vid, true)->active = active;
  }
  std::map<int64_t, MsgPtr> msgs;
  auto load_msg = [&](int64_t id) -> MsgPtr {
    auto it = msgs.find(id);
    if (it != msgs.end()) return it->second;
    MsgRow r;
    if (!store_.selectMessage(id, &r)) return nullptr;
    auto m = std::make_shared<Message>();
    m->id = (u64)r.id;
    m->exchange = r.exchange;
    m->rk = r.routing;
    m->props = r.header.size() >= 10 ? r.header.substr(10) : std::string("\0\0", 2);
    m->body = r.body;
    m->persistent = true;
    m->stored = true;
    m->ts_ms = r.tstamp;
    m->expire_at = r.expire_at;
    msgs[id] = m;
    return m;
  };
  for (auto& qid : store_.queueIds()) {
    QueueMetaRow meta;
    std::vector<QueueMsgRow> rows, unacks;
    if (!store_.selectQueue(qid, &meta, &rows, &unacks)) continue;
    std::string vh, name;
    split_id(qid, &vh, &name);
    Vhost* v = vhost(vh.empty() ? cfg_.default_vhost : vh, true);
    auto q = std::make_unique<Queue>();
    q->vhost = v->name;
    q->name = name;
    q->id = qid;
    q->durable = true;
    q->ttl = meta.ttl;
    // orphaned unacks are requeued first, redelivered (fixes SURVEY §3.6 / A.Q31)
    std::sort(unacks.begin(), unacks.end(), [](const QueueMsgRow& a, const QueueMsgRow& b) { return a.offset < b.offset; });
    i64 maxoff = meta.lconsumed;
    for (auto& u : unacks) {
      MsgPtr m = load_msg(u.msgid);
      if (!m) continue;
      ++m->refs;
      q->ready.push_back(QEntry{m, u.offset, m->expire_at, true});
      queued_bytes_ += m->body.size();
      maxoff = std::max<i64>(maxoff, u.offset);
      store_.deleteQueueUnack(qid, u.msgid);
      store_.insertQueueMsg(qid, u.offset, u.msgid, u.size, 0);
    }
    for (auto& r : rows) {
      MsgPtr m = load_msg(r.msgid);
      if (!m) continue;
      ++m->refs;
      q->ready.push_back(QEntry{m, r.offset, r.expire_at, false});
      queued_bytes_ += m->body.size();
      maxoff = std::max<i64>(maxoff, r.offset);
    }
    q->next_offset = maxoff + 1;
    v->queues[name] = std::move(q);
  }
  for (auto& xid : store_.exchangeIds()) {
    ExchangeRow xr;
    std::vector<BindRow> binds;
    if (!store_.selectExchange(xid, &xr, &binds)) continue;
    std::string vh, name;
    split_id(xid, &vh, &name);
    Vhost* v = vhost(vh.empty() ? cfg_.default_vhost : vh, true);
    Exchange* x = find_exchange(v, name);
    if (!x) {
      auto e = std::make_unique<Exchange>();
      e->vhost = v->name;
      e->name = name;
      e->type = xr.tpe;
      e->durable = true;
      e->auto_delete = xr.autodel;
      e->internal = xr.internal;
      e->id = xid;
      x = e.get();
      v->exchanges[name] = std::move(e);
    }
    for (auto& b : binds) {   // re-subscribe (ExchangeEntity.scala:137-165)
      std::string qvh, qname;
      split_id(b.queue, &qvh, &qname);
      Queue* q = find_queue(v, qname);
      if (!q) continue;
      Binding bb;
      bb.key = b.key;
      bb.q = q;
      bb.words = split_words(b.key);
      for (auto& kv : b.args) bb.args.emplace_back(kv.first, Value::str(kv.second));
      x->bindings.push_back(bb);
    }
    x->reindex();
  }
  for (auto& kv : msgs)   // refer counts as recovered
    store_.updateMessageReferCount(kv.first, kv.second->refs);
  store_.sync();
}

}  // namespace cmq

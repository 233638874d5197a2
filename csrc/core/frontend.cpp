#include "frontend.hpp"

#include "persist.hpp"
#include "../kernels/xchg_host.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <pthread.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/ioctl.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace cmq {

namespace {
i64 now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
i64 wall_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}
double secs_since(i64 t0) { return (now_ns() - t0) * 1e-9; }
// marks the stepper as blocked on the GPU (step results, egress copies) for healthy()
struct GpuWait {
  std::atomic<i64>& since;
  explicit GpuWait(std::atomic<i64>& s) : since(s) { since = now_ns(); }
  ~GpuWait() { since = 0; }
};
const char HEARTBEAT_FRAME[8] = {8, 0, 0, 0, 0, 0, 0, (char)0xCE};
constexpr u64 LISTENER = ~0ull, WAKE = ~0ull - 1;
}  // namespace

enum : int { M_FREE = 0, M_HOST = 1, M_DATA = 2, M_DEAD = 3 };

struct FeConn {
  int fd = -1;
  u32 id = 0;
  int io = 0;
  std::atomic<int> mode{M_FREE};
  std::atomic<u32> gen{0};   // bumped when the slot is freed: egress of older steps is stale
  // IO-thread owned
  bool in_ready = false;
  bool rdhup = false;
  // guarded by mu
  std::mutex mu;
  std::string out;
  size_t out_pos = 0;
  std::string inject;    // bytes for the data plane ahead of the socket's (handshake leftovers)
  std::string hostbuf;   // host-mode bytes not yet taken by the control plane
  bool host_notified = false;
  // stepper-owned: read by IO threads only inside the gather phase, by the control plane
  // only while paused
  u32 carry = 0, inflight = 0;
  bool paused = false, kicked = false;
  u64 inj_step = 0;       // the step whose gather took the last inject() bytes (FE_INJECTED)
  bool wblocked = false;  // egress back-pressure flag raised on the device (mu held)
  // heartbeats
  std::atomic<i64> last_rx{0}, last_tx{0};
  std::atomic<u32> hb_s{0};
  // per-connection read budget per step (0: the front end's per_conn_read); the control
  // plane lowers it for publisher-confirm channels (set_read_cap)
  std::atomic<u64> read_cap{0};
};

struct FeIo {
  int epfd = -1, evfd = -1;
  std::thread th;
  std::mutex qmu;
  std::vector<u32> adopt;     // new connections to register (accepted by thread 0)
  std::vector<u32> pending;   // connections to put on the ready list (kick / data mode)
  std::vector<u32> closing;   // close() requests
  std::vector<u32> ready;     // data connections with unread socket bytes or pending input
  std::vector<u32> owned;
  std::vector<SegIn> segs;    // this phase's gathered segments
  u64 phase_seen = 0;
  i64 last_hb = 0;
};

static void poke(int evfd) {
  u64 one = 1;
  ssize_t r = ::write(evfd, &one, 8);
  (void)r;
}

// ============================================================================ lifecycle
Frontend::Frontend(const FrontendCfg& cfg, const CmqEngineApi* api) : cfg_(cfg), api_(api) {
  if (!api_ || api_->abi != CMQ_STEP_ABI) throw std::runtime_error("frontend: engine C API missing or ABI mismatch");
  c_max_ = api_->c_max;
  held_cnt_.assign(c_max_, 0);
  notify_.reset(new std::atomic<u8>[c_max_]());
  if (cfg_.io_threads < 1) cfg_.io_threads = 1;
  if (!cfg_.max_slot || cfg_.max_slot > c_max_ - 2) cfg_.max_slot = c_max_ - 2;
  conns_.resize(c_max_);
  for (u32 i = 0; i < c_max_; ++i) {
    conns_[i].reset(new FeConn());
    conns_[i]->id = i;
    conns_[i]->io = (int)(i % (u32)cfg_.io_threads);
  }
  for (u32 i = cfg_.max_slot; i >= 1; --i) free_.push_back(i);
  const u64 arena_bytes = ((api_->ingress_cap + 64 + 4095) / 4096) * 4096;
  // egress by reference: deliveries of the same step's bodies (back 0) are sent from the
  // arena they arrived in (NARENA arenas keep it unchanged until that egress is written)
  if (cfg_.egress_ref && api_->set_egress_ref && api_->set_egress_ref(api_->eng, 0, cfg_.egress_ref_min) == 0) {
    narena_ = NARENA;
    ref_on_ = true;
  }
  else if (api_->set_egress_ref)
    api_->set_egress_ref(api_->eng, -1, 0);
  for (int k = 0; k < narena_; ++k) {
    arena_[k] = (u8*)aligned_alloc(4096, arena_bytes);
    if (!arena_[k]) throw std::runtime_error("frontend: arena allocation failed");
    // page-locked: the step's H2D is a DMA straight from the arena (a pageable source is
    // staged through a bounce buffer by a CPU copy inside submit: ~80 us of a 1.7 MB step,
    // measured).  The engine's submit waits for the H2D of the step two back before
    // reusing its buffers, so by the time an arena is gathered into again (three steps
    // later) its copy is done
    if (api_->host_register && api_->host_register(api_->eng, arena_[k], arena_bytes) == 0) arena_pinned_[k] = true;
  }
  lfd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (lfd_ < 0) throw std::runtime_error("frontend: socket failed");
  int one = 1;
  setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  if (cfg_.reuseport) setsockopt(lfd_, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)cfg_.port);
  if (inet_pton(AF_INET, cfg_.host.c_str(), &a.sin_addr) != 1) a.sin_addr.s_addr = htonl(INADDR_ANY);
  if (::bind(lfd_, (sockaddr*)&a, sizeof a) < 0) throw std::runtime_error(std::string("frontend: bind: ") + strerror(errno));
  if (::listen(lfd_, 4096) < 0) throw std::runtime_error("frontend: listen failed");
  socklen_t l = sizeof a;
  getsockname(lfd_, (sockaddr*)&a, &l);
  port_ = ntohs(a.sin_port);
  for (int i = 0; i < cfg_.io_threads; ++i) {
    std::unique_ptr<FeIo> io(new FeIo());
    io->epfd = epoll_create1(EPOLL_CLOEXEC);
    io->evfd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = WAKE;
    epoll_ctl(io->epfd, EPOLL_CTL_ADD, io->evfd, &ev);
    if (i == 0) {
      ev.events = EPOLLIN;
      ev.data.u64 = LISTENER;
      epoll_ctl(io->epfd, EPOLL_CTL_ADD, lfd_, &ev);
    }
    io_.push_back(std::move(io));
  }
}

Frontend::~Frontend() {
  stop();
  {   // (a front end that was attached to a store but never started has its copier only)
    std::lock_guard<std::mutex> g(pc_mu_);
    pc_stop_ = true;
  }
  pc_cv_.notify_all();
  if (pc_th_.joinable()) pc_th_.join();
  for (auto& c : conns_)
    if (c->fd >= 0) ::close(c->fd);
  for (auto& io : io_) {
    if (io->epfd >= 0) ::close(io->epfd);
    if (io->evfd >= 0) ::close(io->evfd);
  }
  if (lfd_ >= 0) ::close(lfd_);
  for (auto* a : arena_) free(a);   // (free(nullptr) for unused ones)
}

void Frontend::start() {
  if (running_.exchange(true)) return;
  for (int i = 0; i < (int)io_.size(); ++i) io_[i]->th = std::thread([this, i] { io_loop(i); });
  if (api_->world > 1 && api_->native_xchg) stepper_ = std::thread([this] { stepper_sharded(); });
  else stepper_ = std::thread([this] { stepper(); });
}

void Frontend::stop() {
  if (!running_.exchange(false)) return;
  {
    std::lock_guard<std::mutex> g(st_mu_);
    wake_ = true;
  }
  st_cv_.notify_all();
  pause_cv_.notify_all();
  {   // an IO phase in progress completes: IO threads finish it before they look at running_
    std::lock_guard<std::mutex> g(ph_mu_);
  }
  if (stepper_.joinable()) stepper_.join();
  for (auto& io : io_) {
    poke(io->evfd);
    if (io->th.joinable()) io->th.join();
  }
  ev_cv_.notify_all();
  {
    std::lock_guard<std::mutex> g(pc_mu_);
    pc_stop_ = true;
  }
  pc_cv_.notify_all();
  if (pc_th_.joinable()) pc_th_.join();   // (drains the queued copies first)
  // the engine is alive until the front end is stopped (and no step is in flight now)
  for (int k = 0; k < narena_; ++k)
    if (arena_pinned_[k]) { api_->host_unregister(api_->eng, arena_[k]); arena_pinned_[k] = false; }
}

bool Frontend::check(int rc) {
  if (rc >= 0) return true;
  FeEvent e;
  e.kind = FE_ERROR;
  e.data = api_->error(api_->eng);
  failed_ = true;
  post(std::move(e));
  return false;
}

void Frontend::post(FeEvent&& e) {
  {
    std::lock_guard<std::mutex> g(ev_mu_);
    events_.push_back(std::move(e));
  }
  ev_cv_.notify_one();
}

void Frontend::wake_stepper() {
  {
    std::lock_guard<std::mutex> g(st_mu_);
    wake_ = true;
  }
  st_cv_.notify_one();
}

// ============================================================================ control-plane API
std::vector<FeEvent> Frontend::poll_events(int timeout_ms) {
  std::unique_lock<std::mutex> g(ev_mu_);
  if (events_.empty() && timeout_ms != 0)
    ev_cv_.wait_for(g, std::chrono::milliseconds(timeout_ms < 0 ? 1000 : timeout_ms),
                    [&] { return !events_.empty() || !running_; });
  std::vector<FeEvent> out(std::make_move_iterator(events_.begin()), std::make_move_iterator(events_.end()));
  events_.clear();
  return out;
}

std::string Frontend::take(u32 conn) {
  if (conn >= c_max_) return {};
  FeConn& c = *conns_[conn];
  std::lock_guard<std::mutex> g(c.mu);
  std::string s;
  s.swap(c.hostbuf);
  c.host_notified = false;
  return s;
}

// egress back-pressure: above wblock_high bytes queued for a socket the device stops
// dequeuing to that connection (its messages wait in HBM); below wblock_low it resumes
void Frontend::wblock_update(FeConn& c) {
  const size_t pend = c.out.size() - c.out_pos;
  if (!c.wblocked && pend > cfg_.wblock_high) {
    c.wblocked = true;
    if (api_->wblock) api_->wblock[c.id] = 1;
  } else if (c.wblocked && pend < cfg_.wblock_low) {
    c.wblocked = false;
    if (api_->wblock) api_->wblock[c.id] = 0;
    wake_stepper();
  }
}

bool Frontend::write_some(FeConn& c) {
  struct WB { Frontend* f; FeConn& c; ~WB() { f->wblock_update(c); } } wb{this, c};
  while (c.out_pos < c.out.size()) {
    ssize_t k = ::send(c.fd, c.out.data() + c.out_pos, c.out.size() - c.out_pos, MSG_NOSIGNAL);
    if (k > 0) {
      c.out_pos += (size_t)k;
      tx_bytes_ += (u64)k;
      continue;
    }
    if (k < 0 && errno == EINTR) continue;
    if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {   // EPOLLOUT edge resumes
      // a consumer that never catches up never empties its queue: drop the sent prefix once
      // it is half the buffer (else the string keeps every byte ever sent to it, and each
      // growth copies them all -- multi-ms stalls of this IO thread in a cold drain)
      if (c.out_pos >= (256u << 10) && 2 * c.out_pos >= c.out.size()) {
        c.out.erase(0, c.out_pos);
        c.out_pos = 0;
      }
      return false;
    }
    c.out.clear();
    c.out_pos = 0;
    return false;   // broken: the IO thread sees EPOLLERR/HUP and drops it
  }
  c.out.clear();
  c.out_pos = 0;
  c.last_tx = now_ns();
  return true;
}

void Frontend::scatter_conn(FeConn& c, const u8* data, u32 n) {
  std::lock_guard<std::mutex> g(c.mu);
  if (c.fd < 0) return;
  if (c.out_pos >= c.out.size()) {   // nothing queued: write straight from the egress slot
    c.out.clear();
    c.out_pos = 0;
    u32 o = 0;
    while (o < n) {
      ssize_t k = ::send(c.fd, data + o, n - o, MSG_NOSIGNAL);
      if (k > 0) { o += (u32)k; continue; }
      if (k < 0 && errno == EINTR) continue;
      break;
    }
    tx_bytes_ += o;
    c.last_tx = now_ns();
    if (o < n) c.out.append((const char*)data + o, n - o);
  } else {
    c.out.append((const char*)data, n);
  }
  wblock_update(c);
}

// first gather entry whose insertion point is at or after `off` (dst never decreases)
static u32 gath_lower(const EgressRef* g, u32 n, u32 off) {
  u32 lo = 0, hi = n;
  while (lo < hi) {
    const u32 mid = (lo + hi) >> 1;
    if (g[mid].dst < off) lo = mid + 1; else hi = mid;
  }
  return lo;
}

void Frontend::scatter_ref(FeConn& c, const u8* base, const ConnOut& o, const Scatter& sc) {
  const EgressRef* g = (const EgressRef*)(base + sc.gath_off);
  const u32 end = o.off + o.len;
  std::vector<iovec> v;
  u32 pos = o.off;
  for (u32 k = gath_lower(g, sc.gath_n, o.off); k < sc.gath_n && g[k].dst < end; ++k) {
    if (!g[k].len) continue;
    if (g[k].dst > pos) v.push_back(iovec{(void*)(base + pos), (size_t)(g[k].dst - pos)});
    v.push_back(iovec{(void*)(uintptr_t)g[k].src, (size_t)g[k].len});
    pos = g[k].dst;
  }
  if (end > pos) v.push_back(iovec{(void*)(base + pos), (size_t)(end - pos)});
  std::lock_guard<std::mutex> gd(c.mu);
  if (c.fd < 0) return;
  size_t i = 0;
  if (c.out_pos >= c.out.size()) {   // nothing queued: straight from the slot and the arena
    c.out.clear();
    c.out_pos = 0;
    u64 sent = 0;
    while (i < v.size()) {
      msghdr m{};
      m.msg_iov = &v[i];
      m.msg_iovlen = std::min<size_t>(v.size() - i, 1024);   // (IOV_MAX)
      ssize_t k = ::sendmsg(c.fd, &m, MSG_NOSIGNAL);
      if (k < 0 && errno == EINTR) continue;
      if (k <= 0) break;
      sent += (u64)k;
      size_t left = (size_t)k;
      while (i < v.size() && left >= v[i].iov_len) { left -= v[i].iov_len; ++i; }
      if (left) { v[i].iov_base = (u8*)v[i].iov_base + left; v[i].iov_len -= left; }
    }
    tx_bytes_ += sent;
    c.last_tx = now_ns();
  }
  for (; i < v.size(); ++i) c.out.append((const char*)v[i].iov_base, v[i].iov_len);   // the rest waits
  wblock_update(c);
}

void Frontend::materialize(Scatter& sc, const u8* egress, u64 bytes) {
  if (!sc.gath_n) {
    sc.own.assign((const char*)egress, bytes);
    sc.egress = nullptr;
    return;
  }
  const EgressRef* g = (const EgressRef*)(egress + sc.gath_off);
  std::string own;
  u32 k = 0;
  for (auto& o : sc.co) {   // (connection regions lie in ascending offset order)
    if (!o.len) continue;
    const u32 start = (u32)own.size(), end = o.off + o.len;
    u32 pos = o.off;
    k = gath_lower(g, sc.gath_n, o.off);
    for (; k < sc.gath_n && g[k].dst < end; ++k) {
      if (!g[k].len) continue;
      own.append((const char*)egress + pos, g[k].dst - pos);
      own.append((const char*)(uintptr_t)g[k].src, g[k].len);
      pos = g[k].dst;
    }
    own.append((const char*)egress + pos, end - pos);
    o = ConnOut{start, (u32)own.size() - start};
  }
  sc.own.swap(own);
  sc.egress = nullptr;
  sc.gath_n = 0;
  sc.gath_off = 0;
}

// the connections a submitted step unpauses get their carries re-presented by the next
// gather (Python kicks them when it stages the unpause, but inside a light section that
// kick can be spent on a step submitted before the batch carrying the unpause closed --
// the connection would then sit paused-free with its next command stuck in the carry)
void Frontend::kick_unpaused(int p) {
  if (!api_->unpaused) return;
  const u32* l = nullptr;
  const u32 n = api_->unpaused(api_->eng, p, &l);
  for (u32 k = 0; k < n && l; ++k) kick(l[k]);
}

// egress by reference for the next submitted step only when it gathered enough bytes
void Frontend::ref_for_step(u64 used) {
  if (narena_ != NARENA) return;
  const bool on = used >= cfg_.egress_ref_step_min;
  if (on == ref_on_) return;
  // (below the threshold spilled bodies still go from the host spill ring: large, and not
  // in HBM -- rendering them would read them across PCIe and send them back again)
  api_->set_egress_ref(api_->eng, on ? 0 : -2, cfg_.egress_ref_min);
  ref_on_ = on;
}

void Frontend::send(u32 conn, const char* data, size_t n) {
  if (conn >= c_max_ || !n) return;
  FeConn& c = *conns_[conn];
  std::lock_guard<std::mutex> g(c.mu);
  if (c.fd < 0) return;
  c.out.append(data, n);
  write_some(c);
}

void Frontend::send_after(u32 conn, const char* data, size_t n) {
  if (conn >= c_max_ || !n) return;
  {
    std::lock_guard<std::mutex> g(ctl_mu_);
    // behind the steps in flight and the next one, which carries the control writes the
    // command staged (Engine::pack_deltas): the reply never overtakes its own table changes.
    // With batch ids: exactly behind the egress of the step that applied the command's
    // write batch -- before the next step's, where a consumer it activated first gets
    // deliveries (k_stage flips cons_active 2 -> 1): no Basic.Deliver before its ConsumeOk
    const u64 batch = api_->dl_state ? api_->dl_state(api_->eng, 0) : 0;
    ctl_out_.push_back(CtlOut{sub_step_.load() + 1, conn, conns_[conn]->gen.load(), std::string(data, n), batch});
  }
  wake_stepper();
}

// (control plane, stepper paused, staged writes applied) every held reply goes out now,
// in order, behind the egress the pause already wrote
void Frontend::flush_ctl() {
  std::deque<CtlOut> go;
  {
    std::lock_guard<std::mutex> g(ctl_mu_);
    go.swap(ctl_out_);
  }
  for (auto& o : go)
    if (o.gen == conns_[o.conn]->gen.load()) send(o.conn, o.data.data(), o.data.size());
}

std::vector<u64> Frontend::ctl_state() {
  std::lock_guard<std::mutex> g(ctl_mu_);
  return {(u64)ctl_out_.size(), ctl_out_.empty() ? 0 : ctl_out_.front().after, sub_step_.load(), fin_step_.load()};
}

// a held reply waits for a step not submitted yet: the stepper must submit one
bool Frontend::ctl_needs_step() {
  std::lock_guard<std::mutex> g(ctl_mu_);
  return !ctl_out_.empty() && ctl_out_.back().after > sub_step_.load();
}

void Frontend::wake() { wake_stepper(); }

bool Frontend::ctl_pending() {
  std::lock_guard<std::mutex> g(ctl_mu_);
  return !ctl_out_.empty();
}

// (stepper) control replies whose steps have all finished go out behind those steps'
// egress: one Scatter at the end of this IO phase's list, in reply order per connection
void Frontend::release_ctl() {
  std::vector<CtlOut> go;
  {
    std::lock_guard<std::mutex> g(ctl_mu_);
    // the egress queued so far covers steps <= out_step_ and write batches <= out_batch_; a
    // connection with bytes in held (write-behind) steps keeps its replies behind them --
    // per connection, so a durable broker whose steps are nearly always held still answers
    // the other connections' control commands (replies keep their order per connection)
    std::vector<u32> blocked;
    for (auto it = ctl_out_.begin(); it != ctl_out_.end();) {
      const u32 c = it->conn;
      const bool ok = it->after <= out_step_ && it->batch <= out_batch_ && (c >= c_max_ || held_cnt_[c] == 0) &&
                      std::find(blocked.begin(), blocked.end(), c) == blocked.end();
      if (!ok) {
        blocked.push_back(c);
        ++it;
        continue;
      }
      go.push_back(std::move(*it));
      it = ctl_out_.erase(it);
    }
  }
  if (go.empty()) return;
  Scatter sc;
  sc.co.assign(c_max_, ConnOut{0, 0});
  sc.gen.assign(c_max_, 0);
  for (u32 c = 0; c < c_max_; ++c) sc.gen[c] = conns_[c]->gen.load();
  // per connection contiguous (its replies keep their order)
  std::vector<std::vector<size_t>> by(c_max_);
  for (size_t k = 0; k < go.size(); ++k) by[go[k].conn].push_back(k);
  for (u32 c = 0; c < c_max_; ++c) {
    if (by[c].empty()) continue;
    const u32 off = (u32)sc.own.size();
    for (size_t k : by[c])
      if (go[k].gen == sc.gen[c]) sc.own += go[k].data;   // (a closed connection's: dropped)
    sc.co[c] = ConnOut{off, (u32)sc.own.size() - off};
  }
  if (!sc.own.empty()) out_.push_back(std::move(sc));
}

void Frontend::send_egress(const u8* egress, const ConnOut* co, u32 n_slots) {
  for (u32 i = 0; i < n_slots && i < c_max_; ++i)
    if (co[i].len) send(i, (const char*)egress + co[i].off, co[i].len);
}

void Frontend::set_data_mode(u32 conn, const std::string& leftover) {
  if (conn >= c_max_) return;
  FeConn& c = *conns_[conn];
  {
    std::lock_guard<std::mutex> g(c.mu);
    if (c.fd < 0) return;
    c.inject = leftover + c.hostbuf;
    c.hostbuf.clear();
    c.host_notified = false;
    c.carry = c.inflight = 0;
    c.paused = false;
    c.kicked = !c.inject.empty();
    c.mode = M_DATA;
  }
  FeIo& io = *io_[c.io];
  {
    std::lock_guard<std::mutex> g(io.qmu);
    io.pending.push_back(conn);
  }
  poke(io.evfd);
  wake_stepper();
}

void Frontend::set_host_mode(u32 conn) {
  if (conn >= c_max_) return;
  FeConn& c = *conns_[conn];
  std::lock_guard<std::mutex> g(c.mu);
  if (c.mode == M_DATA) c.mode = M_HOST;
  c.inject.clear();
  FeIo& io = *io_[c.io];
  std::lock_guard<std::mutex> g2(io.qmu);
  io.pending.push_back(conn);   // its socket may hold bytes: read them as host bytes now
  poke(io.evfd);
}

void Frontend::set_heartbeat(u32 conn, u32 seconds) {
  if (conn < c_max_) conns_[conn]->hb_s = seconds;
}

void Frontend::set_read_cap(u32 conn, u64 bytes) {
  if (conn < c_max_) conns_[conn]->read_cap = bytes;
}

void Frontend::close(u32 conn, i64 gen) {
  if (conn == 0 || conn >= c_max_) return;
  if (gen >= 0 && conns_[conn]->gen.load() != (u32)gen) return;   // a stale close: slot freed since
  FeIo& io = *io_[conns_[conn]->io];
  {
    std::lock_guard<std::mutex> g(io.qmu);
    io.closing.push_back(conn);
  }
  poke(io.evfd);
}

void Frontend::inject(u32 conn, const std::string& bytes) {
  if (conn == 0 || conn >= c_max_) return;
  FeConn& c = *conns_[conn];
  {
    std::lock_guard<std::mutex> g(c.mu);
    c.inject += bytes;
    c.carry = c.inflight = 0;
    c.paused = false;
    c.kicked = true;
    c.mode = M_DATA;
  }
  notify_[conn] = 1;
  FeIo& io = *io_[c.io];
  {
    std::lock_guard<std::mutex> g(io.qmu);
    io.pending.push_back(conn);
  }
  poke(io.evfd);
  wake_stepper();
}

void Frontend::queue_get(u32 conn, u32 chslot, u32 q, u32 noack, u64 id) {
  {
    std::lock_guard<std::mutex> g(get_mu_);
    gets_.push_back(PendGet{GetReq{conn, chslot, q, noack}, id});
  }
  wake_stepper();
}

void Frontend::cancel_gets(u32 conn) {
  std::lock_guard<std::mutex> g(get_mu_);
  gets_.erase(std::remove_if(gets_.begin(), gets_.end(), [&](const PendGet& x) { return x.r.conn == conn; }),
              gets_.end());
}

bool Frontend::gets_pending() {
  std::lock_guard<std::mutex> g(get_mu_);
  return !gets_.empty();
}

// stepper thread, right before api_->submit: the step takes the oldest requests
void Frontend::stage_gets(Inflight& f) {
  if (!api_->stage_gets) return;
  std::vector<GetReq> rs;
  {
    std::lock_guard<std::mutex> g(get_mu_);
    if (gets_.empty()) return;
    const size_t n = std::min<size_t>(gets_.size(), GET_STEP_MAX);
    for (size_t i = 0; i < n; ++i) {
      rs.push_back(gets_[i].r);
      f.gets.emplace_back(gets_[i].r.conn, gets_[i].id);
    }
    gets_.erase(gets_.begin(), gets_.begin() + n);
  }
  if (api_->stage_gets(api_->eng, rs.data(), (u32)rs.size()) != 0) {
    check(-1);
    f.gets.clear();
  }
}

void Frontend::kick(u32 conn) {
  if (conn >= c_max_) return;
  FeConn& c = *conns_[conn];
  c.paused = false;
  c.kicked = true;
  FeIo& io = *io_[c.io];
  {
    std::lock_guard<std::mutex> g(io.qmu);
    io.pending.push_back(conn);
  }
  wake_stepper();
}

void Frontend::pause() {
  std::unique_lock<std::mutex> g(st_mu_);
  ++pause_req_;
  wake_ = true;
  st_cv_.notify_all();
  pause_cv_.wait(g, [&] { return paused_ || !running_ || failed_; });
}

void Frontend::resume() {
  {
    std::lock_guard<std::mutex> g(st_mu_);
    if (pause_req_ > 0) --pause_req_;
    wake_ = true;
  }
  st_cv_.notify_all();
}

void Frontend::release(u64 step) {
  u64 cur = released_.load();
  while (step > cur && !released_.compare_exchange_weak(cur, step)) {
  }
  have_released_ = true;
  wake_stepper();
}

void Frontend::attach_persist(PersistWorker* w) {
  persist_ = w;
  w->on_commit([this](u64 step) { release(step); });
  if (!pc_th_.joinable()) pc_th_ = std::thread([this] { copier(); });
}

void Frontend::copier() {
  pthread_setname_np(pthread_self(), "cmq-pcopy");
  std::unique_lock<std::mutex> g(pc_mu_);
  while (true) {
    pc_cv_.wait(g, [&] { return !pc_q_.empty() || pc_stop_; });
    if (pc_q_.empty()) break;
    PCopy c = pc_q_.front();
    pc_q_.pop_front();
    ++pc_active_;
    g.unlock();
    std::string a, b;
    if (c.plen) a.assign((const char*)c.persist, c.plen);
    if (c.clen) b.assign((const char*)c.consumed, c.clen);
    persist_->submit(c.step, std::move(a), std::move(b));
    g.lock();
    --pc_active_;
    pc_done_cv_.notify_all();
  }
}

void Frontend::post_copy(const PCopy& c) {
  {
    std::lock_guard<std::mutex> g(pc_mu_);
    pc_q_.push_back(c);
  }
  pc_cv_.notify_one();
}

// before the engine reuses a record slot: at most `max_pending` copies still to run
void Frontend::wait_copies(size_t max_pending) {
  if (!pc_th_.joinable()) return;
  std::unique_lock<std::mutex> g(pc_mu_);
  pc_done_cv_.wait(g, [&] { return pc_q_.size() + pc_active_ <= max_pending; });
}

FeStats Frontend::stats() {
  std::lock_guard<std::mutex> g(stats_mu_);
  FeStats s = stats_;
  s.rx_bytes = rx_bytes_;
  s.tx_bytes = tx_bytes_;
  return s;
}

u64 Frontend::pending_out() const {
  u64 t = 0;
  for (auto& c : conns_) {
    std::lock_guard<std::mutex> g(c->mu);
    t += c->out.size() - c->out_pos;
  }
  return t;
}

// ============================================================================ IO threads
void Frontend::accept_all(FeIo& io0) {
  for (;;) {
    sockaddr_in a{};
    socklen_t l = sizeof a;
    int fd = ::accept4(lfd_, (sockaddr*)&a, &l, SOCK_NONBLOCK | SOCK_CLOEXEC);
    if (fd < 0) return;
    u32 id = 0;
    {
      std::lock_guard<std::mutex> g(free_mu_);
      const u64 fin = fin_step_.load();
      while (!quarantine_.empty() && quarantine_.front().first <= fin) {
        free_.push_back(quarantine_.front().second);
        quarantine_.pop_front();
      }
      if (!free_.empty()) { id = free_.back(); free_.pop_back(); }
    }
    if (!id) { ::close(fd); continue; }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    if (cfg_.sndbuf) setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &cfg_.sndbuf, sizeof cfg_.sndbuf);
    if (cfg_.rcvbuf) setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &cfg_.rcvbuf, sizeof cfg_.rcvbuf);
    FeConn& c = *conns_[id];
    {
      std::lock_guard<std::mutex> g(c.mu);
      c.fd = fd;
      c.out.clear();
      c.out_pos = 0;
      c.inject.clear();
      c.hostbuf.clear();
      c.host_notified = false;
    }
    c.in_ready = false;
    c.rdhup = false;
    c.wblocked = false;
    if (api_->wblock) api_->wblock[id] = 0;
    c.carry = c.inflight = 0;
    c.paused = c.kicked = false;
    c.hb_s = 0;
    c.last_rx = c.last_tx = now_ns();
    c.mode = M_HOST;
    FeEvent e;
    e.kind = FE_OPEN;
    e.conn = id;
    post(std::move(e));
    FeIo& io = *io_[c.io];
    if (&io == &io0) {
      io.owned.push_back(id);
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLOUT | EPOLLRDHUP | EPOLLET;
      ev.data.u64 = id;
      epoll_ctl(io.epfd, EPOLL_CTL_ADD, fd, &ev);
    } else {
      {
        std::lock_guard<std::mutex> g(io.qmu);
        io.adopt.push_back(id);
      }
      poke(io.evfd);
    }
  }
}

void Frontend::drop(FeConn& c, bool notify) {
  std::lock_guard<std::mutex> g(c.mu);
  if (c.fd < 0) return;
  epoll_ctl(io_[c.io]->epfd, EPOLL_CTL_DEL, c.fd, nullptr);
  ::close(c.fd);
  c.fd = -1;
  c.mode = M_DEAD;
  const u32 g2 = c.gen.fetch_add(1) + 1;
  c.read_cap = 0;
  c.out.clear();
  c.out_pos = 0;
  c.inject.clear();
  c.wblocked = false;
  if (api_->wblock) api_->wblock[c.id] = 0;
  if (notify) {
    FeEvent e;
    e.kind = FE_CLOSED;
    e.conn = c.id;
    e.a = g2;   // the control plane's close(conn, gen) of this slot is stale once it moved on
    post(std::move(e));
  }
}

// bytes of a host-mode connection to its host buffer.  The control plane may switch the
// connection to the data plane meanwhile (set_data_mode moves the host buffer to the
// inject queue under c.mu): bytes read after that go to the inject queue too (to_data: the
// caller marks the connection ready), never to a host buffer nobody reads any more
static void host_read(Frontend* fe, FeConn& c, std::atomic<u64>& rx, bool& eof, bool& notify, bool& to_data) {
  char buf[1 << 16];
  for (;;) {
    ssize_t k = ::recv(c.fd, buf, sizeof buf, 0);
    if (k > 0) {
      rx += (u64)k;
      std::lock_guard<std::mutex> g(c.mu);
      if (c.mode == M_DATA) {
        c.inject.append(buf, (size_t)k);
        to_data = true;
        continue;
      }
      c.hostbuf.append(buf, (size_t)k);
      if (!c.host_notified) { c.host_notified = true; notify = true; }
      continue;
    }
    if (k == 0) eof = true;
    else if (errno == EINTR) continue;
    else if (errno != EAGAIN && errno != EWOULDBLOCK) eof = true;
    break;
  }
  (void)fe;
}

void Frontend::io_loop(int i) {
  FeIo& io = *io_[i];
  char tname[16];
  snprintf(tname, sizeof tname, "cmq-io%d", i);
  pthread_setname_np(pthread_self(), tname);
  epoll_event evs[512];
  while (true) {
    const bool run = running_.load();
    int n = epoll_wait(io.epfd, evs, 512, run ? 50 : 2);
    // ---- queued requests
    std::vector<u32> adopt, pend, closing;
    {
      std::lock_guard<std::mutex> g(io.qmu);
      adopt.swap(io.adopt);
      pend.swap(io.pending);
      closing.swap(io.closing);
    }
    for (u32 id : adopt) {
      FeConn& c = *conns_[id];
      io.owned.push_back(id);
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLOUT | EPOLLRDHUP | EPOLLET;
      ev.data.u64 = id;
      epoll_ctl(io.epfd, EPOLL_CTL_ADD, c.fd, &ev);
    }
    for (u32 id : pend) {
      FeConn& c = *conns_[id];
      if (c.mode == M_DATA) {
        if (!c.in_ready) { c.in_ready = true; io.ready.push_back(id); }
      } else if (c.mode == M_HOST && c.fd >= 0) {
        bool eof = false, notify = false, to_data = false;
        host_read(this, c, rx_bytes_, eof, notify, to_data);
        if (notify) { FeEvent e; e.kind = FE_HOST; e.conn = id; post(std::move(e)); }
        if (to_data && !c.in_ready) { c.in_ready = true; io.ready.push_back(id); }
        if (eof) drop(c, true);
      }
    }
    for (u32 id : closing) {
      FeConn& c = *conns_[id];
      {
        std::lock_guard<std::mutex> g(c.mu);
        if (c.mode == M_FREE) continue;   // closed twice: the slot is freed (or reused) once
        if (c.fd >= 0) {
          write_some(c);
          epoll_ctl(io.epfd, EPOLL_CTL_DEL, c.fd, nullptr);
          ::close(c.fd);
          c.fd = -1;
        }
        c.mode = M_FREE;
        c.gen.fetch_add(1);
        c.read_cap = 0;
        c.out.clear();
        c.out_pos = 0;
        c.wblocked = false;
        if (api_->wblock) api_->wblock[id] = 0;
        c.inject.clear();
        c.hostbuf.clear();
      }
      c.in_ready = false;
      io.owned.erase(std::remove(io.owned.begin(), io.owned.end(), id), io.owned.end());
      io.ready.erase(std::remove(io.ready.begin(), io.ready.end(), id), io.ready.end());
      // reusable once the steps in flight now have finished (their results name this slot)
      std::lock_guard<std::mutex> g(free_mu_);
      quarantine_.emplace_back(sub_step_.load(), id);
    }
    // ---- socket events
    bool data_ready = false;
    for (int k = 0; k < n; ++k) {
      u64 id = evs[k].data.u64;
      if (id == WAKE) {
        u64 v;
        while (::read(io.evfd, &v, 8) > 0) {
        }
        continue;
      }
      if (id == LISTENER) { accept_all(io); continue; }
      FeConn& c = *conns_[id];
      if (c.fd < 0) continue;
      const u32 e = evs[k].events;
      if (e & EPOLLOUT) {
        std::lock_guard<std::mutex> g(c.mu);
        if (c.fd >= 0 && c.out_pos < c.out.size()) write_some(c);
      }
      if (e & (EPOLLRDHUP | EPOLLHUP | EPOLLERR)) c.rdhup = true;
      if (!(e & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR))) continue;
      c.last_rx = now_ns();
      const int m = c.mode;
      if (m == M_DATA) {
        if (!c.in_ready) { c.in_ready = true; io.ready.push_back((u32)id); }
        data_ready = true;
      } else if (m == M_HOST) {
        bool eof = false, notify = false, to_data = false;
        host_read(this, c, rx_bytes_, eof, notify, to_data);
        if (notify) { FeEvent ev; ev.kind = FE_HOST; ev.conn = (u32)id; post(std::move(ev)); }
        if (to_data) {   // switched to the data plane while reading: its next step takes them
          if (!c.in_ready) { c.in_ready = true; io.ready.push_back((u32)id); }
          data_ready = true;
        }
        if (eof) drop(c, true);
      }
    }
    if (data_ready) wake_stepper();
    // ---- IO phase requested by the stepper
    const u64 ph = ph_id_.load(std::memory_order_acquire);
    if (ph != io.phase_seen) {
      io.phase_seen = ph;
      io.segs.clear();
      // scatter: the egress of finished steps, in step order, for this thread's connections
      // (async phase: after the gather has released the stepper; the Scatter objects live
      // in out_prev_ until every IO thread has passed the next phase)
      const std::vector<Scatter*> scat = *ph_scat_;
      const bool async = ph_async_;
      auto scatter = [&] {
        for (Scatter* sc : scat) {
          // the step's D2H was issued by the stepper, which did not wait for it (stash_pend)
          if (sc->wait_slot >= 0) api_->egress_ready(api_->eng, sc->wait_slot);
          const u8* base = sc->own.empty() ? sc->egress : (const u8*)sc->own.data();
          for (u32 id : io.owned) {
            const ConnOut& o = sc->co[id];
            if (o.len) {
              FeConn& c = *conns_[id];
              if (!sc->gen.empty() && sc->gen[id] != c.gen.load()) continue;   // closed since: stale
              if (c.mode != M_DATA && c.mode != M_HOST) continue;
              if (sc->gath_n) scatter_ref(c, base, o, *sc);
              else scatter_conn(c, base + o.off, o.len);
            }
          }
        }
      };
      if (!async) scatter();
      if (ph_gather_) {
        std::vector<u32> keep;
        for (u32 id : io.ready) {
          FeConn& c = *conns_[id];
          c.in_ready = false;
          if (c.mode != M_DATA) continue;
          gather_conn(io, c, ph_arena_, ph_cap_);
          if (c.in_ready) keep.push_back(id);
        }
        io.ready.swap(keep);
      }
      if (ph_left_.fetch_sub(1) == 1) {
        std::lock_guard<std::mutex> g(ph_mu_);
        ph_cv_.notify_all();
      }
      if (async) scatter();
    }
    if (!run && stepper_done_) break;
    // ---- heartbeats (every 100 ms): send when idle for hb/2, drop after 2*hb of silence
    const i64 t = now_ns();
    if (t - io.last_hb > 100000000) {
      io.last_hb = t;
      for (u32 id : io.owned) {
        FeConn& c = *conns_[id];
        const u32 hb = c.hb_s;
        if (!hb || c.fd < 0) continue;
        const i64 hbn = (i64)hb * 1000000000;
        if (t - c.last_rx > 2 * hbn) { drop(c, true); continue; }
        if (t - c.last_tx >= hbn / 2) {
          std::lock_guard<std::mutex> g(c.mu);
          if (c.out_pos >= c.out.size()) {
            c.out.append(HEARTBEAT_FRAME, 8);
            write_some(c);
          }
        }
      }
    }
  }
}

// one connection's bytes for this step: queued inject bytes, then what its socket holds,
// within the per-connection budget; reserved densely in the shared arena
void Frontend::gather_conn(FeIo& io, FeConn& c, u8* arena, u64 cap) {
  u64 lim = cfg_.per_conn_read;
  const u64 rc = c.read_cap.load(std::memory_order_relaxed);
  if (rc && rc < lim) lim = rc;
  const u64 room = api_->carry_cap > (u64)c.carry + c.inflight ? api_->carry_cap - c.carry - c.inflight : 0;
  if (lim > room) lim = room;
  if (c.paused) {   // behind a control command: bytes wait in the socket (TCP back-pressure)
    c.in_ready = true;
    return;
  }
  std::string inj;
  {
    std::lock_guard<std::mutex> g(c.mu);
    if (!c.inject.empty()) {
      if (c.inject.size() <= lim) inj.swap(c.inject);
      else { inj = c.inject.substr(0, lim); c.inject.erase(0, lim); c.in_ready = true; }
      c.inj_step = ph_step_;
    }
  }
  int avail = 0;
  if (c.fd >= 0 && ioctl(c.fd, FIONREAD, &avail) < 0) avail = 0;
  u64 want = (u64)avail;
  if (inj.size() + want > lim) { want = lim > inj.size() ? lim - inj.size() : 0; if (avail) c.in_ready = true; }
  const u64 total = inj.size() + want;
  const bool eof = avail == 0 && c.rdhup;
  if (total == 0 && !c.kicked) {
    if (eof) drop(c, true);
    return;
  }
  // work-buffer budget: the device stages this connection's carry (<= carry + bytes still
  // in flight) in front of the new bytes
  const u64 wneed = (u64)c.carry + c.inflight + 48;
  if (ph_carry_.fetch_add(wneed) + wneed > api_->carry_budget) {
    ph_carry_.fetch_sub(wneed);
    std::lock_guard<std::mutex> g(c.mu);
    c.inject.insert(0, inj);
    c.in_ready = true;
    return;
  }
  // reserve a segment slot and arena bytes
  const u32 si = ph_nseg_.fetch_add(1);
  if (si >= api_->seg_max) {
    ph_nseg_.fetch_sub(1);
    ph_carry_.fetch_sub(wneed);
    std::lock_guard<std::mutex> g(c.mu);
    c.inject.insert(0, inj);
    c.in_ready = true;
    return;
  }
  const u64 need = (total + 15) & ~15ull;
  u64 off = ph_used_.load();
  while (true) {
    if (off + need > cap) {
      ph_nseg_.fetch_sub(1);
      ph_carry_.fetch_sub(wneed);
      std::lock_guard<std::mutex> g(c.mu);
      c.inject.insert(0, inj);
      c.in_ready = true;
      return;
    }
    if (ph_used_.compare_exchange_weak(off, off + need)) break;
  }
  u8* dst = arena + off;
  if (!inj.empty()) memcpy(dst, inj.data(), inj.size());
  u64 got = 0;
  while (got < want) {
    ssize_t k = ::recv(c.fd, dst + inj.size() + got, want - got, 0);
    if (k > 0) { got += (u64)k; continue; }
    if (k < 0 && errno == EINTR) continue;
    break;
  }
  const u64 len = inj.size() + got;
  rx_bytes_ += got;
  if (got) c.last_rx = now_ns();
  c.kicked = false;
  io.segs.push_back(SegIn{c.id, (u32)len, off});
  if (eof && !c.in_ready) drop(c, true);
}

void Frontend::io_phase(std::vector<Scatter*>& scat, bool gather, bool async) {
  ph_scat_ = &scat;
  ph_gather_ = gather;
  ph_async_ = async && gather && !scat.empty();
  ph_arena_ = arena_[arena_i_];
  ph_cap_ = api_->ingress_cap;
  if (api_->log_bytes) {
    // ingress throttle: the device drops a step's publishes when the body log cannot take
    // them (the oldest live message pins the log tail), so near a full log only a trickle
    // is read (acks still get through and free it); TCP pushes back on publishers
    u64 used;
    {
      std::lock_guard<std::mutex> g(stats_mu_);
      used = stats_.log_used;
    }
    // two steps may already be in flight with up to ingress_cap each
    const u64 reserve = 2 * api_->ingress_cap + (api_->log_bytes >> 6);
    const u64 freeb = api_->log_bytes > used + reserve ? api_->log_bytes - used - reserve : 0;
    if (freeb < ph_cap_) ph_cap_ = std::max<u64>(freeb, 256u << 10);
  }
  ph_step_ = step_no_ + 1;   // the step these segments go into (f.step = ++step_no_)
  ph_used_ = 0;
  ph_nseg_ = 0;
  ph_carry_ = 0;
  ph_left_ = (int)io_.size();
  ph_id_.fetch_add(1, std::memory_order_release);
  for (auto& io : io_) poke(io->evfd);
  {
    std::unique_lock<std::mutex> g(ph_mu_);
    ph_cv_.wait(g, [&] { return ph_left_.load() == 0; });
  }
  // every IO thread passed this phase, so the previous async scatter is written; this
  // phase's egress stays alive while the IO threads write it (async) or is done
  out_prev_.clear();
  if (ph_async_) out_prev_.swap(out_);
  out_.clear();
}

// log2 µs bin of a duration in seconds (FeStats.h_*)
static void hbin(u64* h, double s) {
  u64 us = (u64)(s * 1e6);
  int k = 0;
  while (us > 1 && k < 31) { us >>= 1; ++k; }
  h[k]++;
}

// ============================================================================ stepper
void Frontend::finish_oldest(std::deque<Inflight>& inflight) {
  if (pend_valid_ && !stash_pend(true)) return;   // its egress is written by the next IO phase
  Inflight f = std::move(inflight.front());
  inflight.pop_front();
  const int p = f.p;
  i64 t0 = now_ns();
  {
    GpuWait gw(gpu_wait_since_);
    if (!check(api_->wait_results(api_->eng, p))) return;
  }
  double w = secs_since(t0);
  const Counters& c = *api_->counters(api_->eng, p);
  if (!f.gets.empty()) {   // Basic.Get answers of this step
    const GetOut* go = api_->get_out(api_->eng, p);
    for (size_t k = 0; k < f.gets.size(); ++k) {
      FeEvent e;
      e.kind = FE_GET;
      e.conn = f.gets[k].first;
      e.a = (u64)go[k].status | ((u64)go[k].msg_count << 32);
      e.b = f.gets[k].second;
      post(std::move(e));
    }
  }
  const SegOut* so = api_->seg_out(api_->eng, p);
  for (size_t k = 0; k < f.segs.size(); ++k) {
    const SegOut& s = so[k];
    if (s.conn >= c_max_) continue;
    FeConn& cc = *conns_[s.conn];
    cc.carry = s.carry;
    const u32 len = f.segs[k].second;
    cc.inflight = cc.inflight > len ? cc.inflight - len : 0;
    if (s.status & SS_CTRL) cc.paused = true;
    if (notify_[s.conn] && cc.fd < 0) {   // an injected pseudo-connection's bytes were stepped
      std::lock_guard<std::mutex> g(cc.mu);
      // only once the step that took the LAST injected bytes has finished (an inject
      // larger than one step's read budget spans several steps)
      if (cc.inject.empty() && f.step >= cc.inj_step) {
        notify_[s.conn] = 0;
        FeEvent e;
        e.kind = FE_INJECTED;
        e.conn = s.conn;
        e.a = s.carry;
        post(std::move(e));
      }
    }
    if (s.status & (SS_FRAME_ERROR | SS_UNEXPECTED | SS_TOO_LARGE)) {
      FeEvent e;
      e.kind = FE_STATUS;
      e.conn = s.conn;
      e.a = s.status;
      post(std::move(e));
    }
    if (cc.carry && !cc.paused && !(s.status & (SS_FRAME_ERROR | SS_UNEXPECTED | SS_TOO_LARGE)) &&
        (s.status & SS_OVERFLOW)) {   // per-step capacity hit: re-present the carry next step
      cc.kicked = true;
      FeIo& io = *io_[cc.io];
      std::lock_guard<std::mutex> g(io.qmu);
      io.pending.push_back(s.conn);
    }
  }
  u32 nc = c.n_ctrl;
  if (nc > api_->seg_max * 2) nc = api_->seg_max * 2;
  if (nc) {
    const CtrlRec* cr = api_->ctrl_rec(api_->eng, p);
    const u8* cb = api_->ctrl(api_->eng, p);
    for (u32 k = 0; k < nc; ++k) {
      FeEvent e;
      e.conn = cr[k].conn;
      if (cr[k].off == 0xffffffffu) {
        e.kind = FE_EVENT;
        e.a = cr[k].len;
        e.b = cr[k].seg;
      } else if (cr[k].seg & CTRL_TXBUF) {
        e.kind = FE_TXBUF;
        e.a = cr[k].seg & ~CTRL_TXBUF;
        e.data.assign((const char*)cb + cr[k].off, cr[k].len);
      } else {
        e.kind = FE_CTRL;
        e.a = (cr[k].seg & CTRL_DGET) ? 1 : 0;   // a step-decoded Basic.Get: connection not paused
        e.data.assign((const char*)cb + cr[k].off, cr[k].len);
      }
      post(std::move(e));
    }
  }
  if (c.n_grow && api_->grow_host) {
    FeEvent e;
    e.kind = FE_GROW;
    e.data.assign((const char*)api_->grow_host(api_->eng, p), sizeof(RingMove) * std::min<u32>(c.n_grow, GROW_MAX));
    post(std::move(e));
  }
  bool needs_commit = false;
  if (api_->persist && (c.n_persist || c.n_consumed)) {
    if (c.n_persist_overflow || c.n_persist > api_->persist_max || c.n_consumed > api_->persist_max) {
      // the device dropped store records of this step: committing the rest and releasing
      // its confirms would acknowledge messages that are not durable (or keep rows of
      // consumed ones).  Fail closed: the stepper stops, nothing of this step is released
      FeEvent e;
      e.kind = FE_ERROR;
      e.data = "persist record buffer overflow (step " + std::to_string(f.step) + ": " +
               std::to_string(c.n_persist) + " persist / " + std::to_string(c.n_consumed) +
               " consumed records > persist_max " + std::to_string(api_->persist_max) + ")";
      failed_ = true;
      post(std::move(e));
      return;
    }
    if (persist_) {   // copied off the stepper (the slot outlives this step by PSLOTS - 1)
      post_copy(PCopy{f.step, c.n_persist ? api_->persist_host(api_->eng, p) : nullptr,
                      c.n_persist ? (size_t)c.persist_used : 0,
                      c.n_consumed ? (const u8*)api_->consumed_host(api_->eng, p) : nullptr,
                      c.n_consumed ? (size_t)c.n_consumed * sizeof(ConsumedRec) : 0});
    } else {
      FeEvent e;
      e.kind = FE_PERSIST;
      e.a = f.step;
      e.b = 0;
      if (c.n_persist) e.data.assign((const char*)api_->persist_host(api_->eng, p), c.persist_used);
      if (c.n_consumed)
        e.data2.assign((const char*)api_->consumed_host(api_->eng, p), (size_t)c.n_consumed * sizeof(ConsumedRec));
      post(std::move(e));
    }
    needs_commit = true;
  }
  const int slot = api_->egress_slot(api_->eng, p);
  const ConnOut* co = api_->conn_out(api_->eng, p);
  Held h;
  h.step = f.step;
  h.batch_hi = f.batch_hi;
  h.needs_commit = needs_commit;
  h.sc.co.assign(co, co + c_max_);
  h.sc.gen = std::move(f.gen);
  h.sc.egress = api_->egress_host(api_->eng, slot);
  if (c.n_ref && c.egress_bytes > c.gath_off) {   // deliveries referencing arena bodies
    h.sc.gath_off = c.gath_off;
    h.sc.gath_n = (u32)((c.egress_bytes - c.gath_off) / sizeof(EgressRef));
  }
  if (needs_commit && api_->conn_conf) {
    const u32* cf = api_->conn_conf(api_->eng, p);
    h.conf.assign(cf, cf + c_max_);
  }
  if (c.egress_bytes && !check(api_->egress_copy(api_->eng, p))) return;
  {
    std::lock_guard<std::mutex> g(stats_mu_);
    stats_.steps++;
    stats_.published += c.n_pubs;
    stats_.spill_moved += c.spill_moved;
    stats_.delivered += c.n_deliv;
    stats_.egress_bytes += c.egress_bytes;
    stats_.live_bytes = c.live_bytes;
    stats_.dropped_nomem += c.n_dropped_nomem;
    stats_.ring_full += c.n_ring_full;
    stats_.unroutable += c.n_unroutable;
    stats_.routed += c.n_routed_msgs;
    stats_.expired += c.n_expired;
    stats_.ctrl += c.n_ctrl;
    stats_.live_msgs = c.n_live_msgs;
    stats_.log_used = c.log_head - c.log_tail;
    stats_.wait_s += w;
    hbin(stats_.h_wait, w);
    stats_.max_wait_s = std::max(stats_.max_wait_s, w);
    for (int k = 0; k < 32; ++k) stats_.lat_hist[k] += c.lat_hist[k];
    if (needs_commit) stats_.held_steps++;
  }
  // busy: keep stepping while the device still has work (backlog, carry, deliveries)
  bool busy = !f.segs.empty() || c.n_deliv || c.egress_bytes || c.n_ctrl;
  pend_slot_ = slot;
  pend_valid_ = true;
  pend_bytes_ = c.egress_bytes;
  pend_ = std::move(h);
  last_busy_ = busy;
  fin_step_.store(f.step);
}

void Frontend::stepper() {
  pthread_setname_np(pthread_self(), "cmq-stepper");
  std::deque<Inflight> inflight;
  i64 last_step = now_ns();
  while (running_ && !failed_) {
    // ---- exclusive access for the control plane: drain, write out, park
    bool want_pause;
    {
      std::lock_guard<std::mutex> g(st_mu_);
      want_pause = pause_req_ > 0;
    }
    if (want_pause) {
      while (!inflight.empty() && !failed_) finish_oldest(inflight);
      wait_copies(0);   // a host-run step may reuse any record slot
      flush_pending(false);
      std::unique_lock<std::mutex> g(st_mu_);
      paused_ = true;
      pause_cv_.notify_all();
      st_cv_.wait(g, [&] { return pause_req_ == 0 || !running_; });
      paused_ = false;
      wake_ = true;
      continue;
    }
    // ---- idle: nothing in flight, nothing to write, nothing readable
    const bool host_work = api_->host_work && api_->host_work(api_->eng) > 0;   // staged control writes
    if (inflight.empty() && !pend_valid_ && out_.empty() && !last_busy_ && !releasable() && !gets_pending() &&
        !host_work && !ctl_pending()) {
      std::unique_lock<std::mutex> g(st_mu_);
      const double idle = cfg_.idle_step_ms > 0 ? cfg_.idle_step_ms : 1000.0;
      st_cv_.wait_for(g, std::chrono::microseconds((i64)(idle * 1000)),
                      [&] { return wake_ || pause_req_ > 0 || !running_; });
      bool woke = wake_;
      wake_ = false;
      if (pause_req_ > 0 || !running_) continue;
      if (!woke) {
        if (now_ns() - last_step < (i64)(idle * 1e6)) continue;
        // open connections: the idle step period; none: a TTL sweep (K12 at the queue heads
        // in k_dequeue) every sweep_ms while the device still holds messages
        i64 live;
        {
          std::lock_guard<std::mutex> sg(stats_mu_);
          live = stats_.live_bytes;
        }
        idle_tick_ = any_data_conn() || (live > 0 && now_ns() - last_step >= (i64)(cfg_.sweep_ms * 1e6));
        if (!idle_tick_) continue;
      }
    } else {
      std::lock_guard<std::mutex> g(st_mu_);
      wake_ = false;
    }
    // ---- IO phase: write the oldest finished step's egress, gather the next step
    std::vector<Scatter*> scat;
    if (!collect_scatter(scat)) break;
    i64 t0 = now_ns();
    io_phase(scat, true, cfg_.async_scatter);
    double tio = secs_since(t0);
    std::vector<SegIn> segs;
    std::vector<std::pair<u32, u32>> seglens;
    for (auto& io : io_) {
      for (auto& s : io->segs) {
        segs.push_back(s);
        seglens.emplace_back(s.conn, s.len);
        conns_[s.conn]->inflight += s.len;
      }
    }
    const u64 used = ph_used_.load();
    const bool submit = !segs.empty() || last_busy_ || idle_tick_ || gets_pending() ||
                        (api_->host_work && api_->host_work(api_->eng) > 0) || ctl_needs_step();
    idle_tick_ = false;
    bool submitted = false;
    if (submit) {
      // the gathered bytes start crossing PCIe now, while the oldest step finishes (the
      // engine orders the copy behind the last reader of that ingress buffer on the GPU)
      if (inflight.size() >= 2 && used && api_->prefetch &&
          !check(api_->prefetch(api_->eng, arena_[arena_i_], used)))
        break;
      if (inflight.size() >= 2) finish_oldest(inflight);
      if (failed_) break;
      i64 t1 = now_ns();
      Inflight f;
      stage_gets(f);
      wait_copies(PSLOTS - 3);   // the slot this submit takes was last used PSLOTS steps back
      ref_for_step(used);
      int p = api_->submit(api_->eng, segs.data(), (u32)segs.size(), arena_[arena_i_], used, wall_ms(), cfg_.worker);
      if (!check(p)) break;
      {
        std::lock_guard<std::mutex> g(stats_mu_);
        const double ts = secs_since(t1);
        stats_.submit_s += ts;
        stats_.io_phase_s += tio;
        stats_.gather_segs += segs.size();
        if (segs.empty() && !last_busy_) stats_.idle_steps++;
        hbin(stats_.h_submit, ts);
        hbin(stats_.h_io, tio);
        stats_.max_io_s = std::max(stats_.max_io_s, tio);
        if (last_submit_) {
          const double per = (t1 - last_submit_) * 1e-9;
          hbin(stats_.h_period, per);
          stats_.max_period_s = std::max(stats_.max_period_s, per);
        }
        last_submit_ = t1;
      }
      kick_unpaused(p);
      f.p = p;
      f.step = ++step_no_;
      f.batch_hi = api_->dl_state ? api_->dl_state(api_->eng, 1) : 0;
      sub_step_.store(step_no_);
      f.segs = std::move(seglens);
      f.gen.resize(c_max_);
      for (u32 k = 0; k < c_max_; ++k) f.gen[k] = conns_[k]->gen.load();
      inflight.push_back(std::move(f));
      arena_i_ = (arena_i_ + 1) % narena_;
      last_step = now_ns();
      submitted = true;
      last_busy_ = false;
    }
    // ---- results: the older step once two are in flight (or when nothing new went out)
    if (inflight.size() >= 2 || (!submitted && !inflight.empty())) finish_oldest(inflight);
  }
  // stopping: complete what is in flight so the engine is idle
  while (!inflight.empty() && !failed_) finish_oldest(inflight);
  flush_pending(true);
  stepper_done_ = true;
  std::lock_guard<std::mutex> g(st_mu_);
  paused_ = true;
  pause_cv_.notify_all();
}

// ============================================================================ sharded broker
void Frontend::request_sync() {
  sync_req_ = true;
  wake_stepper();
}

void Frontend::sync_done() {
  {
    std::lock_guard<std::mutex> g(st_mu_);
    sync_go_ = true;
  }
  st_cv_.notify_all();
}

bool Frontend::healthy(double stuck_s) const {
  if (failed_) return false;
  if (persist_ && persist_->failed()) return false;   // the store cannot commit: fail over
  const i64 t = gpu_wait_since_.load();
  return !t || (now_ns() - t) < (i64)(stuck_s * 1e9);
}

void Frontend::inject_fault(int kind, u64 steps) {
  std::lock_guard<std::mutex> g(st_mu_);
  fault_kind_ = kind;
  fault_at_ = step_no_ + steps;
}

// an injected fault whose step has come (stepper thread)
bool Frontend::fault_due() {
  int kind;
  {
    std::lock_guard<std::mutex> g(st_mu_);
    if (!fault_kind_ || step_no_ < fault_at_) return false;
    kind = fault_kind_;
    fault_kind_ = 0;
  }
  if (kind == 2) _exit(86);
  if (kind == 3) {   // a wedged GPU: the stepper never returns from a device wait
    gpu_wait_since_ = now_ns();
    while (running_) std::this_thread::sleep_for(std::chrono::milliseconds(50));
    return true;
  }
  FeEvent e;
  e.kind = FE_ERROR;
  e.data = "injected engine failure";
  failed_ = true;
  post(std::move(e));
  return true;
}

void Frontend::drain(std::deque<Inflight>& inflight) {
  while (!inflight.empty() && !failed_) finish_oldest(inflight);
}

// every rank parks here at the same step: the control plane syncs (or fails over), then
// sync_done() resumes the steps
void Frontend::park_sync(int kind, u64 step) {
  FeEvent e;
  e.kind = kind;
  e.a = step;
  post(std::move(e));
  std::unique_lock<std::mutex> g(st_mu_);
  paused_ = true;
  pause_cv_.notify_all();
  st_cv_.wait(g, [&] { return sync_go_ || !running_; });
  sync_go_ = false;
  paused_ = false;
  wake_ = true;
}

// Sharded steps: every rank takes part in every exchange, so the steppers tick in
// lockstep -- continuously while any rank is busy (the busy flag travels in the count
// exchange), every idle_step_ms otherwise.  Step t: gather -> submit (H2D + phase A) ->
// exchange of step t-1 (records of t-1's phase A; flags) -> phase B (imports it).
// A sync request (replicated control ops pending on some rank) travels the same way:
// when the OR-ed flags carry XF_SYNC every rank runs one empty flush step (imports the
// last exchange; nothing stays in flight), drains, and parks for the control plane.
void Frontend::stepper_sharded() {
  pthread_setname_np(pthread_self(), "cmq-stepper");
  std::deque<Inflight> inflight;
  // drop the pending exchange of parity q: 0, -1 error (reported), -2 the asynchronous
  // exchange still in flight failed (its phase B imported nothing): a failover
  auto dropx = [&](int q) -> int {
    const int r = api_->drop_exchange(api_->eng, q);
    if (r == -1) check(-1);
    return r;
  };
  while (running_ && !failed_) {
    bool want_pause;
    {
      std::lock_guard<std::mutex> g(st_mu_);
      want_pause = pause_req_ > 0;
    }
    if (want_pause) {   // local exclusive access (a pending exchange may stay pending)
      drain(inflight);
      flush_pending(false);
      std::unique_lock<std::mutex> g(st_mu_);
      paused_ = true;
      pause_cv_.notify_all();
      st_cv_.wait(g, [&] { return pause_req_ == 0 || !running_; });
      paused_ = false;
      wake_ = true;
      continue;
    }
    // ---- pace: idle ranks tick every idle_step_ms (the whole cluster is idle)
    if (!(last_busy_ || cluster_busy_ || sync_req_ || releasable() || gets_pending())) {
      std::unique_lock<std::mutex> g(st_mu_);
      const double idle = cfg_.idle_step_ms > 0 ? cfg_.idle_step_ms : 1.0;
      st_cv_.wait_for(g, std::chrono::microseconds((i64)(idle * 1000)),
                      [&] { return wake_ || pause_req_ > 0 || !running_; });
      wake_ = false;
      if (pause_req_ > 0 || !running_) continue;
    } else {
      std::lock_guard<std::mutex> g(st_mu_);
      wake_ = false;
    }
    if (fault_due()) break;
    // ---- IO phase
    std::vector<Scatter*> scat;
    if (!collect_scatter(scat)) break;
    i64 t0 = now_ns();
    io_phase(scat, true);   // sync: flush steps may reuse egress slots before the next phase
    double tio = secs_since(t0);
    std::vector<SegIn> segs;
    std::vector<std::pair<u32, u32>> seglens;
    for (auto& io : io_) {
      for (auto& sg : io->segs) {
        segs.push_back(sg);
        seglens.emplace_back(sg.conn, sg.len);
        conns_[sg.conn]->inflight += sg.len;
      }
    }
    const bool local_busy = !segs.empty() || last_busy_ || gets_pending();
    if (inflight.size() >= 2) finish_oldest(inflight);
    if (failed_) break;
    // ---- step t: H2D + phase A
    i64 t1 = now_ns();
    int p;
    Inflight f;
    stage_gets(f);
    {
      GpuWait gw(gpu_wait_since_);
      wait_copies(PSLOTS - 3);
      ref_for_step(ph_used_.load());
      p = api_->submit(api_->eng, segs.data(), (u32)segs.size(), arena_[arena_i_], ph_used_.load(), wall_ms(),
                       cfg_.worker);
    }
    if (!check(p)) break;
    arena_i_ = (arena_i_ + 1) % narena_;
    kick_unpaused(p);
    f.p = p;
    f.step = ++step_no_;
    f.batch_hi = api_->dl_state ? api_->dl_state(api_->eng, 1) : 0;
    sub_step_.store(step_no_);
    f.segs = std::move(seglens);
    f.gen.resize(c_max_);
    for (u32 k = 0; k < c_max_; ++k) f.gen[k] = conns_[k]->gen.load();
    // ---- exchange of step t-1, then phase B of t.  A sync request only counts once it
    // travelled in an exchange: the first step after a sync has none, and a rank must
    // never park for a sync its peers did not see
    const bool want_sync = sync_req_.load();
    u32 flags = (want_sync ? XF_SYNC : 0u) | (local_busy ? XF_BUSY : 0u), orf = flags & ~XF_SYNC;
    bool xfail = false;
    i64 t2 = now_ns();
    if (xpend_ >= 0) {
      int rc = api_->exchange(api_->eng, xpend_, flags, &orf);
      if (rc == -1) { check(-1); break; }
      if (rc == -2) {
        xfail = true;
        if (dropx(xpend_) == -1) break;
      } else if (orf & XF_SYNC) {
        sync_req_ = false;   // served by this sync (later requests join its control batch)
      }
    }
    double tx = secs_since(t2);
    if (!check(api_->launch_b(api_->eng, p))) break;
    inflight.push_back(std::move(f));
    xpend_ = p;
    last_busy_ = false;
    {
      std::lock_guard<std::mutex> g(stats_mu_);
      stats_.submit_s += secs_since(t1) - tx;
      stats_.io_phase_s += tio;
      stats_.gather_segs += segs.size();
      stats_.xchg_s += tx;
      stats_.xchg_steps++;
      if (segs.empty() && !local_busy) stats_.idle_steps++;
    }
    if (!xfail && (orf & XF_SYNC)) {
      // ---- flush: empty no-dispatch steps import the pending exchange (and, with device
      // links, the link records / acks that travel one exchange later); nothing stays
      // pending, so the control plane may change replicated tables
      const int nflush = api_->links ? 2 : 1;
      bool bad = false;
      for (int k = 0; k < nflush && !xfail; ++k) {
        if (inflight.size() >= 2) finish_oldest(inflight);
        if (failed_) { bad = true; break; }
        int p2;
        {
          GpuWait gw(gpu_wait_since_);
          wait_copies(PSLOTS - 3);
          p2 = api_->flush_submit ? api_->flush_submit(api_->eng, wall_ms(), cfg_.worker)
                                  : api_->submit(api_->eng, nullptr, 0, arena_[arena_i_], 0, wall_ms(), cfg_.worker);
        }
        if (!check(p2)) { bad = true; break; }
        u32 dummy = 0;
        int rc = api_->exchange(api_->eng, xpend_, 0, &dummy);
        if (rc == -1) { check(-1); bad = true; break; }
        if (rc == -2) { xfail = true; if (dropx(xpend_) == -1) { bad = true; break; } }
        if (!check(api_->launch_b(api_->eng, p2))) { bad = true; break; }
        Inflight f2;
        kick_unpaused(p2);
        f2.p = p2;
        f2.step = ++step_no_;
        f2.batch_hi = api_->dl_state ? api_->dl_state(api_->eng, 1) : 0;
        f2.gen.resize(c_max_);
        for (u32 j = 0; j < c_max_; ++j) f2.gen[j] = conns_[j]->gen.load();
        inflight.push_back(std::move(f2));
        xpend_ = p2;
      }
      if (bad) break;
      if (xpend_ >= 0) {   // packed nothing (asynchronous: the last flush exchange lands first)
        const int r = dropx(xpend_);
        if (r == -1) break;
        if (r == -2) xfail = true;
      }
      xpend_ = -1;
      {
        std::lock_guard<std::mutex> g(stats_mu_);
        stats_.flush_steps++;
        if (!xfail) stats_.syncs++;
      }
      if (!xfail) {
        drain(inflight);
        flush_pending(false);
        park_sync(FE_SYNC, step_no_);
        cluster_busy_ = true;   // step right after a sync (replies, unpaused connections)
        continue;
      }
    }
    if (xfail) {   // a peer is gone: nothing of the failed exchange was imported anywhere
      if (xpend_ >= 0 && dropx(xpend_) == -1) break;
      xpend_ = -1;
      drain(inflight);
      flush_pending(false);
      {
        std::lock_guard<std::mutex> g(stats_mu_);
        stats_.xfails++;
      }
      park_sync(FE_XFAIL, step_no_);
      cluster_busy_ = true;
      continue;
    }
    cluster_busy_ = (orf & XF_BUSY) != 0;
    // idle cluster: this step's results and egress go out now, not at the next tick
    if (!cluster_busy_ && !local_busy) {
      drain(inflight);
      flush_pending(false);
    }
  }
  drain(inflight);
  flush_pending(true);
  stepper_done_ = true;
  std::lock_guard<std::mutex> g(st_mu_);
  paused_ = true;
  pause_cv_.notify_all();
}

// the finished step's egress (D2H complete) and any released held steps, oldest first
bool Frontend::stash_pend(bool copy) {
  if (!pend_valid_) return true;
  pend_valid_ = false;
  // replies due behind the egress already queued go first: this step's egress may hold
  // deliveries a reply must precede (a ConsumeOk before its consumer's first delivery)
  release_ctl();
  out_step_ = std::max(out_step_, pend_.step);
  out_batch_ = std::max(out_batch_, pend_.batch_hi);
  // the common case (no copy, nothing held): the IO threads wait for the D2H themselves
  // before writing the slot out, so the stepper goes on to gather and submit meanwhile
  const bool defer = !copy && !pend_.needs_commit && held_total_ == 0 && api_->egress_ready != nullptr;
  if (pend_bytes_ && !defer) {
    GpuWait gw(gpu_wait_since_);
    if (!check(api_->egress_wait_slot(api_->eng, pend_slot_))) return false;
  }
  if (!pend_.needs_commit && held_total_ == 0) {
    if (copy) {   // the slot may be reused before it is written: copy
      materialize(pend_.sc, pend_.sc.egress, pend_bytes_);
    } else if (pend_bytes_ && defer) {
      pend_.sc.wait_slot = pend_slot_;
    }
    out_.push_back(std::move(pend_.sc));
    return true;
  }
  // write-behind: only the connections with publisher confirms in this step wait for the
  // commit (deliveries need no durability), plus any connection that still has older
  // held bytes (its stream stays in order)
  Scatter now;
  now.co.assign(c_max_, ConnOut{0, 0});
  now.gen = pend_.sc.gen;
  bool now_any = false, held_any = false;
  for (u32 c = 0; c < c_max_; ++c) {
    if (!pend_.sc.co[c].len) continue;
    const bool gated = pend_.needs_commit && (pend_.conf.empty() || pend_.conf[c] != 0);
    if (gated || held_cnt_[c]) {
      ++held_cnt_[c];
      ++held_total_;
      held_any = true;
    } else {
      now.co[c] = pend_.sc.co[c];
      pend_.sc.co[c].len = 0;
      now_any = true;
    }
  }
  if (now_any) {
    now.egress = pend_.sc.egress;
    now.gath_n = pend_.sc.gath_n;
    now.gath_off = pend_.sc.gath_off;
    if (copy) materialize(now, pend_.sc.egress, pend_bytes_);
    out_.push_back(std::move(now));
  }
  if (held_any) {
    materialize(pend_.sc, pend_.sc.egress, pend_bytes_);
    held_.push_back(std::move(pend_));
  }
  return true;
}

u64 Frontend::nack_confirms(Scatter& sc) {
  if (sc.own.empty()) return 0;
  u8* b = (u8*)&sc.own[0];
  u64 n = 0;
  for (auto& o : sc.co) {
    u64 p = o.off;
    const u64 end = (u64)o.off + o.len;
    while (p + 8 <= end) {
      const u32 size = ((u32)b[p + 3] << 24) | ((u32)b[p + 4] << 16) | ((u32)b[p + 5] << 8) | b[p + 6];
      if (p + 8 + size > end) break;
      // a method frame Basic.Ack (60/80, 13 argument bytes): only publisher confirms
      if (b[p] == 1 && size == 13 && b[p + 7] == 0 && b[p + 8] == 60 && b[p + 9] == 0 && b[p + 10] == 80) {
        b[p + 10] = 120;
        b[p + 19] &= 1;   // multiple kept, requeue 0
        ++n;
      }
      p += 8 + size;
    }
  }
  return n;
}

bool Frontend::collect_scatter(std::vector<Scatter*>& scat) {
  if (!stash_pend(false)) return false;
  const u64 rel = released_.load();
  // a failed store never commits again: the held steps it did not commit go out now, their
  // confirms as Basic.Nack (they were held forever)
  const bool pfail = persist_ && persist_->failed();
  while (!held_.empty() && (pfail || !held_.front().needs_commit || held_.front().step <= rel)) {
    Scatter& sc = held_.front().sc;
    if (pfail && held_.front().needs_commit && held_.front().step > rel) {
      const u64 k = nack_confirms(sc);
      std::lock_guard<std::mutex> g(stats_mu_);
      stats_.store_fail_nacks += k;
    }
    for (u32 c = 0; c < c_max_; ++c)
      if (sc.co[c].len) { --held_cnt_[c]; --held_total_; }
    out_.push_back(std::move(sc));
    held_.pop_front();
  }
  release_ctl();
  for (auto& sc : out_) scat.push_back(&sc);
  return true;
}

bool Frontend::releasable() const {
  return !held_.empty() && (!held_.front().needs_commit || held_.front().step <= released_.load() ||
                            (persist_ && persist_->failed()));
}

bool Frontend::any_data_conn() const {
  for (auto& c : conns_)
    if (c->mode == M_DATA) return true;
  return false;
}

void Frontend::flush_pending(bool final) {
  if (final) {   // shutting down: the engine goes idle, nothing more is written
    if (pend_valid_ && pend_bytes_) api_->egress_wait_slot(api_->eng, pend_slot_);
    pend_valid_ = false;
    out_.clear();
    return;
  }
  std::vector<Scatter*> scat;
  if (!collect_scatter(scat)) return;
  // an empty phase still waits out the last async scatter: control replies written after
  // this are ordered behind every earlier delivery
  if (!scat.empty() || !out_prev_.empty()) io_phase(scat, false);
}

// ============================================================================ EchoEngine
EchoEngine::~EchoEngine() { x_stop(); }

void EchoEngine::xchg_setup(const std::string& name, const std::vector<int>& members, int timeout_ms, bool async) {
  x_stop();
  shm_.reset();
  members_ = members;
  std::sort(members_.begin(), members_.end());
  shm_.reset(new cmqx::ShmXchg(name, members_, (int)rank_, 1 << 20, timeout_ms));
  xseq_ = 0;
  imports_.clear();
  async_ = async;
  if (async_) xth_ = std::thread([this] { x_loop(); });
}

void EchoEngine::x_stop() {
  {
    std::lock_guard<std::mutex> g(xmu_);
    xstop_ = true;
    xcv_.notify_all();
  }
  if (xth_.joinable()) xth_.join();
  std::lock_guard<std::mutex> g(xmu_);
  xstop_ = xjob_ = xbusy_ = xres_ = false;
  b_wait_[0] = b_wait_[1] = b_due_[0] = b_due_[1] = false;
}

// forwarded segments of the step of parity q, per member: [u32 conn][u32 len][bytes] records
std::vector<std::string> EchoEngine::pack_fwd(int q) {
  Io& io = io_[q];
  const int n = (int)members_.size();
  std::vector<std::string> blocks(n);
  for (int i = 0; i < n; ++i) {
    if (members_[i] == (int)rank_) continue;
    for (auto& rec : io.fwd[members_[i]]) {
      u32 h[2] = {rec.first, (u32)rec.second.size()};
      blocks[i].append((const char*)h, 8);
      blocks[i] += rec.second;
    }
  }
  return blocks;
}

// the last job's result (waits for it); 0 / flags 0 when none is uncollected
int EchoEngine::collect(u32* orf) {
  std::unique_lock<std::mutex> g(xmu_);
  xcv_.wait(g, [&] { return !xjob_ && !xbusy_; });
  *orf = 0;
  if (!xres_) return 0;
  xres_ = false;
  *orf = xres_orf_;
  return xres_rc_;
}

void EchoEngine::x_loop() {
  std::unique_lock<std::mutex> g(xmu_);
  while (true) {
    xcv_.wait(g, [&] { return xstop_ || xjob_; });
    if (!xjob_) return;
    std::vector<std::string> blocks = std::move(xblocks_);
    const u32 fl = xflags_;
    const int dst = xdst_;
    xjob_ = false;
    xbusy_ = true;
    g.unlock();
    u32 orf = 0;
    std::vector<std::pair<u32, std::string>> im;
    const int rc = exchange_blocks(blocks, fl, &orf, &im);
    if (rc) im.clear();   // phase B imports nothing
    g.lock();
    ximports_ = std::move(im);
    b_wait_[dst] = false;
    if (b_due_[dst]) {   // launched before its exchange finished: it runs now
      b_due_[dst] = false;
      run_b(dst, ximports_);
    }
    xbusy_ = false;
    xres_ = true;
    xres_rc_ = rc;
    xres_orf_ = orf;
    xcv_.notify_all();
  }
}

// the shared-memory exchange of the step of parity q
int EchoEngine::exchange(int q, u32 flags, u32* orf) {
  Io& io = io_[q];
  if (!io.ready) { err_ = "exchange: no phase-A step of this parity"; return -1; }
  std::vector<std::string> blocks = pack_fwd(q);
  if (!async_) {
    const int rc = exchange_blocks(blocks, flags, orf, &imports_);
    if (rc == 0) io.ready = false;
    return rc;
  }
  const int rc = collect(orf);
  if (rc) return rc;
  io.ready = false;
  std::lock_guard<std::mutex> g(xmu_);
  xblocks_ = std::move(blocks);
  xflags_ = flags;
  xdst_ = q ^ 1;
  b_wait_[q ^ 1] = true;
  xjob_ = true;
  xcv_.notify_all();
  return 0;
}

int EchoEngine::exchange_blocks(std::vector<std::string>& blocks, u32 flags, u32* orf,
                                std::vector<std::pair<u32, std::string>>* imports) {
  const int n = (int)members_.size();
  int me = 0;
  for (int i = 0; i < n; ++i) if (members_[i] == (int)rank_) me = i;
  std::vector<u32> hs((size_t)n * cmqx::XH_WORDS, 0), hr((size_t)n * cmqx::XH_WORDS, 0);
  for (int i = 0; i < n; ++i) {
    hs[(size_t)i * cmqx::XH_WORDS + 1] = (u32)blocks[i].size();
    hs[(size_t)i * cmqx::XH_WORDS + 5] = flags;
    hs[(size_t)i * cmqx::XH_WORDS + 6] = (u32)xseq_;
  }
  int rc = shm_->counts(hs.data(), hr.data());
  if (rc) return rc;
  u32 o = 0;
  for (int i = 0; i < n; ++i) {
    o |= hr[(size_t)i * cmqx::XH_WORDS + 5];
    if (i != me && hr[(size_t)i * cmqx::XH_WORDS + 6] != (u32)xseq_) { err_ = "exchange out of lockstep"; return -1; }
  }
  *orf = o;
  u8* box = shm_->box(me);
  uint64_t* dir = shm_->dir(me);
  u64 off = 0;
  for (int i = 0; i < n; ++i) {
    dir[i] = off;
    memcpy(box + off, blocks[i].data(), blocks[i].size());
    off += blocks[i].size();
  }
  rc = shm_->barrier();
  if (rc) return rc;
  imports->clear();
  for (int i = 0; i < n; ++i) {
    if (i == me) continue;
    const u8* src = shm_->box(i) + shm_->dir(i)[me];
    const u32 len = hr[(size_t)i * cmqx::XH_WORDS + 1];
    for (u32 k = 0; k + 8 <= len;) {
      u32 h[2];
      memcpy(h, src + k, 8);
      imports->emplace_back(h[0], std::string((const char*)src + k + 8, h[1]));
      k += 8 + h[1];
    }
  }
  ++xseq_;
  return 0;
}

// phase B: imported records become egress of their connection slot in this step
void EchoEngine::launch_b(int p) {
  if (async_) {
    std::lock_guard<std::mutex> g(xmu_);
    if (b_wait_[p]) { b_due_[p] = true; return; }   // after its exchange (x_loop)
    run_b(p, ximports_);   // (its exchange finished first, or none: nothing to import)
    return;
  }
  run_b(p, imports_);
}

void EchoEngine::run_b(int p, std::vector<std::pair<u32, std::string>>& imports) {
  Io& io = io_[p];
  std::string& eg = slot_[slot_of_[p]];
  for (auto& im : imports) {
    if (im.first >= io.co.size()) continue;
    ConnOut& c = io.co[im.first];
    std::string prev = c.len ? eg.substr(c.off, c.len) : std::string();
    c.off = (u32)eg.size();
    c.len = (u32)(prev.size() + im.second.size());
    eg += prev;
    eg += im.second;
    io.ctr.n_deliv++;
    ++imported;
  }
  imports.clear();
  io.ctr.egress_bytes = (u32)eg.size();
}

EchoEngine::EchoEngine(u32 c_max, u32 seg_max, u64 ingress_cap, u32 carry_cap, u32 world, u32 rank)
    : world_(world), rank_(rank) {
  api_.abi = CMQ_STEP_ABI;
  api_.world = world;
  api_.rank = rank;
  api_.native_xchg = world > 1 ? 1u : 0u;
  api_.c_max = c_max;
  api_.seg_max = seg_max;
  api_.carry_cap = carry_cap;
  api_.ingress_cap = ingress_cap;
  api_.ctrl_cap = 1 << 20;
  api_.carry_budget = 64ull << 20;
  api_.log_bytes = 0;
  api_.eng = this;
  paused_.assign(c_max, 0);
  wblock_.assign(c_max, 0);
  api_.wblock = wblock_.data();
  for (auto& io : io_) { io.so.resize(seg_max); io.co.resize(c_max); }
  api_.submit = [](void* e, const SegIn* sg, u32 n, const u8* pay, u64 len, i64, u32) -> int {
    EchoEngine& E = *(EchoEngine*)e;
    const int p = (int)(E.seq_ & 1);
    const int slot = (int)(E.seq_ % 3);
    E.slot_of_[p] = slot;
    ++E.seq_;
    ++E.steps;
    Io& io = E.io_[p];
    io.ctr = Counters{};
    io.cr.clear();
    io.ctrl.clear();
    std::fill(io.co.begin(), io.co.end(), ConnOut{0, 0});
    std::string& eg = E.slot_[slot];
    eg.clear();
    if (n > E.api_.seg_max) { E.err_ = "too many segments"; return -1; }
    for (auto& f : io.fwd) f.clear();
    io.ready = E.world_ > 1;
    for (u32 k = 0; k < n; ++k) {
      const SegIn& s = sg[k];
      if (s.src + s.len > len) { E.err_ = "segment outside the payload"; return -1; }
      SegOut o{};
      o.conn = s.conn;
      std::string b((const char*)pay + s.src, s.len);
      size_t xp = b.find("XR");
      if (E.world_ > 1 && xp != std::string::npos && xp + 2 < b.size() && b[xp + 2] >= '0' && b[xp + 2] <= '9') {
        const u32 dst = (u32)(b[xp + 2] - '0');
        if (dst < E.world_ && dst != E.rank_) io.fwd[dst].emplace_back(s.conn, b.substr(xp + 3));
        b.resize(xp);
      }
      if (E.paused_[s.conn]) o.status = SS_PAUSED;
      size_t cpos = b.find("CTRL");
      if (!E.paused_[s.conn] && cpos != std::string::npos) {   // control command: pause, hand to host
        CtrlRec r{s.conn, (u32)io.ctrl.size(), 4, (u32)k};
        io.ctrl += "CTRL";
        io.cr.push_back(r);
        o.status |= SS_CTRL;
        E.paused_[s.conn] = 1;
        b.resize(cpos);
      }
      if (E.wblock_[s.conn]) o.status |= SS_PAUSED;   // back-pressured: nothing delivered
      if (!b.empty() && !(o.status & SS_PAUSED)) {
        io.co[s.conn] = ConnOut{(u32)eg.size(), (u32)b.size()};
        eg += b;
        io.ctr.n_deliv++;
      }
      io.so[k] = o;
    }
    io.ctr.n_ctrl = (u32)io.cr.size();
    io.ctr.egress_bytes = (u32)eg.size();
    return p;
  };
  api_.wait_results = [](void* e, int p) -> int {   // (asynchronous: phase B ran)
    EchoEngine& E = *(EchoEngine*)e;
    if (!E.async_) return 0;
    std::unique_lock<std::mutex> g(E.xmu_);
    E.xcv_.wait(g, [&] { return !E.b_due_[p]; });
    return 0;
  };
  api_.egress_slot = [](void* e, int p) -> int { return ((EchoEngine*)e)->slot_of_[p]; };
  api_.egress_copy = [](void*, int) -> int { return 0; };
  api_.egress_wait_slot = [](void*, int) -> int { return 0; };
  api_.error = [](void* e) -> const char* { return ((EchoEngine*)e)->err_.c_str(); };
  api_.counters = [](void* e, int p) -> const Counters* { return &((EchoEngine*)e)->io_[p].ctr; };
  api_.seg_out = [](void* e, int p) -> const SegOut* { return ((EchoEngine*)e)->io_[p].so.data(); };
  api_.conn_out = [](void* e, int p) -> const ConnOut* { return ((EchoEngine*)e)->io_[p].co.data(); };
  api_.ctrl_rec = [](void* e, int p) -> const CtrlRec* { return ((EchoEngine*)e)->io_[p].cr.data(); };
  api_.ctrl = [](void* e, int p) -> const u8* { return (const u8*)((EchoEngine*)e)->io_[p].ctrl.data(); };
  api_.egress_host = [](void* e, int slot) -> const u8* { return (const u8*)((EchoEngine*)e)->slot_[slot].data(); };
  api_.persist_host = [](void*, int) -> const u8* { return nullptr; };
  api_.grow_host = [](void*, int) -> const RingMove* { return nullptr; };
  api_.conn_conf = nullptr;   // every connection's egress is commit-gated
  api_.consumed_host = [](void*, int) -> const ConsumedRec* { return nullptr; };
  api_.exchange = [](void* e, int q, u32 flags, u32* orf) -> int { return ((EchoEngine*)e)->exchange(q, flags, orf); };
  api_.drop_exchange = [](void* e, int q) -> int {
    EchoEngine& E = *(EchoEngine*)e;
    E.io_[q].ready = false;
    E.imports_.clear();
    if (!E.async_) return 0;
    u32 orf = 0;
    return E.collect(&orf);   // the job in flight (its phase B has run)
  };
  api_.launch_b = [](void* e, int p) -> int { ((EchoEngine*)e)->launch_b(p); return 0; };
  api_.links = 0;
  api_.flush_submit = nullptr;
  api_.host_register = nullptr;
  api_.host_unregister = nullptr;
  api_.egress_ready = nullptr;
  api_.host_work = nullptr;
}

void EchoEngine::unpause(u32 conn) {
  if (conn < paused_.size()) paused_[conn] = 0;
}

}  // namespace cmq

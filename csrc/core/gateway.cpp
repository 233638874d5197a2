#include "gateway.hpp"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <stdexcept>

namespace cmq {

Gateway::Gateway(const std::string& host, int port, uint32_t max_conns, bool reuseport)
    : max_conns_(max_conns) {
  lfd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (lfd_ < 0) throw std::runtime_error("socket failed");
  int one = 1;
  setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  if (reuseport) setsockopt(lfd_, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) a.sin_addr.s_addr = htonl(INADDR_ANY);
  if (::bind(lfd_, (sockaddr*)&a, sizeof a) < 0) throw std::runtime_error(std::string("bind: ") + strerror(errno));
  if (::listen(lfd_, 4096) < 0) throw std::runtime_error("listen failed");
  socklen_t l = sizeof a;
  getsockname(lfd_, (sockaddr*)&a, &l);
  port_ = ntohs(a.sin_port);
  epfd_ = epoll_create1(EPOLL_CLOEXEC);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.u64 = 0;   // 0 = listener
  epoll_ctl(epfd_, EPOLL_CTL_ADD, lfd_, &ev);
  conns_.resize(max_conns_);
  for (uint32_t i = max_conns_ - 1; i >= 1; --i) free_.push_back(i);
}

Gateway::~Gateway() {
  for (auto& c : conns_)
    if (c.fd >= 0) ::close(c.fd);
  if (lfd_ >= 0) ::close(lfd_);
  if (epfd_ >= 0) ::close(epfd_);
}

void Gateway::accept_all(GwPoll& r) {
  for (;;) {
    sockaddr_in a{};
    socklen_t l = sizeof a;
    int fd = ::accept4(lfd_, (sockaddr*)&a, &l, SOCK_NONBLOCK | SOCK_CLOEXEC);
    if (fd < 0) return;
    if (free_.empty()) { ::close(fd); continue; }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    uint32_t id = free_.back();
    free_.pop_back();
    GwConn& c = conns_[id];
    c = GwConn{};
    c.fd = fd;
    c.id = id;
    by_fd_[fd] = id;
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = id;
    epoll_ctl(epfd_, EPOLL_CTL_ADD, fd, &ev);
    r.opened.push_back(id);
  }
}

void Gateway::drop(GwConn& c, GwPoll* r) {
  if (c.fd < 0) return;
  epoll_ctl(epfd_, EPOLL_CTL_DEL, c.fd, nullptr);
  ::close(c.fd);
  by_fd_.erase(c.fd);
  c.fd = -1;
  c.dead = true;
  c.out.clear();
  c.out_pos = 0;
  if (r) r->closed.push_back(c.id);
  pending_free_.push_back(c.id);   // reusable after the host has seen the close
}

GwPoll Gateway::poll(int timeout_ms, uint8_t* buf, uint64_t cap, uint64_t per_conn_cap) {
  GwPoll r;
  free_.insert(free_.end(), pending_free_.begin(), pending_free_.end());
  pending_free_.clear();
  epoll_event evs[1024];
  int n = epoll_wait(epfd_, evs, 1024, timeout_ms);
  uint64_t off = 0;
  for (int i = 0; i < n; ++i) {
    uint64_t id = evs[i].data.u64;
    if (id == 0) { accept_all(r); continue; }
    GwConn& c = conns_[id];
    if (c.fd < 0) continue;
    if (evs[i].events & EPOLLOUT) write_some(c);
    if (!(evs[i].events & (EPOLLIN | EPOLLHUP | EPOLLERR))) continue;
    if (c.rpause && !(evs[i].events & (EPOLLHUP | EPOLLERR))) continue;
    uint64_t start = (off + 15) & ~15ull;
    uint64_t room = cap > start ? cap - start : 0;
    if (room > per_conn_cap) room = per_conn_cap;
    if (room == 0) continue;   // buffer full: level-triggered epoll reports it next poll
    uint64_t got = 0;
    bool eof = false;
    while (got < room) {
      ssize_t k = ::recv(c.fd, buf + start + got, room - got, 0);
      if (k > 0) { got += (uint64_t)k; continue; }
      if (k == 0) eof = true;
      else if (errno == EINTR) continue;
      else if (errno != EAGAIN && errno != EWOULDBLOCK) eof = true;
      break;
    }
    rx_bytes += got;
    if (got) {
      if (c.data) {
        r.segs.push_back(GwSeg{c.id, (uint32_t)got, start});
        off = start + got;
      } else {
        r.handshake.emplace_back(c.id, std::string((const char*)buf + start, got));
      }
    }
    if (eof) drop(c, &r);
  }
  r.used = off;
  return r;
}

bool Gateway::write_some(GwConn& c) {
  while (c.out_pos < c.out.size()) {
    ssize_t k = ::send(c.fd, c.out.data() + c.out_pos, c.out.size() - c.out_pos, MSG_NOSIGNAL);
    if (k > 0) { c.out_pos += (size_t)k; tx_bytes += (uint64_t)k; continue; }
    if (k < 0 && errno == EINTR) continue;
    if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLOUT;
      ev.data.u64 = c.id;
      epoll_ctl(epfd_, EPOLL_CTL_MOD, c.fd, &ev);
      return false;
    }
    drop(c, nullptr);
    return false;
  }
  c.out.clear();
  c.out_pos = 0;
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.u64 = c.id;
  epoll_ctl(epfd_, EPOLL_CTL_MOD, c.fd, &ev);
  return true;
}

void Gateway::send(uint32_t conn, const char* data, size_t n) {
  if (conn >= conns_.size()) return;
  GwConn& c = conns_[conn];
  if (c.fd < 0 || n == 0) return;
  bool was_empty = c.out_pos >= c.out.size();
  c.out.append(data, n);
  if (was_empty) dirty_.push_back(conn);
}

uint64_t Gateway::send_egress(const uint8_t* egress, const uint32_t* conn_out, uint32_t n_slots) {
  uint64_t total = 0;
  for (uint32_t i = 0; i < n_slots && i < conns_.size(); ++i) {
    uint32_t o = conn_out[2 * i], l = conn_out[2 * i + 1];
    if (!l) continue;
    send(i, (const char*)egress + o, l);
    total += l;
  }
  return total;
}

void Gateway::flush() {
  std::vector<uint32_t> d;
  d.swap(dirty_);
  for (uint32_t id : d) {
    GwConn& c = conns_[id];
    if (c.fd < 0) continue;
    if (!write_some(c) && c.fd >= 0) dirty_.push_back(id);
  }
}

void Gateway::set_data_mode(uint32_t conn, bool on) {
  if (conn < conns_.size()) conns_[conn].data = on;
}

void Gateway::set_read_paused(uint32_t conn, bool on) {
  if (conn < conns_.size()) conns_[conn].rpause = on;
}

void Gateway::close(uint32_t conn) {
  if (conn < conns_.size()) {
    GwConn& c = conns_[conn];
    if (c.fd >= 0) {
      write_some(c);
      drop(c, nullptr);
    }
  }
}

uint64_t Gateway::pending_bytes() const {
  uint64_t t = 0;
  for (auto& c : conns_) t += c.out.size() - c.out_pos;
  return t;
}

}  // namespace cmq

#include "tls_proxy.hpp"

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
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace cmq {

struct TlsProxy::Pair {
  int cfd = -1, ufd = -1;
  SSL* ssl = nullptr;
  bool handshaken = false, closing = false;
  std::string c2u, u2c;   // decrypted client bytes -> broker; broker bytes -> client (plaintext)
  size_t c2u_pos = 0, u2c_pos = 0;
  bool ssl_want_write = false;
};

static void set_nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK); }

TlsProxy::TlsProxy(const TlsProxyCfg& cfg) : cfg_(cfg) {
  SSL_library_init();
  SSL_load_error_strings();
  ctx_ = SSL_CTX_new(TLS_server_method());
  if (!ctx_) throw std::runtime_error("tls proxy: SSL_CTX_new failed");
  SSL_CTX_set_mode(ctx_, SSL_MODE_ENABLE_PARTIAL_WRITE | SSL_MODE_ACCEPT_MOVING_WRITE_BUFFER);
  if (!cfg_.p12.empty()) {
    FILE* f = fopen(cfg_.p12.c_str(), "rb");
    if (!f) throw std::runtime_error("tls proxy: cannot open keystore " + cfg_.p12);
    PKCS12* p12 = d2i_PKCS12_fp(f, nullptr);
    fclose(f);
    EVP_PKEY* pkey = nullptr;
    X509* cert = nullptr;
    if (!p12 || !PKCS12_parse(p12, cfg_.p12_password.c_str(), &pkey, &cert, nullptr))
      throw std::runtime_error("tls proxy: cannot parse PKCS12 keystore");
    SSL_CTX_use_certificate(ctx_, cert);
    SSL_CTX_use_PrivateKey(ctx_, pkey);
    X509_free(cert);
    EVP_PKEY_free(pkey);
    PKCS12_free(p12);
  } else if (SSL_CTX_use_certificate_chain_file(ctx_, cfg_.cert.c_str()) != 1 ||
             SSL_CTX_use_PrivateKey_file(ctx_, cfg_.key.c_str(), SSL_FILETYPE_PEM) != 1) {
    throw std::runtime_error("tls proxy: cannot load TLS certificate/key");
  }
  lfd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  int one = 1;
  setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)cfg_.port);
  if (inet_pton(AF_INET, cfg_.host.c_str(), &a.sin_addr) != 1) a.sin_addr.s_addr = htonl(INADDR_ANY);
  if (::bind(lfd_, (sockaddr*)&a, sizeof a) < 0 || ::listen(lfd_, 1024) < 0)
    throw std::runtime_error("tls proxy: cannot listen on " + cfg_.host + ":" + std::to_string(cfg_.port));
  socklen_t l = sizeof a;
  getsockname(lfd_, (sockaddr*)&a, &l);
  port_ = ntohs(a.sin_port);
  epfd_ = epoll_create1(EPOLL_CLOEXEC);
  evfd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = lfd_;
  epoll_ctl(epfd_, EPOLL_CTL_ADD, lfd_, &ev);
  ev.data.fd = evfd_;
  epoll_ctl(epfd_, EPOLL_CTL_ADD, evfd_, &ev);
}

TlsProxy::~TlsProxy() {
  stop();
  std::vector<Pair*> all;
  for (auto& kv : by_fd_)
    if (kv.first == kv.second->cfd) all.push_back(kv.second);
  for (Pair* p : all) close_pair(p);
  if (lfd_ >= 0) ::close(lfd_);
  if (epfd_ >= 0) ::close(epfd_);
  if (evfd_ >= 0) ::close(evfd_);
  if (ctx_) SSL_CTX_free(ctx_);
}

void TlsProxy::start() {
  if (running_.exchange(true)) return;
  th_ = std::thread([this] { loop(); });
}

void TlsProxy::stop() {
  if (!running_.exchange(false)) return;
  unsigned long long one = 1;
  ssize_t r = ::write(evfd_, &one, 8);
  (void)r;
  if (th_.joinable()) th_.join();
}

void TlsProxy::accept_all() {
  for (;;) {
    int cfd = ::accept4(lfd_, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
    if (cfd < 0) return;
    int ufd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)cfg_.upstream_port);
    inet_pton(AF_INET, cfg_.upstream_host.c_str(), &a.sin_addr);
    if (ufd < 0 || ::connect(ufd, (sockaddr*)&a, sizeof a) < 0) {   // loopback: immediate
      if (ufd >= 0) ::close(ufd);
      ::close(cfd);
      continue;
    }
    set_nonblock(ufd);
    int one = 1;
    setsockopt(cfd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    setsockopt(ufd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    Pair* p = new Pair();
    p->cfd = cfd;
    p->ufd = ufd;
    p->ssl = SSL_new(ctx_);
    SSL_set_fd(p->ssl, cfd);
    SSL_set_accept_state(p->ssl);
    by_fd_[cfd] = p;
    by_fd_[ufd] = p;
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = cfd;
    epoll_ctl(epfd_, EPOLL_CTL_ADD, cfd, &ev);
    ev.data.fd = ufd;
    epoll_ctl(epfd_, EPOLL_CTL_ADD, ufd, &ev);
    ++accepted_;
    pump(p);
  }
}

void TlsProxy::close_pair(Pair* p) {
  for (int fd : {p->cfd, p->ufd}) {
    if (fd < 0) continue;
    epoll_ctl(epfd_, EPOLL_CTL_DEL, fd, nullptr);
    by_fd_.erase(fd);
    ::close(fd);
  }
  if (p->ssl) SSL_free(p->ssl);
  delete p;
}

// interest: read a side while its destination buffer has room, write while bytes are pending
void TlsProxy::arm(Pair* p) {
  epoll_event ev{};
  ev.data.fd = p->cfd;
  ev.events = (p->c2u.size() - p->c2u_pos < cfg_.buffer ? EPOLLIN : 0u) |
              ((p->u2c_pos < p->u2c.size() || p->ssl_want_write) ? EPOLLOUT : 0u);
  epoll_ctl(epfd_, EPOLL_CTL_MOD, p->cfd, &ev);
  ev.data.fd = p->ufd;
  ev.events = (p->u2c.size() - p->u2c_pos < cfg_.buffer ? EPOLLIN : 0u) | (p->c2u_pos < p->c2u.size() ? EPOLLOUT : 0u);
  epoll_ctl(epfd_, EPOLL_CTL_MOD, p->ufd, &ev);
}

void TlsProxy::pump(Pair* p) {
  char buf[1 << 16];
  bool dead = false;
  p->ssl_want_write = false;
  if (!p->handshaken) {
    int r = SSL_do_handshake(p->ssl);
    if (r == 1) {
      p->handshaken = true;
    } else {
      int e = SSL_get_error(p->ssl, r);
      if (e == SSL_ERROR_WANT_WRITE) p->ssl_want_write = true;
      else if (e != SSL_ERROR_WANT_READ) dead = true;
    }
  }
  bool progress = true;
  while (!dead && p->handshaken && progress) {
    progress = false;
    // client -> broker
    while (p->c2u.size() - p->c2u_pos < cfg_.buffer) {
      int k = SSL_read(p->ssl, buf, sizeof buf);
      if (k > 0) { p->c2u.append(buf, (size_t)k); progress = true; continue; }
      int e = SSL_get_error(p->ssl, k);
      if (e == SSL_ERROR_WANT_WRITE) p->ssl_want_write = true;
      else if (e != SSL_ERROR_WANT_READ) dead = true;
      break;
    }
    while (p->c2u_pos < p->c2u.size()) {
      ssize_t k = ::send(p->ufd, p->c2u.data() + p->c2u_pos, p->c2u.size() - p->c2u_pos, MSG_NOSIGNAL);
      if (k > 0) { p->c2u_pos += (size_t)k; progress = true; continue; }
      if (k < 0 && (errno == EAGAIN || errno == EINTR)) break;
      dead = true;
      break;
    }
    if (p->c2u_pos == p->c2u.size()) { p->c2u.clear(); p->c2u_pos = 0; }
    // broker -> client
    while (!dead && p->u2c.size() - p->u2c_pos < cfg_.buffer) {
      ssize_t k = ::recv(p->ufd, buf, sizeof buf, 0);
      if (k > 0) { p->u2c.append(buf, (size_t)k); progress = true; continue; }
      if (k == 0) p->closing = true;
      else if (errno != EAGAIN && errno != EINTR) dead = true;
      break;
    }
    while (!dead && p->u2c_pos < p->u2c.size()) {
      int k = SSL_write(p->ssl, p->u2c.data() + p->u2c_pos, (int)std::min<size_t>(p->u2c.size() - p->u2c_pos, 1 << 20));
      if (k > 0) { p->u2c_pos += (size_t)k; progress = true; continue; }
      int e = SSL_get_error(p->ssl, k);
      if (e == SSL_ERROR_WANT_WRITE || e == SSL_ERROR_WANT_READ) p->ssl_want_write = e == SSL_ERROR_WANT_WRITE;
      else dead = true;
      break;
    }
    if (p->u2c_pos == p->u2c.size()) { p->u2c.clear(); p->u2c_pos = 0; }
  }
  if (dead || (p->closing && p->u2c.empty())) {
    close_pair(p);
    return;
  }
  arm(p);
}

void TlsProxy::loop() {
  epoll_event evs[256];
  while (running_) {
    int n = epoll_wait(epfd_, evs, 256, 100);
    for (int i = 0; i < n; ++i) {
      int fd = evs[i].data.fd;
      if (fd == lfd_) { accept_all(); continue; }
      if (fd == evfd_) continue;
      auto it = by_fd_.find(fd);
      if (it == by_fd_.end()) continue;
      pump(it->second);
    }
  }
}

}  // namespace cmq

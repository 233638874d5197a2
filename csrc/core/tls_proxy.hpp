// AMQPS for the GPU-path server: a TLS terminator in front of the pipelined front end.
//
// The reference serves AMQP and AMQPS from the same engine (AMQPServer.scala:70-92,
// Amqp.scala:177-210 TLS BidiFlow per connection).  The GPU front end gathers raw
// socket bytes straight into the pinned ingress arena, so TLS is terminated here instead:
// one epoll thread accepts TLS clients (PEM or PKCS12 keystore, like broker.cpp), and
// relays decrypted bytes to the broker's plain listener over loopback and back.  The
// broker sees an ordinary AMQP connection; SASL EXTERNAL still answers "" like the
// reference (SaslMechanism.scala:90-98).
#pragma once
#include <atomic>
#include <string>
#include <thread>
#include <unordered_map>

typedef struct ssl_ctx_st SSL_CTX;
typedef struct ssl_st SSL;

namespace cmq {

struct TlsProxyCfg {
  std::string host = "127.0.0.1";
  int port = 0;                      // TLS listener (0 = any)
  std::string upstream_host = "127.0.0.1";
  int upstream_port = 5672;
  std::string cert, key, p12, p12_password;
  size_t buffer = 1 << 20;           // per direction per connection
};

class TlsProxy {
 public:
  explicit TlsProxy(const TlsProxyCfg& cfg);
  ~TlsProxy();
  int port() const { return port_; }
  void start();
  void stop();
  unsigned long long connections() const { return accepted_; }

 private:
  struct Pair;
  void loop();
  void accept_all();
  void pump(Pair* p);
  void arm(Pair* p);
  void close_pair(Pair* p);

  TlsProxyCfg cfg_;
  SSL_CTX* ctx_ = nullptr;
  int lfd_ = -1, epfd_ = -1, evfd_ = -1, port_ = 0;
  std::thread th_;
  std::atomic<bool> running_{false};
  std::unordered_map<int, Pair*> by_fd_;
  std::atomic<unsigned long long> accepted_{0};
};

}  // namespace cmq

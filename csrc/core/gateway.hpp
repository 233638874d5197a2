// Batched socket front end for the GPU data plane.
//
// One call to poll() accepts new connections and drains every readable socket into a
// caller-provided pinned buffer, one contiguous 16-byte-aligned segment per connection:
// the result is exactly the SegIn list the HIP engine consumes, so ingress bytes go
// from the kernel's socket buffers to the GPU with a single copy and no per-connection
// Python work.  send_egress() writes a whole step's rendered egress (one host buffer +
// per-connection {offset, length}) to the sockets.  Connections still in the AMQP
// handshake are returned separately (handshake_bytes) so the control plane can answer
// Start/Tune/Open before switching them to data mode.
//
// Reference counterpart: the Akka-Streams TCP stage feeding FrameStage
// (chana-mq-server/.../engine/FrameStage.scala:272-320, Amqp.scala) — here batched
// across connections per step instead of per connection.
#pragma once
#include <cstdint>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace cmq {

struct GwSeg {            // layout of dp_common.h SegIn
  uint32_t conn, len;
  uint64_t src;
};

struct GwConn {
  int fd = -1;
  uint32_t id = 0;
  bool data = false;      // bytes go to the data plane (else: handshake bytes to the host)
  bool dead = false;
  bool rpause = false;    // reads paused (ingress back-pressure: the data plane still holds a backlog)
  std::string out;        // pending egress
  size_t out_pos = 0;
};

struct GwPoll {
  std::vector<GwSeg> segs;
  uint64_t used = 0;
  std::vector<std::pair<uint32_t, std::string>> handshake;
  std::vector<uint32_t> opened, closed;
};

class Gateway {
 public:
  Gateway(const std::string& host, int port, uint32_t max_conns, bool reuseport);
  ~Gateway();
  int port() const { return port_; }
  GwPoll poll(int timeout_ms, uint8_t* buf, uint64_t cap, uint64_t per_conn_cap);
  void send(uint32_t conn, const char* data, size_t n);
  // egress: host buffer + ConnOut {off, len} per connection slot [0, n_slots)
  uint64_t send_egress(const uint8_t* egress, const uint32_t* conn_out, uint32_t n_slots);
  void flush();
  void set_data_mode(uint32_t conn, bool on);
  void set_read_paused(uint32_t conn, bool on);
  void close(uint32_t conn);
  uint64_t pending_bytes() const;
  uint64_t rx_bytes = 0, tx_bytes = 0;

 private:
  void accept_all(GwPoll& r);
  void drop(GwConn& c, GwPoll* r);
  bool write_some(GwConn& c);
  int lfd_ = -1, epfd_ = -1, port_ = 0;
  uint32_t max_conns_;
  std::vector<GwConn> conns_;          // by slot id (0 unused)
  std::vector<uint32_t> free_, pending_free_;
  std::unordered_map<int, uint32_t> by_fd_;
  std::vector<uint32_t> dirty_;        // slots with pending output
};

}  // namespace cmq

// Native AMQP 0-9-1 broker: epoll (+OpenSSL) transport, connection state machine,
// method handlers, exchanges/queues/bindings, delivery loop, acks, confirms, tx,
// heartbeats, back-pressure and Cassandra-schema persistence.
//
// This is the CPU host path (BASELINE config 1) and the control plane that the GPU
// data plane plugs into.  Reference counterparts (all under /root/reference):
//   transport            chana-mq-base/.../Amqp.scala, ConnectionContext.scala
//   connection engine    chana-mq-server/.../engine/FrameStage.scala (C22a-r)
//   SASL                 chana-mq-server/.../engine/SaslMechanism.scala
//   session model        chana-mq-base/.../model/AMQ{Connection,Channel,Consumer}.scala
//   entities             chana-mq-server/.../entity/{Vhost,Exchange,Queue,Message}Entity.scala
//   routing              chana-mq-server/.../engine/QueueMatcher.scala
//   ids                  chana-mq-server/.../service/IdGenerator.scala
// Unlike the reference's actor-per-entity design, all broker state is owned by one
// event-loop thread (no locks on the hot path); other threads talk to it through a
// command queue woken by an eventfd.
#pragma once
#include <atomic>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "codec.hpp"
#include "store.hpp"

typedef struct ssl_st SSL;
typedef struct ssl_ctx_st SSL_CTX;

namespace cmq {

struct BrokerConfig {
  std::string host = "0.0.0.0";
  int port = 5672;                 // chana.mq.amqp.server.port
  bool amqp_enable = true;
  int tls_port = 5671;             // chana.mq.amqps.server.port
  bool tls_enable = false;
  std::string tls_cert, tls_key;   // PEM
  std::string tls_p12, tls_p12_password;  // PKCS12 keystore (chana.mq.ssl.keystore/password)
  u16 channel_max = 0;             // chana.mq.amqp.connection.channel-max (0 = 65535)
  u32 frame_max = 131072;          // ...frame-max
  u32 frame_min = 4096;            // ...frame-min
  u16 heartbeat = 30;              // ...heartbeat (s)
  std::string default_vhost = "AMQ.DEFAULT";  // chana.mq.amqp.vhost.default-id
  std::string data_dir;            // "" = memory only
  bool fsync = true;
  u32 worker_id = 0;               // snowflake worker (<=1023)
  u64 mem_high_watermark = 0;      // bytes of queued message data; 0 = off
  u64 mem_low_watermark = 0;
  bool flow_channel = false;       // back-pressure via Channel.Flow (else Connection.Blocked)
  u32 max_connections = 0;         // 0 = unlimited
  bool hash_wildcard = true;       // topic '#' (false = reference parity: literal '#')
  std::string product = "chana.mq";
  std::string version = "0.1.0";
};

class IdGenerator {   // snowflake: ms<<22 | worker<<12 | seq  (IdGenerator.scala:28-83)
 public:
  explicit IdGenerator(u32 worker) : worker_(worker & 1023) {}
  u64 next();
 private:
  u32 worker_;
  i64 last_ms_ = -1;
  u32 seq_ = 0;
};

struct Queue;
struct Conn;
struct Exchange;

struct Message {
  u64 id = 0;
  std::string exchange, rk, props, body;
  bool persistent = false;
  i64 expire_at = 0;
  i64 ts_ms = 0;
  int refs = 0;         // queues holding it (ready + unacked)
  bool stored = false;  // msgs row exists
};
using MsgPtr = std::shared_ptr<Message>;

struct QEntry {
  MsgPtr m;
  i64 offset;
  i64 expire_at;
  bool redelivered;
};

struct Consumer {
  std::string tag;
  Conn* conn;
  u16 ch;
  Queue* q;
  bool no_ack;
  bool exclusive;
  u32 unacked = 0;
};

struct Queue {
  std::string vhost, name, id;
  bool durable = false, exclusive = false, auto_delete = false;
  Conn* owner = nullptr;
  i64 ttl = 0;
  Table args;
  std::deque<QEntry> ready;
  i64 next_offset = 0;
  std::vector<Consumer*> consumers;
  size_t rr = 0;
  bool had_consumer = false;
  u64 unacked = 0;
  u64 bytes = 0;
  u64 published = 0, delivered = 0, acked = 0;
};

struct Binding {
  std::string key;
  Queue* q = nullptr;         // queue destination
  Exchange* x = nullptr;      // exchange destination (Exchange.Bind extension)
  std::vector<std::string> words;
  Table args;
};

struct Exchange {
  std::string vhost, name, type, id;
  bool durable = false, auto_delete = false, internal = false;
  Table args;
  std::vector<Binding> bindings;
  std::unordered_map<std::string, std::vector<size_t>> direct;  // key -> binding indices
  void reindex();
};

struct Vhost {
  std::string name;
  bool active = true;
  std::map<std::string, std::unique_ptr<Exchange>> exchanges;
  std::map<std::string, std::unique_ptr<Queue>> queues;
};

struct Unacked {
  MsgPtr m;
  std::string qname;
  i64 offset;
  Consumer* c;          // may be null after cancel
  std::string ctag;
};

struct PendingPub {
  std::string exchange, rk;
  bool mandatory, immediate;
  std::string props, body;
};

struct Channel {
  u16 id = 0;
  bool closing = false;
  bool flow_out = true;        // server delivers (client Channel.Flow)
  bool flow_in = true;         // client may publish (server Channel.Flow)
  bool confirm = false, tx = false;
  u64 next_tag = 1;
  std::map<u64, Unacked> unacked;
  u32 prefetch_count = 0, prefetch_size = 0;
  bool global = false;
  u32 unacked_count = 0;
  u64 pub_seq = 0, confirmed = 0, confirm_pending_sync = 0;
  std::map<std::string, std::unique_ptr<Consumer>> consumers;
  // content assembly (CommandAssembler.scala:33-130)
  bool have_method = false, have_header = false;
  Method method;
  u64 body_size = 0;
  std::string props, body;
  // tx
  std::vector<PendingPub> tx_pubs;
  std::vector<std::tuple<u16, u64, bool, bool>> tx_acks;  // (method id, tag, multiple, requeue)
};

enum ConnState { CS_HANDSHAKE, CS_START_SENT, CS_TUNE_SENT, CS_OPEN, CS_CLOSING, CS_CLOSED };

struct Conn {
  u64 id;
  int fd;
  SSL* ssl = nullptr;
  bool tls_handshaken = false;
  ConnState state = CS_HANDSHAKE;
  std::string in;
  size_t in_pos = 0;
  std::string out;
  size_t out_pos = 0;
  u32 frame_max = 131072;
  u16 channel_max = 65535;
  u16 heartbeat = 0;
  i64 last_rx = 0, last_tx = 0, close_deadline = 0;
  Vhost* vhost = nullptr;
  std::string user, peer;
  Table client_props;
  std::map<u16, Channel> channels;
  std::set<Queue*> exclusive_queues;
  bool cap_blocked = false, cap_cancel_notify = false;
  bool blocked = false;        // reading paused by back-pressure
  bool want_write = false;
  bool dead = false;
  FrameParser parser;
  u64 published = 0, delivered = 0;
};

struct BrokerStats {
  u64 published = 0, routed = 0, unroutable = 0, delivered = 0, acked = 0, requeued = 0, expired = 0;
  u64 returned = 0, confirms = 0, connections = 0, channels = 0, bytes_in = 0, bytes_out = 0;
};

class Broker {
 public:
  explicit Broker(const BrokerConfig& cfg);
  ~Broker();
  int listen_port() const { return bound_port_; }
  int listen_tls_port() const { return bound_tls_port_; }
  void start();                 // bind + spawn the event-loop thread
  void stop();
  bool running() const { return running_; }
  // thread-safe admin API (AdminApi.scala): executed on the loop thread
  bool create_vhost(const std::string& name);
  bool delete_vhost(const std::string& name);
  std::string stats_json();
  std::string queues_json();

 private:
  friend struct BrokerTestAccess;
  void loop();
  void post(std::function<void()> fn);
  void drain_posted();
  void setup_listeners();
  void setup_tls();
  void accept_all(int lfd, bool tls);
  void on_readable(Conn* c);
  void on_writable(Conn* c);
  void process_input(Conn* c);
  void flush(Conn* c);
  void close_conn(Conn* c);
  void reap();
  void timers(i64 now);
  void kick_write(Conn* c);

  // protocol
  void handle_frame(Conn* c, Frame& f);
  void dispatch(Conn* c, Channel* ch, Method& m);
  void on_connection(Conn* c, Method& m);
  void on_channel(Conn* c, u16 chid, Method& m);
  void on_exchange(Conn* c, Channel& ch, Method& m);
  void on_queue(Conn* c, Channel& ch, Method& m);
  void on_basic(Conn* c, Channel& ch, Method& m);
  void on_publish(Conn* c, Channel& ch, const Method& m, std::string&& props, std::string&& body);
  void send_method(Conn* c, u16 ch, const Method& m);
  void send_connection_close(Conn* c, u16 code, const std::string& text, u16 cls, u16 mid);
  void send_channel_close(Conn* c, Channel& ch, u16 code, const std::string& text, u16 cls, u16 mid);

  // entities
  Vhost* vhost(const std::string& name, bool create);
  void ensure_standard_exchanges(Vhost* v);
  Exchange* find_exchange(Vhost* v, const std::string& name);
  Queue* find_queue(Vhost* v, const std::string& name);
  void delete_queue(Queue* q, bool notify);
  void delete_exchange(Exchange* x);
  void unbind_queue_everywhere(Queue* q);
  void route(Exchange* x, const std::string& rk, const Props& pr, std::vector<Queue*>& out, int depth = 0);
  void enqueue(Queue* q, const MsgPtr& m, bool redelivered = false);
  void mark_dirty(Queue* q) { dirty_.insert(q); }
  void deliver(Queue* q);
  bool consumer_credit(Consumer* c);
  void send_deliver(Consumer* c, QEntry& e);
  void release(const std::string& qname, Vhost* v, const MsgPtr& m, i64 offset, bool was_unacked);
  void ack(Conn* c, Channel& ch, u64 tag, bool multiple);
  void reject(Conn* c, Channel& ch, u64 tag, bool multiple, bool requeue);
  void requeue_unacked(Conn* c, Channel& ch, std::vector<u64> tags);
  void cancel_consumer(Conn* c, Channel& ch, const std::string& tag, bool notify);
  void close_channel_state(Conn* c, Channel& ch);
  void expire_head(Queue* q, i64 now);
  void check_memory();
  void confirm_flush();

  // persistence
  void persist_exchange(Exchange* x);
  void persist_bind(Exchange* x, const Binding& b);
  void persist_queue_meta(Queue* q);
  void recover();

  BrokerConfig cfg_;
  IdGenerator ids_;
  Store store_;
  std::map<std::string, std::unique_ptr<Vhost>> vhosts_;
  std::unordered_map<int, std::unique_ptr<Conn>> conns_;
  std::set<Queue*> dirty_;
  std::set<Conn*> confirm_conns_;
  u64 next_conn_id_ = 1;
  u64 queued_bytes_ = 0;
  bool mem_alarm_ = false;
  int epfd_ = -1, lfd_ = -1, tls_lfd_ = -1, evfd_ = -1;
  int bound_port_ = -1, bound_tls_port_ = -1;
  SSL_CTX* ssl_ctx_ = nullptr;
  std::thread thr_;
  std::atomic<bool> running_{false}, stop_{false};
  std::mutex post_mu_;
  std::vector<std::function<void()>> posted_;
  i64 last_timer_ = 0;
  u64 ctag_seq_ = 0;
  BrokerStats stats_;
};

}  // namespace cmq

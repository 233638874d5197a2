// Embedded, schema-identical replacement for the reference's Cassandra store.
//
// Same tables / keys / column types as chana-mq-server/src/main/resources/create-cassantra.cql
// and the same 22 operations as trait DBOpService (chana-mq-server/.../store/package.scala:15-43),
// with Cassandra row semantics that matter to the broker: upsert by primary key,
// clustering order ASC on queues.offset, and per-row TTL (USING TTL seconds).
// Durability: every mutation is appended to a CRC-checked write-ahead log; sync() is a
// group-commit fsync the broker calls before it sends publisher confirms for persistent
// messages (SURVEY §3.3 "confirm only after the durable write").  open() replays the log;
// compact() rewrites it from the live tables.
#pragma once
#include <cstdint>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <tuple>
#include <vector>

namespace cmq {

struct MsgRow {            // msgs
  int64_t id = 0;
  int64_t tstamp = 0;      // header timestamp, epoch ms (CassandraOpService.scala:406-411)
  std::string header;      // BasicProperties.writeTo: weight u16 | bodySize u64 | flags | props (no class id)
  std::string body;
  std::string exchange, routing;
  bool durable = false;
  int32_t refer = 0;
  int64_t expire_at = 0;   // from USING TTL; 0 = none
};
struct QueueMsgRow {       // queues / queues_deleted / queue_unacks / queue_unacks_deleted
  int64_t offset = 0, msgid = 0;
  int32_t size = 0;
  int64_t expire_at = 0;
};
struct QueueMetaRow {      // queue_metas
  int64_t lconsumed = -1;
  std::set<std::string> consumers;
  bool durable = false;
  int64_t ttl = 0;
};
struct QueueMetaDeletedRow {  // queue_metas_deleted (nconsumer int: SURVEY A.Q22 fixed)
  int64_t lconsumed = -1;
  int32_t nconsumer = 0;
  bool durable = false;
};
struct ExchangeRow {       // exchanges
  std::string tpe;
  bool durable = false, autodel = false, internal = false;
  std::map<std::string, std::string> args;
};
struct BindRow { std::string queue, key; std::map<std::string, std::string> args; };

class Store {
 public:
  Store() = default;
  ~Store();
  // dir == "" -> memory only (the in-memory fake of SURVEY §4.2 item 5)
  void open(const std::string& dir, bool fsync_enabled = true);
  void close();
  void sync();             // group commit
  void compact();          // rewrite the WAL from live rows
  bool persistent() const { return fd_ >= 0; }
  int64_t now_ms() const;

  // ---- messages
  void insertMessage(const MsgRow& m, int64_t ttl_ms);
  void insertMessage(MsgRow&& m, int64_t ttl_ms);
  void updateMessageReferCount(int64_t id, int32_t refer);
  bool selectMessage(int64_t id, MsgRow* out);
  void deleteMessage(int64_t id);
  // ---- queues
  void insertQueueMeta(const std::string& q, int64_t lconsumed, const std::set<std::string>& consumers,
                       bool durable, int64_t ttl);
  void insertQueueMsg(const std::string& q, int64_t offset, int64_t msgid, int32_t size, int64_t ttl_ms);
  void insertLastConsumed(const std::string& q, int64_t lconsumed);
  void consumedQueueMessages(const std::string& q, int64_t lconsumed, const std::vector<QueueMsgRow>& unacks);
  bool selectQueue(const std::string& q, QueueMetaRow* meta, std::vector<QueueMsgRow>* msgs,
                   std::vector<QueueMsgRow>* unacks);
  void forceDeleteQueue(const std::string& q);
  void pendingDeleteQueue(const std::string& q);
  void deleteConsumedQueueMsgs(const std::string& q, int64_t upto_offset);
  void insertQueueUnack(const std::string& q, int64_t offset, int64_t msgid, int32_t size);
  void deleteQueueUnack(const std::string& q, int64_t msgid);
  void deleteQueueMsg(const std::string& q, int64_t offset);
  // ---- exchanges
  void insertExchange(const std::string& id, const ExchangeRow& x);
  void insertBind(const std::string& id, const std::string& queue, const std::string& key,
                  const std::map<std::string, std::string>& args);
  bool selectExchange(const std::string& id, ExchangeRow* x, std::vector<BindRow>* binds);
  void deleteBind(const std::string& id, const std::string& queue, const std::string& key);
  void deleteBindsOfQueue(const std::string& queue);
  void deleteExchange(const std::string& id);
  // ---- vhosts
  void insertVhost(const std::string& id, bool active);
  bool selectVhost(const std::string& id, bool* active);
  void deleteVhost(const std::string& id);

  // ---- recovery / inspection
  std::vector<std::string> vhostIds();
  std::vector<std::string> exchangeIds();
  std::vector<std::string> queueIds();
  size_t rowCount(const std::string& table);
  uint64_t walBytes() const { return wal_bytes_ + wbuf_.size(); }
  std::vector<int64_t> messageIds();

 private:
  void append(uint8_t op, const std::string& payload);
  void append_wal(uint8_t op, const std::string& payload);
  void apply(uint8_t op, const std::string& payload);
  void replay();
  void write_all(const std::string& rec);
  void flush_wal();
  std::string wbuf_;       // WAL records not yet written

  std::recursive_mutex mu_;
  int fd_ = -1;
  std::string path_;
  bool fsync_ = true;
  bool dirty_ = false;
  bool replaying_ = false;
  uint64_t wal_bytes_ = 0;

  std::map<int64_t, MsgRow> msgs_;
  std::map<std::string, std::map<int64_t, QueueMsgRow>> queues_, queues_deleted_;
  std::map<std::string, QueueMetaRow> queue_metas_;
  std::map<std::string, QueueMetaDeletedRow> queue_metas_deleted_;
  std::map<std::string, std::map<int64_t, QueueMsgRow>> queue_unacks_, queue_unacks_deleted_;  // key msgid
  std::map<std::string, ExchangeRow> exchanges_;
  std::map<std::string, std::map<std::pair<std::string, std::string>, BindRow>> binds_;
  std::map<std::string, bool> vhosts_;
};

}  // namespace cmq

// Embedded, schema-identical replacement for the reference's Cassandra store.
//
// Same tables / keys / column types as chana-mq-server/src/main/resources/create-cassantra.cql
// and the same 22 operations as trait DBOpService (chana-mq-server/.../store/package.scala:15-43),
// with Cassandra row semantics that matter to the broker: upsert by primary key,
// clustering order ASC on queues.offset, and per-row TTL (USING TTL seconds).
// Durability: every mutation is appended to a CRC-checked write-ahead log; sync() is a
// group-commit fsync the broker calls before it sends publisher confirms for persistent
// messages (SURVEY §3.3 "confirm only after the durable write").  open() replays the log.
//
// Reclamation (the reference's Cassandra drops deleted rows itself,
// CassandraOpService.scala:395-417): the WAL is compacted in the background once it is
// auto_ratio x the live rows (and >= auto_min bytes).  A compaction snapshots the live
// rows into a new file in short locked chunks while appends continue into the old WAL,
// then copies the old WAL's tail written since the switch point (mostly unlocked) and
// atomically renames the new file over it.  Every record is an upsert / delete / field
// set by key, so replaying the tail over a snapshot that already saw some of those
// changes yields the same rows; group commits are never blocked for a whole rewrite.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "bodylog.hpp"

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
  // body in the body log (bodylog.hpp) instead of in this row: header/body/exchange/routing
  // are read back from (bseg, boff, blen) by selectMessage; bseg < 0 = inline row
  int64_t bseg = -1;
  uint64_t boff = 0;
  uint32_t blen = 0;
};
// a persistent message of the GPU write-behind whose bytes are a device persist record
// (step_abi.h PersistHdr + exchange | routing key | properties | body)
struct BodyRef { int64_t id, tstamp; const char* rec; uint32_t len; int32_t refer; };
// one row change of the write-behind's batched path (Store::applyRows); q indexes the
// batch's queue ids
enum RowOpKind : uint8_t {
  ROW_QMSG_INS, ROW_QMSG_DEL, ROW_QUNACK_INS, ROW_QUNACK_DEL, ROW_MSG_DEL, ROW_MSG_REFER /* refer in size */,
  ROW_MSG_REF /* msgs row in the body log: refer in q, (seg, offset, size) the body, tstamp */
};
struct RowOp {
  uint8_t op, pad[3];
  uint32_t q;
  int64_t offset, msgid;
  int32_t size;
  uint32_t seg;
  int64_t tstamp;
};
static_assert(sizeof(RowOp) == 40, "RowOp layout (WAL format)");
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

struct CompactStats {
  uint64_t runs = 0, last_before = 0, last_after = 0, tail_bytes = 0;
  double last_s = 0, max_lock_s = 0;
  uint64_t failures = 0;        // background runs that failed (ENOSPC, EIO, rename, ...)
  std::string last_error;
};

class Store {
 public:
  Store() = default;
  ~Store();
  // dir == "" -> memory only (the in-memory fake of SURVEY §4.2 item 5)
  void open(const std::string& dir, bool fsync_enabled = true);
  void close();
  void sync();             // group commit (may start a background compaction)
  void compact();          // rewrite the WAL from live rows now (waits for it)
  // background compaction policy: WAL > ratio x live estimate and > min_bytes (ratio 0 = off)
  void set_auto_compact(double ratio, uint64_t min_bytes) { auto_ratio_ = ratio; auto_min_ = min_bytes; }
  // a byte budget for the store on disk (WAL appends + body log), 0 = none: writes past it
  // fail like a full disk (ENOSPC), which the write-behind reports as a store failure --
  // operators cap a store this way; tests use it to fill a store deterministically
  void set_quota(uint64_t bytes);
  void wait_compaction();
  CompactStats compactStats();
  uint64_t liveEstimate();
  bool persistent() const { return fd_ >= 0; }
  int64_t now_ms() const;

  // ---- messages
  void insertMessage(const MsgRow& m, int64_t ttl_ms);
  void insertMessage(MsgRow&& m, int64_t ttl_ms);
  // bodies to the body log (written by its stripes from the given records, which must stay
  // valid until the next sync()), rows to the WAL.  Needs a store on disk
  void insertMessageRefs(const BodyRef* refs, size_t n);
  // start writing bodies to the body log (locations now, durable by the next sync())
  void placeBodies(const char* const* recs, const uint32_t* lens, size_t n, BodyLog::Loc* out);
  // a group of row changes as one WAL record, applied in order
  void applyRows(const std::vector<const std::string*>& qids, const RowOp* ops, size_t n);
  bool hasBodyLog() const { return body_ != nullptr; }
  void configureBodyLog(int stripes, uint64_t seg_bytes) { if (body_) body_->configure(stripes, seg_bytes); }
  BodyLog::Stats bodyStats() { return body_ ? body_->stats() : BodyLog::Stats{}; }
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
  // ---- *_deleted tables (pendingDeleteQueue copies; Cassandra interop import/export)
  std::vector<std::string> deletedQueueIds();
  bool selectDeletedQueue(const std::string& q, QueueMetaDeletedRow* meta, std::vector<QueueMsgRow>* msgs,
                          std::vector<QueueMsgRow>* unacks);
  void insertDeletedQueueMeta(const std::string& q, int64_t lconsumed, int32_t nconsumer, bool durable);
  void insertDeletedQueueMsg(const std::string& q, int64_t offset, int64_t msgid, int32_t size);
  void insertDeletedQueueUnack(const std::string& q, int64_t offset, int64_t msgid, int32_t size);

  // ---- change feed (store/cassandra_live.py, the live Cassandra mirror): with it on, every
  // change marks the key of the row (or the partition, for range / whole-queue changes) it
  // touched; mirrorTake hands over up to max_keys marked keys of each kind and clears them,
  // and the mirror reads those rows' current state back (select*) and writes it -- repeated
  // changes to one row between two takes cost one write (a publish acked before the take:
  // none).  Replay and compaction mark nothing.
  struct MirrorKeys {
    std::vector<int64_t> msgs;
    std::vector<std::pair<std::string, int64_t>> qmsgs, qunacks;   // (queue, offset) / (queue, msgid)
    std::vector<std::string> qmetas, qparts, xs, vhosts, deleted;
  };
  void setMirror(bool on);
  MirrorKeys mirrorTake(size_t max_keys);
  size_t mirrorPending();
  bool selectQueueMsg(const std::string& q, int64_t offset, QueueMsgRow* out);
  bool selectQueueUnack(const std::string& q, int64_t msgid, QueueMsgRow* out);
  bool selectQueueMeta(const std::string& q, QueueMetaRow* out);

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
  void put_msg(MsgRow&& m);
  void apply_rows(const std::vector<const std::string*>& qids, const RowOp* ops, size_t n);           // upsert into msgs_ (body log accounting)
  void drop_msg(std::map<int64_t, MsgRow>::iterator it);
  void flush_wal();
  void maybe_compact();               // mu_ held
  void compact_run();                 // the compaction (background thread or compact())
  bool snapshot_chunk(int table, std::string& key, int64_t& sub, std::string& out);
  std::string wbuf_;       // WAL records not yet written
  uint64_t msg_bytes_ = 0;            // live message row bytes (liveEstimate)
  double auto_ratio_ = 4.0;
  uint64_t auto_min_ = 256ull << 20;
  uint64_t auto_backoff_ = 0;         // after a failed background run: retry once the WAL passes this
  std::thread compact_th_;
  std::atomic<bool> compacting_{false}, compact_stop_{false};
  std::string close_error_;          // what the final sync of close() reported (it never throws)
  CompactStats cstats_;

  std::recursive_mutex mu_;
  int fd_ = -1;
  std::string path_;
  bool fsync_ = true;
  bool dirty_ = false;
  bool replaying_ = false;
  uint64_t wal_bytes_ = 0;
  uint64_t quota_ = 0;
  std::atomic<uint64_t> quota_used_{0};

  std::unique_ptr<BodyLog> body_;     // with a store on disk
  std::map<int64_t, MsgRow> msgs_;
  std::map<std::string, std::map<int64_t, QueueMsgRow>> queues_, queues_deleted_;
  std::map<std::string, QueueMetaRow> queue_metas_;
  std::map<std::string, QueueMetaDeletedRow> queue_metas_deleted_;
  std::map<std::string, std::map<int64_t, QueueMsgRow>> queue_unacks_, queue_unacks_deleted_;  // key msgid
  std::map<std::string, ExchangeRow> exchanges_;
  std::map<std::string, std::map<std::pair<std::string, std::string>, BindRow>> binds_;
  std::map<std::string, bool> vhosts_;

  // change feed (setMirror)
  bool mirror_ = false;
  std::set<int64_t> md_msgs_;
  std::set<std::pair<std::string, int64_t>> md_qmsgs_, md_qunacks_;
  std::set<std::string> md_qmetas_, md_qparts_, md_xs_, md_vhosts_, md_deleted_;
  bool marking() const { return mirror_ && !replaying_; }
};

}  // namespace cmq

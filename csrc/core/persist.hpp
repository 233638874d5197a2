// Native write-behind persistence for the GPU data plane (BASELINE config 4).
//
// The device emits, per step, one PersistHdr record per enqueue of a persistent message
// into a durable queue (packed with the message bytes) and one ConsumedRec per persistent
// message that changes state in a durable queue (step_abi.h).  PersistWorker turns them
// into rows of the Cassandra-schema store (store.hpp — the tables of the reference's
// create-cassantra.cql) on its own thread: it applies every pending batch, commits them
// with one fsync (group commit) and then releases the held egress of those steps to the
// front end, so a publisher confirm never leaves before its message is durable
// (CassandraOpService.scala:395-417 insertMessage / insertQueueMsg; FrameStage.scala:571-596
// confirms after the entities answered).  Steps keep running while the commit is in flight.
//
// Rows are addressed by (queue, message id) -> the queue offset they were stored at, since
// device queue positions change on requeue; a message row is deleted when the last queue
// row referencing it goes (MessageEntity.scala:134-166 refer counting).
//
// Group commit coalescing: the batches that queued up while the previous fsync ran are
// applied as one group, and a row born in the group is only written at its end — a
// persistent message published, delivered and acked within one group never reaches the
// WAL (nothing to recover), so the store's work falls as the load rises.
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../kernels/step_abi.h"
#include "flatmap.hpp"
#include "store.hpp"

namespace cmq {

class PersistWorker {
 public:
  explicit PersistWorker(Store* store);
  ~PersistWorker();
  void start();
  void stop();
  // committed steps are reported here (the front end releases their held egress)
  void on_commit(std::function<void(u64)> cb) { commit_cb_ = std::move(cb); }
  void set_queue(u32 slot, const std::string& qid);   // durable queue slot -> entity id ("" = none)
  void seed_row(const std::string& qid, i64 msgid, i64 offset, i32 size, bool unack, int refs);
  // records of step `step` (0 = a host-run step / Basic.Get: no egress held)
  void submit(u64 step, std::string persist, std::string consumed);
  void drain();                                       // every submitted batch committed
  // a group commit starts once its oldest batch is this old (0 = at once): messages
  // consumed within the window never reach the disk, at the price of later confirms
  void set_group_delay(double ms) { delay_us_ = (i64)(ms * 1000.0); }
  u64 rows() const { return rows_; }
  u64 commits() const { return commits_; }
  u64 bytes() const { return bytes_; }
  double busy_s() const { return busy_s_; }
  // busy time split: applying the batches / writing the group's rows / WAL write + fsync
  double apply_s() const { return apply_s_; }
  double flush_s() const { return flush_s_; }
  double sync_s() const { return sync_s_; }
  // a group commit failed (ENOSPC / EIO on the WAL or the body log, a segment that could
  // not be created): nothing of that group or later is reported committed, so their
  // publisher confirms are never released; the broker reads this through stats / healthy
  bool failed() const { return failed_.load(); }
  std::string error() const {
    std::lock_guard<std::mutex> g(mu_);
    return err_;
  }

 private:
  struct Batch { u64 step; std::string persist, consumed; std::chrono::steady_clock::time_point t; };
  struct Row { i64 offset; i32 size; bool unack; };
  struct RowKey {
    u32 q; i64 id;
    bool operator==(const RowKey& o) const { return q == o.q && id == o.id; }
  };
  struct RowHash {
    size_t operator()(const RowKey& k) const { return HashI64()(k.id ^ ((i64)k.q << 48)); }
  };
  struct Born { PersistHdr h; bool unack; };                  // row of this group, not yet written
  struct BornMsg { const char* rec; PersistHdr h; int refs; };  // rec: the record holding the bytes
  void loop();
  void apply(const Batch& b);
  void flush_born();
  u32 gq(u32 slot);
  void op(u8 kind, u32 q, i64 offset, i64 msgid, i32 size);

  Store* st_;
  std::function<void(u64)> commit_cb_;
  mutable std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::deque<Batch> q_;
  u64 submitted_ = 0, committed_ = 0;
  bool running_ = false;
  std::thread th_;
  std::mutex qid_mu_;
  std::vector<std::string> qid_;                      // by queue slot
  std::unordered_map<std::string, u32> slot_of_;      // queue id -> slot
  FlatMap<i64, int, HashI64> refs_;                   // msg id -> durable queue rows (in the store)
  FlatMap<RowKey, Row, RowHash> rows_by_;             // (queue slot, msg id) -> stored row
  FlatMap<RowKey, Born, RowHash> born_;               // this group's rows
  FlatMap<i64, BornMsg, HashI64> born_msg_;           // this group's messages
  // the group's row changes, applied to the store as one WAL record
  std::vector<RowOp> ops_;
  std::vector<int> qlocal_;                           // queue slot -> index in gq_ (-1)
  std::vector<const std::string*> gq_;
  std::vector<u32> gslots_;
  std::vector<const char*> recs_;
  std::vector<uint32_t> lens_;
  std::vector<i64> mids_;
  std::vector<BodyLog::Loc> locs_;
  std::atomic<u64> rows_{0}, commits_{0}, bytes_{0};
  double busy_s_ = 0, apply_s_ = 0, flush_s_ = 0, sync_s_ = 0;
  std::atomic<i64> delay_us_{0};
  std::atomic<bool> failed_{false};
  std::string err_;                                   // (mu_) what failed first
};

}  // namespace cmq

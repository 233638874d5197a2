#include "persist.hpp"

#include <chrono>
#include <climits>
#include <cstring>

namespace cmq {

PersistWorker::PersistWorker(Store* store)
    : st_(store), refs_(INT64_MIN), rows_by_(RowKey{~0u, INT64_MIN}), born_(RowKey{~0u, INT64_MIN}),
      born_msg_(INT64_MIN) {}

PersistWorker::~PersistWorker() { stop(); }

void PersistWorker::start() {
  std::lock_guard<std::mutex> g(mu_);
  if (running_) return;
  running_ = true;
  th_ = std::thread([this] { loop(); });
}

void PersistWorker::stop() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!running_) return;
    running_ = false;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
}

void PersistWorker::set_queue(u32 slot, const std::string& qid) {
  std::lock_guard<std::mutex> g(qid_mu_);
  if (slot >= qid_.size()) {
    qid_.resize(slot + 1);
    qlocal_.resize(slot + 1, -1);
  }
  if (!qid_[slot].empty()) slot_of_.erase(qid_[slot]);
  if (qid.empty() || qid != qid_[slot]) {   // slot freed / reused: its old rows are gone
    std::vector<RowKey> gone;
    rows_by_.for_each([&](const RowKey& k, Row&) { if (k.q == slot) gone.push_back(k); });
    for (auto& k : gone) rows_by_.erase(k);
  }
  qid_[slot] = qid;
  if (!qid.empty()) slot_of_[qid] = slot;
}

void PersistWorker::seed_row(const std::string& qid, i64 msgid, i64 offset, i32 size, bool unack, int refs) {
  std::lock_guard<std::mutex> g(qid_mu_);
  auto it = slot_of_.find(qid);
  if (it == slot_of_.end()) return;
  rows_by_[RowKey{it->second, msgid}] = Row{offset, size, unack};
  refs_[msgid] = refs;
}

void PersistWorker::submit(u64 step, std::string persist, std::string consumed) {
  {
    std::lock_guard<std::mutex> g(mu_);
    q_.push_back(Batch{step, std::move(persist), std::move(consumed), std::chrono::steady_clock::now()});
    ++submitted_;
  }
  cv_.notify_one();
}

void PersistWorker::drain() {
  std::unique_lock<std::mutex> g(mu_);
  const u64 want = submitted_;
  done_cv_.wait(g, [&] { return committed_ >= want || !running_ || failed_.load(); });
}

void PersistWorker::loop() {
  std::unique_lock<std::mutex> g(mu_);
  while (true) {
    cv_.wait(g, [&] { return !q_.empty() || !running_; });
    if (q_.empty() && !running_) break;
    const i64 delay = delay_us_.load();
    if (delay > 0 && running_) {   // let the group gather (a deep queue goes at once)
      const auto until = q_.front().t + std::chrono::microseconds(delay);
      cv_.wait_until(g, until, [&] { return !running_ || q_.size() >= 256; });
    }
    std::deque<Batch> work;
    work.swap(q_);
    if (failed_) {   // a group already failed: later ones are never reported committed
      committed_ += work.size();
      done_cv_.notify_all();
      continue;
    }
    g.unlock();
    auto t0 = std::chrono::steady_clock::now(), t1 = t0, t2 = t0;
    u64 top = 0;
    try {
      {
        std::lock_guard<std::mutex> qg(qid_mu_);
        for (auto& b : work) {
          apply(b);
          if (b.step > top) top = b.step;
        }
        t1 = std::chrono::steady_clock::now();
        flush_born();   // rows that outlived the group (their batches are still alive here)
      }
      t2 = std::chrono::steady_clock::now();
      st_->sync();   // group commit: one fsync for every batch that was waiting (+ the body log's)
    } catch (std::exception& e) {
      // ENOSPC / EIO (sticky in the body log) or a segment that could not be created: the
      // group is not durable.  Its steps' confirms stay held (no commit callback), the
      // worker reports failed() and the broker fails over instead of std::terminate
      g.lock();
      if (!failed_) err_ = e.what();
      failed_ = true;
      committed_ += work.size();
      done_cv_.notify_all();
      continue;
    }
    ++commits_;
    auto t3 = std::chrono::steady_clock::now();
    apply_s_ += std::chrono::duration<double>(t1 - t0).count();
    flush_s_ += std::chrono::duration<double>(t2 - t1).count();
    sync_s_ += std::chrono::duration<double>(t3 - t2).count();
    busy_s_ += std::chrono::duration<double>(t3 - t0).count();
    if (top && commit_cb_) commit_cb_(top);
    g.lock();
    committed_ += work.size();
    done_cv_.notify_all();
  }
}

// the group's index of a queue slot (RowOp.q)
u32 PersistWorker::gq(u32 slot) {
  int& l = qlocal_[slot];
  if (l < 0) {
    l = (int)gq_.size();
    gq_.push_back(&qid_[slot]);
    gslots_.push_back(slot);
  }
  return (u32)l;
}

void PersistWorker::op(u8 kind, u32 q, i64 offset, i64 msgid, i32 size) {
  RowOp o{};
  o.op = kind;
  o.q = q;
  o.offset = offset;
  o.msgid = msgid;
  o.size = size;
  ops_.push_back(o);
}

void PersistWorker::apply(const Batch& b) {
  // ---- enqueues of persistent messages into durable queues: held as this group's rows.
  // A message's bytes ride only its first record of the step (the others are headers,
  // size == sizeof(PersistHdr)): find them first
  const u8* p = (const u8*)b.persist.data();
  size_t off = 0, n = b.persist.size();
  FlatMap<i64, const char*, HashI64> bytes_of(INT64_MIN, n / 4096 + 16);
  while (off + sizeof(PersistHdr) <= n) {
    PersistHdr h;
    memcpy(&h, p + off, sizeof h);
    if (h.size < sizeof(PersistHdr) || off + h.size > n) break;
    if (h.size > sizeof(PersistHdr)) bytes_of[h.msg_id] = (const char*)p + off;   // the full record
    off += h.size;
  }
  off = 0;
  while (off + sizeof(PersistHdr) <= n) {
    PersistHdr h;
    memcpy(&h, p + off, sizeof h);
    if (h.size < sizeof(PersistHdr) || off + h.size > n) break;
    const char* const* bo = bytes_of.find(h.msg_id);
    const char* rec = bo ? *bo : (const char*)p + off;
    off += h.size;
    if (h.q >= qid_.size() || qid_[h.q].empty()) continue;
    if (int* rf = refs_.find(h.msg_id)) {   // a message already in the store gains a queue row
      const int refs = ++*rf;
      const u32 lq = gq(h.q);
      op(ROW_MSG_REFER, lq, 0, h.msg_id, refs);
      op(ROW_QMSG_INS, lq, (i64)h.qpos, h.msg_id, (i32)h.body_len);
      rows_by_[RowKey{h.q, h.msg_id}] = Row{(i64)h.qpos, (i32)h.body_len, false};
      ++rows_;
      continue;
    }
    bool fresh = false;
    BornMsg& bm = born_msg_.get(h.msg_id, &fresh);
    if (fresh) bm = BornMsg{rec, h, 0};
    ++bm.refs;
    born_[RowKey{h.q, h.msg_id}] = Born{h, false};
    ++rows_;
  }
  // ---- state changes: 0 consumed/acked, 1 expired, 2 dropped, 3 delivered awaiting ack, 4 requeued
  const size_t nc = b.consumed.size() / sizeof(ConsumedRec);
  for (size_t k = 0; k < nc; ++k) {
    ConsumedRec r;
    memcpy(&r, b.consumed.data() + k * sizeof(ConsumedRec), sizeof r);
    if (r.q >= qid_.size() || qid_[r.q].empty()) continue;
    const RowKey key{r.q, r.msg_id};
    if (Born* bi = born_.find(key)) {   // the row never reached the store: update it in memory
      if (r.kind == 3) bi->unack = true;
      else if (r.kind == 4) bi->unack = false;
      else {
        born_.erase(key);
        BornMsg* bm = born_msg_.find(r.msg_id);
        if (bm && --bm->refs <= 0) born_msg_.erase(r.msg_id);
      }
      continue;
    }
    Row* row = rows_by_.find(key);
    if (!row) continue;
    const u32 lq = gq(r.q);
    if (r.kind == 3) {
      if (!row->unack) {
        op(ROW_QUNACK_INS, lq, row->offset, r.msg_id, row->size);
        op(ROW_QMSG_DEL, lq, row->offset, r.msg_id, 0);
        row->unack = true;
      }
      continue;
    }
    if (r.kind == 4) {
      if (row->unack) {
        op(ROW_QUNACK_DEL, lq, row->offset, r.msg_id, 0);
        op(ROW_QMSG_INS, lq, row->offset, r.msg_id, row->size);
        row->unack = false;
      }
      continue;
    }
    if (row->unack) op(ROW_QUNACK_DEL, lq, row->offset, r.msg_id, 0);
    else op(ROW_QMSG_DEL, lq, row->offset, r.msg_id, 0);
    rows_by_.erase(key);
    int* rf = refs_.find(r.msg_id);
    const int left = rf ? *rf - 1 : 0;
    if (left <= 0) {
      if (rf) refs_.erase(r.msg_id);
      op(ROW_MSG_DEL, lq, 0, r.msg_id, 0);
    } else {
      *rf = left;
      op(ROW_MSG_REFER, lq, 0, r.msg_id, left);
    }
  }
}

// the group's surviving messages and rows go to the store (before its one fsync)
void PersistWorker::flush_born() {
  if (!born_msg_.empty() && st_->hasBodyLog()) {   // bytes straight from the batches to the body log
    recs_.clear();
    lens_.clear();
    mids_.clear();
    born_msg_.for_each([&](const i64& id, BornMsg& bm) {
      PersistHdr full;
      memcpy(&full, bm.rec, sizeof full);   // the record holding the bytes
      recs_.push_back(bm.rec);
      lens_.push_back(full.size);
      mids_.push_back(id);
    });
    locs_.resize(recs_.size());
    st_->placeBodies(recs_.data(), lens_.data(), recs_.size(), locs_.data());
    for (size_t i = 0; i < mids_.size(); ++i) {
      const BornMsg& bm = *born_msg_.find(mids_[i]);
      RowOp o{};
      o.op = ROW_MSG_REF;
      o.q = (u32)bm.refs;
      o.msgid = mids_[i];
      o.offset = (i64)locs_[i].off;
      o.size = (i32)locs_[i].len;
      o.seg = locs_[i].seg;
      o.tstamp = bm.h.ts_ms;
      ops_.push_back(o);
      refs_[mids_[i]] = bm.refs;
      bytes_ += bm.h.body_len;
    }
  } else if (!born_msg_.empty()) {   // memory-only store: the row holds the bytes
    born_msg_.for_each([&](const i64& id, BornMsg& bm) {
      const PersistHdr& h = bm.h;
      const char* d = bm.rec + sizeof(PersistHdr);
      MsgRow m;
      m.id = id;
      m.tstamp = h.ts_ms;
      m.exchange.assign(d, h.ex_len);
      m.routing.assign(d + h.ex_len, h.rk_len);
      m.header.assign(2, '\0');   // weight u16 | body size u64 | props
      for (int i = 7; i >= 0; --i) m.header.push_back((char)((u64)h.body_len >> (8 * i)));
      m.header.append(d + h.ex_len + h.rk_len, h.props_len);
      m.body.assign(d + h.ex_len + h.rk_len + h.props_len, h.body_len);
      m.durable = true;
      m.refer = bm.refs;
      st_->insertMessage(std::move(m), 0);
      refs_[id] = bm.refs;
      bytes_ += h.body_len;
    });
  }
  born_.for_each([&](const RowKey& k, Born& b) {
    const PersistHdr& h = b.h;
    op(b.unack ? ROW_QUNACK_INS : ROW_QMSG_INS, gq(k.q), (i64)h.qpos, k.id, (i32)h.body_len);
    rows_by_[k] = Row{(i64)h.qpos, (i32)h.body_len, b.unack};
  });
  born_.clear();
  born_msg_.clear();
  st_->applyRows(gq_, ops_.data(), ops_.size());
  ops_.clear();
  for (u32 s : gslots_) qlocal_[s] = -1;
  gslots_.clear();
  gq_.clear();
}

}  // namespace cmq

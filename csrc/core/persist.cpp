#include "persist.hpp"

#include <chrono>
#include <cstring>

namespace cmq {

namespace {
std::string be64(u64 v) {
  std::string s(8, '\0');
  for (int i = 7; i >= 0; --i) { s[i] = (char)(v & 0xff); v >>= 8; }
  return s;
}
}  // namespace

PersistWorker::PersistWorker(Store* store) : st_(store) {}

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
  if (slot >= qid_.size()) qid_.resize(slot + 1);
  if (!qid_[slot].empty()) slot_of_.erase(qid_[slot]);
  if (qid.empty() || qid != qid_[slot])   // slot freed / reused: its old rows are gone
    for (auto it = rows_by_.begin(); it != rows_by_.end();)
      it = it->first.q == slot ? rows_by_.erase(it) : std::next(it);
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
    q_.push_back(Batch{step, std::move(persist), std::move(consumed)});
    ++submitted_;
  }
  cv_.notify_one();
}

void PersistWorker::drain() {
  std::unique_lock<std::mutex> g(mu_);
  const u64 want = submitted_;
  done_cv_.wait(g, [&] { return committed_ >= want || !running_; });
}

void PersistWorker::loop() {
  std::unique_lock<std::mutex> g(mu_);
  while (true) {
    cv_.wait(g, [&] { return !q_.empty() || !running_; });
    if (q_.empty() && !running_) break;
    std::deque<Batch> work;
    work.swap(q_);
    g.unlock();
    auto t0 = std::chrono::steady_clock::now();
    u64 top = 0;
    {
      std::lock_guard<std::mutex> qg(qid_mu_);
      for (auto& b : work) {
        apply(b);
        if (b.step > top) top = b.step;
      }
      flush_born();   // rows that outlived the group (their batches are still alive here)
    }
    st_->sync();   // group commit: one fsync for every batch that was waiting
    ++commits_;
    busy_s_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (top && commit_cb_) commit_cb_(top);
    g.lock();
    committed_ += work.size();
    done_cv_.notify_all();
  }
}

void PersistWorker::apply(const Batch& b) {
  // ---- enqueues of persistent messages into durable queues: held as this group's rows.
  // A message's bytes ride only its first record of the step (the others are headers,
  // size == sizeof(PersistHdr)): find them first
  const u8* p = (const u8*)b.persist.data();
  size_t off = 0, n = b.persist.size();
  std::unordered_map<i64, const char*> bytes_of;
  while (off + sizeof(PersistHdr) <= n) {
    PersistHdr h;
    memcpy(&h, p + off, sizeof h);
    if (h.size < sizeof(PersistHdr) || off + h.size > n) break;
    if (h.size > sizeof(PersistHdr)) bytes_of.emplace(h.msg_id, (const char*)p + off + sizeof(PersistHdr));
    off += h.size;
  }
  off = 0;
  while (off + sizeof(PersistHdr) <= n) {
    PersistHdr h;
    memcpy(&h, p + off, sizeof h);
    if (h.size < sizeof(PersistHdr) || off + h.size > n) break;
    auto bo = bytes_of.find(h.msg_id);
    const char* d = bo != bytes_of.end() ? bo->second : (const char*)p + off + sizeof(PersistHdr);
    off += h.size;
    if (h.q >= qid_.size() || qid_[h.q].empty()) continue;
    auto rf = refs_.find(h.msg_id);
    if (rf != refs_.end()) {   // a message already in the store gains a queue row
      st_->updateMessageReferCount(h.msg_id, ++rf->second);
      st_->insertQueueMsg(qid_[h.q], (i64)h.qpos, h.msg_id, (i32)h.body_len, 0);
      rows_by_[RowKey{h.q, h.msg_id}] = Row{(i64)h.qpos, (i32)h.body_len, false};
      ++rows_;
      continue;
    }
    auto& bm = born_msg_[h.msg_id];
    if (bm.refs == 0) { bm.d = d; bm.h = h; }
    ++bm.refs;
    born_[RowKey{h.q, h.msg_id}] = Born{d, h, false};
    ++rows_;
  }
  // ---- state changes: 0 consumed/acked, 1 expired, 2 dropped, 3 delivered awaiting ack, 4 requeued
  const size_t nc = b.consumed.size() / sizeof(ConsumedRec);
  for (size_t k = 0; k < nc; ++k) {
    ConsumedRec r;
    memcpy(&r, b.consumed.data() + k * sizeof(ConsumedRec), sizeof r);
    if (r.q >= qid_.size() || qid_[r.q].empty()) continue;
    const RowKey key{r.q, r.msg_id};
    auto bi = born_.find(key);
    if (bi != born_.end()) {   // the row never reached the store: update it in memory
      if (r.kind == 3) bi->second.unack = true;
      else if (r.kind == 4) bi->second.unack = false;
      else {
        born_.erase(bi);
        auto bm = born_msg_.find(r.msg_id);
        if (bm != born_msg_.end() && --bm->second.refs <= 0) born_msg_.erase(bm);
      }
      continue;
    }
    const std::string& qid = qid_[r.q];
    auto it = rows_by_.find(key);
    if (it == rows_by_.end()) continue;
    Row& row = it->second;
    if (r.kind == 3) {
      if (!row.unack) {
        st_->insertQueueUnack(qid, row.offset, r.msg_id, row.size);
        st_->deleteQueueMsg(qid, row.offset);
        row.unack = true;
      }
      continue;
    }
    if (r.kind == 4) {
      if (row.unack) {
        st_->deleteQueueUnack(qid, r.msg_id);
        st_->insertQueueMsg(qid, row.offset, r.msg_id, row.size, 0);
        row.unack = false;
      }
      continue;
    }
    if (row.unack) st_->deleteQueueUnack(qid, r.msg_id);
    else st_->deleteQueueMsg(qid, row.offset);
    rows_by_.erase(it);
    auto rf = refs_.find(r.msg_id);
    int left = rf == refs_.end() ? 0 : rf->second - 1;
    if (left <= 0) {
      if (rf != refs_.end()) refs_.erase(rf);
      st_->deleteMessage(r.msg_id);
    } else {
      rf->second = left;
      st_->updateMessageReferCount(r.msg_id, left);
    }
  }
}

// the group's surviving messages and rows go to the store (before its one fsync)
void PersistWorker::flush_born() {
  for (auto& kv : born_msg_) {
    const PersistHdr& h = kv.second.h;
    const char* d = kv.second.d;
    MsgRow m;
    m.id = h.msg_id;
    m.tstamp = h.ts_ms;
    m.exchange.assign(d, h.ex_len);
    m.routing.assign(d + h.ex_len, h.rk_len);
    m.header = std::string(2, '\0') + be64(h.body_len);   // weight u16 | body size u64 | props
    m.header.append(d + h.ex_len + h.rk_len, h.props_len);
    m.body.assign(d + h.ex_len + h.rk_len + h.props_len, h.body_len);
    m.durable = true;
    m.refer = kv.second.refs;
    st_->insertMessage(std::move(m), 0);
    refs_[h.msg_id] = kv.second.refs;
    bytes_ += h.body_len;
  }
  for (auto& kv : born_) {
    const PersistHdr& h = kv.second.h;
    const std::string& qid = qid_[h.q];
    if (kv.second.unack) st_->insertQueueUnack(qid, (i64)h.qpos, h.msg_id, (i32)h.body_len);
    else st_->insertQueueMsg(qid, (i64)h.qpos, h.msg_id, (i32)h.body_len, 0);
    rows_by_[kv.first] = Row{(i64)h.qpos, (i32)h.body_len, kv.second.unack};
  }
  born_.clear();
  born_msg_.clear();
}

}  // namespace cmq

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
  qid_[slot] = qid;
}

void PersistWorker::seed_row(const std::string& qid, i64 msgid, i64 offset, i32 size, bool unack, int refs) {
  std::lock_guard<std::mutex> g(qid_mu_);
  rows_by_[{qid, msgid}] = Row{offset, size, unack};
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
  // ---- enqueues of persistent messages into durable queues
  const u8* p = (const u8*)b.persist.data();
  size_t off = 0, n = b.persist.size();
  while (off + sizeof(PersistHdr) <= n) {
    PersistHdr h;
    memcpy(&h, p + off, sizeof h);
    if (h.size < sizeof(PersistHdr) || off + h.size > n) break;
    const char* d = (const char*)p + off + sizeof(PersistHdr);
    off += h.size;
    const std::string& qid = h.q < qid_.size() ? qid_[h.q] : std::string();
    if (qid.empty()) continue;
    int& refs = refs_[h.msg_id];
    if (refs == 0) {
      MsgRow m;
      m.id = h.msg_id;
      m.tstamp = h.ts_ms;
      m.exchange.assign(d, h.ex_len);
      m.routing.assign(d + h.ex_len, h.rk_len);
      m.header = std::string(2, '\0') + be64(h.body_len);   // weight u16 | body size u64 | props
      m.header.append(d + h.ex_len + h.rk_len, h.props_len);
      m.body.assign(d + h.ex_len + h.rk_len + h.props_len, h.body_len);
      m.durable = true;
      m.refer = 1;
      st_->insertMessage(std::move(m), 0);
      bytes_ += h.body_len;
    } else {
      st_->updateMessageReferCount(h.msg_id, refs + 1);
    }
    ++refs;
    st_->insertQueueMsg(qid, (i64)h.qpos, h.msg_id, (i32)h.body_len, 0);
    rows_by_[{qid, h.msg_id}] = Row{(i64)h.qpos, (i32)h.body_len, false};
    ++rows_;
  }
  // ---- state changes: 0 consumed/acked, 1 expired, 2 dropped, 3 delivered awaiting ack, 4 requeued
  const size_t nc = b.consumed.size() / sizeof(ConsumedRec);
  for (size_t k = 0; k < nc; ++k) {
    ConsumedRec r;
    memcpy(&r, b.consumed.data() + k * sizeof(ConsumedRec), sizeof r);
    const std::string& qid = r.q < qid_.size() ? qid_[r.q] : std::string();
    if (qid.empty()) continue;
    auto it = rows_by_.find({qid, r.msg_id});
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

}  // namespace cmq

// Embedded Cassandra-schema store with a CRC-checked write-ahead log (see store.hpp).
#include "store.hpp"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <climits>
#include <libgen.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <stdexcept>

#include <nmmintrin.h>

#include "codec.hpp"
#include "../kernels/step_abi.h"

namespace cmq {

namespace {
enum Op : uint8_t {
  OP_MSG_INS = 1, OP_MSG_REFER, OP_MSG_DEL, OP_QMETA_INS, OP_QMSG_INS, OP_QLAST, OP_QCONSUMED, OP_QFORCE_DEL,
  OP_QPENDING_DEL, OP_QDEL_CONSUMED, OP_QUNACK_INS, OP_QUNACK_DEL, OP_X_INS, OP_BIND_INS, OP_BIND_DEL,
  OP_BIND_DEL_Q, OP_X_DEL, OP_VH_INS, OP_VH_DEL, OP_QMSG_DEL, OP_QDMETA_INS, OP_QDMSG_INS, OP_QDUNACK_INS,
  OP_MSG_REF,  // a msgs row whose bytes are in the body log (bodylog.hpp)
  OP_ROWS      // a group of RowOps (little-endian: u32 nq | nq x (u32 len | id) | u32 n | n x RowOp)
};

// CRC-32C (Castagnoli, init/xorout 0xFFFFFFFF) on the SSE4.2 crc32 instruction: the
// record check is on the persistence hot path (every 4 KB message body of BASELINE
// config 4), where zlib's table-driven CRC-32 ran at < 1 GB/s
__attribute__((target("sse4.2"))) uint32_t crc32(const char* p, size_t n) {
  uint64_t c = 0xFFFFFFFFu;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, (uint8_t)*p++);
  return c32 ^ 0xFFFFFFFFu;
}
uint32_t crc32(const std::string& s) { return crc32(s.data(), s.size()); }

// round-1 WALs (no header): records checked with CRC-32 (reflected 0xEDB88320); replayed
// once and rewritten in the current format
uint32_t crc32_legacy(const std::string& s) {
  static uint32_t tab[256];
  static bool init = false;
  if (!init) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      tab[i] = c;
    }
    init = true;
  }
  uint32_t c = 0xFFFFFFFFu;
  for (unsigned char ch : s) c = tab[(c ^ ch) & 0xff] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

// a WAL starts with this header (format 2: CRC-32C records)
const char WAL_MAGIC[8] = {'C', 'M', 'Q', 'W', 'A', 'L', '2', '\n'};

void w_map(Writer& w, const std::map<std::string, std::string>& m) {
  w.lng((u32)m.size());
  for (auto& kv : m) { w.longstr(kv.first); w.longstr(kv.second); }
}
std::map<std::string, std::string> r_map(Reader& r) {
  std::map<std::string, std::string> m;
  u32 n = r.lng();
  for (u32 i = 0; i < n; ++i) { std::string k = r.longstr(); m[k] = r.longstr(); }
  return m;
}

// one framed WAL record: u32 len | op | payload | CRC-32C(op | payload)
void add_rec(std::string& buf, uint8_t op, const std::string& payload) {
  const u32 len = (u32)payload.size() + 1;
  const size_t at = buf.size();
  buf.resize(at + 4 + len + 4);
  char* r = &buf[at];
  for (int i = 0; i < 4; ++i) r[i] = (char)(len >> (24 - 8 * i));
  r[4] = (char)op;
  memcpy(r + 5, payload.data(), payload.size());
  const u32 c = crc32(r + 4, len);
  for (int i = 0; i < 4; ++i) r[4 + len + i] = (char)(c >> (24 - 8 * i));
}

// record payloads (the encoders of the operations; compaction re-emits rows with them)
std::string enc_msg(const MsgRow& m, int64_t ttl_ms, int64_t now) {
  Writer w;
  w.b.reserve(64 + m.header.size() + m.body.size() + m.exchange.size() + m.routing.size());
  w.llng((u64)m.id); w.llng((u64)m.tstamp); w.longstr(m.header); w.longstr(m.body); w.longstr(m.exchange);
  w.longstr(m.routing); w.octet(m.durable); w.lng((u32)m.refer);
  // Cassandra TTL is whole seconds (CassandraOpService.scala:157-159); keep ms precision internally
  w.llng((u64)ttl_ms); w.llng((u64)now);
  return std::move(w.done());
}
std::string enc_ref(const MsgRow& m, int64_t ttl_ms, int64_t now) {
  Writer w;
  w.llng((u64)m.id); w.llng((u64)m.tstamp); w.octet(m.durable); w.lng((u32)m.refer);
  w.llng((u64)ttl_ms); w.llng((u64)now);
  w.lng((u32)m.bseg); w.llng(m.boff); w.lng(m.blen);
  return std::move(w.done());
}
// the row's columns from its body-log record (a device persist record)
bool dec_body(const std::string& rec, MsgRow* m) {
  if (rec.size() < sizeof(PersistHdr)) return false;
  PersistHdr h;
  memcpy(&h, rec.data(), sizeof h);
  const size_t need = sizeof h + h.ex_len + h.rk_len + h.props_len + (size_t)h.body_len;
  if (need > rec.size()) return false;
  const char* d = rec.data() + sizeof h;
  m->exchange.assign(d, h.ex_len);
  m->routing.assign(d + h.ex_len, h.rk_len);
  m->header.assign(2, '\0');   // weight u16 | body size u64 | props (persist.cpp)
  for (int i = 7; i >= 0; --i) m->header.push_back((char)((u64)h.body_len >> (8 * i)));
  m->header.append(d + h.ex_len + h.rk_len, h.props_len);
  m->body.assign(d + h.ex_len + h.rk_len + h.props_len, h.body_len);
  return true;
}
std::string enc_qmeta(const std::string& q, int64_t lconsumed, const std::set<std::string>& consumers, bool durable,
                      int64_t ttl) {
  Writer w;
  w.longstr(q); w.llng((u64)lconsumed); w.lng((u32)consumers.size());
  for (auto& c : consumers) w.longstr(c);
  w.octet(durable); w.llng((u64)ttl);
  return std::move(w.done());
}
std::string enc_qmsg(const std::string& q, int64_t offset, int64_t msgid, int32_t size, int64_t ttl_ms, int64_t now) {
  Writer w;
  w.longstr(q); w.llng((u64)offset); w.llng((u64)msgid); w.lng((u32)size); w.llng((u64)ttl_ms); w.llng((u64)now);
  return std::move(w.done());
}
std::string enc_qrow(const std::string& q, int64_t offset, int64_t msgid, int32_t size) {
  Writer w;
  w.longstr(q); w.llng((u64)offset); w.llng((u64)msgid); w.lng((u32)size);
  return std::move(w.done());
}
std::string enc_x(const std::string& id, const ExchangeRow& x) {
  Writer w;
  w.longstr(id); w.longstr(x.tpe); w.octet(x.durable); w.octet(x.autodel); w.octet(x.internal); w_map(w, x.args);
  return std::move(w.done());
}
std::string enc_bind(const std::string& id, const std::string& queue, const std::string& key,
                     const std::map<std::string, std::string>& args) {
  Writer w;
  w.longstr(id); w.longstr(queue); w.longstr(key); w_map(w, args);
  return std::move(w.done());
}
std::string enc_vh(const std::string& id, bool active) {
  Writer w;
  w.longstr(id); w.octet(active);
  return std::move(w.done());
}
std::string enc_qdmeta(const std::string& q, const QueueMetaDeletedRow& d) {
  Writer w;
  w.longstr(q); w.llng((u64)d.lconsumed); w.lng((u32)d.nconsumer); w.octet(d.durable);
  return std::move(w.done());
}
uint64_t msg_size(const MsgRow& m) { return 64 + m.header.size() + m.body.size() + m.exchange.size() + m.routing.size(); }
int64_t ttl_left(int64_t expire_at, int64_t now) { return expire_at ? std::max<int64_t>(1, expire_at - now) : 0; }

void write_fd(int fd, const char* p, size_t n) {
  while (n) {
    ssize_t k = ::write(fd, p, n);
    if (k < 0) { if (errno == EINTR) continue; throw std::runtime_error("store: WAL write failed"); }
    p += k;
    n -= (size_t)k;
  }
}
// bytes [from, to) of the WAL file `src` appended to `dst`
void copy_range(int src, int dst, uint64_t from, uint64_t to) {
  std::string buf(1 << 20, '\0');
  while (from < to) {
    size_t want = (size_t)std::min<uint64_t>(buf.size(), to - from);
    ssize_t k = ::pread(src, &buf[0], want, (off_t)from);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) throw std::runtime_error("store: WAL read failed during compaction");
    write_fd(dst, buf.data(), (size_t)k);
    from += (uint64_t)k;
  }
}
double mono_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

Store::~Store() { close(); }

void Store::wait_compaction() {
  if (compact_th_.joinable() && compact_th_.get_id() != std::this_thread::get_id()) compact_th_.join();
}

int64_t Store::now_ms() const {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::system_clock::now().time_since_epoch()).count();
}

void Store::open(const std::string& dir, bool fsync_enabled) {
  std::lock_guard<std::recursive_mutex> g(mu_);
  fsync_ = fsync_enabled;
  if (dir.empty()) return;
  ::mkdir(dir.c_str(), 0755);
  path_ = dir + "/chanamq.wal";
  fd_ = ::open(path_.c_str(), O_RDWR | O_CREAT | O_APPEND, 0644);
  if (fd_ < 0) throw std::runtime_error("store: cannot open " + path_);
  body_.reset(new BodyLog(dir + "/bodies", fsync_enabled));
  if (quota_) body_->set_quota(&quota_used_, quota_);
  replay();
  body_->open_existing();
}

void Store::close() {
  compact_stop_ = true;
  wait_compaction();
  compact_stop_ = false;
  std::lock_guard<std::recursive_mutex> g(mu_);
  if (fd_ >= 0) {
    // the fds close even when the last sync fails (a sticky body-log error): close() runs
    // from the destructor too, where an exception would terminate the process
    try {
      sync();
    } catch (std::exception& e) {
      close_error_ = e.what();
    }
    ::close(fd_);
    fd_ = -1;
  }
  if (body_) body_->close();
}

void Store::set_quota(uint64_t bytes) {
  std::lock_guard<std::recursive_mutex> g(mu_);
  quota_ = bytes;
  quota_used_ = wal_bytes_;
  if (body_) body_->set_quota(&quota_used_, bytes);
}

void Store::write_all(const std::string& rec) {
  if (quota_ && quota_used_.fetch_add(rec.size()) + rec.size() > quota_)
    throw std::runtime_error("store: WAL write failed: No space left on device (store quota of " +
                             std::to_string(quota_) + " bytes)");
  write_fd(fd_, rec.data(), rec.size());
  wal_bytes_ += rec.size();
}

// WAL records are buffered in memory and written in large chunks: by sync() (the group
// commit, before confirms leave) or when the buffer passes 16 MB
void Store::append(uint8_t op, const std::string& payload) {
  apply(op, payload);
  append_wal(op, payload);
}

void Store::append_wal(uint8_t op, const std::string& payload) {
  if (fd_ < 0 || replaying_) return;
  add_rec(wbuf_, op, payload);
  dirty_ = true;
  if (wbuf_.size() > (16u << 20)) flush_wal();
}

void Store::flush_wal() {
  if (fd_ >= 0 && !wbuf_.empty()) write_all(wbuf_);
  wbuf_.clear();
}

void Store::sync() {
  std::lock_guard<std::recursive_mutex> g(mu_);
  flush_wal();
  if (fd_ >= 0 && dirty_) {
    if (fsync_) ::fdatasync(fd_);
    dirty_ = false;
  }
  if (body_) {   // the group's bodies (written by the stripes meanwhile) are durable too
    std::string err;
    if (!body_->wait(&err)) throw std::runtime_error("store: " + err);
    body_->reap();   // segments whose last row went in a record now on disk
  }
  maybe_compact();
}

uint64_t Store::liveEstimate() {
  std::lock_guard<std::recursive_mutex> g(mu_);
  uint64_t rows = 0;
  for (auto& kv : queues_) rows += kv.second.size();
  for (auto& kv : queue_unacks_) rows += kv.second.size();
  for (auto& kv : binds_) rows += kv.second.size();
  return msg_bytes_ + 96 * rows + 256 * (queue_metas_.size() + exchanges_.size() + vhosts_.size());
}

CompactStats Store::compactStats() {
  std::lock_guard<std::recursive_mutex> g(mu_);
  return cstats_;
}

void Store::maybe_compact() {
  if (auto_ratio_ <= 0 || fd_ < 0 || compacting_ || compact_stop_ || wal_bytes_ < auto_min_) return;
  if (wal_bytes_ < auto_backoff_) return;
  if ((double)wal_bytes_ < auto_ratio_ * (double)liveEstimate()) return;
  if (compact_th_.joinable()) compact_th_.join();   // the previous run has finished
  compacting_ = true;
  // A background run must never let an exception escape the thread (std::terminate
  // would take the broker down with unsynced state).  A failed run (typically ENOSPC
  // while writing the second copy) is recorded and auto-compaction backs off until the
  // WAL has grown by half again; the live WAL is untouched by a failed run.
  compact_th_ = std::thread([this] {
    try {
      compact_run();
    } catch (std::exception& e) {
      std::lock_guard<std::recursive_mutex> g(mu_);
      cstats_.failures++;
      cstats_.last_error = e.what();
      auto_backoff_ = wal_bytes_ + wal_bytes_ / 2;
      std::fprintf(stderr, "chanamq store: background compaction failed (%s); retry after %llu WAL bytes\n",
                   e.what(), (unsigned long long)auto_backoff_);
    }
  });
}

void Store::replay() {
  replaying_ = true;
  std::string data;
  ::lseek(fd_, 0, SEEK_SET);
  char buf[1 << 16];
  ssize_t k;
  while ((k = ::read(fd_, buf, sizeof buf)) > 0) data.append(buf, (size_t)k);
  const bool v2 = data.size() >= sizeof WAL_MAGIC && memcmp(data.data(), WAL_MAGIC, sizeof WAL_MAGIC) == 0;
  const bool legacy = !v2 && !data.empty();
  if (data.empty()) {   // a new WAL: the format header first
    std::string h(WAL_MAGIC, sizeof WAL_MAGIC);
    write_all(h);
  }
  size_t pos = v2 ? sizeof WAL_MAGIC : 0, good = data.empty() ? sizeof WAL_MAGIC : pos;
  while (pos + 9 <= data.size()) {
    const u8* p = (const u8*)data.data() + pos;
    u32 len = (u32(p[0]) << 24) | (u32(p[1]) << 16) | (u32(p[2]) << 8) | p[3];
    if (len == 0 || pos + 4 + len + 4 > data.size()) break;
    std::string body = data.substr(pos + 4, len);
    const u8* q = p + 4 + len;
    u32 crc = (u32(q[0]) << 24) | (u32(q[1]) << 16) | (u32(q[2]) << 8) | q[3];
    if (crc != (legacy ? crc32_legacy(body) : crc32(body))) break;  // torn tail: stop at the last good record
    apply((uint8_t)body[0], body.substr(1));
    pos += 8 + len;
    good = pos;
  }
  if (!data.empty() && good < data.size() && ::ftruncate(fd_, (off_t)good) != 0)
    throw std::runtime_error("store: cannot truncate the torn WAL tail");
  wal_bytes_ = good;
  ::lseek(fd_, 0, SEEK_END);
  replaying_ = false;
  if (legacy) compact();   // rewrite a round-1 WAL in the current format
}

void Store::compact() {
  wait_compaction();
  {
    std::lock_guard<std::recursive_mutex> g(mu_);
    if (fd_ < 0) return;
    compacting_ = true;
  }
  compact_run();
}

// live rows of table `t` after the continuation point (key, sub) as WAL records; false
// when the table is done.  Chunks bound the time mu_ is held.
bool Store::snapshot_chunk(int t, std::string& key, int64_t& sub, std::string& out) {
  const int64_t now = now_ms();
  const size_t budget = 8u << 20;
  const size_t start = out.size();
  switch (t) {
    case 0: for (auto& kv : vhosts_) add_rec(out, OP_VH_INS, enc_vh(kv.first, kv.second)); return false;
    case 1: for (auto& kv : exchanges_) add_rec(out, OP_X_INS, enc_x(kv.first, kv.second)); return false;
    case 2:
      for (auto& kv : binds_)
        for (auto& b : kv.second) add_rec(out, OP_BIND_INS, enc_bind(kv.first, b.second.queue, b.second.key, b.second.args));
      return false;
    case 3:
      for (auto& kv : queue_metas_)
        add_rec(out, OP_QMETA_INS, enc_qmeta(kv.first, kv.second.lconsumed, kv.second.consumers, kv.second.durable,
                                             kv.second.ttl));
      return false;
    case 4:
    case 5: {   // queue rows (by offset) / unacks (by msg id), continued at (queue, last key)
      auto& tab = t == 4 ? queues_ : queue_unacks_;
      for (auto qi = tab.lower_bound(key); qi != tab.end(); ++qi) {
        if (qi->first != key) sub = LLONG_MIN;
        key = qi->first;
        for (auto it = qi->second.upper_bound(sub); it != qi->second.end(); ++it) {
          const QueueMsgRow& r = it->second;
          if (t == 4) {
            if (!r.expire_at || r.expire_at > now)
              add_rec(out, OP_QMSG_INS, enc_qmsg(key, r.offset, r.msgid, r.size, ttl_left(r.expire_at, now), now));
          } else {
            add_rec(out, OP_QUNACK_INS, enc_qrow(key, r.offset, r.msgid, r.size));
          }
          sub = it->first;
          if (out.size() - start > budget) return true;
        }
      }
      return false;
    }
    case 6: {   // messages, continued at the last id
      for (auto it = msgs_.upper_bound(sub); it != msgs_.end(); ++it) {
        if (!it->second.expire_at || it->second.expire_at > now)
          add_rec(out, it->second.bseg >= 0 ? OP_MSG_REF : OP_MSG_INS,
                  it->second.bseg >= 0 ? enc_ref(it->second, ttl_left(it->second.expire_at, now), now)
                                       : enc_msg(it->second, ttl_left(it->second.expire_at, now), now));
        sub = it->first;
        if (out.size() - start > budget) return true;
      }
      return false;
    }
    case 7:
      for (auto& kv : queue_metas_deleted_) add_rec(out, OP_QDMETA_INS, enc_qdmeta(kv.first, kv.second));
      for (auto& kv : queues_deleted_)
        for (auto& r : kv.second) add_rec(out, OP_QDMSG_INS, enc_qrow(kv.first, r.second.offset, r.second.msgid, r.second.size));
      for (auto& kv : queue_unacks_deleted_)
        for (auto& r : kv.second)
          add_rec(out, OP_QDUNACK_INS, enc_qrow(kv.first, r.second.offset, r.second.msgid, r.second.size));
      return false;
    default: return false;
  }
}

void Store::compact_run() {
  const double t0 = mono_s();
  double max_lock = 0;
  std::string tmp;
  int nfd = -1;
  uint64_t switch_off = 0, before = 0;
  try {
    {
      std::lock_guard<std::recursive_mutex> g(mu_);
      if (fd_ < 0) { compacting_ = false; return; }
      flush_wal();
      switch_off = before = wal_bytes_;
      tmp = path_ + ".compact";
      nfd = ::open(tmp.c_str(), O_RDWR | O_CREAT | O_TRUNC | O_APPEND, 0644);
      if (nfd < 0) throw std::runtime_error("store: compact open failed");
    }
    // ---- snapshot of the live rows (short locked chunks; appends continue meanwhile)
    std::string out(WAL_MAGIC, sizeof WAL_MAGIC);
    uint64_t written = 0;
    for (int t = 0; t <= 7; ++t) {
      std::string key;
      int64_t sub = LLONG_MIN;
      bool more = true;
      while (more) {
        {
          std::lock_guard<std::recursive_mutex> g(mu_);
          const double l0 = mono_s();
          more = snapshot_chunk(t, key, sub, out);
          max_lock = std::max(max_lock, mono_s() - l0);
        }
        if (out.size() > (4u << 20)) { write_fd(nfd, out.data(), out.size()); written += out.size(); out.clear(); }
        if (compact_stop_) throw std::runtime_error("store closing");
      }
    }
    write_fd(nfd, out.data(), out.size());
    written += out.size();
    out.clear();
    // ---- the old WAL's records since the switch point, then swap files under the lock
    uint64_t copied = switch_off;
    while (true) {
      uint64_t cur;
      int oldfd;
      {
        std::lock_guard<std::recursive_mutex> g(mu_);
        const double l0 = mono_s();
        flush_wal();
        cur = wal_bytes_;
        oldfd = fd_;
        if (cur - copied <= (4u << 20) || compact_stop_) {
          copy_range(fd_, nfd, copied, cur);
          if (fsync_) ::fdatasync(nfd);
          if (::rename(tmp.c_str(), path_.c_str()) != 0) throw std::runtime_error("store: compact rename failed");
          if (fsync_) {   // the rename itself is durable
            std::string dir = path_;
            int dfd = ::open(dirname(&dir[0]), O_RDONLY | O_DIRECTORY);
            if (dfd >= 0) { ::fsync(dfd); ::close(dfd); }
          }
          ::close(fd_);
          fd_ = nfd;
          nfd = -1;
          wal_bytes_ = written + (cur - switch_off);
          dirty_ = false;
          cstats_.runs++;
          cstats_.last_before = before + (cur - switch_off);
          cstats_.last_after = wal_bytes_;
          cstats_.tail_bytes = cur - switch_off;
          max_lock = std::max(max_lock, mono_s() - l0);
          cstats_.max_lock_s = std::max(cstats_.max_lock_s, max_lock);
          cstats_.last_s = mono_s() - t0;
          auto_backoff_ = 0;
          compacting_ = false;
          return;
        }
      }
      copy_range(oldfd, nfd, copied, cur);   // bytes already in the file: no lock needed
      copied = cur;
    }
  } catch (std::exception&) {
    if (nfd >= 0) { ::close(nfd); ::unlink(tmp.c_str()); }
    compacting_ = false;
    if (!compact_stop_) throw;
  }
}

// ------------------------------------------------------------------ apply (row semantics)
void Store::apply(uint8_t op, const std::string& pl) {
  Reader r((const u8*)pl.data(), pl.size());
  int64_t now = now_ms();
  switch (op) {
    case OP_MSG_INS: {
      MsgRow m;
      m.id = (int64_t)r.llng(); m.tstamp = (int64_t)r.llng(); m.header = r.longstr(); m.body = r.longstr();
      m.exchange = r.longstr(); m.routing = r.longstr(); m.durable = r.octet(); m.refer = (int32_t)r.lng();
      int64_t ttl = (int64_t)r.llng();
      int64_t at = (int64_t)r.llng();
      m.expire_at = ttl > 0 ? at + ttl : 0;
      put_msg(std::move(m));
      break;
    }
    case OP_MSG_REF: {
      MsgRow m;
      m.id = (int64_t)r.llng(); m.tstamp = (int64_t)r.llng(); m.durable = r.octet(); m.refer = (int32_t)r.lng();
      int64_t ttl = (int64_t)r.llng();
      int64_t at = (int64_t)r.llng();
      m.expire_at = ttl > 0 ? at + ttl : 0;
      m.bseg = (int64_t)r.lng(); m.boff = r.llng(); m.blen = r.lng();
      if (!body_) break;   // a memory-only store never wrote one
      put_msg(std::move(m));
      break;
    }
    case OP_MSG_REFER: { int64_t id = (int64_t)r.llng(); int32_t ref = (int32_t)r.lng();
      auto it = msgs_.find(id); if (it != msgs_.end()) it->second.refer = ref;
      if (marking()) md_msgs_.insert(id);
      break; }
    case OP_MSG_DEL: {
      auto it = msgs_.find((int64_t)r.llng());
      if (it != msgs_.end()) drop_msg(it);
      break;
    }
    case OP_QMETA_INS: {
      std::string q = r.longstr();
      QueueMetaRow m;
      m.lconsumed = (int64_t)r.llng();
      u32 n = r.lng();
      for (u32 i = 0; i < n; ++i) m.consumers.insert(r.longstr());
      m.durable = r.octet(); m.ttl = (int64_t)r.llng();
      queue_metas_[q] = m;
      if (marking()) md_qmetas_.insert(q);
      break;
    }
    case OP_QMSG_INS: {
      std::string q = r.longstr();
      QueueMsgRow m;
      m.offset = (int64_t)r.llng(); m.msgid = (int64_t)r.llng(); m.size = (int32_t)r.lng();
      int64_t ttl = (int64_t)r.llng(), at = (int64_t)r.llng();
      m.expire_at = ttl > 0 ? at + ttl : 0;
      queues_[q][m.offset] = m;
      if (marking()) md_qmsgs_.emplace(q, m.offset);
      break;
    }
    case OP_QMSG_DEL: {
      std::string q = r.longstr();
      const int64_t off = (int64_t)r.llng();
      queues_[q].erase(off);
      if (marking()) md_qmsgs_.emplace(q, off);
      break;
    }
    case OP_QLAST: {
      std::string q = r.longstr();
      queue_metas_[q].lconsumed = (int64_t)r.llng();
      if (marking()) md_qmetas_.insert(q);
      break;
    }
    case OP_QCONSUMED: {
      // lconsumed := L; rows with offset <= L removed; unacks inserted (correct columns: A.Q21)
      std::string q = r.longstr();
      int64_t L = (int64_t)r.llng();
      queue_metas_[q].lconsumed = L;
      auto& rows = queues_[q];
      rows.erase(rows.begin(), rows.upper_bound(L));
      u32 n = r.lng();
      for (u32 i = 0; i < n; ++i) {
        QueueMsgRow u;
        u.offset = (int64_t)r.llng(); u.msgid = (int64_t)r.llng(); u.size = (int32_t)r.lng();
        queue_unacks_[q][u.msgid] = u;
      }
      if (marking()) { md_qmetas_.insert(q); md_qparts_.insert(q); }
      break;
    }
    case OP_QFORCE_DEL: {
      std::string q = r.longstr();
      queues_.erase(q); queue_metas_.erase(q); queue_unacks_.erase(q);
      if (marking()) { md_qmetas_.insert(q); md_qparts_.insert(q); }
      break;
    }
    case OP_QPENDING_DEL: {  // copy to *_deleted tables, then delete (CassandraOpService.scala:561-604)
      std::string q = r.longstr();
      auto mi = queue_metas_.find(q);
      if (mi != queue_metas_.end()) {
        QueueMetaDeletedRow d;
        d.lconsumed = mi->second.lconsumed; d.nconsumer = (int32_t)mi->second.consumers.size();
        d.durable = mi->second.durable;
        queue_metas_deleted_[q] = d;
      }
      for (auto& kv : queues_[q]) queues_deleted_[q][kv.first] = kv.second;
      for (auto& kv : queue_unacks_[q]) queue_unacks_deleted_[q][kv.first] = kv.second;
      queues_.erase(q); queue_metas_.erase(q); queue_unacks_.erase(q);
      if (marking()) { md_qmetas_.insert(q); md_qparts_.insert(q); md_deleted_.insert(q); }
      break;
    }
    case OP_QDEL_CONSUMED: {
      std::string q = r.longstr();
      int64_t L = (int64_t)r.llng();
      auto& rows = queues_[q];
      rows.erase(rows.begin(), rows.upper_bound(L));
      if (marking()) md_qparts_.insert(q);
      break;
    }
    case OP_QUNACK_INS: {
      std::string q = r.longstr();
      QueueMsgRow u;
      u.offset = (int64_t)r.llng(); u.msgid = (int64_t)r.llng(); u.size = (int32_t)r.lng();
      queue_unacks_[q][u.msgid] = u;
      if (marking()) md_qunacks_.emplace(q, u.msgid);
      break;
    }
    case OP_QUNACK_DEL: {
      std::string q = r.longstr();
      const int64_t mid = (int64_t)r.llng();
      queue_unacks_[q].erase(mid);
      if (marking()) md_qunacks_.emplace(q, mid);
      break;
    }
    case OP_X_INS: {
      std::string id = r.longstr();
      ExchangeRow x;
      x.tpe = r.longstr(); x.durable = r.octet(); x.autodel = r.octet(); x.internal = r.octet();
      x.args = r_map(r);
      exchanges_[id] = x;
      if (marking()) md_xs_.insert(id);
      break;
    }
    case OP_BIND_INS: {
      std::string id = r.longstr();
      BindRow b;
      b.queue = r.longstr(); b.key = r.longstr(); b.args = r_map(r);
      binds_[id][{b.queue, b.key}] = b;
      if (marking()) md_xs_.insert(id);
      break;
    }
    case OP_BIND_DEL: {
      std::string id = r.longstr(), q = r.longstr(), k = r.longstr();
      binds_[id].erase({q, k});
      if (marking()) md_xs_.insert(id);
      break;
    }
    case OP_BIND_DEL_Q: {
      std::string q = r.longstr();
      for (auto& kv : binds_)
        for (auto it = kv.second.begin(); it != kv.second.end();) {
          if (it->first.first == q) {
            if (marking()) md_xs_.insert(kv.first);
            it = kv.second.erase(it);
          } else {
            ++it;
          }
        }
      break;
    }
    case OP_X_DEL: {
      std::string id = r.longstr();
      exchanges_.erase(id); binds_.erase(id);
      if (marking()) md_xs_.insert(id);
      break;
    }
    case OP_QDMETA_INS: {
      std::string q = r.longstr();
      QueueMetaDeletedRow d;
      d.lconsumed = (int64_t)r.llng(); d.nconsumer = (int32_t)r.lng(); d.durable = r.octet();
      queue_metas_deleted_[q] = d;
      if (marking()) md_deleted_.insert(q);
      break;
    }
    case OP_QDMSG_INS:
    case OP_QDUNACK_INS: {
      std::string q = r.longstr();
      QueueMsgRow u;
      u.offset = (int64_t)r.llng(); u.msgid = (int64_t)r.llng(); u.size = (int32_t)r.lng();
      if (op == OP_QDMSG_INS) queues_deleted_[q][u.offset] = u;
      else queue_unacks_deleted_[q][u.msgid] = u;
      if (marking()) md_deleted_.insert(q);
      break;
    }
    case OP_ROWS: {
      const char* d = pl.data();
      const size_t n = pl.size();
      size_t at = 0;
      auto u32at = [&](uint32_t* v) { if (at + 4 > n) return false; memcpy(v, d + at, 4); at += 4; return true; };
      uint32_t nq = 0, nops = 0;
      if (!u32at(&nq)) break;
      std::vector<std::string> names(nq);
      std::vector<const std::string*> qids(nq);
      for (uint32_t i = 0; i < nq; ++i) {
        uint32_t len = 0;
        if (!u32at(&len) || at + len > n) return;
        names[i].assign(d + at, len);
        qids[i] = &names[i];
        at += len;
      }
      if (!u32at(&nops) || at + (size_t)nops * sizeof(RowOp) > n) break;
      std::vector<RowOp> ops(nops);
      memcpy(ops.data(), d + at, (size_t)nops * sizeof(RowOp));
      apply_rows(qids, ops.data(), nops);
      break;
    }
    case OP_VH_INS: {
      std::string id = r.longstr();
      vhosts_[id] = r.octet();
      if (marking()) md_vhosts_.insert(id);
      break;
    }
    case OP_VH_DEL: {
      std::string id = r.longstr();
      vhosts_.erase(id);
      if (marking()) md_vhosts_.insert(id);
      break;
    }
    default: break;
  }
  (void)now;
}

// ------------------------------------------------------------------ operations
#define LOCK std::lock_guard<std::recursive_mutex> g(mu_)

void Store::insertMessage(const MsgRow& m, int64_t ttl_ms) {
  LOCK;
  append(OP_MSG_INS, enc_msg(m, ttl_ms, now_ms()));
}
// hot path of the GPU write-behind (persist.cpp): the row moves into the table instead of
// being re-decoded from its WAL record
void Store::insertMessage(MsgRow&& m, int64_t ttl_ms) {
  LOCK;
  const int64_t now = now_ms();
  append_wal(OP_MSG_INS, enc_msg(m, ttl_ms, now));
  m.expire_at = ttl_ms > 0 ? now + ttl_ms : 0;
  m.bseg = -1;
  put_msg(std::move(m));
}

void Store::put_msg(MsgRow&& m) {
  auto it = msgs_.find(m.id);
  if (it != msgs_.end()) drop_msg(it);
  msg_bytes_ += msg_size(m);
  if (m.bseg >= 0 && body_) body_->ref(BodyLog::Loc{(uint32_t)m.bseg, m.blen, m.boff});
  const int64_t id = m.id;
  msgs_.emplace(id, std::move(m));
  if (marking()) md_msgs_.insert(id);
}

void Store::drop_msg(std::map<int64_t, MsgRow>::iterator it) {
  msg_bytes_ -= msg_size(it->second);
  if (it->second.bseg >= 0 && body_) body_->unref(BodyLog::Loc{(uint32_t)it->second.bseg, it->second.blen, it->second.boff});
  if (marking()) md_msgs_.insert(it->first);
  msgs_.erase(it);
}

void Store::apply_rows(const std::vector<const std::string*>& qids, const RowOp* ops, size_t n) {
  std::vector<std::map<int64_t, QueueMsgRow>*> qm(qids.size(), nullptr), qu(qids.size(), nullptr);
  auto rows = [&](uint32_t q) -> std::map<int64_t, QueueMsgRow>& {
    if (!qm[q]) qm[q] = &queues_[*qids[q]];
    return *qm[q];
  };
  auto unacks = [&](uint32_t q) -> std::map<int64_t, QueueMsgRow>& {
    if (!qu[q]) qu[q] = &queue_unacks_[*qids[q]];
    return *qu[q];
  };
  for (size_t i = 0; i < n; ++i) {
    const RowOp& o = ops[i];
    const bool qok = o.q < qids.size();
    switch (o.op) {
      case ROW_QMSG_INS:
        if (qok) {
          auto& t = rows(o.q);
          t.insert_or_assign(t.end(), o.offset, QueueMsgRow{o.offset, o.msgid, o.size, 0});
          if (marking()) md_qmsgs_.emplace(*qids[o.q], o.offset);
        }
        break;
      case ROW_QMSG_DEL:
        if (qok) {
          rows(o.q).erase(o.offset);
          if (marking()) md_qmsgs_.emplace(*qids[o.q], o.offset);
        }
        break;
      case ROW_QUNACK_INS:
        if (qok) {
          unacks(o.q)[o.msgid] = QueueMsgRow{o.offset, o.msgid, o.size, 0};
          if (marking()) md_qunacks_.emplace(*qids[o.q], o.msgid);
        }
        break;
      case ROW_QUNACK_DEL:
        if (qok) {
          unacks(o.q).erase(o.msgid);
          if (marking()) md_qunacks_.emplace(*qids[o.q], o.msgid);
        }
        break;
      case ROW_MSG_DEL: {
        auto it = msgs_.find(o.msgid);
        if (it != msgs_.end()) drop_msg(it);
        break;
      }
      case ROW_MSG_REFER: {
        auto it = msgs_.find(o.msgid);
        if (it != msgs_.end()) it->second.refer = o.size;
        if (marking()) md_msgs_.insert(o.msgid);
        break;
      }
      case ROW_MSG_REF: {
        if (!body_) break;
        MsgRow m;
        m.id = o.msgid;
        m.tstamp = o.tstamp;
        m.durable = true;
        m.refer = (int32_t)o.q;
        m.bseg = o.seg;
        m.boff = (uint64_t)o.offset;
        m.blen = (uint32_t)o.size;
        put_msg(std::move(m));
        break;
      }
      default: break;
    }
  }
}

void Store::applyRows(const std::vector<const std::string*>& qids, const RowOp* ops, size_t n) {
  if (!n) return;
  LOCK;
  apply_rows(qids, ops, n);
  if (fd_ < 0) return;
  size_t bytes = 8 + n * sizeof(RowOp);
  for (auto* q : qids) bytes += 4 + q->size();
  std::string pl(bytes, '\0');
  char* d = &pl[0];
  uint32_t v = (uint32_t)qids.size();
  memcpy(d, &v, 4);
  d += 4;
  for (auto* q : qids) {
    v = (uint32_t)q->size();
    memcpy(d, &v, 4);
    memcpy(d + 4, q->data(), q->size());
    d += 4 + q->size();
  }
  v = (uint32_t)n;
  memcpy(d, &v, 4);
  memcpy(d + 4, ops, n * sizeof(RowOp));
  append_wal(OP_ROWS, pl);
}

void Store::placeBodies(const char* const* recs, const uint32_t* lens, size_t n, BodyLog::Loc* out) {
  LOCK;
  if (!body_) throw std::runtime_error("store: the body log needs a store on disk");
  body_->put(recs, lens, n, out);
  dirty_ = true;
}

void Store::insertMessageRefs(const BodyRef* refs, size_t n) {
  LOCK;
  if (!body_) throw std::runtime_error("store: the body log needs a store on disk");
  std::vector<const char*> recs(n);
  std::vector<uint32_t> lens(n);
  std::vector<BodyLog::Loc> locs(n);
  for (size_t i = 0; i < n; ++i) { recs[i] = refs[i].rec; lens[i] = refs[i].len; }
  body_->put(recs.data(), lens.data(), n, locs.data());
  dirty_ = true;
  const int64_t now = now_ms();
  for (size_t i = 0; i < n; ++i) {
    MsgRow m;
    m.id = refs[i].id;
    m.tstamp = refs[i].tstamp;
    m.durable = true;
    m.refer = refs[i].refer;
    m.bseg = locs[i].seg;
    m.boff = locs[i].off;
    m.blen = locs[i].len;
    append_wal(OP_MSG_REF, enc_ref(m, 0, now));
    put_msg(std::move(m));
  }
}

void Store::updateMessageReferCount(int64_t id, int32_t refer) {
  LOCK; Writer w; w.llng((u64)id); w.lng((u32)refer); append(OP_MSG_REFER, w.done());
}
bool Store::selectMessage(int64_t id, MsgRow* out) {
  LOCK;
  auto it = msgs_.find(id);
  if (it == msgs_.end()) return false;
  if (it->second.expire_at && it->second.expire_at <= now_ms()) return false;
  *out = it->second;
  if (it->second.bseg >= 0) {   // the bytes are in the body log
    std::string rec;
    if (!body_ || !body_->read(BodyLog::Loc{(uint32_t)it->second.bseg, it->second.blen, it->second.boff}, &rec) ||
        !dec_body(rec, out))
      return false;   // a torn body: its message was never confirmed
  }
  return true;
}
void Store::deleteMessage(int64_t id) { LOCK; Writer w; w.llng((u64)id); append(OP_MSG_DEL, w.done()); }

void Store::insertQueueMeta(const std::string& q, int64_t lconsumed, const std::set<std::string>& consumers,
                            bool durable, int64_t ttl) {
  LOCK;
  Writer w;
  w.longstr(q); w.llng((u64)lconsumed); w.lng((u32)consumers.size());
  for (auto& c : consumers) w.longstr(c);
  w.octet(durable); w.llng((u64)ttl);
  append(OP_QMETA_INS, w.done());
}
void Store::insertQueueMsg(const std::string& q, int64_t offset, int64_t msgid, int32_t size, int64_t ttl_ms) {
  LOCK;
  Writer w;
  w.longstr(q); w.llng((u64)offset); w.llng((u64)msgid); w.lng((u32)size); w.llng((u64)ttl_ms);
  w.llng((u64)now_ms());
  append(OP_QMSG_INS, w.done());
}
void Store::deleteQueueMsg(const std::string& q, int64_t offset) {
  LOCK; Writer w; w.longstr(q); w.llng((u64)offset); append(OP_QMSG_DEL, w.done());
}
void Store::insertLastConsumed(const std::string& q, int64_t l) {
  LOCK; Writer w; w.longstr(q); w.llng((u64)l); append(OP_QLAST, w.done());
}
void Store::consumedQueueMessages(const std::string& q, int64_t l, const std::vector<QueueMsgRow>& unacks) {
  LOCK;
  Writer w;
  w.longstr(q); w.llng((u64)l); w.lng((u32)unacks.size());
  for (auto& u : unacks) { w.llng((u64)u.offset); w.llng((u64)u.msgid); w.lng((u32)u.size); }
  append(OP_QCONSUMED, w.done());
}
bool Store::selectQueue(const std::string& q, QueueMetaRow* meta, std::vector<QueueMsgRow>* msgs,
                        std::vector<QueueMsgRow>* unacks) {
  LOCK;
  auto mi = queue_metas_.find(q);
  if (mi == queue_metas_.end()) return false;
  if (meta) *meta = mi->second;
  int64_t now = now_ms();
  if (msgs) {
    msgs->clear();
    auto qi = queues_.find(q);
    if (qi != queues_.end())
      for (auto it = qi->second.upper_bound(mi->second.lconsumed); it != qi->second.end(); ++it)
        if (!it->second.expire_at || it->second.expire_at > now) msgs->push_back(it->second);
  }
  if (unacks) {
    unacks->clear();
    auto ui = queue_unacks_.find(q);
    if (ui != queue_unacks_.end())
      for (auto& kv : ui->second) unacks->push_back(kv.second);
  }
  return true;
}
void Store::forceDeleteQueue(const std::string& q) { LOCK; Writer w; w.longstr(q); append(OP_QFORCE_DEL, w.done()); }
void Store::pendingDeleteQueue(const std::string& q) { LOCK; Writer w; w.longstr(q); append(OP_QPENDING_DEL, w.done()); }
void Store::deleteConsumedQueueMsgs(const std::string& q, int64_t upto) {
  LOCK; Writer w; w.longstr(q); w.llng((u64)upto); append(OP_QDEL_CONSUMED, w.done());
}
void Store::insertQueueUnack(const std::string& q, int64_t offset, int64_t msgid, int32_t size) {
  LOCK; Writer w; w.longstr(q); w.llng((u64)offset); w.llng((u64)msgid); w.lng((u32)size);
  append(OP_QUNACK_INS, w.done());
}
void Store::deleteQueueUnack(const std::string& q, int64_t msgid) {
  LOCK; Writer w; w.longstr(q); w.llng((u64)msgid); append(OP_QUNACK_DEL, w.done());
}
// ---- change feed
void Store::setMirror(bool on) {
  LOCK;
  mirror_ = on;
  if (!on) {
    md_msgs_.clear(); md_qmsgs_.clear(); md_qunacks_.clear(); md_qmetas_.clear(); md_qparts_.clear();
    md_xs_.clear(); md_vhosts_.clear(); md_deleted_.clear();
  }
}

size_t Store::mirrorPending() {
  LOCK;
  return md_msgs_.size() + md_qmsgs_.size() + md_qunacks_.size() + md_qmetas_.size() + md_qparts_.size() +
         md_xs_.size() + md_vhosts_.size() + md_deleted_.size();
}

Store::MirrorKeys Store::mirrorTake(size_t max_keys) {
  LOCK;
  MirrorKeys k;
  auto take = [&](auto& set, auto& out) {
    auto it = set.begin();
    for (size_t n = 0; it != set.end() && n < max_keys; ++n) out.push_back(*it++);
    set.erase(set.begin(), it);
  };
  // a whole partition rewritten covers that queue's single-row keys (taken with it)
  take(md_qparts_, k.qparts);
  std::set<std::string> parts(k.qparts.begin(), k.qparts.end());
  auto take_rows = [&](std::set<std::pair<std::string, int64_t>>& set, std::vector<std::pair<std::string, int64_t>>& out) {
    size_t n = 0;
    for (auto it = set.begin(); it != set.end() && n < max_keys;) {
      if (!parts.count(it->first)) { out.push_back(*it); ++n; }
      it = set.erase(it);
    }
  };
  take_rows(md_qmsgs_, k.qmsgs);
  take_rows(md_qunacks_, k.qunacks);
  take(md_msgs_, k.msgs);
  take(md_qmetas_, k.qmetas);
  take(md_xs_, k.xs);
  take(md_vhosts_, k.vhosts);
  take(md_deleted_, k.deleted);
  return k;
}

bool Store::selectQueueMsg(const std::string& q, int64_t offset, QueueMsgRow* out) {
  LOCK;
  auto qi = queues_.find(q);
  if (qi == queues_.end()) return false;
  auto it = qi->second.find(offset);
  if (it == qi->second.end() || (it->second.expire_at && it->second.expire_at <= now_ms())) return false;
  *out = it->second;
  return true;
}

bool Store::selectQueueUnack(const std::string& q, int64_t msgid, QueueMsgRow* out) {
  LOCK;
  auto qi = queue_unacks_.find(q);
  if (qi == queue_unacks_.end()) return false;
  auto it = qi->second.find(msgid);
  if (it == qi->second.end()) return false;
  *out = it->second;
  return true;
}

bool Store::selectQueueMeta(const std::string& q, QueueMetaRow* out) {
  LOCK;
  auto it = queue_metas_.find(q);
  if (it == queue_metas_.end()) return false;
  *out = it->second;
  return true;
}

void Store::insertExchange(const std::string& id, const ExchangeRow& x) {
  LOCK; Writer w; w.longstr(id); w.longstr(x.tpe); w.octet(x.durable); w.octet(x.autodel); w.octet(x.internal);
  w_map(w, x.args); append(OP_X_INS, w.done());
}
void Store::insertBind(const std::string& id, const std::string& queue, const std::string& key,
                       const std::map<std::string, std::string>& args) {
  LOCK; Writer w; w.longstr(id); w.longstr(queue); w.longstr(key); w_map(w, args); append(OP_BIND_INS, w.done());
}
bool Store::selectExchange(const std::string& id, ExchangeRow* x, std::vector<BindRow>* binds) {
  LOCK;
  auto it = exchanges_.find(id);
  if (it == exchanges_.end()) return false;
  if (x) *x = it->second;
  if (binds) {
    binds->clear();
    auto bi = binds_.find(id);
    if (bi != binds_.end())
      for (auto& kv : bi->second) binds->push_back(kv.second);
  }
  return true;
}
void Store::deleteBind(const std::string& id, const std::string& queue, const std::string& key) {
  LOCK; Writer w; w.longstr(id); w.longstr(queue); w.longstr(key); append(OP_BIND_DEL, w.done());
}
void Store::deleteBindsOfQueue(const std::string& queue) {
  LOCK; Writer w; w.longstr(queue); append(OP_BIND_DEL_Q, w.done());
}
void Store::deleteExchange(const std::string& id) { LOCK; Writer w; w.longstr(id); append(OP_X_DEL, w.done()); }
void Store::insertVhost(const std::string& id, bool active) { LOCK; append(OP_VH_INS, enc_vh(id, active)); }
bool Store::selectVhost(const std::string& id, bool* active) {
  LOCK;
  auto it = vhosts_.find(id);
  if (it == vhosts_.end()) return false;
  if (active) *active = it->second;
  return true;
}
void Store::deleteVhost(const std::string& id) { LOCK; Writer w; w.longstr(id); append(OP_VH_DEL, w.done()); }

std::vector<std::string> Store::deletedQueueIds() {
  LOCK;
  std::set<std::string> ids;
  for (auto& kv : queue_metas_deleted_) ids.insert(kv.first);
  for (auto& kv : queues_deleted_) if (!kv.second.empty()) ids.insert(kv.first);
  for (auto& kv : queue_unacks_deleted_) if (!kv.second.empty()) ids.insert(kv.first);
  return std::vector<std::string>(ids.begin(), ids.end());
}
bool Store::selectDeletedQueue(const std::string& q, QueueMetaDeletedRow* meta, std::vector<QueueMsgRow>* msgs,
                               std::vector<QueueMsgRow>* unacks) {
  LOCK;
  auto mi = queue_metas_deleted_.find(q);
  if (meta) *meta = mi != queue_metas_deleted_.end() ? mi->second : QueueMetaDeletedRow{};
  if (msgs) {
    msgs->clear();
    auto it = queues_deleted_.find(q);
    if (it != queues_deleted_.end()) for (auto& kv : it->second) msgs->push_back(kv.second);
  }
  if (unacks) {
    unacks->clear();
    auto it = queue_unacks_deleted_.find(q);
    if (it != queue_unacks_deleted_.end()) for (auto& kv : it->second) unacks->push_back(kv.second);
  }
  return mi != queue_metas_deleted_.end();
}
void Store::insertDeletedQueueMeta(const std::string& q, int64_t lconsumed, int32_t nconsumer, bool durable) {
  LOCK;
  QueueMetaDeletedRow d;
  d.lconsumed = lconsumed; d.nconsumer = nconsumer; d.durable = durable;
  append(OP_QDMETA_INS, enc_qdmeta(q, d));
}
void Store::insertDeletedQueueMsg(const std::string& q, int64_t offset, int64_t msgid, int32_t size) {
  LOCK; append(OP_QDMSG_INS, enc_qrow(q, offset, msgid, size));
}
void Store::insertDeletedQueueUnack(const std::string& q, int64_t offset, int64_t msgid, int32_t size) {
  LOCK; append(OP_QDUNACK_INS, enc_qrow(q, offset, msgid, size));
}

std::vector<std::string> Store::vhostIds() {
  LOCK; std::vector<std::string> v; for (auto& kv : vhosts_) v.push_back(kv.first); return v;
}
std::vector<std::string> Store::exchangeIds() {
  LOCK; std::vector<std::string> v; for (auto& kv : exchanges_) v.push_back(kv.first); return v;
}
std::vector<std::string> Store::queueIds() {
  LOCK; std::vector<std::string> v; for (auto& kv : queue_metas_) v.push_back(kv.first); return v;
}
std::vector<int64_t> Store::messageIds() {
  LOCK; std::vector<int64_t> v; for (auto& kv : msgs_) v.push_back(kv.first); return v;
}
size_t Store::rowCount(const std::string& t) {
  LOCK;
  auto count2 = [](const std::map<std::string, std::map<int64_t, QueueMsgRow>>& m) {
    size_t n = 0; for (auto& kv : m) n += kv.second.size(); return n; };
  if (t == "msgs") return msgs_.size();
  if (t == "queues") return count2(queues_);
  if (t == "queues_deleted") return count2(queues_deleted_);
  if (t == "queue_unacks") return count2(queue_unacks_);
  if (t == "queue_unacks_deleted") return count2(queue_unacks_deleted_);
  if (t == "queue_metas") return queue_metas_.size();
  if (t == "queue_metas_deleted") return queue_metas_deleted_.size();
  if (t == "exchanges") return exchanges_.size();
  if (t == "binds") { size_t n = 0; for (auto& kv : binds_) n += kv.second.size(); return n; }
  if (t == "vhosts") return vhosts_.size();
  throw std::runtime_error("unknown table " + t);
}

}  // namespace cmq

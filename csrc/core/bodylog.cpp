#include "bodylog.hpp"

#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <stdexcept>

#include <nmmintrin.h>

namespace cmq {

namespace {
const uint32_t MAGIC = 0x42514D43u;   // "CMQB"
double mono() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

// pwritev of the whole vector, continuing after short writes
bool pwritev_all(int fd, iovec* iov, int cnt, uint64_t off, std::string* err) {
  while (cnt > 0) {
    ssize_t k = ::pwritev(fd, iov, cnt, (off_t)off);
    if (k < 0) {
      if (errno == EINTR) continue;
      *err = std::string("body log write: ") + strerror(errno);
      return false;
    }
    off += (uint64_t)k;
    size_t left = (size_t)k;
    while (cnt > 0 && left >= iov->iov_len) { left -= iov->iov_len; ++iov; --cnt; }
    if (cnt > 0 && left) { iov->iov_base = (char*)iov->iov_base + left; iov->iov_len -= left; }
  }
  return true;
}
}  // namespace

__attribute__((target("sse4.2"))) uint32_t crc32c(const char* p, size_t n) {
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

BodyLog::BodyLog(std::string dir, bool fsync) : dir_(std::move(dir)), fsync_(fsync) {}

BodyLog::~BodyLog() { close(); }

void BodyLog::configure(int stripes, uint64_t seg_bytes) {
  std::lock_guard<std::mutex> g(mu_);
  if (started_) return;   // fixed once the first body is written
  nstripes_ = std::max(1, std::min(stripes, 64));
  seg_bytes_ = std::max<uint64_t>(seg_bytes, 1u << 20);
}

std::string BodyLog::path(uint32_t seg) const {
  char b[32];
  snprintf(b, sizeof b, "/%010u.seg", seg);
  return dir_ + b;
}

// the directory entry of a new segment file is durable before a row names it: fsync of
// the bodies directory after its mkdir and after each segment creation (rare: one per
// seg_bytes of a stripe), ahead of the group commit that references the segment
void BodyLog::sync_dir_locked() {
  if (!fsync_) return;
  if (dfd_ < 0) dfd_ = ::open(dir_.c_str(), O_RDONLY | O_DIRECTORY);
  if (dfd_ >= 0) ::fsync(dfd_);
}

void BodyLog::start_locked() {
  if (started_) return;
  if (::mkdir(dir_.c_str(), 0755) == 0 && fsync_) {   // a new directory: its parent's entry too
    const size_t sl = dir_.find_last_of('/');
    const int pfd = ::open(sl == std::string::npos ? "." : dir_.substr(0, sl ? sl : 1).c_str(), O_RDONLY | O_DIRECTORY);
    if (pfd >= 0) { ::fsync(pfd); ::close(pfd); }
  }
  st_ = std::vector<Stripe>(nstripes_);
  for (int k = 0; k < nstripes_; ++k) st_[k].th = std::thread([this, k] { run(k); });
  started_ = true;
}

void BodyLog::roll_locked(Stripe& s) {
  const uint32_t seg = next_seg_++;
  const int fd = ::open(path(seg).c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) throw std::runtime_error("body log: cannot create " + path(seg));
  sync_dir_locked();
  std::lock_guard<std::mutex> a(amu_);
  if (s.fd >= 0) {
    s.retired.push_back(s.fd);
    Seg& old = segs_[s.seg];
    old.current = false;
    if (old.live_n == 0) dead_.push_back(s.seg);
  }
  segs_[seg].current = true;
  s.fd = fd;
  s.seg = seg;
  s.off = 0;
}

void BodyLog::put(const char* const* recs, const uint32_t* lens, size_t n, Loc* out) {
  if (!n) return;
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i) total += FRAME + lens[i];
  std::lock_guard<std::mutex> g(mu_);
  if (q_lim_ && (!err_.empty() || q_used_->fetch_add(total) + total > q_lim_)) {
    if (err_.empty()) err_ = "body log write: No space left on device (store quota of " + std::to_string(q_lim_) + " bytes)";
    for (size_t i = 0; i < n; ++i) out[i] = Loc{};
    return;
  }
  start_locked();
  // contiguous chunks of about equal bytes, one per stripe (small groups use fewer)
  const int k = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)nstripes_, total / (256u << 10)));
  const uint64_t per = (total + k - 1) / k;
  size_t i = 0;
  for (int c = 0; c < k && i < n; ++c) {
    Stripe& s = st_[rr_];
    rr_ = (rr_ + 1) % nstripes_;
    uint64_t bytes = 0;
    size_t j = i;
    while (j < n && (bytes < per || c == k - 1)) bytes += FRAME + lens[j++];
    if (s.fd < 0 || (s.off && s.off + bytes > seg_bytes_)) roll_locked(s);
    Job job;
    job.fd = s.fd;
    job.off = s.off;
    job.recs.assign(recs + i, recs + j);
    job.lens.assign(lens + i, lens + j);
    for (size_t t = i; t < j; ++t) {
      out[t] = Loc{s.seg, lens[t], s.off};
      s.off += FRAME + lens[t];
    }
    {
      std::lock_guard<std::mutex> a(amu_);
      segs_[s.seg].size = s.off;
      stats_.written += bytes;
      stats_.records += j - i;
    }
    s.q.push_back(std::move(job));
    ++pending_;
    i = j;
  }
  cv_.notify_all();
}

void BodyLog::run(int k) {
  std::unique_lock<std::mutex> g(mu_);
  Stripe& s = st_[k];
  std::vector<int> touched;
  std::vector<uint32_t> frames;
  std::vector<iovec> iov;
  uint64_t done = 0;
  while (true) {
    cv_.wait(g, [&] { return !s.q.empty() || stop_; });
    if (s.q.empty()) break;   // stop_ and nothing left
    std::string err;
    double w0 = 0, ws = 0;
    while (!s.q.empty()) {
      Job j = std::move(s.q.front());
      s.q.pop_front();
      g.unlock();
      const double t0 = mono();
      const size_t n = j.recs.size();
      frames.resize(4 * n);
      for (size_t t = 0; t < n; ++t) {
        frames[4 * t] = MAGIC;
        frames[4 * t + 1] = j.lens[t];
        frames[4 * t + 2] = crc32c(j.recs[t], j.lens[t]);
        frames[4 * t + 3] = 0;
      }
      uint64_t off = j.off;
      for (size_t t0r = 0; t0r < n && err.empty(); t0r += 512) {   // IOV_MAX is 1024
        const size_t t1 = std::min(n, t0r + 512);
        iov.clear();
        uint64_t bytes = 0;
        for (size_t t = t0r; t < t1; ++t) {
          iov.push_back(iovec{&frames[4 * t], FRAME});
          iov.push_back(iovec{(void*)j.recs[t], j.lens[t]});
          bytes += FRAME + j.lens[t];
        }
        pwritev_all(j.fd, iov.data(), (int)iov.size(), off, &err);
        off += bytes;
      }
      if (std::find(touched.begin(), touched.end(), j.fd) == touched.end()) touched.push_back(j.fd);
      w0 += mono() - t0;
      g.lock();
      ++done;
    }
    std::vector<int> retired;
    retired.swap(s.retired);   // every job of a rolled segment was queued before the roll
    g.unlock();
    const double s0 = mono();
    if (fsync_)
      for (int fd : touched)
        if (::fdatasync(fd) != 0 && err.empty()) err = std::string("body log fdatasync: ") + strerror(errno);
    for (int fd : retired) ::close(fd);
    touched.clear();
    ws = mono() - s0;
    {
      std::lock_guard<std::mutex> a(amu_);
      stats_.write_s += w0;
      stats_.sync_s += ws;
    }
    g.lock();
    if (!err.empty() && err_.empty()) err_ = err;
    pending_ -= done;
    done = 0;
    done_cv_.notify_all();
  }
}

bool BodyLog::wait(std::string* err) {
  std::unique_lock<std::mutex> g(mu_);
  done_cv_.wait(g, [&] { return pending_ == 0; });
  if (!err_.empty()) {
    if (err) *err = err_;
    return false;
  }
  return true;
}

void BodyLog::ref(const Loc& l) {
  std::lock_guard<std::mutex> a(amu_);
  Seg& s = segs_[l.seg];
  s.live_n++;
  s.live_bytes += l.len;
}

void BodyLog::unref(const Loc& l) {
  std::lock_guard<std::mutex> a(amu_);
  auto it = segs_.find(l.seg);
  if (it == segs_.end() || it->second.live_n == 0) return;
  Seg& s = it->second;
  s.live_n--;
  s.live_bytes -= std::min<uint64_t>(s.live_bytes, l.len);
  if (s.live_n == 0 && !s.current) dead_.push_back(l.seg);
}

void BodyLog::reap() {
  std::vector<std::pair<int, std::string>> out;
  {
    std::lock_guard<std::mutex> a(amu_);
    for (uint32_t seg : dead_) {
      auto it = segs_.find(seg);
      if (it == segs_.end() || it->second.live_n || it->second.current) continue;
      out.emplace_back(it->second.rfd, path(seg));
      stats_.reclaimed += it->second.size;
      segs_.erase(it);
    }
    dead_.clear();
  }
  if (out.empty()) return;
  std::lock_guard<std::mutex> r(rmu_);
  if (!reap_th_.joinable()) {
    reap_stop_ = false;
    reap_th_ = std::thread([this] { reaper(); });
  }
  for (auto& e : out) reap_q_.push_back(std::move(e));
  rcv_.notify_one();
}

void BodyLog::reaper() {
  std::unique_lock<std::mutex> r(rmu_);
  while (true) {
    rcv_.wait(r, [&] { return reap_stop_ || !reap_q_.empty(); });
    if (reap_q_.empty()) return;   // (stop: after the queue drained)
    auto e = std::move(reap_q_.front());
    reap_q_.pop_front();
    r.unlock();
    if (e.first >= 0) ::close(e.first);
    ::unlink(e.second.c_str());
    r.lock();
  }
}

bool BodyLog::read(const Loc& l, std::string* rec) {
  {
    std::unique_lock<std::mutex> g(mu_);   // a record of a group still being written
    done_cv_.wait(g, [&] { return pending_ == 0; });
  }
  int fd;
  {
    std::lock_guard<std::mutex> a(amu_);
    auto it = segs_.find(l.seg);
    if (it == segs_.end()) { stats_.bad_reads++; return false; }
    if (it->second.rfd < 0) it->second.rfd = ::open(path(l.seg).c_str(), O_RDONLY);
    fd = it->second.rfd;
  }
  std::string buf(FRAME + l.len, '\0');
  size_t got = 0;
  while (fd >= 0 && got < buf.size()) {
    ssize_t k = ::pread(fd, &buf[got], buf.size() - got, (off_t)(l.off + got));
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) break;
    got += (size_t)k;
  }
  uint32_t f[4];
  if (got == buf.size()) memcpy(f, buf.data(), sizeof f);
  if (got != buf.size() || f[0] != MAGIC || f[1] != l.len || f[2] != crc32c(buf.data() + FRAME, l.len)) {
    std::lock_guard<std::mutex> a(amu_);
    stats_.bad_reads++;
    return false;
  }
  rec->assign(buf, FRAME, l.len);
  return true;
}

void BodyLog::open_existing() {
  DIR* d = ::opendir(dir_.c_str());
  if (!d) return;
  std::lock_guard<std::mutex> g(mu_);
  std::lock_guard<std::mutex> a(amu_);
  while (dirent* e = ::readdir(d)) {
    unsigned id = 0;
    char tail[8] = {0};
    if (sscanf(e->d_name, "%10u.%3s", &id, tail) != 2 || strcmp(tail, "seg") != 0) continue;
    next_seg_ = std::max<uint32_t>(next_seg_, id + 1);
    const std::string p = path(id);
    auto it = segs_.find(id);
    if (it == segs_.end() || it->second.live_n == 0) {   // nothing refers to it any more
      ::unlink(p.c_str());
      if (it != segs_.end()) segs_.erase(it);
      continue;
    }
    struct stat sb;
    if (::stat(p.c_str(), &sb) == 0) it->second.size = (uint64_t)sb.st_size;
  }
  ::closedir(d);
}

BodyLog::Stats BodyLog::stats() {
  std::lock_guard<std::mutex> a(amu_);
  Stats s = stats_;
  for (auto& kv : segs_) {
    s.live_bytes += kv.second.live_bytes;
    s.live_records += kv.second.live_n;
    s.disk_bytes += kv.second.size;
  }
  s.segments = segs_.size();
  return s;
}

void BodyLog::close() {
  bool started;
  {
    std::lock_guard<std::mutex> g(mu_);
    started = started_;
    stop_ = true;
  }
  cv_.notify_all();
  if (started) {
    for (auto& s : st_)
      if (s.th.joinable()) s.th.join();
    for (auto& s : st_) {
      if (s.fd >= 0) ::close(s.fd);
      for (int fd : s.retired) ::close(fd);
    }
  }
  if (dfd_ >= 0) { ::close(dfd_); dfd_ = -1; }
  {
    std::unique_lock<std::mutex> r(rmu_);
    reap_stop_ = true;
    rcv_.notify_all();
    r.unlock();
    if (reap_th_.joinable()) reap_th_.join();
  }
  std::lock_guard<std::mutex> g(mu_);
  std::lock_guard<std::mutex> a(amu_);
  st_.clear();
  started_ = stop_ = false;
  for (auto& kv : segs_) {
    if (kv.second.rfd >= 0) ::close(kv.second.rfd);
    kv.second.rfd = -1;
    if (kv.second.current && !kv.second.live_n) dead_.push_back(kv.first);
    kv.second.current = false;
  }
}

}  // namespace cmq

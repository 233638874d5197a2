// Host side of the per-step cross-rank exchange of a sharded broker: a POSIX
// shared-memory all-to-all between the rank processes of one host.
//
// The production path between GPUs is RCCL over xGMI (engine.hip, RcclXchg: direct
// ncclSend / ncclRecv of device buffers).  This backend serves the rehearsal of N ranks
// on fewer GPUs (several processes on one MI355X, as in the CI box) and CPU tests: each
// rank owns one mailbox in a shared segment; a collective = write own mailbox, barrier,
// read the parts addressed to this rank.  The count exchange double-buffers its header
// area, and the bulk data area is reused safely because the next count exchange's
// barrier is only passed once every rank has finished reading it.
//
// Failure model: every barrier wait is bounded (timeout_ms) and reports -2, so a dead
// peer surfaces as an exchange failure in the stepper (frontend.cpp), never as a hang.
// After a membership change the survivors open a new segment (new name) over the live
// ranks.  Plain C++ (no HIP): included by the engine (hipcc) and the core (g++) builds.
#pragma once
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace cmqx {

constexpr int XH_WORDS = 16;       // u32 header words per (source, destination) pair
constexpr int XMAX = 16;           // ranks (dp_state.h WORLD_MAX)

struct ShmCtl {                    // first 4 KB of the segment
  std::atomic<uint32_t> arrive;
  std::atomic<uint32_t> gen;
  uint32_t n;                      // ranks in this group
  uint32_t magic;
};

class ShmXchg {
 public:
  // name: shm object name shared by the group; members: logical ranks (sorted, this rank
  // included); box_bytes: mailbox bytes per rank (data area)
  ShmXchg(const std::string& name, const std::vector<int>& members, int me, size_t box_bytes, int timeout_ms)
      : name_(name), members_(members), me_(me), timeout_ms_(timeout_ms) {
    if (members_.empty() || members_.size() > (size_t)XMAX) throw std::runtime_error("shm xchg: bad group");
    idx_ = (int)(std::find(members_.begin(), members_.end(), me_) - members_.begin());
    if (idx_ >= (int)members_.size()) throw std::runtime_error("shm xchg: this rank is not a member");
    box_ = (box_bytes + 4095) & ~(size_t)4095;
    hdr_ = 2 * (size_t)XMAX * XMAX * XH_WORDS * 4 + (size_t)XMAX * 8 * 2;   // 2 header areas + directory
    hdr_ = (hdr_ + 4095) & ~(size_t)4095;
    per_ = hdr_ + box_;
    total_ = 4096 + per_ * members_.size();
    std::string nm = "/" + name_;
    fd_ = ::shm_open(nm.c_str(), O_CREAT | O_RDWR, 0600);
    if (fd_ < 0) throw std::runtime_error("shm xchg: shm_open " + nm + " failed");
    struct stat st;
    if (::fstat(fd_, &st) == 0 && (size_t)st.st_size < total_ && ::ftruncate(fd_, (off_t)total_) != 0)
      throw std::runtime_error("shm xchg: ftruncate failed");
    base_ = (uint8_t*)::mmap(nullptr, total_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
    if (base_ == MAP_FAILED) throw std::runtime_error("shm xchg: mmap failed");
    ctl_ = (ShmCtl*)base_;
    gen_seen_ = ctl_->gen.load();
  }
  ~ShmXchg() {
    if (base_ && base_ != MAP_FAILED) ::munmap(base_, total_);
    if (fd_ >= 0) ::close(fd_);
    // (normally unlinked after the first exchange; a group that never exchanged)
    std::string nm = "/" + name_;
    if (idx_ == 0 && !unlinked_) ::shm_unlink(nm.c_str());
  }
  ShmXchg(const ShmXchg&) = delete;
  ShmXchg& operator=(const ShmXchg&) = delete;

  const std::vector<int>& members() const { return members_; }
  int index_of(int logical) const {
    for (size_t i = 0; i < members_.size(); ++i)
      if (members_[i] == logical) return (int)i;
    return -1;
  }
  size_t box_bytes() const { return box_; }
  // data area of member `i`
  uint8_t* box(int i) { return base_ + 4096 + per_ * (size_t)i + hdr_; }
  // header area (parity k) of member i: [dest member][XH_WORDS] u32
  uint32_t* hdr(int i, int k) { return (uint32_t*)(base_ + 4096 + per_ * (size_t)i) + (size_t)(k & 1) * XMAX * XMAX * XH_WORDS; }
  // directory of member i: u64 [XMAX] offsets of its data for each destination member
  uint64_t* dir(int i) {
    return (uint64_t*)(base_ + 4096 + per_ * (size_t)i + 2 * (size_t)XMAX * XMAX * XH_WORDS * 4);
  }

  // all members arrive; 0, or -2 after timeout_ms (a peer is gone)
  int barrier() {
    const uint32_t n = (uint32_t)members_.size();
    const uint32_t g = ctl_->gen.load(std::memory_order_acquire);
    if (ctl_->arrive.fetch_add(1, std::memory_order_acq_rel) + 1 == n) {
      ctl_->arrive.store(0, std::memory_order_relaxed);
      ctl_->gen.store(g + 1, std::memory_order_release);
      return 0;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; ++spin) {
      if (ctl_->gen.load(std::memory_order_acquire) != g) return 0;
      if (spin < 2000) { sched_yield(); continue; }
      timespec ts{0, 20000};
      nanosleep(&ts, nullptr);
      if ((spin & 63) == 0 &&
          std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count() >
              timeout_ms_)
        return withdraw(g);
    }
  }

  // Timed out: take this rank's arrival back, so the generation cannot complete without
  // it and every member reports the same outcome (all pass, or all time out and drop the
  // step's exchange together).  If the last member arrived meanwhile, the generation did
  // complete and this rank passes too.
  int withdraw(uint32_t g) {
    uint32_t a = ctl_->arrive.load(std::memory_order_acquire);
    while (true) {
      if (ctl_->gen.load(std::memory_order_acquire) != g) return 0;
      if (a == 0) {   // the completing member reset the count: its gen store follows
        sched_yield();
        a = ctl_->arrive.load(std::memory_order_acquire);
        continue;
      }
      if (ctl_->arrive.compare_exchange_weak(a, a - 1, std::memory_order_acq_rel, std::memory_order_acquire))
        return ctl_->gen.load(std::memory_order_acquire) != g ? 0 : -2;
    }
  }

  // count exchange: send[dest member][XH_WORDS] -> recv[src member][XH_WORDS]
  int counts(const uint32_t* send, uint32_t* recv) {
    const int k = (int)(seq_++ & 1);
    const int n = (int)members_.size();
    memcpy(hdr(idx_, k), send, (size_t)n * XH_WORDS * 4);
    std::atomic_thread_fence(std::memory_order_release);
    int rc = barrier();
    if (rc) return rc;
    if (!unlinked_) {   // every member has it mapped now: drop the name (nothing left in
      unlinked_ = true; // /dev/shm if a process is killed later)
      if (idx_ == 0) ::shm_unlink(("/" + name_).c_str());
    }
    for (int s = 0; s < n; ++s) memcpy(recv + (size_t)s * XH_WORDS, hdr(s, k) + (size_t)idx_ * XH_WORDS, XH_WORDS * 4);
    return 0;
  }

 private:
  std::string name_;
  std::vector<int> members_;
  int me_ = 0, idx_ = 0, timeout_ms_ = 10000;
  size_t box_ = 0, hdr_ = 0, per_ = 0, total_ = 0;
  int fd_ = -1;
  uint8_t* base_ = nullptr;
  ShmCtl* ctl_ = nullptr;
  uint32_t gen_seen_ = 0;
  uint64_t seq_ = 0;
  bool unlinked_ = false;
};

}  // namespace cmqx

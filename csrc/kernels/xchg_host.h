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
  // the barrier: generation << 32 | arrivals in it, one word, so an arrival, a withdrawal,
  // the completion (the last arrival moves it to (gen + 1, 0) in the same CAS) and the
  // abort of a generation nobody can complete any more are each one atomic step
  std::atomic<uint64_t> state;
  uint32_t n;                      // ranks in this group
  uint32_t magic;
  // how generation g ended, at [g % OUTCOMES]: g << 1 | aborted.  Written by the member
  // that completed g (after its CAS) or aborted it (before its CAS; an aborted generation
  // can never complete); a member that finds the state past its generation reads it here
  std::atomic<uint64_t> outcome[64];
};
constexpr uint64_t OUTCOMES = 64;

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
    gen_ = 0;   // a group's segment is new (fresh name): every member starts at generation 0
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

  // all members arrive; 0, or -2 after timeout_ms (a peer is gone).  Every member reports
  // the same outcome for a generation: it completes only by the n-th arrival, and a member
  // that timed out first takes its arrival back (withdraw), so the generation can no longer
  // complete -- the others time out too.  Arrivals carry the generation they are for
  // (gen_), so a member that failed generation g and comes back for g + 1 never counts
  // towards g: it aborts g instead, and a peer still waiting in g fails it.
  int barrier() {
    const uint64_t n = members_.size();
    const uint64_t b = gen_;
    uint64_t s = ctl_->state.load(std::memory_order_acquire);
    while (true) {
      const uint64_t g = s >> 32, c = s & 0xffffffffull;
      if (g > b) return settle(b);   // the group left b without this member (aborted)
      uint64_t nxt;
      if (g < b) {
        // generation g is still open but this member already failed it (it only moves
        // past g by failing it): nobody can complete g any more -- abort it, arrive in b
        for (uint64_t k = g; k < b; ++k) ctl_->outcome[k % OUTCOMES].store(k << 1 | 1, std::memory_order_release);
        nxt = n == 1 ? ((b + 1) << 32) : ((b << 32) | 1);
      } else {
        nxt = c + 1 == n ? ((b + 1) << 32) : s + 1;
      }
      if (ctl_->state.compare_exchange_weak(s, nxt, std::memory_order_acq_rel, std::memory_order_acquire)) {
        if ((nxt >> 32) == b + 1) {   // this arrival completed b
          ctl_->outcome[b % OUTCOMES].store(b << 1, std::memory_order_release);
          gen_ = b + 1;
          return 0;
        }
        break;
      }
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; ++spin) {
      if ((ctl_->state.load(std::memory_order_acquire) >> 32) != b) return settle(b);
      if (spin < 2000) { sched_yield(); continue; }
      timespec ts{0, 20000};
      nanosleep(&ts, nullptr);
      if ((spin & 63) == 0 &&
          (abort_.load(std::memory_order_relaxed) ||
           std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count() >
               timeout_ms_))
        return withdraw(b);
    }
  }

  // Timed out in generation b: take this rank's arrival back, so b cannot complete without
  // it.  If b completed (or was aborted) meanwhile, that outcome stands for this rank too.
  int withdraw(uint64_t b) {
    uint64_t s = ctl_->state.load(std::memory_order_acquire);
    while ((s >> 32) == b) {
      if (ctl_->state.compare_exchange_weak(s, s - 1, std::memory_order_acq_rel, std::memory_order_acquire)) {
        gen_ = b + 1;
        return -2;
      }
    }
    return settle(b);
  }

  // the state left generation b: completed (0) or aborted (-2), as recorded in the outcome
  // ring (its writer may still be between its CAS and that store: wait for it, bounded)
  int settle(uint64_t b) {
    gen_ = b + 1;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; ++spin) {
      const uint64_t o = ctl_->outcome[b % OUTCOMES].load(std::memory_order_acquire);
      if ((o >> 1) == b) return (o & 1) ? -2 : 0;
      sched_yield();
      if ((spin & 63) == 0 &&
          std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count() >
              timeout_ms_)
        return -2;
    }
  }

  // a waiting barrier gives up now (as after its timeout): the owner is shutting down
  void abort() { abort_.store(true, std::memory_order_relaxed); }

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
  std::atomic<bool> abort_{false};
  size_t box_ = 0, hdr_ = 0, per_ = 0, total_ = 0;
  int fd_ = -1;
  uint8_t* base_ = nullptr;
  ShmCtl* ctl_ = nullptr;
  uint64_t gen_ = 0;                 // the barrier generation this member's next call is for
  uint64_t seq_ = 0;
  bool unlinked_ = false;
};

}  // namespace cmqx

// RCCL backend of the per-step exchange (engine.hip): librccl is opened at run time
// (dlopen) and driven with grouped ncclSend / ncclRecv on a dedicated exchange stream --
// one point-to-point transfer per live peer and region, exactly the records each peer
// needs (no all-to-all padding), over xGMI between the MI355X of a node.
//
// The unique id comes from the launcher's c10d store (Python passes its 128 bytes);
// membership changes build a new communicator over the survivors (ncclCommAbort of the
// old one first).  Host waits are bounded: a peer that stops answering surfaces as -2 from
// wait() (the stepper fails over) instead of a stream that never drains.
#pragma once
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace cmqx {

typedef int ncclResult_t;
typedef struct ncclComm* ncclComm_t;
struct ncclUniqueId { char internal[128]; };
enum : int { nccl_int8 = 0 };

struct RcclLib {
  void* h = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
  bool standin = false;   // the test-only stand-in (tests/rccl_standin), not RCCL

  static RcclLib& get() {
    static RcclLib lib;
    if (!lib.h) lib.open();
    return lib;
  }
  template <class F>
  void sym(F& f, const char* n) {
    f = (F)dlsym(h, n);
    if (!f) throw std::runtime_error(std::string("librccl: missing symbol ") + n);
  }
  void open() {
    // CHANAMQ_RCCL_LIB: another library with the same entry points first -- the tests'
    // shared-memory stand-in that lets several ranks share one GPU (RCCL refuses that).
    // chanamq_amd.ops.load() refuses the override unless CHANAMQ_RCCL_STANDIN_OK=1
    const char* over = getenv("CHANAMQ_RCCL_LIB");
    if (over && *over) {
      if (!(h = dlopen(over, RTLD_NOW | RTLD_LOCAL)))
        throw std::runtime_error(std::string("CHANAMQ_RCCL_LIB: dlopen failed: ") + dlerror());
    } else {
      const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so"};
      for (const char* n : names)
        if ((h = dlopen(n, RTLD_NOW | RTLD_GLOBAL))) break;
    }
    if (!h) throw std::runtime_error("librccl not found (dlopen)");
    standin = dlsym(h, "cmq_rccl_standin") != nullptr;
    sym(GetUniqueId, "ncclGetUniqueId");
    sym(CommInitRank, "ncclCommInitRank");
    sym(Send, "ncclSend");
    sym(Recv, "ncclRecv");
    sym(GroupStart, "ncclGroupStart");
    sym(GroupEnd, "ncclGroupEnd");
    sym(CommAbort, "ncclCommAbort");
    sym(CommDestroy, "ncclCommDestroy");
    sym(CommGetAsyncError, "ncclCommGetAsyncError");
    sym(GetErrorString, "ncclGetErrorString");
  }
};

inline std::string rccl_unique_id() {
  ncclUniqueId id;
  RcclLib& L = RcclLib::get();
  ncclResult_t r = L.GetUniqueId(&id);
  if (r) throw std::runtime_error(std::string("ncclGetUniqueId: ") + L.GetErrorString(r));
  return std::string(id.internal, sizeof id.internal);
}

struct XPart { void* ptr; uint64_t bytes; };   // one region to / from one peer

class RcclXchg {
 public:
  // members: logical ranks of the communicator (sorted); comm rank = index in members
  RcclXchg(const std::string& uid, const std::vector<int>& members, int me, int timeout_ms)
      : members_(members), timeout_ms_(timeout_ms) {
    if (uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("rccl xchg: unique id must be 128 bytes");
    idx_ = -1;
    for (size_t i = 0; i < members_.size(); ++i)
      if (members_[i] == me) idx_ = (int)i;
    if (idx_ < 0) throw std::runtime_error("rccl xchg: this rank is not a member");
    ncclUniqueId id;
    memcpy(id.internal, uid.data(), sizeof id.internal);
    RcclLib& L = RcclLib::get();
    // high priority: a hardware queue of its own, never s_comp_'s (the asynchronous exchange
    // parks phase B there in k_xwait until this stream's counts and bulk are done)
    int plo = 0, phi = 0;
    if (hipDeviceGetStreamPriorityRange(&plo, &phi) != hipSuccess ||
        hipStreamCreateWithPriority(&s_, hipStreamNonBlocking, phi) != hipSuccess)
      throw std::runtime_error("rccl xchg: stream");
    if (hipEventCreateWithFlags(&ev_, hipEventDisableTiming) != hipSuccess) throw std::runtime_error("rccl xchg: event");
    ncclResult_t r = L.CommInitRank(&comm_, (int)members_.size(), id, idx_);
    if (r) throw std::runtime_error(std::string("ncclCommInitRank: ") + L.GetErrorString(r));
    if (hipMalloc(&dh_send_, 4ull * 16 * 16 * 16) != hipSuccess || hipMalloc(&dh_recv_, 4ull * 16 * 16 * 16) != hipSuccess)
      throw std::runtime_error("rccl xchg: header buffers");
    if (hipHostMalloc(&hh_, 4ull * 16 * 16 * 16 * 2, hipHostMallocPortable) != hipSuccess)
      throw std::runtime_error("rccl xchg: pinned header buffer");
  }
  ~RcclXchg() {
    if (comm_) (void)RcclLib::get().CommAbort(comm_);   // teardown: never wait on peers
    if (dh_send_) (void)hipFree(dh_send_);
    if (dh_recv_) (void)hipFree(dh_recv_);
    if (hh_) (void)hipHostFree(hh_);
    (void)hipEventDestroy(ev_);
    (void)hipStreamDestroy(s_);
  }
  RcclXchg(const RcclXchg&) = delete;
  RcclXchg& operator=(const RcclXchg&) = delete;

  hipStream_t stream() const { return s_; }
  hipEvent_t event() const { return ev_; }
  const std::vector<int>& members() const { return members_; }
  int index() const { return idx_; }

  // count exchange: send[member][words] -> recv[member][words] (blocking, bounded)
  int counts(const uint32_t* send, uint32_t* recv, int words) {
    const int n = (int)members_.size();
    const size_t row = 4ull * words;
    uint32_t* hs = (uint32_t*)hh_;
    uint32_t* hr = hs + 16 * 16 * 16;
    memcpy(hs, send, row * n);
    if (hipMemcpyAsync(dh_send_, hs, row * n, hipMemcpyHostToDevice, s_) != hipSuccess) return -1;
    RcclLib& L = RcclLib::get();
    if (L.GroupStart()) return -1;
    int bad = 0;   // a failed enqueue inside the group: the group still ends, then fails
    for (int i = 0; i < n; ++i) {
      if (i == idx_) continue;
      bad |= L.Send((const char*)dh_send_ + row * i, row, nccl_int8, i, comm_, s_) != 0;
      bad |= L.Recv((char*)dh_recv_ + row * i, row, nccl_int8, i, comm_, s_) != 0;
    }
    if (L.GroupEnd() || bad) { abort(); return -2; }
    if (hipMemcpyAsync(hr, dh_recv_, row * n, hipMemcpyDeviceToHost, s_) != hipSuccess) return -1;
    if (hipEventRecord(ev_, s_) != hipSuccess) return -1;
    int rc = wait(ev_);
    if (rc) return rc;
    memcpy(recv, hr, row * n);
    memcpy(recv + (size_t)idx_ * words, send + (size_t)idx_ * words, row);   // self: as sent
    return 0;
  }

  // bulk: parts to send / receive per peer member, in matching order on both sides;
  // stream-ordered (the caller waits on event() or makes its stream wait on it)
  int bulk(const std::vector<std::vector<XPart>>& sends, const std::vector<std::vector<XPart>>& recvs) {
    RcclLib& L = RcclLib::get();
    if (L.GroupStart()) return -1;
    const int n = (int)members_.size();
    int bad = 0;
    for (int i = 0; i < n; ++i) {
      if (i == idx_) continue;
      for (const XPart& p : sends[i])
        if (p.bytes) bad |= L.Send(p.ptr, p.bytes, nccl_int8, i, comm_, s_) != 0;
      for (const XPart& p : recvs[i])
        if (p.bytes) bad |= L.Recv(p.ptr, p.bytes, nccl_int8, i, comm_, s_) != 0;
    }
    if (L.GroupEnd() || bad) { abort(); return -2; }
    if (hipEventRecord(ev_, s_) != hipSuccess) return -1;
    return 0;
  }

  // bounded host wait on an event of the exchange stream; -2: a peer stopped answering
  // (the communicator is aborted so its kernels stop spinning)
  int wait(hipEvent_t e) {
    RcclLib& L = RcclLib::get();
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; ++spin) {
      hipError_t q = hipEventQuery(e);
      if (q == hipSuccess) return 0;
      if (q != hipErrorNotReady) return -1;
      if ((spin & 255) == 255) {
        ncclResult_t ae = 0;
        if (L.CommGetAsyncError(comm_, &ae) == 0 && ae != 0 && ae != 7 /* ncclInProgress */) { abort(); return -2; }
        auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
        if (ms > timeout_ms_) { abort(); return -2; }
      }
    }
  }

  void abort() {
    if (comm_ && !aborted_) { (void)RcclLib::get().CommAbort(comm_); aborted_ = true; comm_ = nullptr; }
  }

 private:
  std::vector<int> members_;
  int idx_ = 0, timeout_ms_ = 10000;
  ncclComm_t comm_ = nullptr;
  bool aborted_ = false;
  hipStream_t s_ = nullptr;
  hipEvent_t ev_ = nullptr;
  void* dh_send_ = nullptr;
  void* dh_recv_ = nullptr;
  void* hh_ = nullptr;
};

}  // namespace cmqx

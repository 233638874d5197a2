// TEST-ONLY stand-in for librccl: the ten entry points csrc/kernels/xchg_rccl.h resolves
// (ncclGetUniqueId ... ncclGetErrorString), implemented over POSIX shared memory and
// hipMemcpy, so the engine's RCCL exchange (RcclXchg: grouped send/recv, bounded waits,
// CommAbort + a new communicator on failover) can run with several ranks on ONE GPU --
// real RCCL refuses that ("Duplicate GPU detected").  It moves bytes; it is not a
// performance model of xGMI, and no number measured through it is a scaling number.
//
// Selected only by CHANAMQ_RCCL_LIB=<this .so> (xchg_rccl.h) together with
// CHANAMQ_RCCL_STANDIN_OK=1 (chanamq_amd.ops.load refuses it otherwise).
//
// Semantics kept from NCCL: calls between ncclGroupStart / ncclGroupEnd form one group;
// per peer, sends and receives match in call order.  Stricter than NCCL on purpose: at
// ncclGroupEnd the receiver checks that the peer's group carries exactly as many parts
// of exactly the sizes it posted, in the same order -- any mismatch fails the call
// (ncclInvalidUsage) with a message on stderr, so an exchange whose two sides disagree
// cannot pass a test by accident.  Data moves synchronously inside ncclGroupEnd (after the
// streams the calls named have drained); every wait is bounded and honours CommAbort.
//
// Layout of a communicator's segment: Hdr (one Chan per ordered pair (src, dst)), then one
// mailbox of box_bytes per pair.  A sender waits for its previous message on the pair
// to be taken, writes its parts and publishes seq; the receiver waits for that seq.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace {

typedef int ncclResult_t;
enum : int { ncclSuccess = 0, ncclUnhandledCudaError = 1, ncclSystemError = 2, ncclInternalError = 3,
             ncclInvalidArgument = 4, ncclInvalidUsage = 5, ncclRemoteError = 6 };
struct ncclUniqueId { char internal[128]; };
constexpr char MAGIC[8] = {'C', 'M', 'Q', 'S', 'T', 'N', 'D', 0};
constexpr int MAXR = 16, MAXP = 16;

struct Chan {
  std::atomic<uint64_t> posted, taken;
  uint32_t nparts, pad;
  uint64_t sizes[MAXP];
};
struct Hdr {
  std::atomic<uint32_t> aborted;
  uint32_t n;
  uint64_t box_bytes;
  Chan ch[MAXR * MAXR];
};

}  // namespace

struct ncclComm {
  std::string name;
  int n = 0, rank = 0;
  Hdr* h = nullptr;
  uint8_t* boxes = nullptr;
  size_t map_bytes = 0;
  ncclResult_t err = ncclSuccess;
  uint64_t seq_send[MAXR] = {}, seq_recv[MAXR] = {};
  Chan& chan(int src, int dst) { return h->ch[src * MAXR + dst]; }
  uint8_t* box(int src, int dst) { return boxes + (size_t)(src * n + dst) * h->box_bytes; }
};

namespace {

struct Op { bool send; void* ptr; size_t bytes; int peer; ncclComm* comm; hipStream_t s; };
thread_local int g_depth = 0;
thread_local std::vector<Op> g_ops;

int timeout_ms() {
  const char* e = getenv("CHANAMQ_RCCL_STANDIN_TIMEOUT_MS");
  return e && *e ? atoi(e) : 30000;
}
uint64_t box_bytes() {
  const char* e = getenv("CHANAMQ_RCCL_STANDIN_BOX_MB");
  return (uint64_t)(e && *e ? atoi(e) : 48) << 20;
}

// wait until pred() or the communicator is aborted / the deadline passes
template <class P>
ncclResult_t wait_for(ncclComm* c, P pred, const char* what, int peer) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t spin = 0; !pred(); ++spin) {
    if (c->h->aborted.load(std::memory_order_acquire)) return ncclRemoteError;
    if (spin > 2000) std::this_thread::sleep_for(std::chrono::microseconds(50));
    if ((spin & 1023) == 1023 &&
        std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms())) {
      fprintf(stderr, "rccl stand-in: rank %d timed out %s peer %d\n", c->rank, what, peer);
      return ncclRemoteError;
    }
  }
  return ncclSuccess;
}

ncclResult_t run_group(std::vector<Op>& ops) {
  if (ops.empty()) return ncclSuccess;
  ncclComm* c = ops[0].comm;
  for (auto& o : ops)
    if (o.comm != c) return ncclInvalidUsage;   // (the engine never mixes communicators)
  if (c->err) return c->err;
  std::vector<hipStream_t> ss;
  for (auto& o : ops) {
    bool seen = false;
    for (auto s : ss) seen |= s == o.s;
    if (!seen) ss.push_back(o.s);
  }
  for (auto s : ss)
    if (hipStreamSynchronize(s) != hipSuccess) return c->err = ncclUnhandledCudaError;
  // sends: per peer, the group's parts in call order into the (me -> peer) mailbox
  for (int p = 0; p < c->n; ++p) {
    std::vector<const Op*> mine;
    for (auto& o : ops)
      if (o.send && o.peer == p) mine.push_back(&o);
    if (mine.empty()) continue;
    if (mine.size() > MAXP) return c->err = ncclInvalidUsage;
    Chan& ch = c->chan(c->rank, p);
    const uint64_t seq = c->seq_send[p];
    ncclResult_t r = wait_for(c, [&] { return ch.taken.load(std::memory_order_acquire) == seq; }, "posting to", p);
    if (r) return c->err = r;
    uint64_t off = 0;
    for (size_t k = 0; k < mine.size(); ++k) {
      if (off + mine[k]->bytes > c->h->box_bytes) {
        fprintf(stderr, "rccl stand-in: rank %d -> %d: %zu bytes exceed the %llu-byte mailbox "
                "(CHANAMQ_RCCL_STANDIN_BOX_MB)\n", c->rank, p, (size_t)(off + mine[k]->bytes),
                (unsigned long long)c->h->box_bytes);
        return c->err = ncclInvalidUsage;
      }
      // (on the op's own stream, as RCCL's kernels would run: never the null stream, whose
      // hardware queue may be the one a spinning kernel of the engine holds)
      if (mine[k]->bytes && (hipMemcpyAsync(c->box(c->rank, p) + off, mine[k]->ptr, mine[k]->bytes, hipMemcpyDefault,
                                            mine[k]->s) != hipSuccess ||
                             hipStreamSynchronize(mine[k]->s) != hipSuccess))
        return c->err = ncclUnhandledCudaError;
      ch.sizes[k] = mine[k]->bytes;
      off += (mine[k]->bytes + 63) & ~63ull;
    }
    ch.nparts = (uint32_t)mine.size();
    ch.posted.store(seq + 1, std::memory_order_release);
    c->seq_send[p] = seq + 1;
  }
  // receives: per peer, the peer's group for me must match what I posted part for part
  for (int p = 0; p < c->n; ++p) {
    std::vector<const Op*> mine;
    for (auto& o : ops)
      if (!o.send && o.peer == p) mine.push_back(&o);
    if (mine.empty()) continue;
    Chan& ch = c->chan(p, c->rank);
    const uint64_t seq = c->seq_recv[p];
    ncclResult_t r = wait_for(c, [&] { return ch.posted.load(std::memory_order_acquire) == seq + 1; }, "waiting for",
                              p);
    if (r) return c->err = r;
    bool ok = ch.nparts == mine.size();
    for (size_t k = 0; ok && k < mine.size(); ++k) ok = ch.sizes[k] == mine[k]->bytes;
    if (!ok) {
      fprintf(stderr, "rccl stand-in: rank %d <- %d: send/recv mismatch: peer sent %u parts [", c->rank, p, ch.nparts);
      for (uint32_t k = 0; k < ch.nparts && k < MAXP; ++k) fprintf(stderr, " %llu", (unsigned long long)ch.sizes[k]);
      fprintf(stderr, " ], this rank posted %zu [", mine.size());
      for (auto* o : mine) fprintf(stderr, " %zu", o->bytes);
      fprintf(stderr, " ]\n");
      c->h->aborted.store(1, std::memory_order_release);   // the peers fail too: loudly
      return c->err = ncclInvalidUsage;
    }
    uint64_t off = 0;
    for (size_t k = 0; k < mine.size(); ++k) {
      if (mine[k]->bytes && (hipMemcpyAsync(mine[k]->ptr, c->box(p, c->rank) + off, mine[k]->bytes, hipMemcpyDefault,
                                            mine[k]->s) != hipSuccess ||
                             hipStreamSynchronize(mine[k]->s) != hipSuccess))
        return c->err = ncclUnhandledCudaError;
      off += (mine[k]->bytes + 63) & ~63ull;
    }
    ch.taken.store(seq + 1, std::memory_order_release);
    c->seq_recv[p] = seq + 1;
  }
  return ncclSuccess;
}

}  // namespace

extern "C" {

// marker the engine reports (so nothing measured through the stand-in is mistaken for RCCL)
int cmq_rccl_standin() { return 1; }

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  memset(id->internal, 0, sizeof id->internal);
  memcpy(id->internal, MAGIC, sizeof MAGIC);
  std::random_device rd;
  char name[64];
  snprintf(name, sizeof name, "/cmq-rccl-standin-%d-%08x%08x", (int)getpid(), rd(), rd());
  memcpy(id->internal + 8, name, strlen(name) + 1);
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm** out, int n, ncclUniqueId id, int rank) {
  if (memcmp(id.internal, MAGIC, sizeof MAGIC) != 0 || n < 1 || n > MAXR || rank < 0 || rank >= n)
    return ncclInvalidArgument;
  auto* c = new ncclComm();
  c->name = std::string(id.internal + 8);
  c->n = n;
  c->rank = rank;
  const uint64_t bb = box_bytes();
  c->map_bytes = sizeof(Hdr) + (size_t)n * n * bb;   // (sparse: only the pages a step writes)
  int fd = shm_open(c->name.c_str(), O_CREAT | O_RDWR, 0600);
  if (fd < 0) { delete c; return ncclSystemError; }
  if (ftruncate(fd, (off_t)c->map_bytes) != 0) { close(fd); delete c; return ncclSystemError; }
  void* m = mmap(nullptr, c->map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (m == MAP_FAILED) { delete c; return ncclSystemError; }
  c->h = (Hdr*)m;
  c->boxes = (uint8_t*)m + sizeof(Hdr);
  if (c->h->box_bytes == 0) { c->h->n = (uint32_t)n; c->h->box_bytes = bb; }   // (zero-filled by ftruncate)
  if (c->h->n != (uint32_t)n || c->h->box_bytes != bb) {
    munmap(m, c->map_bytes);
    delete c;
    return ncclInvalidUsage;
  }
  *out = c;
  return ncclSuccess;
}

ncclResult_t ncclGroupStart() { ++g_depth; return ncclSuccess; }

ncclResult_t ncclGroupEnd() {
  if (g_depth <= 0) return ncclInvalidUsage;
  if (--g_depth) return ncclSuccess;
  std::vector<Op> ops;
  ops.swap(g_ops);
  return run_group(ops);
}

static ncclResult_t enqueue(bool send, void* ptr, size_t bytes, int dtype, int peer, ncclComm* c, hipStream_t s) {
  if (!c || dtype != 0 || peer < 0 || peer >= c->n || peer == c->rank) return ncclInvalidArgument;
  g_ops.push_back(Op{send, ptr, bytes, peer, c, s});
  if (g_depth) return ncclSuccess;
  std::vector<Op> ops;
  ops.swap(g_ops);
  return run_group(ops);
}

ncclResult_t ncclSend(const void* buf, size_t count, int dtype, int peer, ncclComm* c, hipStream_t s) {
  return enqueue(true, (void*)buf, count, dtype, peer, c, s);
}

ncclResult_t ncclRecv(void* buf, size_t count, int dtype, int peer, ncclComm* c, hipStream_t s) {
  return enqueue(false, buf, count, dtype, peer, c, s);
}

ncclResult_t ncclCommAbort(ncclComm* c) {
  if (!c) return ncclSuccess;
  if (c->h) {
    c->h->aborted.store(1, std::memory_order_release);
    munmap(c->h, c->map_bytes);
    if (c->rank == 0) shm_unlink(c->name.c_str());
  }
  delete c;
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm* c) { return ncclCommAbort(c); }

ncclResult_t ncclCommGetAsyncError(ncclComm* c, ncclResult_t* e) {
  *e = c ? c->err : ncclInvalidArgument;
  return ncclSuccess;
}

const char* ncclGetErrorString(ncclResult_t r) {
  switch (r) {
    case ncclSuccess: return "success (stand-in)";
    case ncclInvalidArgument: return "invalid argument (stand-in)";
    case ncclInvalidUsage: return "invalid usage: send/recv mismatch or mailbox overflow (stand-in)";
    case ncclRemoteError: return "remote error: peer aborted or timed out (stand-in)";
    case ncclSystemError: return "system error: shared memory (stand-in)";
    default: return "error (stand-in)";
  }
}

}  // extern "C"

// MI355X (gfx950) AMQP 0-9-1 data plane: the broker hot path as a fixed-shape,
// hipGraph-capturable kernel pipeline.
//
//   K0 stage        carry + new TCP bytes -> contiguous per-connection work segment
//   K1 frame_scan   speculative frame-boundary scan + chain resolution (LDS), command
//                   assembly (method -> header -> bodies), control barrier, carry-out
//                   (FrameParser.scala:86-157, CommandAssembler.scala:56-130)
//   K3/K4 decode    Basic.Publish / Ack / Nack / Reject args + content-header
//                   properties (Basic.scala:36-59, BasicProperties.scala:42-96)
//   K6 route        direct (device hash), fanout (CSR), topic (int8 MFMA word-hash
//                   prefilter + exact word matcher)  (QueueMatcher.scala, ExchangeEntity.scala:287-331)
//   K13 ids         snowflake ids (IdGenerator.scala:55-83)
//   K7 enqueue      stable radix sort by queue -> per-queue HBM ring append (QueueEntity.scala:271-316)
//   K9 acks         per-channel unacked windows, ack/nack/reject (AMQChannel.scala:109-174)
//   K8/K12 dequeue  credit-limited round-robin pull with TTL skip (QueueEntity.scala:318-393)
//   K9 tags         stable sort by channel -> delivery tags
//   K5 render       Deliver / Return / confirm-Ack frames written straight into
//                   host-mapped egress memory (AMQCommand.scala:30-59)
//   K10 confirms    one coalesced Basic.Ack per channel per step (FrameStage.scala:571-596)
//   K11 refcount    body refcount + free-list / log reclamation (MessageEntity.scala:134-166)
//
// Every kernel reads its dynamic sizes from device counters, so grids are fixed by
// EngineCfg and the whole step is captured once into a hipGraph (engine.cpp).
#include "dp_state.h"

#define INVALID 0xffffffffu
#define FNV64_BASIS 0xcbf29ce484222325ULL
#define FNV64_PRIME 0x100000001b3ULL

// ============================================================================ helpers
DEV u32 lane_id() { return __lane_id(); }
DEV u64 lanemask_lt() {
  u32 l = __lane_id();
  return l ? ((~0ull) >> (64 - l)) : 0ull;
}
DEV u32 be16(const u8* p) { return (u32(p[0]) << 8) | u32(p[1]); }
DEV u32 be32(const u8* p) {
  return (u32(p[0]) << 24) | (u32(p[1]) << 16) | (u32(p[2]) << 8) | u32(p[3]);
}
DEV u64 be64(const u8* p) { return (u64(be32(p)) << 32) | u64(be32(p + 4)); }
DEV void wr16(u8* p, u32 v) { p[0] = u8(v >> 8); p[1] = u8(v); }
DEV void wr32(u8* p, u32 v) { p[0] = u8(v >> 24); p[1] = u8(v >> 16); p[2] = u8(v >> 8); p[3] = u8(v); }
DEV void wr64(u8* p, u64 v) { wr32(p, u32(v >> 32)); wr32(p + 4, u32(v)); }
DEV u32 align16(u32 x) { return (x + 15u) & ~15u; }

DEV u64 exch_hash(u32 vhost, const u8* name, u32 n) {
  u64 h = FNV64_BASIS ^ (u64(vhost) * 0x9E3779B97F4A7C15ULL);
  for (u32 i = 0; i < n; ++i) { h ^= name[i]; h *= FNV64_PRIME; }
  return h;
}
DEV u32 fnv1a32(const u8* p, u32 n) {
  u32 h = 0x811c9dc5u;
  for (u32 i = 0; i < n; ++i) { h ^= p[i]; h *= 0x01000193u; }
  return h;
}

struct __attribute__((packed, aligned(1))) U4 { u32 x, y, z, w; };

// unaligned-source, unaligned-dest byte copy by the 64 lanes of one wave (kept minimal:
// it is inlined into the store / render / pack kernels, and a batched variant with 8
// loads in flight raised their VGPR count and cost them ~20% at 1 KB messages, measured)
DEV void wave_copy(u8* dst, const u8* src, u32 n) {
  u32 lane = lane_id();
  u32 nv = n >> 4;
  for (u32 i = lane; i < nv; i += 64) {
    U4 v = *(const U4*)(src + (u64)i * 16);
    *(U4*)(dst + (u64)i * 16) = v;
  }
  for (u32 i = (nv << 4) + lane; i < n; i += 64) dst[i] = src[i];
}

// same, by the G lanes (lane = 0..G-1) of a lane group
template <u32 G>
DEV void group_copy(u8* dst, const u8* src, u32 n, u32 lane) {
  u32 nv = n >> 4;
  for (u32 i = lane; i < nv; i += G) {
    U4 v = *(const U4*)(src + (u64)i * 16);
    *(U4*)(dst + (u64)i * 16) = v;
  }
  for (u32 i = (nv << 4) + lane; i < n; i += G) dst[i] = src[i];
}

// same, by all threads of a block
DEV void block_copy(u8* dst, const u8* src, u32 n, u32 tid, u32 nt) {
  u32 nv = n >> 4;
  for (u32 i = tid; i < nv; i += nt) {
    U4 v = *(const U4*)(src + (u64)i * 16);
    *(U4*)(dst + (u64)i * 16) = v;
  }
  for (u32 i = (nv << 4) + tid; i < n; i += nt) dst[i] = src[i];
}

// Saturating reservation for counters that restart at 0 every step (control bytes,
// delivery slots, egress budget): one atomicAdd and no give-back.  The caller owns
// [cur, cur + want) and is granted its part below cap, so granted ranges never overlap
// and the total granted is exactly min(sum of requests, cap) whatever the arrival order.
// The counter itself may end above cap: every reader clamps.  (A CAS loop serialises
// ~1000 queue blocks on one L2 line — 2.9 ms per step at 1024 fan-out queues — and an
// add-then-give-back fast path lets a transient overshoot inflate other threads' bases.)
DEV u32 reserve_sat(u32* p, u32 want, u32 cap, u32* base) {
  u32 cur = want ? atomicAdd(p, want) : __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  *base = cur;
  if (cur >= cap) return 0;
  return want < cap - cur ? want : cap - cur;
}
DEV u64 reserve_sat64(u64* p, u64 want, u64 cap) {
  u64 cur = atomicAdd((unsigned long long*)p, (unsigned long long)want);
  if (cur >= cap) return 0;
  return want < cap - cur ? want : cap - cur;
}

// exact CAS reservation for counters that persist across steps and are also decremented
// (per-channel delivery windows): grant min(want, cap - *p).  Contention is per channel.
DEV u32 reserve_upto(u32* p, u32 want, u32 cap, u32* base) {
  u32 cur = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (true) {
    u32 avail = cur < cap ? cap - cur : 0;
    u32 g = want < avail ? want : avail;
    if (g == 0) { *base = cur; return 0; }
    u32 prev = atomicCAS(p, cur, cur + g);
    if (prev == cur) { *base = cur; return g; }
    cur = prev;
  }
}

// exclusive block scan (NT threads), returns this thread's offset; total via ref
template <int NT>
DEV u32 block_scan(u32 v, u32* lds, u32& total) {
  u32 lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  u32 x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    u32 y = __shfl_up(x, o, 64);
    if (lane >= (u32)o) x += y;
  }
  if (lane == 63) lds[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    u32 run = 0;
    for (int i = 0; i < NT / 64; ++i) { u32 t = lds[i]; lds[i] = run; run += t; }
    lds[NT / 64] = run;
  }
  __syncthreads();
  u32 res = lds[w] + x - v;
  total = lds[NT / 64];
  __syncthreads();
  return res;
}

DEV u64 shfl_xor64(u64 v, int m) {
  return ((u64)(u32)__shfl_xor((int)(v >> 32), m, 64) << 32) | (u32)__shfl_xor((int)(u32)v, m, 64);
}
DEV u64 shfl64(u64 v, u32 src) {
  u32 lo = __shfl((u32)v, src, 64), hi = __shfl((u32)(v >> 32), src, 64);
  return (u64(hi) << 32) | lo;
}
DEV i64 wave_sum64(i64 v) {
  u64 x = (u64)v;
  for (int o = 32; o > 0; o >>= 1) {
    u32 lo = __shfl_xor((u32)x, o, 64), hi = __shfl_xor((u32)(x >> 32), o, 64);
    x += (u64(hi) << 32) | lo;
  }
  return (i64)x;
}
// all 64 lanes must call these (wave-uniform control flow); one atomic per distinct index
DEV void wave_add_u32(u32* arr, u32 idx, u32 v, bool valid) {
  u64 pend = __ballot(valid);
  while (pend) {
    u32 leader = __ffsll((unsigned long long)pend) - 1;
    u32 b = __shfl(idx, leader, 64);
    bool mine = valid && idx == b && ((pend >> lane_id()) & 1);
    u32 x = mine ? v : 0;
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    if (lane_id() == leader) atomicAdd(&arr[b], x);
    pend &= ~__ballot(mine);
  }
}
DEV void wave_sub_u32(u32* arr, u32 idx, u32 v, bool valid) {
  u64 pend = __ballot(valid);
  while (pend) {
    u32 leader = __ffsll((unsigned long long)pend) - 1;
    u32 b = __shfl(idx, leader, 64);
    bool mine = valid && idx == b && ((pend >> lane_id()) & 1);
    u32 x = mine ? v : 0;
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    if (lane_id() == leader) atomicSub(&arr[b], x);
    pend &= ~__ballot(mine);
  }
}
DEV void wave_add_i64(i64* arr, u64 idx, i64 v, bool valid) {
  u64 pend = __ballot(valid);
  while (pend) {
    u32 leader = __ffsll((unsigned long long)pend) - 1;
    u64 b = shfl64(idx, leader);
    bool mine = valid && idx == b && ((pend >> lane_id()) & 1);
    i64 x = wave_sum64(mine ? v : 0);
    if (lane_id() == leader) atomicAdd((unsigned long long*)&arr[b], (unsigned long long)x);
    pend &= ~__ballot(mine);
  }
}
// wave-uniform reservation of `cnt` (per lane) slots from one counter: returns lane's base
DEV u32 wave_reserve(u32* ctr, bool want, u32* total_out = nullptr) {
  u64 m = __ballot(want);
  u32 n = __popcll(m);
  u32 base = 0;
  if (n) {
    u32 leader = __ffsll((unsigned long long)m) - 1;
    if (lane_id() == leader) base = atomicAdd(ctr, n);
    base = __shfl(base, leader, 64);
  }
  if (total_out) *total_out = n;
  return base + __popcll(m & lanemask_lt());
}

// a message's slot: the HBM body log, or the host spill ring for a spilled cold body
DEV const u8* msg_slot(const DS& d, u64 log_off) {
  return (log_off & SPILL_BIT) ? d.spill + ((log_off & ~SPILL_BIT) % d.spill_bytes) : d.log + (log_off % d.log_bytes);
}

// live-bytes accounting of a freed slot in the spill ring
DEV void spill_free(const DS& d, u64 log_off, u32 slot_bytes) {
  const u64 blk = ((log_off & ~SPILL_BIT) / d.log_block) % d.n_spill_blocks;
  atomicAdd((unsigned long long*)&d.spill_live[blk], (unsigned long long)(-(i64)slot_bytes));
}

// ---- message release (K11): refcount -1, free slot + table index at zero
DEV void release_msg(const DS& d, u32 msg) {
  if (msg == INVALID) return;
  i32 old = atomicSub(&d.msgs[msg].refcnt, 1);
  if (old == 1) {
    MsgEnt& m = d.msgs[msg];
    if (m.log_off & COLD_BIT) {
      atomicAdd((unsigned long long*)&d.cold_live[((m.log_off & ~COLD_BIT) >> COLD_SEG_SHIFT) % COLD_SEGS],
                (unsigned long long)(-(i64)m.slot_bytes));
    } else if (m.log_off & SPILL_BIT) {
      spill_free(d, m.log_off, m.slot_bytes);
    } else {
      u64 blk = (m.log_off / d.log_block) % d.n_log_blocks;
      atomicAdd((unsigned long long*)&d.log_live[blk], (unsigned long long)(-(i64)m.slot_bytes));
      atomicAdd((unsigned long long*)d.live_bytes, (unsigned long long)(-(i64)m.slot_bytes));
    }
    u32 slot = atomicAdd(d.msg_free_top, 1u);
    d.msg_free[slot] = msg;
    atomicAdd(&d.ctr->n_freed, 1u);
  }
}

// wave-uniform release: refcount atomics per lane, one free-list reservation and one
// live-bytes atomic per distinct log block per wave (avoids serialising on hot words)
DEV void wave_release(const DS& d, u32 msg, bool valid) {
  bool freed = false, spilled = false;
  u64 blk = 0;
  i64 sb = 0;
  if (valid && msg != INVALID) {
    i32 old = atomicSub(&d.msgs[msg].refcnt, 1);
    if (old == 1) {
      freed = true;
      const u64 lo = d.msgs[msg].log_off;
      sb = d.msgs[msg].slot_bytes;
      spilled = (lo & (SPILL_BIT | COLD_BIT)) != 0;
      if (lo & COLD_BIT)   // (rare: bodies in the cold store)
        atomicAdd((unsigned long long*)&d.cold_live[((lo & ~COLD_BIT) >> COLD_SEG_SHIFT) % COLD_SEGS],
                  (unsigned long long)(-sb));
      else if (spilled) spill_free(d, lo, (u32)sb);   // (rare: cold bodies)
      else blk = (lo / d.log_block) % d.n_log_blocks;
    }
  }
  u64 fm = __ballot(freed);
  if (!fm) return;
  u32 nf;
  u32 pos = wave_reserve(d.msg_free_top, freed, &nf);
  if (freed) d.msg_free[pos] = msg;
  i64 tot = wave_sum64(freed && !spilled ? sb : 0);
  if (lane_id() == __ffsll((unsigned long long)fm) - 1) {
    atomicAdd(&d.ctr->n_freed, nf);
    if (tot) atomicAdd((unsigned long long*)d.live_bytes, (unsigned long long)(-tot));
  }
  wave_add_i64(d.log_live, blk, -sb, freed && !spilled);
}

// ---- K13 snowflake ids: id = ms << 22 | worker << 12 | seq (IdGenerator.scala:14-34).
// The reference's generator allows 4096 ids per ms per node and waits for the next ms
// (IdGenerator.scala:55-83); one MI355X publishes ~10x that.  A GPU therefore owns
// ID_WORKERS worker ids (group g = StepIn.worker owns g*64 .. g*64+63): 2^18 ids per ms
// (262 M msgs/s), so the virtual position (ms << 18 | slot) never outruns the wall clock
// and ids stay unique across restarts (the host seeds id_next above recovered ids).
DEV u64 snowflake_id(u64 pos, u32 group) {
  const u64 ms = pos >> ID_SLOT_BITS;
  const u64 worker = (u64)(group & (1023 / ID_WORKERS)) * ID_WORKERS + ((pos >> 12) & (ID_WORKERS - 1));
  return (ms << 22) | (worker << 12) | (pos & 4095);
}

// ============================================================================ topic words
// Java String.split("\\.") semantics (QueueMatcher.scala:69-71): trailing empty
// words dropped, "" -> [""], "..." -> [].
struct Words { u32 eff; u32 count; };
DEV Words words_of(const u8* s, u32 n) {
  Words w;
  if (n == 0) { w.eff = 0; w.count = 1; return w; }
  u32 e = n;
  while (e > 0 && s[e - 1] == '.') --e;
  w.eff = e;
  if (e == 0) { w.count = 0; return w; }
  u32 c = 1;
  for (u32 i = 0; i < e; ++i) c += (s[i] == '.');
  w.count = c;
  return w;
}
DEV u32 word_len(const u8* s, u32 off, u32 eff) {
  u32 i = off;
  while (i < eff && s[i] != '.') ++i;
  return i - off;
}
DEV bool word_eq(const u8* a, u32 al, const u8* b, u32 bl) {
  if (al != bl) return false;
  for (u32 i = 0; i < al; ++i)
    if (a[i] != b[i]) return false;
  return true;
}
// exact topic match: '*' = one word, '#' = zero or more words (when hash_wild),
// greedy backtracking (glob algorithm over words). Golden: models/matcher.py words_match.
DEV bool topic_match(const u8* pat, u32 plen, const u8* key, u32 klen, bool hash_wild) {
  Words pw = words_of(pat, plen), kw = words_of(key, klen);
  u32 pend = pw.eff + 1, kend = kw.eff + 1;  // cursor == end -> exhausted
  u32 p = pw.count ? 0 : pend, k = kw.count ? 0 : kend;
  u32 sp = INVALID, sk = 0;
  while (k < kend) {
    u32 kl = word_len(key, k, kw.eff);
    if (p < pend) {
      u32 pl = word_len(pat, p, pw.eff);
      bool is_hash = hash_wild && pl == 1 && pat[p] == '#';
      bool is_star = pl == 1 && pat[p] == '*';
      if (is_hash) { p += pl + 1; sp = p; sk = k; continue; }
      if (is_star || word_eq(pat + p, pl, key + k, kl)) { p += pl + 1; k += kl + 1; continue; }
    }
    if (sp != INVALID) {
      sk += word_len(key, sk, kw.eff) + 1;
      k = sk;
      p = sp;
      continue;
    }
    return false;
  }
  while (p < pend) {
    u32 pl = word_len(pat, p, pw.eff);
    if (hash_wild && pl == 1 && pat[p] == '#') { p += pl + 1; continue; }
    return false;
  }
  return true;
}

// ============================================================================ deferred control writes
// The control plane's table writes (connection / channel / consumer state) staged while
// steps run, packed per step by the host (Engine::pack_deltas): applied by k_stage before
// the step reads anything, so no pipeline drain is needed for them.  Layout:
//   DeltaHead | DeltaRec[nrec] | u32 dirty channel slots[ndirty] (16-B padded) | data chunks
// Records never overlap (the host keeps the last write of every byte), so they are applied
// in parallel: 16-byte chunk i belongs to record r with chunk0[r] <= i < chunk0[r + 1].
struct DeltaHead { u32 nrec, ndirty, nchunk, pad; };
struct DeltaRec { u64 dst; u32 len; u32 chunk0; };
#define DELTA_REC_MAX 1024   // records per step (the host keeps the rest for later steps)
DEV void apply_deltas(const DS& d, const u8* buf, u32 tid, u32 nt, DeltaRec* lrec) {
  const DeltaHead h = *(const DeltaHead*)buf;
  const DeltaRec* recs = (const DeltaRec*)(buf + sizeof(DeltaHead));
  const u32* dirty = (const u32*)(recs + h.nrec);
  const uint4* data = (const uint4*)((const u8*)dirty + ((4u * h.ndirty + 15u) & ~15u));
  for (u32 r = tid; r < h.nrec; r += nt) lrec[r] = recs[r];
  __syncthreads();
  for (u32 i = tid; i < h.nchunk; i += nt) {
    u32 lo = 0, hi = h.nrec;   // last record with chunk0 <= i
    while (hi - lo > 1) {
      const u32 mid = (lo + hi) >> 1;
      if (lrec[mid].chunk0 <= i) lo = mid; else hi = mid;
    }
    const DeltaRec r = lrec[lo];
    const u32 off = (i - r.chunk0) * 16u;
    const u32 n = r.len - off < 16u ? r.len - off : 16u;
    const uint4 v = data[i];
    u8* dst = (u8*)(uintptr_t)(r.dst + off);
    const u32 w[4] = {v.x, v.y, v.z, v.w};
    if (((uintptr_t)dst & 3) == 0 && (n & 3) == 0) {
      for (u32 k = 0; k < n / 4; ++k) ((u32*)dst)[k] = w[k];
    } else {
      for (u32 k = 0; k < n; ++k) dst[k] = (u8)(w[k >> 2] >> (8 * (k & 3)));
    }
  }
  __syncthreads();
  // closing channels: on the dirty list (k_chan_advance requeues their unacked deliveries)
  for (u32 k = tid; k < h.ndirty; k += nt) {
    const u32 ch = dirty[k];
    if (atomicExch(&d.ch_dirty[ch], 1u) == 0) d.dirty_list[atomicAdd(d.n_dirty, 1u)] = ch;
  }
  __threadfence();   // (rare: steps with control writes) every later read of the block sees them
  __syncthreads();
}
// between steps (the control plane holds the engine): the staged writes now
__global__ __launch_bounds__(1024) void k_apply_deltas(DS d, const u8* buf) {
  __shared__ DeltaRec lrec[DELTA_REC_MAX];
  apply_deltas(d, buf, threadIdx.x, 1024, lrec);
}

// ============================================================================ K0' ingress wait
// the step's ingress payload copy, queued by the host on an SDMA engine through HSA (Engine
// h2d_hsa): waited for here, on the device, between k_stage and the frame scan.  No marker
// on a HIP stream and no cross-queue barrier sits between two steps' copies, so they run back
// to back on their engine (12.7 MB each: 237.7 us per copy this way vs 262 us with
// hipMemcpyAsync + event + stream wait, bench/micro/h2d_chain_probe.hip, profiles/r6_z).
// The SDMA engine writes HBM behind the L2s: every block (16 of them, two per XCD) ends with
// a system-scope acquire, dropping its XCD's stale lines before any kernel reads the slot.
// Bounded: a copy that never completes lets the step run on and the host's check of the
// signal at collection (Engine::wait_results) reports it
__global__ __launch_bounds__(64) void k_h2d_wait(DS d) {
  const u64 sig = d.in->h2d_sig, sig2 = d.in->h2d_sig2;   // (sig2: a payload split over two engines)
  if (!sig) return;
  const u32 lim = d.in->h2d_polls ? d.in->h2d_polls : (1u << 24);
  if (threadIdx.x == 0)
    for (u32 it = 0; it < lim; ++it) {
      if (__hip_atomic_load((const i64*)sig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0 &&
          (!sig2 || __hip_atomic_load((const i64*)sig2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0))
        break;
      __builtin_amdgcn_s_sleep(4);
    }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

// ============================================================================ K0 step init
// one block: resets the step counters and lays the step's segments out in the work buffer
// (segment k at the prefix of the 16-aligned sizes carry + new bytes + 32 of the segments
// before it).  The copy itself is done by k_frame_scan's block for the segment, which
// stages the bytes through its LDS anyway (was: a grid-wide copy kernel, 12 us per 16.7 MB
// step, whose output the frame scan then read back)
__global__ __launch_bounds__(1024) void k_stage(DS d) {
  __shared__ u32 lds[1024 / 64 + 1];
  __shared__ StepIn s_in;
  __shared__ DeltaRec lrec[DELTA_REC_MAX];
  const u32 tid = threadIdx.x;
  // the step's descriptors from the host's mapped staging (one PCIe round), written to
  // their device copies for every later kernel of the step
  if (tid == 0) {
    s_in = *d.in_h;
    *d.in = s_in;
  }
  __syncthreads();
  if (s_in.delta_bytes) apply_deltas(d, d.delta_h, tid, 1024, lrec);   // control writes first
  const u32 nseg = s_in.nseg;
  {
    u32* c = (u32*)d.ctr;
    for (u32 k = tid; k < sizeof(Counters) / 4; k += 1024)
      if (k * 4 < offsetof(Counters, log_head)) c[k] = 0;
    if (tid == 0) {   // (per-parity scratch only: the link-ack counts and the id floor are
                      // reset by k_marks, in the step's routing half)
      d.ctr->n_grow = 0; d.tot[TS_NMOVE] = 0; d.tot[TS_NDEFER] = 0; d.tot[TS_TTL_BUDGET] = 0;
      d.tot[TS_NDGET] = 0;
      d.tot[TS_SPILL_USED] = 0;
      d.ctr->spill_moved = 0;
      d.ctr->n_ref = 0; d.ctr->gath_off = 0; d.ctr->ref_bytes = 0;
      *d.egress_budget = 0;
    }
    // connections whose control command the host has answered resume with this step (the
    // frame scan, the only reader and writer of the flag, runs after this kernel)
    const u32 nunp = s_in.nunp;
    for (u32 k = tid; k < nunp; k += 1024) {
      const u32 c = d.unpause_req[k];
      if (c < d.c_max) d.conn_paused[c] = 0;
    }
  }
  u32 total = 0;
  u32 cl0 = 0, len0 = 0;   // this thread's first segment (the usual step has <= 1024): the
                           // layout pass below reuses it instead of a second PCIe read
  for (u32 k = tid; k < nseg; k += 1024) {
    const SegIn sg = d.segs_h[k];
    ((SegIn*)d.segs)[k] = sg;
    const u32 cl = d.carry_len[sg.conn];
    if (k == tid) { cl0 = cl; len0 = sg.len; }
    total += align16(cl + sg.len + 32);
  }
  u32 all_t;
  block_scan<1024>(total, lds, all_t);
  if (tid == 0) d.tot[15] = all_t;  // work bytes used
  if (all_t > d.work_cap) return;   // host sizes steps so this never triggers
  u32 run = 0;
  for (u32 b0 = 0; b0 < nseg; b0 += 1024) {
    const u32 k = b0 + tid;
    u32 cl = 0, len = 0, v = 0;
    if (k < nseg) {
      if (b0 == 0) {
        cl = cl0;
        len = len0;
      } else {
        const SegIn sg = d.segs_h[k];
        cl = d.carry_len[sg.conn];
        len = sg.len;
      }
      v = align16(cl + len + 32);
    }
    u32 all;
    __syncthreads();   // lds of the previous scan
    const u32 o = block_scan<1024>(v, lds, all);
    if (k < nseg) { d.seg_total[k] = cl + len; d.seg_start[k] = run + o; }
    run += all;
  }
}

// ============================================================================ K1 frame scan
struct FInfo { u32 type, ch, size; bool complete, valid_hdr; };

DEV FInfo frame_at(const u8* b, u32 p, u32 L, u32 fmax) {
  FInfo f;
  f.complete = false;
  f.valid_hdr = false;
  f.type = 0; f.ch = 0; f.size = 0;
  if (p + 7 > L) return f;  // partial header
  f.type = b[p];
  f.ch = be16(b + p + 1);
  f.size = be32(b + p + 3);
  bool tok = f.type == 1 || f.type == 2 || f.type == 3 || f.type == 8;
  bool sok = fmax == 0 || f.size + 8 <= fmax;
  f.valid_hdr = tok && sok;
  if (f.valid_hdr && (u64)p + 8 + f.size <= L) f.complete = (b[p + 7 + f.size] == 0xCE);
  return f;
}

DEV i32 chan_lookup(const DS& d, u32 conn, u32 ch) {
  const u32* m = d.chmap + (u64)conn * d.chmap_size;
  u32 mask = d.chmap_size - 1;
  u32 h = (ch * 0x9E3779B1u) >> 7;
  for (u32 i = 0; i < d.chmap_size; ++i) {
    u32 e = m[(h + i) & mask];
    if (e == 0) return -1;
    if ((e >> 16) == ch && (e & 0x8000u)) return (i32)(conn * d.chpc + (e & 0x7fffu));
  }
  return -1;
}

// candidate screen: one u16 mask per 16 work bytes; bit j set when byte j looks like a
// frame header (type 1/2/3/8, size within the broker frame-max).  Reads 32 bytes (the
// header of a frame starting at byte 15 ends in the next word); segments are padded
// by >= 32 bytes in the work buffer
// SWAR: 0x80 in every byte of v that is zero (exact per byte: no borrow between bytes)
DEV u32 zero_bytes(u32 v) { return ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v | 0x7F7F7F7Fu); }
// bits 0..3 = bytes 0..3 of v hold a frame type (1, 2, 3 or 8); the multiply gathers the
// four 0x80 flags (bits 0, 8, 16, 24 after the shift) into bits 21..24 without carries
DEV u32 type_nibble(u32 v) {
  const u32 h = (zero_bytes(v & 0xFCFCFCFCu) & ~zero_bytes(v)) | zero_bytes(v ^ 0x08080808u);
  return (((h >> 7) * 0x00204081u) >> 21) & 0xFu;
}
DEV u32 cand_bits(uint4 A, uint4 B, u32 fm) {
  const u32 w[6] = {A.x, A.y, A.z, A.w, B.x, B.y};
  u32 m = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    u32 h = type_nibble(w[i]);
    // the rare type hits: big-endian size from bytes k+3..k+6 of the 4i-byte window
    while (h) {
      const u32 k = __ffs(h) - 1;
      h &= h - 1;
      const u32 v = k == 0 ? __builtin_amdgcn_alignbyte(w[i + 1], w[i], 3)
                           : __builtin_amdgcn_alignbyte(w[i + 2], w[i + 1], k - 1);
      const u32 sz = __builtin_bswap32(v);
      if (fm == 0 || sz <= fm - 8) m |= 1u << (4 * i + k);
    }
  }
  return m;
}
DEV u32 cand_word(const u8* w16, u32 fm) {
  const uint4* q = (const uint4*)w16;
  return cand_bits(q[0], q[1], fm);
}

#define FS_MARK(k) \
  do { if (tid == 0 && d.dbg) d.dbg[(u64)s * 16 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
constexpr u32 FS_AM_MAX = 8192;  // 128 KB segment; 16 KB of LDS
// Segments up to FS_STAGE bytes (the screen's 32-byte read-ahead included) are copied
// into LDS by the screen pass itself, and every later phase reads the segment's bytes
// from LDS instead of HBM (frame headers, method ids, body sizes, control bytes: ~15
// dependent global round trips per segment before).  The block's LDS is one pool carved
// per segment: staged segments hold up to FS_CAND_STAGED candidates next to the 72 KB
// stage, other segments CAND_MAX candidates (a 128 KB segment of 1-byte messages)
constexpr u32 FS_STAGE = 72u << 10;
constexpr u32 FS_CAND_STAGED = 6144;
// candidate arrays: wend + cpos (u32), chain / screen mask (u16), csucc (i16), claim (u8)
constexpr u32 fs_cand_bytes(u32 cmax, u32 amw) { return cmax * 4 * 2 + (cmax > amw ? cmax : amw) * 2 + cmax * 2 + cmax; }
constexpr u32 FS_POOL_STAGED = FS_STAGE + fs_cand_bytes(FS_CAND_STAGED, FS_STAGE / 16);
constexpr u32 FS_POOL_FULL = fs_cand_bytes(CAND_MAX, FS_AM_MAX);
constexpr u32 FS_POOL = ((FS_POOL_STAGED > FS_POOL_FULL ? FS_POOL_STAGED : FS_POOL_FULL) + 15) & ~15u;
static_assert(FS_POOL <= 156u << 10, "k_frame_scan LDS pool");
// one block of FS_NT threads per segment: 16 waves (4 per SIMD) hide the screen's
// dependent integer chains, which one wave per SIMD could not
#define FS_NT 1024
// a content publish whose whole command (method + header + body frames) cannot fit the
// connection's carry: the host assembles it (FE_CTRL of its method + header frames; the
// body is read on the host and enqueued as an MF_HOSTPUB record)
DEV bool big_publish(const DS& d, u32 msize, u32 hsize, u64 bsz, u32 fmax) {
  const u64 fb = fmax > 8 ? fmax - 8 : 0;
  const u64 nb = bsz == 0 ? 0 : (fb ? (bsz + fb - 1) / fb : 1);
  return (u64)msize + 8 + hsize + 8 + bsz + 8 * nb > d.carry_cap;
}

// bytes [sh, sh + 16) of the 32 bytes a:b (sh 0..15): a two-level word barrel shift (by 2
// words, then 1 -- named registers and selects: an indexed word array here was lowered to
// a scratch-memory table, 48 bytes per lane), then four dword funnel shifts
DEV uint4 shift_pair(uint4 a, uint4 b, u32 sh) {
  const u32 q = sh >> 2, r = sh & 3;
  const bool q2 = (q & 2) != 0, q1 = (q & 1) != 0;
  const u32 s0 = q2 ? a.z : a.x, s1 = q2 ? a.w : a.y, s2 = q2 ? b.x : a.z;
  const u32 s3 = q2 ? b.y : a.w, s4 = q2 ? b.z : b.x, s5 = q2 ? b.w : b.y;
  const u32 w0 = q1 ? s1 : s0, w1 = q1 ? s2 : s1, w2 = q1 ? s3 : s2, w3 = q1 ? s4 : s3, w4 = q1 ? s5 : s4;
  if (!r) return make_uint4(w0, w1, w2, w3);
  return make_uint4(__builtin_amdgcn_alignbyte(w1, w0, r), __builtin_amdgcn_alignbyte(w2, w1, r),
                    __builtin_amdgcn_alignbyte(w3, w2, r), __builtin_amdgcn_alignbyte(w4, w3, r));
}
// word c (bytes [16c, 16c + 16)) of a segment = the connection's carry (cl bytes, C
// 16-aligned) then its new ingress bytes (N 16-aligned; reading up to 32 bytes past them
// stays inside the ingress slot's slack); bytes past the segment are don't-care
DEV uint4 seg_word(const u8* C, u32 cl, const u8* N, u32 c) {
  const u32 b0 = c * 16;
  if (b0 + 16 <= cl) return *(const uint4*)(C + b0);
  if (b0 >= cl) {
    const u32 o = b0 - cl, k = o >> 4, sh = o & 15;
    const uint4 a = ((const uint4*)N)[k];
    return sh ? shift_pair(a, ((const uint4*)N)[k + 1], sh) : a;
  }
  u32 v[4] = {0, 0, 0, 0};   // the word holding the carry's end and the new bytes' start
#pragma unroll
  for (u32 j = 0; j < 16; ++j) {
    const u32 i = b0 + j;
    const u32 x = i < cl ? C[i] : N[i - cl];
    v[j >> 2] |= x << (8 * (j & 3));
  }
  return make_uint4(v[0], v[1], v[2], v[3]);
}

// Basic.Get the step can serve itself: a named queue of the connection's vhost (the default
// exchange's direct binding of that name), owned by this rank, not another connection's
// exclusive queue.  An empty name (the channel's last declared queue) and every error case
// go to the host.  Method args at b + p + 7: class, method, ticket, queue shortstr, bits.
DEV bool dget_resolve(const DS& d, u32 conn, const u8* b, u32 p, u32 size, u32& q, u32& noack) {
  if (size < 8) return false;
  const u32 a = p + 7 + 6, n = b[a], end = p + 7 + size;
  if (n == 0 || a + 1 + n + 1 > end) return false;
  const u8* name = b + a + 1;
  const u32 vh = d.conn_vhost[conn];
  const u64 hk = exch_hash(vh, name, 0);   // the vhost's default exchange ("")
  i32 xs = -1;
  for (u32 j = 0; j <= d.xhash_mask; ++j) {
    const u32 slot = (u32)(hk + j) & d.xhash_mask;
    const i32 v = d.x_hval[slot];
    if (v < 0) break;
    if (d.x_hkey[slot] == hk) { xs = v; break; }
  }
  if (xs < 0 || d.x_type[xs] != EX_DIRECT) return false;
  const u64 k = fnv1a64_dev(name, n) ^ (u64(xs) * 0x9E3779B97F4A7C15ULL);
  for (u32 j = 0; j <= d.dhash_mask; ++j) {
    const u32 s = (u32)(k + j) & d.dhash_mask;
    const i32 ex = d.d_exch[s];
    if (ex < 0) return false;
    if (ex == xs && d.d_key[s] == k && word_eq(d.kpool + d.d_kb_off[s], d.d_kb_len[s], name, n)) {
      if (d.d_q_n[s] != 1) return false;
      const u32 qq = d.d_q[d.d_q_off[s]];
      const u32 ex_owner = d.q_excl[qq];
      if (!d.q_active[qq] || d.q_owner[qq] != d.my_rank || (ex_owner && ex_owner != conn + 1)) return false;
      q = qq;
      noack = b[a + 1 + n] & 1u;
      return true;
    }
  }
  return false;
}

DEV void frame_scan_seg(const DS& d, const u32 s) {
  __shared__ uint4 fs_pool[FS_POOL / 16];
  __shared__ u32 sc[FS_NT / 64 + 1];
  __shared__ u32 sh_m, sh_over, sh_ok, sh_nf, sh_stop, sh_brk;
  __shared__ u32 sh_cmd_base, sh_frag_base, sh_ncmd;
  __shared__ u32 sh_get0, sh_gch, sh_gq, sh_gna, sh_gbase;   // Basic.Get: the segment's first, its key
  __shared__ u32 sh_split;   // split mode: bytes [0, sh_split) are in the work buffer

  const u32 tid = threadIdx.x;
  const u32 conn = d.segs[s].conn;
  const u32 L = d.seg_total[s];
  const u32 seg_len = d.segs[s].len, seg_cl = L - seg_len, src = d.segs[s].src;
  // the step's new bytes are read where their H2D put them: the ingress slots follow the
  // work buffers in one allocation, so a u32 offset from d.work reaches them, and every
  // later reader (decode, route-store, returns, gets) takes a frame's bytes from there.  A
  // segment with no carry is scanned in place (nothing goes to the work buffer); one with a
  // carry is staged in LDS by the screen and only its head -- the carry and the frame that
  // straddles into the new bytes -- is written to the work buffer (split mode, OFF below):
  // the work copy of the step's bytes is gone.  Single GPU (sharded steps read imports
  // beside the work buffer).
  const u64 ing_rel = (u64)d.in->ingress - (u64)d.work;
  const bool ing_ok = d.scan_inplace && d.world == 1 && (u64)d.in->ingress > (u64)d.work && ing_rel + src + L + 64 < (1ull << 32) &&
                      d.tot[15] <= d.work_cap;
  const bool inplace = ing_ok && seg_cl == 0 && L > 0;
  const u32 wbase = inplace ? (u32)(ing_rel + src) : d.seg_start[s];
  const u8* const bg = d.work + wbase;   // the segment in HBM: the work buffer or its ingress slot
  const u8* b = bg;                      // switched to the LDS stage after the screen
  // the pool for this segment: [stage] wend cpos chain/amask csucc claim
  const u32 nm16 = (L + 15) >> 4;
  const bool staged = nm16 * 16 + 32 <= FS_STAGE;
  const u32 cmax = staged ? FS_CAND_STAGED : CAND_MAX;
  u8* const pool = (u8*)fs_pool;
  uint4* const fs_stage = fs_pool;
  // per accepted candidate: its frame end | complete << 31 (phase b reuses it instead of
  // re-reading the header); ~0u = recompute
  u32* const wend = (u32*)(pool + (staged ? FS_STAGE : 0u));
  u32* const cpos = wend + cmax;
  // chain (first written in phase c) aliases amask (used only in phase a, which ends on a
  // __syncthreads)
  u16* const chain_am = (u16*)(cpos + cmax);
  u16* const chain = chain_am;
  u16* const amask = chain_am;
  int16_t* const csucc = (int16_t*)(chain_am + (staged ? FS_CAND_STAGED : (CAND_MAX > FS_AM_MAX ? CAND_MAX : FS_AM_MAX)));
  u8* const claim = (u8*)(csucc + cmax);
  const u32 fmax = d.conn_frame_max[conn];
  FS_MARK(15);
  const u8* const seg_C = d.carry + (u64)conn * d.carry_cap;
  const u8* const seg_N = (const u8*)d.in->ingress + d.segs[s].src;
  // the common segment is copied into the work buffer by the screen pass itself: one read
  // of the sources, the work copy, the LDS stage and the candidate mask from the same
  // registers (was: a copy pass, then the screen re-reading the copy)
  const bool fit = d.tot[15] <= d.work_cap;
  const bool fuse = fit && !inplace && L > 0 && ((L + 15) >> 4) <= FS_AM_MAX && !d.conn_paused[conn];
  const bool split = fuse && staged && ing_ok;   // (the screen then leaves the work buffer alone)
  if (fit && !fuse && !inplace) {
    // the segment into the work buffer (fused k_stage copy): the connection's carry, then
    // its new ingress bytes.  k_decode / k_route_store read publishes from there
    u8* const dst = d.work + wbase;
    if (seg_cl) block_copy(dst, seg_C, seg_cl, tid, FS_NT);
    if (seg_len) block_copy(dst + seg_cl, seg_N, seg_len, tid, FS_NT);
  }
  __threadfence_block();
  __syncthreads();
  SegOut so;
  so.conn = conn; so.status = 0; so.consumed = 0; so.carry = L; so.ncmds = 0; so.err_off = 0;
  so.pad[0] = so.pad[1] = 0;

  if (d.conn_paused[conn]) {
    // hold everything; write carry back (k_stage already appended new bytes)
    if (L > d.carry_cap) { so.status = SS_TOO_LARGE; so.carry = 0; }
    else block_copy(d.carry + (u64)conn * d.carry_cap, b, L, tid, FS_NT);
    if (tid == 0) {
      so.status |= SS_PAUSED;
      d.carry_len[conn] = so.carry;
      d.seg_out[s] = so;
      d.seg_cmd_base[s] = INVALID;
      d.seg_npub[s] = 0;
      d.seg_nack[s] = 0;
    }
    return;
  }
  if (L == 0) {
    if (tid == 0) {
      d.carry_len[conn] = 0; d.seg_out[s] = so; d.seg_cmd_base[s] = INVALID; d.seg_npub[s] = 0; d.seg_nack[s] = 0;
    }
    return;
  }
  if (tid == 0) { sh_m = 0; sh_over = 0; }
  __syncthreads();

  FS_MARK(0);
  // ---- (a) candidates: screen the segment (one mask bit per byte that looks like a frame
  // header), validate them against the connection's frame-max / end marker, append the
  // trailing positions that can only hold a partial header.  cpos = accepted positions in
  // order; wend[i] = candidate i's frame end | complete << 31 (~0u: phase b re-reads it)
  {
    const u32 nm = (L + 15) >> 4;
    const u32 per = (nm + FS_NT - 1) / FS_NT;
    const u32 c0 = tid * per;
    const u32 c1 = c0 + per < nm ? c0 + per : nm;
    const u32 lim = L >= 7 ? L - 6 : 0;   // full-header positions are p < lim
    const bool use_am = nm <= FS_AM_MAX;
    const u32 fmg = d.frame_max_global;
    if (use_am) {   // candidate screen of the segment into LDS (fused k_cand), coalesced reads
      const uint4* W = (const uint4*)bg;   // 16-aligned; >= 32 bytes of padding after the segment
      uint4* const WD = (uint4*)(d.work + wbase);
      // every word is read from memory once: a lane's next word (the screen looks 16 bytes
      // ahead) is its neighbour lane's word, the wave's last lane reads it itself -- all 256
      // segment blocks screen at once, so the double read made this phase HBM-bound
      const u32 ln = lane_id();
      // (wave-uniform trip count: every lane of a wave takes part in the shuffles)
      for (u32 cb = tid - ln; cb < nm; cb += FS_NT * 4) {
        const u32 cc = cb + ln;
        uint4 x[4], y[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {   // every load of the batch in flight before any use
          const u32 c = cc + k * FS_NT;   // (c == nm: the word after the segment, read as slack)
          x[k] = make_uint4(0, 0, 0, 0);
          y[k] = make_uint4(0, 0, 0, 0);
          if (c <= nm) x[k] = fuse ? seg_word(seg_C, seg_cl, seg_N, c) : W[c];
          if (ln == 63 && c < nm) y[k] = fuse ? seg_word(seg_C, seg_cl, seg_N, c + 1) : W[c + 1];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint4 nx = make_uint4(__shfl_down(x[k].x, 1), __shfl_down(x[k].y, 1), __shfl_down(x[k].z, 1),
                                      __shfl_down(x[k].w, 1));
          if (ln != 63) y[k] = nx;
          const u32 c = cc + k * FS_NT;
          if (c < nm) {
            amask[c] = (u16)cand_bits(x[k], y[k], fmg);
            if (staged) fs_stage[c] = x[k];
            if (fuse && !split) WD[c] = x[k];
          }
        }
      }
      if (fuse && !staged) __threadfence_block();   // the later phases read the work copy
      if (staged && tid < 2) fs_stage[nm + tid] = make_uint4(0, 0, 0, 0);   // the screen's read-ahead
      __syncthreads();
      if (staged) b = (const u8*)fs_stage;
    }
    FS_MARK(12);
    // raw candidates per thread (its words are contiguous: the scan keeps position order)
    u32 rc = 0;
    if (use_am)
      for (u32 c = c0; c < c1; ++c) {
        u32 mk = amask[c];
        if (c * 16 + 16 > lim) mk &= lim > c * 16 ? (1u << (lim - c * 16)) - 1u : 0u;
        rc += __popc(mk);
      }
    u32 rtot;
    u32 roff = block_scan<FS_NT>(rc, sc, rtot);
    FS_MARK(13);
    u32 tot = 0;
    if (use_am && rtot <= cmax) {
      // every raw candidate validated in parallel (one thread each), then compacted in
      // place chunk by chunk: accepted entries only move left, after the chunk was read
      for (u32 c = c0; c < c1; ++c) {
        u32 mk = amask[c];
        while (mk) {
          const u32 j = __ffs(mk) - 1;
          mk &= mk - 1;
          const u32 p = c * 16 + j;
          if (p >= lim) break;
          cpos[roff++] = p;
        }
      }
      __syncthreads();
      FS_MARK(14);
      for (u32 k0 = 0; k0 < rtot; k0 += FS_NT) {
        const u32 i = k0 + tid;
        bool ok = false;
        u32 p = 0, we = ~0u;
        if (i < rtot) {
          p = cpos[i];
          const FInfo f = frame_at(b, p, L, fmax);
          ok = f.valid_hdr && (f.complete || (u64)p + 8 + f.size > L);
          const u64 e64 = (u64)p + 8 + f.size;
          we = e64 < 0x7fffffffull ? ((f.complete ? 0x80000000u : 0u) | (u32)e64) : ~0u;
        }
        u32 all;
        const u32 o = block_scan<FS_NT>(ok ? 1u : 0u, sc, all);
        if (ok) { cpos[tot + o] = p; wend[tot + o] = we; }
        tot += all;
      }
    } else {
      // very long segment (no LDS mask) or more raw candidates than cmax: each
      // thread validates its own words, twice (count, then emit)
      u32 cnt = 0;
      for (u32 c = c0; c < c1; ++c) {
        u32 mk = use_am ? (u32)amask[c] : cand_word(b + c * 16, fmg);
        u32 acc = 0;
        while (mk) {
          u32 j = __ffs(mk) - 1;
          mk &= mk - 1;
          u32 p = c * 16 + j;
          if (p >= lim) break;
          FInfo f = frame_at(b, p, L, fmax);
          if (f.valid_hdr && (f.complete || (u64)p + 8 + f.size > L)) { ++cnt; acc |= 1u << j; }
        }
        if (use_am) amask[c] = (u16)acc;
      }
      u32 off = block_scan<FS_NT>(cnt, sc, tot);
      for (u32 c = c0; c < c1; ++c) {
        u32 mk = use_am ? (u32)amask[c] : cand_word(b + c * 16, fmg);
        while (mk) {
          u32 j = __ffs(mk) - 1;
          mk &= mk - 1;
          u32 p = c * 16 + j;
          if (p >= lim) break;
          bool acc = use_am;
          if (!use_am) {
            FInfo f = frame_at(b, p, L, fmax);
            acc = f.valid_hdr && (f.complete || (u64)p + 8 + f.size > L);
          }
          if (acc) {
            if (off < cmax) { cpos[off] = p; wend[off] = ~0u; }
            ++off;
          }
        }
      }
    }
    __syncthreads();
    if (tid == 0) {
      u32 nmc = tot;
      for (u32 p = lim; p < L; ++p) {
        if (nmc < cmax) { cpos[nmc] = p; wend[nmc] = ~0u; }
        ++nmc;
      }
      if (nmc > cmax) { sh_over = 1; nmc = cmax; }
      sh_m = nmc;
    }
    __syncthreads();
  }
  FS_MARK(1);
  const u32 m = sh_m;
  const bool over = sh_over != 0;

  // ---- (b) successor of every candidate (-1 exact end, -2 partial/unknown, -3 broken)
  for (u32 i = tid; i < m; i += FS_NT) {
    u32 p = cpos[i];
    bool complete;
    u32 e;
    const u32 we = wend[i];
    if (we != ~0u) {
      complete = (we >> 31) != 0;
      e = we & 0x7fffffffu;
    } else {
      FInfo f = frame_at(b, p, L, fmax);
      complete = f.complete;
      e = p + 8 + f.size;
    }
    i32 sx;
    if (!complete) sx = -2;
    else {
      if (e == L) sx = -1;
      else {
        u32 lo = i + 1, hi = m;  // successor lies strictly after i
        while (lo < hi) { u32 mid = (lo + hi) >> 1; if (cpos[mid] < e) lo = mid + 1; else hi = mid; }
        if (lo < m && cpos[lo] == e) sx = (i32)lo;
        else sx = (over && e > cpos[m - 1]) ? -2 : -3;
      }
    }
    csucc[i] = (int16_t)sx;
  }
  FS_MARK(2);
  // ---- (c) chain.  A failure is a candidate whose successor is not the next candidate;
  // between failures the chain runs through consecutive candidates.  The failures are
  // compacted in order (into wend, dead after (b)), then one thread walks failure to
  // failure -- one step per jump over false candidates (e.g. timestamp bytes inside a
  // header that look like a frame running past the segment end), not one per frame --
  // recording runs, which all threads expand into chain[].  A single run starting at 0
  // is the implicit chain (frame f = candidate f)
  constexpr u32 FS_RUNS = 1024;            // run records at the top of wend
  const u32 FS_FAIL_MAX = cmax - 2 * FS_RUNS;
  __syncthreads();   // csucc / wend of (b) complete
  FS_MARK(9);
  {
    const u32 per = (m + FS_NT - 1) / FS_NT;
    const u32 i0 = tid * per < m ? tid * per : m;
    const u32 i1 = i0 + per < m ? i0 + per : m;
    u32 nfl = 0;
    for (u32 i = i0; i < i1; ++i) nfl += csucc[i] != (i32)(i + 1);
    u32 tfl;
    u32 o = block_scan<FS_NT>(nfl, sc, tfl);
    for (u32 i = i0; i < i1; ++i)
      if (csucc[i] != (i32)(i + 1) && o < FS_FAIL_MAX) wend[o++] = i;
    __syncthreads();
    // per failure x (candidate F[x] = wend[x]) with a successor: the first failure at or
    // after that successor, in parallel (binary search over F); kept in chain[] (free
    // until the expansion below), 0xFFFF = the chain ends at this failure
    if (tfl <= FS_FAIL_MAX)
      for (u32 x = tid; x < tfl; x += FS_NT) {
        const i32 sx = csucc[wend[x]];
        u32 nx = 0xFFFFu;
        if (sx >= 0) {
          u32 lo = x + 1, hi = tfl;   // successors lie after the failure
          while (lo < hi) { u32 mid = (lo + hi) >> 1; if (wend[mid] < (u32)sx) lo = mid + 1; else hi = mid; }
          nx = lo;   // < tfl: the last candidate is a failure
        }
        chain[x] = (u16)nx;
      }
    __syncthreads();
    FS_MARK(10);
    if (tid == 0) {
      u32 nf = 0, brk = 0, nrun = 0;
      if (m == 0 || cpos[0] != 0) {
        brk = 1;  // first bytes are not a frame header
      } else if (tfl <= FS_FAIL_MAX) {
        // failure to failure: the run [i, F[x]], then the run from F[x]'s successor
        u32 i = 0, x = 0;
        while (true) {
          const u32 k = wend[x], nx = chain[x];
          if (nrun < FS_RUNS) { wend[FS_FAIL_MAX + 2 * nrun] = i; wend[FS_FAIL_MAX + 2 * nrun + 1] = nf; }
          ++nrun;
          nf += k - i + 1;
          if (nx == 0xFFFFu) { brk = csucc[k] == -3; break; }
          i = (u32)csucc[k];
          x = nx;
        }
      }
      if (m != 0 && cpos[0] == 0 && (tfl > FS_FAIL_MAX || nrun > FS_RUNS)) {
        nf = 0; brk = 0; nrun = FS_RUNS + 1;   // pathological: serial walk
        i32 i = 0;
        while (true) {
          chain[nf++] = (u16)i;
          i32 sx = csucc[i];
          if (sx >= 0) { i = sx; continue; }
          if (sx == -3) brk = 1;
          break;
        }
      }
      sh_nf = nf;
      sh_brk = brk;
      sh_ok = nrun;
    }
    __syncthreads();
    FS_MARK(11);
    const u32 nrun = sh_ok;
    if (nrun > 1 && nrun <= FS_RUNS) {
      for (u32 r = tid; r < nrun; r += FS_NT) {
        const u32 ci = wend[FS_FAIL_MAX + 2 * r], f0 = wend[FS_FAIL_MAX + 2 * r + 1];
        const u32 f1 = r + 1 < nrun ? wend[FS_FAIL_MAX + 2 * r + 3] : sh_nf;
        for (u32 f = f0; f < f1; ++f) chain[f] = (u16)(ci + (f - f0));
      }
    }
    __syncthreads();
  }
  FS_MARK(3);
  const u32 nf = sh_nf;
  const bool implicit_chain = sh_ok == 1;
#define CPOS(f) (cpos[implicit_chain ? (f) : chain[f]])

  // ---- (d) commands: each method frame walks its content frames
  for (u32 f = tid; f < nf; f += FS_NT) claim[f] = 0;
  if (tid == 0) { sh_stop = (nf << 3) | 7; sh_get0 = INVALID; }  // (frame << 3) | reason; 7 = none
  __syncthreads();
  // stop reasons: 0 = after control, 1 = incomplete, 2 = unexpected frame, 3 = frame error,
  // 4 = before a command that may not follow the segment's Basic.Gets in one step
  for (u32 f = tid; f < nf; f += FS_NT) {
    u32 p = CPOS(f);
    FInfo fi = frame_at(b, p, L, fmax);
    if (!fi.complete) {
      if (fi.type == 1 || fi.type == 8 || !fi.valid_hdr) atomicMin(&sh_stop, (f << 3) | 1);
      continue;
    }
    if (fi.type == 8) { claim[f] = 1; continue; }
    if (fi.type != 1) continue;
    claim[f] = 1;
    if (fi.size < 4) { atomicMin(&sh_stop, (f << 3) | 3); continue; }
    u32 cls = be16(b + p + 7), mid = be16(b + p + 9);
    bool content = (cls == 60 && mid == 40);
    bool data = (cls == 60 && (mid == 40 || mid == 80 || mid == 90 || mid == 120)) && fi.ch != 0 &&
                chan_lookup(d, conn, fi.ch) >= 0;
    if (cls == 60 && mid == 70 && fi.ch != 0 && chan_lookup(d, conn, fi.ch) >= 0) {
      u32 gq, gna;
      if (dget_resolve(d, conn, b, p, fi.size, gq, gna)) { atomicMin(&sh_get0, f); continue; }
    }
    if (!content) {
      if (!data) atomicMin(&sh_stop, ((f + 1) << 3) | 0);
      continue;
    }
    // header then bodies on the same channel
    u32 g = f + 1;
    if (g >= nf) { atomicMin(&sh_stop, (f << 3) | 1); continue; }
    u32 hp = CPOS(g);
    FInfo hi = frame_at(b, hp, L, fmax);
    if (!hi.complete) { atomicMin(&sh_stop, (f << 3) | 1); continue; }
    if (hi.type != 2 || hi.ch != fi.ch || hi.size < 14) { atomicMin(&sh_stop, (f << 3) | 2); continue; }
    claim[g] = 1;
    u64 bsz = be64(b + hp + 7 + 4);
    if (data && big_publish(d, fi.size, hi.size, bsz, fmax)) {   // host-assembled: stop after its header
      atomicMin(&sh_stop, ((g + 1) << 3) | 0);
      continue;
    }
    u64 got = 0;
    u32 e = g;
    bool bad = false, incomplete = false;
    while (got < bsz) {
      ++e;
      if (e >= nf) { incomplete = true; break; }
      u32 bp = CPOS(e);
      FInfo bi = frame_at(b, bp, L, fmax);
      if (!bi.complete) { incomplete = true; break; }
      if (bi.type != 3 || bi.ch != fi.ch) { atomicMin(&sh_stop, (f << 3) | 2); bad = true; break; }
      claim[e] = 1;
      got += bi.size;
      if (got > bsz) { atomicMin(&sh_stop, (f << 3) | 3); bad = true; break; }
    }
    if (incomplete) atomicMin(&sh_stop, (f << 3) | 1);
    (void)bad;
    if (!data) atomicMin(&sh_stop, ((e + 1) << 3) | 0);
  }
  __syncthreads();
  for (u32 f = tid; f < nf; f += FS_NT) {
    if (claim[f]) continue;
    FInfo fi = frame_at(b, CPOS(f), L, fmax);
    if (fi.complete) atomicMin(&sh_stop, (f << 3) | 2);
  }
  __syncthreads();
  if (sh_get0 != INVALID) {   // (block-uniform) the segment serves Basic.Gets in this step
    // they all ask the same (channel, queue, no-ack) -- any two then answer alike, whichever
    // is served first -- and nothing but such Gets follows the first in this step (an ack
    // after a Get may name its delivery tag, which the step assigns later); the rest of the
    // segment waits in the carry for the next step
    const u32 g0 = sh_get0;
    if (tid == g0 % FS_NT) {
      const u32 p = CPOS(g0);
      FInfo fi = frame_at(b, p, L, fmax);
      u32 gq = 0, gna = 0;
      dget_resolve(d, conn, b, p, fi.size, gq, gna);
      sh_gch = fi.ch; sh_gq = gq; sh_gna = gna;
    }
    __syncthreads();
    for (u32 f = g0 + 1 + tid; f < nf; f += FS_NT) {
      const u32 p = CPOS(f);
      if (b[p] != 1) continue;   // content and heartbeat frames go with their method / nothing
      FInfo fi = frame_at(b, p, L, fmax);
      bool same = false;
      if (fi.complete && fi.size >= 4 && be16(b + p + 7) == 60 && be16(b + p + 9) == 70 && fi.ch == sh_gch) {
        u32 gq, gna;
        same = dget_resolve(d, conn, b, p, fi.size, gq, gna) && gq == sh_gq && gna == sh_gna;
      }
      if (!same) atomicMin(&sh_stop, (f << 3) | 4);
    }
    __syncthreads();
  }
  FS_MARK(4);
  u32 stop = sh_stop;
  u32 kf = stop >> 3, reason = stop & 7;
  if (kf > nf) kf = nf;
  if (reason == 7 && sh_brk) { reason = 3; }  // chain ended on a broken frame

  // consumed bytes: up to frame kf (or the end of the chain)
  u32 consumed;
  if (kf < nf) consumed = CPOS(kf);
  else if (nf == 0) consumed = 0;
  else {
    u32 lp = CPOS(nf - 1);
    FInfo lf = frame_at(b, lp, L, fmax);
    consumed = lf.complete ? lp + 8 + lf.size : lp;
  }
  if (reason == 3 || reason == 2) {
    so.status |= (reason == 3) ? SS_FRAME_ERROR : SS_UNEXPECTED;
    so.err_off = consumed;
  }
  if (over && reason != 0 && kf == nf) so.status |= SS_OVERFLOW;
  if (reason == 4) so.status |= SS_OVERFLOW;   // the carry is re-presented to the next step

  // split mode: the work buffer gets the carry and the frame that runs from it into the new
  // bytes (frames start inside the carry only before that point); later frames are read from
  // the ingress slot
  if (split) {
    if (tid == 0) sh_split = seg_cl;
    __syncthreads();
    for (u32 f = tid; f < nf; f += FS_NT) {
      const u32 p = CPOS(f);
      if (p >= seg_cl) continue;
      const FInfo fi = frame_at(b, p, L, fmax);
      const u64 e = fi.complete ? (u64)p + 8 + fi.size : (u64)L;
      atomicMax(&sh_split, (u32)(e < L ? e : L));
    }
    __syncthreads();
    uint4* const WD = (uint4*)(d.work + wbase);
    const u32 nw = (sh_split + 15) >> 4;
    for (u32 w = tid; w < nw; w += FS_NT) WD[w] = fs_stage[w];
    __syncthreads();
  }
  const u32 sp = split ? sh_split : inplace ? 0u : L + 1u;
  // a frame's offset from d.work (frames lie wholly below sp or at / above it)
  auto OFF = [&](u32 pos) -> u32 { return pos < sp ? wbase + pos : (u32)(ing_rel + src + pos - seg_cl); };
  FS_MARK(5);
  // ---- (e) emit commands for method frames < kf
  u32 run = 0, frun = 0;
  if (tid == 0) { sh_cmd_base = INVALID; sh_ncmd = 0; }
  __syncthreads();
  // count first -- unless the commands fit one emit chunk (the common case): then the emit
  // pass reserves them itself, from the scans it runs anyway
  const bool one = kf <= FS_NT;   // (block-uniform)
  u32 my_cmds = 0, my_frags = 0;
  for (u32 f = tid; f < kf && !one; f += FS_NT) {
    u32 p = CPOS(f);
    if (b[p] != 1) continue;
    ++my_cmds;
    if (be16(b + p + 7) == 60 && be16(b + p + 9) == 40) {
      // frags: frames after header until the next method
      u32 e = f + 2;
      while (e < kf && b[CPOS(e)] == 3) { ++my_frags; ++e; }
    }
  }
  u32 tc = 0, tfr = 0;
  if (!one) {
    block_scan<FS_NT>(my_cmds, sc, tc);
    block_scan<FS_NT>(my_frags, sc, tfr);
  }
  // one uncontended atomicAdd per block (a CAS loop here serialises all blocks);
  // on overflow the reserved in-range slots are filled with CK_NONE and the whole
  // segment is carried to the next step
  if (!one && tid == 0) {
    u32 cb = tc ? atomicAdd(&d.ctr->n_cmds, tc) : 0;
    u32 fb = tfr ? atomicAdd(&d.ctr->n_frags, tfr) : 0;
    sh_frag_base = fb;
    sh_cmd_base = cb;
    sh_ncmd = (cb + tc > d.cmd_max || fb + tfr > d.frag_max) ? 1u : 0u;
  }
  __syncthreads();
  if (sh_ncmd && tc > 0) {
    u32 cb = sh_cmd_base;
    for (u32 i = cb + tid; i < cb + tc && i < d.cmd_max; i += FS_NT) {
      d.cmds[i].kind = CK_NONE;
      d.cmd_is_pub[i] = 0;
      d.cmd_is_ack[i] = 0;
    }
    if (tid == 0) sh_cmd_base = INVALID;
    __syncthreads();
  }
  if (sh_cmd_base == INVALID && tc > 0) {
    so.status |= SS_OVERFLOW;
    so.status &= ~(SS_FRAME_ERROR | SS_UNEXPECTED);
    consumed = 0;
    kf = 0;
    reason = 7;
  }
  FS_MARK(6);
  const i64 now = d.in->now_ms;
  u32 npub_run = 0, nack_run = 0;   // the segment's publishes / acks so far (their ordinals)
  for (u32 f0 = 0; f0 < kf; f0 += FS_NT) {
    u32 f = f0 + tid;
    u32 is_cmd = 0, nfr = 0;
    u32 p = 0;
    // every command's kind first: the publish / ack ordinals within the segment come out of
    // the same block scan as the command index (no grid-wide rank scan over the commands)
    Cmd c;
    FInfo fi;
    u32 cls = 0, mid = 0, hp = 0, gq = 0, gna = 0;
    FInfo hi;
    if (f < kf) {
      p = CPOS(f);
      if (b[p] == 1) {
        is_cmd = 1;
        if (be16(b + p + 7) == 60 && be16(b + p + 9) == 40) {
          u32 e = f + 2;
          while (e < kf && b[CPOS(e)] == 3) { ++nfr; ++e; }
        }
      }
    }
    if (is_cmd) {
      fi = frame_at(b, p, L, fmax);
      cls = be16(b + p + 7);
      mid = be16(b + p + 9);
      const i32 chs = fi.ch ? chan_lookup(d, conn, fi.ch) : -1;
      c.pad[0] = (u32)chs;
      if (cls == 60 && mid == 40 && chs >= 0) c.kind = CK_PUBLISH;
      else if (cls == 60 && mid == 70 && chs >= 0 && dget_resolve(d, conn, b, p, fi.size, gq, gna)) c.kind = CK_GET;
      else if (cls == 60 && mid == 80 && chs >= 0) c.kind = CK_ACK;
      else if (cls == 60 && mid == 90 && chs >= 0) c.kind = CK_REJECT;
      else if (cls == 60 && mid == 120 && chs >= 0) c.kind = CK_NACK;
      else c.kind = CK_CONTROL;
      if (c.kind != CK_CONTROL && c.kind != CK_GET && d.ch_tx[chs]) c.kind = CK_TXBUF;   // held until Tx.Commit
      if (cls == 60 && mid == 40) {
        hp = CPOS(f + 1);
        hi = frame_at(b, hp, L, fmax);
        // a publish too large for the carry is a control command: the host assembles it
        if ((c.kind == CK_PUBLISH || c.kind == CK_TXBUF) && big_publish(d, fi.size, hi.size, be64(b + hp + 7 + 4), fmax))
          c.kind = CK_CONTROL;
      }
    }
    const u32 is_pub = is_cmd && c.kind == CK_PUBLISH;
    const u32 is_ack = is_cmd && (c.kind == CK_ACK || c.kind == CK_NACK || c.kind == CK_REJECT);
    // one scan of three 11-bit counters (<= FS_NT each per chunk): commands | pubs | acks
    u32 tpk, tf;
    const u32 rpk = block_scan<FS_NT>(is_cmd | (is_pub << 11) | (is_ack << 22), sc, tpk);
    u32 fr = block_scan<FS_NT>(nfr, sc, tf);
    const u32 r = rpk & 0x7ffu, tcnt = tpk & 0x7ffu;
    if (one) {   // the segment's only chunk: reserve its commands / fragments now (as above)
      if (tid == 0) {
        const u32 cb = tcnt ? atomicAdd(&d.ctr->n_cmds, tcnt) : 0;
        const u32 fb = tf ? atomicAdd(&d.ctr->n_frags, tf) : 0;
        sh_frag_base = fb;
        sh_cmd_base = cb;
        sh_ncmd = (cb + tcnt > d.cmd_max || fb + tf > d.frag_max) ? 1u : 0u;
      }
      __syncthreads();
      if (sh_ncmd && tcnt > 0) {   // (block-uniform) overflow: nothing is emitted, all carried
        const u32 cb = sh_cmd_base;
        for (u32 i = cb + tid; i < cb + tcnt && i < d.cmd_max; i += FS_NT) {
          d.cmds[i].kind = CK_NONE;
          d.cmd_is_pub[i] = 0;
          d.cmd_is_ack[i] = 0;
        }
        __syncthreads();
        if (tid == 0) sh_cmd_base = INVALID;
        so.status |= SS_OVERFLOW;
        so.status &= ~(SS_FRAME_ERROR | SS_UNEXPECTED);
        consumed = 0;
        kf = 0;
        reason = 7;
        break;
      }
      if (tcnt == 0 && tid == 0) sh_cmd_base = INVALID;
    }
    // the segment's Basic.Gets: a contiguous DGet range per chunk, in wire order
    u32 gi = INVALID;
    if (sh_get0 != INVALID) {   // (block-uniform)
      const u32 is_get = is_cmd && c.kind == CK_GET;
      u32 tg;
      const u32 rg = block_scan<FS_NT>(is_get, sc, tg);
      if (tid == 0) sh_gbase = tg ? atomicAdd(&d.tot[TS_NDGET], tg) : 0;
      __syncthreads();
      if (is_get) gi = sh_gbase + rg;
    }
    if (is_cmd) {
      c.conn = conn;
      c.ch = fi.ch;
      c.m_off = OFF(p) + 7;
      c.m_len = fi.size;
      c.h_off = 0; c.h_len = 0; c.frag0 = 0; c.nfrag = 0; c.body_size = 0;
      c.seg = s;
      c.raw_off = OFF(p);
      // ordinals within the segment: k_decode numbers publishes / acks segment-major
      c.pad[1] = npub_run + ((rpk >> 11) & 0x7ffu);
      c.pad[2] = nack_run + (rpk >> 22);
      u32 endp = p + 8 + fi.size;
      if (cls == 60 && mid == 40) {
        c.h_off = OFF(hp) + 7;
        c.h_len = hi.size;
        c.body_size = (u32)be64(b + hp + 7 + 4);
        c.frag0 = sh_frag_base + frun + fr;
        c.nfrag = nfr;
        endp = hp + 8 + hi.size;
        for (u32 k = 0; k < nfr; ++k) {
          u32 bp = CPOS(f + 2 + k);
          FInfo bi = frame_at(b, bp, L, fmax);
          Frag fg;
          fg.off = OFF(bp) + 7;
          fg.len = bi.size;
          d.frags[c.frag0 + k] = fg;
          endp = bp + 8 + bi.size;
        }
      }
      c.raw_len = endp - p;
      const u32 ci = sh_cmd_base + run + r;
      if (gi != INVALID) {
        if (gi < DGET_MAX) {
          DGet g;
          g.conn = conn; g.chslot = c.pad[0]; g.q = gq; g.noack = gna;
          g.raw_off = c.raw_off; g.raw_len = c.raw_len; g.seg = s; g.pad = 0;
          d.dget[gi] = g;
        } else {
          c.kind = CK_CONTROL;   // the step's DGet list is full: the host serves it (not paused)
        }
      }
      d.cmds[ci] = c;
      // classification for the rank scan of the large-segment-count path (k_decode)
      d.cmd_is_pub[ci] = is_pub;
      d.cmd_is_ack[ci] = is_ack;
      if (c.kind == CK_CONTROL || c.kind == CK_TXBUF) {
        u32 cbase;
        u32 g = reserve_sat(&d.ctr->ctrl_bytes, c.raw_len, (u32)d.ctrl_cap, &cbase);
        u32 ri = atomicAdd(&d.ctr->n_ctrl, 1u);
        CtrlRec rec;
        rec.conn = conn;
        if (g == c.raw_len) {
          for (u32 k = 0; k < c.raw_len; ++k) d.ctrl[cbase + k] = b[p + k];
          rec.off = cbase; rec.len = c.raw_len;
          rec.seg = c.kind == CK_TXBUF ? (CTRL_TXBUF | p) : gi != INVALID ? (CTRL_DGET | s) : s;
        } else {   // control buffer full: an event, the host closes the connection (506)
          rec.off = INVALID; rec.len = 506; rec.seg = 0;
        }
        if (ri < d.seg_max * 2) d.ctrl_rec[ri] = rec;
      }
    }
    run += tcnt;
    frun += tf;
    npub_run += (tpk >> 11) & 0x7ffu;
    nack_run += tpk >> 22;
  }
  if (tid == 0 && kf > 0) d.conn_last_rx[conn] = now;
  if (reason == 0) so.status |= SS_CTRL;
  if (tid == 0) {   // the segment's publish / ack counts: k_decode numbers them segment-major
    d.seg_cmd_base[s] = (run && sh_cmd_base != INVALID) ? sh_cmd_base : INVALID;
    d.seg_npub[s] = d.seg_cmd_base[s] == INVALID ? 0u : npub_run;
    d.seg_nack[s] = d.seg_cmd_base[s] == INVALID ? 0u : nack_run;
  }

  FS_MARK(7);
  // ---- (f) carry out: bytes [consumed, L)
  u32 rest = L - consumed;
  if (rest > d.carry_cap) { so.status |= SS_TOO_LARGE; rest = 0; }
  else if (split) {   // [consumed, sp) from the work copy, the rest from the ingress slot (sp >= carry)
    u8* const cd = d.carry + (u64)conn * d.carry_cap;
    if (consumed < sp) block_copy(cd, d.work + wbase + consumed, sp - consumed, tid, FS_NT);
    const u32 from = consumed > sp ? consumed : sp;
    if (from < L) block_copy(cd + (from - consumed), seg_N + (from - seg_cl), L - from, tid, FS_NT);
  } else block_copy(d.carry + (u64)conn * d.carry_cap, bg + consumed, rest, tid, FS_NT);   // 16-B moves from HBM
  FS_MARK(8);
  if (tid == 0) {
    so.consumed = consumed;
    so.carry = rest;
    so.ncmds = run;
    d.carry_len[conn] = rest;
    if (reason == 0) d.conn_paused[conn] = 1;
    d.seg_out[s] = so;
  }
#undef CPOS
}

// block-stride over the segments: the grid is capped below seg_max (a 1024-thread block
// per segment slot of the capacity would mostly launch idle waves)
__global__ __launch_bounds__(FS_NT) void k_frame_scan(DS d) {
  const u32 nseg = d.in->nseg;
  for (u32 s = blockIdx.x; s < nseg; s += gridDim.x) {
    frame_scan_seg(d, s);
    __syncthreads();   // the next segment reuses the LDS
  }
}

// a Basic.Get the frame scan decoded that its step cannot serve (delivery window full, cold
// queue head, step full, queue gone): its bytes go to the host as a control record flagged
// CTRL_DGET -- the connection is not paused -- and the host serves it with a later step
DEV void dget_to_host(const DS& d, u32 k) {
  const DGet g = d.dget[k];
  u32 cbase;
  const u32 got = reserve_sat(&d.ctr->ctrl_bytes, g.raw_len, (u32)d.ctrl_cap, &cbase);
  const u32 ri = atomicAdd(&d.ctr->n_ctrl, 1u);
  CtrlRec rec;
  rec.conn = g.conn;
  if (got == g.raw_len) {
    for (u32 k = 0; k < g.raw_len; ++k) d.ctrl[cbase + k] = d.work[g.raw_off + k];
    rec.off = cbase; rec.len = g.raw_len; rec.seg = CTRL_DGET | g.seg;
  } else {   // control buffer full: an event, the host closes the connection (506)
    rec.off = INVALID; rec.len = 506; rec.seg = 0;
  }
  if (ri < d.seg_max * 2) d.ctrl_rec[ri] = rec;
}

// ============================================================================ K3 classify / decode
DEV void set_counts(const DS& d, u32 np, u32 na) {
  d.ctr->n_pubs = np < d.pub_max ? np : d.pub_max;
  d.ctr->n_acks = na < d.ack_max ? na : d.ack_max;
  // routing phase 0: the step's own publishes
  d.tot[TS_RANGE_LO] = 0;
  d.tot[TS_RANGE_HI] = d.ctr->n_pubs;
  d.tot[TS_PAIR_BASE] = 0;
  d.tot[TS_PAIR_N] = 0;
  d.tot[TS_NIMPORT] = 0;
}

DEV bool skip_shortstr(const u8* p, u32& o, u32 end) {
  if (o + 1 > end) return false;
  o += 1 + p[o];
  return o <= end;
}

// topic key vector (8 words x 32 bits, +-1), built only if topic bindings exist
DEV u32 build_keyvec(const DS& d, const u8* key, u32 len, u32 pi) {
  Words kw = words_of(key, len);
  if (d.tb_max) {
    // 32 int8 lanes per word (+1 / -1 per hash bit), written as two 16-B stores
    uint4* kv = (uint4*)(d.pub_keyvec + (u64)pi * TOPIC_K);
    u16* kwo = d.pub_kwoff + (u64)pi * TOPIC_WORDS;   // (offset << 8 | length) per word
    u32 off = 0;
    u32 wi = 0;
    if (kw.count) {
      while (wi < TOPIC_WORDS && off <= kw.eff) {
        u32 wl = word_len(key, off, kw.eff);
        u32 h = fnv1a32(key + off, wl);
        kwo[wi] = (u16)((off << 8) | (wl & 255));
        u32 pk[8];
#pragma unroll
        for (int g = 0; g < 8; ++g) {
          u32 v = 0;
#pragma unroll
          for (int bb = 0; bb < 4; ++bb) v |= (((h >> (g * 4 + bb)) & 1) ? 0x01u : 0xffu) << (8 * bb);
          pk[g] = v;
        }
        kv[wi * 2] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
        kv[wi * 2 + 1] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
        off += wl + 1;
        ++wi;
      }
    }
    for (; wi < TOPIC_WORDS; ++wi) {
      kv[wi * 2] = make_uint4(0, 0, 0, 0);
      kv[wi * 2 + 1] = make_uint4(0, 0, 0, 0);
    }
  }
  return kw.count;
}

// ---- 32-byte register windows of a publish's method arguments and routing key.  The
// byte loops above cost one memory round trip per byte wherever a loop's exit depends on
// the byte (word_len, the trailing-'.' strip), ~20 dependent trips per publish at one
// thread per command; here two 16-byte loads bring the bytes in and every loop below is
// unrolled over compile-time positions (register selects, no scratch).  Callers guarantee
// 32 readable bytes at the window start (the work buffer has 4 KB of slack past work_cap).
// named words, not an array: no dynamic index can pin the window to scratch memory
struct Win32 { u32 w0, w1, w2, w3, w4, w5, w6, w7; };
DEV Win32 load_win(const u8* p) {
  const U4 a = *(const U4*)p, b = *(const U4*)(p + 16);
  return Win32{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
}
// word k < 8: folds to one register for a compile-time k, a select chain otherwise
DEV u32 win_word(const Win32& s, u32 k) {
  // selects over values (a ?: over the members themselves selects their addresses)
  const u32 a0 = s.w0, a1 = s.w1, a2 = s.w2, a3 = s.w3, a4 = s.w4, a5 = s.w5, a6 = s.w6, a7 = s.w7;
  const u32 lo = k < 2 ? (k == 0 ? a0 : a1) : (k == 2 ? a2 : a3);
  const u32 hi = k < 6 ? (k == 4 ? a4 : a5) : (k == 6 ? a6 : a7);
  return k < 4 ? lo : hi;
}
// byte i < 32 of the window
DEV u32 win_byte(const Win32& s, u32 i) { return (win_word(s, i >> 2) >> (8 * (i & 3))) & 255u; }
DEV u32 win_get(const Win32& s, u32 i) { return win_byte(s, i); }
// FNV-1a 64 of bytes [S, S + n) of the window (S + n <= 32)
template <u32 S>
DEV u64 win_fnv64(const Win32& s, u32 n, u64 h) {
#pragma unroll
  for (u32 i = 0; i + S < 32; ++i) {
    if (i < n) {   // predicated, not a break: the loop stays fully unrolled (constant indices)
      h ^= win_byte(s, i + S);
      h *= FNV64_PRIME;
    }
  }
  return h;
}

// build_keyvec for a routing key of n <= 32 bytes held in a window: same rows, same count
DEV u32 build_keyvec_win(const DS& d, const Win32& s, u32 n, u32 pi) {
  const u32 lenmask = n >= 32 ? ~0u : ((1u << n) - 1u);
  u32 dots = 0;
#pragma unroll
  for (u32 i = 0; i < 32; ++i) dots |= (win_byte(s, i) == '.' ? 1u : 0u) << i;
  dots &= lenmask;
  const u32 nd = ~dots & lenmask;                 // trailing '.' stripped (words_of)
  const u32 eff = nd ? 32u - __clz(nd) : 0u;
  const u32 effmask = eff >= 32 ? ~0u : ((1u << eff) - 1u);
  const u32 de = dots & effmask;
  const u32 count = n == 0 ? 1u : (eff == 0 ? 0u : 1u + __popc(de));
  if (!d.tb_max) return count;
  // per-word FNV-1a 32 in one pass: a '.' commits the running hash to its word slot
  u32 hw[TOPIC_WORDS];
#pragma unroll
  for (u32 k = 0; k < TOPIC_WORDS; ++k) hw[k] = 0x811c9dc5u;
  u32 h = 0x811c9dc5u, wi = 0;
#pragma unroll
  for (u32 i = 0; i < 32; ++i) {
    const u32 c = win_byte(s, i);
    const bool in = i < eff, dot = in && c == '.';
#pragma unroll
    for (u32 k = 0; k < TOPIC_WORDS; ++k) hw[k] = (dot && wi == k) ? h : hw[k];
    wi += dot ? 1u : 0u;
    h = dot ? 0x811c9dc5u : (in ? (h ^ c) * 0x01000193u : h);
  }
#pragma unroll
  for (u32 k = 0; k < TOPIC_WORDS; ++k) hw[k] = wi == k ? h : hw[k];
  const u32 nw = count < TOPIC_WORDS ? count : TOPIC_WORDS;
  uint4* kv = (uint4*)(d.pub_keyvec + (u64)pi * TOPIC_K);
  u16* kwo = d.pub_kwoff + (u64)pi * TOPIC_WORDS;
  u32 off = 0;
#pragma unroll
  for (u32 k = 0; k < TOPIC_WORDS; ++k) {
    if (k < nw) {
      const u32 rest = off >= 32 ? 0u : (de & ~((1u << off) - 1u));   // separators at or after off
      u32 e = rest ? (u32)(__ffs(rest) - 1) : eff;
      if (e > eff) e = eff;
      const u32 wl = e - off;
      kwo[k] = (u16)((off << 8) | (wl & 255));
      u32 pk[8];
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        u32 v = 0;
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) v |= (((hw[k] >> (g * 4 + bb)) & 1) ? 0x01u : 0xffu) << (8 * bb);
        pk[g] = v;
      }
      kv[k * 2] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
      kv[k * 2 + 1] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
      off = e + 1;
    } else {
      kv[k * 2] = make_uint4(0, 0, 0, 0);
      kv[k * 2 + 1] = make_uint4(0, 0, 0, 0);
    }
  }
  return count;
}

// K9 ack mark (AMQChannel.scala:128-174): single tag -> its window slot; multiple -> the
// record (tag resolved) stays in d.acks and the channel's [first, last] ack index range
// grows, so k_chan_advance resolves the step's multiple settles in wire order (ack index
// = command order): a tag's fate is the first settle covering it, e.g. Nack(4, requeue)
// then Ack(8) requeues 1-4.  Marks only depend on earlier steps' deliveries.
DEV void apply_ack(const DS& d, Ack a, u32 ai) {
  const u32 ch = a.chslot;
  if (ch == INVALID) { d.acks[ai] = a; return; }
  const u64 nt = d.ch_next_tag[ch];
  u64 tag = a.tag;
  if (tag == 0 && a.multiple) tag = nt - 1;  // ack everything outstanding
  a.tag = tag;
  d.acks[ai] = a;
  const bool requeue = (a.kind != CK_ACK) && a.requeue;
  if (a.multiple) {
    atomicMin(&d.ch_mlo[ch], ai);
    atomicMax(&d.ch_mhi[ch], ai);
  } else if (tag >= d.ch_uhead[ch] && tag < nt) {
    USlot& u = d.uwin[(u64)ch * (d.ucap_mask + 1) + ((tag - 1) & d.ucap_mask)];
    atomicCAS(&u.state, (u32)US_PENDING, requeue ? (u32)US_REQUEUE : (u32)US_ACKED);
  }
  if (atomicExch(&d.ch_dirty[ch], 1u) == 0) {
    u32 k = atomicAdd(d.n_dirty, 1u);
    d.dirty_list[k] = ch;
  }
  atomicAdd(&d.ctr->n_acked, 1u);
}

// publishes are numbered in segment order (segment s's publishes follow those of the
// segments before it), not in the order the frame-scan blocks reserved their commands:
// queue order across connections is then deterministic (the golden model's order)
__global__ __launch_bounds__(256) void k_decode(DS d) {
  __shared__ u32 spref[DEC_SEG_LDS];
  __shared__ u32 sprefa[DEC_SEG_LDS];
  __shared__ u32 lds[256 / 64 + 1];
  const u32 nseg = d.in->nseg;
  const bool seg_order = nseg <= DEC_SEG_LDS;
  u32 n0 = d.ctr->n_cmds;
  n0 = n0 < d.cmd_max ? n0 : d.cmd_max;
  if (!d.rank_scan) {
    // segment-major numbering from the frame scan's per-segment ordinals: every busy block
    // (and block 0, which sets the step's counts) scans the segments' publish / ack counts
    if (blockIdx.x != 0 && blockIdx.x * 256 >= n0) return;   // whole block idle
    u32 run = 0, runa = 0;
    for (u32 b0 = 0; b0 < nseg; b0 += 256) {
      const u32 k = b0 + threadIdx.x;
      const u32 v = k < nseg ? d.seg_npub[k] : 0, va = k < nseg ? d.seg_nack[k] : 0;
      u32 all, alla;
      const u32 o = block_scan<256>(v, lds, all);
      const u32 oa = block_scan<256>(va, lds, alla);
      if (k < nseg) { spref[k] = run + o; sprefa[k] = runa + oa; }
      run += all;
      runa += alla;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) set_counts(d, run, runa);   // fused: counts + phase-0 range
    __syncthreads();
    if (blockIdx.x * 256 >= n0) return;
  } else {
    if (blockIdx.x == 0 && threadIdx.x == 0) set_counts(d, d.tot[4], d.tot[5]);
    if (blockIdx.x * 256 >= n0) return;   // whole block idle
    if (seg_order) {
      u32 run = 0;
      for (u32 b0 = 0; b0 < nseg; b0 += 256) {
        const u32 k = b0 + threadIdx.x;
        const u32 v = k < nseg ? d.seg_npub[k] : 0;
        u32 all;
        const u32 o = block_scan<256>(v, lds, all);
        if (k < nseg) spref[k] = run + o;
        run += all;
      }
      __syncthreads();
    }
  }
  u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  u32 n = d.ctr->n_cmds;
  if (n > d.cmd_max) n = d.cmd_max;
  if (i >= n) return;
  const Cmd c = d.cmds[i];
  const u8* w = d.work;
  if (c.kind == CK_PUBLISH) {
    u32 pi;
    if (!d.rank_scan) {
      pi = spref[c.seg] + c.pad[1];
    } else {
      pi = d.cmd_pub_rank[i];
      if (seg_order && c.seg < nseg && d.seg_cmd_base[c.seg] != INVALID)
        pi = spref[c.seg] + (pi - d.cmd_pub_rank[d.seg_cmd_base[c.seg]]);
    }
    if (pi >= d.pub_max) return;
    Pub pb;
    pb.conn = c.conn;
    pb.chslot = c.pad[0];
    pb.frag0 = c.frag0;
    pb.nfrag = c.nfrag;
    pb.body_size = c.body_size;
    pb.flags = 0;
    pb.expire_ms = 0;
    pb.ts_ms = 0;
    pb.nq = 0; pb.slot_bytes = 0; pb.msg = INVALID; pb.pad = 0; pb.xid = 0;
    // method args: class u16, method u16, ticket u16, exchange ss, rk ss, bits
    // (skip_shortstr inlined over register windows: [ex_len][exchange][rk_len] in one,
    // exchange names up to 30 bytes; the routing key and the bits octet in a second)
    u32 o = c.m_off + 6, end = c.m_off + c.m_len;
    const u32 o0 = o;
    const Win32 ma = load_win(w + o0);
    bool ok = o <= end;
    pb.ex_off = o + 1;
    const u32 b0 = ok && o < end ? win_byte(ma, 0) : 0u;
    pb.ex_len = b0;
    if (ok) { if (o + 1 > end) ok = false; else { o += 1 + b0; ok = o <= end; } }
    pb.rk_off = o + 1;
    const u32 b1 = ok && o < end ? (o - o0 < 32 ? win_get(ma, o - o0) : (u32)w[o]) : 0u;
    pb.rk_len = b1;
    if (ok) { if (o + 1 > end) ok = false; else { o += 1 + b1; ok = o <= end; } }
    const Win32 rkw = load_win(w + pb.rk_off);
    u32 bits = (ok && o < end) ? (o - pb.rk_off < 32 ? win_get(rkw, o - pb.rk_off) : (u32)w[o]) : 0u;
    if (bits & 1) pb.flags |= MF_MANDATORY;
    if (bits & 2) pb.flags |= MF_IMMEDIATE;
    // exchange
    i32 xs = -1;
    if (ok) {
      const u32 vh = d.conn_vhost[c.conn];
      u64 hk = pb.ex_len <= 31 ? win_fnv64<1>(ma, pb.ex_len, FNV64_BASIS ^ (u64(vh) * 0x9E3779B97F4A7C15ULL))
                               : exch_hash(vh, w + pb.ex_off, pb.ex_len);
      u32 mask = d.xhash_mask;
      for (u32 j = 0; j <= mask; ++j) {
        u32 slot = (u32)(hk + j) & mask;
        i32 v = d.x_hval[slot];
        if (v < 0) break;
        if (d.x_hkey[slot] == hk) { xs = v; break; }
      }
    }
    pb.exch = ok ? xs : -2;
    pb.keyhash = pb.rk_len <= 32 ? win_fnv64<0>(rkw, pb.rk_len, FNV64_BASIS) : fnv1a64_dev(w + pb.rk_off, pb.rk_len);
    // properties (flags chain then values), read through a 32-byte register window of the
    // header payload (one pair of loads instead of one dependent load per field)
    u32 ho = c.h_off + 12, hend = c.h_off + c.h_len;
    pb.props_off = ho;
    pb.props_len = hend > ho ? hend - ho : 0;
    const Win32 pw = load_win(w + ho);
    auto pbyte = [&](u32 q) -> u32 { const u32 o = q - ho; return o < 32 ? win_byte(pw, o) : (u32)w[q]; };
    u32 fl = 0;   // the first property-flags word (continuation words are skipped)
    u32 nfl = 0;
    u32 q = ho;
    while (q + 2 <= hend) {
      u32 fw = (pbyte(q) << 8) | pbyte(q + 1);
      q += 2;
      if (nfl == 0) fl = fw;
      ++nfl;
      if (!(fw & 1)) break;
    }
    bool pok = true;
    // field order: 15 ctype ss, 14 cenc ss, 13 headers tbl, 12 dmode oct, 11 prio oct,
    // 10 corr ss, 9 replyto ss, 8 expiration ss, 7 msgid ss, 6 timestamp u64, 5 type,
    // 4 userid, 3 appid, 2 clusterid
    for (int bit = 15; bit >= 2 && pok; --bit) {
      if (!(fl & (1u << bit))) continue;
      switch (bit) {
        case 13: {
          if (q + 4 > hend) { pok = false; break; }
          u32 tl = (pbyte(q) << 24) | (pbyte(q + 1) << 16) | (pbyte(q + 2) << 8) | pbyte(q + 3);
          q += 4 + tl;
          pok = q <= hend;
          break;
        }
        case 12:
          if (q + 1 > hend) { pok = false; break; }
          if (pbyte(q) == 2) pb.flags |= MF_PERSIST;
          q += 1;
          break;
        case 11: q += 1; pok = q <= hend; break;
        case 8: {
          if (q + 1 > hend) { pok = false; break; }
          u32 sl = pbyte(q);
          if (q + 1 + sl > hend) { pok = false; break; }
          i64 v = 0;
          bool digits = sl > 0 && sl <= 18;
          for (u32 k = 0; k < sl && digits; ++k) {
            u32 ch = pbyte(q + 1 + k);
            if (ch < '0' || ch > '9') digits = false;
            else v = v * 10 + (ch - '0');
          }
          if (digits) pb.expire_ms = d.in->now_ms + v;
          q += 1 + sl;
          break;
        }
        case 6: {
          if (q + 8 > hend) { pok = false; break; }
          u64 ts = 0;
#pragma unroll
          for (u32 k = 0; k < 8; ++k) ts = (ts << 8) | pbyte(q + k);
          pb.ts_ms = (i64)ts * 1000;
          pb.flags |= MF_HAS_TS;
          q += 8;
          break;
        }
        default:
          if (q + 1 > hend) { pok = false; break; }
          q += 1 + pbyte(q);
          pok = q <= hend;
      }
    }
    pb.nwords = pb.rk_len <= 32 ? build_keyvec_win(d, rkw, pb.rk_len, pi) : build_keyvec(d, w + pb.rk_off, pb.rk_len, pi);
    // egress by reference: a body that is one run of this step's new ingress bytes (not in
    // the connection's carry) keeps its host address -- its deliveries can be sent from
    // there instead of crossing PCIe back (render_deliv)
    if (c.nfrag == 1 && d.in->ingress_host && d.in->ref_back != 0xffffffffu && c.body_size >= d.in->ref_min &&
        c.seg < nseg) {
      const Frag fg = d.frags[c.frag0];
      const u32 w0 = d.seg_start[c.seg], cl = d.seg_total[c.seg] - d.segs[c.seg].len;
      const u64 ing_rel = (u64)d.in->ingress - (u64)d.work;
      if (fg.len == c.body_size && d.scan_inplace && (u64)d.in->ingress > (u64)d.work && fg.off >= ing_rel) {
        pb.flags |= MF_HREF;   // (read in place from the ingress slot: its payload offset)
        pb.pad = (u32)(fg.off - ing_rel);
      } else if (fg.len == c.body_size && fg.off >= w0 + cl && fg.off < w0 + d.seg_total[c.seg]) {
        pb.flags |= MF_HREF;
        pb.pad = (u32)(d.segs[c.seg].src + (fg.off - w0 - cl));
      }
    }
    d.pubs[pi] = pb;   // (its channel's confirm count: k_marks)
  } else if (c.kind == CK_ACK || c.kind == CK_NACK || c.kind == CK_REJECT) {
    const u32 ai = d.rank_scan ? d.cmd_ack_rank[i] : sprefa[c.seg] + c.pad[2];
    if (ai >= d.ack_max) return;
    Ack a;
    a.chslot = c.pad[0];
    a.kind = c.kind;
    u32 o = c.m_off + 4;
    bool ok = c.m_len >= 13;
    a.tag = ok ? be64(w + o) : 0;
    u32 bits = ok ? w[o + 8] : 0;
    if (c.kind == CK_ACK) { a.multiple = bits & 1; a.requeue = 0; }
    else if (c.kind == CK_REJECT) { a.multiple = 0; a.requeue = bits & 1; }
    else { a.multiple = bits & 1; a.requeue = (bits >> 1) & 1; }
    d.acks[ai] = a;   // marked in the channel's window by k_marks (k_chan_advance resolves it)
  }
}

// K9 marks + K10 confirm counts of the step's commands: the first kernel of the step's
// routing half.  k_decode only records acks and publishes, so the ingest half never
// touches delivery-side state and can run next to the previous step's k_chan_advance /
// k_render (engine overlap).  Also the routing half's per-step resets.
// (fused into k_route_store, phase 0: the marks only have to precede k_chan_advance, and
// the snowflake id floor moved into log_reserve, its one reader -- a launch less per step)
DEV void marks_range(const DS& d, u32 i0, u32 stride) {
  if (i0 == 0 && d.links)
    for (u32 r = 0; r < WORLD_MAX; ++r) d.lk_cnt[r] = 0;
  const u32 na = d.ctr->n_acks, np = d.ctr->n_pubs;
  const u32 n = na > np ? na : np;
  for (u32 i = i0; i < n; i += stride) {
    if (i < na) apply_ack(d, d.acks[i], i);
    if (i < np) {
      const u32 ch = d.pubs[i].chslot;
      if (ch != INVALID && d.ch_confirm[ch]) atomicAdd(&d.ch_pub_cnt[ch], 1u);
    }
  }
}
__global__ __launch_bounds__(256) void k_marks(DS d) { marks_range(d, blockIdx.x * 256 + threadIdx.x, gridDim.x * 256); }

// ============================================================================ scans
// single-block multi-array exclusive scan; n read from device; totals -> tot[slot+k]
// lo != null: scan elements [*lo, *n) (absolute indices), else [0, *n)
// NA <= 4: arrays in[k] / out[k].  NA = 8 (per-rank pairs): array k is in[k & 1] +
// (k >> 1) * stride
struct ScanArgs { const u32* in[4]; u32* out[4]; const u32* n; const u32* lo; u32 narr; u32 nmax; u32 tot_slot; u64 stride; };
// Single-pass exclusive scan over up to NA arrays, 4 elements per thread, 4096-element
// tiles (NA = 8: the per-rank counts of the cross-GPU pack, 4 ranks per launch; 16 arrays
// spill registers; 1024-element tiles lengthen the look-back chain), tiles chained by
// decoupled look-back: each tile publishes its aggregate, then its inclusive prefix, in a
// per-(array, tile) status word tagged with the launch epoch, so the status array never
// needs clearing.  Tickets (not blockIdx) order the tiles, so a tile only ever waits on
// tiles whose blocks are already running.
//   status word = epoch << 34 | flag << 32 | value   (flag 1 = aggregate, 2 = inclusive)
#define SCAN_TILE 4096
// one tile of the scan (1024 threads); true (block-uniform) in the block that holds the
// last data tile, after its totals are written
template <int NA, int EPT>
DEV bool scan_tile(const ScanArgs& a, u32* tot, u64* status, u32* ctl, u32 smax) {
  constexpr u32 TILE = 1024 * EPT;
  __shared__ u32 s_tile, s_epoch;
  __shared__ u32 s_excl[NA];
  __shared__ u32 wsum[NA][1024 / 64 + 1];
  const u32 tid = threadIdx.x;
  if (tid == 0) {
    s_epoch = atomicAdd(&ctl[1], 0u);
    s_tile = atomicAdd(&ctl[0], 1u);
  }
  __syncthreads();
  const u32 tile = s_tile, epoch = s_epoch & 0x3fffffffu;
  const bool last_block = tile == gridDim.x - 1;
  u32 n = a.n ? *a.n : a.nmax;
  if (n > a.nmax) n = a.nmax;
  // lo: elements [lo, lo + n) -- applied at each access (rewriting the argument struct's
  // pointers would copy it to scratch memory)
  const u32 lo = a.lo ? *a.lo : 0u;
  n = n > lo ? n - lo : 0;
  const u32 base = tile * TILE;
  const bool data = base < n || tile == 0;
  if (data) {
    const u32 i = base + tid * EPT;
    u32 v[NA][EPT], off[NA], sm[NA];
    // every array's loads in flight at once, then one block scan of the sums together
#pragma clang loop unroll(full)
    for (int k = 0; k < NA; ++k) {
#pragma clang loop unroll(full)
      for (int e = 0; e < EPT; ++e) v[k][e] = 0;
      if ((u32)k >= a.narr) continue;
      const u32* in = (NA <= 4 ? a.in[k & 3] : a.in[k & 1] + (u64)(k >> 1) * a.stride) + lo;
      if (EPT == 4 && i + 3 < n && !(((uintptr_t)(in + i)) & 15)) {
        uint4 x = *(const uint4*)(in + i);
        v[k][0] = x.x; v[k][EPT > 1 ? 1 : 0] = x.y; v[k][EPT > 2 ? 2 : 0] = x.z; v[k][EPT > 3 ? 3 : 0] = x.w;
      } else {
#pragma clang loop unroll(full)
        for (int e = 0; e < EPT; ++e)
          if (i + e < n) v[k][e] = in[i + e];
      }
    }
    const u32 ln = tid & 63, w = tid >> 6;
    u32 x[NA];
#pragma clang loop unroll(full)
    for (int k = 0; k < NA; ++k) {
      u32 t = 0;
#pragma clang loop unroll(full)
      for (int e = 0; e < EPT; ++e) t += v[k][e];
      sm[k] = t;
      x[k] = t;
    }
#pragma clang loop unroll(full)
    for (int o = 1; o < 64; o <<= 1) {
#pragma clang loop unroll(full)
      for (int k = 0; k < NA; ++k) {
        u32 y = __shfl_up(x[k], o, 64);
        if (ln >= (u32)o) x[k] += y;
      }
    }
    if (ln == 63) {
#pragma clang loop unroll(full)
      for (int k = 0; k < NA; ++k) wsum[k][w] = x[k];
    }
    __syncthreads();
    if (tid < NA) {
      u32 run = 0;
      for (u32 j = 0; j < 1024 / 64; ++j) { u32 t = wsum[tid][j]; wsum[tid][j] = run; run += t; }
      wsum[tid][1024 / 64] = run;
    }
    __syncthreads();
#pragma clang loop unroll(full)
    for (int k = 0; k < NA; ++k) off[k] = wsum[k][w] + x[k] - sm[k];
    // look-back, one wave per array: the wave's 64 lanes read the 64 preceding tiles'
    // status words at once, so a tile waits one round trip for all its (concurrently
    // running) predecessors instead of a chain of them
    const u32 wv = tid >> 6, lane = tid & 63;
    if (wv < a.narr && wv < (u32)NA) {
      const u32 k = wv;
      const u32 A = wsum[k][1024 / 64];   // the tile's aggregate of array k
      // agent-scope (coherent across the XCDs' L2s) relaxed status words: a word carries
      // its own value, nothing else has to become visible with it, so no release fence
      // (an agent-scope release writes back the whole L2: ~1 us per tile, measured)
      u64* st = status + (u64)k * smax;
      const u64 tag = (u64)epoch << 34;
      u32 excl = 0;
      if (tile > 0) {
        if (lane == 0)
          __hip_atomic_store(&st[tile], tag | (1ull << 32) | A, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        u32 top = tile;   // predecessors [0, top) not yet summed
        while (top > 0) {
          const bool has = lane < top;
          const u32 j = has ? top - 1 - lane : 0;   // lane 0 = nearest predecessor
          u64 w = 0;
          if (has) {
            do {
              w = __hip_atomic_load(&st[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } while ((w >> 34) != epoch || ((w >> 32) & 3) == 0);
          }
          const u64 incl = __ballot(has && ((w >> 32) & 3) == 2);
          // sum lanes up to (and including) the nearest inclusive prefix, or the window
          const u32 last = incl ? (u32)(__ffsll((unsigned long long)incl) - 1) : 63u;
          u32 v = (has && lane <= last) ? (u32)w : 0u;
          for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
          excl += v;
          if (incl) break;
          top = top > 64 ? top - 64 : 0;
        }
      }
      if (lane == 0) {
        __hip_atomic_store(&st[tile], tag | (2ull << 32) | (excl + A), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_excl[k] = excl;
        if (base + TILE >= n) tot[a.tot_slot + k] = excl + A;   // the last data tile
      }
    }
    __syncthreads();
#pragma clang loop unroll(full)
    for (int k = 0; k < NA; ++k) {
      if ((u32)k >= a.narr) continue;   // (continue, not break: a single-exit loop unrolls)
      u32 o0 = s_excl[k] + off[k];
      u32* out = (NA <= 4 ? a.out[k & 3] : a.out[k & 1] + (u64)(k >> 1) * a.stride) + lo;
      if (EPT == 4) {
        uint4 o;
        o.x = o0; o.y = o0 + v[k][0]; o.z = o.y + v[k][EPT > 1 ? 1 : 0]; o.w = o.z + v[k][EPT > 2 ? 2 : 0];
        if (i + 3 < n && !(((uintptr_t)(out + i)) & 15)) *(uint4*)(out + i) = o;
        else {
          if (i < n) out[i] = o.x;
          if (i + 1 < n) out[i + 1] = o.y;
          if (i + 2 < n) out[i + 2] = o.z;
          if (i + 3 < n) out[i + 3] = o.w;
        }
      } else {
#pragma clang loop unroll(full)
        for (int e = 0; e < EPT; ++e) {
          if (i + e < n) out[i + e] = o0;
          o0 += v[k][e];
        }
      }
    }
  }
  if (last_block && tid == 0) {   // every block has its ticket: reset for the next launch
    atomicExch(&ctl[0], 0u);
    atomicExch(&ctl[1], epoch + 1);
  }
  return data && base + TILE >= n;
}

template <int NA, int EPT>
__global__ __launch_bounds__(1024) void k_scan(ScanArgs a, u32* tot, u64* status, u32* ctl, u32 smax) {
  (void)scan_tile<NA, EPT>(a, tot, status, ctl, smax);
}

// the route phase's scan (pub_nq, pub_slot, pub_routed, pub_ret_sz) with the phase's
// body-log / message-table reservation done by the block of the last data tile once its
// totals are out (fused: k_route<1> used to reserve, so k_route<1> + k_store can be one)
DEV void log_reserve(const DS& d);
__global__ __launch_bounds__(1024) void k_scan_route(ScanArgs a, u32* tot, u64* status, u32* ctl, u32 smax, DS d) {
  const bool last = scan_tile<4, 4>(a, tot, status, ctl, smax);
  if (last) {
    __syncthreads();   // the totals (tot[0..3]) were written by lane 0 of waves 0..3
    if (threadIdx.x == 0) log_reserve(d);
  }
}

// ============================================================================ radix sort
// stable LSD radix sort of (key, val) u32 pairs, DB bits per pass (8, or 9..11 for keys
// of 9..11 bits in one pass instead of two);
// n from device.  Per-tile digit histograms; the last occupied tile to finish turns them
// into the offsets of the occupied tiles (fused k_rs_offsets).  hist and hscan are both
// tile-major (hist[t * D + digit], hscan[t * D + digit]): the tiles write and the offsets
// pass reads / writes contiguous words, and the queue starts (k_ring_plan / k_enqueue) are
// row 0.  The offsets block keeps up to RS_RT tiles' counts in registers: one round of
// loads, one block scan, one round of stores.
constexpr u32 RS_RT = 16;
template <int DB> struct RsNt { static constexpr u32 v = DB > 10 ? 1024u : (DB > 9 ? 512u : 256u); };
template <int DB>
DEV void rs_offsets(const u32* hist, u32* hscan, u32 T, u32* lds) {
  constexpr u32 NT = RsNt<DB>::v, D = 1u << DB, PER = D / NT;   // consecutive digits per thread
  const u32 d0 = threadIdx.x * PER;
  u32 tot[PER];
#pragma unroll
  for (u32 j = 0; j < PER; ++j) tot[j] = 0;
  if (T <= RS_RT) {
    u32 h[RS_RT][PER];
#pragma unroll
    for (u32 a = 0; a < RS_RT; ++a)
#pragma unroll
      for (u32 j = 0; j < PER; ++j) h[a][j] = a < T ? hist[a * D + d0 + j] : 0u;
#pragma unroll
    for (u32 a = 0; a < RS_RT; ++a)
#pragma unroll
      for (u32 j = 0; j < PER; ++j) tot[j] += h[a][j];
    u32 sum = 0;
#pragma unroll
    for (u32 j = 0; j < PER; ++j) sum += tot[j];
    u32 all;
    u32 run = block_scan<NT>(sum, lds, all);
#pragma unroll
    for (u32 j = 0; j < PER; ++j) { const u32 x = tot[j]; tot[j] = run; run += x; }   // digit starts
#pragma unroll
    for (u32 a = 0; a < RS_RT; ++a) {
      if (a >= T) break;
#pragma unroll
      for (u32 j = 0; j < PER; ++j) { hscan[a * D + d0 + j] = tot[j]; tot[j] += h[a][j]; }
    }
    return;
  }
  // many tiles: two passes over the histograms, RB tiles at a time
  constexpr u32 RB = 8;
  u32 t = 0;
  for (; t + RB <= T; t += RB) {
    u32 h[RB][PER];
#pragma unroll
    for (u32 a = 0; a < RB; ++a)
#pragma unroll
      for (u32 j = 0; j < PER; ++j) h[a][j] = hist[(t + a) * D + d0 + j];
#pragma unroll
    for (u32 a = 0; a < RB; ++a)
#pragma unroll
      for (u32 j = 0; j < PER; ++j) tot[j] += h[a][j];
  }
  for (; t < T; ++t) {
#pragma unroll
    for (u32 j = 0; j < PER; ++j) tot[j] += hist[t * D + d0 + j];
  }
  u32 sum = 0;
#pragma unroll
  for (u32 j = 0; j < PER; ++j) sum += tot[j];
  u32 all;
  u32 run = block_scan<NT>(sum, lds, all);
#pragma unroll
  for (u32 j = 0; j < PER; ++j) { const u32 x = tot[j]; tot[j] = run; run += x; }   // digit starts
  for (t = 0; t < T; ++t) {
    u32 h[PER];
#pragma unroll
    for (u32 j = 0; j < PER; ++j) h[j] = hist[t * D + d0 + j];
#pragma unroll
    for (u32 j = 0; j < PER; ++j) { hscan[t * D + d0 + j] = tot[j]; tot[j] += h[j]; }
  }
}

template <int DB>
__global__ __launch_bounds__(RsNt<DB>::v) void k_rs_hist(const u32* keys, const u32* np, u32 shift, u32* hist,
                                                        u32* hscan, u32* ticket, u32 ntiles) {
  constexpr u32 NT = RsNt<DB>::v, D = 1u << DB;
  __shared__ u32 cnt[D];
  __shared__ u32 lds[NT / 64 + 1];
  __shared__ u32 s_last;
  u32 tid = threadIdx.x, t = blockIdx.x;
  u32 n = *np;
  u32 T = (n + SORT_TILE - 1) / SORT_TILE;
  if (T > ntiles) T = ntiles;
  if (t >= T) return;   // only occupied tiles take part (and take a ticket)
  bool last = false;
  for (; t < T; t += gridDim.x) {   // tile-stride: the grid is capped below ntiles
    for (u32 k = tid; k < D; k += NT) cnt[k] = 0;
    __syncthreads();
    u32 base = t * SORT_TILE;
    for (u32 j = 0; j < SORT_TILE / NT; ++j) {
      u32 i = base + j * NT + tid;
      if (i < n) atomicAdd(&cnt[(keys[i] >> shift) & (D - 1)], 1u);
    }
    __syncthreads();
    // agent-coherent stores + a workgroup-scope release (wait for them) before the
    // ticket: no L2 writeback per tile (__threadfence: +11 us at 15 tiles, measured)
    for (u32 k = tid; k < D; k += NT)
      __hip_atomic_store(&hist[t * D + k], cnt[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    if (tid == 0) s_last = atomicAdd(ticket, 1u) == T - 1;
    __syncthreads();
    last = last || s_last;
  }
  if (!last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (tid == 0) *ticket = 0;
  rs_offsets<DB>(hist, hscan, T, lds);
}

template <int DB>
__global__ __launch_bounds__(256) void k_rs_scatter(const u32* kin, const u32* vin, u32* kout, u32* vout,
                                                    const u32* np, u32 shift, const u32* hscan,
                                                    u32 ntiles) {
  constexpr u32 D = 1u << DB;
  __shared__ u32 wc[4][D];
  const u32 tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const u32 n = *np;
  for (u32 t = blockIdx.x; t * SORT_TILE < n; t += gridDim.x) {   // tile-stride (capped grid)
    const u32 base = t * SORT_TILE;
    __syncthreads();   // wc of the previous tile
    for (u32 i = tid; i < 4 * D; i += 256) ((u32*)wc)[i] = 0;
    __syncthreads();
    u32 wbase = base + w * (SORT_TILE / 4);
    // pass 1: per-wave digit counts
    for (u32 c = 0; c < SORT_TILE / 256; ++c) {
      u32 i = wbase + c * 64 + lane;
      bool valid = i < n;
      u32 dg = valid ? (kin[i] >> shift) & (D - 1) : 0;
      u64 peers = __ballot(valid);
#pragma unroll
      for (u32 bb = 0; bb < DB; ++bb) {
        u64 m = __ballot((dg >> bb) & 1);
        peers &= ((dg >> bb) & 1) ? m : ~m;
      }
      bool leader = valid && ((peers & lanemask_lt()) == 0);
      if (leader) wc[w][dg] += __popcll(peers);
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    for (u32 dg = tid; dg < D; dg += 256) {
      u32 run = hscan[t * D + dg];
      for (u32 ww = 0; ww < 4; ++ww) { u32 x = wc[ww][dg]; wc[ww][dg] = run; run += x; }
    }
    __syncthreads();
    for (u32 c = 0; c < SORT_TILE / 256; ++c) {
      u32 i = wbase + c * 64 + lane;
      bool valid = i < n;
      u32 key = valid ? kin[i] : 0;
      u32 dg = (key >> shift) & (D - 1);
      u64 peers = __ballot(valid);
#pragma unroll
      for (u32 bb = 0; bb < DB; ++bb) {
        u64 m = __ballot((dg >> bb) & 1);
        peers &= ((dg >> bb) & 1) ? m : ~m;
      }
      u32 basepos = ((volatile u32*)wc[w])[dg];
      u32 rank = __popcll(peers & lanemask_lt());
      if (valid) {
        kout[basepos + rank] = key;
        vout[basepos + rank] = vin[i];
      }
      __builtin_amdgcn_wave_barrier();
      bool leader = valid && ((peers & lanemask_lt()) == 0);
      if (leader) ((volatile u32*)wc[w])[dg] = basepos + __popcll(peers);
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// ============================================================================ K6 route
// topic prefilter on MFMA: score[p][b] = keyvec[p] . patvec[b] over 256 int8 lanes;
// a pattern word contributes +32 iff its 32-bit word hash equals the key's.
typedef int v4i __attribute__((ext_vector_type(4)));
DEV void topic_tile(const DS& d, u32 i0, u32 j0, u32 jt, u32 ntb, u32 npub, u32 lane) {
  v4i acc = {0, 0, 0, 0};
  const i8* A = d.pub_keyvec + (u64)(i0 + (lane & 15)) * TOPIC_K + (lane >> 4) * 16;
  const i8* B = d.t_mat + (u64)(j0 + (lane & 15)) * TOPIC_K + (lane >> 4) * 16;
#pragma unroll
  for (int kk = 0; kk < TOPIC_K / 64; ++kk) {
    v4i a = *(const v4i*)(A + kk * 64);
    v4i bv = *(const v4i*)(B + kk * 64);
    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bv, acc, 0, 0, 0);
  }
  i32 ex = d.t_expect[j0 + (lane & 15)];
  u64 m0 = __ballot(acc[0] == ex), m1 = __ballot(acc[1] == ex);
  u64 m2 = __ballot(acc[2] == ex), m3 = __ballot(acc[3] == ex);
  if (lane < 16) {  // row = i0 + 4*g + r with g = lane/4, r = lane%4
    u32 g = lane >> 2, r = lane & 3;
    u64 mm = r == 0 ? m0 : r == 1 ? m1 : r == 2 ? m2 : m3;
    u32 rr = i0 + g * 4 + r;
    if (rr < npub) d.pub_match[(u64)rr * ntb + jt] = (u16)((mm >> (16 * g)) & 0xffff);
  }
}

// the topic prefilter tiles of one group of 16 publishes [g0, g0 + 16) (all binding tiles,
// spread over the block's 16 waves); tiles whose publishes all arrived routed (MF_ONEQ /
// MF_RESTORE) or are not topic-routed have nothing to match.  The rows are written to
// pub_match (global: k_route_store re-reads them for publishes with > 8 queues) and made
// visible to the block's waves before they route.
DEV void topic_group(const DS& d, u32 g0, u32 n, u32 w, u32 lane) {
  // the prefilter tiles of the bindings in use only (the tables are packed from row 0): a
  // step of a few publishes on a 4096-row table cost ~68 us here (profiles/r5_coldprof/)
  const u32 nused = d.t_count[0] < d.tb_pad ? d.t_count[0] : d.tb_pad;
  const u32 ntb = d.tb_max ? d.tb_pad >> 4 : 0u;   // (pub_match row stride: every tile)
  const u32 nt = d.tb_max ? (nused + 15) >> 4 : 0u;
  if (nt == 0) return;
  const u32 pi = g0 + lane;
  const bool need = lane < 16 && pi < n && !(d.pubs[pi].flags & (MF_ONEQ | MF_RESTORE));
  if (!__ballot(need)) return;
  for (u32 jt = w; jt < nt; jt += 16) topic_tile(d, g0, jt * 16, jt, ntb, n, lane);
}


// exact check behind an MFMA prefilter hit: same word count (checked) and every non-'*'
// pattern word byte-equal to the key word at its position.  Word offsets are precomputed
// (host: t_woff, decode: pub_kwoff), so the compares of all words issue together instead
// of walking both strings byte by byte.
// bytes of a publish: the step's work buffer, or for a record imported from another
// rank the all-to-all receive buffer itself (k_import_route copies nothing)
DEV const u8* pub_src(const DS& d, const Pub& pb) { return (pb.flags & MF_IMPORTED) ? d.recv_pay : d.work; }

// word i (offset << 8 | length) of a row of TOPIC_WORDS u16 held in one 16-byte load
DEV u32 woff_at(const uint4& v, u32 i) {
  const u32 w = i < 2 ? v.x : i < 4 ? v.y : i < 6 ? v.z : v.w;
  return (w >> (16 * (i & 1))) & 0xffffu;
}

// a binding is a candidate for a publish when its pattern needs the full matcher (flags
// bit 0: '#', long keys) or the word counts agree and the MFMA prefilter bit is set: two
// small loads per binding lane (flags, prefilter row), nothing else for the non-candidates
DEV bool topic_cand(const DS& d, const Pub& pb, u32 pidx, u32 t, u32& fl) {
  fl = d.t_flags[t];
  const u16 mw = d.pub_match[(u64)pidx * (d.tb_pad >> 4) + (t >> 4)];
  return (fl & 1) || ((((fl >> 8) & 0xffu) == pb.nwords) && ((mw >> (t & 15)) & 1));
}

// exact check of a candidate: both word-offset rows (one 16-byte load each) and the
// pattern offset in one round, the word lengths checked without memory, then every byte
// compare issued together (was: word offsets one by one, each a round trip)
DEV bool topic_verify(const DS& d, const Pub& pb, u32 pidx, u32 t, u32 fl) {
  const uint4 pw = *(const uint4*)(d.t_woff + (u64)t * TOPIC_WORDS);
  const uint4 kw = *(const uint4*)(d.pub_kwoff + (u64)pidx * TOPIC_WORDS);
  const u32 kb = d.t_kb_off[t];
  if (fl & 1)   // pattern the prefilter cannot express: full matcher
    return topic_match(d.kpool + kb, d.t_kb_len[t], pub_src(d, pb) + pb.rk_off, pb.rk_len, d.hash_wildcard != 0);
  const u32 nw = pb.nwords < TOPIC_WORDS ? pb.nwords : TOPIC_WORDS;
  const u32 star = (fl >> 16) & 0xffu;
  bool lens_ok = true;
#pragma unroll
  for (u32 i = 0; i < TOPIC_WORDS; ++i)
    if (i < nw && !((star >> i) & 1)) lens_ok &= (woff_at(pw, i) & 255) == (woff_at(kw, i) & 255);
  if (!lens_ok) return false;
  const u8* pat = d.kpool + kb;
  const u8* key = pub_src(d, pb) + pb.rk_off;
  u32 diff = 0;
#pragma unroll
  for (u32 i = 0; i < TOPIC_WORDS; ++i) {
    if (i >= nw || ((star >> i) & 1)) continue;
    const u32 pe = woff_at(pw, i), ke = woff_at(kw, i);
    const u32 len = pe & 255;
    const u8* a = pat + (pe >> 8);
    const u8* b = key + (ke >> 8);
    for (u32 k0 = 0; k0 < len; k0 += 8) {
#pragma unroll
      for (u32 j = 0; j < 8; ++j)
        if (k0 + j < len) diff |= (u32)(a[k0 + j] ^ b[k0 + j]);
    }
  }
  return diff == 0;
}

DEV i32 direct_find(const DS& d, const Pub& pb) {
  u64 k = pb.keyhash ^ (u64(pb.exch) * 0x9E3779B97F4A7C15ULL);
  u32 mask = d.dhash_mask;
  for (u32 j = 0; j <= mask; ++j) {
    u32 s = (u32)(k + j) & mask;
    i32 ex = d.d_exch[s];
    if (ex < 0) return -1;
    if (ex == pb.exch && d.d_key[s] == k &&
        word_eq(d.kpool + d.d_kb_off[s], d.d_kb_len[s], pub_src(d, pb) + pb.rk_off, pb.rk_len))
      return (i32)s;
  }
  return -1;
}

// pass 0: count queues; pass 1: write pairs
// Publishes [tot[RANGE_LO], tot[RANGE_HI]): phase 0 = the step's own, phase 1 = records
// imported from other ranks (sharded queues; only locally owned queues are emitted).
// One wave per publish: the lanes walk the exchange's candidate list (direct queue list,
// fanout list, or topic bindings with their MFMA prefilter bits) 64 entries at a time, so
// a publish costs a few dependent loads instead of one serial chain per binding.
DEV u32 wave_or(u32 v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o);
  return v;
}

template <int PASS>
struct RouteAcc {
  u32 nq = 0, nq_all = 0, rmask = 0;
  u32 nrem = 0, rq = INVALID;   // remote queues matched, the first of them
  bool has_cons = false;
};

// emit one candidate queue per lane (valid lanes), preserving lane order.  qo / qc: the
// queue's owner and consumer count when the caller loaded them already (INVALID: load)
template <int PASS>
DEV void route_emit(const DS& d, RouteAcc<PASS>& a, u32 p, u32 wbase, u32 srank, u32 q, bool valid, u32 lane,
                    u32 qo = INVALID, u32 qc = INVALID) {
  const u32 me = d.my_rank;
  u32 owner = (valid && d.world > 1) ? (qo != INVALID ? qo : d.q_owner[q]) : me;
  bool remote = valid && owner != me;
  bool local = valid && !remote;
  a.rmask |= wave_or(remote ? (1u << owner) : 0u);
  const u64 rm = __ballot(remote);
  if (rm) {
    if (a.rq == INVALID) a.rq = (u32)__shfl((int)q, (int)(__ffsll((unsigned long long)rm) - 1));
    a.nrem += (u32)__popcll(rm);
  }
  u64 lm = __ballot(local);
  bool cons = local && (qc != INVALID ? qc : d.q_cons_n[q]) != 0;
  if (__ballot(cons || remote)) a.has_cons = true;
  u32 pos = a.nq + (u32)__popcll(lm & lanemask_lt());
  if (local) {
    if (PASS) {
      if (wbase + pos >= d.pair_max) return;   // pair table full: store_one trims refcnt
      d.pair_k[0][wbase + pos] = (q << d.rank_bits) | srank;
      d.pair_v[0][wbase + pos] = p;
    } else if (pos < 8) {
      d.pub_qc[(u64)p * 8 + pos] = q;
    }
  }
  a.nq += (u32)__popcll(lm);
  a.nq_all += (u32)__popcll(__ballot(valid));
}

template <int PASS>
DEV void route_one(const DS& d, u32 p, u32 lane) {
  Pub& pb = d.pubs[p];
  // pass 0 of an imported record that arrived with its queue ran in import_one
  if (PASS == 0 && (pb.flags & MF_IMPORTED) && (pb.flags & (MF_ONEQ | MF_RESTORE))) return;
  const u32 wbase = PASS ? d.tot[TS_PAIR_BASE] + d.pub_pair_off[p] : 0;
  // pair key = queue << rank_bits | (source rank >= this rank) (engine.hip): with the
  // stable sort and the generation order (own publishes, then imports by source rank) a
  // queue's messages are ordered by (source rank, connection, publish order) whichever
  // rank owns it
  const u32 srank = d.rank_bits ? (((pb.flags & MF_IMPORTED) ? pb.pad : d.my_rank) >= d.my_rank ? 1u : 0u) : 0u;
  if (PASS == 1) {
    if (lane == 0 && d.pub_ret_sz[p]) atomicMin(&d.conn_ret_min[pb.conn], d.pub_ret_off[p]);
    u32 nq0 = d.pub_nq[p];
    if (nq0 == 0) return;
    if (wbase >= d.pair_max) return;  // capacity: log_reserve clamps the pair count
    const u32 fit = d.pair_max - wbase < nq0 ? d.pair_max - wbase : nq0;
    if (nq0 <= 8) {  // routing result cached by pass 0
      if (lane < fit) {
        d.pair_k[0][wbase + lane] = (d.pub_qc[(u64)p * 8 + lane] << d.rank_bits) | srank;
        d.pair_v[0][wbase + lane] = p;
      }
      return;
    }
  }
  RouteAcc<PASS> a;
  const i32 ex = pb.exch;
  if (pb.flags & (MF_RESTORE | MF_ONEQ)) {   // recovered / origin-routed: exactly its queue
    route_emit<PASS>(d, a, p, wbase, srank, (u32)pb.keyhash, lane == 0, lane);
  } else if (ex >= 0) {
    u32 xt = d.x_type[ex];
    if (xt == EX_DIRECT || xt == EX_FANOUT) {
      u32 o = 0, c = 0;
      const u32* list;
      if (xt == EX_DIRECT) {
        i32 s = lane == 0 ? direct_find(d, pb) : 0;
        s = __shfl(s, 0);
        if (s >= 0) { o = d.d_q_off[s]; c = d.d_q_n[s]; }
        list = d.d_q;
      } else {
        o = d.x_fan_off[ex]; c = d.x_fan_n[ex];
        list = d.fan_q;
      }
      for (u32 k0 = 0; k0 < c; k0 += 64) {
        bool v = k0 + lane < c;
        u32 q = v ? list[o + k0 + lane] : 0;
        route_emit<PASS>(d, a, p, wbase, srank, q, v, lane);
      }
    } else {
      u32 o = d.x_t_off[ex], c = d.x_t_n[ex];
      u32 lastq = INVALID;
      for (u32 k0 = 0; k0 < c; k0 += 64) {
        bool v = k0 + lane < c;
        u32 t = o + k0 + lane;
        u32 q = INVALID, fl = 0, qo = INVALID, qc = INVALID;
        bool hit = false;
        if (v) {
          q = d.t_queue[t];
          if (topic_cand(d, pb, p, t, fl)) {
            // the queue's owner / consumer count load alongside the exact check's loads
            qo = d.world > 1 ? d.q_owner[q] : d.my_rank;
            qc = d.q_cons_n[q];
            hit = topic_verify(d, pb, p, t, fl);
          }
        }
        // bindings are sorted by queue: a queue is emitted once, by its first hit
        u64 hm = __ballot(hit);
        u64 below = hm & lanemask_lt();
        u32 qb = (u32)__shfl((int)q, below ? 63 - __clzll(below) : 0);  // nearest lower hit
        u32 qtop = (u32)__shfl((int)q, hm ? 63 - __clzll(hm) : 0);     // highest hit
        bool emit = hit && (below ? qb : lastq) != q;
        route_emit<PASS>(d, a, p, wbase, srank, q, emit, lane, qo, qc);
        if (hm) lastq = qtop;
      }
    }
  }
  if (PASS == 0 && lane == 0) {
    u32 nq = a.nq, rmask = a.rmask;
    u32 ret = 0;
    if (!(pb.flags & MF_IMPORTED))   // a single remote queue travels with the record (MF_ONEQ)
      pb.xid = a.nrem == 1 ? (u64)a.rq : ~0ull;
    if (pb.flags & MF_IMPORTED) {
      rmask = 0;  // imported records are never forwarded again
    } else if (ex < 0 && !(pb.flags & MF_RESTORE)) {
      atomicAdd(&d.ctr->n_unknown_exchange, 1u);
      u32 ri = atomicAdd(&d.ctr->n_ctrl, 1u);
      CtrlRec rec;
      rec.conn = pb.conn; rec.off = INVALID; rec.len = 404; rec.seg = pb.chslot;
      if (ri < d.seg_max * 2) d.ctrl_rec[ri] = rec;
    } else if (a.nq_all == 0) {
      atomicAdd(&d.ctr->n_unroutable, 1u);
      if (pb.flags & MF_MANDATORY) ret = 312;
    } else if ((pb.flags & MF_IMMEDIATE) && !a.has_cons) {
      ret = 313;
      nq = 0;  // spec behaviour: not enqueued (SURVEY A.Q16/CHANGES.md)
    }
    d.pub_ret[p] = ret;
    if (d.world > 1) d.pub_rmask[p] = ret ? 0 : rmask;
    u32 meta = align16(pb.ex_len + pb.rk_len + pb.props_len);
    u32 slot = nq ? align16(meta + pb.body_size) : 0;
    d.pub_nq[p] = nq;
    d.pub_slot[p] = slot;
    d.pub_routed[p] = nq ? 1 : 0;
    pb.nq = nq;
    pb.slot_bytes = slot;
    u32 rsz = 0;
    if (ret) {
      // bytes in the connection's return region; the offset comes from the publish-order
      // scan of pub_ret_sz (returns keep publish order within a connection)
      u32 tl = ret == 312 ? 49u : 72u;  // reply texts (ErrorCodes.scala:23-31)
      u32 sz = (8 + 4 + 2 + 1 + tl + 1 + pb.ex_len + 1 + pb.rk_len) /*method*/ +
               (8 + 12 + pb.props_len) /*header*/;
      u32 fm = d.conn_frame_max[pb.conn];
      u32 fmb = fm ? fm - 8 : 0xffffffffu;
      u32 nb = pb.body_size ? (pb.body_size + fmb - 1) / fmb : 0;
      sz += pb.body_size + 8 * nb;
      atomicAdd(&d.conn_ret_bytes[pb.conn], sz);
      rsz = sz;
      u32 ri = atomicAdd(&d.ctr->n_returns, 1u);
      if (ri < d.pub_max) d.ret_list[ri] = p;
    }
    d.pub_ret_sz[p] = rsz;
  }
}

// routing pass 0 (count queues, destination ranks) of the step's own publishes, 16 per
// 1024-thread block: the group's topic prefilter tiles on MFMA (fused k_topic_mfma), then
// one wave per publish.  Pass 1 runs fused with the store (k_route_store) after
// k_scan_route reserved the phase's log region.  The imports' pass 0 is k_import_route.
#ifndef ROUTE_WPE   // k_route occupancy target: 8 (two blocks per CU, 64 VGPRs, 12 VGPRs spilled)
#define ROUTE_WPE 8     // or 4 (one block per CU, no spill): A/B through CHANAMQ_DP_SO
#endif
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(ROUTE_WPE))) void k_route(DS d) {
  // the wave index as a scalar: each wave's publish index, and every pointer derived from
  // it, then lives in SGPRs (as a VGPR value it pushed the wave router past 64 VGPRs and
  // into scratch)
  const u32 lane = lane_id(), w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 lo = d.tot[TS_RANGE_LO];
  u32 n = d.tot[TS_RANGE_HI];
  if (n > d.pub_cap) n = d.pub_cap;
  // a block past the step's publishes leaves before any per-wave set-up: the grid is sized
  // for capacity (2048 blocks), and the register allocator spills loop-invariant state to
  // scratch in the prologue -- 1 KB of HBM writes per idle wave otherwise (PMC WRITE_SIZE)
  if (lo + blockIdx.x * 16 >= n) return;
  for (u32 g0 = lo + blockIdx.x * 16; g0 < n; g0 += gridDim.x * 16) {
    topic_group(d, g0, n, w, lane);
    __threadfence_block();
    __syncthreads();
    if (g0 + w < n) route_one<0>(d, g0 + w, lane);
    __syncthreads();   // the next group's tiles overwrite nothing this group reads, but keep waves together
  }
}

// reserve the step's contiguous body-log region and message-table indices
DEV void log_reserve(const DS& d) {
  u32 total = d.tot[1];     // slot bytes
  u32 routed = d.tot[2];    // routed messages
  u32 np = d.tot[TS_PAIR_BASE] + d.tot[0];
  d.tot[TS_PAIR_N] = np < d.pair_max ? np : d.pair_max;
  d.ctr->n_pairs = d.tot[TS_PAIR_N];
  // snowflake virtual position base for this step (ID_SLOT_BITS slots per wall-clock ms):
  // never below the step's clock (was k_marks; idempotent for a second routing phase)
  const u64 floor_pos = d.in->id_ms << ID_SLOT_BITS;
  const u64 cur = *d.id_next > floor_pos ? *d.id_next : floor_pos;
  *d.id_base = cur;
  *d.id_next = cur + routed;
  u64 head = *d.log_head, tail = *d.log_tail;
  u64 phys = head % d.log_bytes;
  if (phys + total > d.log_bytes) head += d.log_bytes - phys;
  bool ok = (head + total - tail <= d.log_bytes) && routed <= *d.msg_free_top;
  if (!ok || total == 0) {
    *d.log_step_base = ok ? head : INVALID;
    if (!ok) d.ctr->n_dropped_nomem += routed;
    return;
  }
  *d.log_step_base = head;
  *d.log_head = head + total;
  d.tot[8] = *d.msg_free_top;
  *d.msg_free_top = d.tot[8] - routed;
  d.ctr->n_routed_msgs += routed;
  atomicAdd((unsigned long long*)d.live_bytes, (unsigned long long)total);
}

// live bytes per log block (fused k_live_add), by one wave: the phase's slots are
// contiguous from the step base (slot p at base + pub_slot_off[p]) and a slot counts in
// the block where it starts, as release_msg subtracts it.  Lane l owns log block b0 + l:
// its bytes = S(end of the block) - S(start), S(x) = pub_slot_off of the first slot
// starting at or after x (a prefix sum; binary search, all lanes in parallel).
DEV void live_add_blocks(const DS& d, u32 lane) {
  const u64 head = *d.log_step_base;
  const u32 total = d.tot[1];
  if (head == INVALID || total == 0) return;
  const u32 lo = d.tot[TS_RANGE_LO];
  u32 hi = d.tot[TS_RANGE_HI];
  if (hi > d.pub_cap) hi = d.pub_cap;
  const u64 b0 = head / d.log_block, b1 = (head + total - 1) / d.log_block;
  for (u64 g = b0; g <= b1; g += 64) {
    const u64 bk = g + lane;
    u64 s_end = 0, s_beg = 0;
    if (bk <= b1) {
      auto S = [&](u64 x) -> u64 {
        u32 a = lo, b = hi;
        while (a < b) { u32 mid = (a + b) >> 1; if ((u64)d.pub_slot_off[mid] < x) a = mid + 1; else b = mid; }
        return a < hi ? (u64)d.pub_slot_off[a] : (u64)total;
      };
      s_end = bk == b1 ? (u64)total : S((bk + 1) * d.log_block - head);
      s_beg = bk == b0 ? 0 : S(bk * d.log_block - head);
      if (s_end > s_beg)
        atomicAdd((unsigned long long*)&d.log_live[bk % d.n_log_blocks], (unsigned long long)(s_end - s_beg));
    }
  }
}

// one wave per publish: write its queue pairs (route pass 1), then allocate the message,
// fill its MsgEnt and copy exchange / rk / props / body into the log (fused k_route<1> +
// k_store: one pass over the phase's publishes)
DEV void store_one_pre(const DS& d, u32 p, u32 lane, const Pub& pb, u32 nq, u32 rr, u32 soff, u32 wbase);
DEV void live_add_blocks(const DS& d, u32 lane);
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void k_route_store(DS d, u32 marks) {
  u32 lane = lane_id();
  if (blockIdx.x == 0 && threadIdx.x < 64) live_add_blocks(d, lane);
  // phase 0 (the step's own commands): K9 ack marks + K10 confirm counts (fused k_marks)
  if (marks) marks_range(d, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x);
  u32 n = d.tot[TS_RANGE_HI];
  if (n > d.pub_cap) n = d.pub_cap;
  const u32 nw = (gridDim.x * blockDim.x) >> 6;
  // (wave-uniform, made scalar: the publish's loads and pointers stay in SGPRs)
  const u32 wave = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  for (u32 p = d.tot[TS_RANGE_LO] + wave; p < n; p += nw) {
    // the store's loads go out before pass 1's pair stores (which the compiler cannot
    // move them past: every table is a global pointer of DS), one round instead of two
    const Pub pb = d.pubs[p];
    const u32 nq = d.pub_nq[p];
    const u32 rr = d.pub_routed_rank[p];
    const u32 soff = d.pub_slot_off[p];
    const u32 wbase = d.tot[TS_PAIR_BASE] + d.pub_pair_off[p];
    route_one<1>(d, p, lane);
    store_one_pre(d, p, lane, pb, nq, rr, soff, wbase);
  }
}

DEV void store_one_pre(const DS& d, u32 p, u32 lane, const Pub& pb, u32 nq, u32 rr, u32 soff, u32 wbase) {
  if (nq == 0) return;
  u64 base = *d.log_step_base;
  if (base == INVALID) {   // body log / message table full: dropped, confirmed with Basic.Nack
    if (lane == 0) {
      d.pubs[p].msg = INVALID;
      if (pb.chslot != INVALID) d.ch_pub_fail[pb.chslot] = 1u;
    }
    return;
  }
  u32 msg = d.msg_free[d.tot[8] - 1 - rr];
  u64 off = base + soff;
  u8* slot = d.log + (off % d.log_bytes);
  const u8* w = pub_src(d, pb);
  u32 meta = align16(pb.ex_len + pb.rk_len + pb.props_len);
  if ((pb.flags & (MF_IMPORTED | MF_SLOTFMT)) == (MF_IMPORTED | MF_SLOTFMT)) {
    // a record already in slot layout, 16-aligned on both sides: one vector copy
    const uint4* src = (const uint4*)(w + pb.ex_off);
    uint4* dst = (uint4*)slot;
    for (u32 i = lane; i < (pb.slot_bytes >> 4); i += 64) dst[i] = src[i];
  } else {
    wave_copy(slot, w + pb.ex_off, pb.ex_len);
    wave_copy(slot + pb.ex_len, w + pb.rk_off, pb.rk_len);
    wave_copy(slot + pb.ex_len + pb.rk_len, w + pb.props_off, pb.props_len);
    u32 bo = meta;
    for (u32 k = 0; k < pb.nfrag; ++k) {
      Frag fg = d.frags[pb.frag0 + k];
      wave_copy(slot + bo, w + fg.off, fg.len);
      bo += fg.len;
    }
  }
  if (lane == 0) {
    MsgEnt m;
    m.log_off = off;
    u64 pos = (*d.id_base) + rr;
    m.msg_id = (pb.flags & MF_RESTORE) ? pb.xid : snowflake_id(pos, d.in->worker);
    m.ts_ms = pb.ts_ms;
    m.slot_bytes = pb.slot_bytes;
    m.body_len = pb.body_size;
    m.body_off = meta;
    m.props_len = (u16)pb.props_len;
    m.ex_len = (u8)pb.ex_len;
    m.rk_len = (u8)pb.rk_len;
    // pairs past the pair table were not written (route_one): those queues never get
    // the message, so it holds only the references that were enqueued, and the
    // publisher gets Basic.Nack
    const u32 fit = wbase >= d.pair_max ? 0u : (d.pair_max - wbase < pb.nq ? d.pair_max - wbase : pb.nq);
    m.refcnt = (i32)(fit ? fit : 1u);
    m.flags = pb.flags;
    m.pub_step = (u32)d.in->step;
    m.pad = 0;
    m.href = (pb.flags & (MF_HREF | MF_IMPORTED)) == MF_HREF ? d.in->ingress_host + pb.pad : 0ull;
    d.msgs[msg] = m;
    u32 pmsg = msg;
    if (fit < pb.nq) {
      atomicAdd(&d.ctr->n_ring_full, pb.nq - fit);
      if (pb.chslot != INVALID) d.ch_pub_fail[pb.chslot] = 1u;
    }
    if (!fit) {   // freed by k_post: this kernel's waves are still popping the free list
      pmsg = INVALID;
      d.defer_free[atomicAdd(&d.tot[TS_NDEFER], 1u)] = msg;
    }
    d.pubs[p].msg = pmsg;
  }
}

// ============================================================================ sharded queues
// Cross-rank exchange of publishes (SURVEY §3.4 / BASELINE config 3).  Each queue has one
// owning rank; bindings are replicated.  Phase A (the step's own publishes) emits pairs for
// local queues and marks remote owners in pub_rmask; the packers below serialise each such
// publish once per destination rank into [RDesc][payload] send buffers, laid out
// destination-major so one RCCL all_to_all_single moves them.  Phase B imports the
// received records as publishes and routes them against local queues only.

// Per-destination record / byte offsets of the step's own publishes (phase A), without
// any inter-block waiting: a block per 1024-publish tile ranks its records per wave and
// destination (ballot: records, shuffle scan: payload bytes), scans the 16 waves' totals
// in LDS and writes tile-relative offsets for the destinations each publish goes to, plus
// the tile's 2W aggregates.  The last tile to finish (ticket) turns the aggregates into
// per-tile prefixes (one wave per value, 64 tiles per round) and the totals
// (tot[TS_XSCAN + 2r], tot[TS_XSCAN + 2r + 1]); k_pack adds the prefix of its tile.
// The tile aggregates are agent-coherent relaxed stores ordered before the ticket by a
// workgroup-scope release: no L2 writeback per tile.
constexpr u32 PK_TILE = 1024;
__global__ __launch_bounds__(1024) void k_pack_scan(DS d, u32* agg, u32* ticket) {
  __shared__ u32 wtot[16][2 * WORLD_MAX];
  __shared__ u32 s_last;
  const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  u32 n = d.ctr->n_pubs;
  if (n > d.pub_max) n = d.pub_max;
  const u32 W = d.world, V = 2 * W;
  const u32 T = n ? (n + PK_TILE - 1) / PK_TILE : 1;   // tile 0 always runs (publishes totals)
  const u32 tile = blockIdx.x;
  if (tile >= T) return;
  const u32 p = tile * PK_TILE + tid;
  u32 m = 0, sz = 0;
  if (p < n) {
    m = d.pub_rmask[p];
    if (m) {
      const Pub& pb = d.pubs[p];
      sz = align16(align16(pb.ex_len + pb.rk_len + pb.props_len) + pb.body_size);   // slot layout
    }
  }
  u32 myc[WORLD_MAX], myb[WORLD_MAX];
#pragma unroll
  for (u32 r = 0; r < WORLD_MAX; ++r) {
    myc[r] = myb[r] = 0;
    if (r >= W) continue;
    const u32 bit = (m >> r) & 1u;
    const u64 bal = __ballot(bit);
    myc[r] = (u32)__popcll(bal & lanemask_lt());
    const u32 v = bit ? sz : 0u;
    u32 x = v;
#pragma unroll
    for (u32 o = 1; o < 64; o <<= 1) {
      const u32 y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    myb[r] = x - v;
    const u32 bt = (u32)__shfl((int)x, 63);
    if (lane == 0) { wtot[w][2 * r] = (u32)__popcll(bal); wtot[w][2 * r + 1] = bt; }
  }
  __syncthreads();
  if (tid < V) {   // value tid: exclusive offsets of the 16 waves, the tile aggregate
    u32 run = 0;
    for (u32 ww = 0; ww < 16; ++ww) { const u32 t = wtot[ww][tid]; wtot[ww][tid] = run; run += t; }
    __hip_atomic_store(&agg[(u64)tile * 2 * WORLD_MAX + tid], run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
#pragma unroll
  for (u32 r = 0; r < WORLD_MAX; ++r) {
    if (r >= W || !((m >> r) & 1u)) continue;
    d.xp_cnt_off[(u64)r * d.pub_cap + p] = wtot[w][2 * r] + myc[r];
    d.xp_byt_off[(u64)r * d.pub_cap + p] = wtot[w][2 * r + 1] + myb[r];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // the agent-coherent agg stores are done
  __syncthreads();
  if (tid == 0) s_last = atomicAdd(ticket, 1u) == T - 1;
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (tid == 0) *ticket = 0;
  // aggregates -> per-tile exclusive prefixes, in place; totals
  for (u32 v = w; v < V; v += 16) {
    u32 carry = 0;
    for (u32 t0 = 0; t0 < T; t0 += 64) {
      const u32 t = t0 + lane;
      const u32 a = t < T ? __hip_atomic_load(&agg[(u64)t * 2 * WORLD_MAX + v], __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT) : 0u;
      u32 x = a;
#pragma unroll
      for (u32 o = 1; o < 64; o <<= 1) {
        const u32 y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      if (t < T) agg[(u64)t * 2 * WORLD_MAX + v] = carry + x - a;
      carry += (u32)__shfl((int)x, 63);
    }
    if (lane == 0) d.tot[TS_XSCAN + v] = carry;
  }
}

// one wave per local publish with remote owners: write one record per destination.
// Fused k_pack_bases: every block turns the per-rank totals of k_pack_scan into destination bases
// itself (one wave, lane r = rank r, one load round trip and a shuffle scan); block 0
// also publishes the send counts to the host-visible words
DEV void pack_one(const DS& d, u32 p, u32 lane, const u32* s_base);
__global__ __launch_bounds__(256) void k_pack(DS d) {
  __shared__ u32 s_base[2 * WORLD_MAX];
  const u32 tid = threadIdx.x, lane = lane_id();
  if (tid < 64) {
    const bool v = lane < d.world;
    const u32 c = v ? d.tot[TS_XSCAN + 2 * lane] : 0u, b = v ? d.tot[TS_XSCAN + 2 * lane + 1] : 0u;
    u32 sc = c, sb = b;
#pragma unroll
    for (u32 o = 1; o < WORLD_MAX; o <<= 1) {
      const u32 yc = __shfl_up(sc, o, 64), yb = __shfl_up(sb, o, 64);
      if (lane >= o) { sc += yc; sb += yb; }
    }
    if (v) { s_base[lane] = sc - c; s_base[WORLD_MAX + lane] = sb - b; }
    if (blockIdx.x == 0) {
      if (v) { d.xs_base[lane] = sc - c; d.xs_base[WORLD_MAX + lane] = sb - b; d.xchg[lane] = c; d.xchg[WORLD_MAX + lane] = b; }
      const u32 dsum = (u32)__shfl((int)sc, (int)d.world - 1), psum = (u32)__shfl((int)sb, (int)d.world - 1);
      if (lane == 0) d.xchg[4 * WORLD_MAX] = (dsum > d.xfer_desc_max || psum > d.xfer_bytes) ? 1u : 0u;
    }
  }
  __syncthreads();
  const u32 n = d.ctr->n_pubs, nw = (gridDim.x * blockDim.x) >> 6;
  for (u32 p = (blockIdx.x * blockDim.x + tid) >> 6; p < n; p += nw) pack_one(d, p, lane, s_base);
}

DEV void pack_one(const DS& d, u32 p, u32 lane, const u32* s_base) {
  u32 m = d.pub_rmask[p];
  if (!m) return;
  const Pub pb = d.pubs[p];
  const u8* w = d.work;
  while (m) {
    u32 r = __builtin_ctz(m);
    m &= m - 1;
    // tile prefix (k_pack_scan) + offset within the tile
    const u32* tp = d.pk_agg + (u64)(p / PK_TILE) * 2 * WORLD_MAX;
    u32 di = s_base[r] + tp[2 * r] + d.xp_cnt_off[(u64)r * d.pub_cap + p];
    u32 rel = tp[2 * r + 1] + d.xp_byt_off[(u64)r * d.pub_cap + p];
    u64 po = (u64)s_base[WORLD_MAX + r] + rel;
    // the record is laid out as the owner's body-log slot (MF_SLOTFMT)
    const u32 meta = align16(pb.ex_len + pb.rk_len + pb.props_len);
    u32 sz = align16(meta + pb.body_size);
    if (di >= d.xfer_desc_max || po + sz > d.xfer_bytes) continue;  // overflow flagged by k_pack_bases
    u8* o = d.send_pay + po;
    wave_copy(o, w + pb.ex_off, pb.ex_len);
    wave_copy(o + pb.ex_len, w + pb.rk_off, pb.rk_len);
    wave_copy(o + pb.ex_len + pb.rk_len, w + pb.props_off, pb.props_len);
    o += meta;
    for (u32 k = 0; k < pb.nfrag; ++k) {
      Frag fg = d.frags[pb.frag0 + k];
      wave_copy(o, w + fg.off, fg.len);
      o += fg.len;
    }
    if (lane == 0) {
      RDesc rd{};
      rd.pay_off = rel;
      rd.body_len = pb.body_size;
      rd.props_len = pb.props_len;
      rd.exch = pb.exch;
      rd.flags = (pb.flags & (MF_PERSIST | MF_HAS_TS)) | MF_SLOTFMT;
      if (pb.xid != ~0ull) {   // the owner skips re-routing: its one queue is known
        rd.flags |= MF_ONEQ;
        rd.tq = (u32)pb.xid;
      }
      rd.ex_len = (u8)pb.ex_len;
      rd.rk_len = (u8)pb.rk_len;
      rd.expire_ms = pb.expire_ms;
      rd.ts_ms = pb.ts_ms;
      d.send_desc[di] = rd;
    }
  }
}

// Phase B head: one kernel imports the received records and applies the received link
// acks (fused k_import_prep + k_link_acks).  Every block derives the per-source bases from
// the received counts (host-mapped xchg) itself -- one wave, lane r = source r, one load
// round trip and a shuffle scan -- and block 0 also publishes the import range for the
// kernels after it.  xr: [0,W) record bases, [W,2W) byte bases, [2W,3W) publish records
// of each source (the link deliveries after them have payload offsets past the publish
// bytes, [3W,4W): native exchange, engine.hip exchange()).  The same kernel runs routing
// pass 0 of the imports (fused k_topic_mfma + k_route): 16 records per 1024-thread block
// -- 16 threads import them, the block computes their topic tiles, one wave per record
// routes it (records that arrived with their queue were routed by import_one and return
// at once)
DEV void import_one(const DS& d, u32 i, const u32* xr);
DEV void link_ack_one(const DS& d, u32 i);
__global__ __launch_bounds__(1024) void k_import_route(DS d) {
  __shared__ u32 xr[4 * WORLD_MAX];
  __shared__ u32 s_n, s_k;
  const u32 tid = threadIdx.x;
  if (tid < 64) {
    const u32 lane = tid;
    const bool v = lane < d.world;
    const u32 cn = v ? d.xchg[XC_RECV_N + lane] : 0u, cb = v ? d.xchg[XC_RECV_B + lane] : 0u;
    const u32 an = v ? d.xchg[XC_RECV_AN + lane] : 0u, ab = v ? d.xchg[XC_RECV_AB + lane] : 0u;
    const u32 rk = (v && d.links) ? d.xchg[XC_RACK_N + lane] : 0u;
    u32 sn = cn, sb = cb, sk = rk;
#pragma unroll
    for (u32 o = 1; o < WORLD_MAX; o <<= 1) {
      const u32 yn = __shfl_up(sn, o, 64), yb = __shfl_up(sb, o, 64), yk = __shfl_up(sk, o, 64);
      if (lane >= o) { sn += yn; sb += yb; sk += yk; }
    }
    if (v) { xr[lane] = sn - cn; xr[WORLD_MAX + lane] = sb - cb; xr[2 * WORLD_MAX + lane] = an; xr[3 * WORLD_MAX + lane] = ab; }
    const u32 last = d.world - 1;
    const u32 dsum = (u32)__shfl((int)sn, (int)last), psum = (u32)__shfl((int)sb, (int)last);
    const u32 nk = (u32)__shfl((int)sk, (int)last);
    const bool fits = dsum <= d.import_max && psum <= d.import_bytes;
    const u32 ni = fits ? dsum : 0u;
    const u32 kcap = (d.world - 1) * d.lk_cap;
    const u32 nr = d.links ? (nk < kcap ? nk : kcap) : 0u;
    if (lane == 0) { s_n = ni; s_k = nr; }
    if (blockIdx.x == 0) {
      if (v)
        for (u32 k = 0; k < 4; ++k) d.xr_base[k * WORLD_MAX + lane] = xr[k * WORLD_MAX + lane];
      if (lane == 0) {
        if (!fits) d.ctr->n_dropped_nomem += dsum;
        d.tot[TS_NRACK] = nr;
        d.tot[TS_NIMPORT] = ni;
        d.tot[TS_IMPORT_BASE] = 0;   // imported bytes stay in the receive buffer (pub_src)
        d.tot[TS_RANGE_LO] = d.ctr->n_pubs;
        d.tot[TS_RANGE_HI] = d.ctr->n_pubs + ni;
        d.tot[TS_PAIR_BASE] = d.tot[TS_PAIR_N];
      }
    }
  }
  __syncthreads();
  const u32 n = s_n, nk = s_k;
  const u32 g = blockIdx.x * blockDim.x + tid, gs = gridDim.x * blockDim.x;
  for (u32 i = g; i < nk; i += gs) link_ack_one(d, i);
  const u32 base = d.ctr->n_pubs, lane = tid & 63, w = tid >> 6;
  for (u32 g0 = blockIdx.x * 16; g0 < n; g0 += gridDim.x * 16) {
    if (tid < 16 && g0 + tid < n) import_one(d, g0 + tid, xr);
    __threadfence_block();
    __syncthreads();
    topic_group(d, base + g0, base + n, w, lane);
    __threadfence_block();
    __syncthreads();
    if (g0 + w < n) route_one<0>(d, base + g0 + w, lane);
    __syncthreads();
  }
}

// one thread per received record -> imported Publish whose bytes stay in recv_pay (no
// copy: a thread builds the record's key hash / key vector, as k_decode does per publish)
DEV void import_one(const DS& d, u32 i, const u32* xr) {
  u32 src = 0;
  for (u32 r = 1; r < d.world; ++r)
    if (xr[r] <= i) src = r;
  const RDesc rd = d.recv_desc[i];
  const u32 lpart = i - xr[src] >= xr[2 * WORLD_MAX + src] ? xr[3 * WORLD_MAX + src] : 0u;
  const u32 roff = xr[WORLD_MAX + src] + lpart + rd.pay_off;
  const u32 wo = roff;   // offsets relative to recv_pay (MF_IMPORTED, pub_src)
  u32 pi = d.ctr->n_pubs + i;
  Pub pb;
  pb.conn = INVALID;
  pb.chslot = INVALID;
  pb.exch = rd.exch;
  pb.ex_off = wo;
  pb.ex_len = rd.ex_len;
  pb.rk_off = wo + rd.ex_len;
  pb.rk_len = rd.rk_len;
  pb.props_off = pb.rk_off + rd.rk_len;
  pb.props_len = rd.props_len;
  u32 fi = d.frag_max + i;  // imported bodies live past the step's own fragments
  d.frags[fi] = Frag{(rd.flags & MF_SLOTFMT) ? wo + align16(rd.ex_len + rd.rk_len + rd.props_len)
                                            : pb.props_off + rd.props_len, rd.body_len};
  pb.frag0 = fi;
  pb.nfrag = rd.body_len ? 1 : 0;
  pb.body_size = rd.body_len;
  pb.flags = rd.flags | MF_IMPORTED;
  pb.expire_ms = rd.expire_ms;
  pb.ts_ms = rd.ts_ms;
  const u8* key = d.recv_pay + roff + rd.ex_len;
  const bool routed = rd.flags & (MF_RESTORE | MF_ONEQ);   // target queue in tq, no matching
  pb.keyhash = routed ? (u64)rd.tq : fnv1a64_dev(key, rd.rk_len);
  pb.nwords = routed ? 0u : build_keyvec(d, key, rd.rk_len, pi);
  pb.nq = 0; pb.slot_bytes = 0; pb.msg = INVALID; pb.xid = rd.xid;
  pb.pad = src;  // source rank (pair ordering)
  if (rd.flags & MF_HOSTPUB) {   // the publisher's channel: confirm counting, Nack on a drop
    pb.chslot = rd.pad[0];
    pb.conn = rd.pad[1];
    if (pb.chslot < d.c_max * d.chpc && d.ch_confirm[pb.chslot]) atomicAdd(&d.ch_pub_cnt[pb.chslot], 1u);
  }
  if (routed) {
    // routing pass 0 for a record that arrived with its queue (what route_one<0> computes
    // for it: one local queue, no return, never forwarded); route_one<0> skips it
    const u32 q = rd.tq;
    const u32 nq = (d.world == 1 || d.q_owner[q] == d.my_rank) ? 1u : 0u;
    const u32 slot = nq ? align16(align16(pb.ex_len + pb.rk_len + pb.props_len) + pb.body_size) : 0u;
    pb.nq = nq;
    pb.slot_bytes = slot;
    d.pub_qc[(u64)pi * 8] = q;
    d.pub_nq[pi] = nq;
    d.pub_slot[pi] = slot;
    d.pub_routed[pi] = nq;
    d.pub_ret[pi] = 0;
    d.pub_ret_sz[pi] = 0;
    if (d.world > 1) d.pub_rmask[pi] = 0;
  }
  d.pubs[pi] = pb;
}

// ============================================================================ K7 enqueue
__global__ void k_qfirst(DS d, u32 src) {
  u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  u32 n = d.tot[TS_PAIR_N];
  if (i >= n) return;
  const u32* k = d.pair_k[src];
  const u32 rb = d.rank_bits;
  if (i == 0 || (k[i - 1] >> rb) != (k[i] >> rb)) d.q_first[k[i] >> rb] = i;
}

// publish p's entry at position `rank` of this step's entries for queue q (`last`: the
// queue's last pair, which moves q_tail); returns the message to release if the ring is full
// a pair's enqueue in two halves: every load (the publish, the queue's ring state), then
// the stores -- so a kernel can have the loads of several pairs in flight at once
struct EnqLoad {
  u32 msg = INVALID, flags = 0, chslot = INVALID;
  u64 head = 0, tail = 0, mask = 0, ring_off = 0;
  i64 expire_ms = 0, ttl = 0;
  bool durable = false;
};
DEV EnqLoad enq_load(const DS& d, u32 q, u32 p) {
  const Pub& pb = d.pubs[p];
  EnqLoad e;
  e.msg = pb.msg;
  e.flags = pb.flags;
  e.chslot = pb.chslot;
  e.expire_ms = pb.expire_ms;
  // the queue's last pair moves q_tail in this kernel: every pair reads the tail that
  // k_ring_plan recorded before the enqueue, never q_tail itself
  e.head = d.q_head[q];
  e.tail = d.q_enq_tail[q];
  e.mask = d.q_ring_mask[q];
  e.ring_off = d.q_ring_off[q];
  e.ttl = d.q_ttl[q];
  e.durable = d.persist && d.q_durable[q];
  return e;
}
DEV u32 enq_store(const DS& d, const EnqLoad& l, u32 q, u32 rank, bool last, PersistRec* pr) {
  const u64 cap = l.mask + 1;
  const u64 freec = cap - (l.tail - l.head);
  u32 drop = INVALID;
  if (l.msg == INVALID) return INVALID;
  if (rank < freec) {
    u64 pos = l.tail + rank;
    Desc ds;
    ds.msg = l.msg;
    ds.flags = (l.flags & MF_REDELIVERED) ? 1u : 0u;
    i64 e = l.expire_ms;
    if (l.ttl > 0) { i64 qe = d.in->now_ms + l.ttl; e = (e == 0 || qe < e) ? qe : e; }
    ds.expire_ms = e;
    d.ring[l.ring_off + (pos & l.mask)] = ds;
    if (l.durable && (l.flags & MF_PERSIST) && !(l.flags & MF_RESTORE)) {
      pr->msg = l.msg; pr->q = q; pr->qpos = pos; pr->expire_ms = e;
    }
  } else {
    drop = l.msg;
    if (l.chslot != INVALID) d.ch_pub_fail[l.chslot] = 1u;   // confirmed with Basic.Nack
  }
  if (last) {
    u64 cnt = rank + 1;
    u64 nt = l.tail + (cnt < freec ? cnt : freec);
    d.q_tail[q] = nt;
  }
  return drop;
}
DEV u32 enqueue_at(const DS& d, u32 q, u32 p, u32 rank, bool last, PersistRec* pr) {
  return enq_store(d, enq_load(d, q, p), q, rank, last, pr);
}
DEV u32 enqueue_one(const DS& d, u32 src, u32 i, u32 n, PersistRec* pr, u32 hs_ntiles) {
  const u32* kk = d.pair_k[src];
  const u32 rb = d.rank_bits;
  u32 q = kk[i] >> rb;
  u32 p = d.pair_v[src][i];
  // single-pass sort (queue|rank key <= 8 bits): the queue's first pair is where digit
  // (q << rank_bits) starts; otherwise k_qfirst recorded it
  u32 first = hs_ntiles ? d.hist_scan[q << rb] : d.q_first[q];
  return enqueue_at(d, q, p, i - first, (i + 1 == n) || (kk[i + 1] >> rb) != q, pr);
}

// ---- unbounded queues (QueueEntity.scala:271-316 keeps a growing Vector): before the
// step's enqueue, the last pair of every queue checks that the queue's ring holds this
// step's entries; if not, the ring moves to one of >= 2x the needed size taken from the
// ring pool (one bump pointer shared with the host's allocator), within the queue's
// max_capacity.  Positions stay absolute (entry pos lives at off + (pos & mask)), so
// unacked windows, requeues and store rows keep their queue offsets.
DEV void plan_queue(const DS& d, u32 q, u64 cnt);
DEV void ring_plan_one(const DS& d, u32 src, u32 hs_ntiles, u32 i, u32 n) {
  const u32* kk = d.pair_k[src];
  const u32 rb = d.rank_bits;
  const u32 q = kk[i] >> rb;
  if (i + 1 < n && (kk[i + 1] >> rb) == q) return;   // not the queue's last pair
  const u32 first = hs_ntiles ? d.hist_scan[q << rb] : d.q_first[q];
  plan_queue(d, q, (u64)(i - first) + 1);
}
// queue q takes cnt entries this step: record its tail before the enqueue, grow its ring
DEV void plan_queue(const DS& d, u32 q, u64 cnt) {
  const u64 head = d.q_head[q], tail = d.q_tail[q];
  d.q_enq_tail[q] = tail;
  const u64 mask = d.q_ring_mask[q], cap = mask + 1;
  const u64 need = tail - head + cnt;
  if (need <= cap) return;
  const u64 limit = d.q_max_cap[q] ? d.q_max_cap[q] : d.ring_pool;
  u64 want = cap;
  while (want < 2 * need && want * 2 <= limit) want *= 2;
  if (want <= cap) return;                            // at max_capacity: the overflow drops (nack)
  unsigned long long* top = (unsigned long long*)d.ring_top;
  u64 off = __hip_atomic_load(top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (true) {
    if (off + want > d.ring_pool) return;            // pool exhausted: drops (nack)
    u64 prev = atomicCAS(top, off, off + want);
    if (prev == off) break;
    off = prev;
  }
  RingMove mv;
  mv.q = q; mv.pad = 0;
  mv.old_off = d.q_ring_off[q]; mv.old_mask = mask;
  mv.new_off = off; mv.new_mask = want - 1;
  mv.head = head; mv.tail = tail;
  const u32 mi = atomicAdd(&d.tot[TS_NMOVE], 1u);
  d.moves[mi] = mv;                                  // mi < q_max: one move per queue
  d.q_ring_off[q] = off;
  d.q_ring_mask[q] = want - 1;
  const u32 gi = atomicAdd(&d.ctr->n_grow, 1u);      // the host reclaims the old ring
  if (gi < GROW_MAX) d.grow_h[gi] = mv;
  __threadfence();   // the move is visible to the last block of k_ring_plan (which copies)
}

// the last (occupied) block to finish copies every moved ring's live entries (fused
// k_ring_moves: growth is rare, so one block does it and the common step saves a launch)
// Grid-stride over the pairs with a capped grid (the graph's grid is sized for pair_max;
// a block per 256 pairs of the capacity would mostly launch waves with nothing to do)
__global__ __launch_bounds__(256) void k_ring_plan(DS d, u32 src, u32 hs_ntiles) {
  __shared__ u32 s_last;
  const u32 n = d.tot[TS_PAIR_N];
  u32 nb = (n + 255) / 256;
  if (nb > gridDim.x) nb = gridDim.x;   // blocks taking part
  if (blockIdx.x >= nb) return;
  for (u32 i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) ring_plan_one(d, src, hs_ntiles, i, n);
  // a thread that planned a ring move fenced it itself (rare); the common step only waits
  // for its own stores before the ticket (no L2 writeback per block)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(&d.tot[TS_RP_TICKET], 1u) == nb - 1;
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (threadIdx.x == 0) d.tot[TS_RP_TICKET] = 0;
  const u32 nm = d.tot[TS_NMOVE];
  for (u32 m = 0; m < nm; ++m) {
    const RingMove mv = d.moves[m];
    for (u64 pos = mv.head + threadIdx.x; pos < mv.tail; pos += 256)
      d.ring[mv.new_off + (pos & mv.new_mask)] = d.ring[mv.old_off + (pos & mv.old_mask)];
  }
}

__global__ void k_enqueue(DS d, u32 src, u32 hs_ntiles) {
  const u32 n = d.tot[TS_PAIR_N];
  const u32 stride = gridDim.x * blockDim.x;
  // whole waves iterate together (the wave collectives below need every lane)
  for (u32 b = blockIdx.x * blockDim.x; b < n; b += stride) {
    const u32 i = b + threadIdx.x;
    PersistRec pr;
    pr.msg = INVALID;
    u32 drop = i < n ? enqueue_one(d, src, i, n, &pr, hs_ntiles) : INVALID;
    wave_release(d, drop, drop != INVALID);
    if (drop != INVALID) atomicAdd(&d.ctr->n_ring_full, 1u);
    if (d.persist) {
      bool want = pr.msg != INVALID;
      u32 k = wave_reserve(&d.ctr->n_persist, want);
      if (want && k < d.persist_max) d.prec[k] = pr;
    }
  }
}

// ---- single-pass sort (queue | rank key <= 11 bits) with the enqueue fused: k_ring_plan
// and k_enqueue fold into the sort's two kernels.  The histogram's last block knows every
// queue's pair count (its digit range) and plans the rings; the scatter knows every pair's
// sorted position -- its rank in its queue -- and writes the ring entry itself, so the
// sorted pair arrays are never materialised.  Two launches a step instead of four.
DEV void plan_rings_block(const DS& d, const u32* hscan, u32 n, u32 D, u32 tid, u32 nt) {
  const u32 rb = d.rank_bits;
  for (u32 q = tid; q < d.q_max && (q << rb) < D; q += nt) {
    // the digit starts (row 0 of hscan) were stored by this block: agent-scope loads
    const u32 first = __hip_atomic_load(&hscan[q << rb], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const u32 nx = ((q + 1) << rb) < D
                       ? __hip_atomic_load(&hscan[(q + 1) << rb], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                       : n;
    if (nx > first) plan_queue(d, q, nx - first);
  }
  __syncthreads();
  const u32 nm = __hip_atomic_load(&d.tot[TS_NMOVE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!nm) return;   // (block-uniform) rings that grew: copy their live entries over
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  for (u32 m = 0; m < nm; ++m) {
    const RingMove mv = d.moves[m];
    for (u64 pos = mv.head + tid; pos < mv.tail; pos += nt)
      d.ring[mv.new_off + (pos & mv.new_mask)] = d.ring[mv.old_off + (pos & mv.old_mask)];
  }
}

template <int DB>
__global__ __launch_bounds__(RsNt<DB>::v) void k_rs_hist_plan(DS d, const u32* keys, const u32* np, u32* hist,
                                                             u32* hscan, u32* ticket, u32 ntiles) {
  constexpr u32 NT = RsNt<DB>::v, D = 1u << DB;
  __shared__ u32 cnt[D];
  __shared__ u32 lds[NT / 64 + 1];
  __shared__ u32 s_last;
  u32 tid = threadIdx.x, t = blockIdx.x;
  const u32 n = *np;
  u32 T = (n + SORT_TILE - 1) / SORT_TILE;
  if (T > ntiles) T = ntiles;
  if (T == 0) {   // no pairs: nothing to plan (the queues' tails stay)
    return;
  }
  if (t >= T) return;
  bool last = false;
  for (; t < T; t += gridDim.x) {
    for (u32 k = tid; k < D; k += NT) cnt[k] = 0;
    __syncthreads();
    const u32 base = t * SORT_TILE;
    for (u32 j = 0; j < SORT_TILE / NT; ++j) {
      const u32 i = base + j * NT + tid;
      if (i < n) atomicAdd(&cnt[keys[i] & (D - 1)], 1u);
    }
    __syncthreads();
    for (u32 k = tid; k < D; k += NT)
      __hip_atomic_store(&hist[t * D + k], cnt[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    if (tid == 0) s_last = atomicAdd(ticket, 1u) == T - 1;
    __syncthreads();
    last = last || s_last;
  }
  if (!last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (tid == 0) *ticket = 0;
  rs_offsets<DB>(hist, hscan, T, lds);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __syncthreads();
  plan_rings_block(d, hscan, n, D, tid, NT);
}

template <int DB>
__global__ __launch_bounds__(256) void k_rs_scatter_enq(DS d, const u32* kin, const u32* vin, const u32* np,
                                                       const u32* hscan) {
  constexpr u32 D = 1u << DB, CH = SORT_TILE / 256;   // CH items per lane
  __shared__ u32 wc[4][D];
  const u32 tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const u32 n = *np, rb = d.rank_bits;
  const u64 lt = lanemask_lt();
  for (u32 t = blockIdx.x; t * SORT_TILE < n; t += gridDim.x) {   // tile-stride (capped grid)
    const u32 base = t * SORT_TILE;
    __syncthreads();
    for (u32 i = tid; i < 4 * D; i += 256) ((u32*)wc)[i] = 0;
    __syncthreads();
    const u32 wbase = base + w * (SORT_TILE / 4);
    // the lane's CH pairs loaded at once, and kept: the rank pass and the enqueue reuse them
    // (was: each of the CH rounds re-read its pair, then walked its queue's state -- ~3
    // dependent memory trips a round, CH rounds in series: the kernel's 12-13 us floor)
    u32 key[CH], val[CH];
    u64 pe[CH];
#pragma unroll
    for (u32 c = 0; c < CH; ++c) {
      const u32 i = wbase + c * 64 + lane;
      key[c] = i < n ? kin[i] : 0u;
      val[c] = i < n ? vin[i] : 0u;
    }
#pragma unroll
    for (u32 c = 0; c < CH; ++c) {   // per-wave digit counts
      const bool valid = wbase + c * 64 + lane < n;
      const u32 dg = key[c] & (D - 1);
      u64 peers = __ballot(valid);
#pragma unroll
      for (u32 bb = 0; bb < DB; ++bb) {
        const u64 m = __ballot((dg >> bb) & 1);
        peers &= ((dg >> bb) & 1) ? m : ~m;
      }
      pe[c] = peers;
      if (valid && ((peers & lt) == 0)) wc[w][dg] += __popcll(peers);
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    for (u32 dg = tid; dg < D; dg += 256) {
      u32 run = hscan[t * D + dg];
      for (u32 ww = 0; ww < 4; ++ww) { const u32 x = wc[ww][dg]; wc[ww][dg] = run; run += x; }
    }
    __syncthreads();
    // every pair's position in digit order (LDS only), then every load the enqueue needs --
    // its queue's first pair / next digit start, the publish, the queue's ring state -- issued
    // together for the lane's CH pairs, then the ring stores
    u32 pos[CH];
#pragma unroll
    for (u32 c = 0; c < CH; ++c) {
      const bool valid = wbase + c * 64 + lane < n;
      const u32 dg = key[c] & (D - 1);
      const u32 basepos = ((volatile u32*)wc[w])[dg];
      pos[c] = basepos + __popcll(pe[c] & lt);
      __builtin_amdgcn_wave_barrier();
      if (valid && ((pe[c] & lt) == 0)) ((volatile u32*)wc[w])[dg] = basepos + __popcll(pe[c]);
      __builtin_amdgcn_wave_barrier();
    }
    EnqLoad el[CH];
    u32 first[CH], nx[CH];
#pragma unroll
    for (u32 c = 0; c < CH; ++c) {
      const bool valid = wbase + c * 64 + lane < n;
      const u32 q = key[c] >> rb;
      first[c] = valid ? hscan[q << rb] : 0u;
      nx[c] = valid ? (((q + 1) << rb) < D ? hscan[(q + 1) << rb] : n) : 0u;
      el[c] = valid ? enq_load(d, q, val[c]) : EnqLoad{};
    }
#pragma unroll
    for (u32 c = 0; c < CH; ++c) {
      const bool valid = wbase + c * 64 + lane < n;
      PersistRec pr;
      pr.msg = INVALID;
      u32 drop = INVALID;
      if (valid) drop = enq_store(d, el[c], key[c] >> rb, pos[c] - first[c], pos[c] + 1 == nx[c], &pr);
      wave_release(d, drop, drop != INVALID);
      if (drop != INVALID) atomicAdd(&d.ctr->n_ring_full, 1u);
      if (d.persist) {
        const bool want = pr.msg != INVALID;
        const u32 k = wave_reserve(&d.ctr->n_persist, want);
        if (want && k < d.persist_max) d.prec[k] = pr;
      }
    }
  }
}

// a persistent message changed state in a durable queue: record it for the store
// (kind 0 consumed/acked, 1 expired, 2 dropped, 3 delivered awaiting ack, 4 requeued)
DEV bool wants_record(const DS& d, u32 msg, u32 q, bool valid) {
  return d.persist && valid && msg != INVALID && d.q_durable[q] && (d.msgs[msg].flags & MF_PERSIST);
}
DEV void consumed_rec_at(const DS& d, u32 msg, u32 q, u64 qpos, u32 kind, u32 k) {
  ConsumedRec r;
  r.msg_id = (i64)d.msgs[msg].msg_id;
  r.qpos = qpos;
  r.q = q;
  r.kind = kind;
  r.pad[0] = r.pad[1] = 0;
  d.crec[k] = r;
}
// X3: a shadow message left its queue (consumed, expired, dropped): ack it at the owner
DEV void link_consumed(const DS& d, u32 msg, u32 q, u32 kind, bool valid) {
  if (d.links && valid && msg != INVALID && kind <= 2u) {
    const u32 ow = d.q_link_owner[q];
    if (ow) {
      const u32 k = atomicAdd(&d.lk_cnt[ow - 1], 1u);
      if (k < d.lk_cap) {
        AckRec a;
        a.tq = q;
        a.pad = 0;
        a.xid = d.msgs[msg].msg_id;
        d.lk_send[(u64)(ow - 1) * d.lk_cap + k] = a;
      }
    }
  }
}
DEV void wave_consumed(const DS& d, u32 msg, u32 q, u64 qpos, u32 kind, bool valid) {
  link_consumed(d, msg, q, kind, valid);
  if (!d.persist) return;
  bool want = wants_record(d, msg, q, valid);
  u32 k = wave_reserve(&d.ctr->n_consumed, want);
  if (want && k < d.persist_max) consumed_rec_at(d, msg, q, qpos, kind, k);
}


// ============================================================================ K9 window advance
// one block (4 waves) per dirty channel: resolve marks, release/requeue, advance the
// window head over the contiguous run of finished slots, 256 slots per iteration
#define MS_MAX 256   // multiple settles per channel per step resolved exactly (more: folded)
struct MsLds {
  u64 up[MS_MAX];
  u32 rq[MS_MAX];
  u32 wc[4];
  u32 rc[4];     // store records per wave of the current chunk
  u32 rbase;     // their block reservation (INVALID: budget exhausted)
  u32 n, nb;
  unsigned long long ovf_a, ovf_r;
};
DEV void chan_advance_one(const DS& d, u32 ch, u32 tid, u32 lane, u32 w, u32* s_first, u32* s_done, MsLds& ms);
__global__ __launch_bounds__(256) void k_chan_advance(DS d) {
  __shared__ u32 s_first[4];
  __shared__ u32 s_done[4];
  __shared__ MsLds ms;
  const u32 tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const u32 nd = *d.n_dirty;
  for (u32 wv = blockIdx.x; wv < nd; wv += gridDim.x) chan_advance_one(d, d.dirty_list[wv], tid, lane, w, s_first,
                                                                        s_done, ms);
}

// the channel's multiple settles of this step (ack indices [lo, hi]) in wire order, reduced
// to record-breaking uptos: ms.up[0..nb) increasing, the first one >= t decides tag t
DEV void collect_settles(const DS& d, u32 ch, u32 tid, u32 lane, u32 w, MsLds& ms) {
  const u32 lo = d.ch_mlo[ch], hi = d.ch_mhi[ch];
  if (tid == 0) { ms.n = 0; ms.nb = 0; ms.ovf_a = 0; ms.ovf_r = 0; }
  __syncthreads();
  if (lo == INVALID) return;   // block-uniform
  for (u32 base = lo; base <= hi; base += 256) {
    const u32 i = base + tid;
    bool take = false;
    Ack a;
    a.tag = 0; a.kind = 0; a.requeue = 0;
    if (i <= hi) {
      a = d.acks[i];
      take = a.chslot == ch && a.multiple;
    }
    const bool rq = (a.kind != CK_ACK) && a.requeue;
    const u64 m = __ballot(take);
    if (lane == 0) ms.wc[w] = (u32)__popcll(m);
    __syncthreads();
    u32 pos = ms.n + (u32)__popcll(m & lanemask_lt());
    for (u32 k = 0; k < w; ++k) pos += ms.wc[k];
    if (take) {
      if (pos < MS_MAX) { ms.up[pos] = a.tag; ms.rq[pos] = rq; }
      else atomicMax(rq ? &ms.ovf_r : &ms.ovf_a, (unsigned long long)a.tag);
    }
    __syncthreads();
    if (tid == 0) ms.n += ms.wc[0] + ms.wc[1] + ms.wc[2] + ms.wc[3];
    __syncthreads();
  }
  if (tid == 0) {
    const u32 n = ms.n < MS_MAX ? ms.n : MS_MAX;
    u64 top = 0;
    u32 nb = 0;
    for (u32 k = 0; k < n; ++k)
      if (ms.up[k] > top) { ms.up[nb] = ms.up[k]; ms.rq[nb] = ms.rq[k]; ++nb; top = ms.up[k]; }
    const u64 oa = ms.ovf_a, orq = ms.ovf_r;   // past MS_MAX: the larger cover, appended
    const u64 om = oa > orq ? oa : orq;
    if (om > top && nb < MS_MAX) { ms.up[nb] = om; ms.rq[nb] = orq > oa; ++nb; }
    ms.nb = nb;
    d.ch_mlo[ch] = INVALID;
    d.ch_mhi[ch] = 0;
  }
  __syncthreads();
}

// k_chan_advance's share of a step's consumed-store records: persist_max minus what the
// later producers can take (deliveries <= deliv_max in k_dv_write / k_post, the durable
// TTL skip <= persist_max / 4 in k_dequeue); the engine sizes persist_max so this is
// >= deliv_max / 2.  Reserved per 256-slot chunk, never past the budget (CAS).
DEV u32 ca_reserve(const DS& d, u32 n) {
  const u32 lim = d.persist_max - d.deliv_max - (d.persist_max >> 2) - 64u;
  u32 cur = *(volatile u32*)&d.ctr->n_consumed;
  while (true) {
    if (cur + n > lim) return INVALID;
    const u32 prev = atomicCAS(&d.ctr->n_consumed, cur, cur + n);
    if (prev == cur) return cur;
    cur = prev;
  }
}

DEV void chan_advance_one(const DS& d, u32 ch, u32 tid, u32 lane, u32 w, u32* s_first, u32* s_done, MsLds& ms) {
  collect_settles(d, ch, tid, lane, w, ms);
  const u32 nb = ms.nb;
  const u64 head = d.ch_uhead[ch], nt = d.ch_next_tag[ch];
  const u64 aup = d.ch_ack_upto[ch], rup = d.ch_req_upto[ch];
  USlot* win = d.uwin + (u64)ch * (d.ucap_mask + 1);
  bool contiguous = true;
  bool deferred = false;   // block-uniform: the record budget ran out at some chunk
  u64 newhead = head;
  u32 manual_done = 0;
  for (u64 t0 = head; t0 < nt; t0 += 256) {
    const u64 t = t0 + tid;
    const bool valid = t < nt;
    u32 st = US_FREE;
    USlot u;
    u.state = US_FREE; u.msg = INVALID; u.q = 0; u.cons = 0; u.qpos = 0; u.expire_ms = 0;
    if (valid) {
      u = win[(t - 1) & d.ucap_mask];
      st = u.state;
      if (st == US_PENDING) {   // host marks (between steps) first, then this step's settles
        if (t <= aup) st = US_ACKED;
        else if (t <= rup) st = US_REQUEUE;
        else
          for (u32 k = 0; k < nb; ++k)
            if (t <= ms.up[k]) { st = ms.rq[k] ? US_REQUEUE : US_ACKED; break; }
      }
    }
    const bool acked = valid && st == US_ACKED;
    const bool req = valid && st == US_REQUEUE;
    // store records of this chunk, reserved for the whole block within the step's budget.
    // Past the budget the channel keeps its decided marks (ACKED / REQUEUE slot states,
    // which the next step resolves first) and stays dirty (a burst of settles
    // of durable persistent messages must not overflow persist_max and stop the broker)
    u32 rec_k = INVALID;
    const bool want_rec = wants_record(d, u.msg, u.q, acked || req);
    if (d.persist) {   // kernel-uniform
      const u64 rm = __ballot(want_rec);
      if (lane == 0) ms.rc[w] = (u32)__popcll(rm);
      __syncthreads();
      if (tid == 0) {
        const u32 tot = ms.rc[0] + ms.rc[1] + ms.rc[2] + ms.rc[3];
        ms.rbase = deferred ? INVALID : (tot ? ca_reserve(d, tot) : 0u);
      }
      __syncthreads();
      if (ms.rbase == INVALID) deferred = true;
      if (!deferred) {
        rec_k = ms.rbase + (u32)__popcll(rm & lanemask_lt());
        for (u32 k = 0; k < w; ++k) rec_k += ms.rc[k];
      }
    }
    if (deferred) {   // block-uniform
      if (valid && (st == US_ACKED || st == US_REQUEUE) && st != u.state) win[(t - 1) & d.ucap_mask].state = st;
      contiguous = false;
      continue;
    }
    // requeue list (one reservation per wave)
    u32 rtot;
    u32 ri = wave_reserve(d.req_n, req, &rtot);
    bool req_ok = req && ri < d.req_max;
    if (req_ok) {
      ReqItem r;
      r.q = u.q; r.msg = u.msg; r.qpos = u.qpos; r.expire_ms = u.expire_ms;
      d.req[ri] = r;
    }
    wave_add_u32(d.req_q_n, u.q, 1u, req_ok);
    link_consumed(d, u.msg, u.q, acked ? 0u : (req_ok ? 4u : 2u), acked || req);
    if (want_rec) consumed_rec_at(d, u.msg, u.q, u.qpos, acked ? 0u : (req_ok ? 4u : 2u), rec_k);
    wave_release(d, u.msg, acked || (req && !req_ok));
    wave_sub_u32(d.cons_unacked, u.cons, 1u, acked || req);
    manual_done += __popcll(__ballot(acked || req));
    if (lane == 0 && rtot) atomicAdd(&d.ctr->n_requeue, rtot);
    if (acked || req) st = US_DONE;
    if (valid && st != u.state) win[(t - 1) & d.ucap_mask].state = st;
    if (contiguous) {   // block-uniform
      // both ballots wave-wide (a ballot inside the lane-0 branch would see one lane)
      const u64 notdone = __ballot(valid && st != US_DONE);
      const u32 nvalid = (u32)__popcll(__ballot(valid));
      if (lane == 0) {
        s_first[w] = notdone ? (u32)(__ffsll((unsigned long long)notdone) - 1) : 64u;
        s_done[w] = nvalid;
      }
      __syncthreads();
      u32 adv = 0;
      bool stop = false;
      for (u32 k = 0; k < 4 && !stop; ++k) {
        if (s_first[k] < 64) { adv += s_first[k]; stop = true; }
        else adv += s_done[k];
      }
      newhead += adv;
      if (stop) contiguous = false;
      __syncthreads();
    }
  }
  if (lane == 0 && manual_done) atomicSub(&d.ch_unacked[ch], manual_done);
  if (tid == 0) {
    atomicSub(&d.ch_win[ch], (u32)(newhead - head));
    d.ch_uhead[ch] = newhead;
    if (deferred) d.def_list[atomicAdd(&d.tot[TS_NCADEF], 1u)] = ch;   // stays dirty: k_dequeue re-lists it
    else d.ch_dirty[ch] = 0;
  }
}

// ============================================================================ K8 dequeue
DEV u32 deliver_size(const DS& d, u32 cons, const MsgEnt& m, u32 conn) {
  // a link pseudo-connection ships [ex][rk][props][body] as a restore record (render_deliv)
  if (d.links && d.conn_link[conn]) return align16(m.ex_len + m.rk_len + m.props_len + m.body_len);
  // cons_max = a Basic.GetOk: no consumer tag, a 4-byte message-count instead
  u32 mp = (cons == d.cons_max ? 4 + 4 : 4 + 1 + d.cons_tag_len[cons]) + 8 + 1 + 1 + m.ex_len + 1 + m.rk_len;
  u32 sz = 8 + mp + 8 + 12 + m.props_len;
  u32 fm = d.conn_frame_max[conn];
  u32 fmb = fm ? fm - 8 : 0xffffffffu;
  u32 nb = m.body_len ? (m.body_len + fmb - 1) / fmb : 0;
  return sz + m.body_len + 8 * nb;
}

// egress by reference: the delivery of message m to connection conn is rendered without its
// body (the host sends those bytes from the publishing step's ingress payload): a body the
// publish decode marked (MsgEnt.href), published at most ref_back steps ago, no shorter than
// ref_min and within one body frame of the connection.  Link pseudo-connections ship
// restore records, never references.  k_dv_write and render_deliv must agree: same inputs
// Returns the body's host address, or 0 (rendered whole).  A body in the host spill ring
// is referenced there whatever its age: a freed ring byte is reused only SPILL_LAG steps
// later (spill_reserve), after every egress that can reference it was written out
DEV u64 deliv_href(const DS& d, const MsgEnt& m, u32 conn) {
  if (d.in->ref_back == 0xffffffffu || m.body_len < d.in->ref_min) return 0;
  if (d.links && d.conn_link[conn]) return 0;
  const u32 fm = d.conn_frame_max[conn];
  if (fm != 0 && m.body_len > fm - 8) return 0;
  if ((m.log_off & (SPILL_BIT | COLD_BIT)) == SPILL_BIT && d.spill_host)
    return d.spill_host + ((m.log_off & ~SPILL_BIT) % d.spill_bytes) + m.body_off;
  if (d.in->ref_back & REF_SPILL_ONLY) return 0;   // (ingress bodies inline this step)
  if (!m.href || (u32)d.in->step - m.pub_step > d.in->ref_back) return 0;
  return m.href;
}

// give back channel reservations for `take` messages not delivered after all
DEV void unreserve(const DS& d, u32 c, u32 take) {
  u32 ch = d.cons_ch[c];
  atomicSub(&d.ch_win[ch], take);
  if (!d.cons_noack[c]) { atomicSub(&d.ch_unacked[ch], take); d.cons_unacked[c] -= take; }
}

// one block per queue: TTL skip (K12, wave 0), credit-limited round-robin split over the
// consumers (thread 0, deterministic consumer order), egress byte budget (block-parallel
// sizes), then one delivery run per granted consumer.  k_runs orders the runs by channel
// and k_dv_write expands them into Deliv records at their final positions, so no sort
// over individual deliveries is needed (QueueEntity.scala:318-393, FrameStage.scala:380-406).
#define REQ_BLK 1024
DEV void requeue_compact(const DS& d);
DEV void requeue_queue(const DS& d, u32 q, u64* kpos, u32* kidx, u32* cnt_p);
// one queue's share of a spill (4 waves): every queued message past the first `hot` entries
// (of a queue with consumers) whose slot lies below log position `lim` -- its body to the
// host spill ring, the message switched to it; at most `budget` bytes per launch across
// all queues (budget 0: no limit)
DEV bool spill_reserve(const DS& d, u32 sz, u64* pos);
DEV void spill_queue(const DS& d, u32 q, u64 lim, u32 hot, u32 budget, u64* moved) {
  const u32 lane = lane_id(), w = threadIdx.x >> 6;
  if (!d.q_active[q]) return;
  // (agent scope: in k_dequeue this block's requeue may just have moved the head)
  const u64 head = __hip_atomic_load(&d.q_head[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const u64 tail = d.q_tail[q], mask = d.q_ring_mask[q];
  const Desc* ring = d.ring + d.q_ring_off[q];
  const u64 skip = d.q_cons_n[q] ? hot : 0;
  // Resume at the queue's cursor: every entry before it is tiered already, so a deep
  // backlog is not walked again each step (it was: ~10 ms per step for a 90 K-entry queue
  // of spilled and cold bodies, profiles/r5_coldprof/).  A queue's log offsets grow along
  // the queue (requeues only go lower), so the first entry at or past `lim` ends the walk.
  __shared__ unsigned long long s_open;
  if (threadIdx.x == 0) s_open = ~0ull;
  __syncthreads();
  const u64 start0 = head + skip;
  u64 cur = d.q_spill_cur[q];
  if (cur < start0 || cur > tail) cur = start0;   // (the head passed it, or the slot was reset)
  u64 open = ~0ull;   // this wave's first entry left in the log
  for (u64 i = cur + w; i < tail; i += 4) {
    const u32 msg = ring[i & mask].msg;
    if (msg == INVALID || msg >= d.msg_max) continue;
    MsgEnt& m = d.msgs[msg];
    const u64 lo = __hip_atomic_load(&m.log_off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lo & (SPILL_BIT | COLD_BIT)) continue;
    if (lo >= lim) { open = i; break; }
    const u32 sz = m.slot_bytes;
    u64 pos = 0;
    u32 ok = 0;
    if (lane == 0) {
      ok = (!budget || atomicAdd(&d.tot[TS_SPILL_USED], sz) + sz <= budget) ? 1u : 0u;
      if (ok) ok = spill_reserve(d, sz, &pos) ? 1u : 0u;
    }
    ok = (u32)__shfl((int)ok, 0);
    if (!ok) { open = i; break; }   // the spill ring is full, or this step's budget is spent
    pos = shfl64(pos, 0);
    wave_copy(d.spill + (pos % d.spill_bytes), d.log + (lo % d.log_bytes), sz);
    __threadfence_system();   // the copy reached host memory before the slot is switched
    if (lane == 0 &&
        atomicCAS((unsigned long long*)&m.log_off, (unsigned long long)lo, (unsigned long long)(SPILL_BIT | pos)) == lo) {
      atomicAdd((unsigned long long*)&d.log_live[(lo / d.log_block) % d.n_log_blocks], (unsigned long long)(-(i64)sz));
      atomicAdd((unsigned long long*)&d.spill_live[(pos / d.log_block) % d.n_spill_blocks], (unsigned long long)sz);
      atomicAdd((unsigned long long*)d.live_bytes, (unsigned long long)(-(i64)sz));
      atomicAdd((unsigned long long*)moved, (unsigned long long)sz);
    }
  }
  if (lane == 0 && open != ~0ull) atomicMin(&s_open, (unsigned long long)open);
  __syncthreads();
  if (threadIdx.x == 0) d.q_spill_cur[q] = s_open == ~0ull ? tail : (u64)s_open;
}

// true: the block wrote runs with plain stores (the fused k_runs' ticket needs an
// agent-scope release); false: at most q_nruns[q] = 0, stored agent-coherent
// a consumer's dispatch inputs, loaded by the block's other waves while wave 0 walks the
// TTL head (thread 0's credit loop then reads them from LDS: only its atomics stay serial)
struct DqCons { u32 c, ch, ok, noack, pc, glob, unacked; };
DEV bool dequeue_queue(const DS& d) {
  __shared__ u32 g_cons[RUNS_PER_Q];
  __shared__ u32 g_n[RUNS_PER_Q];
  __shared__ DqCons g_ci[RUNS_PER_Q];
  __shared__ u64 s_head;
  __shared__ u32 s_ngr;
  __shared__ unsigned long long s_bytes;
  __shared__ u64 kpos[REQ_BLK];
  __shared__ u32 kidx[REQ_BLK];
  __shared__ u32 rq_cnt, rq_last;
  const u32 q = blockIdx.x, tid = threadIdx.x, lane = lane_id();
  if (q == 0 && tid == 0) {   // fused k_reset_dirty (k_chan_advance consumed the list)
    // channels it deferred (store-record budget) start the next step's list
    const u32 nd = d.tot[TS_NCADEF];
    for (u32 k = 0; k < nd; ++k) d.dirty_list[k] = d.def_list[k];
    *d.n_dirty = nd;
    d.tot[TS_NCADEF] = 0;
  }
  // fused k_requeue: requeued deliveries go back in front of their queues' heads before this
  // step's dispatch, in queue-offset order.  Every block takes the ticket (req_n only
  // changes in the compaction, which runs after every block has read it); the last one
  // compacts the unconsumed items
  if (*d.req_n != 0) {
    if (q < d.q_max && d.req_q_n[q] != 0) requeue_queue(d, q, kpos, kidx, &rq_cnt);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    if (tid == 0) rq_last = atomicAdd(&d.tot[TS_REQ_TICKET], 1u) == gridDim.x - 1;
    __syncthreads();
    if (rq_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      if (tid == 0) d.tot[TS_REQ_TICKET] = 0;
      requeue_compact(d);
      __syncthreads();
    }
  }
  if (q >= d.q_max) return false;
  const u32 ndg = d.tot[TS_NDGET] < DGET_MAX ? d.tot[TS_NDGET] : DGET_MAX;   // Basic.Gets decoded this step
  if (!d.q_active[q]) {
    if (tid == 0) {
      __hip_atomic_store(&d.q_nruns[q], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // a Basic.Get staged for a queue deleted since: answered GONE (never left RETRY, which
      // the host would resubmit forever -- or serve from whatever queue reuses the slot)
      const u32 ng = d.in->nget < GET_STEP_MAX ? d.in->nget : GET_STEP_MAX;
      for (u32 i = 0; i < ng; ++i)
        if (d.get_req[i].q == q) d.get_out_h[i] = GetOut{GS_GONE, 0u};
      for (u32 k = 0; k < ndg; ++k)
        if (d.dget[k].q == q) dget_to_host(d, k);
    }
    return false;
  }
  const bool nodisp = (d.in->flags & SF_NODISPATCH) != 0;
  if (d.in->spill_frac && d.spill_bytes) {   // (kernel-uniform) the step's share of body tiering
    const u64 lim = *d.log_tail + (((u64)d.log_bytes * d.in->spill_frac) >> 16);
    spill_queue(d, q, lim, d.in->spill_hot, d.in->spill_budget, &d.ctr->spill_moved);
    __syncthreads();
  }
  if (nodisp && d.links && d.q_link_owner[q]) {   // a live link shadow: its acks could not travel
    if (tid == 0) {
      __hip_atomic_store(&d.q_nruns[q], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (u32 k = 0; k < ndg; ++k)
        if (d.dget[k].q == q) dget_to_host(d, k);
    }
    return false;
  }
  // agent-scope load: the requeue above (this block's thread 0) may have moved the head
  // after this wave read the line
  u64 head = __hip_atomic_load(&d.q_head[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const u64 tail = d.q_tail[q];
  const u64 mask = d.q_ring_mask[q];
  const Desc* ring = d.ring + d.q_ring_off[q];
  const i64 now = d.in->now_ms;
  if (tid < 64) {   // TTL skip at the head (K12)
    // durable queues: every skipped persistent entry is a store record (ConsumedRec); a
    // purge of a deep queue marks its whole backlog expired, so the skip takes at most a
    // quarter of the step's record buffer (reserved 64 at a time) and the next steps
    // continue it -- the record buffer never overflows (the store would miss deletions)
    const bool budget = d.persist && d.q_durable[q];
    while (head < tail) {
      if (budget) {
        u32 ok = 1;
        if (lane == 0) ok = atomicAdd(&d.tot[TS_TTL_BUDGET], 64u) + 64u <= (d.persist_max >> 2);
        if (!__shfl(ok, 0, 64)) break;
      }
      u64 idx = head + lane;
      bool valid = idx < tail;
      Desc ds;
      ds.msg = INVALID; ds.expire_ms = 0; ds.flags = 0;
      if (valid) ds = ring[idx & mask];
      bool exp = valid && ds.expire_ms != 0 && ds.expire_ms <= now;
      u64 live = __ballot(valid && !exp);
      u32 nexp = live ? (__ffsll((unsigned long long)live) - 1) : __popcll(__ballot(valid));
      wave_consumed(d, ds.msg, q, idx, 1u, lane < nexp);
      wave_release(d, ds.msg, lane < nexp);
      if (lane == 0 && nexp) atomicAdd(&d.ctr->n_expired, nexp);
      head += nexp;
      if (live) break;
    }
    if (lane == 0) { s_head = head; s_bytes = 0; }
  } else if (!nodisp && tid - 64 < RUNS_PER_Q) {   // the consumers' inputs, beside the TTL walk
    const u32 j = tid - 64, mall0 = d.q_cons_n[q];
    if (j < mall0) {
      const u32 c = d.q_cons[d.q_cons_off[q] + (d.q_rr[q] % mall0 + j) % mall0];
      const u32 ch = d.cons_ch[c];
      DqCons ci;
      ci.c = c;
      ci.ch = ch;
      // wblock: the front end's socket backlog for this connection is above its high
      // watermark (host-mapped, written by the IO threads): its messages stay queued in HBM
      // (cons_active 2: staged by a light control section this step -- it takes deliveries
      // from the next step on, behind its Basic.ConsumeOk)
      ci.ok = d.cons_active[c] == 1u && d.ch_flow[ch] && !d.conn_wblock[ch / d.chpc];
      ci.noack = d.cons_noack[c];
      ci.pc = d.ch_prefetch[ch];
      ci.glob = d.ch_global[ch];
      ci.unacked = d.cons_unacked[c];
      g_ci[j] = ci;
    }
  }
  __syncthreads();
  head = s_head;
  // Basic.Get requests of this queue, in request order, ahead of its consumers (the
  // reference's Pull(1) with the channel's next delivery tag, FrameStage.scala:1199-1229):
  // each answer is one run of cnt 1 on the requester's channel (consumer slot cons_max),
  // rendered as GetOk + header + body by k_render; EMPTY / RETRY / WINDOW_FULL go back
  // to the host through the step's host-mapped GetOut (the host initialised them RETRY)
  u32 ngr = 0;
  if (d.in->nget || ndg) {   // kernel-uniform
    if (tid == 0) {
      const u32 ng = d.in->nget < GET_STEP_MAX ? d.in->nget : GET_STEP_MAX;
      const u64 clim = d.q_cold_lim[q];   // a cold head waits for the host's page-in (RETRY)
      u64 h = head;
      // the host-staged requests (their connections were paused: nothing of theirs was
      // decoded this step), then the step's own Basic.Gets in wire order
      for (u32 i = 0; i < ng + ndg; ++i) {
        const bool dev = i >= ng;
        const u32 dk = dev ? i - ng : 0u;
        GetReq rq;
        if (dev) {
          rq.conn = d.dget[dk].conn; rq.chslot = d.dget[dk].chslot; rq.q = d.dget[dk].q; rq.noack = d.dget[dk].noack;
        } else {
          rq = d.get_req[i];
        }
        if (rq.q != q) continue;
        GetOut o;
        o.status = GS_RETRY;
        o.msg_count = 0;
        if (!nodisp && h == tail) {
          o.status = GS_EMPTY;
        } else if (!nodisp && h < clim && ngr < RUNS_PER_Q / 2 && rq.chslot < d.c_max * d.chpc) {
          const u32 ch = rq.chslot;
          const u32 sz = deliver_size(d, d.cons_max, d.msgs[ring[h & mask].msg], ch / d.chpc);
          u32 wb, db;
          if (sz > d.egress_cap / 2) {
            o.status = GS_NO_SPACE;
          } else if (!reserve_upto(&d.ch_win[ch], 1u, d.ucap_mask + 1, &wb)) {
            o.status = GS_WINDOW_FULL;
          } else if (reserve_sat64(d.egress_budget, sz, d.egress_cap) < sz ||
                     !reserve_sat(&d.ctr->n_deliv, 1u, d.deliv_max, &db)) {
            atomicSub(&d.ch_win[ch], 1u);   // step full: the host retries with a later step
          } else {
            if (!rq.noack) { atomicAdd(&d.ch_unacked[ch], 1u); atomicAdd(&d.cons_unacked[d.cons_max], 1u); }
            const u64 left = tail - h - 1;
            Run rn;
            rn.ch = ch;
            rn.cons = left < 0xffffffffull ? (u32)left : 0xffffffffu;
            rn.cnt = 1;
            rn.q = q;
            rn.qpos = h;
            rn.noack = rq.noack ? 1u : 0u;
            rn.flags = RUN_GET;
            d.runs[(u64)q * RUNS_PER_Q + ngr] = rn;
            ++ngr;
            ++h;
            o.status = GS_OK;
            o.msg_count = rn.cons;
          }
        }
        if (!dev) {
          d.get_out_h[i] = o;
        } else if (o.status == GS_EMPTY && reserve_sat64(d.egress_budget, 13, d.egress_cap) == 13) {
          atomicAdd(&d.conn_gempty[rq.conn], 1u);   // Basic.GetEmpty, rendered by render_confirms
          d.conn_gempty_ch[rq.conn] = d.ch_num[rq.chslot];
        } else if (o.status != GS_OK) {
          dget_to_host(d, dk);
        }
      }
      s_head = h;
      s_ngr = ngr;
    }
    __syncthreads();
    head = s_head;
    ngr = s_ngr;
  }
  const u32 mall = d.q_cons_n[q];
  // bodies from q_cold_lim on may be in the cold store: delivered once paged back in
  const u64 dlim = d.q_cold_lim[q] < tail ? d.q_cold_lim[q] : tail;
  const u64 avail = dlim > head ? dlim - head : 0;
  if (mall == 0 || avail == 0 || nodisp) {
    if (tid == 0) { d.q_head[q] = head; d.q_nruns[q] = ngr; }
    return true;
  }
  const u32 m = mall > RUNS_PER_Q - ngr ? RUNS_PER_Q - ngr : mall;
  const u32 r = d.q_rr[q] % mall;
  // (1) counts by credit (the consumers' inputs came in beside the TTL walk: g_ci)
  if (tid == 0) {
    u64 remaining = avail;
    for (u32 j = 0; j < m; ++j) {
      const DqCons ci = g_ci[j];
      u32 c = ci.c;
      g_cons[j] = c;
      g_n[j] = 0;
      if (remaining == 0) continue;
      u32 ch = ci.ch;
      if (!ci.ok) continue;
      u64 share = (remaining + (m - j) - 1) / (m - j);
      u32 want = (u32)(share < d.deliver_cap ? share : d.deliver_cap);
      const u32 dcb = d.in->dcap_bytes;
      if (dcb && want > 1 && !(d.links && d.conn_link[ch / d.chpc])) {   // byte cap (StepIn.dcap_bytes)
        const u32 s0 = deliver_size(d, c, d.msgs[ring[(head + (avail - remaining)) & mask].msg], ch / d.chpc);
        const u32 lim = s0 >= dcb ? 1u : dcb / s0;
        want = want < lim ? want : lim;
      }
      bool noack = ci.noack;
      u32 pc = ci.pc;
      if (!noack && pc && !ci.glob) {
        u32 used = ci.unacked;
        u32 cr = used < pc ? pc - used : 0;
        want = want < cr ? want : cr;
      }
      u32 wb;
      u32 g = reserve_upto(&d.ch_win[ch], want, d.ucap_mask + 1, &wb);
      if (!noack && pc && ci.glob && g) {
        u32 ub;
        u32 g2 = reserve_upto(&d.ch_unacked[ch], g, pc, &ub);
        if (g2 < g) atomicSub(&d.ch_win[ch], g - g2);
        g = g2;
      } else if (!noack && g) {
        atomicAdd(&d.ch_unacked[ch], g);
      }
      if (!noack && g) d.cons_unacked[c] += g;
      g_n[j] = g;
      remaining -= g;
    }
  }
  __syncthreads();
  // (2) egress bytes of every granted entry, block-parallel per consumer run
  {
    u32 mine = 0;
    u64 qp = head;
    for (u32 j = 0; j < m; ++j) {
      const u32 cnt = g_n[j];
      if (!cnt) continue;
      const u32 c = g_cons[j];
      const u32 conn = g_ci[j].ch / d.chpc;
      // four entries a thread per round, their ring loads then their message loads in flight
      // together (a round trip each per entry in series before)
      constexpr u32 U = 4;
      for (u32 k0 = tid; k0 < cnt; k0 += 256 * U) {
        u32 mg[U];
#pragma unroll
        for (u32 u = 0; u < U; ++u) {
          const u32 k = k0 + u * 256;
          mg[u] = k < cnt ? ring[(qp + k) & mask].msg : INVALID;
        }
#pragma unroll
        for (u32 u = 0; u < U; ++u)
          if (mg[u] != INVALID) mine += deliver_size(d, c, d.msgs[mg[u]], conn);
      }
      qp += cnt;
    }
    for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o, 64);
    if (lane == 0 && mine) atomicAdd(&s_bytes, (unsigned long long)mine);
  }
  __syncthreads();
  if (tid == 0) {
    const u64 bytes = s_bytes;
    const u64 gb = reserve_sat64(d.egress_budget, bytes, d.egress_cap);
    if (gb < bytes) {
      // egress budget nearly spent: keep the longest prefix of the queue's granted
      // entries (in run order) whose frames fit in what this queue was granted
      u64 left = gb;
      u64 qp = head;
      bool full = false;
      for (u32 j = 0; j < m; ++j) {
        u32 cnt = g_n[j];
        if (!cnt) continue;
        u32 c = g_cons[j];
        u32 conn = d.cons_ch[c] / d.chpc;
        u32 keep = 0;
        while (!full && keep < cnt) {
          u32 sz = deliver_size(d, c, d.msgs[ring[(qp + keep) & mask].msg], conn);
          if (sz > left) { full = true; break; }
          left -= sz;
          ++keep;
        }
        if (keep < cnt) unreserve(d, c, cnt - keep);
        g_n[j] = keep;
        qp += keep;
      }
    }
    // (3) delivery slots (capacity), trimmed from the last run backwards; k_runs
    // rewrites n_deliv with the exact total of the kept runs
    u32 total = 0;
    for (u32 j = 0; j < m; ++j) total += g_n[j];
    u32 db;
    u32 gt = reserve_sat(&d.ctr->n_deliv, total, d.deliv_max, &db);
    u32 excess = total - gt;
    for (int j = (int)m - 1; j >= 0 && excess; --j) {
      u32 take = g_n[j] < excess ? g_n[j] : excess;
      if (!take) continue;
      unreserve(d, g_cons[j], take);
      g_n[j] -= take;
      excess -= take;
    }
    // (4) runs, in round-robin order (after this step's Basic.Get answers)
    u32 nr = ngr;
    u64 qp = head;
    for (u32 j = 0; j < m; ++j) {
      u32 cnt = g_n[j];
      if (!cnt) continue;
      u32 c = g_cons[j];
      Run rn;
      rn.ch = d.cons_ch[c];
      rn.cons = c;
      rn.cnt = cnt;
      rn.q = q;
      rn.qpos = qp;
      rn.noack = d.cons_noack[c];
      rn.flags = 0;
      d.runs[(u64)q * RUNS_PER_Q + nr] = rn;
      ++nr;
      qp += cnt;
    }
    d.q_nruns[q] = nr;
    d.q_head[q] = qp;
    d.q_rr[q] = (r + 1) % mall;
  }
  return true;
}

// K8 dequeue, one block per queue; the last block to finish (ticket) then lays out the
// step's delivery runs (fused k_runs: a launch less per step)
template <u32 NT> DEV void runs_body(const DS& d, u64* key_lds, u32 key_cap, u32* lds);
#define DQ_RUN_LDS 2048   // runs sorted in the fused k_runs' LDS (more: the global-memory sort)
__global__ __launch_bounds__(256) void k_dequeue(DS d) {
  __shared__ u64 key_lds[DQ_RUN_LDS];
  __shared__ u32 lds[256 / 64 + 1];
  __shared__ u32 s_last;
  const bool wrote = dequeue_queue(d);
  // every block's runs and counts reach the device-wide coherence point before its ticket
  // (agent scope: the last block may run on another XCD, whose L2 does not see this one's);
  // a block that wrote no runs stored its zero count agent-coherent and skips the L2
  // write-back that release costs
  if (wrote) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  else __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(&d.tot[TS_DQ_TICKET], 1u) == gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (threadIdx.x == 0) d.tot[TS_DQ_TICKET] = 0;
  runs_body<256>(d, key_lds, DQ_RUN_LDS, lds);
}

// ============================================================================ runs -> deliveries
// One block: gather the step's runs (queue order, then round-robin order), sort them by
// channel (bitonic on (channel << 32 | run slot): ties keep queue order, the stable order
// of the reference's per-channel delivery), lay out their deliveries contiguously, and
// record the first delivery of every channel / first and last of every connection.
DEV void bitonic_sort_u64(u64* k, u32 np2, u32 tid, u32 nt) {
  for (u32 sz = 2; sz <= np2; sz <<= 1) {
    for (u32 j = sz >> 1; j > 0; j >>= 1) {
      for (u32 i = tid; i < np2; i += nt) {
        u32 ij = i ^ j;
        if (ij > i) {
          bool up = (i & sz) == 0;
          u64 a = k[i], b = k[ij];
          if ((a > b) == up) { k[i] = b; k[ij] = a; }
        }
      }
      __syncthreads();
    }
  }
}

template <u32 NT>
DEV void runs_body(const DS& d, u64* key_lds, u32 key_cap, u32* lds) {
  const u32 tid = threadIdx.x;
  // pass 1: total runs
  u32 R = 0;
  for (u32 b0 = 0; b0 < d.q_max; b0 += NT) {
    u32 qq = b0 + tid;
    u32 v = qq < d.q_max ? d.q_nruns[qq] : 0;
    u32 all;
    u32 off = block_scan<NT>(v, lds, all);
    for (u32 j = 0; j < v; ++j) {
      const u32 slot = qq * RUNS_PER_Q + j;
      const u32 pos = R + off + j;
      const u64 k = ((u64)d.runs[slot].ch << 32) | slot;
      if (pos < key_cap) key_lds[pos] = k;
      d.run_key[pos] = k;
    }
    R += all;
  }
  __syncthreads();
  u32 np2 = 1;
  while (np2 < R) np2 <<= 1;
  const bool in_lds = np2 <= key_cap;
  u64* key = in_lds ? key_lds : d.run_key;
  for (u32 i = R + tid; i < np2; i += NT) key[i] = ~0ull;
  __syncthreads();
  if (R > 1) bitonic_sort_u64(key, np2, tid, NT);
  // pass 2: delivery offsets in run order
  u32 run = 0;
  for (u32 b0 = 0; b0 < R; b0 += NT) {
    const u32 s = b0 + tid;
    u32 cnt = 0, slot = 0;
    if (s < R) { slot = (u32)key[s]; cnt = d.runs[slot].cnt; }
    u32 all;
    u32 off = block_scan<NT>(cnt, lds, all);
    if (s < R) {
      const u32 start = run + off;
      d.run_order[s] = slot;
      d.run_start[s] = start;
      const u32 ch = (u32)(key[s] >> 32);
      const u32 conn = ch / d.chpc;
      const u32 pch = s > 0 ? (u32)(key[s - 1] >> 32) : INVALID;
      const u32 nch = s + 1 < R ? (u32)(key[s + 1] >> 32) : INVALID;
      if (pch != ch) d.ch_first[ch] = start;
      if (pch == INVALID || pch / d.chpc != conn) d.conn_dfirst[conn] = start;
      if (nch == INVALID || nch / d.chpc != conn) d.conn_dlast[conn] = start + cnt - 1;
    }
    run += all;
  }
  if (tid == 0) {
    d.tot[TS_NRUNS] = R;
    d.ctr->n_deliv = run;   // the saturating slot counter may have ended above deliv_max
  }
}
__global__ __launch_bounds__(1024) void k_runs(DS d) {
  __shared__ u64 key_lds[RUN_SORT_LDS];
  __shared__ u32 lds[1024 / 64 + 1];
  runs_body<1024>(d, key_lds, RUN_SORT_LDS, lds);
}

DEV void wave_consumed(const DS& d, u32 msg, u32 q, u64 qpos, u32 kind, bool valid);
// thread per delivery: expand its run (binary search), assign the channel's next delivery
// tag, fill the unacked window slot, size the rendered frames
#define DVW_LDS 512   // runs staged in LDS per block (more: searched in global memory)
__global__ __launch_bounds__(256) void k_dv_write(DS d) {
  __shared__ u32 s_start[DVW_LDS];
  __shared__ Run s_run[DVW_LDS];
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  const u32 n = d.ctr->n_deliv;
  const bool valid = i < n;
  u32 lat = 0, nref = 0, rbytes = 0;
  Deliv dv;
  dv.msg = INVALID; dv.q = 0; dv.qpos = 0; dv.flags = 2;
  const u32 R = d.tot[TS_NRUNS];
  // the step's runs (run order) staged in LDS by the block: one coalesced load of the
  // starts and the runs instead of a chain of dependent global loads per delivery (the
  // binary search's probes, then run_order -> runs)
  const bool lds_runs = R <= DVW_LDS;
  if (lds_runs && blockIdx.x * blockDim.x < n) {   // (block-uniform)
    for (u32 s = threadIdx.x; s < R; s += blockDim.x) {
      s_start[s] = d.run_start[s];
      s_run[s] = d.runs[d.run_order[s]];
    }
    __syncthreads();
  }
  if (valid) {
    u32 lo = 0, hi = R;   // last s with run_start[s] <= i
    while (hi - lo > 1) {
      u32 mid = (lo + hi) >> 1;
      if ((lds_runs ? s_start[mid] : d.run_start[mid]) <= i) lo = mid; else hi = mid;
    }
    const Run rn = lds_runs ? s_run[lo] : d.runs[d.run_order[lo]];
    const u32 k = i - (lds_runs ? s_start[lo] : d.run_start[lo]);
    const Desc ds = d.ring[d.q_ring_off[rn.q] + ((rn.qpos + k) & d.q_ring_mask[rn.q])];
    const u32 ch = rn.ch;
    const u64 tag = d.ch_next_tag[ch] + (i - d.ch_first[ch]);
    const bool get = rn.flags & RUN_GET;
    const u32 cons = get ? d.cons_max : rn.cons;   // Basic.Get: the reserved slot cons_max
    dv.chslot = ch;
    dv.cons = rn.cons;   // Basic.Get: the message-count of the GetOk
    dv.msg = ds.msg;
    dv.q = rn.q;
    dv.qpos = rn.qpos + k;
    dv.expire_ms = ds.expire_ms;
    dv.tag = tag;
    dv.flags = (ds.flags & 1) | (rn.noack ? 2u : 0u) | (get ? DV_GET : 0u);
    USlot u;
    u.state = rn.noack ? US_DONE : US_PENDING;
    u.msg = ds.msg;
    u.q = rn.q;
    u.cons = cons;
    u.qpos = dv.qpos;
    u.expire_ms = ds.expire_ms;
    d.uwin[(u64)ch * (d.ucap_mask + 1) + ((tag - 1) & d.ucap_mask)] = u;
    const MsgEnt& m = d.msgs[ds.msg];
    const bool ref = deliv_href(d, m, ch / d.chpc) != 0;
    const u32 sz = deliver_size(d, cons, m, ch / d.chpc) - (ref ? m.body_len : 0u);
    dv.size = sz;
    d.dv_size[i] = sz;
    if (ref) { nref = 1; rbytes = m.body_len; }
    d.deliv[i] = dv;
    lat = (u32)d.in->step - m.pub_step;
    // the channel's last delivery this step: the window needs a k_chan_advance pass
    bool last = i + 1 == n ||
                (k + 1 == rn.cnt && (lo + 1 >= R || (lds_runs ? s_run[lo + 1].ch : d.runs[d.run_order[lo + 1]].ch) != ch));
    if (last) {
      // auto-ack channel with nothing pending (no manual delivery awaiting a settle, no
      // deferred marks): every slot up to this tag is done, so the window head moves here
      // and k_chan_advance has nothing to walk for it
      if (rn.noack && d.ch_unacked[ch] == 0 && d.ch_dirty[ch] == 0) {
        const u64 head = d.ch_uhead[ch];
        atomicSub(&d.ch_win[ch], (u32)(tag + 1 - head));
        d.ch_uhead[ch] = tag + 1;
      } else if (atomicExch(&d.ch_dirty[ch], 1u) == 0) {
        u32 kk = atomicAdd(d.n_dirty, 1u);
        d.dirty_list[kk] = ch;
      }
    }
  } else if (i < d.deliv_max) {
    d.dv_size[i] = 0;
  }
  if (d.persist)   // manual-ack delivery of a persistent message: its row becomes an unack
    wave_consumed(d, dv.msg, dv.q, dv.qpos, 3u, valid && !(dv.flags & 2));
  wave_add_u32(d.ctr->lat_hist, lat < LAT_BINS ? lat : LAT_BINS - 1, 1u, valid);
  {   // referenced deliveries / body bytes of the step (one atomic per wave)
    u32 nr = nref;
    u64 rb = rbytes;
    for (int o = 32; o > 0; o >>= 1) { nr += __shfl_xor(nr, o, 64); rb += shfl_xor64(rb, o); }
    if (lane_id() == 0 && nr) {
      atomicAdd(&d.ctr->n_ref, nr);
      atomicAdd((unsigned long long*)&d.ctr->ref_bytes, (unsigned long long)rb);
    }
  }
}

// per connection: egress size = returns + confirms + deliveries
__global__ void k_conn_sizes(DS d) {
  u32 c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= d.c_max) return;
  u32 conf = 0;
  for (u32 l = 0; l < d.chpc; ++l) {
    u32 ch = c * d.chpc + l;
    if (d.ch_pub_cnt[ch] && d.ch_confirm[ch]) conf += 21;
  }
  d.conn_conf_bytes[c] = conf;
  u32 dl = 0;
  u32 f = d.conn_dfirst[c];
  if (f != INVALID) {
    u32 l = d.conn_dlast[c];
    dl = d.dv_off[l] + d.dv_size[l] - d.dv_off[f];
  }
  d.conn_total[c] = d.conn_ret_bytes[c] + conf + dl + 13u * d.conn_gempty[c];
}

// the step's D2H size: its rendered bytes, then -- when any delivery references a host
// body -- the gather table (one EgressRef per delivery), so one copy carries both
DEV void set_egress_bytes(const DS& d, u32 eb) {
  if (d.ctr->n_ref) {
    u32 nd = d.ctr->n_deliv;
    if (nd > d.deliv_max) nd = d.deliv_max;
    const u32 go = align16(eb);
    d.ctr->gath_off = go;
    eb = go + 16u * nd;
  }
  d.ctr->egress_bytes = eb;
}

// single block (c_max <= CONN_LAYOUT_MAX): k_conn_sizes + scan of conn_total + k_conn_out
#define CONN_LAYOUT_MAX 8192
__global__ __launch_bounds__(1024) void k_conn_layout(DS d) {
  __shared__ u32 lds[1024 / 64 + 1];
  // exclusive scan of the deliveries' rendered sizes (fused k_scan: one block walks the
  // step's deliveries 16K at a time -- 16 per thread, all loads of a pass in flight at
  // once, one block scan per pass: a step's deliveries usually take one pass)
  {
    u32 n = d.ctr->n_deliv;
    if (n > d.deliv_max) n = d.deliv_max;
    u32 acc = 0;
    constexpr u32 EPT = 16;
    for (u32 b0 = 0; b0 < n; b0 += 1024 * EPT) {
      const u32 i0 = b0 + threadIdx.x * EPT;
      u32 v[EPT];
      if (i0 + EPT <= n) {   // dv_size is 16-byte aligned and i0 a multiple of 16
        const uint4* src = (const uint4*)(d.dv_size + i0);
#pragma unroll
        for (u32 k = 0; k < EPT / 4; ++k) {
          const uint4 x = src[k];
          v[4 * k] = x.x; v[4 * k + 1] = x.y; v[4 * k + 2] = x.z; v[4 * k + 3] = x.w;
        }
      } else {
#pragma unroll
        for (u32 k = 0; k < EPT; ++k) v[k] = i0 + k < n ? d.dv_size[i0 + k] : 0u;
      }
      u32 sum = 0;
#pragma unroll
      for (u32 k = 0; k < EPT; ++k) sum += v[k];
      u32 all;
      u32 o = acc + block_scan<1024>(sum, lds, all);
      if (i0 + EPT <= n) {
        uint4* dst = (uint4*)(d.dv_off + i0);
#pragma unroll
        for (u32 k = 0; k < EPT / 4; ++k) {
          uint4 x;
          x.x = o; o += v[4 * k];
          x.y = o; o += v[4 * k + 1];
          x.z = o; o += v[4 * k + 2];
          x.w = o; o += v[4 * k + 3];
          dst[k] = x;
        }
      } else {
#pragma unroll
        for (u32 k = 0; k < EPT; ++k) {
          if (i0 + k < n) d.dv_off[i0 + k] = o;
          o += v[k];
        }
      }
      acc += all;
      __syncthreads();   // lds of the next pass's scan
    }
    if (threadIdx.x == 0) d.tot[6] = acc;
    __syncthreads();
  }
  u32 run = 0;
  for (u32 b0 = 0; b0 < d.c_max; b0 += 1024) {
    const u32 c = b0 + threadIdx.x;
    u32 total = 0;
    if (c < d.c_max) {
      u32 conf = 0;
      for (u32 l = 0; l < d.chpc; ++l) {
        u32 ch = c * d.chpc + l;
        if (d.ch_pub_cnt[ch] && d.ch_confirm[ch]) conf += 21;
      }
      d.conn_conf_bytes[c] = conf;
      u32 dl = 0;
      u32 f = d.conn_dfirst[c];
      if (f != INVALID) {
        u32 l = d.conn_dlast[c];
        dl = d.dv_off[l] + d.dv_size[l] - d.dv_off[f];
      }
      total = d.conn_ret_bytes[c] + conf + dl + 13u * d.conn_gempty[c];
      d.conn_total[c] = total;
    }
    u32 all;
    const u32 off = block_scan<1024>(total, lds, all);
    if (c < d.c_max) {
      ConnOut o;
      o.off = run + off;
      o.len = d.links && d.conn_link[c] ? 0u : total;   // links: their bytes go to lsend_*
      d.conn_base[c] = o.off;
      d.conn_out[c] = o;
      if (c == d.c_max - 1) set_egress_bytes(d, o.off + total);
    }
    run += all;
  }
}

__global__ void k_conn_out(DS d) {
  u32 c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= d.c_max) return;
  ConnOut o;
  o.off = d.conn_base[c];
  o.len = d.links && d.conn_link[c] ? 0u : d.conn_total[c];
  d.conn_out[c] = o;
  if (c == d.c_max - 1) set_egress_bytes(d, o.off + d.conn_total[c]);
}

// ============================================================================ links (X2/X3)
// one wave: record / payload bases of every link pseudo-connection's deliveries in this
// parity's link send buffers, destination-major (the host reads the per-destination
// totals from xchg and sends each destination's region to it in the next exchange)
__global__ __launch_bounds__(64) void k_link_bases(DS d) {
  const u32 lane = threadIdx.x;
  const u32 nl = *d.n_link_conns;
  u32 c = INVALID, dest = INVALID, n = 0, b = 0;
  if (lane < nl && lane < 64) {
    c = d.link_conns[lane];
    const u32 lk = d.conn_link[c];
    const u32 f = d.conn_dfirst[c];
    if (lk) {
      dest = lk - 1;
      if (f != INVALID) { n = d.conn_dlast[c] - f + 1; b = d.conn_total[c]; }
    }
  }
  u32 npre = 0, bpre = 0, tn = 0, tb = 0;
  for (u32 j = 0; j < 64; ++j) {
    const u32 dj = __shfl(dest, j, 64), nj = __shfl(n, j, 64), bj = __shfl(b, j, 64);
    if (j < lane && dj == dest) { npre += nj; bpre += bj; }
    if (dj == lane) { tn += nj; tb += bj; }
  }
  u32 basen = 0, baseb = 0;
  for (u32 r = 0; r < 64; ++r) {
    const u32 x = __shfl(tn, r, 64), y = __shfl(tb, r, 64);
    if (r < lane) { basen += x; baseb += y; }
  }
  if (lane < d.world) {
    d.link_dbase[lane] = baseb;
    d.xchg[XC_LINK_N + lane] = tn;
    d.xchg[XC_LINK_B + lane] = tb;
  }
  const u32 sl = dest < 64 ? dest : 0;
  const u32 dbn = __shfl(basen, sl, 64);
  if (c != INVALID) {
    d.link_nbase[c] = dbn + npre;
    d.link_bbase[c] = bpre;
  }
}

// owner side, phase B (k_import_route): an ack a connection side sent for a link pseudo channel
// (the device form of Basic.Ack on the owner's pseudo channel; k_chan_advance settles)
DEV void link_ack_one(const DS& d, u32 i) {
  const AckRec a = d.rack[i];
  if (a.tq >= d.q_max) return;
  const u32 ch = d.q_link_ch[a.tq];
  if (ch == INVALID || (u32)(a.xid >> 40) != d.q_link_epoch[a.tq]) return;
  const u64 tag = a.xid & ((1ull << 40) - 1);
  if (tag < d.ch_uhead[ch] || tag >= d.ch_next_tag[ch]) return;
  USlot* u = &d.uwin[(u64)ch * (d.ucap_mask + 1) + ((tag - 1) & d.ucap_mask)];
  if (atomicCAS(&u->state, (u32)US_PENDING, (u32)US_ACKED) == US_PENDING &&
      atomicExch(&d.ch_dirty[ch], 1u) == 0)
    d.dirty_list[atomicAdd(d.n_dirty, 1u)] = ch;
}

// ============================================================================ K5 render
DEV u32 put_frame_hdr(u8* o, u32 type, u32 ch, u32 size) {
  o[0] = (u8)type;
  wr16(o + 1, ch);
  wr32(o + 3, size);
  return 7;
}

// one group of RD_G lanes per delivery i (< n_deliv), lane = 0..RD_G-1: with egress by
// reference a delivery is ~100 bytes of frames, so a whole wave per delivery left 3/4 of
// its lanes idle (four deliveries per wave now)
#define RD_G 16
DEV void render_deliv(const DS& d, u32 i, u32 lane) {
  const Deliv dv = d.deliv[i];
  const u32 ch = dv.chslot;
  const MsgEnt m = d.msgs[dv.msg];
  u32 conn = ch / d.chpc;
  u32 f = d.conn_dfirst[conn];
  const u8* slot = msg_slot(d, m.log_off);
  // gather entry of this delivery (the table exists when some delivery of the step
  // references its body; dst of an unreferenced one = its end, so dst never decreases)
  const u64 href = deliv_href(d, m, conn);
  const bool ref = href != 0;
  EgressRef* gt = d.ctr->n_ref ? (EgressRef*)((u8*)d.in->egress + d.ctr->gath_off) : nullptr;
  if (d.links && d.conn_link[conn]) {   // X2: a restore record for the shadow queue
    if (gt && lane == 0) gt[i] = EgressRef{0ull, d.conn_base[conn], 0u};
    const u32 dest = d.conn_link[conn] - 1;
    const u32 po = d.link_bbase[conn] + (d.dv_off[i] - d.dv_off[f]);
    u8* lo = d.lsend_pay + (u64)d.link_dbase[dest] + po;
    const u32 meta = m.ex_len + m.rk_len + m.props_len;
    group_copy<RD_G>(lo, slot, meta, lane);
    group_copy<RD_G>(lo + meta, slot + m.body_off, m.body_len, lane);
    if (lane == 0) {
      RDesc rd{};
      rd.pay_off = po;
      rd.body_len = m.body_len;
      rd.props_len = m.props_len;
      rd.exch = -1;
      rd.flags = MF_RESTORE | ((dv.flags & 1) ? MF_REDELIVERED : 0u);
      rd.ex_len = m.ex_len;
      rd.rk_len = m.rk_len;
      rd.expire_ms = dv.expire_ms;
      rd.ts_ms = m.ts_ms;
      rd.xid = ((u64)d.conn_link_epoch[conn] << 40) | (dv.tag & ((1ull << 40) - 1));
      rd.tq = d.conn_link_tq[conn];
      d.lsend_desc[d.link_nbase[conn] + (i - f)] = rd;
    }
    return;
  }
  u64 off = (u64)d.conn_base[conn] + d.conn_ret_bytes[conn] + d.conn_conf_bytes[conn] + d.dv_off[i] -
            d.dv_off[f];
  if (gt && lane == 0)   // (a referenced body goes after its body frame's 7-byte header)
    gt[i] = ref ? EgressRef{href, (u32)(off + dv.size - 1u), m.body_len} : EgressRef{0ull, (u32)(off + dv.size), 0u};
  if (off + dv.size > d.egress_cap) return;  // never: dequeue reserves an egress byte budget
  u8* o = (u8*)d.in->egress + off;
  u32 chno = d.ch_num[ch];
  const bool get = dv.flags & DV_GET;   // Basic.GetOk (60/71): no consumer tag, message-count last
  u32 taglen = get ? 0u : d.cons_tag_len[dv.cons];
  u32 mp = (get ? 4 + 4 : 4 + 1 + taglen) + 8 + 1 + 1 + m.ex_len + 1 + m.rk_len;
  u64 dtag = dv.tag;
  // method frame: scalar fields by lane 0, the variable-length strings (consumer tag,
  // exchange, routing key) by all lanes in parallel (no serial byte-load chains)
  const u32 p_tag = 7 + 4 + (get ? 0 : 1), p_ex = p_tag + taglen + 8 + 1 + 1, p_rk = p_ex + m.ex_len + 1;
  if (lane == 0) {
    put_frame_hdr(o, 1, chno, mp);
    wr16(o + 7, 60); wr16(o + 9, get ? 71 : 60);
    if (!get) o[11] = (u8)taglen;
    wr64(o + p_tag + taglen, dtag);
    o[p_tag + taglen + 8] = (dv.flags & 1) ? 1 : 0;
    o[p_ex - 1] = m.ex_len;
    o[p_rk - 1] = m.rk_len;
    u32 p = p_rk + m.rk_len;
    if (get) { wr32(o + p, dv.cons); p += 4; }
    o[p++] = 0xCE;
    p += put_frame_hdr(o + p, 2, chno, 12 + m.props_len);
    wr16(o + p, 60); wr16(o + p + 2, 0); wr64(o + p + 4, m.body_len);
  }
  if (!get) {
    const u8* tg = d.tpool + d.cons_tag_off[dv.cons];
    for (u32 k = lane; k < taglen; k += RD_G) o[p_tag + k] = tg[k];
  }
  for (u32 k = lane; k < m.ex_len; k += RD_G) o[p_ex + k] = slot[k];
  for (u32 k = lane; k < m.rk_len; k += RD_G) o[p_rk + k] = slot[m.ex_len + k];
  u32 hp = 8 + mp + 7 + 12;
  group_copy<RD_G>(o + hp, slot + m.ex_len + m.rk_len, m.props_len, lane);
  if (lane == 0) o[hp + m.props_len] = 0xCE;
  u32 bp = hp + m.props_len + 1;
  u32 fm = d.conn_frame_max[conn];
  u32 fmb = fm ? fm - 8 : 0xffffffffu;
  if (ref) {   // one body frame whose payload the host inserts: header, then the frame end
    if (lane == 0) {
      put_frame_hdr(o + bp, 3, chno, m.body_len);
      o[bp + 7] = 0xCE;
    }
    return;
  }
  const u8* body = slot + m.body_off;
  for (u32 b0 = 0; b0 < m.body_len; b0 += fmb) {
    u32 bl = m.body_len - b0 < fmb ? m.body_len - b0 : fmb;
    if (lane == 0) put_frame_hdr(o + bp, 3, chno, bl);
    group_copy<RD_G>(o + bp + 7, body + b0, bl, lane);
    if (lane == 0) o[bp + 7 + bl] = 0xCE;
    bp += bl + 8;
  }
}

// confirms: one thread per connection writes its channels' coalesced confirm frames:
// Basic.Ack(last, multiple) when every publish of the channel in this step was stored,
// else Basic.Nack(last, multiple, requeue=0) over the step's whole range — a publisher
// may resend a nacked message, it never loses an acked one (FrameStage.scala:571-596
// confirms everything it asked the entities to store; drops are ours: ring full, no memory)
DEV void render_confirms(const DS& d, u32 c) {
  const u32 ng = d.conn_gempty[c];
  if (ng) {   // Basic.GetEmpty (60/72, empty cluster-id) frames close the connection's region
    u8* e = (u8*)d.in->egress + (u64)d.conn_base[c] + d.conn_total[c] - 13u * ng;
    const u32 chno = d.conn_gempty_ch[c];
    for (u32 k = 0; k < ng; ++k, e += 13) {
      put_frame_hdr(e, 1, chno, 5);
      wr16(e + 7, 60); wr16(e + 9, 72);
      e[11] = 0;
      e[12] = 0xCE;
    }
  }
  u32 conf = d.conn_conf_bytes[c];
  u8* o = (u8*)d.in->egress + (u64)d.conn_base[c] + d.conn_ret_bytes[c];
  u32 p = 0;
  for (u32 l = 0; l < d.chpc; ++l) {
    u32 ch = c * d.chpc + l;
    u32 cnt = d.ch_pub_cnt[ch];
    const bool fail = d.ch_pub_fail[ch] != 0;
    if (fail) d.ch_pub_fail[ch] = 0;
    if (!cnt) continue;
    d.ch_pub_cnt[ch] = 0;
    if (!d.ch_confirm[ch]) continue;
    u64 last = d.ch_confirm_next[ch] + cnt - 1;
    d.ch_confirm_next[ch] = last + 1;
    u32 chno = d.ch_num[ch];
    if (p + 21 > conf) break;
    put_frame_hdr(o + p, 1, chno, 13);
    wr16(o + p + 7, 60); wr16(o + p + 9, fail ? 120 : 80);
    wr64(o + p + 11, last);
    o[p + 19] = cnt > 1 ? 1 : 0;
    o[p + 20] = 0xCE;
    p += 21;
    atomicAdd(&d.ctr->n_confirm_frames, 1u);
  }
}

// returns: one wave per returned publish (Basic.Return 312/313 + header + body)
DEV void render_return(const DS& d, u32 i, u32 lane) {
  u32 p = d.ret_list[i];
  const Pub pb = d.pubs[p];
  u32 code = d.pub_ret[p];
  u8* o = (u8*)d.in->egress + (u64)d.conn_base[pb.conn] + (d.pub_ret_off[p] - d.conn_ret_min[pb.conn]);
  const u8* w = d.work;
  // channel number from the publish command's frame
  u32 chno = d.ch_num[pb.chslot];
  const char* txt = code == 312 ? "The exchange cannot route the result of a Publish"
                                : "The exchange cannot deliver to a consumer when the immediate flag is set";
  u32 tl = 0;
  while (txt[tl]) ++tl;
  u32 mp = 4 + 2 + 1 + tl + 1 + pb.ex_len + 1 + pb.rk_len;
  if (lane == 0) {
    u32 q = 0;
    q += put_frame_hdr(o, 1, chno, mp);
    wr16(o + q, 60); wr16(o + q + 2, 50); q += 4;
    wr16(o + q, code); q += 2;
    o[q++] = (u8)tl;
    for (u32 k = 0; k < tl; ++k) o[q + k] = (u8)txt[k];
    q += tl;
    o[q++] = (u8)pb.ex_len;
    for (u32 k = 0; k < pb.ex_len; ++k) o[q + k] = w[pb.ex_off + k];
    q += pb.ex_len;
    o[q++] = (u8)pb.rk_len;
    for (u32 k = 0; k < pb.rk_len; ++k) o[q + k] = w[pb.rk_off + k];
    q += pb.rk_len;
    o[q++] = 0xCE;
    q += put_frame_hdr(o + q, 2, chno, 12 + pb.props_len);
    wr16(o + q, 60); wr16(o + q + 2, 0); wr64(o + q + 4, pb.body_size);
  }
  u32 hp = 8 + mp + 7 + 12;
  wave_copy(o + hp, w + pb.props_off, pb.props_len);
  if (lane == 0) o[hp + pb.props_len] = 0xCE;
  u32 bp = hp + pb.props_len + 1;
  u32 fm = d.conn_frame_max[pb.conn];
  u32 fmb = fm ? fm - 8 : 0xffffffffu;
  // body from ingress fragments, re-split at the connection's frame size
  u32 fi = 0, fo = 0;
  for (u32 b0 = 0; b0 < pb.body_size; b0 += fmb) {
    u32 bl = pb.body_size - b0 < fmb ? pb.body_size - b0 : fmb;
    if (lane == 0) put_frame_hdr(o + bp, 3, chno, bl);
    u32 done = 0;
    while (done < bl) {
      Frag fg = d.frags[pb.frag0 + fi];
      u32 take = fg.len - fo < bl - done ? fg.len - fo : bl - done;
      wave_copy(o + bp + 7 + done, w + fg.off + fo, take);
      done += take;
      fo += take;
      if (fo == fg.len) { ++fi; fo = 0; }
    }
    if (lane == 0) o[bp + 7 + bl] = 0xCE;
    bp += bl + 8;
  }
}

// blocks [0, RC_RET_BLOCKS): returns, grid-stride, one wave each; the rest: confirms,
// one thread per connection
#define RC_RET_BLOCKS 512
DEV void render_rc(const DS& d, u32 blk);
// one launch for all egress rendering: returns / confirms blocks first, then one wave per
// delivery (the two write disjoint byte ranges of each connection's egress)
__global__ __launch_bounds__(256) void k_render(DS d, u32 n_rc) {
  if (blockIdx.x < n_rc) { render_rc(d, blockIdx.x); return; }
  const u32 n = d.ctr->n_deliv;
  const u32 ng = ((gridDim.x - n_rc) * blockDim.x) / RD_G;
  const u32 g = ((blockIdx.x - n_rc) * blockDim.x + threadIdx.x) / RD_G;
  const u32 lane = threadIdx.x % RD_G;
  for (u32 i = g; i < n; i += ng) render_deliv(d, i, lane);
}
DEV void render_rc(const DS& d, u32 blk) {
  if (blk >= RC_RET_BLOCKS) {
    u32 c = (blk - RC_RET_BLOCKS) * blockDim.x + threadIdx.x;
    if (c < d.c_max) render_confirms(d, c);
    return;
  }
  u32 n = d.ctr->n_returns;
  if (n > d.pub_max) n = d.pub_max;
  const u32 lane = lane_id();
  for (u32 i = (blk * blockDim.x + threadIdx.x) >> 6; i < n; i += RC_RET_BLOCKS * 4) render_return(d, i, lane);
}

// ============================================================================ post / final
// (a last-block ticket here to fold k_host_out in costs more than the launch it saves:
// hundreds of blocks serialise on the ticket word)
DEV void final_step(const DS& d);
DEV void host_out_copies(const DS& d, u64 gtid, u64 gsz);
// fin (no persistence: nothing runs after it): the host-visible copies and, by the last
// block to finish (ticket), the log tail + counters (fused k_host_out)
__global__ __launch_bounds__(256) void k_post(DS d, u32 fin) {
  __shared__ u32 s_last;
  u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  u32 n = d.ctr->n_deliv;
  u32 msg = INVALID, q = 0;
  u64 qpos = 0;
  bool aa = false;
  if (i < n) {
    const Deliv& dv = d.deliv[i];
    aa = dv.flags & 2;
    msg = dv.msg;
    q = dv.q;
    qpos = dv.qpos;
    const u32 ch = dv.chslot;
    if (i + 1 == n || d.deliv[i + 1].chslot != ch) d.ch_next_tag[ch] = dv.tag + 1;
  }
  wave_consumed(d, msg, q, qpos, 0u, aa);
  wave_release(d, msg, aa);
  const u32 nd = d.tot[TS_NDEFER], gs = gridDim.x * blockDim.x;
  for (u32 b = 0; b < nd; b += gs)   // grid-uniform trip count (wave_release ballots)
    wave_release(d, b + i < nd ? d.defer_free[b + i] : INVALID, b + i < nd);
  // consumers a light control section activated (cons_active 2, applied by this or an
  // earlier step's k_stage) take deliveries from the next step on: this step's dequeue (it
  // ran before this kernel) rendered none for them, so its egress -- behind which the front
  // end releases the Basic.ConsumeOk (Frontend::send_after) -- never holds a Basic.Deliver
  // that overtakes the ConsumeOk.  (Here and not in the next step's k_stage: with the
  // overlapped engine that k_stage may run beside this step's k_dequeue; a step that stages
  // writes waits for the previous step's routing half, so no 2 written after this point is
  // flipped by it)
  for (u32 c = i; c < d.cons_max; c += gridDim.x * blockDim.x)
    if (d.cons_active[c] == 2u) d.cons_active[c] = 1u;
  // reset per-connection scratch (fused k_post2)
  if (i < d.c_max) {
    d.conn_dfirst[i] = INVALID;
    d.conn_dlast[i] = INVALID;
    d.conn_ret_bytes[i] = 0;
    d.conn_ret_min[i] = INVALID;
    d.conn_gempty[i] = 0;
  }
  if (!fin) return;
  host_out_copies(d, i, (u64)gridDim.x * blockDim.x);
  // every block's releases are done (their atomics returned) before its ticket
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(&d.tot[TS_POST_TICKET], 1u) == gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (threadIdx.x == 0) {
    d.tot[TS_POST_TICKET] = 0;
    final_step(d);
  }
}


DEV void final_step(const DS& d) {
  // advance the log tail over fully released blocks (K11)
  u64 head = *d.log_head, tail = *d.log_tail;
  while (tail < head) {
    u64 blk_idx = tail / d.log_block;
    if (blk_idx == head / d.log_block) break;
    if (d.log_live[blk_idx % d.n_log_blocks] > 0) break;
    tail = (blk_idx + 1) * d.log_block;
  }
  if (tail > head) tail = head;
  *d.log_tail = tail;
  if (d.spill_bytes) {   // the spill ring's tail, the same way
    const u64 sh = *d.spill_head;
    u64 st = *d.spill_tail;
    while (st < sh) {
      const u64 bi = st / d.log_block;
      if (bi == sh / d.log_block) break;
      if (d.spill_live[bi % d.n_spill_blocks] > 0) break;
      st = (bi + 1) * d.log_block;
    }
    *d.spill_tail = st > sh ? sh : st;
    d.spill_tail_lag[d.in->step % SPILL_LAG] = *d.spill_tail;
  }
  Counters* c = d.ctr;
  c->log_head = head;
  c->log_tail = tail;
  c->msg_free_top = *d.msg_free_top;
  c->n_live_msgs = d.msg_max - *d.msg_free_top;
  c->live_bytes = *d.live_bytes;
  c->n_dget = d.tot[TS_NDGET];
  if (d.links)
    for (u32 r = 0; r < d.world; ++r) d.xchg[XC_ACK_N + r] = d.lk_cnt[r] < d.lk_cap ? d.lk_cnt[r] : d.lk_cap;
  *d.ctr_host = *c;
  // open the step's egress gate: the SDMA engine, polling it, starts the D2H of this
  // step's egress now.  The rendered bytes left their L2s at the earlier kernels' ends;
  // the system-scope release covers this kernel's own stores (vector store, system scope)
  const u64 gate = d.in->gate;
  if (gate) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store((i64*)gate, (i64)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// persistence: size + pack the step's persist records (header + message bytes) into the
// host-mapped persist buffer; the host writes them to the store before it releases the
// step's publisher confirms (write-behind with confirm gating)
__global__ void k_persist_size(DS d) {
  u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  u32 n = d.ctr->n_persist;
  if (n > d.persist_max) n = d.persist_max;
  if (i >= n) return;
  // a message's bytes travel once per step: with its first record (claimed through the
  // otherwise unused MsgEnt.pad, zeroed when the message is stored); its other queues'
  // records are headers only (PersistHdr.size == sizeof(PersistHdr))
  MsgEnt& m = d.msgs[d.prec[i].msg];
  const u32 bytes = (m.ex_len + m.rk_len + m.props_len + m.body_len + 7u) & ~7u;
  const bool first = atomicCAS(&m.pad, 0u, 1u) == 0u;
  d.ps_size[i] = (u32)sizeof(PersistHdr) + (first ? bytes : 0u);
}

__global__ __launch_bounds__(256) void k_persist_pack(DS d) {
  u32 lane = lane_id();
  u32 n = d.ctr->n_persist;
  if (n > d.persist_max) n = d.persist_max;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    u64 used = d.tot[TS_PERSIST];
    d.ctr->persist_used = (u32)(used < d.persist_bytes ? used : d.persist_bytes);
  }
  const u32 nw = (gridDim.x * blockDim.x) >> 6;
  for (u32 i = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < n; i += nw) {
    const PersistRec r = d.prec[i];
    const MsgEnt m = d.msgs[r.msg];
    u64 off = d.ps_off[i];
    u32 sz = d.ps_size[i];
    if (off + sz > d.persist_bytes) {
      if (lane == 0) atomicAdd(&d.ctr->n_persist_overflow, 1u);
      continue;
    }
    u8* o = d.ps_persist[d.in->pslot] + off;
    const u8* slot = msg_slot(d, m.log_off);
    if (lane == 0) {
      PersistHdr h;
      h.msg_id = (i64)m.msg_id; h.ts_ms = m.ts_ms; h.qpos = r.qpos; h.expire_ms = r.expire_ms;
      h.q = r.q; h.body_len = m.body_len; h.props_len = m.props_len; h.ex_len = m.ex_len; h.rk_len = m.rk_len;
      h.size = sz;
      *(PersistHdr*)o = h;
    }
    if (sz == sizeof(PersistHdr)) continue;   // header only: the bytes ride the message's first record
    u32 meta = m.ex_len + m.rk_len + m.props_len;
    wave_copy(o + sizeof(PersistHdr), slot, meta);
    wave_copy(o + sizeof(PersistHdr) + meta, slot + m.body_off, m.body_len);
  }
}

// egress D2H on a few workgroups (copy_engine=2): 16-B loads from HBM, 16-B stores into
// mapped pinned memory; PCIe is the limit, so a handful of CUs saturate it
__global__ __launch_bounds__(256) void k_copy_out(u8* dst, const u8* src, u64 n) {
  const u64 gtid = blockIdx.x * blockDim.x + threadIdx.x, gsz = (u64)gridDim.x * blockDim.x;
  const u64 nv = n >> 4;
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  for (u64 i = gtid; i < nv; i += gsz) ((v4u*)dst)[i] = __builtin_nontemporal_load(((const v4u*)src) + i);
  for (u64 i = (nv << 4) + gtid; i < n; i += gsz) dst[i] = src[i];
}

// the same, sized on the device (the step's egress byte count): launched right behind the
// step's kernels, with no host round trip between render and copy (copy_engine=2, overlap)
__global__ __launch_bounds__(256) void k_copy_out_dev(u8* dst, const u8* src, const Counters* c) {
  const u64 n = c->egress_bytes;
  const u64 gtid = blockIdx.x * blockDim.x + threadIdx.x, gsz = (u64)gridDim.x * blockDim.x;
  const u64 nv = n >> 4;
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  for (u64 i = gtid; i < nv; i += gsz) ((v4u*)dst)[i] = __builtin_nontemporal_load(((const v4u*)src) + i);
  for (u64 i = (nv << 4) + gtid; i < n; i += gsz) dst[i] = src[i];
}

// copy the step's small host-visible results to their host-mapped mirrors in one pass
// (16-B stores, grid-stride) once the whole step has run
DEV void copy16(u8* dst, const u8* src, u64 n, u64 gtid, u64 gsz) {
  u64 nv = n >> 4;
  for (u64 i = gtid; i < nv; i += gsz) ((uint4*)dst)[i] = ((const uint4*)src)[i];
  for (u64 i = (nv << 4) + gtid; i < n; i += gsz) dst[i] = src[i];
}

DEV void host_out_copies(const DS& d, u64 gtid, u64 gsz);
__global__ __launch_bounds__(256) void k_host_out(DS d) {
  if (blockIdx.x == 0 && threadIdx.x == 0) final_step(d);   // log tail, counters -> host
  host_out_copies(d, blockIdx.x * blockDim.x + threadIdx.x, (u64)gridDim.x * blockDim.x);
}

DEV void host_out_copies(const DS& d, u64 gtid, u64 gsz) {
  u32 nseg = d.in->nseg;
  copy16((u8*)d.seg_out_h, (const u8*)d.seg_out, (u64)nseg * sizeof(SegOut), gtid, gsz);
  copy16((u8*)d.conn_out_h, (const u8*)d.conn_out, (u64)d.c_max * sizeof(ConnOut), gtid, gsz);
  copy16((u8*)d.conn_conf_h, (const u8*)d.conn_conf_bytes, (u64)d.c_max * 4, gtid, gsz);
  u32 nc = d.ctr->n_ctrl;
  if (nc > d.seg_max * 2) nc = d.seg_max * 2;
  copy16((u8*)d.ctrl_rec_h, (const u8*)d.ctrl_rec, (u64)nc * sizeof(CtrlRec), gtid, gsz);
  u64 cb = d.ctr->ctrl_bytes;
  if (cb > d.ctrl_cap) cb = d.ctrl_cap;
  copy16(d.ctrl_h, d.ctrl, cb, gtid, gsz);
  if (d.persist) {
    u32 nr = d.ctr->n_consumed;
    if (nr > d.persist_max) nr = d.persist_max;
    copy16((u8*)d.ps_crec[d.in->pslot], (const u8*)d.crec, (u64)nr * sizeof(ConsumedRec), gtid, gsz);
  }
}

// ============================================================================ Basic.Get
// Basic.Get (60/70) between steps, while the connection is paused behind the command
// (FrameStage.scala:1199-1229: Pull(1) -> GetOk / GetEmpty; QueueEntity.scala:318-393).
// One wave: TTL skip of up to 64 head entries (K12), then the head message gets the
// channel's next delivery tag.  Manual ack: a pending window slot that Basic.Ack/Nack/
// Reject/Recover/channel close resolve exactly like a consumer delivery (k_chan_advance);
// no-ack: a done slot, the message is released now.  GetOk + content header + body frames
// (split at the connection's frame-max) are rendered into `out` (host-mapped).
// Consumer bookkeeping uses the spare consumer slot cons_max.
__global__ __launch_bounds__(64) void k_basic_get(DS d, u32 q, u32 ch, u32 noack, i64 now, u8* out, u64 out_cap,
                                                  GetRes* res) {
  u32 lane = lane_id();
  u64 head = d.q_head[q], tail = d.q_tail[q];
  const u64 mask = d.q_ring_mask[q];
  const Desc* ring = d.ring + d.q_ring_off[q];
  u32 nexp = 0;
  bool more_expired = false;
  if (head < tail) {
    u64 idx = head + lane;
    bool valid = idx < tail;
    Desc ds;
    ds.msg = INVALID; ds.expire_ms = 0; ds.flags = 0;
    if (valid) ds = ring[idx & mask];
    bool exp = valid && ds.expire_ms != 0 && ds.expire_ms <= now;
    u64 live = __ballot(valid && !exp);
    nexp = live ? (__ffsll((unsigned long long)live) - 1) : __popcll(__ballot(valid));
    more_expired = !live && head + nexp < tail;
    bool mine = lane < nexp;
    bool rec = mine && d.q_durable[q] && (d.msgs[ds.msg].flags & MF_PERSIST);
    u64 rm = __ballot(rec);
    if (rec) {
      ConsumedRec r;
      r.msg_id = (i64)d.msgs[ds.msg].msg_id;
      r.qpos = idx;
      r.q = q;
      r.kind = 1;
      r.pad[0] = r.pad[1] = 0;
      res->exp[__popcll(rm & lanemask_lt())] = r;
    }
    wave_release(d, ds.msg, mine);
    if (lane == 0) res->n_exp = __popcll(rm);
    head += nexp;
  } else if (lane == 0) {
    res->n_exp = 0;
  }
  if (head >= tail || more_expired) {
    if (lane == 0) {
      d.q_head[q] = head;
      res->status = more_expired ? GET_RETRY : GET_EMPTY;
      res->msg_count = (u32)(tail - head);
      res->out_len = 0;
    }
    return;
  }
  if (head >= d.q_cold_lim[q] && (d.msgs[ring[head & mask].msg].log_off & COLD_BIT)) {
    if (lane == 0) {   // the host pages the queue's head back in, then asks again
      d.q_head[q] = head;
      res->status = GET_COLD;
      res->msg_count = (u32)(tail - head);
      res->out_len = 0;
    }
    return;
  }
  const Desc ds = ring[head & mask];
  const MsgEnt m = d.msgs[ds.msg];
  const u32 conn = ch / d.chpc;
  const u32 ucap = d.ucap_mask + 1;
  const u32 msg_count = (u32)(tail - head - 1);
  u32 mp = 4 + 8 + 1 + 1 + m.ex_len + 1 + m.rk_len + 4;
  u32 fm = d.conn_frame_max[conn];
  u32 fmb = fm ? fm - 8 : 0xffffffffu;
  u32 nb = m.body_len ? (m.body_len + fmb - 1) / fmb : 0;
  u64 need = 8ull + mp + 8 + 12 + m.props_len + m.body_len + 8ull * nb;
  u32 st = need > out_cap ? GET_NO_SPACE : (d.ch_win[ch] >= ucap ? GET_WINDOW_FULL : GET_OK);
  if (st != GET_OK) {
    if (lane == 0) {
      d.q_head[q] = head;
      res->status = st;
      res->msg_count = (u32)(tail - head);
      res->out_len = 0;
    }
    return;
  }
  const u64 tag = d.ch_next_tag[ch];
  const bool redelivered = ds.flags & 1;
  if (lane == 0) {
    d.ch_next_tag[ch] = tag + 1;
    d.ch_win[ch] += 1;
    USlot u;
    u.state = noack ? US_DONE : US_PENDING;
    u.msg = ds.msg;
    u.q = q;
    u.cons = d.cons_max;
    u.qpos = head;
    u.expire_ms = ds.expire_ms;
    d.uwin[(u64)ch * ucap + ((tag - 1) & d.ucap_mask)] = u;
    if (!noack) { d.ch_unacked[ch] += 1; d.cons_unacked[d.cons_max] += 1; }
    if (d.ch_dirty[ch] == 0) {   // k_chan_advance walks the window at the next step
      d.ch_dirty[ch] = 1;
      u32 k = *d.n_dirty;
      d.dirty_list[k] = ch;
      *d.n_dirty = k + 1;
    }
    d.q_head[q] = head + 1;
    res->status = GET_OK;
    res->msg_count = msg_count;
    res->out_len = (u32)need;
    res->tag = tag;
    res->msg_id = (i64)m.msg_id;
    res->qpos = head;
    res->persist = d.q_durable[q] && (m.flags & MF_PERSIST) ? 1u : 0u;
  }
  // render: GetOk(tag, redelivered, exchange, routing-key, message-count) + header + body
  const u8* slot = msg_slot(d, m.log_off);
  const u32 chno = d.ch_num[ch];
  if (lane == 0) {
    u32 p = 0;
    p += put_frame_hdr(out + p, 1, chno, mp);
    wr16(out + p, 60); wr16(out + p + 2, 71); p += 4;
    wr64(out + p, tag); p += 8;
    out[p++] = redelivered ? 1 : 0;
    out[p++] = m.ex_len;
    for (u32 k = 0; k < m.ex_len; ++k) out[p + k] = slot[k];
    p += m.ex_len;
    out[p++] = m.rk_len;
    for (u32 k = 0; k < m.rk_len; ++k) out[p + k] = slot[m.ex_len + k];
    p += m.rk_len;
    wr32(out + p, msg_count); p += 4;
    out[p++] = 0xCE;
    p += put_frame_hdr(out + p, 2, chno, 12 + m.props_len);
    wr16(out + p, 60); wr16(out + p + 2, 0); wr64(out + p + 4, m.body_len);
  }
  u32 hp = 8 + mp + 7 + 12;
  wave_copy(out + hp, slot + m.ex_len + m.rk_len, m.props_len);
  if (lane == 0) out[hp + m.props_len] = 0xCE;
  u32 bp = hp + m.props_len + 1;
  const u8* body = slot + m.body_off;
  for (u32 b0 = 0; b0 < m.body_len; b0 += fmb) {
    u32 bl = m.body_len - b0 < fmb ? m.body_len - b0 : fmb;
    if (lane == 0) put_frame_hdr(out + bp, 3, chno, bl);
    wave_copy(out + bp + 7, body + b0, bl);
    if (lane == 0) out[bp + 7 + bl] = 0xCE;
    bp += bl + 8;
  }
  wave_release(d, ds.msg, noack && lane == 0);
}

// ============================================================================ spill (between steps)
// reserve `sz` bytes in the spill ring (never across its wrap), false when it is full
DEV bool spill_reserve(const DS& d, u32 sz, u64* pos) {
  unsigned long long cur = __hip_atomic_load(d.spill_head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the tail of SPILL_LAG steps ago (the oldest of the history): bytes freed since may still
  // be referenced by an egress not yet written out (spilled bodies are sent from the ring)
  u64 tail = *d.spill_tail;
  for (u32 k = 0; k < SPILL_LAG; ++k) tail = d.spill_tail_lag[k] < tail ? d.spill_tail_lag[k] : tail;
  while (true) {
    u64 h = cur;
    const u64 phys = h % d.spill_bytes;
    if (phys + sz > d.spill_bytes) h += d.spill_bytes - phys;
    if (h + sz - tail > d.spill_bytes) return false;
    const unsigned long long prev = atomicCAS((unsigned long long*)d.spill_head, cur, (unsigned long long)(h + sz));
    if (prev == cur) { *pos = h; return true; }
    cur = prev;
  }
}

// Cold bodies to host memory (host-driven, between steps, when the HBM log fills): one
// block per queue, one wave per ring entry whose body sits in the log below position
// `lim` -- the oldest part, which pins the log tail: the log is a ring, only its tail
// frees space -- skipping the first `hot` entries of a queue that has consumers (about to
// be delivered; a backlog without consumers moves from its head).
// The slot is copied into the spill ring (pinned host memory), then MsgEnt.log_off is
// switched with a CAS (a message in several queues moves once; a lost race leaves a
// never-live gap the spill tail passes).  Its log block loses the bytes, so the next
// step's final_step can advance the log tail.  Unacked deliveries stay in the log.
__global__ __launch_bounds__(256) void k_spill(DS d, u64 lim, u32 hot, unsigned long long* moved) {
  const u32 q = blockIdx.x;
  if (q >= d.q_max || d.spill_bytes == 0) return;
  spill_queue(d, q, lim, hot, 0, (u64*)moved);
}

// ============================================================================ cold store (between steps)
// Third body tier (MessageEntity.scala:174-186: idle bodies go to the store and are
// read back on demand).  Out: k_cold_pick lists spilled bodies of single-queue,
// non-persistent messages at least `hot` entries behind their queue's head; the host
// writes them from the pinned ring to the cold store; k_cold_commit switches each
// MsgEnt to COLD_BIT | store offset, frees its ring bytes and lowers q_cold_lim.
// Candidates are taken from the oldest part of the ring (slot position below `lim`, like
// k_spill's log limit): the ring is a FIFO, so only freeing its tail end makes room; a
// queue with consumers keeps its first `hot` entries resident.
// `lim` counts from the ring's tail; nothing is picked while the ring holds less than
// `min_used` bytes (the cold thread asks every 10 ms without reading the ring state)
__global__ __launch_bounds__(256) void k_cold_pick(DS d, u32 hot, u64 lim_rel, u64 min_used, ColdRec* out, u32 max_n,
                                                   u32* n_out, unsigned long long* bytes, u64 max_bytes) {
  const u32 q = blockIdx.x, lane = lane_id(), w = threadIdx.x >> 6;
  if (q >= d.q_max || !d.q_active[q] || d.spill_bytes == 0) return;
  if (*d.spill_head - *d.spill_tail < min_used) return;
  const u64 lim = *d.spill_tail + lim_rel;
  const u64 head = d.q_head[q], tail = d.q_tail[q], mask = d.q_ring_mask[q];
  const Desc* ring = d.ring + d.q_ring_off[q];
  const u64 skip = d.q_cons_n[q] ? hot : 0;
  // resume past the queue's cold prefix (cursor): a deep cold backlog is not walked again
  // at every call (it was: up to ~370 us between two steps, profiles/r5_coldprof/)
  __shared__ unsigned long long s_open;
  if (threadIdx.x == 0) s_open = ~0ull;
  __syncthreads();
  const u64 start0 = head + skip;
  u64 cur = d.q_cold_cur[q];
  if (cur < start0 || cur > tail) cur = start0;   // (the head passed it, or the slot was reset)
  u64 open = ~0ull;   // this wave's first entry that is not cold (or where it stopped)
  for (u64 b = cur + (u64)w * 64; b < tail; b += 256) {
    const u64 i = b + lane;
    bool want = false, cold = false;
    u32 msg = INVALID, sz = 0;
    u64 lo = 0;
    if (i < tail) {
      msg = ring[i & mask].msg;
      cold = msg == INVALID || msg >= d.msg_max;
      if (!cold) {
        const MsgEnt& m = d.msgs[msg];
        lo = m.log_off;
        sz = m.slot_bytes;
        cold = (lo & COLD_BIT) != 0;
        want = (lo & SPILL_BIT) && !(lo & COLD_BIT) && (lo & ~SPILL_BIT) < lim && m.refcnt == 1 &&
               !(m.flags & MF_PERSIST);
      }
    }
    const u64 nc = __ballot(i < tail && !cold);
    if (nc && open == ~0ull) open = b + (u64)(__ffsll((unsigned long long)nc) - 1);
    const u32 k = wave_reserve(n_out, want);
    bool ok = want && k < max_n;
    if (ok) ok = atomicAdd(bytes, (unsigned long long)sz) + sz <= max_bytes;
    if (want && k < max_n) {   // (a record of bytes 0 is skipped by the host)
      ColdRec r;
      r.msg = ok ? msg : INVALID; r.q = q; r.qpos = i; r.pos = lo & ~SPILL_BIT; r.cold = 0;
      r.bytes = ok ? sz : 0; r.pad = 0;
      out[k] = r;
    }
    if (__ballot(want && !ok)) {   // the batch is full
      if (b < open) open = b;
      break;
    }
  }
  if (lane == 0 && open != ~0ull) atomicMin(&s_open, (unsigned long long)open);
  __syncthreads();
  if (threadIdx.x == 0) d.q_cold_cur[q] = s_open == ~0ull ? tail : (u64)s_open;
}

__global__ void k_cold_commit(DS d, const ColdRec* recs, u32 n) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ColdRec r = recs[i];
  if (!r.bytes || r.msg >= d.msg_max) return;
  // (picked a few steps ago by the cold thread: an entry delivered since then stays spilled)
  if (d.q_head[r.q] > r.qpos) return;
  MsgEnt& m = d.msgs[r.msg];
  const u64 expect = SPILL_BIT | r.pos;
  if (atomicCAS((unsigned long long*)&m.log_off, (unsigned long long)expect, (unsigned long long)(COLD_BIT | r.cold)) !=
      expect)
    return;
  spill_free(d, expect, r.bytes);
  atomicAdd((unsigned long long*)&d.cold_live[(r.cold >> COLD_SEG_SHIFT) % COLD_SEGS], (unsigned long long)r.bytes);
  atomicMin((unsigned long long*)&d.q_cold_lim[r.q], (unsigned long long)r.qpos);
}

// In: for every queue held at q_cold_lim, the cold entries among its next `window`
// positions get a slot in the spill ring (in queue order; the scan stops where the ring
// is full) and are listed for the host, which reads their bodies into those slots;
// k_cold_in then switches them back to SPILL_BIT and moves q_cold_lim past the scan
// (to ~0 when it reached the tail: entries behind the tail are never cold)
__global__ __launch_bounds__(64) void k_cold_scan(DS d, u32 window, ColdRec* out, u32 max_n, u32* n_out,
                                                  u64* scan_end) {
  const u32 q = blockIdx.x, lane = lane_id();
  if (q >= d.q_max) return;
  const u64 lim = d.q_cold_lim[q];
  if (lim == ~0ull) return;
  const u64 head = d.q_head[q], tail = d.q_tail[q], mask = d.q_ring_mask[q];
  const Desc* ring = d.ring + d.q_ring_off[q];
  const u64 start = lim > head ? lim : head;
  const u64 stop = tail < head + window ? tail : head + window;
  u64 end = start;
  for (u64 b = start; b < stop; b += 64) {
    const u64 i = b + lane;
    u32 msg = INVALID, sz = 0;
    u64 lo = 0;
    bool cold = false;
    if (i < stop) {
      msg = ring[i & mask].msg;
      if (msg != INVALID && msg < d.msg_max) {
        lo = d.msgs[msg].log_off;
        sz = d.msgs[msg].slot_bytes;
        cold = (lo & COLD_BIT) != 0;
      }
    }
    // one ring reservation for the wave's cold bodies, in lane order
    u32 off = cold ? sz : 0;
    for (int o = 1; o < 64; o <<= 1) {
      const u32 y = __shfl_up(off, o, 64);
      if (lane >= (u32)o) off += y;
    }
    const u32 total = __shfl(off, 63, 64);
    off -= cold ? sz : 0;
    u64 pos = 0;
    u32 ok = 1, k0 = 0;
    const u64 cm = __ballot(cold);
    const u32 nc = (u32)__popcll(cm);
    if (lane == 0 && nc) {
      k0 = atomicAdd(n_out, nc);
      ok = k0 + nc <= max_n && spill_reserve(d, total, &pos) ? 1u : 0u;
    }
    ok = (u32)__shfl((int)ok, 0);
    pos = shfl64(pos, 0);
    k0 = (u32)__shfl((int)k0, 0);
    const u32 k = k0 + (u32)__popcll(cm & lanemask_lt());
    // the reserved bytes count as live from here: steps that run before k_cold_in (the
    // cold thread reads the store meanwhile) must not move the ring's tail over them
    if (cold && ok) atomicAdd((unsigned long long*)&d.spill_live[((pos + off) / d.log_block) % d.n_spill_blocks],
                              (unsigned long long)sz);
    if (cold && k < max_n) {   // (not ok: a record of bytes 0, skipped by the host)
      ColdRec r;
      r.msg = ok ? msg : INVALID; r.q = q; r.qpos = i; r.pos = pos + off; r.cold = lo & ~COLD_BIT;
      r.bytes = ok ? sz : 0; r.pad = 0;
      out[k] = r;
    }
    if (!ok) break;   // ring (or the batch) full: the rest waits for the next call
    end = b + 64 < stop ? b + 64 : stop;
  }
  if (lane == 0) scan_end[q] = end == tail ? ~0ull : end;
}

__global__ void k_cold_in(DS d, const ColdRec* recs, u32 n, const u64* scan_end) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const ColdRec r = recs[i];
    if (r.bytes && r.msg < d.msg_max) {
      // still the cold message the scan listed (not purged since): back to its ring slot;
      // else the slot's reservation is returned
      const unsigned long long expect = COLD_BIT | r.cold;
      if (atomicCAS((unsigned long long*)&d.msgs[r.msg].log_off, expect, (unsigned long long)(SPILL_BIT | r.pos)) ==
          expect)
        atomicAdd((unsigned long long*)&d.cold_live[(r.cold >> COLD_SEG_SHIFT) % COLD_SEGS],
                  (unsigned long long)(-(i64)r.bytes));
      else
        spill_free(d, SPILL_BIT | r.pos, r.bytes);
    }
  }
  if (i < d.q_max && scan_end[i] != 0) d.q_cold_lim[i] = scan_end[i];   // (0: not scanned)
}

// ============================================================================ asynchronous exchange
// Phase B of a sharded step waits here (one wave, ahead of its graph) until the exchange
// thread finished the exchange it imports: the thread writes the received counts, then the
// job's sequence number into host-mapped flag[0].  Bounded: after ~20 s the wave gives up
// and sets flag[1] (the exchange thread always releases its job, so only a lost thread
// would get there; the host reports it), so a stuck host can never wedge the queue.
// lim: s_memrealtime ticks (100 MHz) after which the job counts as lost (the host derives
// it from the exchange timeout); phase B then imports nothing -- its receive counts are
// zeroed here too (the host zeroed them before handing the job over; a job that finishes
// after the give-up must not have them imported), and the next exchange() call throws
__global__ __launch_bounds__(64) void k_xwait(const u32* flag, u32 seq, u32* gave_up, u64 lim, u32* xchg, u32 world) {
  const u64 t0 = __builtin_amdgcn_s_memrealtime();   // 100 MHz
  while (true) {
    const u32 v = __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if ((int)(v - seq) >= 0) return;
    if (__builtin_amdgcn_s_memrealtime() - t0 > lim) {
      const u32 r = threadIdx.x;
      if (r < world && r < WORLD_MAX) {
        __hip_atomic_store(&xchg[XC_RECV_N + r], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&xchg[XC_RECV_B + r], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&xchg[XC_RECV_AN + r], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&xchg[XC_RECV_AB + r], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&xchg[XC_RACK_N + r], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      if (threadIdx.x == 0) __hip_atomic_store(gave_up, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __threadfence_system();
      return;
    }
    __builtin_amdgcn_s_sleep(32);
  }
}

// the cold thread's copy of a pick / scan: the listed records into host-mapped memory
__global__ void k_side_out(const ColdRec* recs, const u32* cnt, u32 max_n, u32* out, u32* out_cnt) {
  u32 n = *cnt;
  if (n > max_n) n = max_n;
  const u32 words = n * (u32)(sizeof(ColdRec) / 4);
  const u32* src = (const u32*)recs;
  for (u32 i = blockIdx.x * blockDim.x + threadIdx.x; i < words; i += gridDim.x * blockDim.x) out[i] = src[i];
  if (blockIdx.x == 0 && threadIdx.x == 0) out_cnt[0] = n;
}

// ============================================================================ requeue (pre-step)
// run by k_dequeue (fused k_requeue): the block of a queue with requeued items gathers
// them, bitonic-sorts by queue position and pushes them back in front of the head with
// the redelivered flag (QueueEntity.scala:415-446); the last block compacts the rest
DEV void requeue_queue(const DS& d, u32 q, u64* kpos, u32* kidx, u32* cnt_p) {
  u32& cnt = *cnt_p;
  u32 tid = threadIdx.x;
  if (tid == 0) cnt = 0;
  __syncthreads();
  u32 n = *d.req_n;
  if (n > d.req_max) n = d.req_max;
  for (u32 i = tid; i < n; i += 256) {
    if (d.req[i].q == q) {
      u32 k = atomicAdd(&cnt, 1u);
      if (k < REQ_BLK) { kpos[k] = d.req[i].qpos; kidx[k] = i; }
    }
  }
  __syncthreads();
  u32 m = cnt < REQ_BLK ? cnt : REQ_BLK;
  u32 np2 = 1;
  while (np2 < m) np2 <<= 1;
  for (u32 i = m + tid; i < np2; i += 256) { kpos[i] = ~0ull; kidx[i] = INVALID; }
  __syncthreads();
  for (u32 k = 2; k <= np2; k <<= 1) {
    for (u32 j = k >> 1; j > 0; j >>= 1) {
      for (u32 i = tid; i < np2; i += 256) {
        u32 ij = i ^ j;
        if (ij > i) {
          bool up = (i & k) == 0;
          if ((kpos[i] > kpos[ij]) == up) {
            u64 t = kpos[i]; kpos[i] = kpos[ij]; kpos[ij] = t;
            u32 x = kidx[i]; kidx[i] = kidx[ij]; kidx[ij] = x;
          }
        }
      }
      __syncthreads();
    }
  }
  u64 head = d.q_head[q], tail = d.q_tail[q];
  u64 mask = d.q_ring_mask[q];
  u64 freec = mask + 1 - (tail - head);
  u32 k = m < freec ? m : (u32)freec;
  for (u32 i = tid; i < k; i += 256) {
    const ReqItem r = d.req[kidx[i]];
    Desc ds;
    ds.msg = r.msg;
    ds.flags = 1;
    ds.expire_ms = r.expire_ms;
    d.ring[d.q_ring_off[q] + ((head - k + i) & mask)] = ds;
    // consumed (agent-coherent: the compacting block of another XCD reads it after the ticket)
    __hip_atomic_store(&d.req[kidx[i]].q, INVALID, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (tid == 0) {
    d.q_head[q] = head - k;
    d.req_q_n[q] -= k;
  }
}

DEV void requeue_compact(const DS& d) {
  // one block of 256: compact the remaining (unconsumed) requeue items
  __shared__ u32 lds[256 / 64 + 1];
  u32 n = *d.req_n;
  if (n == 0) return;
  if (n > d.req_max) n = d.req_max;
  u32 run = 0;
  for (u32 b0 = 0; b0 < n; b0 += 256) {
    u32 i = b0 + threadIdx.x;
    // (fields as scalars: an aggregate copy across the scan's barriers was lowered to scratch)
    u32 rq = INVALID, rm = 0;
    u64 rp = 0;
    i64 re = 0;
    if (i < n) { rq = d.req[i].q; rm = d.req[i].msg; rp = d.req[i].qpos; re = d.req[i].expire_ms; }
    u32 keep = (i < n && rq != INVALID) ? 1 : 0;
    u32 all;
    u32 off = block_scan<256>(keep, lds, all);
    __syncthreads();
    if (keep) {   // run + off <= i: safe forward compaction
      ReqItem& o = d.req[run + off];
      o.q = rq; o.msg = rm; o.qpos = rp; o.expire_ms = re;
    }
    __syncthreads();
    run += all;
  }
  if (threadIdx.x == 0) *d.req_n = run;
}

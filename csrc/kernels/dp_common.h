// Shared device/host definitions for the MI355X AMQP data plane.
// Layouts here are mirrored by chanamq_amd/engine/layout.py (numpy dtypes);
// tests/test_layout.py checks sizes/offsets.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "step_abi.h"


#define DEV __device__ __forceinline__

// ---- command kinds (data-plane classification of an assembled command)
enum : u32 {
  CK_NONE = 0,
  CK_PUBLISH = 1,   // Basic.Publish (60/40)
  CK_ACK = 2,       // Basic.Ack (60/80)
  CK_REJECT = 3,    // Basic.Reject (60/90)
  CK_NACK = 4,      // Basic.Nack (60/120)
  CK_CONTROL = 5,   // everything else: bytes go to the host control plane
  CK_TXBUF = 6,     // publish / ack / nack / reject on a transactional channel: raw bytes
                    // to the host (buffered until Tx.Commit), connection not paused
  CK_GET = 7,       // Basic.Get (60/70) of a local queue named in the command: served in the
                    // step (DGet list), connection not paused
};

// ---- exchange types (constants.py EX_*)
enum : u32 { EX_DIRECT = 0, EX_FANOUT = 1, EX_TOPIC = 2, EX_HEADERS = 3 };


// ---- message flags
enum : u32 {
  MF_PERSIST = 1, MF_MANDATORY = 2, MF_IMMEDIATE = 4, MF_HAS_TS = 8, MF_IMPORTED = 16,
  MF_RESTORE = 32,      // recovered from the store: enqueue into exactly RDesc.tq, keep RDesc.xid
  MF_REDELIVERED = 64,  // enqueue with the redelivered flag (recovered unacks)
  MF_ONEQ = 128,        // cross-rank record routed at its origin to exactly one queue: RDesc.tq
  MF_SLOTFMT = 256,     // cross-rank record laid out as a body-log slot ([ex][rk][props] padded
                        // to 16, then the body): the owner stores it with one aligned copy
  MF_HOSTPUB = 512,     // a publish assembled by the host (larger than the connection carry):
                        // routed by its exchange, publisher channel in RDesc.pad[0], conn pad[1]
  MF_HREF = 1024        // (Pub only) the body is one contiguous run of this step's new ingress
                        // bytes, at payload offset Pub.pad: MsgEnt.href = StepIn.ingress_host + it
};

// ---- unacked slot states
enum : u32 { US_FREE = 0, US_PENDING = 1, US_ACKED = 2, US_REQUEUE = 3, US_DONE = 4 };


// StepIn.ref_back flag: only bodies in the host spill ring go by reference this step
#define REF_SPILL_ONLY 0x80000000u
struct StepIn {         // host -> device per step (96 B)
  u32 nseg;
  u32 flags;
  i64 now_ms;
  u64 step;
  u64 id_ms;            // epoch ms for snowflake ids
  u32 worker;           // snowflake worker id (rank)
  u32 nget;             // Basic.Get requests of this step (DS.get_req, <= GET_STEP_MAX)
  u64 egress;           // device pointer: this step's egress slot (engine rotates slots)
  u32 nunp;             // connections to unpause before this step's frame scan (DS.unpause_req)
  u32 pslot;            // host persist slot of this step (DS.ps_persist / ps_crec, rotating)
  u64 ingress;          // device pointer: this step's ingress slot (engine rotates INGRESS_SLOTS)
  // the value word of this step's egress gate (an HSA signal, 1 while armed; 0 = none): the
  // step's last kernel stores 0 once every byte is rendered, which releases the egress D2H
  // the host queued on the SDMA engine at launch -- no host round trip between render and
  // copy
  u64 gate;
  // deferred control writes (DS.delta_h of this parity, packed by the host): bytes, 0 = none.
  // k_stage applies them first, before the step reads any table
  u32 delta_bytes;
  // body tier upkeep riding the step (k_dequeue, no pipeline drain): queued bodies in the
  // oldest spill_frac / 65536 of the HBM log, past the first spill_hot entries of a queue
  // with consumers, move to the host spill ring, at most spill_budget bytes this step
  u32 spill_frac;
  u32 spill_hot;
  u32 spill_budget;
  // egress by reference (bodies are not sent back over PCIe): a delivery whose
  // body is a run of the host ingress payload of a step no more than ref_back steps back
  // (0xffffffff: off) and at least ref_min bytes long is rendered without its body bytes --
  // the step's gather table (EgressRef, after the rendered bytes) tells the host where they
  // go.  ingress_host = this step's payload in host memory (0: its bodies are not referable)
  u32 ref_back;
  u32 ref_min;
  u64 ingress_host;
  // a consumer takes at most max(1, dcap_bytes / s) deliveries this step, s = the rendered
  // size of the first one (0: no byte cap): bounds one connection's egress per step, so a
  // deep-backlog drain does not stretch the front end's IO phase for everyone else
  u32 dcap_bytes;
  u32 h2d_polls;        // k_h2d_wait's poll budget (0: 2^24, ~20 s; tests lower it)
  // the value word of the HSA completion signal of this step's ingress copy when the host
  // queued it on an SDMA engine itself (0: a runtime copy the step's stream waits for):
  // k_h2d_wait holds the step's frame scan until it reads 0
  u64 h2d_sig;
  u64 h2d_sig2;         // the second half's copy of a payload split over two engines (0: none)
};
static_assert(sizeof(StepIn) == 128, "StepIn layout");



struct Cmd {            // one assembled command (device internal)
  u32 conn;
  u32 ch;               // channel number
  u32 kind;
  u32 m_off;            // method payload offset in work buffer (absolute)
  u32 m_len;
  u32 h_off;            // content-header payload offset
  u32 h_len;
  u32 frag0;            // first body fragment
  u32 nfrag;
  u32 body_size;
  u32 seg;
  u32 raw_off;          // first byte of the command's first frame (for control copies)
  u32 raw_len;
  u32 pad[3];
};

struct Frag { u32 off, len; };

struct Pub {            // decoded Basic.Publish
  u32 conn;
  u32 chslot;           // -1 if unknown
  i32 exch;             // exchange slot, -1 unknown
  u32 rk_off;           // routing key bytes in work buffer
  u32 rk_len;
  u32 ex_off;           // exchange name bytes in work buffer
  u32 ex_len;
  u32 props_off;        // property bytes (flags + values) in work buffer
  u32 props_len;
  u32 frag0, nfrag;
  u32 body_size;
  u32 flags;            // MF_*
  u32 nwords;           // routing-key word count (topic)
  i64 expire_ms;        // absolute, 0 = never
  i64 ts_ms;
  u64 keyhash;          // fnv1a64(routing key); MF_RESTORE: target queue slot
  u32 nq;               // queues routed to
  u32 slot_bytes;       // bytes reserved in the body log
  u32 msg;              // message-table index, -1 if not stored
  u32 pad;
  u64 xid;              // MF_RESTORE: message id to keep; local publish (route pass 0):
                        // its only remote queue, ~0 if it routed to none or several
};

// cross-rank publish record (sharded queues): the ingress rank ships each publish once
// per destination rank that owns >= 1 of its queues; the owner re-routes it against its
// replicated binding tables restricted to local queues.  Payload = [ex][rk][props][body].
struct RDesc {
  u32 pay_off;          // payload offset within the sender's region for this destination
  u32 body_len;
  u32 props_len;
  i32 exch;             // exchange slot (identical on every rank: replicated control plane)
  u32 flags;            // MF_* of the original publish
  u8 ex_len, rk_len;
  u16 pad0;
  i64 expire_ms;
  i64 ts_ms;
  u64 xid;              // MF_RESTORE: the message id to keep
  u32 tq;               // MF_RESTORE / MF_ONEQ: target queue slot
  u32 pad[3];
};
static_assert(sizeof(RDesc) == 64, "RDesc layout");

// persistence (durable queue x persistent message): one record per enqueue, packed with
// the message bytes into the host-mapped persist buffer at the end of the step
struct PersistRec { u32 msg; u32 q; u64 qpos; i64 expire_ms; };

struct Ack { u32 chslot; u32 kind; u64 tag; u32 multiple; u32 requeue; };

#define SPILL_BIT (1ull << 63)   // MsgEnt.log_off: the slot lives in the host spill ring
// MsgEnt.log_off: the slot lives in the cold store on disk (third body tier, below the
// spill ring): never rendered -- k_dequeue holds a queue's deliveries at q_cold_lim, the
// first position that may be cold, until the host pages the bodies back into the ring
#define COLD_BIT (1ull << 62)
#define COLD_SEG_SHIFT 30        // cold store segments (files) of 1 GiB
#define COLD_SEGS 16384          // -> 16 TiB of cold bodies per GPU
struct ColdRec { u32 msg; u32 q; u64 qpos; u64 pos; u64 cold; u32 bytes; u32 pad; };
struct MsgEnt {         // message table (one per stored message; body stored once per rank)
  u64 log_off;          // start of slot in body log (| SPILL_BIT: in the host spill ring)
  u64 msg_id;           // snowflake id
  i64 ts_ms;
  u32 slot_bytes;
  u32 body_len;
  u32 body_off;         // offset of body inside the slot (16-aligned)
  u16 props_len;
  u8 ex_len;
  u8 rk_len;
  i32 refcnt;
  u32 flags;
  u32 pub_step;         // step the message was published (latency histogram)
  u32 pad;
  u64 href;             // host address of the body in its step's ingress payload (0: none)
};
static_assert(sizeof(MsgEnt) == 64, "MsgEnt layout");

struct Desc {           // queue ring entry
  u32 msg;
  u32 flags;            // bit0 redelivered
  i64 expire_ms;
};

struct Deliv {          // one delivery produced by the dequeue kernel
  u32 chslot;
  u32 cons;
  u32 msg;
  u32 q;
  u64 qpos;             // queue position (for requeue ordering)
  i64 expire_ms;
  u64 tag;              // delivery tag (assigned in k_tags)
  u32 flags;            // bit0 redelivered, bit1 autoack
  u32 size;             // rendered bytes
};

struct Run {            // consecutive queue entries granted to one consumer this step
  u32 ch;               // channel slot
  u32 cons;             // RUN_GET: the queue's ready count left (Basic.GetOk message-count)
  u32 cnt;
  u32 q;
  u64 qpos;             // queue position of the first entry
  u32 noack;
  u32 flags;            // RUN_GET: one Basic.Get answer (consumer slot cons_max)
};
#define RUN_GET 1u
#define DV_GET 4u       // Deliv.flags: a Basic.GetOk (Deliv.cons = message-count)

struct USlot {          // per-channel unacked window slot
  u32 state;
  u32 msg;
  u32 q;
  u32 cons;
  u64 qpos;
  i64 expire_ms;
};

struct ReqItem { u32 q; u32 msg; u64 qpos; i64 expire_ms; };

// Basic.Get result (k_basic_get -> host-mapped); exp[] = persistent messages of durable
// queues dropped by the TTL skip (their store rows go, like ConsumedRec kind 1)
#define GET_EXP_MAX 64
enum : u32 { GET_EMPTY = 0, GET_OK = 1, GET_RETRY = 2, GET_NO_SPACE = 3, GET_WINDOW_FULL = 4, GET_COLD = 5 };
struct GetRes {
  u32 status;
  u32 msg_count;        // ready messages left in the queue
  u32 out_len;          // rendered GetOk + header + body bytes
  u32 n_exp;
  u64 tag;
  i64 msg_id;
  u64 qpos;
  u32 persist;          // durable queue x persistent message
  u32 pad;
  ConsumedRec exp[GET_EXP_MAX];
};


// ---- FNV-1a 64 (host mirror: chanamq_amd/engine/layout.py fnv1a64)
DEV u64 fnv1a64_dev(const u8* p, u32 n, u64 h = 0xcbf29ce484222325ULL) {
  for (u32 i = 0; i < n; ++i) { h ^= p[i]; h *= 0x100000001b3ULL; }
  return h;
}

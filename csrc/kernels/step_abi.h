// Host-visible step ABI of the MI355X data plane: the structs the engine exchanges with
// the host every step, and the C entry points through which the native front end
// (csrc/core/frontend.cpp, built by g++ into _core) drives the engine (csrc/kernels/
// engine.hip, built by hipcc into _dataplane) without Python on the per-step path.
// Plain C++ (no HIP headers): included by both builds.
#pragma once
#include <cstdint>

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;
typedef int32_t i32;
typedef int8_t i8;
typedef int64_t i64;

// ---- per-segment status bits (SegOut.status)
enum : u32 {
  SS_OK = 0,
  SS_PAUSED = 1,        // connection paused behind a control command
  SS_CTRL = 2,          // a control command was emitted (connection now paused)
  SS_FRAME_ERROR = 4,   // malformed frame (501); host closes connection
  SS_UNEXPECTED = 8,    // frame sequence error (505)
  SS_TOO_LARGE = 16,    // command exceeds carry capacity (host fallback)
  SS_OVERFLOW = 32,     // per-step capacity hit; remainder carried
  SS_CHANNEL = 64,      // data command on a channel the device does not know (sent as control)
};

#define CTRL_TXBUF 0x80000000u   // CtrlRec.seg flag: CK_TXBUF record, low bits = wire position
#define CTRL_DGET 0x40000000u    // CtrlRec.seg flag: a Basic.Get the step decoded but could not
                                 // serve (the connection is not paused: the host serves it)

struct SegIn {          // host -> device, one per connection with bytes this step
  u32 conn;
  u32 len;              // new bytes
  u64 src;              // offset of the new bytes in the ingress payload
};

struct SegOut {         // device -> host per segment
  u32 conn;
  u32 status;
  u32 consumed;         // bytes of the virtual segment consumed
  u32 carry;            // carry length after this step
  u32 ncmds;
  u32 err_off;          // offset of the first malformed frame
  u32 pad[2];
};

// persistence: header of one packed persist record in the host-mapped persist buffer
struct PersistHdr {     // host-visible header of one packed persist record (48 B)
  i64 msg_id;
  i64 ts_ms;
  u64 qpos;
  i64 expire_ms;
  u32 q;
  u32 body_len;
  u16 props_len;
  u8 ex_len, rk_len;
  u32 size;             // bytes of this record including the header (8-aligned)
};
static_assert(sizeof(PersistHdr) == 48, "PersistHdr layout");

// a persistent message changed state in a durable queue (kind 0 consumed/acked, 1 expired,
// 2 dropped, 3 delivered awaiting ack, 4 requeued)
struct ConsumedRec { i64 msg_id; u64 qpos; u32 q; u32 kind; u32 pad[2]; };
static_assert(sizeof(ConsumedRec) == 32, "ConsumedRec layout");

struct Counters {       // per-step counters (device -> host)
  u32 n_cmds, n_frags, n_pubs, n_acks;
  u32 n_ctrl, ctrl_bytes, n_pairs, n_deliv;
  u32 egress_bytes, n_returns, n_confirm_frames, n_freed;
  u32 n_requeue, n_unroutable, n_dropped_nomem, n_expired;
  u32 n_routed_msgs, n_unknown_exchange, n_ring_full, n_acked;
  u32 n_persist, n_consumed, persist_used, n_persist_overflow;
  u32 lat_hist[32];     // deliveries by (deliver_step - publish_step), last bin = overflow
  u64 log_head, log_tail;
  u32 msg_free_top, n_live_msgs;
  i64 live_bytes;       // body-log slot bytes of live messages (exact, unlike head - tail)
  u32 n_grow;           // rings grown this step (grow_host list of RingMove)
  u32 n_dget;           // Basic.Gets decoded (and served or handed to the host) this step
  u64 spill_moved;      // body bytes this step moved to the host spill ring (StepIn.spill_*)
  // egress by reference: deliveries rendered without their body bytes (0: no gather table),
  // those bodies' bytes, and where the gather table (EgressRef[n_deliv]) starts in the
  // step's egress.  egress_bytes = bytes to copy D2H (rendered bytes + table); the wire
  // bytes are egress_bytes - table + ref_bytes
  u32 n_ref, gath_off;
  u64 ref_bytes;
};

struct CtrlRec { u32 conn; u32 off; u32 len; u32 seg; };

// a queue ring grown (moved) by the device this step: live entries [head, tail) copied from
// the old ring to the new one; the host returns the old range to its allocator
struct RingMove { u32 q, pad; u64 old_off, old_mask, new_off, new_mask, head, tail; };

struct ConnOut { u32 off; u32 len; };
// one gather entry per delivery of a step whose deliveries reference host bodies
// (Counters.n_ref > 0): the `len` body bytes at host address `src` go at offset `dst` of the
// step's rendered egress (before the byte there); len 0 = the delivery is rendered whole.
// dst never decreases along the table (deliveries are in egress order)
struct EgressRef { u64 src; u32 dst; u32 len; };
static_assert(sizeof(EgressRef) == 16, "EgressRef layout");

// Basic.Get served inside a step (k_dequeue, before the queue's consumers): the front end
// stages up to GET_STEP_MAX requests with a submit; the device answers each in the step's
// host-mapped GetOut (OK: GetOk + header + body rendered into the connection's egress like
// a delivery; EMPTY: the host sends Basic.GetEmpty; RETRY: resubmit with a later step).
// Reference: FrameStage.scala:1199-1229, QueueEntity.scala:318-393
#define GET_STEP_MAX 256
struct GetReq { u32 conn; u32 chslot; u32 q; u32 noack; };
// GONE: the request's queue slot is no longer active (deleted since the request was
// staged): the host answers it from its own view of the queue, never retries it
enum : u32 { GS_EMPTY = 0, GS_OK = 1, GS_RETRY = 2, GS_NO_SPACE = 3, GS_WINDOW_FULL = 4, GS_GONE = 5 };
struct GetOut { u32 status; u32 msg_count; };

// C entry points of one Engine (engine.hip: Engine::c_api).  All return 0 / a parity on
// success and -1 on error (message: error()).  Parity p = the double-buffered step IO set
// of a submitted step; its host-mapped outputs stay valid until the next submit of p.
#define CMQ_STEP_ABI 9
#define PSLOTS 4                // rotating host store-record slots (a step's records live PSLOTS - 1 more steps)
#define UNPAUSE_STEP_MAX 1024   // connections unpaused per step (StepIn.nunp)
struct CmqEngineApi {
  u32 abi;
  u32 c_max, seg_max, carry_cap, persist, persist_max;
  u64 ingress_cap, ctrl_cap;
  u64 carry_budget;   // per step: sum over the step's connections of (device carry + 48) <= this
  u64 log_bytes;      // HBM body log capacity (Counters.log_head - log_tail = occupancy)
  void* eng;
  int (*submit)(void* eng, const SegIn* segs, u32 nseg, const u8* payload, u64 len, i64 now_ms, u32 worker);
  int (*wait_results)(void* eng, int p);
  int (*egress_slot)(void* eng, int p);                  // egress slot of the last step of parity p
  int (*egress_copy)(void* eng, int p);                  // D2H of that step's rendered bytes
  int (*egress_wait_slot)(void* eng, int slot);
  const char* (*error)(void* eng);
  const Counters* (*counters)(void* eng, int p);
  const SegOut* (*seg_out)(void* eng, int p);
  const ConnOut* (*conn_out)(void* eng, int p);
  const CtrlRec* (*ctrl_rec)(void* eng, int p);
  const u8* (*ctrl)(void* eng, int p);
  const u8* (*egress_host)(void* eng, int slot);
  const u8* (*persist_host)(void* eng, int p);           // packed PersistHdr records (persist=1)
  const ConsumedRec* (*consumed_host)(void* eng, int p);
  u32* wblock;   // host-mapped u32[c_max]: nonzero = do not dequeue to this connection (egress back-pressure)
  const RingMove* (*grow_host)(void* eng, int p);        // rings grown in that step (Counters.n_grow)
  // u32[c_max]: publisher-confirm bytes in each connection's egress of that step — only
  // those connections wait for the step's persistence commit (null = every connection)
  const u32* (*conn_conf)(void* eng, int p);
  // ---- sharded broker (world > 1, engine built with native_xchg): submit() launches only
  // phase A of the step; the front end then calls exchange() for the previous step (count
  // exchange + bulk move, flags OR-reduced over the live ranks; -2 = a peer failed) and
  // launch_b() for this one
  u32 world, rank, native_xchg;
  int (*exchange)(void* eng, int q, u32 flags, u32* or_flags);
  int (*drop_exchange)(void* eng, int q);
  int (*launch_b)(void* eng, int p);
  // remote-consumer links on the device (X2/X3): a control sync flushes with two empty
  // no-dispatch steps (their link records and acks travel one exchange later)
  u32 links;
  int (*flush_submit)(void* eng, i64 now_ms, u32 worker);   // an empty no-dispatch step: parity
  // page-lock a front-end buffer (its ingress arenas: their H2D copy is then an async DMA
  // instead of a staged CPU copy inside submit); 0 or -1
  int (*host_register)(void* eng, void* p, u64 bytes);
  int (*host_unregister)(void* eng, void* p);
  // thread-safe wait for an egress slot's D2H (IO threads, before writing it out): unlike
  // egress_wait_slot it changes no engine state
  int (*egress_ready)(void* eng, int slot);
  // Basic.Get on the step: requests for the next submit (n <= GET_STEP_MAX), and the
  // answers of the last step of parity p (in request order)
  int (*stage_gets)(void* eng, const GetReq* reqs, u32 n);
  const GetOut* (*get_out)(void* eng, int p);
  // the NEXT submit's payload H2D queued now (overlapped single-GPU engine): 1 queued, 0 not
  // applicable, -1 error; that submit must pass the same payload
  int (*prefetch)(void* eng, const u8* payload, u64 len);
  // control writes (or unpauses) staged for the next step: 1 = the stepper should step even
  // without client bytes (null: never)
  int (*host_work)(void* eng);
  // egress by reference: deliveries of bodies from the ingress payload of the last `back`
  // steps (0 = the same step; -1 = off; -2 = only bodies spilled to the host ring), at least
  // min_bytes long, are rendered without them
  // (Counters.n_ref / EgressRef).  The caller keeps those payloads unchanged until the
  // delivering step's egress is written out
  int (*set_egress_ref)(void* eng, int back, u32 min_bytes);
  // staged control-write batches (light control sections): which 0 = the id of the batch
  // staging goes into now, 1 = the highest id every batch up to which a submitted step has
  // taken (a reply tied to batch b may leave once the step that took b has finished)
  u64 (*dl_state)(void* eng, int which);
  // the connections whose unpause the last submit on parity p carried (k_stage clears their
  // flag): the caller re-presents their carries from the next step on -- a light section's
  // kick may have been spent on a step submitted before its batch closed
  u32 (*unpaused)(void* eng, int p, const u32** conns);
};
#define GROW_MAX 4096   // grow requests reported per step

// Device-state descriptor passed by value to every data-plane kernel.
// All arrays are allocated once by Engine (engine.cpp) and sized from EngineCfg;
// nothing is allocated on the step path, so the whole step is hipGraph-capturable.
#pragma once
#include "dp_common.h"

#define CAND_MAX 8192         // frame candidates per segment held in LDS
#define ID_WORKERS 64         // snowflake worker ids per GPU (K13)
#define ID_SLOT_BITS 18       // log2(ID_WORKERS * 4096): id slots per millisecond
#define DEC_SEG_LDS 4096      // k_decode: segment prefixes in LDS up to this many segments
#define SORT_TILE 1024        // radix-sort tile (256 threads x 4): more tiles, more blocks in flight
#define TOPIC_K 256           // topic key vector: 8 words x 32 hash bits (int8 +-1)
#define TOPIC_WORDS 8
#define LAT_BINS 32
#define WORLD_MAX 16          // ranks of one sharded broker (one node: 8 GPUs)
#define INGRESS_SLOTS 3       // rotating ingress payload buffers (StepIn.ingress)
#define EGRESS_SLOTS 4        // rotating egress buffers (render of step t || D2H of t-1 .. t-3)
#define RUNS_PER_Q 64         // consumers served per queue per step (dequeue round-robin window)
#define RUN_SORT_LDS 8192     // runs sorted in LDS by k_runs (more: global-memory sort)
#define SPILL_LAG 6           // steps a freed spill-ring byte stays untouched (egress by reference)

// host-mapped xchg[] words (one array per IO parity).  [XC_SEND_N + r] / [XC_SEND_B + r]:
// records / payload bytes phase A packed for rank r; [XC_RECV_N + r] / [XC_RECV_B + r]:
// received from rank r (host-written before phase B imports them); [XC_OVF]: send
// overflow; [XC_RECV_AN + r] / [XC_RECV_AB + r]: the publish part of what rank r sent
// (the records after it are remote-consumer link deliveries, their payload after its
// bytes); [XC_LINK_N + r] / [XC_LINK_B + r]: link delivery records / bytes this step's
// render packed for rank r; [XC_ACK_N + r]: link acks packed for rank r;
// [XC_RACK_N + r]: link acks received from rank r
enum : u32 {
  XC_SEND_N = 0, XC_SEND_B = WORLD_MAX, XC_RECV_N = 2 * WORLD_MAX, XC_RECV_B = 3 * WORLD_MAX,
  XC_OVF = 4 * WORLD_MAX, XC_RECV_AN = 4 * WORLD_MAX + 4, XC_RECV_AB = 5 * WORLD_MAX + 4,
  XC_LINK_N = 6 * WORLD_MAX + 4, XC_LINK_B = 7 * WORLD_MAX + 4, XC_ACK_N = 8 * WORLD_MAX + 4,
  XC_RACK_N = 9 * WORLD_MAX + 4, XC_WORDS = 10 * WORLD_MAX + 8
};

// tot[] scratch slots (scan totals and phase bookkeeping)
enum : u32 {
  TS_RANGE_LO = 20, TS_RANGE_HI = 21,   // publish index range of the current routing phase
  TS_PAIR_BASE = 22, TS_PAIR_N = 23,    // pair base of the phase / pairs so far
  TS_NIMPORT = 24, TS_IMPORT_BASE = 25, // imported records / their work-buffer base
  TS_PERSIST = 26,                      // packed persist bytes
  TS_NRUNS = 27,                        // delivery runs of the step (k_runs)
  TS_REQ_TICKET = 28,                   // k_requeue finished-block ticket (last block compacts)
  TS_RS_TICKET = 29,                    // k_rs_hist finished-block ticket (last block: offsets)
  TS_NMOVE = 30,                        // rings moved (grown) this step (k_ring_plan)
  TS_NDEFER = 31,                       // stored messages released at the end of the step
  TS_RP_TICKET = 14,                    // k_ring_plan finished-block ticket (last block: ring moves)
  TS_XSCAN = 32,                        // + 2*r: per-destination record / byte totals
  TS_TTL_BUDGET = 64,                   // durable TTL-skip records reserved this step (k_dequeue)
  TS_NRACK = 65,                        // link acks received this step (k_import_route -> link_ack_one)
  TS_PK_TICKET = 66,                    // k_pack_scan finished-tile ticket (last tile: prefixes)
  TS_POST_TICKET = 67,                  // k_post finished-block ticket (last block: final_step)
  TS_NCADEF = 68,                       // channels k_chan_advance deferred (store-record budget)
  TS_NDGET = 69,                        // Basic.Get commands the frame scan decoded (DGet list)
  TS_SPILL_USED = 70,                   // bytes of StepIn.spill_budget reserved this step (k_dequeue)
  TS_DQ_TICKET = 71                     // k_dequeue finished-block ticket (last block: the step's runs)
};

// Basic.Get decoded from a connection's bytes by the frame scan (no host round trip): served
// by k_dequeue with the host-staged requests; GetOk rendered like a delivery, GetEmpty
// rendered at the end of the connection's egress; a Get the step cannot serve (window full,
// cold head, step full) goes to the host as a control record (CTRL_DGET) and is served there
#define DGET_MAX 4096
struct DGet { u32 conn, chslot, q, noack, raw_off, raw_len, seg, pad; };

// remote-consumer link ack (X3): the connection side consumed message `xid` (owner's
// epoch << 40 | owner's delivery tag) of shadow queue `tq`
struct AckRec { u32 tq; u32 pad; u64 xid; };

// StepIn.flags
enum : u32 {
  SF_NODISPATCH = 1   // flush / host step of a sharded node: no grants (nothing rendered or
                      // shipped to links), no TTL skip on live link shadows
};

struct DS {
  // ---------------- sizes
  u32 c_max, chpc, q_max, x_max, cons_max, seg_max;
  u32 carry_cap, cmd_max, frag_max, pub_max, ack_max, pair_max, deliv_max, msg_max;
  u32 ucap_mask, deliver_cap, chmap_size, xhash_mask, dhash_mask, tb_max, tb_pad, req_max;
  u32 q_bits, ch_bits, hash_wildcard, frame_max_global;
  u64 log_bytes, log_block, n_log_blocks, work_cap, ingress_cap, egress_cap, ctrl_cap, ring_pool;

  // ---------------- step io
  StepIn* in;               // device copy of the step's StepIn (k_stage writes it)
  const SegIn* segs;        // device copy of the step's segments (k_stage writes them)
  const StepIn* in_h;       // host-mapped: the host's staging of them (read once, by k_stage)
  const SegIn* segs_h;
  const u8* delta_h;        // host-mapped: this parity's deferred control writes (StepIn.delta_bytes)
  const u8* ingress;
  SegOut* seg_out;          // device; published to seg_out_h at the end of the step
  Counters* ctr;            // device
  Counters* ctr_host;       // host-mapped
  ConnOut* conn_out;        // device [c_max]
  u8* ctrl;                 // device
  CtrlRec* ctrl_rec;        // device [seg_max * 2]
  // host-mapped mirrors, written once by k_host_out after every other kernel: mid-step
  // stores over PCIe would queue behind the previous step's egress DMA
  SegOut* seg_out_h;
  ConnOut* conn_out_h;
  u8* ctrl_h;
  CtrlRec* ctrl_rec_h;
  RingMove* grow_h;         // host-mapped: rings grown this step (the host reclaims the old ones)
  u32* conn_conf_h;         // host-mapped: conn_conf_bytes of the step (confirm-gated connections)
  RingMove* moves;          // this step's ring moves (k_ring_plan -> k_ring_moves)
  u32* defer_free;          // [pub_cap] messages stored without a queue (pair table full): k_post frees
  u64* ring_top;            // ring pool bump pointer (shared with the host allocator)
  u64* q_max_cap;           // per queue ring growth limit (0 = the pool)
  u64* q_enq_tail;          // per queue tail before this step's enqueue (k_ring_plan -> k_enqueue)

  // ---------------- per connection
  u8* carry;                // [c_max][carry_cap]
  u32* carry_len;           // [c_max]
  u32* conn_paused;
  u32* conn_frame_max;
  u32* conn_vhost;
  i64* conn_last_rx;
  u32* chmap;               // [c_max][chmap_size]: (ch<<16)|0x8000|local, 0 = empty
  u32* conn_ret_bytes;      // per step (reset by renderer)
  u32* conn_conf_bytes;
  u32* conn_dfirst;         // first sorted delivery of the connection (0xffffffff none)
  u32* conn_dlast;
  const u32* conn_wblock;   // host-mapped: egress back-pressure per connection (front end)
  u32* conn_total;
  u32* conn_base;

  // ---------------- per segment / work
  u32* seg_start;
  u32* seg_total;
  u32* seg_cmd_base;        // first command of each segment (INVALID: none / overflowed)
  u32* seg_npub;            // publishes of each segment: publishes get segment-ordered indices
  u32* seg_nack;            // acks / nacks / rejects of each segment (segment-ordered indices)
  u32 rank_scan;            // 1: publish / ack indices from a grid-wide rank scan (seg_max > DEC_SEG_LDS)
  u8* work;

  // ---------------- commands
  Cmd* cmds;
  Frag* frags;
  u32* cmd_is_pub;
  u32* cmd_is_ack;
  u32* cmd_pub_rank;
  u32* cmd_ack_rank;

  // ---------------- publishes
  Pub* pubs;
  i8* pub_keyvec;           // [pub_max][TOPIC_K]
  u16* pub_kwoff;           // [pub_max][TOPIC_WORDS] routing-key words: offset << 8 | length
  u16* pub_match;           // [pub_max][tb_pad/16]
  u32* pub_nq;
  u32* pub_qc;              // [pub_max][8] routed queues cached by route pass 0
  u32* pub_slot;
  u32* pub_routed;
  u32* pub_pair_off;
  u32* pub_slot_off;
  u32* pub_routed_rank;
  u32* pub_ret;             // 0 / 312 / 313
  u32* pub_ret_sz;          // rendered Basic.Return bytes of the publish (0 = none)
  u32* pub_ret_off;         // exclusive scan of pub_ret_sz (publish order)
  u32* conn_ret_min;        // per connection: smallest pub_ret_off (0xffffffff none)
  u32* ret_list;            // pub indices with returns
  Ack* acks;

  // ---------------- pairs (msg -> queue), radix-sorted by queue
  u32* pair_k[2];
  u32* pair_v[2];
  u32* q_first;             // [q_max] scratch (0xffffffff)

  // ---------------- exchanges / bindings (replicated, uploaded by host)
  u64* x_hkey;              // [xhash] exchange-name hash
  i32* x_hval;              // [xhash] exchange slot
  u32* x_type;
  u32* x_fan_off; u32* x_fan_n;
  u32* x_t_off; u32* x_t_n;
  u32* fan_q;               // fanout queue lists (sorted, unique)
  u64* d_key;               // [dhash] direct binding hash (keyhash ^ exch*K)
  i32* d_exch;              // [dhash] -1 empty
  u32* d_kb_off; u32* d_kb_len;
  u32* d_q_off; u32* d_q_n;
  u32* d_q;                 // direct queue lists
  u8* kpool;                // key/pattern bytes
  u32* t_queue; u32* t_exch; u32* t_kb_off; u32* t_kb_len; u32* t_flags; i32* t_expect;
  u32* t_count;             // [4] topic bindings in use ([0]; rows 0..n-1 of the tables above)
  i8* t_mat;                // [tb_pad][TOPIC_K]
  u16* t_woff;              // [tb_pad][TOPIC_WORDS] pattern words: offset << 8 | length

  // ---------------- queues
  u64* q_ring_off;          // offset into ring pool
  u64* q_ring_mask;
  u64* q_head;
  u64* q_tail;
  i64* q_ttl;
  u32* q_cons_off; u32* q_cons_n; u32* q_rr; u32* q_active;
  u32* q_cons;              // consumer ids per queue (CSR)
  Desc* ring;               // ring pool

  // ---------------- channels
  u32* ch_confirm;
  u32* ch_pub_cnt;
  u32* ch_pub_fail;         // a publish of this step was dropped (ring full / no memory): confirm with Nack
  u64* ch_confirm_next;
  u64* ch_next_tag;
  u64* ch_uhead;
  u64* ch_ack_upto;
  u64* ch_req_upto;
  u32* ch_mlo;        // this step's multiple settles of the channel: first / last ack index
  u32* ch_mhi;        // (INVALID / 0 when none; reset by k_chan_advance)
  u32* ch_prefetch;
  u32* ch_global;
  u32* ch_flow;
  u32* ch_tx;               // transactional channel (Tx.Select): data commands -> CK_TXBUF
  u32* ch_num;              // AMQP channel number of the slot
  u32* ch_unacked;          // outstanding manual-ack deliveries (global prefetch)
  u32* ch_win;              // window slots in use (reserved)
  u32* ch_dirty;
  u32* dirty_list;
  u32* n_dirty;
  u32* def_list;            // [nch] channels left dirty by k_chan_advance (record budget hit)
  const u32* unpause_req;   // per parity [UNPAUSE_STEP_MAX]: connections k_stage unpauses
  const GetReq* get_req;    // per parity [GET_STEP_MAX]: Basic.Get requests of the step
  GetOut* get_out_h;        // per parity, host-mapped [GET_STEP_MAX]: their answers
  USlot* uwin;              // [chslots][ucap]

  // ---------------- consumers
  u32* cons_q; u32* cons_ch; u32* cons_noack; u32* cons_active; u32* cons_unacked;
  u32* cons_tag_off; u32* cons_tag_len;
  u8* tpool;                // consumer-tag bytes

  // ---------------- messages
  MsgEnt* msgs;
  u32* msg_free;            // free index stack
  u32* msg_free_top;
  u8* log;
  u64* log_head;
  u64* log_tail;
  u64* log_step_base;
  i64* log_live;            // live bytes per log block
  i64* live_bytes;          // live slot bytes in the (HBM) log
  // cold bodies spilled to host memory (spill_bytes > 0): a ring of pinned host memory in
  // log_block blocks, read over PCIe when its messages are delivered (MsgEnt.log_off has
  // SPILL_BIT set and is a position in this ring)
  u8* spill;
  u64 spill_bytes, n_spill_blocks;
  u64* spill_head;
  u64* spill_tail;
  // egress by reference of spilled bodies: the ring's host address, and its tail over the
  // last SPILL_LAG steps -- space freed by a step is reused only SPILL_LAG steps later, after
  // the egress that may still reference it has been written out (spill_reserve)
  u64 spill_host;
  u64* spill_tail_lag;      // [SPILL_LAG]
  i64* spill_live;          // live bytes per spill block
  i64* cold_live;           // [COLD_SEGS] live bytes per cold-store segment (host unlinks freed ones)
  u64* q_cold_lim;          // [q_max] deliveries stop here (~0: nothing of the queue is cold)
  u64* q_spill_cur;         // [q_max] spill_queue resumes here: entries before it are tiered
  u64* q_cold_cur;          // [q_max] k_cold_pick resumes here: entries before it are cold
  u64* id_next;             // snowflake virtual sequence position

  // ---------------- deliveries
  Deliv* deliv;             // in final (channel-sorted) order
  u32* dv_size;             // by sorted position
  u32* dv_off;
  u32* ch_first;            // [chslots] scratch
  // delivery runs: k_dequeue emits one run per (queue, consumer) grant, k_runs orders
  // them by channel, k_dv_write expands them into Deliv records at their final positions
  Run* runs;                // [q_max * RUNS_PER_Q]
  u32* q_nruns;             // [q_max] runs of the queue this step
  u32* run_order;           // [q_max * RUNS_PER_Q] run slots in delivery order
  u32* run_start;           // first delivery index of each ordered run
  u64* run_key;             // global sort space when the runs exceed the LDS sort

  // ---------------- requeue
  ReqItem* req;
  u32* req_n;
  u32* req_q_n;             // per queue count

  // ---------------- scratch
  u32* scan_tmp;            // block sums
  u32* hist;                // radix histograms
  u32* hist_scan;
  u32* tot;                 // scan totals [64]
  u64* egress_budget;       // bytes reserved by dequeue this step (saturating, reserve_sat64)
  u64* dbg;                 // per-segment phase timestamps (s_memrealtime, 100 MHz)

  // ---------------- sharding (cross-rank publish exchange; world == 1: unused)
  u32 world, my_rank, rank_bits, pub_cap, import_max;
  u32 scan_inplace;         // k_frame_scan reads the step's new bytes from the ingress slot (cfg scan_in_place)
  u32 xfer_desc_max;        // records per step, all destinations
  u64 xfer_bytes;           // payload bytes per step, all destinations
  u32* q_owner;             // [q_max] owning rank
  u32* q_excl;              // [q_max] exclusive owner connection + 1 (0: not exclusive)
  DGet* dget;               // per parity [DGET_MAX]: Basic.Get commands of the step (tot[TS_NDGET])
  u32* conn_gempty;         // per connection: Basic.GetEmpty frames to render this step
  u32* conn_gempty_ch;      // per connection: their channel number
  u32* pub_rmask;           // [pub_cap] remote ranks owning >= 1 routed queue
  u32* xp_cnt;              // [world][pub_cap] record for rank r?
  u32* xp_cnt_off;
  u32* xp_byt;              // [world][pub_cap] payload bytes for rank r
  u32* xp_byt_off;
  u32* xs_base;             // [2*WORLD_MAX] send record / byte bases per destination
  u32* pk_agg;              // [pub tiles][2*WORLD_MAX] k_pack_scan tile aggregates -> prefixes
  u32* xr_base;             // [2*WORLD_MAX] recv record / byte bases per source
  u32* xchg;                // host-mapped [4*WORLD_MAX+4]: send counts/bytes (out), recv counts/bytes (in), overflow
  RDesc* send_desc;         // caller-provided (torch tensors: RCCL all-to-all operands)
  u8* send_pay;
  const RDesc* recv_desc;
  const u8* recv_pay;
  u64* id_base;             // snowflake position base of the current routing phase

  // ---------------- persistence (persist == 0: unused)
  u32 persist, persist_max;
  u64 persist_bytes;
  u32* q_durable;           // [q_max]
  PersistRec* prec;         // [persist_max]
  ConsumedRec* crec;        // [persist_max]
  u32* ps_size;             // [persist_max]
  u32* ps_off;
  // host-mapped store records of a step, in PSLOTS slots rotating per step (StepIn.pslot):
  // a step's records stay valid for PSLOTS - 1 further steps, so the front end can hand
  // them to the store without copying them on its stepper thread
  u8* ps_persist[PSLOTS];      // [persist_bytes]
  ConsumedRec* ps_crec[PSLOTS];  // [persist_max]
  u8* persist_h;            // host-mapped [persist_bytes]
  ConsumedRec* crec_h;      // host-mapped [persist_max]

  // ---------------- remote-consumer links (X2/X3; links == 0: unused).  Owner side: a
  // link pseudo-connection's deliveries are not rendered as frames but shipped as restore
  // records (RDesc, MF_RESTORE into the shadow queue, xid = epoch << 40 | tag) in the
  // next exchange; connection side: consumption of a shadow message sends an AckRec back
  // to the owner, whose phase B marks the tag acked in the pseudo channel's window
  u32 links;
  u64 import_bytes;         // receive payload capacity (publishes + link deliveries)
  u32* conn_link;           // [c_max] dest rank + 1 of a link pseudo-connection (0: a client)
  u32* conn_link_tq;        // [c_max] its shadow queue slot (replicated: same slot on every rank)
  u32* conn_link_epoch;     // [c_max]
  u32* link_conns;          // [64] link pseudo-connections of this rank
  u32* n_link_conns;        // [1]
  u32* link_nbase;          // [c_max] first record of the connection's deliveries in lsend_desc
  u32* link_bbase;          // [c_max] payload offset of its deliveries in its destination region
  u32* link_dbase;          // [WORLD_MAX] payload region base of each destination in lsend_pay
  u32* q_link_owner;        // [q_max] connection side: owner rank + 1 of a shadow queue
  u32* q_link_ch;           // [q_max] owner side: pseudo channel slot of the link of shadow q
  u32* q_link_epoch;        // [q_max] owner side: its epoch
  RDesc* lsend_desc;        // [deliv_max] this parity's link records (destination-major)
  u8* lsend_pay;            // [egress_cap]
  AckRec* lk_send;          // [WORLD_MAX][lk_cap] acks per owner rank
  u32 lk_cap;
  u32* lk_cnt;              // [WORLD_MAX] acks packed this step
  const AckRec* rack;       // acks received for this step (contiguous, all sources)
};

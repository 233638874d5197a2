// Native pipelined front end of the GPU broker: sockets -> data-plane steps -> sockets
// with no Python on the per-step path.
//
//   * N IO threads, each with its own edge-triggered epoll set of connections (thread 0
//     also owns the listener).  Per step they gather, in parallel, every readable data
//     connection straight from its socket into one pinned ingress arena (FIONREAD-sized
//     reservations from a shared atomic cursor: one dense buffer, one H2D copy), and
//     scatter the previous step's rendered egress from the host egress slot to the
//     sockets (zero-copy unless a socket is full).
//   * One stepper thread runs the same software pipeline as bench.py: two steps in
//     flight on the GPU (H2D(t+1) || kernels(t) || D2H(t-1)), the IO phase of step t+1
//     overlapping the kernels of step t.  It drives the HIP engine through the C table of
//     step_abi.h (CmqEngineApi), converts step outputs (control commands, tx-held
//     commands, status errors, persistence records) into events for the control plane.
//   * The control plane (Python, server/gpu_broker.py) blocks in poll_events(); before it
//     touches device tables it calls pause(): the stepper finishes the steps in flight,
//     writes their egress and parks, so control replies are ordered after every earlier
//     delivery of the connection.
//   * Persistence write-behind: a step that produced store records is "held": its egress
//     (with the publisher confirms) waits until the control plane has committed the
//     records and calls release(); steps keep running meanwhile.
//
// Per-connection byte budget: at most carry_cap - device_carry - bytes_in_flight is
// gathered for a connection, so a paused connection's backlog never overflows the
// device carry (TCP back-pressure does the rest).
//
// Reference counterpart: the per-connection Akka stream of the reference (Amqp.scala:74-111
// bind, ServerBluePrint.scala:27-43 tick-driven FrameStage), here batched over all
// connections per step.
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../kernels/step_abi.h"

namespace cmqx { class ShmXchg; }

namespace cmq {

enum FeEventKind : int {
  FE_OPEN = 1,      // conn accepted (host mode: its bytes go to the control plane)
  FE_CLOSED = 2,    // peer closed / socket error / heartbeat timeout; call close() to free the slot
  FE_HOST = 3,      // host-mode bytes available: take()
  FE_CTRL = 4,      // control command (raw frames); the device paused the connection
  FE_TXBUF = 5,     // data command of a transactional channel: a = wire position
  FE_EVENT = 6,     // device event: a = code (404 unknown exchange, 506 control overflow), b = channel slot
  FE_STATUS = 7,    // segment error status (SS_FRAME_ERROR / SS_UNEXPECTED / SS_TOO_LARGE): a = status
  FE_PERSIST = 8,   // store records of step a (data = packed PersistHdr records, data2 = ConsumedRec[]);
                    // that step's egress is held until release(a)
  FE_ERROR = 9,     // engine failure (data = message); the stepper stopped
  FE_GROW = 10,     // queues past half their ring (data = u32 slots): the control plane grows them
  // sharded broker (world > 1, native exchange): every rank's stepper parks at the same
  // step and posts one of these; the control plane runs the replicated control-log sync
  // (FE_SYNC) or the failover (FE_XFAIL: an exchange peer did not answer, nothing of that
  // exchange was imported) and then calls sync_done()
  FE_SYNC = 11,
  FE_XFAIL = 12,
  FE_INJECTED = 13,   // the bytes inject()ed into a pseudo-connection were stepped (a = its carry)
  FE_GET = 14,        // a queue_get() was answered by its step: a = status | message_count << 32, b = id
};

enum : u32 { XF_SYNC = 1, XF_BUSY = 2 };   // exchange flags (OR over the live ranks)

struct FeEvent {
  int kind = 0;
  u32 conn = 0;
  u64 a = 0, b = 0;
  std::string data, data2;
};

struct FrontendCfg {
  std::string host = "127.0.0.1";
  int port = 0;
  int io_threads = 4;
  u64 per_conn_read = 256 << 10;   // max bytes gathered per connection per step
  double idle_step_ms = 2.0;       // step period with open data connections and no traffic
  double sweep_ms = 200.0;         // no connections: TTL sweep period while messages are held
  u32 worker = 0;                  // snowflake worker id
  u32 max_slot = 0;                // connection slots 1..max_slot (default c_max - 2)
  bool reuseport = false;
  int sndbuf = 4 << 20, rcvbuf = 4 << 20;
  u64 wblock_high = 8 << 20, wblock_low = 2 << 20;   // egress back-pressure watermarks per connection
  // gather phases of the (unsharded) stepper: each IO thread releases the stepper once its
  // connections are gathered and writes the finished step's egress after that, while the
  // step is submitted (the sockets' send path no longer sits on the step's critical path)
  bool async_scatter = true;
  // egress by reference (step_abi.h set_egress_ref): a delivery of a body that arrived in
  // the same step is rendered without it and sent from the ingress arena with sendmsg
  // iovecs -- the body crosses PCIe once.  Needs NARENA arenas (an arena is gathered into
  // again only after every egress that may reference it is written)
  bool egress_ref = true;
  u32 egress_ref_min = 256;
  // ... only for steps that gathered at least this many bytes: over TCP the iovec walk costs
  // the IO threads more than a small step's D2H costs the PCIe link (gpu_server_e2e config 2:
  // 2.4 MB steps, 3.5 % fewer msgs/s and a 2.4 vs 0.9 ms p99 with references)
  u64 egress_ref_step_min = 8ull << 20;
};

struct FeStats {
  u64 steps = 0, published = 0, delivered = 0, rx_bytes = 0, tx_bytes = 0, egress_bytes = 0;
  u64 spill_moved = 0;   // body bytes moved to the host spill ring by steps (StepIn.spill_*)
  u64 held_steps = 0, idle_steps = 0, gather_segs = 0;
  u64 store_fail_nacks = 0;   // publisher confirms turned into Basic.Nack: their store commit failed
  u64 dropped_nomem = 0, ring_full = 0, unroutable = 0, routed = 0, expired = 0, ctrl = 0;
  i64 live_bytes = 0;
  u64 live_msgs = 0;
  u64 log_used = 0;          // body-log occupancy (head - tail): the oldest live message pins it
  u64 lat_hist[32] = {};
  double io_phase_s = 0, wait_s = 0, submit_s = 0;
  double xchg_s = 0;          // sharded: host time in the per-step exchange
  u64 xchg_steps = 0, syncs = 0, xfails = 0, flush_steps = 0;
  // per-stage latency histograms (bin k: [2^k, 2^(k+1)) µs) -- where a TCP message's time
  // goes: the stepper's period between submits, its IO phase (write the older step's
  // egress, gather the next one), the submit call, and its wait for a step's results
  u64 h_period[32] = {}, h_io[32] = {}, h_submit[32] = {}, h_wait[32] = {};
  double max_period_s = 0, max_io_s = 0, max_wait_s = 0;
};

struct FeConn;
struct FeIo;
class PersistWorker;

class Frontend {
 public:
  Frontend(const FrontendCfg& cfg, const CmqEngineApi* api);
  ~Frontend();
  int port() const { return port_; }
  void start();
  void stop();

  // ---- control-plane API (thread-safe; the bindings release the GIL)
  std::vector<FeEvent> poll_events(int timeout_ms);
  std::string take(u32 conn);                           // host-mode bytes received so far
  void ref_for_step(u64 used);
  void kick_unpaused(int p);
  void send(u32 conn, const char* data, size_t n);      // append to the connection's output
  void send_egress(const u8* egress, const ConnOut* co, u32 n_slots);   // a host-run step's egress
  void set_data_mode(u32 conn, const std::string& leftover);   // bytes now go to the GPU
  void set_host_mode(u32 conn);                          // bytes go to the control plane again
  void set_heartbeat(u32 conn, u32 seconds);
  void set_read_cap(u32 conn, u64 bytes);                // per-step read budget (0: per_conn_read)
  // flush, close the socket, free the slot; gen >= 0: only if the slot's generation is
  // still gen (an FE_CLOSED event's a: the slot may have been freed and reused since)
  void close(u32 conn, i64 gen = -1);
  void kick(u32 conn);                                   // unpaused: re-present its device carry
  // control reply of a command handled while steps keep running (no pause): written after
  // the egress of every step submitted so far, so a Basic.CancelOk / Channel.CloseOk never
  // overtakes a delivery rendered before it.  Any thread.
  void send_after(u32 conn, const char* data, size_t n);
  void wake();                                           // the stepper looks for work (staged control writes)
  void flush_ctl();                                      // (paused) write every held control reply now
  // (held control replies, the first one's step, steps submitted, steps finished)
  std::vector<u64> ctl_state();
  // bytes for a socketless pseudo-connection (committed transactions): stepped with the
  // next step like a client's, FE_INJECTED once that step finished; egress is dropped
  void inject(u32 conn, const std::string& bytes);
  // Basic.Get served inside the next step (k_dequeue): FE_GET answers it once the step
  // finished (GetOk rendered into the connection's egress of that step)
  void queue_get(u32 conn, u32 chslot, u32 q, u32 noack, u64 id);
  void cancel_gets(u32 conn);                            // the connection is gone: drop its requests
  void pause();                                          // exclusive device access (nests)
  void resume();
  void release(u64 step);                                // store commit of steps <= step landed
  // native write-behind: step records go to the worker (not to the control plane) and
  // its group commits release the held egress
  void attach_persist(PersistWorker* w);
  FeStats stats();
  u64 pending_out() const;
  // ---- sharded broker
  void request_sync();                                   // replicated ops are waiting: sync at the next step
  void sync_done();                                      // FE_SYNC / FE_XFAIL handled: steps resume
  // per-step liveness for the failure detector: false once the engine failed or a GPU
  // wait (step results, egress) has been stuck longer than `stuck_s`
  bool healthy(double stuck_s) const;
  // per connection: post FE_INJECTED when its segment was stepped (inject() on the control
  // thread sets it, the stepper clears it)
  std::unique_ptr<std::atomic<u8>[]> notify_;
  // fault injection (tests): after `steps` more steps, kind 1 = engine error, 2 = process
  // exit, 3 = wedge (the stepper blocks inside a GPU wait forever)
  void inject_fault(int kind, u64 steps);

 private:
  friend struct FeIo;
  struct Inflight {
    int p;
    u64 step;
    std::vector<std::pair<u32, u32>> segs;
    std::vector<u32> gen;
    std::vector<std::pair<u32, u64>> gets;   // (conn, id) of the Basic.Gets it serves
    u64 batch_hi = 0;   // staged control-write batches taken by this step and earlier (dl_state 1)
  };
  struct PendGet { GetReq r; u64 id; };
  std::mutex get_mu_;
  std::vector<PendGet> gets_;   // queue_get() requests not yet submitted
  void stage_gets(Inflight& f);   // up to GET_STEP_MAX of them into the step about to be submitted
  bool gets_pending();
  struct Scatter {   // one step's rendered egress, ready to write
    const u8* egress = nullptr;
    std::vector<ConnOut> co;
    std::string own;         // held copy (persistence) or host-run step
    // connection generations when the step was submitted: bytes of a connection that
    // closed since (its slot possibly reused by a new client) are dropped, never written
    std::vector<u32> gen;
    int wait_slot = -1;      // egress slot whose D2H the writer waits for first (-1: ready)
    // egress by reference: gath_n EgressRef entries at gath_off of the egress bytes (0: the
    // bytes are the wire bytes)
    u32 gath_n = 0, gath_off = 0;
  };
  // needs_commit: the step's store records must commit before the confirm-gated part of
  // its egress leaves; conf = that step's confirm bytes per connection (empty = all gated)
  struct Held { u64 step; bool needs_commit; Scatter sc; std::vector<u32> conf; u64 batch_hi = 0; };

  void stepper();
  void stepper_sharded();
  void park_sync(int kind, u64 step);
  void drain(std::deque<Inflight>& inflight);
  bool fault_due();
  void io_loop(int i);
  void io_phase(std::vector<Scatter*>& scat, bool gather, bool async = false);
  void finish_oldest(std::deque<Inflight>& inflight);
  bool collect_scatter(std::vector<Scatter*>& scat);
  bool stash_pend(bool copy);
  void flush_pending(bool final);
  bool releasable() const;
  bool any_data_conn() const;
  void post(FeEvent&& e);
  void wake_stepper();
  void accept_all(FeIo& io);
  void drop(FeConn& c, bool notify);
  bool write_some(FeConn& c);   // mu held
  void wblock_update(FeConn& c);   // mu held
  void scatter_conn(FeConn& c, const u8* data, u32 n);
  // one connection's part of a step's egress, its referenced bodies spliced in (sendmsg)
  void scatter_ref(FeConn& c, const u8* base, const ConnOut& o, const Scatter& sc);
  // the scatter's wire bytes into sc.own (its egress slot / arena may be reused before it
  // is written): bodies spliced in, offsets rewritten
  static void materialize(Scatter& sc, const u8* egress, u64 bytes);
  // the store failed: every publisher confirm (Basic.Ack) in a held step's egress becomes a
  // Basic.Nack -- same frame size, method 80 -> 120, requeue 0 -- so no publish whose rows
  // never reached the disk is acknowledged; returns the frames changed
  static u64 nack_confirms(Scatter& sc);
  void gather_conn(FeIo& io, FeConn& c, u8* arena, u64 cap);
  bool check(int rc);

  FrontendCfg cfg_;
  const CmqEngineApi* api_;
  int lfd_ = -1, port_ = 0;
  u32 c_max_ = 0;
  std::vector<std::unique_ptr<FeConn>> conns_;
  std::vector<std::unique_ptr<FeIo>> io_;
  std::mutex free_mu_;
  std::vector<u32> free_;
  std::thread stepper_;
  std::atomic<bool> running_{false};

  // pinned ingress arenas, gathered into in turn.  3 suffice for the H2D (step t's copy is
  // done before step t+3 gathers); egress by reference needs 4: step t's egress is written
  // by the IO threads after their gather of step t+2 and may still be in progress while
  // step t+3 gathers, and it may reference step t's arena.  One more for margin
  static constexpr int NARENA = 5;
  u8* arena_[NARENA] = {};
  bool arena_pinned_[NARENA] = {};
  int narena_ = 3;
  bool ref_on_ = false;   // egress by reference set on the engine (ref_for_step)
  int arena_i_ = 0;

  // IO phase
  std::mutex ph_mu_;
  std::condition_variable ph_cv_;
  std::atomic<u64> ph_id_{0};
  std::atomic<int> ph_left_{0};
  std::vector<Scatter*>* ph_scat_ = nullptr;
  bool ph_gather_ = false, ph_async_ = false;
  u8* ph_arena_ = nullptr;
  u64 ph_cap_ = 0;
  std::atomic<u64> ph_used_{0};
  u64 ph_step_ = 0;   // step number of the gather phase in progress
  std::atomic<u32> ph_nseg_{0};
  std::atomic<u64> ph_carry_{0};

  // stepper wake-up / pause
  std::mutex st_mu_;
  std::condition_variable st_cv_, pause_cv_;
  bool wake_ = false;
  int pause_req_ = 0;
  bool paused_ = false;

  // events to the control plane
  std::mutex ev_mu_;
  std::condition_variable ev_cv_;
  std::deque<FeEvent> events_;

  // finished step whose egress D2H is in flight
  Held pend_;
  bool pend_valid_ = false;
  int pend_slot_ = 0;
  u64 pend_bytes_ = 0;
  bool last_busy_ = false, idle_tick_ = false;
  std::deque<Scatter> out_;   // egress being written in the current IO phase
  // egress of the last async-scatter phase: IO threads may still be writing it until every
  // one of them has passed the next phase (io_phase frees it then)
  std::deque<Scatter> out_prev_;
  std::atomic<bool> stepper_done_{false};

  // persistence write-behind
  std::deque<Held> held_;
  std::vector<u32> held_cnt_;   // per connection: held entries carrying its bytes (keeps its order)
  u64 held_total_ = 0;
  PersistWorker* persist_ = nullptr;
  // store records handed to the write-behind off the stepper thread: the engine keeps a
  // step's records for PSLOTS - 1 further steps (rotating slots), a copier thread moves
  // them into the worker's batches meanwhile; the stepper only waits when it falls behind
  struct PCopy { u64 step; const u8* persist; size_t plen; const u8* consumed; size_t clen; };
  void copier();
  void post_copy(const PCopy& c);
  void wait_copies(size_t max_pending);
  std::thread pc_th_;
  std::mutex pc_mu_;
  std::condition_variable pc_cv_, pc_done_cv_;
  std::deque<PCopy> pc_q_;
  size_t pc_active_ = 0;
  bool pc_stop_ = false;
  std::atomic<u64> released_{0};
  bool have_released_ = false;

  std::mutex stats_mu_;
  FeStats stats_;
  std::atomic<u64> rx_bytes_{0}, tx_bytes_{0};
  u64 step_no_ = 0;
  // steps submitted / finished so far (control replies and freed connection slots wait
  // for the steps that were in flight when they were produced)
  std::atomic<u64> sub_step_{0}, fin_step_{0};
  // after: released behind the egress of step `after`; batch (light sections, 0: none):
  // and not before the egress of the step that applied that staged-write batch, and never
  // after the egress of any later step (stash_pend releases first)
  struct CtlOut { u64 after; u32 conn; u32 gen; std::string data; u64 batch = 0; };
  std::mutex ctl_mu_;
  std::deque<CtlOut> ctl_out_;
  bool ctl_pending();
  bool ctl_needs_step();
  void release_ctl();
  // step / write batch of the last egress queued for writing (out_ or held_): a reply is
  // released only once the egress of the step it waits for was queued, and before the next
  u64 out_step_ = 0, out_batch_ = 0;
  // closed connection slots: reusable once the steps in flight at their close finished
  std::deque<std::pair<u64, u32>> quarantine_;   // (sub_step_ at close, slot), free_mu_
  i64 last_submit_ = 0;   // (stats: the stepper's period between submits)
  std::atomic<bool> failed_{false};   // read by healthy() (heartbeat thread)

  // sharded broker
  std::atomic<bool> sync_req_{false};
  bool sync_go_ = false;          // st_mu_
  int xpend_ = -1;                // parity of the launched step whose exchange is due
  bool cluster_busy_ = false;
  std::atomic<i64> gpu_wait_since_{0};
  int fault_kind_ = 0;
  u64 fault_at_ = 0;
};

// CPU stand-in for the HIP engine (tests without a GPU): every segment's bytes come back
// to the same connection as egress one step later; a segment containing "CTRL" is
// reported as a control command and pauses the connection like the device does.
// Sharded mode (world > 1, xchg_setup): the bytes after "XR<d>" in a segment are shipped
// to rank d through the real shared-memory exchange (xchg_host.h) and come out there as
// egress of the same connection slot when that rank's phase B imports them -- the
// front end's lockstep stepper, sync points and failover run exactly as with the GPU.
class EchoEngine {
 public:
  EchoEngine(u32 c_max, u32 seg_max, u64 ingress_cap, u32 carry_cap, u32 world = 1, u32 rank = 0);
  ~EchoEngine();
  u64 c_api() { return (u64)&api_; }
  void unpause(u32 conn);
  // async: the Engine's asynchronous exchange, emulated -- exchange() hands the step's
  // records to an exchange thread and returns the previous exchange's result; phase B runs
  // once its exchange finished (on that thread when launch_b came first); wait_results
  // waits for it
  void xchg_setup(const std::string& name, const std::vector<int>& members, int timeout_ms, bool async = false);
  u64 steps = 0, imported = 0;

 private:
  struct Io {
    Counters ctr{};
    std::vector<SegOut> so;
    std::vector<ConnOut> co;
    std::vector<CtrlRec> cr;
    std::string ctrl;
    std::string egress;
    std::vector<std::pair<u32, std::string>> fwd[16];   // phase A: records per destination rank
    bool ready = false;                                  // phase A done, exchange due
  };
  int exchange(int q, u32 flags, u32* orf);
  int exchange_blocks(std::vector<std::string>& blocks, u32 flags, u32* orf,
                      std::vector<std::pair<u32, std::string>>* imports);
  std::vector<std::string> pack_fwd(int q);
  void launch_b(int p);
  void run_b(int p, std::vector<std::pair<u32, std::string>>& imports);
  int collect(u32* orf);
  void x_loop();
  void x_stop();
  bool async_ = false;
  std::thread xth_;
  std::mutex xmu_;
  std::condition_variable xcv_;
  bool xstop_ = false, xjob_ = false, xbusy_ = false, xres_ = false;
  int xres_rc_ = 0, xdst_ = -1;
  u32 xflags_ = 0, xres_orf_ = 0;
  std::vector<std::string> xblocks_;
  std::vector<std::pair<u32, std::string>> ximports_;   // the finished job's records
  bool b_wait_[2] = {false, false};                     // phase B of parity p waits for the job
  bool b_due_[2] = {false, false};                      // ... and was launched (runs after it)
  std::unique_ptr<cmqx::ShmXchg> shm_;
  std::vector<int> members_;
  std::vector<std::pair<u32, std::string>> imports_;
  u32 world_ = 1, rank_ = 0;
  u64 xseq_ = 0;
  CmqEngineApi api_{};
  Io io_[2];
  std::string slot_[3];
  int slot_of_[2] = {0, 0};
  std::vector<u8> paused_;
  std::vector<u32> wblock_;
  u64 seq_ = 0;
  std::string err_;
};

}  // namespace cmq

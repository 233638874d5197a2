// Native host runtime for the MI355X data plane: owns every device/host-mapped
// buffer, launches the step pipeline on a caller-supplied HIP stream and captures
// it once into a hipGraph (steady-state deliver loop = one hipGraphLaunch).
//
// Python sees a pybind11 module `_dataplane` with class Engine (chanamq_amd/ops).
#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include <chrono>
#include <algorithm>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <condition_variable>
#include <thread>
#include <stdexcept>
#include <string>
#include <vector>

#include <hsa/amd_hsa_signal.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include "dataplane.hip"
#include "xchg_host.h"
#include "xchg_rccl.h"

namespace py = pybind11;

#define HIPCHECK(x)                                                                  \
  do {                                                                               \
    hipError_t _e = (x);                                                             \
    if (_e != hipSuccess)                                                            \
      throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(_e));      \
  } while (0)

static u32 ceil_div(u64 a, u64 b) { return (u32)((a + b - 1) / b); }
static u32 next_pow2(u32 x) { u32 p = 1; while (p < x) p <<= 1; return p; }
static u32 bits_for(u64 maxval) { u32 b = 0; while ((1ull << b) <= maxval) ++b; return b; }

// host-side time accounting of the step loop (seconds, per named phase)
struct HostTimer {
  double* acc;
  std::chrono::steady_clock::time_point t0;
  explicit HostTimer(double* a) : acc(a), t0(std::chrono::steady_clock::now()) {}
  ~HostTimer() { *acc += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); }
};

// roctx range over a host scope (rocprofv3 --marker-trace): step phases, copies, Get
struct Range {
  explicit Range(const char* name) { roctxRangePushA(name); }
  ~Range() { roctxRangePop(); }
};

struct Buf {
  void* ptr = nullptr;
  size_t bytes = 0;
  bool host = false;
  bool view = false;   // a named range of another allocation (not freed on its own)
};

// per-step IO sets ("parities"): step t uses set t % npar_.  Two (double buffering) by
// default; three for a single-GPU engine without the overlapped ingest (cfg "parities"): the
// host then submits step t+1 once step t-2 -- not t-1 -- is collected, so the next step's
// ingress H2D never waits for the host to notice the previous step's kernels ending
static constexpr int NPAR_MAX = 3;

class Engine {
 public:
  explicit Engine(py::dict cfg) {
    auto get = [&](const char* k, u64 dflt) -> u64 {
      return cfg.contains(k) ? cfg[k].cast<u64>() : dflt;
    };
    device_ = (int)get("device", 0);
    HIPCHECK(hipSetDevice(device_));
    {
      int ncu = 0;
      if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device_) == hipSuccess && ncu > 0)
        n_cu_ = (u32)ncu;
    }
    d_ = DS{};
    d_.c_max = (u32)get("c_max", 1024);
    d_.chpc = next_pow2((u32)get("chpc", 16));
    d_.q_max = (u32)get("q_max", 4096);
    d_.x_max = (u32)get("x_max", 1024);
    d_.cons_max = (u32)get("cons_max", 16384);
    d_.seg_max = (u32)get("seg_max", 1024);
    d_.carry_cap = (u32)get("carry_cap", 1u << 20);
    d_.cmd_max = (u32)get("cmd_max", 65536);
    d_.frag_max = (u32)get("frag_max", d_.cmd_max * 2);
    d_.pub_max = d_.cmd_max;
    d_.ack_max = d_.cmd_max;
    // sharded queues (world > 1): records imported from other ranks per step
    d_.world = (u32)get("world", 1);
    d_.my_rank = (u32)get("rank", 0);
    if (d_.world < 1 || d_.world > WORLD_MAX || d_.my_rank >= d_.world)
      throw std::runtime_error("world must be 1..16 and rank < world");
    // Each publish is shipped at most once per other rank and its record payload never
    // exceeds its wire bytes, so these defaults cannot overflow (records / bytes per step).
    d_.import_max = d_.world > 1 ? (u32)get("import_max", (d_.world - 1) * d_.pub_max) : 0;
    // exchange_lag = 1: step t's phase B imports the records of step t-1's all-to-all, so
    // phases A and B launch back to back and the collective overlaps the next step's
    // kernels (cross-GPU publishes are delivered one step later)
    lag_ = d_.world > 1 && get("exchange_lag", 0) != 0;
    d_.pub_cap = ((d_.pub_max + d_.import_max + 63) / 64) * 64;
    d_.xfer_desc_max = d_.world > 1 ? (u32)get("xfer_desc_max", (d_.world - 1) * d_.pub_max) : 0;
    // persistence + recovery: restore batches reuse the import path (world == 1: own buffers)
    d_.persist = (u32)get("persist", 0);
    d_.persist_max = d_.persist ? (u32)get("persist_max", d_.cmd_max) : 0;
    d_.persist_bytes = d_.persist ? get("persist_bytes", 64ull << 20) : 0;
    // restore / host-publish records at world 1: recovery batches (persist) and messages
    // larger than a connection's carry, assembled by the host (MF_HOSTPUB)
    restore_max_ = (u32)get("restore_max", d_.persist ? (1u << 14) : 64);
    if (d_.world == 1 && restore_max_) {
      d_.import_max = restore_max_;
      d_.pub_cap = ((d_.pub_max + d_.import_max + 63) / 64) * 64;
    }
    d_.pair_max = (u32)get("pair_max", d_.cmd_max * 4);
    d_.deliv_max = (u32)get("deliv_max", 65536);
    if (d_.persist) {
      // a step's consumed-store records: deliveries (<= deliv_max), the durable TTL skip
      // (<= persist_max / 4) and k_chan_advance's settles, budgeted to what is left and
      // carried to the next step past it -- so the record buffer can never overflow
      const u64 need = 2ull * d_.deliv_max + 4096;
      if (d_.persist_max < need) d_.persist_max = (u32)std::min<u64>(need, 1u << 30);
    }
    // remote-consumer links (X2/X3) on the native exchange: a peer's link deliveries (at
    // most its deliv_max per step) arrive with its publishes and are imported with them
    links_ = d_.world > 1 && get("native_xchg", 0) != 0 && get("links", 0) != 0;
    if (links_) {
      d_.import_max += (d_.world - 1) * d_.deliv_max;
      d_.pub_cap = ((d_.pub_max + d_.import_max + 63) / 64) * 64;
    }
    d_.msg_max = (u32)get("msg_max", 1u << 22);
    u32 ucap = next_pow2((u32)get("ucap", 8192));
    d_.ucap_mask = ucap - 1;
    d_.deliver_cap = (u32)get("deliver_cap", 4096);
    dcap_bytes_ = (u32)get("deliver_cap_bytes", 0);
    d_.chmap_size = next_pow2(d_.chpc * 2);
    u32 xhash = next_pow2(d_.x_max * 2);
    d_.xhash_mask = xhash - 1;
    u32 dhash = next_pow2((u32)get("dhash", 65536));
    d_.dhash_mask = dhash - 1;
    d_.tb_max = (u32)get("tb_max", 4096);
    d_.tb_pad = ((d_.tb_max + 15) / 16) * 16;
    d_.req_max = (u32)get("req_max", 65536);
    d_.hash_wildcard = (u32)get("hash_wildcard", 1);
    d_.frame_max_global = (u32)get("frame_max", 131072);
    d_.log_bytes = get("log_bytes", 1ull << 32);
    d_.log_block = get("log_block", 4ull << 20);
    d_.log_bytes = (d_.log_bytes / d_.log_block) * d_.log_block;
    d_.n_log_blocks = d_.log_bytes / d_.log_block;
    d_.ingress_cap = get("ingress_cap", 64ull << 20);
    d_.xfer_bytes = d_.world > 1 ? get("xfer_bytes", (d_.world - 1) * (d_.ingress_cap + 64))
                                 : (restore_max_ ? get("restore_bytes", 80ull << 20) : 0);
    // work buffer = this step's new bytes + the carries of the connections in the step.
    // carry_cap bounds one connection's (= the largest command assembled on the device,
    // e.g. a multi-MB message); carry_budget bounds their sum per step (the front end
    // gathers within it), so large carries do not multiply by seg_max
    carry_budget_ = std::min<u64>((u64)d_.seg_max * (d_.carry_cap + 64), get("carry_budget", 512ull << 20));
    d_.work_cap = d_.ingress_cap + carry_budget_;
    d_.work_cap = d_.work_cap > (3ull << 30) ? (3ull << 30) : d_.work_cap;  // u32 offsets
    if (d_.work_cap + d_.xfer_bytes + 8192 > (4ull << 30))
      throw std::runtime_error("work buffer + imported bytes must stay below 4 GiB (u32 offsets): lower ingress_cap");
    d_.egress_cap = get("egress_cap", 96ull << 20);
    // receive payload: the peers' publishes + (links) their link deliveries, each bounded
    // by the sender's egress budget
    d_.import_bytes = d_.xfer_bytes + (links_ ? (u64)(d_.world - 1) * d_.egress_cap : 0);
    if (d_.persist) {
      // a step's persist records: one 48-B header per enqueue (<= pair_max) and each
      // message's bytes once (<= the step's work buffer + what it imported), so the
      // packed buffer can never overflow (no fail-closed stop on a burst)
      const u64 need = d_.work_cap + d_.xfer_bytes + 56ull * d_.pair_max + 4096;
      if (d_.persist_bytes < need) d_.persist_bytes = need;
      if (d_.persist_max < d_.pair_max) d_.persist_max = d_.pair_max;
    }
    if (d_.import_bytes + 8192 > (4ull << 30))
      throw std::runtime_error("import buffer must stay below 4 GiB (u32 offsets): lower ingress_cap / egress_cap");
    d_.ctrl_cap = get("ctrl_cap", 4ull << 20);
    d_.ring_pool = get("ring_pool", 1ull << 26);
    u32 fan_max = (u32)get("fan_max", 1u << 20);
    u32 dq_max = (u32)get("dq_max", 1u << 20);
    u64 kpool = get("kpool", 16ull << 20);
    u32 nch = d_.c_max * d_.chpc;
    // pair key = queue << 1 | (source rank >= this rank) at world > 1: the pairs are
    // generated as (this rank's publishes, then imports in source-rank order) and the sort
    // is stable, so one key bit restores (source rank, connection, publish) order per queue
    // (imports from lower ranks, own publishes, higher ranks) -- 9 key bits at q_max 256
    // instead of q_bits + log2(world)
    d_.rank_bits = d_.world > 1 ? 1 : 0;
    d_.q_bits = bits_for(d_.q_max);
    if (d_.q_bits + d_.rank_bits > 32) throw std::runtime_error("q_max too large for sharded pair keys");
    d_.ch_bits = bits_for(nch);
    graph_enabled_ = get("graph", 1) != 0;
    // step IO copies.  copy_engine: 0 = runtime default (a blit kernel that spreads over
    // the whole GPU and, for the egress D2H, holds its CUs for the entire PCIe transfer,
    // stalling the next step's kernels), 1 = hipMemcpyDeviceToDeviceNoCU request,
    // 2 = our own egress copy kernel on copy_wgs workgroups only (stores straight into
    // mapped pinned memory), leaving the rest of the CUs to the step kernels
    // 3 = the egress D2H on an SDMA engine through HSA directly (no CUs involved)
    copy_mode_ = (int)get("copy_engine", 0);   // measured: blit 24.0 M msgs/s, kernel(16 WG) 19.1 M
    sdma_ = copy_mode_ == 1;
    copy_wgs_ = (u32)get("copy_wgs", 16);
    sdma_pref_ = cfg.contains("sdma_engine") ? cfg["sdma_engine"].cast<int>() : -1;
    // (measured: no step-period gain in bench.py, 45.9 / 46.4 vs 45.9 / 46.3 M msgs/s,
    // profiles/r6_sp/ -- the egress D2H shares the link; opt-in)
    h2d_split_cfg_ = get("h2d_split", 0) != 0;
    h2d_split_min_ = get("h2d_split_min", 4u << 20);   // (tests lower it: every payload splits)
    wait_ms_ = (u32)get("wait_timeout_ms", 10000);
    sdma_split_ = cfg.contains("sdma_split") ? std::max(1, std::min(2, cfg["sdma_split"].cast<int>())) : 1;

    // ---- allocations
    auto dev = [&](const char* name, size_t bytes) { return alloc(name, bytes, false); };
    auto hst = [&](const char* name, size_t bytes) { return alloc(name, bytes, true); };
    d_.ctr = (Counters*)dev("ctr", sizeof(Counters));
    // (+ the gather table of egress by reference: one EgressRef per delivery)
    egress_alloc_ = d_.egress_cap + d_.work_cap + (u64)nch * 21 + 4096 + 16ull * d_.deliv_max;
    // the two parities' work buffers and the ingress slots in one allocation, the slots
    // last: a u32 offset from either work buffer reaches them, so a segment without a
    // carry is scanned and read where its H2D put it (k_frame_scan in place: no work copy)
    {
      const u64 wb = (d_.work_cap + 4096 + 255) & ~255ull, ib = (d_.ingress_cap + 64 + 255) & ~255ull;
      u8* base = (u8*)dev("work_all", 2 * wb + INGRESS_SLOTS * ib);
      d_.work = (u8*)view("work", base, d_.work_cap + 4096);   // imports are read in place (k_import_route)
      work_p1_ = (u8*)view("work_p1", base + wb, d_.work_cap + 4096);
      for (int k = 0; k < INGRESS_SLOTS; ++k)
        ingress_slot_[k] = (u8*)view(("ingress_s" + std::to_string(k)).c_str(), base + 2 * wb + k * ib, d_.ingress_cap + 64);
    }
    // per-parity step IO: step t uses set t % npar_, so step t+1's H2D and step t-1's D2H
    // overlap step t's kernels (the graph of each parity is captured once)
    npar_ = (d_.world == 1 && get("overlap", 1) == 0 && get("parities", 2) >= 3) ? 3 : 2;
    for (int p = 0; p < npar_; ++p) {
      std::string sfx = std::to_string(p);
      DS& io = io_[p];
      io.in = (StepIn*)dev(("in" + sfx).c_str(), sizeof(StepIn));
      io.segs = (const SegIn*)dev(("segs" + sfx).c_str(), sizeof(SegIn) * d_.seg_max);
      // ingress payloads rotate over INGRESS_SLOTS buffers by step (StepIn.ingress): the
      // next step's payload goes into a slot whose last reader (three steps back) is known
      // done, so an early H2D never waits on the GPU
      io.ingress = ingress_slot_[p];
      io.seg_out = (SegOut*)dev(("seg_out_d" + sfx).c_str(), sizeof(SegOut) * d_.seg_max);
      io.seg_out_h = (SegOut*)hst(("seg_out" + sfx).c_str(), sizeof(SegOut) * d_.seg_max);
      io.ctr_host = (Counters*)hst(("ctr_host" + sfx).c_str(), sizeof(Counters));
      io.conn_out = (ConnOut*)dev(("conn_out_d" + sfx).c_str(), sizeof(ConnOut) * d_.c_max);
      io.conn_out_h = (ConnOut*)hst(("conn_out" + sfx).c_str(), sizeof(ConnOut) * d_.c_max);
      io.ctrl = (u8*)dev(("ctrl_d" + sfx).c_str(), d_.ctrl_cap);
      io.ctrl_h = (u8*)hst(("ctrl" + sfx).c_str(), d_.ctrl_cap);
      io.ctrl_rec = (CtrlRec*)dev(("ctrl_rec_d" + sfx).c_str(), sizeof(CtrlRec) * d_.seg_max * 2);
      io.ctrl_rec_h = (CtrlRec*)hst(("ctrl_rec" + sfx).c_str(), sizeof(CtrlRec) * d_.seg_max * 2);
      io.grow_h = (RingMove*)hst(("grow" + sfx).c_str(), sizeof(RingMove) * GROW_MAX);
      io.conn_conf_h = (u32*)hst(("conn_conf" + sfx).c_str(), 4ull * d_.c_max);
      io.xchg = (u32*)hst(("xchg" + sfx).c_str(), 4ull * XC_WORDS);
      if (d_.persist && p == 0)
        for (int k = 0; k < PSLOTS; ++k) {   // shared by both parities (rotating per step)
          const std::string ks = std::to_string(k);
          d_.ps_persist[k] = (u8*)hst(("persist" + ks).c_str(), d_.persist_bytes + 64);
          d_.ps_crec[k] = (ConsumedRec*)hst(("consumed" + ks).c_str(), sizeof(ConsumedRec) * (u64)d_.persist_max + 64);
        }
      // the step's descriptors stay in host-mapped memory: k_stage reads them over PCIe
      // and writes the device copies (io.in / io.segs) the later kernels read.  Two H2D
      // copies per step were runtime blit kernels on a third hardware queue, ordered behind
      // the prefetched payload: ~50 us between the payload's arrival and the ingest
      io.in_h = (const StepIn*)hst(("stage_in" + sfx).c_str(), sizeof(StepIn));
      io.segs_h = (const SegIn*)hst(("stage_segs" + sfx).c_str(), sizeof(SegIn) * d_.seg_max + 64);
      stage_in_[p] = (StepIn*)buf("stage_in" + sfx).ptr;
      stage_segs_[p] = (SegIn*)buf("stage_segs" + sfx).ptr;
      // deferred control writes ridden by this parity's steps (pack_deltas)
      io.delta_h = (const u8*)hst(("delta" + sfx).c_str(), DELTA_CAP);
      dl_h_[p] = (u8*)buf("delta" + sfx).ptr;
      // Basic.Get on the step: the requests (H2D with the step) and their answers
      io.get_req = (const GetReq*)dev(("get_req" + sfx).c_str(), sizeof(GetReq) * GET_STEP_MAX);
      io.get_out_h = (GetOut*)hst(("get_out" + sfx).c_str(), sizeof(GetOut) * GET_STEP_MAX);
      stage_gets_[p] = (GetReq*)pinned(("stage_gets" + sfx).c_str(), sizeof(GetReq) * GET_STEP_MAX);
      io.unpause_req = (const u32*)dev(("unpause_req" + sfx).c_str(), 4ull * UNPAUSE_STEP_MAX);
      stage_unp_[p] = (u32*)pinned(("stage_unp" + sfx).c_str(), 4ull * UNPAUSE_STEP_MAX);
    }

    // egress slots rotate per step independently of the IO parity: step t renders into
    // slot t % EGRESS_SLOTS, so its kernels only wait for the D2H of step t-3 (long done)
    // instead of step t-2's, which is still on the copy engine
    for (int e = 0; e < EGRESS_SLOTS; ++e) {
      std::string sfx = std::to_string(e);
      egress_dev_[e] = (u8*)dev(("egress" + sfx).c_str(), egress_alloc_);
      if (copy_mode_ == 2) {
        egress_host_dev_[e] = (u8*)hst(("egress_host" + sfx).c_str(), egress_alloc_);
        egress_host_[e] = (u8*)buf("egress_host" + sfx).ptr;
      } else {
        egress_host_[e] = (u8*)pinned(("egress_host" + sfx).c_str(), egress_alloc_);
      }
    }
    d_.carry = (u8*)dev("carry", (u64)d_.c_max * d_.carry_cap + 64);
    d_.carry_len = (u32*)dev("carry_len", 4ull * d_.c_max);
    d_.conn_paused = (u32*)dev("conn_paused", 4ull * d_.c_max);
    d_.conn_frame_max = (u32*)dev("conn_frame_max", 4ull * d_.c_max);
    d_.conn_vhost = (u32*)dev("conn_vhost", 4ull * d_.c_max);
    d_.conn_last_rx = (i64*)dev("conn_last_rx", 8ull * d_.c_max);
    d_.chmap = (u32*)dev("chmap", 4ull * d_.c_max * d_.chmap_size);
    d_.conn_ret_bytes = (u32*)dev("conn_ret_bytes", 4ull * d_.c_max);
    d_.conn_conf_bytes = (u32*)dev("conn_conf_bytes", 4ull * d_.c_max);
    d_.conn_dfirst = (u32*)dev("conn_dfirst", 4ull * d_.c_max);
    d_.conn_dlast = (u32*)dev("conn_dlast", 4ull * d_.c_max);
    d_.conn_wblock = (const u32*)hst("conn_wblock", 4ull * d_.c_max);
    d_.conn_total = (u32*)dev("conn_total", 4ull * d_.c_max);
    d_.conn_base = (u32*)dev("conn_base", 4ull * d_.c_max);

    d_.seg_start = (u32*)dev("seg_start", 4ull * d_.seg_max);
    d_.seg_total = (u32*)dev("seg_total", 4ull * d_.seg_max);
    d_.seg_cmd_base = (u32*)dev("seg_cmd_base", 4ull * d_.seg_max);
    d_.seg_npub = (u32*)dev("seg_npub", 4ull * d_.seg_max);
    d_.seg_nack = (u32*)dev("seg_nack", 4ull * d_.seg_max);
    // up to DEC_SEG_LDS segments k_decode numbers publishes / acks from the frame scan's
    // per-segment ordinals (segment prefix in LDS): no rank scan over the commands
    d_.rank_scan = d_.seg_max > DEC_SEG_LDS ? 1u : 0u;
    d_.scan_inplace = get("scan_in_place", 1) ? 1u : 0u;

    d_.cmds = (Cmd*)dev("cmds", sizeof(Cmd) * (u64)d_.cmd_max);
    d_.frags = (Frag*)dev("frags", sizeof(Frag) * ((u64)d_.frag_max + d_.import_max));
    d_.cmd_is_pub = (u32*)dev("cmd_is_pub", 4ull * d_.cmd_max);
    d_.cmd_is_ack = (u32*)dev("cmd_is_ack", 4ull * d_.cmd_max);
    d_.cmd_pub_rank = (u32*)dev("cmd_pub_rank", 4ull * d_.cmd_max);
    d_.cmd_ack_rank = (u32*)dev("cmd_ack_rank", 4ull * d_.cmd_max);

    d_.pubs = (Pub*)dev("pubs", sizeof(Pub) * (u64)d_.pub_cap);
    d_.pub_keyvec = (i8*)dev("pub_keyvec", (u64)d_.pub_cap * TOPIC_K + 64);
    d_.pub_kwoff = (u16*)dev("pub_kwoff", 2ull * TOPIC_WORDS * d_.pub_cap + 64);
    d_.pub_match = (u16*)dev("pub_match", 2ull * d_.pub_cap * (d_.tb_pad / 16) + 64);
    d_.pub_nq = (u32*)dev("pub_nq", 4ull * d_.pub_cap);
    d_.pub_qc = (u32*)dev("pub_qc", 32ull * d_.pub_cap);
    d_.pub_slot = (u32*)dev("pub_slot", 4ull * d_.pub_cap);
    d_.pub_routed = (u32*)dev("pub_routed", 4ull * d_.pub_cap);
    d_.pub_pair_off = (u32*)dev("pub_pair_off", 4ull * d_.pub_cap);
    d_.pub_slot_off = (u32*)dev("pub_slot_off", 4ull * d_.pub_cap);
    d_.pub_routed_rank = (u32*)dev("pub_routed_rank", 4ull * d_.pub_cap);
    d_.pub_ret = (u32*)dev("pub_ret", 4ull * d_.pub_cap);
    d_.ret_list = (u32*)dev("ret_list", 4ull * d_.pub_cap);
    d_.pub_ret_sz = (u32*)dev("pub_ret_sz", 4ull * d_.pub_cap);
    d_.pub_ret_off = (u32*)dev("pub_ret_off", 4ull * d_.pub_cap);
    d_.conn_ret_min = (u32*)dev("conn_ret_min", 4ull * d_.c_max);
    u64 xw = d_.world > 1 ? (u64)d_.world * d_.pub_cap : 64;
    d_.q_owner = (u32*)dev("q_owner", 4ull * d_.q_max);
    d_.q_excl = (u32*)dev("q_excl", 4ull * d_.q_max);
    d_.dget = (DGet*)dev("dget", sizeof(DGet) * (u64)DGET_MAX);
    d_.conn_gempty = (u32*)dev("conn_gempty", 4ull * d_.c_max);
    d_.conn_gempty_ch = (u32*)dev("conn_gempty_ch", 4ull * d_.c_max);
    d_.pub_rmask = (u32*)dev("pub_rmask", 4ull * d_.pub_cap);
    d_.xp_cnt = nullptr;   // (per-rank count arrays: k_pack_scan counts in registers)
    d_.xp_cnt_off = (u32*)dev("xp_cnt_off", 4 * xw);
    d_.xp_byt = nullptr;
    d_.xp_byt_off = (u32*)dev("xp_byt_off", 4 * xw);
    // k_pack_scan: per-tile aggregates / prefixes (2 * WORLD_MAX values per 1024 publishes)
    d_.pk_agg = (u32*)dev("pk_agg", 4ull * 2 * WORLD_MAX * (ceil_div(d_.pub_max ? d_.pub_max : 1, 1024) + 1));
    d_.xs_base = (u32*)dev("xs_base", 8ull * WORLD_MAX);
    d_.xr_base = (u32*)dev("xr_base", 16ull * WORLD_MAX);
    d_.id_base = (u64*)dev("id_base", 8);
    d_.q_durable = (u32*)dev("q_durable", 4ull * d_.q_max);
    if (d_.persist) {
      d_.prec = (PersistRec*)dev("prec", sizeof(PersistRec) * (u64)d_.persist_max);
      d_.crec = (ConsumedRec*)dev("crec", sizeof(ConsumedRec) * (u64)d_.persist_max);
      d_.ps_size = (u32*)dev("ps_size", 4ull * d_.persist_max);
      d_.ps_off = (u32*)dev("ps_off", 4ull * d_.persist_max);
    }
    if (d_.world == 1 && restore_max_) {
      d_.recv_desc = (const RDesc*)dev("restore_desc", sizeof(RDesc) * (u64)restore_max_);
      d_.recv_pay = (const u8*)dev("restore_pay", d_.xfer_bytes + 64);
    }
    d_.acks = (Ack*)dev("acks", sizeof(Ack) * (u64)d_.ack_max);

    for (int k = 0; k < 2; ++k) {
      d_.pair_k[k] = (u32*)dev(k ? "pair_k1" : "pair_k0", 4ull * d_.pair_max);
      d_.pair_v[k] = (u32*)dev(k ? "pair_v1" : "pair_v0", 4ull * d_.pair_max);
    }
    d_.q_first = (u32*)dev("q_first", 4ull * d_.q_max);

    d_.x_hkey = (u64*)dev("x_hkey", 8ull * xhash);
    d_.x_hval = (i32*)dev("x_hval", 4ull * xhash);
    d_.x_type = (u32*)dev("x_type", 4ull * d_.x_max);
    d_.x_fan_off = (u32*)dev("x_fan_off", 4ull * d_.x_max);
    d_.x_fan_n = (u32*)dev("x_fan_n", 4ull * d_.x_max);
    d_.x_t_off = (u32*)dev("x_t_off", 4ull * d_.x_max);
    d_.x_t_n = (u32*)dev("x_t_n", 4ull * d_.x_max);
    d_.fan_q = (u32*)dev("fan_q", 4ull * fan_max);
    d_.d_key = (u64*)dev("d_key", 8ull * dhash);
    d_.d_exch = (i32*)dev("d_exch", 4ull * dhash);
    d_.d_kb_off = (u32*)dev("d_kb_off", 4ull * dhash);
    d_.d_kb_len = (u32*)dev("d_kb_len", 4ull * dhash);
    d_.d_q_off = (u32*)dev("d_q_off", 4ull * dhash);
    d_.d_q_n = (u32*)dev("d_q_n", 4ull * dhash);
    d_.d_q = (u32*)dev("d_q", 4ull * dq_max);
    d_.kpool = (u8*)dev("kpool", kpool);
    d_.t_queue = (u32*)dev("t_queue", 4ull * d_.tb_pad);
    d_.t_exch = (u32*)dev("t_exch", 4ull * d_.tb_pad);
    d_.t_kb_off = (u32*)dev("t_kb_off", 4ull * d_.tb_pad);
    d_.t_kb_len = (u32*)dev("t_kb_len", 4ull * d_.tb_pad);
    d_.t_flags = (u32*)dev("t_flags", 4ull * d_.tb_pad);
    d_.t_count = (u32*)dev("t_count", 16);
    {   // (until the first topology upload: every row, as before the count existed)
      const u32 all[4] = {d_.tb_pad, 0, 0, 0};
      HIPCHECK(hipMemcpy(d_.t_count, all, 16, hipMemcpyHostToDevice));
    }
    d_.t_expect = (i32*)dev("t_expect", 4ull * d_.tb_pad);
    d_.t_mat = (i8*)dev("t_mat", (u64)d_.tb_pad * TOPIC_K + 64);
    d_.t_woff = (u16*)dev("t_woff", 2ull * TOPIC_WORDS * d_.tb_pad + 64);

    d_.q_ring_off = (u64*)dev("q_ring_off", 8ull * d_.q_max);
    d_.q_ring_mask = (u64*)dev("q_ring_mask", 8ull * d_.q_max);
    d_.q_head = (u64*)dev("q_head", 8ull * d_.q_max);
    d_.q_tail = (u64*)dev("q_tail", 8ull * d_.q_max);
    d_.q_ttl = (i64*)dev("q_ttl", 8ull * d_.q_max);
    d_.q_cons_off = (u32*)dev("q_cons_off", 4ull * d_.q_max);
    d_.q_cons_n = (u32*)dev("q_cons_n", 4ull * d_.q_max);
    d_.q_rr = (u32*)dev("q_rr", 4ull * d_.q_max);
    d_.q_active = (u32*)dev("q_active", 4ull * d_.q_max);
    d_.q_cons = (u32*)dev("q_cons", 4ull * d_.cons_max);
    d_.ring = (Desc*)dev("ring", sizeof(Desc) * d_.ring_pool);
    d_.ring_top = (u64*)dev("ring_top", 8);
    d_.q_max_cap = (u64*)dev("q_max_cap", 8ull * d_.q_max);
    d_.q_enq_tail = (u64*)dev("q_enq_tail", 8ull * d_.q_max);
    d_.moves = (RingMove*)dev("moves", sizeof(RingMove) * (u64)d_.q_max);
    d_.defer_free = (u32*)dev("defer_free", 4ull * d_.pub_cap);

    d_.ch_confirm = (u32*)dev("ch_confirm", 4ull * nch);
    d_.ch_pub_cnt = (u32*)dev("ch_pub_cnt", 4ull * nch);
    d_.ch_pub_fail = (u32*)dev("ch_pub_fail", 4ull * nch);
    d_.ch_confirm_next = (u64*)dev("ch_confirm_next", 8ull * nch);
    d_.ch_next_tag = (u64*)dev("ch_next_tag", 8ull * nch);
    d_.ch_uhead = (u64*)dev("ch_uhead", 8ull * nch);
    d_.ch_ack_upto = (u64*)dev("ch_ack_upto", 8ull * nch);
    d_.ch_req_upto = (u64*)dev("ch_req_upto", 8ull * nch);
    d_.ch_mlo = (u32*)dev("ch_mlo", 4ull * nch);
    d_.ch_mhi = (u32*)dev("ch_mhi", 4ull * nch);
    d_.ch_prefetch = (u32*)dev("ch_prefetch", 4ull * nch);
    d_.ch_global = (u32*)dev("ch_global", 4ull * nch);
    d_.ch_flow = (u32*)dev("ch_flow", 4ull * nch);
    d_.ch_tx = (u32*)dev("ch_tx", 4ull * nch);
    d_.ch_num = (u32*)dev("ch_num", 4ull * nch);
    d_.ch_unacked = (u32*)dev("ch_unacked", 4ull * nch);
    d_.ch_win = (u32*)dev("ch_win", 4ull * nch);
    d_.ch_dirty = (u32*)dev("ch_dirty", 4ull * nch);
    d_.dirty_list = (u32*)dev("dirty_list", 4ull * nch);
    d_.n_dirty = (u32*)dev("n_dirty", 4);
    d_.def_list = (u32*)dev("def_list", 4ull * nch);
    d_.uwin = (USlot*)dev("uwin", sizeof(USlot) * (u64)nch * ucap);

    d_.cons_q = (u32*)dev("cons_q", 4ull * d_.cons_max);
    d_.cons_ch = (u32*)dev("cons_ch", 4ull * d_.cons_max);
    d_.cons_noack = (u32*)dev("cons_noack", 4ull * d_.cons_max);
    d_.cons_active = (u32*)dev("cons_active", 4ull * d_.cons_max);
    d_.cons_unacked = (u32*)dev("cons_unacked", 4ull * (d_.cons_max + 1));   // [cons_max]: Basic.Get
    d_.cons_tag_off = (u32*)dev("cons_tag_off", 4ull * d_.cons_max);
    d_.cons_tag_len = (u32*)dev("cons_tag_len", 4ull * d_.cons_max);
    d_.tpool = (u8*)dev("tpool", 256ull * d_.cons_max);

    d_.msgs = (MsgEnt*)dev("msgs", sizeof(MsgEnt) * (u64)d_.msg_max);
    d_.msg_free = (u32*)dev("msg_free", 4ull * d_.msg_max);
    d_.msg_free_top = (u32*)dev("msg_free_top", 4);
    d_.log = (u8*)dev("log", d_.log_bytes + 4096);
    d_.log_head = (u64*)dev("log_head", 8);
    d_.log_tail = (u64*)dev("log_tail", 8);
    d_.log_step_base = (u64*)dev("log_step_base", 8);
    d_.log_live = (i64*)dev("log_live", 8ull * d_.n_log_blocks);
    d_.live_bytes = (i64*)dev("live_bytes", 8);
    d_.id_next = (u64*)dev("id_next", 8);
    // cold-body spill ring in pinned host memory (mapped: kernels read / write it over PCIe)
    d_.spill_bytes = (get("spill_bytes", 0) / d_.log_block) * d_.log_block;
    d_.n_spill_blocks = d_.spill_bytes / d_.log_block;
    d_.spill_head = (u64*)dev("spill_head", 8);
    d_.spill_tail = (u64*)dev("spill_tail", 8);
    d_.spill_live = (i64*)dev("spill_live", 8ull * (d_.n_spill_blocks ? d_.n_spill_blocks : 1));
    d_.spill = d_.spill_bytes ? (u8*)hst("spill", d_.spill_bytes + 4096) : nullptr;
    d_.spill_host = d_.spill_bytes ? (u64)buf("spill").ptr : 0;
    d_.spill_tail_lag = (u64*)dev("spill_tail_lag", 8ull * SPILL_LAG);
    spill_moved_ = (unsigned long long*)dev("spill_moved", 8);
    d_.cold_live = (i64*)dev("cold_live", 8ull * COLD_SEGS);
    cold_recs_ = (ColdRec*)dev("cold_recs", sizeof(ColdRec) * COLD_BATCH);
    cold_cnt_ = (u32*)dev("cold_cnt", 16);
    cold_bytes_ = (unsigned long long*)dev("cold_bytes", 8);
    cold_end_ = (u64*)dev("cold_end", 8ull * d_.q_max);
    if (d_.spill_bytes && d_.world == 1) {   // (side operations)
      side_d_ = alloc("cold_side", sizeof(ColdRec) * COLD_BATCH + 64, true);
      side_h_ = buf("cold_side").ptr;
      side_live_h_ = (i64*)pinned("cold_side_live", 8ull * COLD_SEGS);
      HIPCHECK(hipEventCreateWithFlags(&ev_side_, hipEventDisableTiming));
    }
    d_.q_cold_lim = (u64*)dev("q_cold_lim", 8ull * d_.q_max);
    HIPCHECK(hipMemset(d_.q_cold_lim, 0xff, 8ull * d_.q_max));
    d_.q_spill_cur = (u64*)dev("q_spill_cur", 8ull * d_.q_max);
    d_.q_cold_cur = (u64*)dev("q_cold_cur", 8ull * d_.q_max);

    d_.deliv = (Deliv*)dev("deliv", sizeof(Deliv) * (u64)d_.deliv_max);
    {
      const u64 nrun = (u64)d_.q_max * RUNS_PER_Q;
      d_.runs = (Run*)dev("runs", sizeof(Run) * nrun);
      d_.q_nruns = (u32*)dev("q_nruns", 4ull * d_.q_max);
      d_.run_order = (u32*)dev("run_order", 4ull * nrun);
      d_.run_start = (u32*)dev("run_start", 4ull * nrun);
      u64 np2 = 1;
      while (np2 < nrun) np2 <<= 1;
      d_.run_key = (u64*)dev("run_key", 8ull * np2);
    }
    d_.dv_size = (u32*)dev("dv_size", 4ull * d_.deliv_max);
    d_.dv_off = (u32*)dev("dv_off", 4ull * d_.deliv_max);
    d_.ch_first = (u32*)dev("ch_first", 4ull * nch);

    d_.req = (ReqItem*)dev("req", sizeof(ReqItem) * (u64)d_.req_max);
    d_.req_n = (u32*)dev("req_n", 4);
    d_.req_q_n = (u32*)dev("req_q_n", 4ull * d_.q_max);

    ntiles_max_ = ceil_div(d_.pair_max, SORT_TILE);
    d_.hist = (u32*)dev("hist", 4ull * 2048 * ntiles_max_);        // up to 11-bit digits
    d_.hist_scan = (u32*)dev("hist_scan", 4ull * 2048 * ntiles_max_);
    d_.scan_tmp = (u32*)dev("scan_tmp", 4ull * 1024);
    {   // look-back scan state: status words for the largest scan, ticket/epoch
      u64 big = d_.pub_cap > d_.cmd_max ? d_.pub_cap : d_.cmd_max;
      big = big > d_.deliv_max ? big : d_.deliv_max;
      big = big > d_.c_max ? big : d_.c_max;
      scan_smax_ = ceil_div(big, SCAN_TILE) + 1;
      // 4 arrays x smax 4096-tiles, or 16 arrays x 4*smax 1024-tiles
      scan_status_ = (u64*)dev("scan_status", 8ull * 16 * (SCAN_TILE / 1024) * scan_smax_);
      scan_ctl_ = (u32*)dev("scan_ctl", 64);
      // the ingest half's command scan has its own look-back state (it may run next to a
      // scan of the previous step's routing half)
      scan_status_ing_ = (u64*)dev("scan_status_ing", 8ull * 16 * (SCAN_TILE / 1024) * scan_smax_);
      scan_ctl_ing_ = (u32*)dev("scan_ctl_ing", 64);
    }
    d_.tot = (u32*)dev("tot", 4ull * 128);
    d_.egress_budget = (u64*)dev("egress_budget", 8);
    gate_dummy_ = dev("gate_dummy", 64);
    h2d_dummy_ = pinned("h2d_dummy", 64);
    // Basic.Get: rendered frames + result, host-mapped (a stored body never exceeds the
    // carry, which bounds an assembled command)
    get_cap_ = (u64)d_.carry_cap + d_.carry_cap / 64 + 4096;
    get_out_dev_ = (u8*)hst("get_out", get_cap_);
    get_res_dev_ = (GetRes*)hst("get_res", sizeof(GetRes));
    // k_frame_scan phase timestamps (scripts/frame_scan_phases.py): off unless asked for --
    // each mark is a clock read plus a store on the block's critical path
    d_.dbg = get("fs_marks", 0) ? (u64*)dev("dbg", 8ull * 16 * d_.seg_max) : nullptr;

    // the step's ingest buffers exist once per parity: with overlap (world 1), parity
    // t+1's ingest half (k_stage .. k_decode) runs while parity t's routing / delivery half
    // still reads its own commands, publishes, bodies, counters and scratch totals
    dup(&DS::ctr, "ctr", sizeof(Counters));
    dup(&DS::tot, "tot", 4ull * 128);
    dup(&DS::egress_budget, "egress_budget", 8);
    dup(&DS::seg_start, "seg_start", 4ull * d_.seg_max);
    dup(&DS::seg_total, "seg_total", 4ull * d_.seg_max);
    dup(&DS::seg_cmd_base, "seg_cmd_base", 4ull * d_.seg_max);
    dup(&DS::seg_npub, "seg_npub", 4ull * d_.seg_max);
    dup(&DS::seg_nack, "seg_nack", 4ull * d_.seg_max);
    par1_.push_back([this](DS& io) { io.work = work_p1_; });   // (allocated with the ingress slots)
    dup(&DS::cmds, "cmds", sizeof(Cmd) * (u64)d_.cmd_max);
    dup(&DS::frags, "frags", sizeof(Frag) * ((u64)d_.frag_max + d_.import_max));
    dup(&DS::cmd_is_pub, "cmd_is_pub", 4ull * d_.cmd_max);
    dup(&DS::cmd_is_ack, "cmd_is_ack", 4ull * d_.cmd_max);
    dup(&DS::cmd_pub_rank, "cmd_pub_rank", 4ull * d_.cmd_max);
    dup(&DS::cmd_ack_rank, "cmd_ack_rank", 4ull * d_.cmd_max);
    dup(&DS::pubs, "pubs", sizeof(Pub) * (u64)d_.pub_cap);
    dup(&DS::pub_keyvec, "pub_keyvec", (u64)d_.pub_cap * TOPIC_K + 64);
    dup(&DS::pub_kwoff, "pub_kwoff", 2ull * TOPIC_WORDS * d_.pub_cap + 64);
    dup(&DS::acks, "acks", sizeof(Ack) * (u64)d_.ack_max);
    dup(&DS::dget, "dget", sizeof(DGet) * (u64)DGET_MAX);
    for (int p = 0; p < npar_; ++p) {
      DS io = d_;
      if (p == 1)
        for (auto& f : par1_) f(io);
      io.in = io_[p].in; io.segs = io_[p].segs; io.ingress = io_[p].ingress; io.seg_out = io_[p].seg_out;
      io.ctr_host = io_[p].ctr_host; io.conn_out = io_[p].conn_out;
      io.ctrl = io_[p].ctrl; io.ctrl_rec = io_[p].ctrl_rec; io.xchg = io_[p].xchg;
      io.seg_out_h = io_[p].seg_out_h; io.conn_out_h = io_[p].conn_out_h; io.ctrl_h = io_[p].ctrl_h;
      io.ctrl_rec_h = io_[p].ctrl_rec_h; io.grow_h = io_[p].grow_h; io.conn_conf_h = io_[p].conn_conf_h;
      io.get_req = io_[p].get_req; io.get_out_h = io_[p].get_out_h; io.unpause_req = io_[p].unpause_req;
      io.in_h = io_[p].in_h; io.segs_h = io_[p].segs_h; io.delta_h = io_[p].delta_h;
      static_cast<DS&>(io_[p]) = io;
    }
    // native exchange (sharded steps driven by the native front end, csrc/core/frontend.cpp):
    // the engine owns the per-parity send / receive buffers and moves them itself (RCCL or
    // the host shared-memory backend); implies the pipelined (lagged) exchange
    native_x_ = d_.world > 1 && get("native_xchg", 0) != 0;
    if (native_x_) {
      lag_ = true;
      for (int p = 0; p < 2; ++p) {
        std::string sfx = std::to_string(p);
        xs_desc_[p] = (u8*)dev(("xs_desc" + sfx).c_str(), 64ull * d_.xfer_desc_max + 64);
        xs_pay_[p] = (u8*)dev(("xs_pay" + sfx).c_str(), d_.xfer_bytes + 64);
        xr_desc_[p] = (u8*)dev(("xr_desc" + sfx).c_str(), 64ull * d_.import_max + 64);
        xr_pay_[p] = (u8*)dev(("xr_pay" + sfx).c_str(), d_.import_bytes + 64);
      }
      for (int p = 0; p < 2; ++p) {   // parity p packs into S[p], imports R[p^1]
        io_[p].send_desc = (RDesc*)xs_desc_[p]; io_[p].send_pay = xs_pay_[p];
        io_[p].recv_desc = (const RDesc*)xr_desc_[p ^ 1]; io_[p].recv_pay = xr_pay_[p ^ 1];
      }
      xfer_set_ = true;
    }
    if (links_) {
      DS& L = d_;
      L.links = 1;
      L.lk_cap = (u32)get("link_acks", 2ull * d_.deliv_max);
      L.conn_link = (u32*)dev("conn_link", 4ull * d_.c_max);
      L.conn_link_tq = (u32*)dev("conn_link_tq", 4ull * d_.c_max);
      L.conn_link_epoch = (u32*)dev("conn_link_epoch", 4ull * d_.c_max);
      L.link_conns = (u32*)dev("link_conns", 4ull * 64);
      L.n_link_conns = (u32*)dev("n_link_conns", 4);
      L.link_nbase = (u32*)dev("link_nbase", 4ull * d_.c_max);
      L.link_bbase = (u32*)dev("link_bbase", 4ull * d_.c_max);
      L.link_dbase = (u32*)dev("link_dbase", 4ull * WORLD_MAX);
      L.q_link_owner = (u32*)dev("q_link_owner", 4ull * d_.q_max);
      L.q_link_ch = (u32*)dev("q_link_ch", 4ull * d_.q_max);
      L.q_link_epoch = (u32*)dev("q_link_epoch", 4ull * d_.q_max);
      L.lk_cnt = (u32*)dev("lk_cnt", 4ull * WORLD_MAX);
      fill("q_link_ch", 0xff);
      for (int p = 0; p < 2; ++p) {
        std::string sfx = std::to_string(p);
        ls_desc_[p] = (u8*)dev(("ls_desc" + sfx).c_str(), 64ull * d_.deliv_max + 64);
        ls_pay_[p] = (u8*)dev(("ls_pay" + sfx).c_str(), d_.egress_cap + 64);
        lk_send_[p] = (u8*)dev(("lk_send" + sfx).c_str(), 16ull * d_.world * L.lk_cap + 64);
        rack_[p] = (u8*)dev(("rack" + sfx).c_str(), 16ull * d_.world * L.lk_cap + 64);
      }
      for (int p = 0; p < 2; ++p) {
        DS& io = io_[p];
        io.links = 1; io.lk_cap = L.lk_cap;
        io.conn_link = L.conn_link; io.conn_link_tq = L.conn_link_tq; io.conn_link_epoch = L.conn_link_epoch;
        io.link_conns = L.link_conns; io.n_link_conns = L.n_link_conns; io.link_nbase = L.link_nbase;
        io.link_bbase = L.link_bbase; io.link_dbase = L.link_dbase; io.q_link_owner = L.q_link_owner;
        io.q_link_ch = L.q_link_ch; io.q_link_epoch = L.q_link_epoch; io.lk_cnt = L.lk_cnt;
        io.lsend_desc = (RDesc*)ls_desc_[p]; io.lsend_pay = ls_pay_[p]; io.lk_send = (AckRec*)lk_send_[p];
        io.rack = (const AckRec*)rack_[p ^ 1];   // the acks of the exchange this parity imports
      }
    }
    for (int p = 0; p < 2; ++p) io_[p].import_bytes = d_.import_bytes;
    if (copy_mode_ == 3) init_sdma();
    HIPCHECK(hipStreamCreateWithFlags(&s_comp_, hipStreamNonBlocking));
    HIPCHECK(hipStreamCreateWithFlags(&s_h2d_, hipStreamNonBlocking));
    // (non-overlapped single GPU, cfg h2d_alt) odd steps' ingress copies on a second stream:
    // consecutive steps' payloads need not wait for one stream's previous copy to retire
    if (d_.world == 1 && get("overlap", 1) == 0 && get("h2d_alt", 0) != 0)
      HIPCHECK(hipStreamCreateWithFlags(&s_h2d_alt_, hipStreamNonBlocking));
    // (non-overlapped single GPU, HSA egress, cfg h2d_hsa) ingress payloads queued on an SDMA
    // engine through HSA and waited for on the device (k_h2d_wait): consecutive steps' copies
    // run back to back, with no HIP marker / cross-queue barrier between them
    h2d_hsa_ = copy_mode_ == 3 && !sdma_ && d_.world == 1 && get("overlap", 1) == 0 && get("h2d_hsa", 0) != 0;
    if (h2d_hsa_)
      for (int k = 0; k < INGRESS_SLOTS; ++k)
        if (hsa_signal_create(0, 0, nullptr, &ing_sig_[k]) != HSA_STATUS_SUCCESS ||
            hsa_signal_create(0, 0, nullptr, &ing_sig2_[k]) != HSA_STATUS_SUCCESS)
          throw std::runtime_error("hsa_signal_create failed");
    // ingress payloads share the H2D stream: a stream of their own stalled the host for ~6 ms
    // in an early prefetch on some boxes (12+ MB copies; profiles/r4_summary.md)
    s_pre_ = s_h2d_;
    HIPCHECK(hipStreamCreateWithFlags(&s_d2h_, hipStreamNonBlocking));
    {   // the ingest half gets its own (high-priority) hardware queue: next to the routing
        // half of the previous step, not queued behind it
      int lo = 0, hi = 0;
      HIPCHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
      HIPCHECK(hipStreamCreateWithPriority(&s_ing_, hipStreamNonBlocking, hi));
    }
    for (int p = 0; p < npar_; ++p) {
      HIPCHECK(hipEventCreateWithFlags(&ev_ing_[p], hipEventDisableTiming));
      HIPCHECK(hipEventCreateWithFlags(&ev_pre_[p], hipEventDisableTiming));
      HIPCHECK(hipEventCreateWithFlags(&ev_rest_[p], hipEventDisableTiming));
    }
    for (int k = 0; k < INGRESS_SLOTS; ++k)
      HIPCHECK(hipEventCreateWithFlags(&ev_ing_slot_[k], hipEventDisableTiming));
    // overlap (world 1): the step's ingest half runs on its own stream, next to the
    // previous step's routing / delivery half
    overlap_ = d_.world == 1 && get("overlap", 1) != 0;
    // egress by reference (StepIn.ref_back / ref_min): off unless the driver keeps its
    // ingress payloads for it (set_egress_ref)
    ref_back_ = cfg.contains("egress_ref_back") ? cfg["egress_ref_back"].cast<int>() : -1;
    if (ref_back_ > 64) throw std::runtime_error("egress_ref_back: at most 64 steps back");
    ref_min_ = (u32)get("egress_ref_min", 256);
    // egress_gate (HSA SDMA egress, overlapped steps): the step's D2H is queued on the SDMA
    // engine at launch, behind a gate signal the step's last kernel opens (final_step), sized
    // from the recent steps' egress (a host-issued tail copies the rest when a step renders
    // more) -- the host is off the render -> D2H path.  0: the D2H is issued by the host
    // after it saw the step finish (egress_copy)
    // (sharded ranks too: the step's last kernel -- phase B's -- opens the gate the same way)
    gated_ = copy_mode_ == 3 && get("egress_gate", 1) != 0;
    for (int p = 0; p < npar_; ++p) {
      HIPCHECK(hipEventCreateWithFlags(&ev_h2d_[p], hipEventDisableTiming));
      HIPCHECK(hipEventCreateWithFlags(&ev_done_[p], hipEventDisableTiming));
      HIPCHECK(hipEventCreateWithFlags(&ev_a_[p], hipEventDisableTiming));
      HIPCHECK(hipEventCreateWithFlags(&ev_ext_[p], hipEventDisableTiming));
    }
    for (int e = 0; e < EGRESS_SLOTS; ++e) HIPCHECK(hipEventCreateWithFlags(&ev_d2h_[e], hipEventDisableTiming));
    // ---- initial state
    fill("conn_dfirst", 0xff);
    fill("conn_ret_min", 0xff);
    fill("conn_dlast", 0xff);
    fill("x_hval", 0xff);
    fill("ch_mlo", 0xff);
    fill("d_exch", 0xff);
    std::vector<u32> fl(d_.msg_max);
    for (u32 i = 0; i < d_.msg_max; ++i) fl[i] = d_.msg_max - 1 - i;
    HIPCHECK(hipMemcpy(d_.msg_free, fl.data(), 4ull * d_.msg_max, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(d_.msg_free_top, &d_.msg_max, 4, hipMemcpyHostToDevice));
    HIPCHECK(hipDeviceSynchronize());
  }

  ~Engine() {
    x_stop(true);
    // a gated copy never outlives its gate: open every gate, so no SDMA queue waits forever
    // (a step that faulted before its last kernel), then let the copies finish
    if (copy_mode_ == 3)
      for (int e = 0; e < EGRESS_SLOTS; ++e) {
        if (gate_sig_[e].handle) hsa_signal_store_screlease(gate_sig_[e], 0);
        if (sdma_pending_[e] || tail_pending_[e]) {
          try { sdma_wait(e); } catch (const std::exception&) {}   // (reported already)
        }
      }
    for (int k = 0; k < INGRESS_SLOTS; ++k)
      if (ing_sig_[k].handle) {
        if (ing_hsa_[k]) (void)hsa_signal_wait_scacquire(ing_sig_[k], HSA_SIGNAL_CONDITION_EQ, 0, 2000 * block_ticks_,
                                                          HSA_WAIT_STATE_BLOCKED);
        if (ing_split_[k]) (void)hsa_signal_wait_scacquire(ing_sig2_[k], HSA_SIGNAL_CONDITION_EQ, 0, 2000 * block_ticks_,
                                                            HSA_WAIT_STATE_BLOCKED);
      }
    (void)hipStreamSynchronize(s_comp_);
    (void)hipStreamSynchronize(s_h2d_);
    if (s_h2d_alt_) (void)hipStreamSynchronize(s_h2d_alt_);
    (void)hipStreamSynchronize(s_pre_);
    for (int k = 0; k < INGRESS_SLOTS; ++k)
      if (ing_sig_[k].handle) { hsa_signal_destroy(ing_sig_[k]); hsa_signal_destroy(ing_sig2_[k]); }
    (void)hipStreamSynchronize(s_d2h_);
    for (int p = 0; p < npar_; ++p) {
      if (graph_exec_[p]) (void)hipGraphExecDestroy(graph_exec_[p]);
      if (graph_b_[p]) (void)hipGraphExecDestroy(graph_b_[p]);
      (void)hipEventDestroy(ev_a_[p]);
      (void)hipEventDestroy(ev_ext_[p]);
      (void)hipEventDestroy(ev_h2d_[p]);
      (void)hipEventDestroy(ev_done_[p]);
    }
    for (int e = 0; e < EGRESS_SLOTS; ++e) (void)hipEventDestroy(ev_d2h_[e]);
    if (ev_side_) (void)hipEventDestroy(ev_side_);
    if (s_x_) (void)hipStreamDestroy(s_x_);
    if (s_io_) (void)hipStreamDestroy(s_io_);
    (void)hipStreamDestroy(s_comp_);
    (void)hipStreamDestroy(s_h2d_);
    if (s_h2d_alt_) (void)hipStreamDestroy(s_h2d_alt_);
    (void)hipStreamDestroy(s_d2h_);
    for (auto& kv : bufs_) {
      if (kv.second.view) continue;
      if (kv.second.host) (void)hipHostFree(kv.second.ptr);
      else (void)hipFree(kv.second.ptr);
    }
  }

  // page-locked (not mapped into kernels) host buffer: DMA target/source
  void* pinned(const char* name, size_t bytes) {
    Buf b;
    b.bytes = bytes;
    b.host = true;
    HIPCHECK(hipHostMalloc(&b.ptr, bytes, hipHostMallocPortable));
    memset(b.ptr, 0, bytes);
    total_bytes_ += bytes;
    bufs_[name] = b;
    return b.ptr;
  }

  // ------------------------------------------------------------- buffers
  void* alloc(const char* name, size_t bytes, bool host) {
    Buf b;
    b.bytes = bytes;
    b.host = host;
    if (host) {
      HIPCHECK(hipHostMalloc(&b.ptr, bytes, hipHostMallocMapped | hipHostMallocPortable));
      memset(b.ptr, 0, bytes);
    } else {
      HIPCHECK(hipMalloc(&b.ptr, bytes));
      HIPCHECK(hipMemset(b.ptr, 0, bytes));
    }
    total_bytes_ += bytes;
    bufs_[name] = b;
    if (host) {
      void* dp = nullptr;
      HIPCHECK(hipHostGetDevicePointer(&dp, b.ptr, 0));
      return dp;
    }
    return b.ptr;
  }

  // a named device range inside an allocation made with alloc()
  void* view(const char* name, void* ptr, size_t bytes) {
    Buf b;
    b.ptr = ptr;
    b.bytes = bytes;
    b.view = true;
    bufs_[name] = b;
    return ptr;
  }

  const Buf& buf(const std::string& name) const {
    auto it = bufs_.find(name);
    if (it == bufs_.end()) throw std::runtime_error("no buffer " + name);
    return it->second;
  }

  void fill(const std::string& name, int byte) {
    const Buf& b = buf(name);
    if (b.host) memset(b.ptr, byte, b.bytes);
    else HIPCHECK(hipMemset(b.ptr, byte, b.bytes));
  }

  void upload(const std::string& name, py::buffer data, size_t offset) {
    py::buffer_info info = data.request();
    size_t n = (size_t)info.size * info.itemsize;
    const Buf& b = buf(name);
    if (offset + n > b.bytes) throw std::runtime_error("upload overflows " + name);
    if (b.host) memcpy((u8*)b.ptr + offset, info.ptr, n);
    else io_copy((u8*)b.ptr + offset, info.ptr, n, hipMemcpyHostToDevice);
  }

  // table reads / writes from any host thread: on their own non-blocking stream (a
  // legacy-stream copy would conflict with a graph capture running on the stepper thread)
  void io_copy(void* dst, const void* src, size_t n, hipMemcpyKind k) {
    std::lock_guard<std::mutex> g(io_mu_);
    if (!s_io_) HIPCHECK(hipStreamCreateWithFlags(&s_io_, hipStreamNonBlocking));
    HIPCHECK(hipMemcpyAsync(dst, src, n, k, s_io_));
    HIPCHECK(hipStreamSynchronize(s_io_));
  }

  py::bytes download(const std::string& name, size_t offset, size_t n) {
    const Buf& b = buf(name);
    if (n == 0) n = b.bytes - offset;
    if (offset + n > b.bytes) throw std::runtime_error("download overflows " + name);
    std::string out(n, '\0');
    if (b.host) memcpy(&out[0], (u8*)b.ptr + offset, n);
    else io_copy(&out[0], (u8*)b.ptr + offset, n, hipMemcpyDeviceToHost);
    return py::bytes(out);
  }

  // zero-copy numpy view of a host-mapped buffer
  py::array host_view(const std::string& name) {
    const Buf& b = buf(name);
    if (!b.host) throw std::runtime_error(name + " is not host-mapped");
    return py::array(py::dtype("uint8"), {(py::ssize_t)b.bytes}, {(py::ssize_t)1}, b.ptr,
                     py::capsule(b.ptr, [](void*) {}));
  }

  py::dict info() const {
    py::dict o;
    o["c_max"] = d_.c_max; o["chpc"] = d_.chpc; o["q_max"] = d_.q_max; o["x_max"] = d_.x_max;
    o["cons_max"] = d_.cons_max; o["seg_max"] = d_.seg_max; o["carry_cap"] = d_.carry_cap;
    o["cmd_max"] = d_.cmd_max; o["pair_max"] = d_.pair_max; o["deliv_max"] = d_.deliv_max;
    o["msg_max"] = d_.msg_max; o["ucap"] = d_.ucap_mask + 1; o["deliver_cap"] = d_.deliver_cap;
    o["chmap_size"] = d_.chmap_size; o["xhash"] = d_.xhash_mask + 1; o["dhash"] = d_.dhash_mask + 1;
    o["tb_max"] = d_.tb_max; o["tb_pad"] = d_.tb_pad; o["log_bytes"] = d_.log_bytes;
    o["spill_bytes"] = d_.spill_bytes;
    o["ingress_cap"] = d_.ingress_cap; o["egress_cap"] = d_.egress_cap; o["ring_pool"] = d_.ring_pool;
    o["work_cap"] = d_.work_cap; o["total_bytes"] = total_bytes_; o["req_max"] = d_.req_max;
    o["carry_budget"] = carry_budget_;
    o["exchange_lag"] = lag_ ? 1 : 0;
    o["native_xchg"] = native_x_ ? 1 : 0;
    o["rccl_standin"] = (rccl_ && cmqx::RcclLib::get().standin) ? 1 : 0;   // (tests/rccl_standin: not RCCL)
    o["links"] = links_ ? 1 : 0;
    o["import_bytes"] = d_.import_bytes;
    o["world"] = d_.world; o["rank"] = d_.my_rank; o["import_max"] = d_.import_max; o["pub_cap"] = d_.pub_cap;
    o["copy_engine"] = copy_mode_ == 3 ? "hsa-sdma" : copy_mode_ == 2 ? "kernel" : (sdma_ ? "nocu" : "blit");
    o["copy_wgs"] = copy_wgs_;
    o["egress_gate"] = gated_ ? 1 : 0;
    o["egress_ref_back"] = ref_back_;
    o["egress_ref_min"] = ref_min_;
    o["egress_slots"] = EGRESS_SLOTS;
    o["parities"] = npar_;
    { u32 e = 0; while (copy_mode_ == 3 && e < 32 && !(((u32)sdma_engine_ >> e) & 1u)) ++e; o["sdma_engine"] = copy_mode_ == 3 ? (int)e : -1; }
    { u32 e = 0; while (sdma_engine2_ && e < 32 && !(((u32)sdma_engine2_ >> e) & 1u)) ++e; o["sdma_engine2"] = sdma_engine2_ ? (int)e : -1; }
    { u32 e = 0; while (h2d_hsa_ && e < 32 && !(((u32)ing_engine_ >> e) & 1u)) ++e; o["h2d_hsa_engine"] = h2d_hsa_ ? (int)e : -1; }
    { u32 e = 0; while (h2d_hsa_ && ing_engine2_ && e < 32 && !(((u32)ing_engine2_ >> e) & 1u)) ++e;
      o["h2d_hsa_engine2"] = h2d_hsa_ && ing_engine2_ ? (int)e : -1; }
    o["persist"] = d_.persist; o["persist_max"] = d_.persist_max; o["persist_bytes"] = d_.persist_bytes;
    o["restore_max"] = restore_max_;
    o["xfer_desc_max"] = d_.xfer_desc_max; o["xfer_bytes"] = d_.xfer_bytes; o["world_max"] = WORLD_MAX;
    o["sizeof"] = py::dict(py::arg("StepIn") = sizeof(StepIn), py::arg("SegIn") = sizeof(SegIn),
                           py::arg("SegOut") = sizeof(SegOut), py::arg("Counters") = sizeof(Counters),
                           py::arg("CtrlRec") = sizeof(CtrlRec), py::arg("ConnOut") = sizeof(ConnOut),
                           py::arg("MsgEnt") = sizeof(MsgEnt), py::arg("Desc") = sizeof(Desc),
                           py::arg("USlot") = sizeof(USlot), py::arg("Deliv") = sizeof(Deliv),
                           py::arg("Pub") = sizeof(Pub), py::arg("Cmd") = sizeof(Cmd),
                           py::arg("RDesc") = sizeof(RDesc));
    return o;
  }

  // ------------------------------------------------------------- step (pipelined)
  // submit(): stage step t's ingress on the H2D stream and launch parity t&1's graph on
  // the compute stream behind it.  wait_results(p) -> host-mapped SegOut/Counters/ConnOut
  // are valid; egress_copy(p) DMAs exactly the rendered bytes on the D2H stream;
  // egress_wait(p) -> egress_host(p) is valid.
  // defer: queue only the ingress H2D and return; launch(p) starts the step's kernels.  A
  // sharded driver uses the gap to run the previous step's exchange while this step's
  // bytes cross PCIe (the host waits on phase A of t-1, not on H2D(t) + phase A(t))
  int submit(py::buffer segs, u64 payload_ptr, u64 payload_len, i64 now_ms, u64 step, u64 id_ms,
             u32 worker, bool defer, u32 flags) {
    py::buffer_info si = segs.request();
    size_t sb = (size_t)si.size * si.itemsize;
    return submit_raw((const SegIn*)si.ptr, (u32)(sb / sizeof(SegIn)), payload_ptr, payload_len, now_ms, id_ms,
                      worker, defer, flags);
  }

  // step numbers are the engine's own submit sequence (latency histogram, message
  // publish step): identical whether Python or the native front end drives the steps
  int submit_raw(const SegIn* segp, u32 nseg, u64 payload_ptr, u64 payload_len, i64 now_ms, u64 id_ms,
                 u32 worker, bool defer = false, u32 sflags = 0) {
    HostTimer ht(&ht_[0]);
    Range rg("chanamq.step.submit");
    const size_t sb = (size_t)nseg * sizeof(SegIn);
    const u64 step = seq_;
    if (nseg > d_.seg_max) throw std::runtime_error("too many segments");
    if (payload_len > d_.ingress_cap) throw std::runtime_error("ingress payload exceeds ingress_cap");
    int p = (int)(seq_ % (u64)npar_);
    if (inflight_[p]) throw std::runtime_error("submit: results of the previous step of this parity not collected");
    HIPCHECK(hipEventSynchronize(ev_h2d_[p]));  // staging buffers of step t-2 are free
    // the payload first: the H2D is the step's longest stage and nothing below changes what
    // it copies (the slot's last reader, step t - INGRESS_SLOTS, is finished: its results were
    // collected before step t-2's).  It may already be on its way (prefetch): then only the
    // step's descriptors follow it on the H2D stream
    const int is = (int)(seq_ % INGRESS_SLOTS);
    const bool pre = pre_[p];
    if (pre && (pre_seq_[p] != step || pre_ptr_[p] != payload_ptr || pre_len_[p] != payload_len))
      throw std::runtime_error("submit: payload differs from the one prefetched for this step");
    pre_[p] = false;
    {   // overlapped engines move payloads on their own stream (prefetches run ahead of the
        // small per-step copies there; the ingest half waits for both)
      hipStream_t ps = overlap_ ? s_pre_ : h2d_of(step);
      if (payload_len && !pre) ingress_copy(step, is, payload_ptr, payload_len, ps);
      else if (!payload_len) ing_hsa_[is] = false;
    }
    StepIn* in = stage_in_[p];
    *in = StepIn{};
    in->h2d_sig = ing_hsa_[is] ? (u64)&((amd_signal_t*)ing_sig_[is].handle)->value : 0;
    in->h2d_sig2 = ing_hsa_[is] && ing_split_[is] ? (u64)&((amd_signal_t*)ing_sig2_[is].handle)->value : 0;
    if (in->h2d_sig && h2d_fault_) {   // (tests) the step waits on a word no copy completes
      h2d_fault_ = false;
      *(volatile i64*)h2d_dummy_ = 1;
      in->h2d_sig = (u64)h2d_dummy_;
      in->h2d_sig2 = 0;
      in->h2d_polls = 4096;
    }
    h2d_addr_[p] = in->h2d_sig;
    h2d_addr2_[p] = in->h2d_sig2;
    // the step's stream waits for the H2D stream only when a runtime copy of this step is on it
    h2d_hip_[p] = !h2d_hsa_ || (payload_len && !ing_hsa_[is]) || !pend_gets_.empty();
    in->nseg = nseg;
    in->ref_back = ref_back_ >= 0 ? (u32)ref_back_ : ref_back_ == -2 ? REF_SPILL_ONLY : 0xffffffffu;
    in->ref_min = ref_min_;
    in->ingress_host = ref_back_ >= 0 && payload_len ? payload_ptr : 0;
    in->dcap_bytes = dcap_bytes_;
    in->flags = sflags;
    in->now_ms = now_ms;
    in->step = step;
    in->id_ms = id_ms;
    in->worker = worker;
    const int e = (int)(seq_ % EGRESS_SLOTS);
    in->egress = (u64)egress_dev_[e];
    // the slot's previous D2H (step t - EGRESS_SLOTS, long finished) must be complete before
    // its gate is re-armed and its buffer rendered into again
    if (copy_mode_ == 3 && (sdma_pending_[e] || tail_pending_[e])) { HostTimer t(&ht_[1]); sdma_wait(e); }
    spec_[e] = gated_ ? spec_bytes() : 0;
    in->gate = 0;
    if (spec_[e]) {
      hsa_signal_store_screlease(gate_sig_[e], 1);
      in->gate = (u64)&((amd_signal_t*)gate_sig_[e].handle)->value;
      if (gate_fault_) {   // (tests) the last kernel opens a scratch word instead: the copy never starts
        gate_fault_ = false;
        in->gate = (u64)gate_dummy_;
      }
    }
    in->ingress = (u64)ingress_slot_[is];
    in->pslot = (u32)(seq_ % PSLOTS);
    pslot_of_[p] = (int)in->pslot;
    slot_of_[p] = e;
    launch_seq_[p] = step;
    if (sb) memcpy(stage_segs_[p], segp, sb);
    // staged Basic.Get requests ride this step; their answers start out RETRY (a queue the
    // device cannot serve now leaves it so)
    in->nget = (u32)pend_gets_.size();
    if (in->nget) {
      memcpy(stage_gets_[p], pend_gets_.data(), sizeof(GetReq) * in->nget);
      GetOut* go = (GetOut*)buf("get_out" + std::to_string(p)).ptr;
      for (u32 i = 0; i < in->nget; ++i) go[i] = GetOut{GS_RETRY, 0};
      HIPCHECK(hipMemcpyAsync((void*)io_[p].get_req, stage_gets_[p], sizeof(GetReq) * in->nget,
                              hipMemcpyHostToDevice, h2d_of(step)));
      pend_gets_.clear();
    }
    nget_[p] = in->nget;
    {   // body tiering asked for by the control plane rides this step (k_dequeue)
      std::lock_guard<std::mutex> g(dl_mu_);
      in->spill_frac = spill_req_[0];
      in->spill_hot = spill_req_[1];
      in->spill_budget = spill_req_[2];
    }
    // the control writes staged so far (what fits one step) and the connections
    // unpaused with them: a connection resumed in this step finds every write staged
    // before its unpause applied (k_stage applies the writes first)
    u32 nunp = 0;
    in->delta_bytes = pack_deltas(p, stage_unp_[p], &nunp);
    in->nunp = nunp;
    nunp_[p] = nunp;
    if (in->nunp)
      HIPCHECK(hipMemcpyAsync((void*)io_[p].unpause_req, stage_unp_[p], 4ull * in->nunp, hipMemcpyHostToDevice,
                              h2d_of(step)));
    dl_step_[p] = in->delta_bytes;
    if (in->nunp) h2d_hip_[p] = true;
    if (overlap_) HIPCHECK(hipEventRecord(ev_pre_[p], s_pre_));
    HIPCHECK(hipEventRecord(ev_h2d_[p], overlap_ ? s_h2d_ : h2d_of(step)));
    inflight_[p] = true;
    staged_[p] = true;
    ++seq_;
    if (!defer) launch(p);
    return p;
  }

  // Early ingress of the NEXT step (overlapped single-GPU steps): its payload crosses PCIe
  // while the current steps run -- the H2D stream only waits (on the GPU) for the ingest
  // half of the step two back, the last reader of this parity's ingress buffer -- so the
  // copy engine never idles between steps.  The step is then submit()ed with the same
  // payload.  false: not applicable (no overlap), nothing queued.
  // Up to two steps ahead: each call queues the payload of the next step not yet queued
  // (the next submit, then the one after it).
  bool prefetch(u64 payload_ptr, u64 payload_len) {
    if (d_.world != 1 || !payload_len) return false;   // (s_pre_ is s_h2d_: the step waits for it)
    Range rg("chanamq.step.prefetch");
    u64 tgt = seq_;
    int p = (int)(tgt % (u64)npar_);
    if (pre_[p]) {   // the next submit's payload is queued already: the one after it
      tgt = seq_ + 1;
      p = (int)(tgt % (u64)npar_);
      if (pre_[p]) return false;
    }
    if (staged_[p]) throw std::runtime_error("prefetch: this step's payload is already queued");
    if (payload_len > d_.ingress_cap) throw std::runtime_error("ingress payload exceeds ingress_cap");
    // the slot's last reader: the ingest of step tgt - INGRESS_SLOTS, collected by now in
    // the drivers' order (bench / front end prefetch t+1 once t-2 is finished); if not,
    // the copy waits for it on the GPU
    const int is = (int)(tgt % INGRESS_SLOTS);
    hipStream_t ps = overlap_ ? s_pre_ : h2d_of(tgt);
    ingress_copy(tgt, is, payload_ptr, payload_len, ps);
    pre_[p] = true;
    pre_seq_[p] = tgt;
    pre_ptr_[p] = payload_ptr;
    pre_len_[p] = payload_len;
    return true;
  }

  // ---- deferred control writes (no pipeline drain): the control plane stages table writes
  // while steps run; the next submitted step carries them (k_stage applies them first).
  // Any thread.  Writes to the same bytes: the last one wins (records never overlap).
  void stage_write(u64 dst, const u8* data, u64 n) {
    if (!n) return;
    // one record must fit a step's delta buffer with its header (a larger one
    // was never packed and kept the stepper spinning on host_work)
    if (n + 64 > DELTA_CAP) throw std::runtime_error("stage_write: a write larger than one step's delta buffer");
    std::lock_guard<std::mutex> g(dl_mu_);
    if (dl_.empty()) new_batch();
    DlBatch& bt = dl_.back();
    const u64 a = dst, e = dst + n;
    auto it = bt.w.lower_bound(a);
    if (it != bt.w.begin()) --it;
    std::vector<std::pair<u64, std::string>> keep;
    while (it != bt.w.end() && it->first < e) {
      const u64 s0 = it->first, s1 = s0 + it->second.size();
      if (s1 <= a) { ++it; continue; }
      if (s0 < a) keep.emplace_back(s0, it->second.substr(0, a - s0));
      if (s1 > e) keep.emplace_back(e, it->second.substr(e - s0));
      bt.bytes -= it->second.size();
      dl_bytes_ -= it->second.size();
      it = bt.w.erase(it);
    }
    for (auto& kv : keep) {
      bt.bytes += kv.second.size();
      dl_bytes_ += kv.second.size();
      bt.w.emplace(kv.first, std::move(kv.second));
    }
    bt.w.emplace(a, std::string((const char*)data, n));
    bt.bytes += n;
    dl_bytes_ += n;
  }
  void stage_write_buf(const std::string& name, py::buffer data, size_t offset) {
    py::buffer_info info = data.request();
    const size_t n = (size_t)info.size * info.itemsize;
    const Buf& b = buf(name);
    if (offset + n > b.bytes) throw std::runtime_error("stage_write overflows " + name);
    if (b.host) { memcpy((u8*)b.ptr + offset, info.ptr, n); return; }   // host-mapped: direct
    stage_write((u64)b.ptr + offset, (const u8*)info.ptr, n);
  }
  void stage_mark_dirty(u32 ch) {
    if (ch >= d_.c_max * d_.chpc) throw std::runtime_error("stage_mark_dirty: bad channel slot");
    std::lock_guard<std::mutex> g(dl_mu_);
    if (dl_.empty()) new_batch();
    auto& dv = dl_.back().dirty;
    for (u32 c : dv)
      if (c == ch) return;
    dv.push_back(ch);
  }
  // a light control section's staging: everything staged until stage_end() forms one batch
  // that no step takes before the section closed it (a step packing in the middle of a
  // section split a command's consumer rows and q_cons lists over two steps)
  void stage_begin() {
    std::lock_guard<std::mutex> g(dl_mu_);
    ++dl_open_;
    if (dl_.empty() || !dl_.back().open) new_batch();
  }
  void stage_end() {
    std::lock_guard<std::mutex> g(dl_mu_);
    if (dl_open_) --dl_open_;
    if (!dl_open_)
      for (auto& bt : dl_) bt.open = false;
  }
  void new_batch() {   // (dl_mu_ held)
    dl_.emplace_back();
    dl_.back().open = dl_open_ > 0;
    dl_.back().id = dl_next_id_++;
  }
  // batch ids (light sections tie their replies to them, Frontend::send_after): 0 = the
  // batch staging goes into now (the next one to be created when none is open), 1 = every
  // batch up to this id was taken by a submitted step (or applied by flush_deltas)
  u64 dl_state(int which) {
    std::lock_guard<std::mutex> g(dl_mu_);
    if (which == 2) return dl_open_;      // (diagnostics: open light sections, batches queued)
    if (which == 3) return dl_.size();
    if (which == 1) {   // (closed batches with nothing in them count as taken: no step needs to carry them)
      for (auto& bt : dl_)
        if (bt.open || !bt.w.empty() || !bt.dirty.empty() || !bt.unp.empty()) return bt.id - 1;
      return dl_next_id_ - 1;
    }
    // outside a light section nothing is staged for the caller: no batch to wait for
    return (!dl_.empty() && dl_.back().open) ? dl_.back().id : 0;
  }
  // from the next submitted step on, every step moves queued bodies in the oldest frac/65536
  // of the HBM log (past the first `hot` entries of a queue with consumers) to the host
  // spill ring, at most `budget` bytes a step -- spill() without the pipeline drain; frac 0
  // stops it.  Any thread.
  void stage_spill(u32 frac, u32 hot, u32 budget) {
    if (!d_.spill_bytes) return;
    std::lock_guard<std::mutex> g(dl_mu_);
    spill_req_[0] = frac; spill_req_[1] = hot; spill_req_[2] = budget;
  }
  // (records, data bytes, channels to mark) staged and not yet taken by a step
  py::tuple deltas_pending() {
    std::lock_guard<std::mutex> g(dl_mu_);
    size_t nrec = 0, nd = 0;
    for (auto& bt : dl_) { nrec += bt.w.size(); nd += bt.dirty.size(); }
    return py::make_tuple(nrec, dl_bytes_, nd);
  }
  bool host_work() {
    std::lock_guard<std::mutex> g(dl_mu_);
    if (!unp_ready_.empty() || side_queued()) return true;
    for (auto& bt : dl_) {
      if (bt.open) break;   // (staged by a section still running: stage_end wakes the stepper)
      if (!bt.w.empty() || !bt.dirty.empty() || !bt.unp.empty()) return true;
    }
    return false;
  }
  bool has_deltas() {
    std::lock_guard<std::mutex> g(dl_mu_);
    for (auto& bt : dl_)
      if (!bt.w.empty() || !bt.dirty.empty()) return true;
    return false;
  }
  // staged batches, oldest first, into parity p's host-mapped delta buffer: bytes used (0 =
  // none).  The oldest batch may go in part (what does not fit -- records or bytes -- stays
  // for a later step; records are independent bytes, and the control plane keeps a change
  // set within one step by cutting its batches at deltas_pending() limits); later closed
  // batches ride the same step whole, as long as they fit and write no byte an earlier
  // record of the step writes (k_apply_deltas applies a step's records in parallel).  One
  // batch per step capped the light sections at the step rate: under connection / RPC
  // churn on a slower (durable) broker they queued up until a full pause flushed them.
  // A batch's unpauses go with its last records to unp (at most UNPAUSE_STEP_MAX, *nunp) or,
  // with unp null (flush_deltas: no step), to unp_ready_ for the next submitted step.
  u32 pack_deltas(int p, u32* unp, u32* nunp) {
    std::lock_guard<std::mutex> g(dl_mu_);
    u32 nu = 0;
    auto take_unp = [&](std::vector<u32>& v) {
      size_t k = 0;
      for (; k < v.size(); ++k) {
        if (!unp) { unp_ready_.push_back(v[k]); continue; }
        if (nu == UNPAUSE_STEP_MAX) break;
        unp[nu++] = v[k];
      }
      v.erase(v.begin(), v.begin() + k);
    };
    auto done = [&](u32 r) { if (nunp) *nunp = nu; return r; };
    if (unp) take_unp(unp_ready_);
    // a step (unp set) never takes a batch a light section is still staging into;
    // flush_deltas (between steps, the control plane holds the engine) takes everything
    auto usable = [&](const DlBatch& bt) { return !(unp && bt.open); };
    // leading batches with no writes: their unpauses only
    while (!dl_.empty() && usable(dl_.front()) && dl_.front().w.empty() && dl_.front().dirty.empty()) {
      take_unp(dl_.front().unp);
      if (!dl_.front().unp.empty()) return done(0);   // (the step's unpause list is full)
      if (dl_.size() == 1 && dl_.front().open) { dl_.pop_front(); break; }
      dl_.pop_front();
    }
    if (dl_.empty() || !usable(dl_.front()) || (dl_.front().w.empty() && dl_.front().dirty.empty())) return done(0);
    // ---- plan: how many records of the first batch, then which whole batches follow
    u64 nrec = 0, nchunk = 0, ndirty = 0;
    std::map<u64, u64> iv;   // byte ranges [dst, end) written by the records planned so far
    auto overlaps = [&](u64 d0, u64 d1) {
      auto it = iv.lower_bound(d0);
      if (it != iv.end() && it->first < d1) return true;
      if (it != iv.begin() && std::prev(it)->second > d0) return true;
      return false;
    };
    auto need = [&](u64 r, u64 dn, u64 ch) { return 16 + 16 * r + ((4 * dn + 15) & ~15ull) + 16 * ch; };
    DlBatch& b0 = dl_.front();
    const u64 nd0 = std::min<u64>(b0.dirty.size(), 4096);
    u64 n0 = 0;
    for (auto& kv : b0.w) {
      const u64 ch = (kv.second.size() + 15) / 16;
      if (nrec == DELTA_REC_MAX || need(nrec + 1, nd0, nchunk + ch) > DELTA_CAP) break;
      ++nrec;
      nchunk += ch;
      iv[kv.first] = kv.first + kv.second.size();
      ++n0;
    }
    ndirty = nd0;
    size_t nwhole = 0;   // later batches taken whole
    if (n0 == b0.w.size() && nd0 == b0.dirty.size() && b0.unp.size() + nu <= UNPAUSE_STEP_MAX) {
      u32 nu_plan = nu + (u32)b0.unp.size();
      for (size_t k = 1; k < dl_.size(); ++k) {
        DlBatch& bt = dl_[k];
        if (!usable(bt)) break;
        u64 r = nrec, ch = nchunk;
        const u64 dn = ndirty + bt.dirty.size();
        bool ok = dn <= 4096 && nu_plan + bt.unp.size() <= UNPAUSE_STEP_MAX;
        for (auto it = bt.w.begin(); ok && it != bt.w.end(); ++it) {
          ++r;
          ch += (it->second.size() + 15) / 16;
          ok = r <= DELTA_REC_MAX && need(r, dn, ch) <= DELTA_CAP &&
               !overlaps(it->first, it->first + it->second.size());
        }
        if (!ok) break;
        for (auto& kv : bt.w) iv[kv.first] = kv.first + kv.second.size();
        nrec = r;
        nchunk = ch;
        ndirty = dn;
        nu_plan += (u32)bt.unp.size();
        ++nwhole;
      }
    }
    // ---- write: head, records, dirty channels, data
    u8* o = dl_h_[p];
    DeltaHead* h = (DeltaHead*)o;
    h->nrec = (u32)nrec; h->ndirty = (u32)ndirty; h->nchunk = (u32)nchunk; h->pad = 0;
    DeltaRec* recs = (DeltaRec*)(o + sizeof(DeltaHead));
    u32* dirty = (u32*)(recs + nrec);
    u8* data = (u8*)dirty + ((4ull * ndirty + 15) & ~15ull);
    u64 r = 0, c = 0, di = 0;
    auto put = [&](DlBatch& bt, u64 nr, u64 ndr) {
      u64 k = 0;
      for (auto it = bt.w.begin(); it != bt.w.end() && k < nr; ++k) {
        recs[r].dst = it->first;
        recs[r].len = (u32)it->second.size();
        recs[r].chunk0 = (u32)c;
        memcpy(data + 16 * c, it->second.data(), it->second.size());
        c += (it->second.size() + 15) / 16;
        bt.bytes -= it->second.size();
        dl_bytes_ -= it->second.size();
        it = bt.w.erase(it);
        ++r;
      }
      for (u64 k2 = 0; k2 < ndr; ++k2) dirty[di++] = bt.dirty[k2];
      bt.dirty.erase(bt.dirty.begin(), bt.dirty.begin() + ndr);
    };
    put(b0, n0, nd0);
    size_t gone = 0;   // leading batches fully taken (unpauses included)
    for (size_t k = 0; k <= nwhole; ++k) {
      DlBatch& bt = dl_[k];
      if (k) put(bt, bt.w.size(), bt.dirty.size());
      if (!bt.w.empty() || !bt.dirty.empty()) break;   // (the first batch went in part)
      take_unp(bt.unp);   // the whole batch went: its unpauses ride along
      if (!bt.unp.empty()) break;
      ++gone;
    }
    for (size_t k = 0; k < gone; ++k) dl_.pop_front();
    ++dl_steps_;
    return done((u32)((data - o) + 16 * c));
  }
  // between steps (the control plane holds the engine): apply what is staged now
  void flush_deltas() {
    if (!has_deltas()) return;
    if (inflight_[0] || inflight_[1]) throw std::runtime_error("flush_deltas() between steps only");
    sync();
    while (has_deltas()) {
      if (!pack_deltas(0, nullptr, nullptr)) break;
      hipLaunchKernelGGL(k_apply_deltas, dim3(1), dim3(1024), 0, s_comp_, io_[0], io_[0].delta_h);
      HIPCHECK(hipGetLastError());
      HIPCHECK(hipStreamSynchronize(s_comp_));
    }
  }

  // a paused connection (its control command answered) resumes with the next submitted
  // step: k_stage clears its flag before the frame scan reads it, so the host never writes
  // device state while steps are in flight.  Any thread.
  void stage_unpause(u32 conn) {
    if (conn >= d_.c_max) throw std::runtime_error("stage_unpause: bad connection");
    std::lock_guard<std::mutex> g(dl_mu_);
    if (dl_.empty()) new_batch();
    auto& v = dl_.back().unp;   // with the writes staged before it
    for (u32 c : v)
      if (c == conn) return;
    v.push_back(conn);
  }

  // Basic.Get requests for the next submitted step (validated by the caller: a local queue
  // of this rank, a channel slot of an open channel)
  void stage_gets(const GetReq* r, u32 n) {
    if (pend_gets_.size() + n > GET_STEP_MAX) throw std::runtime_error("stage_gets: more than GET_STEP_MAX per step");
    for (u32 i = 0; i < n; ++i) {
      if (r[i].q >= d_.q_max || r[i].chslot >= d_.c_max * d_.chpc) throw std::runtime_error("stage_gets: bad queue / channel");
      pend_gets_.push_back(r[i]);
    }
  }
  py::list get_out_py(int p) {
    const GetOut* go = (const GetOut*)buf("get_out" + std::to_string(p)).ptr;
    py::list l;
    for (u32 i = 0; i < nget_[p]; ++i) l.append(py::make_tuple(go[i].status, go[i].msg_count));
    return l;
  }

  // second half of submit(): the kernels of the staged step of parity p
  void launch(int p) {
    if (!staged_[p]) throw std::runtime_error("launch: no staged step of this parity");
    staged_[p] = false;
    const int e = slot_of_[p];
    // egress slot e (last used by step t-EGRESS_SLOTS) drained before this step's kernels
    // overwrite it; waited for only after this step's ingress H2D is queued, so the H2D
    // and the in-flight D2H overlap on their two SDMA engines
    if (copy_mode_ == 3 && sdma_pending_[e]) { HostTimer t(&ht_[1]); sdma_wait(e); }
    if (overlap_) {
      // ingest half on s_ing_: after this step's H2D and once parity p's buffers are free
      // (the routing half of step t-2); the routing half on s_comp_ behind it and behind
      // the previous step's routing half (stream order), as a single step would run
      // a side operation between the previous step's routing half and this step's ingest
      if (side_queued()) {
        run_side(s_comp_);
        HIPCHECK(hipStreamWaitEvent(s_ing_, ev_side_, 0));
      }
      HIPCHECK(hipStreamWaitEvent(s_ing_, ev_h2d_[p], 0));
      HIPCHECK(hipStreamWaitEvent(s_ing_, ev_pre_[p], 0));
      if (rest_issued_[p]) HIPCHECK(hipStreamWaitEvent(s_ing_, ev_rest_[p], 0));
      // control writes: applied between steps -- after the previous step's routing half
      if (dl_step_[p] && rest_issued_[p ^ 1]) HIPCHECK(hipStreamWaitEvent(s_ing_, ev_rest_[p ^ 1], 0));
      {
        HostTimer t(&ht_[2]);
        if (!graph_ing_[p]) capture_on(s_ing_, &graph_ing_[p], [&] { launch_ingest(s_ing_, io_[p]); });
        HIPCHECK(hipGraphLaunch(graph_ing_[p], s_ing_));
      }
      HIPCHECK(hipEventRecord(ev_ing_[p], s_ing_));
      ing_issued_[p] = true;
      HIPCHECK(hipStreamWaitEvent(s_comp_, ev_ing_[p], 0));
      if (d2h_issued_[e]) HIPCHECK(hipStreamWaitEvent(s_comp_, ev_d2h_[e], 0));
      {
        HostTimer t(&ht_[2]);
        if (!graph_rest_[p]) capture_on(s_comp_, &graph_rest_[p], [&] { launch_rest(s_comp_, io_[p]); });
        HIPCHECK(hipGraphLaunch(graph_rest_[p], s_comp_));
      }
      HIPCHECK(hipEventRecord(ev_rest_[p], s_comp_));
      rest_issued_[p] = true;
      {   // the ingress slot's last reader: the routing half (segments scanned in place)
        const int is = (int)(launch_seq_[p] % INGRESS_SLOTS);
        HIPCHECK(hipEventRecord(ev_ing_slot_[is], s_comp_));
        ing_slot_issued_[is] = true;
      }
      HIPCHECK(hipEventRecord(ev_done_[p], s_comp_));
      gated_copy(e);
      if (copy_mode_ == 2) {   // egress D2H right behind the step, sized on the device
        // (measured slower than the host-issued SDMA copy -- CU stores over PCIe stall
        // behind the next step's kernels: 8.7 vs 32.9 M msgs/s, profiles/r4_bench/pre_*)
        HIPCHECK(hipStreamWaitEvent(s_d2h_, ev_rest_[p], 0));
        hipLaunchKernelGGL(k_copy_out_dev, dim3(copy_wgs_), dim3(256), 0, s_d2h_, egress_host_dev_[e],
                           (const u8*)egress_dev_[e], (const Counters*)io_[p].ctr);
        HIPCHECK(hipEventRecord(ev_d2h_[e], s_d2h_));
        d2h_issued_[e] = true;
        eager_d2h_[p] = true;
      }
      return;
    }
    if (side_h_) run_side(s_comp_);
    if (h2d_hip_[p]) HIPCHECK(hipStreamWaitEvent(s_comp_, ev_h2d_[p], 0));
    if (d2h_issued_[e]) HIPCHECK(hipStreamWaitEvent(s_comp_, ev_d2h_[e], 0));
    if (d_.world > 1 && !xfer_set_) throw std::runtime_error("set_xfer_buffers() before the first sharded step");
    if (graph_enabled_) {
      if (!graph_exec_[p]) capture_main(p);
      HostTimer t(&ht_[2]);
      HIPCHECK(hipGraphLaunch(graph_exec_[p], s_comp_));
    } else {
      launch_main(s_comp_, io_[p]);
    }
    if (d_.world == 1) {   // the ingress slot's last reader (a later prefetch into it waits for it)
      const int is = (int)(launch_seq_[p] % INGRESS_SLOTS);
      HIPCHECK(hipEventRecord(ev_ing_slot_[is], s_comp_));
      ing_slot_issued_[is] = true;
    }
    if (d_.world > 1 && lag_) {
      HIPCHECK(hipEventRecord(ev_a_[p], s_comp_));
      counts_ready_[p] = true;
      if (native_x_) {   // the front end runs the previous step's exchange, then launch_b(p)
        b_due_[p] = true;
        return;
      }
      // phase B right behind phase A: imports the previous step's exchange
      u32* x = (u32*)buf("xchg" + std::to_string(p)).ptr;
      for (u32 r = 0; r < d_.world; ++r) {
        x[2 * WORLD_MAX + r] = x[XC_RECV_AN + r] = lag_recv_.size() == 2 * d_.world ? lag_recv_[r] : 0;
        x[3 * WORLD_MAX + r] = x[XC_RECV_AB + r] = lag_recv_.size() == 2 * d_.world ? lag_recv_[d_.world + r] : 0;
      }
      lag_recv_.clear();
      if (lag_stream_) {
        HIPCHECK(hipEventRecord(ev_ext_[p], (hipStream_t)lag_stream_));
        HIPCHECK(hipStreamWaitEvent(s_comp_, ev_ext_[p], 0));
        lag_stream_ = 0;
      }
      if (graph_enabled_) {
        if (!graph_b_[p]) capture_b(p);
        HIPCHECK(hipGraphLaunch(graph_b_[p], s_comp_));
      } else {
        launch_phase_b(s_comp_, io_[p]);
      }
      HIPCHECK(hipEventRecord(ev_done_[p], s_comp_));
      gated_copy(e);
    } else if (d_.world > 1) {
      HIPCHECK(hipEventRecord(ev_a_[p], s_comp_));
      phase_a_[p] = true;
      counts_ready_[p] = true;
    } else {
      HIPCHECK(hipEventRecord(ev_done_[p], s_comp_));
      gated_copy(e);   // (world 1, one stream: the whole step is one graph)
    }
  }

  // sharded step, after submit(): wait for phase A and return the per-destination send
  // counts [records x world, bytes x world, overflow]
  std::vector<u32> send_counts(int p) {
    if (!counts_ready_[p]) throw std::runtime_error("send_counts: no phase-A step in flight for this parity");
    counts_ready_[p] = false;
    HIPCHECK(hipEventSynchronize(ev_a_[p]));
    const u32* x = (const u32*)buf("xchg" + std::to_string(p)).ptr;
    std::vector<u32> o;
    for (u32 r = 0; r < d_.world; ++r) o.push_back(x[r]);
    for (u32 r = 0; r < d_.world; ++r) o.push_back(x[WORLD_MAX + r]);
    o.push_back(x[4 * WORLD_MAX]);
    return o;
  }

  // sharded step: received [records x world, bytes x world]; the exchange ran on
  // `stream` (0 = already complete); launches phase B behind it
  void submit_b(int p, std::vector<u32> recv, u64 stream) {
    if (!phase_a_[p]) throw std::runtime_error("submit_b: no phase-A step in flight for this parity");
    if (recv.size() != 2 * d_.world) throw std::runtime_error("submit_b: need 2*world counts");
    u32* x = (u32*)buf("xchg" + std::to_string(p)).ptr;
    for (u32 r = 0; r < d_.world; ++r) {
      x[2 * WORLD_MAX + r] = x[XC_RECV_AN + r] = recv[r];
      x[3 * WORLD_MAX + r] = x[XC_RECV_AB + r] = recv[d_.world + r];
    }
    if (stream) {
      HIPCHECK(hipEventRecord(ev_ext_[p], (hipStream_t)stream));
      HIPCHECK(hipStreamWaitEvent(s_comp_, ev_ext_[p], 0));
    }
    if (graph_enabled_) {
      if (!graph_b_[p]) capture_b(p);
      HIPCHECK(hipGraphLaunch(graph_b_[p], s_comp_));
    } else {
      launch_phase_b(s_comp_, io_[p]);
    }
    HIPCHECK(hipEventRecord(ev_done_[p], s_comp_));
    gated_copy(slot_of_[p]);   // (the phase-B render opens the gate)
    phase_a_[p] = false;
  }

  // recovery: enqueue store records (RDesc with MF_RESTORE, payload [ex][rk][props][body])
  // through the import path, between steps; returns the number of messages enqueued
  // cold bodies to the host spill ring, between steps: every queued message past the first
  // `hot` entries of its queue whose slot lies below log position `lim` (k_spill); returns
  // the bytes moved (the log tail advances over the emptied blocks at the next step)
  u64 spill(u64 lim, u32 hot) {
    if (!d_.spill_bytes) return 0;
    if (inflight_[0] || inflight_[1]) throw std::runtime_error("spill() between steps only");
    if (native_x_ && (counts_ready_[0] || counts_ready_[1])) throw std::runtime_error("spill() with an exchange pending");
    Range rg("chanamq.spill");
    sync();
    HIPCHECK(hipMemsetAsync(spill_moved_, 0, 8, s_comp_));
    hipLaunchKernelGGL(k_spill, dim3(d_.q_max), dim3(256), 0, s_comp_, io_[0], lim, hot, spill_moved_);
    HIPCHECK(hipGetLastError());
    unsigned long long moved = 0;
    HIPCHECK(hipMemcpyAsync(&moved, spill_moved_, 8, hipMemcpyDeviceToHost, s_comp_));
    HIPCHECK(hipStreamSynchronize(s_comp_));
    return moved;
  }

  // ---- cold store (third body tier), between steps; the host moves the bytes
  // out: candidate records (ColdRec[], bytes 0 = skip) for the host to write to the store
  // (slots below spill tail + lim)
  py::bytes cold_pick(u32 hot, u64 lim, u32 max_n, u64 max_bytes) {
    if (!d_.spill_bytes) return py::bytes("");
    cold_guard("cold_pick");
    if (max_n > COLD_BATCH) max_n = COLD_BATCH;
    HIPCHECK(hipMemsetAsync(cold_cnt_, 0, 16, s_comp_));
    HIPCHECK(hipMemsetAsync(cold_bytes_, 0, 8, s_comp_));
    hipLaunchKernelGGL(k_cold_pick, dim3(d_.q_max), dim3(256), 0, s_comp_, io_[0], hot, lim, (u64)0, cold_recs_,
                       max_n, cold_cnt_, cold_bytes_, max_bytes);
    return cold_fetch(max_n);
  }
  // ... the host stored them (ColdRec.cold = store offsets): switch the messages over
  void cold_commit(py::buffer recs) {
    const u32 n = cold_upload(recs);
    if (n) hipLaunchKernelGGL(k_cold_commit, blocks(n, 256), dim3(256), 0, s_comp_, io_[0], cold_recs_, n);
    HIPCHECK(hipStreamSynchronize(s_comp_));
  }
  // in: the cold entries near the heads of the held queues, each with a spill-ring slot
  py::bytes cold_scan(u32 window, u32 max_n) {
    if (!d_.spill_bytes) return py::bytes("");
    cold_guard("cold_scan");
    if (max_n > COLD_BATCH) max_n = COLD_BATCH;
    HIPCHECK(hipMemsetAsync(cold_cnt_, 0, 16, s_comp_));
    HIPCHECK(hipMemsetAsync(cold_end_, 0, 8ull * d_.q_max, s_comp_));
    hipLaunchKernelGGL(k_cold_scan, dim3(d_.q_max), dim3(64), 0, s_comp_, io_[0], window, cold_recs_, max_n, cold_cnt_,
                       cold_end_);
    return cold_fetch(max_n);
  }
  // ... the host read their bodies into those slots: back to SPILL_BIT, q_cold_lim moved on
  void cold_in(py::buffer recs) {
    const u32 n = cold_upload(recs);
    const u64 g = n > d_.q_max ? n : d_.q_max;
    hipLaunchKernelGGL(k_cold_in, blocks(g, 256), dim3(256), 0, s_comp_, io_[0], cold_recs_, n, cold_end_);
    HIPCHECK(hipStreamSynchronize(s_comp_));
  }
  // ---- the same four operations beside the steps (no pipeline drain, single GPU): the
  // cold thread posts one (side_*), the next launch() runs it on the compute stream between
  // two steps, side_wait() hands back its records; the steps keep flowing while the host
  // moves bodies between the ring and the store.  A pick is picked up again by the commit
  // only where its entry is still queued (k_cold_commit); k_cold_scan's ring slots count as
  // live until k_cold_in.  SIDE_LIVE copies cold_live (store segment GC).
  enum : int { SIDE_NONE = 0, SIDE_PICK, SIDE_COMMIT, SIDE_SCAN, SIDE_IN, SIDE_LIVE };
  void side_post(int kind, u32 a, u64 b, u64 c, u32 max_n, u64 max_bytes, const ColdRec* recs, u32 n) {
    if (d_.world != 1) throw std::runtime_error("side operations: single-GPU engines only");
    if (!side_h_) throw std::runtime_error("side operations: no spill ring");
    std::lock_guard<std::mutex> g(side_mu_);
    if (side_.kind) throw std::runtime_error("side operation pending (side_wait first)");
    if (n) memcpy((u8*)side_h_ + 64, recs, sizeof(ColdRec) * n);
    side_ = Side{kind, a, b, c, max_n > COLD_BATCH ? COLD_BATCH : max_n, max_bytes, n, false};
  }
  void side_cold_pick(u32 hot, u64 lim_rel, u64 min_used, u32 max_n, u64 max_bytes) {
    side_post(SIDE_PICK, hot, lim_rel, min_used, max_n, max_bytes, nullptr, 0);
  }
  void side_cold_scan(u32 window, u32 max_n) { side_post(SIDE_SCAN, window, 0, 0, max_n, 0, nullptr, 0); }
  void side_cold_commit(py::buffer recs) { side_recs(SIDE_COMMIT, recs); }
  void side_cold_in(py::buffer recs) { side_recs(SIDE_IN, recs); }
  void side_cold_live() { side_post(SIDE_LIVE, 0, 0, 0, 0, 0, nullptr, 0); }
  void side_recs(int kind, py::buffer recs) {
    py::buffer_info bi = recs.request();
    const size_t nb = (size_t)bi.size * bi.itemsize;
    if (nb % sizeof(ColdRec) || nb / sizeof(ColdRec) > COLD_BATCH) throw std::runtime_error("cold: bad ColdRec batch");
    side_post(kind, 0, 0, 0, 0, 0, (const ColdRec*)bi.ptr, (u32)(nb / sizeof(ColdRec)));
  }
  bool side_pending() {
    std::lock_guard<std::mutex> g(side_mu_);
    return side_.kind != SIDE_NONE;
  }
  bool side_queued() {
    std::lock_guard<std::mutex> g(side_mu_);
    return side_.kind && !side_.launched;
  }
  // launch(): the posted operation on stream s, ahead of the step's kernels
  void run_side(hipStream_t s) {
    std::lock_guard<std::mutex> g(side_mu_);
    if (!side_.kind || side_.launched) return;
    ColdRec* hrecs = (ColdRec*)((u8*)side_h_ + 64);
    ColdRec* drecs = (ColdRec*)((u8*)side_d_ + 64);
    switch (side_.kind) {
      case SIDE_PICK:
      case SIDE_SCAN:
        HIPCHECK(hipMemsetAsync(cold_cnt_, 0, 16, s));
        if (side_.kind == SIDE_PICK) {
          HIPCHECK(hipMemsetAsync(cold_bytes_, 0, 8, s));
          hipLaunchKernelGGL(k_cold_pick, dim3(d_.q_max), dim3(256), 0, s, io_[0], side_.a, side_.b, side_.c,
                             cold_recs_, side_.max_n, cold_cnt_, cold_bytes_, side_.max_bytes);
        } else {
          HIPCHECK(hipMemsetAsync(cold_end_, 0, 8ull * d_.q_max, s));
          hipLaunchKernelGGL(k_cold_scan, dim3(d_.q_max), dim3(64), 0, s, io_[0], side_.a, cold_recs_, side_.max_n,
                             cold_cnt_, cold_end_);
        }
        hipLaunchKernelGGL(k_side_out, dim3(64), dim3(256), 0, s, (const ColdRec*)cold_recs_, (const u32*)cold_cnt_,
                           side_.max_n, (u32*)drecs, (u32*)side_d_);
        break;
      case SIDE_COMMIT:
      case SIDE_IN:
        if (side_.n)
          HIPCHECK(hipMemcpyAsync(cold_recs_, hrecs, sizeof(ColdRec) * side_.n, hipMemcpyHostToDevice, s));
        if (side_.kind == SIDE_COMMIT) {
          if (side_.n)
            hipLaunchKernelGGL(k_cold_commit, blocks(side_.n, 256), dim3(256), 0, s, io_[0], cold_recs_, side_.n);
        } else {
          const u64 g2 = side_.n > d_.q_max ? side_.n : d_.q_max;
          hipLaunchKernelGGL(k_cold_in, blocks(g2, 256), dim3(256), 0, s, io_[0], cold_recs_, side_.n, cold_end_);
        }
        break;
      case SIDE_LIVE:
        HIPCHECK(hipMemcpyAsync(side_live_h_, d_.cold_live, 8ull * COLD_SEGS, hipMemcpyDeviceToHost, s));
        break;
    }
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipEventRecord(ev_side_, s));
    side_.launched = true;
    side_cv_.notify_all();
  }
  // the posted operation's result once it ran: ColdRec[] (pick / scan), cold_live bytes
  // (live), b"" (commit / in); None while it has not finished within timeout_s
  py::object side_wait(double timeout_s) {
    int kind = SIDE_NONE;
    hipError_t err = hipSuccess;
    bool done = false;
    {
      py::gil_scoped_release nogil;   // (no Python objects in here)
      std::unique_lock<std::mutex> g(side_mu_);
      kind = side_.kind;
      const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds((i64)(timeout_s * 1e6));
      if (kind && side_cv_.wait_until(g, until, [&] { return side_.launched; })) {
        g.unlock();
        while (true) {
          err = hipEventQuery(ev_side_);
          if (err == hipSuccess) { done = true; break; }
          if (err != hipErrorNotReady || std::chrono::steady_clock::now() > until) break;
          std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
      }
    }
    if (!kind) throw std::runtime_error("side_wait: nothing posted");
    if (err != hipSuccess && err != hipErrorNotReady) HIPCHECK(err);
    if (!done) return py::none();
    std::lock_guard<std::mutex> g(side_mu_);
    side_.kind = SIDE_NONE;
    if (kind == SIDE_PICK || kind == SIDE_SCAN) {
      const u32 n = *(volatile u32*)side_h_;
      return py::bytes((const char*)side_h_ + 64, sizeof(ColdRec) * (size_t)n);
    }
    if (kind == SIDE_LIVE) return py::bytes((const char*)side_live_h_, 8ull * COLD_SEGS);
    return py::bytes("");
  }

  void cold_guard(const char* what) {
    if (inflight_[0] || inflight_[1]) throw std::runtime_error(std::string(what) + "() between steps only");
    if (native_x_ && (counts_ready_[0] || counts_ready_[1]))
      throw std::runtime_error(std::string(what) + "() with an exchange pending");
    sync();
  }
  py::bytes cold_fetch(u32 max_n) {
    u32 n = 0;
    HIPCHECK(hipMemcpyAsync(&n, cold_cnt_, 4, hipMemcpyDeviceToHost, s_comp_));
    HIPCHECK(hipStreamSynchronize(s_comp_));
    if (n > max_n) n = max_n;
    std::string out(sizeof(ColdRec) * (size_t)n, '\0');
    if (n) HIPCHECK(hipMemcpy(&out[0], cold_recs_, out.size(), hipMemcpyDeviceToHost));
    return py::bytes(out);
  }
  u32 cold_upload(py::buffer recs) {
    py::buffer_info bi = recs.request();
    const size_t nb = (size_t)bi.size * bi.itemsize;
    if (nb % sizeof(ColdRec) || nb / sizeof(ColdRec) > COLD_BATCH) throw std::runtime_error("cold: bad ColdRec batch");
    const u32 n = (u32)(nb / sizeof(ColdRec));
    if (n) HIPCHECK(hipMemcpy(cold_recs_, bi.ptr, nb, hipMemcpyHostToDevice));
    return n;
  }

  u32 restore(py::buffer desc, py::buffer pay, i64 now_ms) {
    py::buffer_info di = desc.request(), pi = pay.request();
    u64 db = (u64)di.size * di.itemsize, pb = (u64)pi.size * pi.itemsize;
    u32 n = (u32)(db / sizeof(RDesc));
    // native exchange: restores run at a synchronisation point (no import pending) through
    // parity 0's receive buffers
    const RDesc* rdesc = d_.recv_desc ? d_.recv_desc : (native_x_ ? io_[0].recv_desc : nullptr);
    const u8* rpay = d_.recv_pay ? d_.recv_pay : (native_x_ ? io_[0].recv_pay : nullptr);
    if (!rdesc || n > d_.import_max || pb > d_.xfer_bytes)
      throw std::runtime_error("restore batch exceeds the import buffers (restore_max / restore_bytes)");
    if (inflight_[0] || inflight_[1]) throw std::runtime_error("restore() between steps only");
    if (native_x_ && (counts_ready_[0] || counts_ready_[1]))
      throw std::runtime_error("restore() with an exchange pending");
    sync();
    drain_egress();
    if (db) HIPCHECK(hipMemcpy((void*)rdesc, di.ptr, db, hipMemcpyHostToDevice));
    if (pb) HIPCHECK(hipMemcpy((void*)rpay, pi.ptr, pb, hipMemcpyHostToDevice));
    DS& io = io_[0];
    StepIn& in = *stage_in_[0];   // (k_stage copies it to the device; no step in flight)
    in = StepIn{};
    in.ref_back = 0xffffffffu;   // (no dispatch: nothing rendered)
    in.nseg = 0;
    in.now_ms = now_ms;
    in.step = seq_;
    in.id_ms = now_ms;
    in.worker = 0;
    in.egress = (u64)egress_dev_[0];
    in.ingress = (u64)ingress_slot_[0];
    u32* x = (u32*)buf("xchg0").ptr;
    for (u32 r = 0; r < 2 * WORLD_MAX; ++r) x[2 * WORLD_MAX + r] = x[XC_RECV_AN + r] = 0;
    for (u32 r = 0; r < WORLD_MAX; ++r) x[XC_RACK_N + r] = 0;
    x[2 * WORLD_MAX + d_.my_rank] = x[XC_RECV_AN + d_.my_rank] = n;
    x[3 * WORLD_MAX + d_.my_rank] = x[XC_RECV_AB + d_.my_rank] = (u32)pb;
    launch_ingest(s_comp_, io);
    launch_route(s_comp_, io, d_.pub_max);
    launch_phase_b(s_comp_, io, /*dispatch=*/false);
    HIPCHECK(hipStreamSynchronize(s_comp_));
    const Counters* c = (const Counters*)buf("ctr_host0").ptr;
    return c->n_routed_msgs;
  }

  // Basic.Get between steps: (status, message_count, frames, tag, msg_id, qpos, persist,
  // expired [(msg_id, q, qpos)] of durable x persistent messages dropped by the TTL skip)
  py::tuple basic_get(u32 q, u32 chslot, u32 noack, i64 now_ms) {
    if (inflight_[0] || inflight_[1]) throw std::runtime_error("basic_get() between steps only");
    if (q >= d_.q_max || chslot >= d_.c_max * d_.chpc) throw std::runtime_error("basic_get: bad queue / channel");
    Range rg("chanamq.basic_get");
    sync();
    hipLaunchKernelGGL(k_basic_get, dim3(1), dim3(64), 0, s_comp_, io_[0], q, chslot, noack, now_ms, get_out_dev_,
                       get_cap_, get_res_dev_);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(s_comp_));
    const GetRes& r = *(const GetRes*)buf("get_res").ptr;
    py::list exp;
    for (u32 i = 0; i < r.n_exp && i < GET_EXP_MAX; ++i)
      exp.append(py::make_tuple(r.exp[i].msg_id, r.exp[i].q, r.exp[i].qpos));
    py::bytes frames(r.status == GET_OK ? (const char*)buf("get_out").ptr : "", r.status == GET_OK ? r.out_len : 0);
    return py::make_tuple(r.status, r.msg_count, frames, r.tag, r.msg_id, r.qpos, r.persist, exp);
  }

  // exchange_lag mode: the all-to-all of step t finished on `stream` (0 = complete) with
  // these received counts; the next submit()'s phase B imports it
  void set_import(std::vector<u32> recv, u64 stream) {
    if (recv.size() != 2 * d_.world) throw std::runtime_error("set_import: need 2*world counts");
    lag_recv_ = recv;
    lag_stream_ = stream;
  }

  // per-parity exchange operands (exchange_lag: parity p sends from S[p] and imports R[p^1])
  void set_xfer_parity(int p, u64 send_desc, u64 send_pay, u64 recv_desc, u64 recv_pay) {
    io_[p].send_desc = (RDesc*)send_desc; io_[p].send_pay = (u8*)send_pay;
    io_[p].recv_desc = (const RDesc*)recv_desc; io_[p].recv_pay = (const u8*)recv_pay;
    if (graph_exec_[p]) { HIPCHECK(hipGraphExecDestroy(graph_exec_[p])); graph_exec_[p] = nullptr; }
    if (graph_b_[p]) { HIPCHECK(hipGraphExecDestroy(graph_b_[p])); graph_b_[p] = nullptr; }
    xfer_set_ = true;
  }

  // caller-owned exchange operands (device pointers, e.g. torch tensors used by RCCL)
  void set_xfer_buffers(u64 send_desc, u64 send_pay, u64 recv_desc, u64 recv_pay) {
    d_.send_desc = (RDesc*)send_desc; d_.send_pay = (u8*)send_pay;
    d_.recv_desc = (const RDesc*)recv_desc; d_.recv_pay = (const u8*)recv_pay;
    for (int p = 0; p < npar_; ++p) {
      io_[p].send_desc = d_.send_desc; io_[p].send_pay = d_.send_pay;
      io_[p].recv_desc = d_.recv_desc; io_[p].recv_pay = d_.recv_pay;
      if (graph_exec_[p]) { HIPCHECK(hipGraphExecDestroy(graph_exec_[p])); graph_exec_[p] = nullptr; }
      if (graph_b_[p]) { HIPCHECK(hipGraphExecDestroy(graph_b_[p])); graph_b_[p] = nullptr; }
    }
    xfer_set_ = true;
  }

  // ------------------------------------------------------------- native exchange
  // Sharded steps driven by the native front end: submit(t) stages step t and launches its
  // phase A; exchange(parity of t-1) moves step t-1's cross-rank records (and the link
  // traffic of the step before) between the live ranks; launch_b(t) imports them.  The
  // count exchange carries a flags word per rank (control-sync request, busy), so
  // replicated control ops need no per-tick collective of their own.

  // kind "rccl": arg = 128-byte RCCL unique id; "shm": arg = shared-memory name.
  // members: the live logical ranks (sorted); timeout_ms bounds every host wait;
  // failover: the host also waits (bounded) for the bulk transfer before phase B
  // counts_shm (rccl only): a shared-memory name common to the group -- the per-step count
  // exchange then runs through host shared memory (a spin barrier, ~µs) instead of an
  // RCCL round trip with two PCIe copies; the bulk records stay on RCCL over xGMI.  All
  // ranks of one node (the bench, the sharded server on one host) can use it.
  void xchg_setup(const std::string& kind, const std::string& arg, std::vector<int> members, int timeout_ms,
                  bool failover, const std::string& counts_shm, bool async) {
    if (!native_x_) throw std::runtime_error("xchg_setup: engine built without native_xchg");
    for (int& m : members)
      if (m < 0 || m >= (int)d_.world) throw std::runtime_error("xchg_setup: bad member");
    std::sort(members.begin(), members.end());
    x_stop();   // (a job of the old group finished or failed: its phase B was released)
    if (!s_x_) {
      // high priority: the runtime takes a high-priority stream's hardware queue from a pool
      // of its own, so the exchange never shares a queue with s_comp_ -- where, with the
      // asynchronous exchange, phase B's k_xwait spins until this stream's transfer is done
      // (4 hardware queues per process: a sixth normal stream wraps onto s_comp_'s queue)
      int lo = 0, hi = 0;
      HIPCHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
      HIPCHECK(hipStreamCreateWithPriority(&s_x_, hipStreamNonBlocking, hi));
    }
    rccl_.reset();
    shm_.reset();
    cshm_.reset();
    xtimeout_ms_ = timeout_ms;
    xfailover_ = failover;
    if (kind == "rccl") {
      rccl_.reset(new cmqx::RcclXchg(arg, members, (int)d_.my_rank, timeout_ms));
      if (!counts_shm.empty()) cshm_.reset(new cmqx::ShmXchg(counts_shm, members, (int)d_.my_rank, 4096, timeout_ms));
    } else if (kind == "shm") {
      // a mailbox holds one rank's sends to every peer: records + payload
      // (+ with remote-consumer links: link delivery records, their payload and link acks,
      // as the receive side's import sizing already allows)
      size_t box = 64ull * d_.xfer_desc_max + d_.xfer_bytes + 16ull * (WORLD_MAX + 4) * 16;
      if (links_) box += 64ull * d_.deliv_max + d_.egress_cap + 16ull * d_.world * d_.lk_cap;
      shm_.reset(new cmqx::ShmXchg(arg, members, (int)d_.my_rank, box, timeout_ms));
    } else {
      throw std::runtime_error("xchg_setup: kind must be rccl or shm");
    }
    xmembers_ = members;
    xseq_ = 0;
    x_wait_ = false;
    lag_recv_.clear();
    async_x_ = async;
    if (async_x_) {
      if (!xflag_h_) {
        xflag_d_ = (u32*)alloc("xflag", 64, true);
        xflag_h_ = (u32*)buf("xflag").ptr;
      }
      __atomic_store_n(&xflag_h_[0], xjob_seq_, __ATOMIC_RELEASE);
      xth_ = std::thread([this] { x_loop(); });
    }
  }

  static py::bytes xchg_unique_id() { return py::bytes(cmqx::rccl_unique_id()); }

  // the exchange of the launched step of parity q.  0: done (launch_b imports it);
  // -2: a peer did not answer within the timeout (nothing imported, retry impossible:
  // the caller drops it and fails over).  or_flags: OR of every member's flags.
  //
  // Asynchronous (xchg_setup async=true): the step's exchange is handed
  // to the exchange thread and the call returns the PREVIOUS exchange's result (rc, flags
  // OR) -- one step later, the same on every rank, so lockstep decisions stay identical --
  // after waiting for that job, which normally finished while the last step ran.  launch_b
  // queues phase B behind a device-side wait for its job (k_xwait), so the stepper submits
  // step t+1 while step t's counts and bulk transfer are in flight.  -2 from a finished job:
  // this step is not exchanged (the caller drops it); a failed job releases its phase B
  // with nothing to import.
  int exchange(int q, u32 flags, u32* or_flags) {
    if (!native_x_ || (!rccl_ && !shm_)) throw std::runtime_error("exchange: no native exchange set up");
    if (!counts_ready_[q]) throw std::runtime_error("exchange: no phase-A step of this parity");
    if (!async_x_) {
      const int rc = exchange_now(q, flags, or_flags, -1);
      if (rc == 0) counts_ready_[q] = false;
      return rc;
    }
    HostTimer ht(&ht_[6]);
    int rc = 0;
    u32 orf = 0;
    x_collect(&rc, &orf);
    *or_flags = orf;
    if (rc) return rc;
    counts_ready_[q] = false;
    // what the next phase B (parity q^1) imports starts out as nothing: the job writes the
    // counts when it succeeds; a phase B whose wait gives up imports nothing instead of the
    // counts parity q^1 held two steps ago.  (Its last reader, step t-2, has
    // finished: its results were collected before this step's submit)
    x_recv_counts(q ^ 1, nullptr);
    std::lock_guard<std::mutex> g(xmu_);
    xq_ = q;
    xflags_ = flags;
    xseq_job_ = ++xjob_seq_;
    if (xseq_job_ == 0) xseq_job_ = ++xjob_seq_;   // (0: no wait)
    b_wait_[q ^ 1] = xseq_job_;
    xjob_ = true;
    xcv_.notify_all();
    return 0;
  }

  // the last job's result (waits for it); (0, 0) when none is uncollected
  void x_collect(int* rc, u32* orf) {
    std::unique_lock<std::mutex> g(xmu_);
    xcv_.wait(g, [&] { return !xjob_ && !xbusy_; });
    *rc = 0;
    *orf = 0;
    if (xflag_h_ && __atomic_load_n(&xflag_h_[1], __ATOMIC_ACQUIRE))
      throw std::runtime_error("a phase B gave up waiting for its exchange (exchange thread lost)");
    if (xres_) {
      *rc = xres_rc_;
      *orf = xres_orf_;
      xres_ = false;
      if (xres_rc_ == -1) throw std::runtime_error("exchange thread: " + xerr_);
    }
  }

  void x_loop() {
    HIPCHECK(hipSetDevice(device_));
    std::unique_lock<std::mutex> g(xmu_);
    while (true) {
      xcv_.wait(g, [&] { return xstop_ || xjob_; });
      if (!xjob_) return;
      const int q = xq_;
      const u32 fl = xflags_, seq = xseq_job_;
      xjob_ = false;
      xbusy_ = true;
      g.unlock();
      u32 orf = 0;
      int rc;
      std::string err;
      try {
        std::lock_guard<std::mutex> cg(cap_mu_);
        rc = exchange_now(q, fl, &orf, q ^ 1);
      } catch (const std::exception& e) {
        rc = -1;
        err = e.what();
      }
      if (rc) x_recv_counts(q ^ 1, nullptr);   // phase B imports nothing
      __atomic_store_n(&xflag_h_[0], seq, __ATOMIC_RELEASE);
      g.lock();
      xbusy_ = false;
      xres_ = true;
      xres_rc_ = rc;
      xres_orf_ = orf;
      xerr_ = err;
      xcv_.notify_all();
    }
  }

  // shutdown (abort true): a job still waiting for a peer gives up at once
  void x_stop(bool abort = false) {
    {
      std::lock_guard<std::mutex> g(xmu_);
      xstop_ = true;
      xcv_.notify_all();
      if (abort && (xjob_ || xbusy_)) {
        if (shm_) shm_->abort();
        if (cshm_) cshm_->abort();
      }
    }
    if (xth_.joinable()) xth_.join();
    std::lock_guard<std::mutex> g(xmu_);
    xstop_ = xjob_ = xbusy_ = xres_ = false;
    b_wait_[0] = b_wait_[1] = 0;
  }

  // what phase B of parity p imports: per rank [records, bytes, publish records, publish
  // bytes, link acks]; v null: nothing
  void x_recv_counts(int p, const u32* v) {
    u32* x = (u32*)buf("xchg" + std::to_string(p)).ptr;
    for (u32 r = 0; r < d_.world; ++r) {
      x[XC_RECV_N + r] = v ? v[r] : 0;
      x[XC_RECV_B + r] = v ? v[d_.world + r] : 0;
      x[XC_RECV_AN + r] = v ? v[2 * d_.world + r] : 0;
      x[XC_RECV_AB + r] = v ? v[3 * d_.world + r] : 0;
      x[XC_RACK_N + r] = v ? v[4 * d_.world + r] : 0;
    }
  }

  // dst >= 0 (exchange thread): the received counts go straight into parity dst's xchg
  // words and the RCCL bulk transfer is waited for here, not by phase B's stream
  int exchange_now(int q, u32 flags, u32* or_flags, int dst) {
    Range rg("chanamq.X1.exchange");
    HostTimer ht(&ht_[dst >= 0 ? 8 : 6]);   // (async: the exchange thread's time)
    HIPCHECK(hipEventSynchronize(ev_a_[q]));
    const u32* x = (const u32*)buf("xchg" + std::to_string(q)).ptr;
    if (x[XC_OVF]) throw std::runtime_error("cross-rank send buffers overflowed (xfer_desc_max / xfer_bytes)");
    const int n = (int)xmembers_.size();
    int me = 0;
    for (int i = 0; i < n; ++i)
      if (xmembers_[i] == (int)d_.my_rank) me = i;
    // send regions per destination rank: destination-major prefix over all ranks (k_pack_bases)
    u64 sbn[WORLD_MAX], sbb[WORLD_MAX];
    {
      u64 a = 0, b = 0;
      for (u32 r = 0; r < d_.world; ++r) { sbn[r] = a; sbb[r] = b; a += x[XC_SEND_N + r]; b += x[XC_SEND_B + r]; }
    }
    // link deliveries / acks of the step before (its phase B preceded this phase A): the
    // other parity's link buffers, destination-major (k_link_bases)
    const u32* xl = (const u32*)buf("xchg" + std::to_string(q ^ 1)).ptr;
    u64 lbn[WORLD_MAX], lbb[WORLD_MAX];
    u32 lnn[WORLD_MAX], lnb[WORLD_MAX], lnk[WORLD_MAX];
    {
      u64 a = 0, b = 0;
      for (u32 r = 0; r < d_.world; ++r) {
        lnn[r] = links_ ? xl[XC_LINK_N + r] : 0;
        lnb[r] = links_ ? xl[XC_LINK_B + r] : 0;
        lnk[r] = links_ ? std::min<u32>(xl[XC_ACK_N + r], d_.lk_cap) : 0;
        lbn[r] = a; lbb[r] = b;
        a += lnn[r]; b += lnb[r];
      }
    }
    std::vector<u32> hs((size_t)n * cmqx::XH_WORDS, 0), hr((size_t)n * cmqx::XH_WORDS, 0);
    for (int i = 0; i < n; ++i) {
      u32* h = &hs[(size_t)i * cmqx::XH_WORDS];
      const int r = xmembers_[i];
      if (i != me) {
        h[0] = x[XC_SEND_N + r]; h[1] = x[XC_SEND_B + r];
        h[2] = lnn[r]; h[3] = lnb[r]; h[4] = lnk[r];
      }
      h[5] = flags;
      h[6] = (u32)xseq_;
    }
    int rc;
    {
      Range rc_("chanamq.X1.counts");
      HostTimer hc(&ht_[7]);   // the host's blocking part: waiting for every peer's counts
      rc = cshm_ ? cshm_->counts(hs.data(), hr.data())
                 : rccl_ ? rccl_->counts(hs.data(), hr.data(), cmqx::XH_WORDS) : shm_->counts(hs.data(), hr.data());
    }
    if (rc) return rc;
    u32 orf = 0;
    for (int i = 0; i < n; ++i) {
      const u32* h = &hr[(size_t)i * cmqx::XH_WORDS];
      orf |= h[5];
      if (i != me && h[6] != (u32)xseq_)
        throw std::runtime_error("exchange out of lockstep with rank " + std::to_string(xmembers_[i]));
    }
    *or_flags = orf;
    // receive layout: sources in rank order, each [publish records | link records] and
    // [publish bytes | link bytes]
    u64 rn = 0, rb = 0, rk = 0;
    std::vector<u64> rbn(n), rbb(n), rbk(n);
    for (int i = 0; i < n; ++i) {
      const u32* h = &hr[(size_t)i * cmqx::XH_WORDS];
      rbn[i] = rn; rbb[i] = rb; rbk[i] = rk;
      if (i == me) continue;
      rn += (u64)h[0] + h[2];
      rb += (u64)h[1] + h[3];
      rk += h[4];
    }
    if (rn > d_.import_max || rb > d_.import_bytes || (rk && (!links_ || rk > (u64)d_.world * d_.lk_cap)))
      throw std::runtime_error("exchange: received records exceed the import buffers");
    u8* R_d = xr_desc_[q];
    u8* R_p = xr_pay_[q];
    const u8* S_d = xs_desc_[q];
    const u8* S_p = xs_pay_[q];
    // link buffers: sent from the other parity (step t-1), received with this exchange
    const u8* L_d = links_ ? ls_desc_[q ^ 1] : nullptr;
    const u8* L_p = links_ ? ls_pay_[q ^ 1] : nullptr;
    const u8* K_s = links_ ? lk_send_[q ^ 1] : nullptr;
    u8* RK = links_ ? rack_[q] : nullptr;
    if (rccl_) {
      std::vector<std::vector<cmqx::XPart>> snd(n), rcv(n);
      for (int i = 0; i < n; ++i) {
        if (i == me) continue;
        const int r = xmembers_[i];
        const u32* h = &hr[(size_t)i * cmqx::XH_WORDS];
        // per peer, both sides in this order: publish records, link records, publish
        // payload, link payload, link acks
        snd[i].push_back({(void*)(S_d + 64 * sbn[r]), 64ull * x[XC_SEND_N + r]});
        if (links_) snd[i].push_back({(void*)(L_d + 64 * lbn[r]), 64ull * lnn[r]});
        snd[i].push_back({(void*)(S_p + sbb[r]), (u64)x[XC_SEND_B + r]});
        if (links_) {
          snd[i].push_back({(void*)(L_p + lbb[r]), (u64)lnb[r]});
          snd[i].push_back({(void*)(K_s + 16ull * d_.lk_cap * r), 16ull * lnk[r]});
        }
        rcv[i].push_back({(void*)(R_d + 64 * rbn[i]), 64ull * h[0]});
        if (links_) rcv[i].push_back({(void*)(R_d + 64 * (rbn[i] + h[0])), 64ull * h[2]});
        rcv[i].push_back({(void*)(R_p + rbb[i]), (u64)h[1]});
        if (links_) {
          rcv[i].push_back({(void*)(R_p + rbb[i] + h[1]), (u64)h[3]});
          rcv[i].push_back({(void*)(RK + 16 * rbk[i]), 16ull * h[4]});
        }
      }
      {
        Range rb_("chanamq.X1.bulk");
        rc = rccl_->bulk(snd, rcv);
      }
      if (rc) return rc;
      if (dst < 0) x_wait_ = true;   // (stepper thread only: the exchange thread never touches it)
      if (xfailover_ || dst >= 0) {   // bounded: a peer lost mid-transfer must not wedge the compute stream
        rc = rccl_->wait(rccl_->event());
        if (rc) return rc;
      }
    } else {
      // host backend: my sends into my mailbox (destination blocks), barrier, the blocks
      // addressed to me from every source's mailbox into the receive buffers
      Range rb_("chanamq.X1.bulk_shm");
      u8* box = shm_->box(me);
      uint64_t* dir = shm_->dir(me);
      u64 off = 0;
      for (int i = 0; i < n; ++i) {
        if (i == me) continue;
        const int r = xmembers_[i];
        dir[i] = off;
        const u64 nd = 64ull * x[XC_SEND_N + r], nb = x[XC_SEND_B + r];
        const u64 ld = 64ull * lnn[r], lb = lnb[r], kb = 16ull * lnk[r];
        if (off + nd + ld + nb + 16 + lb + kb > shm_->box_bytes())
          throw std::runtime_error("exchange: shm mailbox too small");
        if (nd) HIPCHECK(hipMemcpyAsync(box + off, S_d + 64 * sbn[r], nd, hipMemcpyDeviceToHost, s_x_));
        off += nd;
        if (ld) HIPCHECK(hipMemcpyAsync(box + off, L_d + 64 * lbn[r], ld, hipMemcpyDeviceToHost, s_x_));
        off += ld;
        if (nb) HIPCHECK(hipMemcpyAsync(box + off, S_p + sbb[r], nb, hipMemcpyDeviceToHost, s_x_));
        off += (nb + 15) & ~15ull;
        if (lb) HIPCHECK(hipMemcpyAsync(box + off, L_p + lbb[r], lb, hipMemcpyDeviceToHost, s_x_));
        off += (lb + 15) & ~15ull;
        if (kb) HIPCHECK(hipMemcpyAsync(box + off, K_s + 16ull * d_.lk_cap * r, kb, hipMemcpyDeviceToHost, s_x_));
        off += kb;
      }
      HIPCHECK(hipStreamSynchronize(s_x_));
      rc = shm_->barrier();
      if (rc) return rc;
      for (int i = 0; i < n; ++i) {
        if (i == me) continue;
        const u32* h = &hr[(size_t)i * cmqx::XH_WORDS];
        const u8* src = shm_->box(i) + shm_->dir(i)[me];
        const u64 nd = 64ull * h[0], nb = h[1], ld = 64ull * h[2], lb = h[3], kb = 16ull * h[4];
        if (nd + ld) HIPCHECK(hipMemcpyAsync(R_d + 64 * rbn[i], src, nd + ld, hipMemcpyHostToDevice, s_x_));
        src += nd + ld;
        if (nb) HIPCHECK(hipMemcpyAsync(R_p + rbb[i], src, nb, hipMemcpyHostToDevice, s_x_));
        src += (nb + 15) & ~15ull;
        if (lb) HIPCHECK(hipMemcpyAsync(R_p + rbb[i] + nb, src, lb, hipMemcpyHostToDevice, s_x_));
        src += (lb + 15) & ~15ull;
        if (kb) HIPCHECK(hipMemcpyAsync(RK + 16 * rbk[i], src, kb, hipMemcpyHostToDevice, s_x_));
      }
      HIPCHECK(hipStreamSynchronize(s_x_));
    }
    // what launch_b writes into the importing step's xchg: per rank [records, bytes,
    // publish records, publish bytes].  A local vector: on the exchange thread (dst >= 0)
    // the stepper's lag_recv_ must not be touched (unsynchronised vector writes)
    std::vector<u32> recv(5 * d_.world, 0);
    for (int i = 0; i < n; ++i) {
      if (i == me) continue;
      const int r = xmembers_[i];
      const u32* h = &hr[(size_t)i * cmqx::XH_WORDS];
      recv[r] = h[0] + h[2];
      recv[d_.world + r] = h[1] + h[3];
      recv[2 * d_.world + r] = h[0];
      recv[3 * d_.world + r] = h[1];
      recv[4 * d_.world + r] = h[4];
    }
    if (dst >= 0) x_recv_counts(dst, recv.data());
    else lag_recv_.swap(recv);
    ++xseq_;
    return 0;
  }

  // the launched step of parity q will not be exchanged (it packed nothing, or a peer
  // failed): the next phase B imports nothing
  // Asynchronous, collect (the stepper): also waits for the job in flight; -2 when it
  // failed (its phase B imported nothing), which the caller handles like a failed exchange.
  // A host-run step of the control plane (collect false) leaves the stepper's uncollected
  // result alone: it carries the flags every rank acts on at the same step.
  int drop_exchange(int q, bool collect = true) {
    counts_ready_[q] = false;
    if (!async_x_) {   // (asynchronous: the exchange thread's job owns no stepper state)
      lag_recv_.clear();
      x_wait_ = false;
    }
    if (!async_x_ || !collect) return 0;
    int rc = 0;
    u32 orf = 0;
    x_collect(&rc, &orf);
    return rc;
  }

  // phase B of the launched step of parity p, importing the last exchange (if any)
  void launch_b(int p) {
    if (!b_due_[p]) throw std::runtime_error("launch_b: no phase-A step of this parity");
    b_due_[p] = false;
    if (async_x_) {   // behind its exchange job (the exchange thread writes the counts)
      const u32 w = b_wait_[p];
      b_wait_[p] = 0;
      // give up only well past every bound the job itself has (counts barrier + bulk
      // barrier + the bulk's own wait, each xtimeout_ms) plus settle: then the job is lost
      const u64 lim = ((u64)xtimeout_ms_ * 3 + 5000) * 100000ull;   // s_memrealtime: 100 MHz
      if (w) hipLaunchKernelGGL(k_xwait, dim3(1), dim3(64), 0, s_comp_, (const u32*)xflag_d_, w, xflag_d_ + 1, lim,
                                io_[p].xchg, d_.world);
      else x_recv_counts(p, nullptr);
    } else {
      x_recv_counts(p, lag_recv_.size() == 5 * d_.world ? lag_recv_.data() : nullptr);
      lag_recv_.clear();
      if (x_wait_ && rccl_) HIPCHECK(hipStreamWaitEvent(s_comp_, rccl_->event(), 0));
      x_wait_ = false;
    }
    if (graph_enabled_) {
      if (!graph_b_[p]) capture_b(p);
      HIPCHECK(hipGraphLaunch(graph_b_[p], s_comp_));
    } else {
      launch_phase_b(s_comp_, io_[p]);
    }
    HIPCHECK(hipEventRecord(ev_done_[p], s_comp_));
    gated_copy(slot_of_[p]);   // (phase B's last kernel opens the gate: sharded ranks gate too)
  }

  // ------------------------------------------------------------- native front end
  // C entry points (step_abi.h) for csrc/core/frontend.cpp: the front end's stepper
  // thread drives submit / wait_results / egress copies directly, without the GIL.  The
  // table lives as long as the Engine; the front end is stopped before the Engine dies.
  u64 c_api() {
    CmqEngineApi& a = api_;
    a.abi = CMQ_STEP_ABI;
    a.c_max = d_.c_max; a.seg_max = d_.seg_max; a.carry_cap = d_.carry_cap;
    a.persist = d_.persist; a.persist_max = d_.persist_max;
    a.ingress_cap = d_.ingress_cap; a.ctrl_cap = d_.ctrl_cap; a.carry_budget = carry_budget_;
    a.log_bytes = d_.log_bytes;
    a.eng = this;
    a.submit = [](void* e, const SegIn* sg, u32 n, const u8* pay, u64 len, i64 now, u32 worker) -> int {
      return ((Engine*)e)->guard([&] { return ((Engine*)e)->submit_raw(sg, n, (u64)pay, len, now, (u64)now, worker); });
    };
    a.prefetch = [](void* e, const u8* pay, u64 len) -> int {
      return ((Engine*)e)->guard([&] { return ((Engine*)e)->prefetch((u64)pay, len) ? 1 : 0; });
    };
    a.wait_results = [](void* e, int p) -> int {
      return ((Engine*)e)->guard([&] { ((Engine*)e)->wait_results(p); return 0; });
    };
    a.egress_slot = [](void* e, int p) -> int { return ((Engine*)e)->egress_slot(p); };
    a.egress_copy = [](void* e, int p) -> int {
      return ((Engine*)e)->guard([&] { ((Engine*)e)->egress_copy(p); return 0; });
    };
    a.egress_wait_slot = [](void* e, int slot) -> int {
      return ((Engine*)e)->guard([&] { ((Engine*)e)->egress_wait_slot(slot); return 0; });
    };
    a.error = [](void* e) -> const char* { return ((Engine*)e)->err_.c_str(); };
    a.counters = [](void* e, int p) -> const Counters* { return ((Engine*)e)->io_[p].ctr_host_h; };
    a.seg_out = [](void* e, int p) -> const SegOut* { return ((Engine*)e)->io_[p].seg_out_hh; };
    a.conn_out = [](void* e, int p) -> const ConnOut* { return ((Engine*)e)->io_[p].conn_out_hh; };
    a.ctrl_rec = [](void* e, int p) -> const CtrlRec* { return ((Engine*)e)->io_[p].ctrl_rec_hh; };
    a.ctrl = [](void* e, int p) -> const u8* { return ((Engine*)e)->io_[p].ctrl_hh; };
    a.egress_host = [](void* e, int slot) -> const u8* { return ((Engine*)e)->egress_host_[slot]; };
    a.persist_host = [](void* e, int p) -> const u8* { return ((Engine*)e)->pslot_host(p); };
    a.consumed_host = [](void* e, int p) -> const ConsumedRec* { return ((Engine*)e)->cslot_host(p); };
    a.wblock = (u32*)buf("conn_wblock").ptr;
    a.grow_host = [](void* e, int p) -> const RingMove* { return ((Engine*)e)->io_[p].grow_hh; };
    a.conn_conf = [](void* e, int p) -> const u32* { return ((Engine*)e)->io_[p].conn_conf_hh; };
    a.world = d_.world;
    a.rank = d_.my_rank;
    a.native_xchg = native_x_ ? 1u : 0u;
    a.exchange = [](void* e, int q, u32 flags, u32* orf) -> int {
      Engine* E = (Engine*)e;
      int rc = 0;
      int g = E->guard([&] { rc = E->exchange(q, flags, orf); return 0; });
      return g < 0 ? -1 : rc;
    };
    a.drop_exchange = [](void* e, int q) -> int {
      Engine* E = (Engine*)e;
      int rc = 0;
      int g = E->guard([&] { rc = E->drop_exchange(q); return 0; });
      return g < 0 ? -1 : rc;
    };
    a.launch_b = [](void* e, int p) -> int {
      return ((Engine*)e)->guard([&] { ((Engine*)e)->launch_b(p); return 0; });
    };
    a.links = links_ ? 1u : 0u;
    a.flush_submit = [](void* e, i64 now, u32 worker) -> int {
      return ((Engine*)e)->guard([&] {
        return ((Engine*)e)->submit_raw(nullptr, 0, 0, 0, now, (u64)now, worker, false, SF_NODISPATCH);
      });
    };
    a.host_register = [](void* e, void* ptr, u64 bytes) -> int {
      return ((Engine*)e)->guard([&] { HIPCHECK(hipHostRegister(ptr, bytes, hipHostRegisterDefault)); return 0; });
    };
    a.host_unregister = [](void* e, void* ptr) -> int {
      return ((Engine*)e)->guard([&] { HIPCHECK(hipHostUnregister(ptr)); return 0; });
    };
    a.egress_ready = [](void* e, int slot) -> int {
      return ((Engine*)e)->guard([&] { ((Engine*)e)->egress_ready(slot); return 0; });
    };
    a.stage_gets = [](void* e, const GetReq* r, u32 n) -> int {
      return ((Engine*)e)->guard([&] { ((Engine*)e)->stage_gets(r, n); return 0; });
    };
    a.get_out = [](void* e, int p) -> const GetOut* { return ((Engine*)e)->io_[p].get_out_hh; };
    a.host_work = [](void* e) -> int { return ((Engine*)e)->host_work() ? 1 : 0; };
    a.dl_state = [](void* e, int which) -> u64 { return ((Engine*)e)->dl_state(which); };
    a.unpaused = [](void* e, int p, const u32** out) -> u32 {
      Engine* en = (Engine*)e;
      if (p < 0 || p > 1) return 0;
      *out = en->stage_unp_[p];
      return en->nunp_[p];
    };
    a.set_egress_ref = [](void* e, int back, u32 min_bytes) -> int {
      return ((Engine*)e)->guard([&] { ((Engine*)e)->set_egress_ref(back, min_bytes); return 0; });
    };
    for (int p = 0; p < npar_; ++p) {
      std::string sfx = std::to_string(p);
      HostIO& h = io_[p];
      h.ctr_host_h = (const Counters*)buf("ctr_host" + sfx).ptr;
      h.seg_out_hh = (const SegOut*)buf("seg_out" + sfx).ptr;
      h.conn_out_hh = (const ConnOut*)buf("conn_out" + sfx).ptr;
      h.ctrl_rec_hh = (const CtrlRec*)buf("ctrl_rec" + sfx).ptr;
      h.ctrl_hh = (const u8*)buf("ctrl" + sfx).ptr;
      h.grow_hh = (const RingMove*)buf("grow" + sfx).ptr;
      h.conn_conf_hh = (const u32*)buf("conn_conf" + sfx).ptr;
      h.get_out_hh = (const GetOut*)buf("get_out" + sfx).ptr;
    }
    return (u64)&api_;
  }

  template <class F>
  int guard(F&& f) {
    try {
      HIPCHECK(hipSetDevice(device_));   // the caller may be any host thread
      return f();
    } catch (std::exception& ex) {
      err_ = ex.what();
      return -1;
    }
  }

  // egress_wait_slot without touching engine state (any thread; the slot's D2H was
  // issued before the caller learnt of the slot)
  void egress_ready(int e) {
    if (copy_mode_ == 3) {
      if (sdma_pending_[e]) bounded_wait(sdma_sig_[e], e, "egress D2H");
      if (tail_pending_[e]) bounded_wait(tail_sig_[e], e, "egress tail D2H");
      return;
    }
    if (d2h_issued_[e]) HIPCHECK(hipEventSynchronize(ev_d2h_[e]));
  }

  void egress_wait_slot(int e) {
    HostTimer ht(&ht_[5]);
    if (copy_mode_ == 3) { sdma_wait(e); return; }
    if (d2h_issued_[e]) HIPCHECK(hipEventSynchronize(ev_d2h_[e]));
  }

  // the egress D2H of slot e, queued now: starts when the step's last kernel opens the gate
  void gated_copy(int e) {
    if (!spec_[e]) return;
    Range rg("chanamq.K5.egress_gated");
    // sdma_split 2: the speculative copy in two halves on two SDMA engines, both released by
    // the same gate, each decrementing the slot's completion signal once
    const u64 n = spec_[e];
    const int k = (sdma_split_ > 1 && sdma_engine2_ && n >= (4u << 20)) ? 2 : 1;
    const u64 half = k == 2 ? ((n / 2) & ~(u64)4095) : n;
    hsa_signal_store_screlease(sdma_sig_[e], k);
    for (int i = 0; i < k; ++i) {
      const u64 off = i ? half : 0, len = i ? n - half : half;
      hsa_status_t st = hsa_amd_memory_async_copy_on_engine((u8*)egress_host_[e] + off, cpu_agent_,
                                                            (u8*)egress_dev_[e] + off, gpu_agent_, len, 1,
                                                            &gate_sig_[e], sdma_sig_[e],
                                                            i ? sdma_engine2_ : sdma_engine_, true);
      if (st != HSA_STATUS_SUCCESS) {
        hsa_signal_store_screlease(sdma_sig_[e], 0);
        throw std::runtime_error("hsa_amd_memory_async_copy_on_engine (gated egress) failed");
      }
    }
    sdma_pending_[e] = true;
    ++eg_stats_[0];
    eg_stats_[2] += spec_[e];
  }

  // non-blocking: the launched step of parity p has finished (its results are readable)
  bool step_done(int p) {
    if (!inflight_[p] || staged_[p] || phase_a_[p] || b_due_[p]) return !inflight_[p];
    return hipEventQuery(ev_done_[p]) == hipSuccess;
  }
  // non-blocking: egress slot e's D2H (and tail) landed in host memory
  bool egress_done_slot(int e) {
    if (copy_mode_ == 3) {
      if (sdma_pending_[e] && hsa_signal_load_scacquire(sdma_sig_[e]) != 0) return false;
      if (tail_pending_[e] && hsa_signal_load_scacquire(tail_sig_[e]) != 0) return false;
      sdma_pending_[e] = tail_pending_[e] = false;
      return true;
    }
    return !d2h_issued_[e] || hipEventQuery(ev_d2h_[e]) == hipSuccess;
  }

  void wait_results(int p) {
    HostTimer ht(&ht_[3]);
    Range rg("chanamq.step.wait_results");
    if (phase_a_[p] || b_due_[p]) throw std::runtime_error("wait_results: phase B of this sharded step not submitted");
    if (staged_[p]) throw std::runtime_error("wait_results: step staged but never launched");
    HIPCHECK(hipEventSynchronize(ev_done_[p]));
    inflight_[p] = false;
    if (h2d_addr_[p]) {   // (k_h2d_wait gives up after its poll budget: the step then ran on a stale slot)
      if (*(volatile const i64*)h2d_addr_[p] != 0 || (h2d_addr2_[p] && *(volatile const i64*)h2d_addr2_[p] != 0)) {
        wait_failed_ = true;
        throw std::runtime_error("ingress copy of step " + std::to_string(launch_seq_[p]) +
                                 " did not complete before its step ran (HSA SDMA copy lost)");
      }
    }
    // egress history of the gated copies' sizing (every finished step, idle ones too)
    const u64 n = ((const Counters*)buf("ctr_host" + std::to_string(p)).ptr)->egress_bytes;
    eg_hist_[eg_hist_i_++ & 3] = n;
    eg_stats_[3] += n;
  }

  u64 egress_copy(int p) {
    HostTimer ht(&ht_[4]);
    Range rg("chanamq.K5.egress_d2h");
    const Counters* c = (const Counters*)buf("ctr_host" + std::to_string(p)).ptr;
    u64 n = c->egress_bytes;
    const int e = slot_of_[p];
    if (spec_[e]) {   // gated: the bulk is on its way already; the host only adds a tail
      if (n > spec_[e]) {
        const u64 off = spec_[e];
        hsa_signal_store_screlease(tail_sig_[e], 1);
        hsa_status_t st = hsa_amd_memory_async_copy_on_engine((u8*)egress_host_[e] + off, cpu_agent_,
                                                              (u8*)egress_dev_[e] + off, gpu_agent_, n - off, 0, nullptr,
                                                              tail_sig_[e], tail_engine_, true);
        if (st != HSA_STATUS_SUCCESS) {
          hsa_signal_store_screlease(tail_sig_[e], 0);
          throw std::runtime_error("hsa_amd_memory_async_copy_on_engine (egress tail) failed");
        }
        tail_pending_[e] = true;
        ++eg_stats_[1];
      }
      return n;
    }
    if (eager_d2h_[p]) {   // already queued behind the step (launch)
      eager_d2h_[p] = false;
      return n;
    }
    HIPCHECK(hipStreamWaitEvent(s_d2h_, ev_done_[p], 0));
    if (n && copy_mode_ == 3) {
      HIPCHECK(hipEventSynchronize(ev_done_[p]));
      // sdma_split 2: large egress split over two SDMA engines, each part decrementing the
      // slot's signal once (measured slower on MI355X: 28.9 vs 38.6 M msgs/s, p99 6.6 ms,
      // profiles/r4_sdma_split.md -- off by default)
      const int k = (n >= (2u << 20) && sdma_engine2_) ? 2 : 1;
      hsa_signal_store_screlease(sdma_sig_[e], k);
      const u64 half = k == 2 ? ((n / 2) & ~(u64)4095) : n;
      for (int i = 0; i < k; ++i) {
        const u64 off = i ? half : 0, len = i ? n - half : half;
        hsa_status_t st = hsa_amd_memory_async_copy_on_engine(
            (u8*)egress_host_[e] + off, cpu_agent_, (u8*)egress_dev_[e] + off, gpu_agent_, len, 0, nullptr,
            sdma_sig_[e], i ? sdma_engine2_ : sdma_engine_, true);
        if (st != HSA_STATUS_SUCCESS) throw std::runtime_error("hsa_amd_memory_async_copy_on_engine failed");
      }
      sdma_pending_[e] = true;
      return n;
    }
    if (n && copy_mode_ == 2)
      hipLaunchKernelGGL(k_copy_out, dim3(copy_wgs_), dim3(256), 0, s_d2h_, egress_host_dev_[e],
                         (const u8*)egress_dev_[e], n);
    else if (n)
      HIPCHECK(hipMemcpyAsync(egress_host_[e], egress_dev_[e], n,
                              sdma_ ? hipMemcpyDeviceToDeviceNoCU : hipMemcpyDeviceToHost, s_d2h_));
    HIPCHECK(hipEventRecord(ev_d2h_[e], s_d2h_));
    d2h_issued_[e] = true;
    return n;
  }

  void egress_wait(int p) {
    HostTimer ht(&ht_[5]);
    const int e = slot_of_[p];
    if (copy_mode_ == 3) { sdma_wait(e); return; }
    HIPCHECK(hipEventSynchronize(ev_d2h_[e]));
  }

  // the slot's D2H (+ its tail) complete
  void sdma_wait(int e) {
    if (sdma_pending_[e]) bounded_wait(sdma_sig_[e], e, "egress D2H");
    if (tail_pending_[e]) bounded_wait(tail_sig_[e], e, "egress tail D2H");
    sdma_pending_[e] = false;
    tail_pending_[e] = false;
  }

  // a copy's completion signal reaching 0: an active spin first (a step's egress lands
  // within its period; a blocked wait would add the interrupt wake-up to every delivery's
  // latency), then blocked waits up to the engine's wait deadline -- past it the copy is
  // declared lost: the slot's gate is opened (a gated copy that never saw its step's last
  // kernel would otherwise hold its SDMA queue forever) and the engine reports an error
  // (the front end's healthy() turns false, a sharded node fails over).  Was: an unbounded
  // active wait, a core spinning forever on a lost gate
  void bounded_wait(hsa_signal_t sig, int e, const char* what) {
    if (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_EQ, 0, spin_ticks_, HSA_WAIT_STATE_ACTIVE) == 0) return;
    const auto t0 = std::chrono::steady_clock::now();
    while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_EQ, 0, block_ticks_, HSA_WAIT_STATE_BLOCKED) != 0) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(wait_ms_)) {
        if (e >= 0 && gate_sig_[e].handle) hsa_signal_store_screlease(gate_sig_[e], 0);
        wait_failed_ = true;
        throw std::runtime_error(std::string(what) + " of egress slot " + std::to_string(e) + " did not complete within " +
                                 std::to_string(wait_ms_) + " ms (gate never opened / copy lost)");
      }
    }
  }
  // fault injection (tests): the next submitted step's egress gate is never opened by its
  // last kernel (it stores to a scratch word instead), as after a step that died before it
  void inject_gate_fault() { gate_fault_ = true; }
  // (tests) the next step's ingress wait polls a word that never reaches 0 (HSA ingress only)
  void inject_h2d_fault() { h2d_fault_ = true; }
  bool wait_failed() const { return wait_failed_; }

  // gated egress: bytes to copy speculatively for the next step -- the largest of the last
  // four steps' egress + 1/16 + 64 KB, in 64 KB units (0 after four steps without egress)
  u64 spec_bytes() const {
    u64 mx = 0;
    for (u64 v : eg_hist_) mx = v > mx ? v : mx;
    if (!mx) return 0;
    const u64 sz = (mx + mx / 16 + (64u << 10) + 65535) & ~(u64)65535;
    return sz < egress_alloc_ ? sz : egress_alloc_;
  }
  // gated egress counters: [gated copies, tail copies, bytes copied speculatively, bytes rendered]
  py::dict egress_stats() const {
    py::dict o;
    o["gated"] = gated_;
    o["gated_copies"] = eg_stats_[0];
    o["tail_copies"] = eg_stats_[1];
    o["spec_bytes"] = eg_stats_[2];
    o["egress_bytes"] = eg_stats_[3];
    return o;
  }

  // egress slot (host view "egress_host<slot>") of the step last submitted with parity p
  int egress_slot(int p) const { return slot_of_[p]; }
  // egress by reference from the next submitted step on (StepIn.ref_back): bodies of the
  // last `back` steps' ingress payloads (-1: off; -2: only bodies in the host spill ring) of
  // at least min_bytes are not rendered;
  // the caller keeps those payloads unchanged until the delivering step's egress is sent
  void set_egress_ref(int back, u32 min_bytes) {
    if (back > 64) throw std::runtime_error("set_egress_ref: at most 64 steps back");
    ref_back_ = back == -2 ? -2 : back < 0 ? -1 : back;
    ref_min_ = min_bytes < 16 ? 16 : min_bytes;
  }
  // store-record slot (host views "persist<slot>" / "consumed<slot>") of that step
  int persist_slot(int p) const { return pslot_of_[p]; }
  const u8* pslot_host(int p) {
    return d_.persist ? (const u8*)buf("persist" + std::to_string(pslot_of_[p])).ptr : nullptr;
  }
  const ConsumedRec* cslot_host(int p) {
    return d_.persist ? (const ConsumedRec*)buf("consumed" + std::to_string(pslot_of_[p])).ptr : nullptr;
  }

  // HSA agents of this device and of the host, an SDMA engine for GPU -> host copies
  void init_sdma() {
    if (hsa_init() != HSA_STATUS_SUCCESS) throw std::runtime_error("hsa_init failed");
    struct Ctx { std::vector<hsa_agent_t> gpus, cpus; } ctx;
    hsa_iterate_agents([](hsa_agent_t a, void* data) {
      hsa_device_type_t t;
      hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
      auto* c = (Ctx*)data;
      if (t == HSA_DEVICE_TYPE_GPU) c->gpus.push_back(a);
      else if (t == HSA_DEVICE_TYPE_CPU) c->cpus.push_back(a);
      return HSA_STATUS_SUCCESS;
    }, &ctx);
    if ((int)ctx.gpus.size() <= device_ || ctx.cpus.empty()) throw std::runtime_error("HSA agents not found");
    {   // bounded_wait: spin 2 ms actively, then block in 1 ms slices
      u64 f = 0;
      if (hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &f) != HSA_STATUS_SUCCESS || !f) f = 100000000ull;
      spin_ticks_ = f / 500;
      block_ticks_ = f / 1000;
    }
    gpu_agent_ = ctx.gpus[device_];
    cpu_agent_ = ctx.cpus[0];
    uint32_t mask = 0;
    if (hsa_amd_memory_copy_engine_status(cpu_agent_, gpu_agent_, &mask) != HSA_STATUS_SUCCESS || !mask)
      throw std::runtime_error("no SDMA engine available for device -> host copies");
    // not the engine of the runtime's own H2D copies: one SDMA engine serialises both
    // directions (measured 54 GB/s total vs 94 GB/s on two engines, bench/pcie_probe.hip)
    // (measured on MI355X: engines 0-3 reach PCIe rate, 8 and 15 a third of it)
    u32 pick = 0;
    if (sdma_pref_ >= 0 && (mask >> sdma_pref_) & 1u) pick = (u32)sdma_pref_;
    else if ((mask >> 1) & 1u) pick = 1;
    else while (!((mask >> pick) & 1u)) ++pick;
    sdma_engine_ = (hsa_amd_sdma_engine_id_t)(1u << pick);
    // a second engine for split egress copies: another full-rate one (0-3), not engine 0
    // (the runtime's H2D engine) when there is a choice
    sdma_engine2_ = (hsa_amd_sdma_engine_id_t)0;
    if (sdma_split_ > 1)
      for (u32 c : {2u, 3u, 0u})
        if (c != pick && ((mask >> c) & 1u)) { sdma_engine2_ = (hsa_amd_sdma_engine_id_t)(1u << c); break; }
    // the tail engine (gated egress): another full-rate engine than the gated copies' --
    // which can sit behind the next step's gate -- and than the runtime's H2D engine 0
    // (nor the split copies' second engine: an engine's queue is in order, and a gated copy
    // waiting there for the next step's gate would hold the tail back by a step)
    tail_engine_ = sdma_engine_;
    for (u32 c : {2u, 3u, 0u})
      if (c != pick && ((mask >> c) & 1u) && (1u << c) != (u32)sdma_engine2_) {
        tail_engine_ = (hsa_amd_sdma_engine_id_t)(1u << c);
        break;
      }
    // the ingress engine (cfg h2d_hsa): engine 0, the runtime's own H2D engine -- the egress
    // engines stay free of it (measured: egress on engine 0 next to the ingress copies halves
    // the throughput, profiles/r6_x); else any full-rate engine the egress does not use
    ing_engine_ = (hsa_amd_sdma_engine_id_t)0;
    for (u32 c : {0u, 3u, 2u, 1u})
      if (((mask >> c) & 1u) && (1u << c) != (u32)sdma_engine_ && (1u << c) != (u32)sdma_engine2_ &&
          (1u << c) != (u32)tail_engine_) {
        ing_engine_ = (hsa_amd_sdma_engine_id_t)(1u << c);
        break;
      }
    if (!ing_engine_) ing_engine_ = tail_engine_;
    // a split payload's second engine (cfg h2d_split, default off): another full-rate one the
    // egress does not use
    ing_engine2_ = (hsa_amd_sdma_engine_id_t)0;
    if (h2d_split_cfg_)
      for (u32 c : {3u, 2u})
        if (((mask >> c) & 1u) && (1u << c) != (u32)ing_engine_ && (1u << c) != (u32)sdma_engine_ &&
            (1u << c) != (u32)sdma_engine2_ && (1u << c) != (u32)tail_engine_) {
          ing_engine2_ = (hsa_amd_sdma_engine_id_t)(1u << c);
          break;
        }
    for (int e = 0; e < EGRESS_SLOTS; ++e)
      if (hsa_signal_create(0, 0, nullptr, &sdma_sig_[e]) != HSA_STATUS_SUCCESS ||
          hsa_signal_create(0, 0, nullptr, &tail_sig_[e]) != HSA_STATUS_SUCCESS ||
          hsa_signal_create(0, 0, nullptr, &gate_sig_[e]) != HSA_STATUS_SUCCESS)
        throw std::runtime_error("hsa_signal_create failed");
  }

  void drain_egress() {
    for (int e = 0; e < EGRESS_SLOTS; ++e) {
      sdma_wait(e);
      if (d2h_issued_[e]) HIPCHECK(hipEventSynchronize(ev_d2h_[e]));
    }
  }

  void sync() {
    HIPCHECK(hipStreamSynchronize(s_h2d_));
    if (s_h2d_alt_) HIPCHECK(hipStreamSynchronize(s_h2d_alt_));
    HIPCHECK(hipStreamSynchronize(s_pre_));
    HIPCHECK(hipStreamSynchronize(s_ing_));
    HIPCHECK(hipStreamSynchronize(s_comp_));
    HIPCHECK(hipStreamSynchronize(s_d2h_));
  }

  // seconds spent in each host phase since the last reset
  py::dict host_times(bool reset) {
    // (asynchronous exchange: "exchange" is the stepper's wait for the previous job,
    // "exchange_thread" and "exchange_counts" the exchange thread's time)
    static const char* names[9] = {"submit", "submit_sdma_wait", "submit_graph_launch", "wait_results",
                                   "egress_copy", "egress_wait", "exchange", "exchange_counts", "exchange_thread"};
    py::dict o;
    for (int i = 0; i < 9; ++i) { o[names[i]] = ht_[i]; if (reset) ht_[i] = 0; }
    return o;
  }

  py::dict counters(int p) const {
    const Counters& c = *(const Counters*)buf("ctr_host" + std::to_string(p)).ptr;
    py::dict o;
#define F(x) o[#x] = c.x
    F(n_cmds); F(n_frags); F(n_pubs); F(n_acks); F(n_ctrl); F(ctrl_bytes); F(n_pairs); F(n_deliv);
    F(egress_bytes); F(n_returns); F(n_confirm_frames); F(n_freed); F(n_requeue); F(n_unroutable);
    F(n_dropped_nomem); F(n_expired); F(n_routed_msgs); F(n_unknown_exchange); F(n_ring_full);
    F(n_acked); F(log_head); F(log_tail); F(msg_free_top); F(n_live_msgs);
    F(n_persist); F(n_consumed); F(persist_used); F(n_persist_overflow);
    F(live_bytes); F(n_grow); F(n_dget); F(spill_moved); F(n_ref); F(gath_off); F(ref_bytes);
#undef F
    std::vector<u32> lat(c.lat_hist, c.lat_hist + LAT_BINS);
    o["lat_hist"] = lat;
    return o;
  }

 private:
  static ScanArgs scan_args(std::initializer_list<std::pair<const u32*, u32*>> arrs, const u32* n, u32 nmax,
                            u32 slot, const u32* lo) {
    if (arrs.size() > 4) throw std::runtime_error("launch_scan: at most 4 arrays");
    ScanArgs a{};
    a.lo = lo;
    u32 k = 0;
    for (auto& p : arrs) { a.in[k] = p.first; a.out[k] = p.second; ++k; }
    a.narr = k;
    a.n = n;
    a.nmax = nmax;
    a.tot_slot = slot;
    return a;
  }
  void launch_scan(hipStream_t s, const DS& d, std::initializer_list<std::pair<const u32*, u32*>> arrs, const u32* n,
                   u32 nmax, u32 slot, const u32* lo = nullptr, bool ingest = false) {
    const ScanArgs a = scan_args(arrs, n, nmax, slot, lo);
    u32 nb = ceil_div(nmax ? nmax : 1, SCAN_TILE);
    hipLaunchKernelGGL((k_scan<4, 4>), dim3(nb), dim3(1024), 0, s, a, d.tot, ingest ? scan_status_ing_ : scan_status_,
                       ingest ? scan_ctl_ing_ : scan_ctl_, scan_smax_);
  }
  // returns index (0/1) of the buffer holding the sorted output
  u32 radix_sort(hipStream_t s, const DS& d, u32** keys, u32** vals, const u32* n, u32 nmax, u32 bits) {
    u32 ntiles = ceil_div(nmax, SORT_TILE);
    if (bits > 8 && bits <= 11) {   // one 9..11-bit pass instead of two 8-bit ones
      if (bits == 9) {
        hipLaunchKernelGGL(k_rs_hist<9>, capped(ntiles, 256), dim3(RsNt<9>::v), 0, s, keys[0], n, 0u, d_.hist,
                           d_.hist_scan, &d.tot[TS_RS_TICKET], ntiles);
        hipLaunchKernelGGL(k_rs_scatter<9>, capped(ntiles, 256), dim3(256), 0, s, keys[0], vals[0], keys[1], vals[1], n,
                           0u, d_.hist_scan, ntiles);
      } else if (bits == 10) {
        hipLaunchKernelGGL(k_rs_hist<10>, capped(ntiles, 256), dim3(RsNt<10>::v), 0, s, keys[0], n, 0u, d_.hist,
                           d_.hist_scan, &d.tot[TS_RS_TICKET], ntiles);
        hipLaunchKernelGGL(k_rs_scatter<10>, capped(ntiles, 256), dim3(256), 0, s, keys[0], vals[0], keys[1], vals[1],
                           n, 0u, d_.hist_scan, ntiles);
      } else {
        hipLaunchKernelGGL(k_rs_hist<11>, capped(ntiles, 256), dim3(RsNt<11>::v), 0, s, keys[0], n, 0u, d_.hist,
                           d_.hist_scan, &d.tot[TS_RS_TICKET], ntiles);
        hipLaunchKernelGGL(k_rs_scatter<11>, capped(ntiles, 256), dim3(256), 0, s, keys[0], vals[0], keys[1], vals[1],
                           n, 0u, d_.hist_scan, ntiles);
      }
      return 1;
    }
    u32 src = 0;
    for (u32 shift = 0; shift < bits; shift += 8) {
      hipLaunchKernelGGL(k_rs_hist<8>, capped(ntiles, 256), dim3(RsNt<8>::v), 0, s, keys[src], n, shift, d_.hist, d_.hist_scan,
                         &d.tot[TS_RS_TICKET], ntiles);
      hipLaunchKernelGGL(k_rs_scatter<8>, capped(ntiles, 256), dim3(256), 0, s, keys[src], vals[src], keys[src ^ 1],
                         vals[src ^ 1], n, shift, d_.hist_scan, ntiles);
      src ^= 1;
    }
    return src;
  }

  static dim3 blocks(u64 n, u32 per) { return dim3(n ? ceil_div(n, per) : 1); }
  // wave-per-item grid-stride kernels: 4 waves per block, at most 8192 blocks
  // wave-per-item grid-stride kernels: 4 waves per block, at most 8192 blocks.  Grids are
  // fixed at graph capture, sized for capacity; the cap keeps a step with a fraction of
  // the capacity from launching (and retiring) 100K+ idle waves, while still giving the
  // latency-bound per-item chains (route, store, render) one wave per item at the usual
  // step sizes (measured: a 2048-block cap made k_route / k_route_store / k_render slower)
  static dim3 wave_blocks(u64 n) { u64 b = n ? ceil_div(n, 4) : 1; return dim3(b > 8192 ? 8192 : (u32)b); }
  static dim3 capped(u64 b, u32 cap) { return dim3(b == 0 ? 1u : (b > cap ? cap : (u32)b)); }

  // frame scan, command assembly, decode (K1-K5)
  void launch_ingest(hipStream_t s, const DS& d) {
    Range rg("chanamq.K1-K4.ingest");
    hipLaunchKernelGGL(k_stage, dim3(1), dim3(1024), 0, s, d);
    if (h2d_hsa_) hipLaunchKernelGGL(k_h2d_wait, dim3(16), dim3(64), 0, s, d);
    // one block per CU fits (154 KB of LDS): more blocks than CUs only queue behind the
    // busy ones, and blocks past the step's segments would still be dispatched one by one
    // after them (the grid is sized for capacity at capture)
    hipLaunchKernelGGL(k_frame_scan, capped(d.seg_max, n_cu_), dim3(FS_NT), 0, s, d);
    if (d.rank_scan)
      launch_scan(s, d, {{d.cmd_is_pub, d.cmd_pub_rank}, {d.cmd_is_ack, d.cmd_ack_rank}}, &d.ctr->n_cmds,
                  d.cmd_max, 4, nullptr, /*ingest=*/true);
    hipLaunchKernelGGL(k_decode, blocks(d.cmd_max, 256), dim3(256), 0, s, d);
  }

  // route + store the publishes of the current phase range (K6); nmax = range capacity.
  // imports: phase B's import + routing pass 0 kernel (k_import_route) instead of k_route
  void launch_route(hipStream_t s, const DS& d, u32 nmax, bool imports = false) {
    Range rg("chanamq.K6-K13.route_store");
    // 16 publishes per block, grid-stride; the grid is the blocks that can be resident
    // (k_route: 2 per CU at 64 VGPRs; k_import_route: 1), not the capacity's groups --
    // the idle blocks of a capacity-sized grid were still dispatched after the busy ones
    const u64 ngroups = ceil_div(nmax ? nmax : 1, 16);
    if (imports) hipLaunchKernelGGL(k_import_route, capped(ngroups, n_cu_), dim3(1024), 0, s, d);   // + prep, link acks
    else hipLaunchKernelGGL(k_route, capped(ngroups, 2 * n_cu_), dim3(1024), 0, s, d);
    // scan of the routing counts + the phase's log reservation, then pairs + store
    const ScanArgs a = scan_args({{d.pub_nq, d.pub_pair_off}, {d.pub_slot, d.pub_slot_off},
                                  {d.pub_routed, d.pub_routed_rank}, {d.pub_ret_sz, d.pub_ret_off}},
                                 &d.tot[TS_RANGE_HI], d.pub_cap, 0, &d.tot[TS_RANGE_LO]);
    hipLaunchKernelGGL(k_scan_route, dim3(ceil_div(d.pub_cap ? d.pub_cap : 1, SCAN_TILE)), dim3(1024), 0, s, a, d.tot,
                       scan_status_, scan_ctl_, scan_smax_, d);
    hipLaunchKernelGGL(k_route_store, wave_blocks(nmax), dim3(256), 0, s, d, imports ? 0u : 1u);
  }

  // serialise publishes with remote owners into the per-destination send buffers
  void launch_pack(hipStream_t s, const DS& d) {
    Range rg("chanamq.X1.pack");
    // per destination rank: record and byte offsets of every publish (one pass, all
    // ranks); k_pack derives the destination bases itself and serialises
    hipLaunchKernelGGL(k_pack_scan, blocks(d.pub_max, PK_TILE), dim3(1024), 0, s, d, d.pk_agg, &d.tot[TS_PK_TICKET]);
    hipLaunchKernelGGL(k_pack, wave_blocks(d.pub_max), dim3(256), 0, s, d);
  }

  // enqueue, acks, dispatch, render (K7-K11)
  // dispatch = false (restore): enqueue only; nothing is delivered or rendered between
  // steps (the restored messages go out with the next step's dispatch)
  void launch_tail(hipStream_t s, const DS& d, bool dispatch = true) {
    Range rg("chanamq.K7-K11.tail");
    u32 nch = d.c_max * d.chpc;
    const u32 pbits = d.q_bits + d.rank_bits;
    if (pbits <= 11) {
      // single-pass sort with the ring plan folded into the histogram's last block and the
      // enqueue into the scatter (k_rs_hist_plan / k_rs_scatter_enq): two launches
      const u32 nt = ceil_div(d.pair_max, SORT_TILE);
      const u32* n = &d.tot[TS_PAIR_N];
      u32* tk = &d.tot[TS_RS_TICKET];
      if (pbits <= 8) {
        hipLaunchKernelGGL(k_rs_hist_plan<8>, capped(nt, 256), dim3(RsNt<8>::v), 0, s, d, d.pair_k[0], n, d_.hist, d_.hist_scan, tk, nt);
        hipLaunchKernelGGL(k_rs_scatter_enq<8>, capped(nt, 256), dim3(256), 0, s, d, d.pair_k[0], d.pair_v[0], n, d_.hist_scan);
      } else if (pbits == 9) {
        hipLaunchKernelGGL(k_rs_hist_plan<9>, capped(nt, 256), dim3(RsNt<9>::v), 0, s, d, d.pair_k[0], n, d_.hist, d_.hist_scan, tk, nt);
        hipLaunchKernelGGL(k_rs_scatter_enq<9>, capped(nt, 256), dim3(256), 0, s, d, d.pair_k[0], d.pair_v[0], n, d_.hist_scan);
      } else if (pbits == 10) {
        hipLaunchKernelGGL(k_rs_hist_plan<10>, capped(nt, 256), dim3(RsNt<10>::v), 0, s, d, d.pair_k[0], n, d_.hist, d_.hist_scan, tk, nt);
        hipLaunchKernelGGL(k_rs_scatter_enq<10>, capped(nt, 256), dim3(256), 0, s, d, d.pair_k[0], d.pair_v[0], n, d_.hist_scan);
      } else {
        hipLaunchKernelGGL(k_rs_hist_plan<11>, capped(nt, 256), dim3(RsNt<11>::v), 0, s, d, d.pair_k[0], n, d_.hist, d_.hist_scan, tk, nt);
        hipLaunchKernelGGL(k_rs_scatter_enq<11>, capped(nt, 256), dim3(256), 0, s, d, d.pair_k[0], d.pair_v[0], n, d_.hist_scan);
      }
    } else {
      u32* pk[2] = {d.pair_k[0], d.pair_k[1]};
      u32* pv[2] = {d.pair_v[0], d.pair_v[1]};
      const u32 psrc = radix_sort(s, d, pk, pv, &d.tot[TS_PAIR_N], d.pair_max, pbits);
      hipLaunchKernelGGL(k_qfirst, blocks(d.pair_max, 256), dim3(256), 0, s, d, psrc);
      hipLaunchKernelGGL(k_ring_plan, capped(ceil_div(d.pair_max, 256), 1024), dim3(256), 0, s, d, psrc, 0u);
      hipLaunchKernelGGL(k_enqueue, capped(ceil_div(d.pair_max, 256), 1024), dim3(256), 0, s, d, psrc, 0u);
    }
    // without persistence nothing runs after k_post: it also writes the host-visible
    // outputs and its last block the counters (fused k_host_out)
    const u32 fin = d.persist ? 0u : 1u;
    if (!dispatch) {
      const u64 pn = d.deliv_max > d.c_max ? d.deliv_max : d.c_max;
      hipLaunchKernelGGL(k_post, blocks(pn, 256), dim3(256), 0, s, d, fin);   // n_deliv = 0: frees only
      if (!fin) hipLaunchKernelGGL(k_host_out, dim3(64), dim3(256), 0, s, d);
      return;
    }
    hipLaunchKernelGGL(k_chan_advance, capped(nch, 1024), dim3(256), 0, s, d);
    // k_dequeue first puts requeued deliveries back in front of their queues' heads, in
    // queue-offset order (QueueEntity.scala:415-446), then dispatches
    hipLaunchKernelGGL(k_dequeue, dim3(d.q_max), dim3(256), 0, s, d);   // (its last block: k_runs)
    hipLaunchKernelGGL(k_dv_write, blocks(d.deliv_max, 256), dim3(256), 0, s, d);
    if (d.c_max <= CONN_LAYOUT_MAX) {
      hipLaunchKernelGGL(k_conn_layout, dim3(1), dim3(1024), 0, s, d);   // + the delivery-size scan
    } else {
      launch_scan(s, d, {{d.dv_size, d.dv_off}}, &d.ctr->n_deliv, d.deliv_max, 6);
      hipLaunchKernelGGL(k_conn_sizes, blocks(d.c_max, 256), dim3(256), 0, s, d);
      launch_scan(s, d, {{d.conn_total, d.conn_base}}, nullptr, d.c_max, 7);
      hipLaunchKernelGGL(k_conn_out, blocks(d.c_max, 256), dim3(256), 0, s, d);
    }
    if (d.links) hipLaunchKernelGGL(k_link_bases, dim3(1), dim3(64), 0, s, d);
    {
      const u32 n_rc = RC_RET_BLOCKS + ceil_div(d.c_max, 256);
      hipLaunchKernelGGL(k_render, dim3(n_rc + wave_blocks(d.deliv_max).x), dim3(256), 0, s, d, n_rc);
    }
    u64 pn = d.deliv_max > d.c_max ? d.deliv_max : d.c_max;
    hipLaunchKernelGGL(k_post, blocks(pn, 256), dim3(256), 0, s, d, fin);
    if (d.persist) {
      hipLaunchKernelGGL(k_persist_size, blocks(d.persist_max, 256), dim3(256), 0, s, d);
      launch_scan(s, d, {{d.ps_size, d.ps_off}}, &d.ctr->n_persist, d.persist_max, TS_PERSIST);
      hipLaunchKernelGGL(k_persist_pack, wave_blocks(d.persist_max), dim3(256), 0, s, d);
      hipLaunchKernelGGL(k_host_out, dim3(64), dim3(256), 0, s, d);
    }
  }

  // world == 1: the whole step; world > 1: phase A (ingest, local route, pack)
  void launch_main(hipStream_t s, const DS& d) {
    launch_ingest(s, d);
    launch_route(s, d, d.pub_max);   // (+ the K9 marks / K10 confirm counts: k_route_store)
    if (d.world > 1) launch_pack(s, d);
    else launch_tail(s, d);
  }

  // world == 1 with overlap: the routing / delivery half of the step (the step's acks /
  // nacks / rejects are marked and its confirms counted in it -- k_route_store, phase 0 --
  // never in the ingest half, so an overlapped ingest never touches delivery-side state)
  void launch_rest(hipStream_t s, const DS& d) {
    launch_route(s, d, d.pub_max);
    launch_tail(s, d);
  }
  void capture_on(hipStream_t st, hipGraphExec_t* ge, const std::function<void()>& f) {
    hipGraph_t g;
    std::lock_guard<std::mutex> cg(cap_mu_);   // (no exchange-thread HIP call inside a capture)
    HIPCHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    f();
    HIPCHECK(hipStreamEndCapture(st, &g));
    HIPCHECK(hipGraphInstantiate(ge, g, nullptr, nullptr, 0));
    HIPCHECK(hipGraphDestroy(g));
  }

  // world > 1, after the all-to-all: import, route against local queues, rest of the step
  void launch_phase_b(hipStream_t s, const DS& d, bool dispatch = true) {
    Range rg("chanamq.X1.import");
    launch_route(s, d, d.import_max, /*imports=*/true);
    launch_tail(s, d, dispatch);
  }

  void capture_main(int p) {
    hipGraph_t g;
    std::lock_guard<std::mutex> cg(cap_mu_);   // (no exchange-thread HIP call inside a capture)
    HIPCHECK(hipStreamBeginCapture(s_comp_, hipStreamCaptureModeThreadLocal));
    launch_main(s_comp_, io_[p]);
    HIPCHECK(hipStreamEndCapture(s_comp_, &g));
    HIPCHECK(hipGraphInstantiate(&graph_exec_[p], g, nullptr, nullptr, 0));
    HIPCHECK(hipGraphDestroy(g));
  }

  void capture_b(int p) {
    hipGraph_t g;
    std::lock_guard<std::mutex> cg(cap_mu_);   // (no exchange-thread HIP call inside a capture)
    HIPCHECK(hipStreamBeginCapture(s_comp_, hipStreamCaptureModeThreadLocal));
    launch_phase_b(s_comp_, io_[p]);
    HIPCHECK(hipStreamEndCapture(s_comp_, &g));
    HIPCHECK(hipGraphInstantiate(&graph_b_[p], g, nullptr, nullptr, 0));
    HIPCHECK(hipGraphDestroy(g));
  }

  int device_ = 0;
  u32 n_cu_ = 256;   // compute units of the device (grid caps of the block-per-segment / group kernels)
  DS d_;
  std::map<std::string, Buf> bufs_;
  u64 total_bytes_ = 0;
  u64 egress_alloc_ = 0;
  int ref_back_ = -1;    // egress by reference: steps back a body may be referenced (-1 off)
  u32 ref_min_ = 256;    // smallest referenced body (smaller ones are cheaper inline)
  u32 ntiles_max_ = 0;
  u32 restore_max_ = 0;
  u64 carry_budget_ = 0;
  u64 get_cap_ = 0;
  u8* get_out_dev_ = nullptr;
  GetRes* get_res_dev_ = nullptr;
  u64* scan_status_ = nullptr;
  unsigned long long* spill_moved_ = nullptr;
  u32* scan_ctl_ = nullptr;
  u32 scan_smax_ = 0;
  bool graph_enabled_ = true;
  bool sdma_ = true;
  hipGraphExec_t graph_exec_[NPAR_MAX] = {};
  hipGraphExec_t graph_b_[NPAR_MAX] = {};
  hipEvent_t ev_a_[NPAR_MAX], ev_ext_[NPAR_MAX];
  bool phase_a_[NPAR_MAX] = {};
  bool counts_ready_[NPAR_MAX] = {};
  bool lag_ = false;
  std::vector<u32> lag_recv_;
  u64 lag_stream_ = 0;
  bool xfer_set_ = false;
  // native exchange
  bool native_x_ = false;
  bool b_due_[NPAR_MAX] = {};   // phase A launched, phase B not yet (native exchange)
  std::unique_ptr<cmqx::RcclXchg> rccl_;
  std::unique_ptr<cmqx::ShmXchg> shm_;
  std::unique_ptr<cmqx::ShmXchg> cshm_;   // rccl + host shared-memory count exchange
  std::vector<int> xmembers_;
  int xtimeout_ms_ = 10000;
  bool xfailover_ = false;
  bool x_wait_ = false;              // phase B waits on the RCCL bulk transfer
  u64 xseq_ = 0;
  // asynchronous exchange (xchg_setup async=true): one job at a time on the exchange thread
  bool async_x_ = false;
  std::thread xth_;
  std::mutex xmu_;
  std::condition_variable xcv_;
  bool xstop_ = false, xjob_ = false, xbusy_ = false, xres_ = false;
  int xq_ = 0, xres_rc_ = 0;
  u32 xflags_ = 0, xres_orf_ = 0, xjob_seq_ = 0, xseq_job_ = 0;
  std::string xerr_;
  u32 b_wait_[NPAR_MAX] = {};           // launch_b(p): the job phase B of parity p waits for (0: none)
  u32* xflag_h_ = nullptr;           // host-mapped [0] last finished job, [1] a device wait gave up
  std::mutex cap_mu_;                // graph captures vs the exchange thread's HIP calls
  hipStream_t s_x_ = nullptr;        // the shared-memory exchange's copies
  std::mutex io_mu_;
  hipStream_t s_io_ = nullptr;       // upload / download
  u32* xflag_d_ = nullptr;
  u8* xs_desc_[2] = {nullptr, nullptr};
  u8* xs_pay_[2] = {nullptr, nullptr};
  u8* xr_desc_[2] = {nullptr, nullptr};
  u8* xr_pay_[2] = {nullptr, nullptr};
  bool links_ = false;
  u8* ls_desc_[2] = {nullptr, nullptr};
  u8* ls_pay_[2] = {nullptr, nullptr};
  u8* lk_send_[2] = {nullptr, nullptr};
  u8* rack_[2] = {nullptr, nullptr};
  struct HostIO : DS {   // per-parity device view + host addresses of its mapped outputs
    const Counters* ctr_host_h = nullptr;
    const SegOut* seg_out_hh = nullptr;
    const ConnOut* conn_out_hh = nullptr;
    const CtrlRec* ctrl_rec_hh = nullptr;
    const u8* ctrl_hh = nullptr;
    const u8* persist_hh = nullptr;
    const ConsumedRec* crec_hh = nullptr;
    const RingMove* grow_hh = nullptr;
    const u32* conn_conf_hh = nullptr;
    const GetOut* get_out_hh = nullptr;
  };
  std::vector<GetReq> pend_gets_;   // Basic.Get requests for the next submit
  // deferred control writes: device address -> bytes (non-overlapping), channels to mark
  static constexpr u64 DELTA_CAP = 4ull << 20;
  std::mutex dl_mu_;
  // open: a light control section is still staging into it (stage_begin .. stage_end); a
  // step never takes an open batch, so one section's change set rides one step whole
  struct DlBatch { std::map<u64, std::string> w; std::vector<u32> dirty, unp; u64 bytes = 0; bool open = false; u64 id = 0; };
  std::vector<u32> unp_ready_;   // unpauses of batches flush_deltas applied (next step)
  u32 spill_req_[3] = {0, 0, 0};   // stage_spill for the next submitted step (dl_mu_)
  // staged writes with the unpauses staged after them; a batch that overflows one step's
  // delta buffer keeps its unpauses until its last write is packed
  std::deque<DlBatch> dl_;
  u32 dl_open_ = 0;   // light sections staging now (stage_begin / stage_end)
  u64 dl_next_id_ = 1;   // id of the next batch (DlBatch.id)
  u64 dl_bytes_ = 0;
  u8* dl_h_[NPAR_MAX] = {};
  u32 dl_step_[NPAR_MAX] = {};
  u64 dl_steps_ = 0;
  static constexpr u32 COLD_BATCH = 1u << 16;   // cold records per pick / scan call
  struct Side { int kind; u32 a; u64 b, c; u32 max_n; u64 max_bytes; u32 n; bool launched; };
  Side side_{SIDE_NONE, 0, 0, 0, 0, 0, 0, false};
  std::mutex side_mu_;
  std::condition_variable side_cv_;
  hipEvent_t ev_side_ = nullptr;
  void* side_h_ = nullptr;      // host-mapped: [count @0][ColdRec[] @64]
  void* side_d_ = nullptr;
  i64* side_live_h_ = nullptr;
  ColdRec* cold_recs_ = nullptr;
  u32* cold_cnt_ = nullptr;
  unsigned long long* cold_bytes_ = nullptr;
  u64* cold_end_ = nullptr;
  // overlapped steps (world 1)
  bool overlap_ = false;
  int npar_ = 2;   // per-step IO sets in use (NPAR_MAX arrays)
 public:
  u32 dcap_bytes_ = 0;   // StepIn.dcap_bytes of the next submitted steps (deliver_cap_bytes)
 private:
  hipStream_t s_ing_ = nullptr;
  hipEvent_t ev_ing_[NPAR_MAX], ev_rest_[NPAR_MAX];
  bool rest_issued_[NPAR_MAX] = {}, ing_issued_[NPAR_MAX] = {};
  bool eager_d2h_[NPAR_MAX] = {};   // the step's egress copy was queued at launch (copy_mode 2)
  bool pre_[NPAR_MAX] = {};
  u8* ingress_slot_[INGRESS_SLOTS] = {};
  u8* work_p1_ = nullptr;
  hipEvent_t ev_ing_slot_[INGRESS_SLOTS];
  bool ing_slot_issued_[INGRESS_SLOTS] = {};
  u64 launch_seq_[NPAR_MAX] = {};          // the step number staged in each parity
  u64 pre_ptr_[NPAR_MAX] = {}, pre_len_[NPAR_MAX] = {}, pre_seq_[NPAR_MAX] = {};
  hipEvent_t ev_pre_[NPAR_MAX];
  hipStream_t s_pre_ = nullptr;
  hipGraphExec_t graph_ing_[NPAR_MAX] = {};
  hipGraphExec_t graph_rest_[NPAR_MAX] = {};
  u64* scan_status_ing_ = nullptr;
  u32* scan_ctl_ing_ = nullptr;
  // parity 1's copies of the per-step buffers (parity 0 keeps d_'s)
  std::vector<std::function<void(DS&)>> par1_;
  template <class T>
  void dup(T* DS::*m, const char* name, size_t bytes) {
    T* p1 = (T*)alloc((std::string(name) + "_p1").c_str(), bytes, false);
    par1_.push_back([m, p1](DS& io) { io.*m = p1; });
  }
  GetReq* stage_gets_[NPAR_MAX] = {};
  u32* stage_unp_[NPAR_MAX] = {};
  u32 nunp_[NPAR_MAX] = {};   // unpauses the last submit on each parity carried
  u32 nget_[NPAR_MAX] = {};
  HostIO io_[NPAR_MAX];
  CmqEngineApi api_{};
  std::string err_;
  u8* egress_dev_[EGRESS_SLOTS] = {};
  u8* egress_host_[EGRESS_SLOTS] = {};
  u8* egress_host_dev_[EGRESS_SLOTS] = {};
  int slot_of_[NPAR_MAX] = {};
  int pslot_of_[NPAR_MAX] = {};
  int copy_mode_ = 0;
  hsa_agent_t gpu_agent_{}, cpu_agent_{};
  hsa_amd_sdma_engine_id_t sdma_engine_{}, sdma_engine2_{};
  int sdma_split_ = 1;
  hsa_signal_t sdma_sig_[EGRESS_SLOTS] = {};
  bool sdma_pending_[EGRESS_SLOTS] = {};
  // gated egress: per slot the gate the step's last kernel opens, the host tail's signal,
  // whether a tail is in flight and the bytes copied speculatively for the slot's step
  bool gated_ = false;
  hsa_signal_t gate_sig_[EGRESS_SLOTS] = {};
  u64 spin_ticks_ = 0, block_ticks_ = 0;   // bounded_wait: active spin / blocked slice (timestamp ticks)
  u32 wait_ms_ = 10000;                    // bounded_wait deadline
  bool wait_failed_ = false, gate_fault_ = false;
  void* gate_dummy_ = nullptr;             // device word a faulted step's gate store lands in
  hsa_signal_t tail_sig_[EGRESS_SLOTS] = {};
  bool tail_pending_[EGRESS_SLOTS] = {};
  u64 spec_[EGRESS_SLOTS] = {};
  hsa_amd_sdma_engine_id_t tail_engine_{};
  u64 eg_hist_[4] = {0, 0, 0, 0};
  u32 eg_hist_i_ = 0;
  u64 eg_stats_[4] = {0, 0, 0, 0};
  u32 copy_wgs_ = 16;
  int sdma_pref_ = -1;
  double ht_[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};   // host_times() phases
  StepIn* stage_in_[NPAR_MAX] = {};
  SegIn* stage_segs_[NPAR_MAX] = {};
  hipStream_t s_comp_ = nullptr, s_h2d_ = nullptr, s_d2h_ = nullptr;
  hipStream_t s_h2d_alt_ = nullptr;   // odd steps' H2D (cfg h2d_alt)
  hipStream_t h2d_of(u64 step) const { return (s_h2d_alt_ && (step & 1)) ? s_h2d_alt_ : s_h2d_; }
  // cfg h2d_hsa: ingress payloads in GPU-mapped host memory go to the SDMA engine through HSA
  bool h2d_hsa_ = false;
  hsa_amd_sdma_engine_id_t ing_engine_{};
  hsa_signal_t ing_sig_[INGRESS_SLOTS] = {};
  bool ing_hsa_[INGRESS_SLOTS] = {};   // the slot's last payload went through HSA (ing_sig_)
  bool h2d_hip_[NPAR_MAX] = {true, true, true};   // the step's stream waits for ev_h2d_
  u64 h2d_addr_[NPAR_MAX] = {};   // the word the step's k_h2d_wait polled (0: none)
  u64 h2d_addr2_[NPAR_MAX] = {};  // (and its second half's, a split payload)
  hsa_amd_sdma_engine_id_t ing_engine2_{};   // a split payload's second engine (0: no split)
  hsa_signal_t ing_sig2_[INGRESS_SLOTS] = {};
  bool ing_split_[INGRESS_SLOTS] = {};
  bool h2d_fault_ = false;
  bool h2d_split_cfg_ = false;
  u64 h2d_split_min_ = 4u << 20;
  void* h2d_dummy_ = nullptr;     // pinned host word of inject_h2d_fault

  // the agent address of a payload in page-locked host memory (hipHostMalloc /
  // hipHostRegister), 0 for pageable memory (the runtime's copy stages that)
  static u64 ingress_src(u64 ptr) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, (const void*)ptr) != hipSuccess) {
      (void)hipGetLastError();
      return 0;
    }
    return a.type == hipMemoryTypeHost && a.devicePointer ? (u64)a.devicePointer : 0;
  }

  // a step's payload into ingress slot is: on the HSA path (k_h2d_wait waits for it on the
  // device) or as a runtime copy on stream ps (the step's stream waits for ev_h2d_)
  void ingress_copy(u64 step, int is, u64 ptr, u64 len, hipStream_t ps) {
    const u64 src = h2d_hsa_ ? ingress_src(ptr) : 0;
    if (src) {
      // the slot's last reader (step - INGRESS_SLOTS, collected long ago in the drivers'
      // order) and its copy are done before the signal is re-armed
      if (step >= INGRESS_SLOTS && ing_slot_issued_[is] && hipEventQuery(ev_ing_slot_[is]) != hipSuccess)
        HIPCHECK(hipEventSynchronize(ev_ing_slot_[is]));
      if (ing_hsa_[is]) bounded_wait(ing_sig_[is], -1, "ingress H2D");
      if (ing_split_[is]) bounded_wait(ing_sig2_[is], -1, "ingress H2D");
      // a large payload in two halves on two engines at once: 56.8 vs 54.9 GB/s on one (the
      // PCIe link is the bound, bench/micro/h2d_chain_probe.hip, profiles/r6_z/h2d_chain3.txt)
      const bool split = ing_engine2_ && len >= h2d_split_min_ && len > 8192;
      const u64 h1 = split ? ((len / 2 + 4095) & ~u64(4095)) : len;
      hsa_signal_store_relaxed(ing_sig_[is], 1);
      if (hsa_amd_memory_async_copy_on_engine(ingress_slot_[is], gpu_agent_, (const void*)src, cpu_agent_, h1, 0,
                                              nullptr, ing_sig_[is], ing_engine_, true) != HSA_STATUS_SUCCESS)
        throw std::runtime_error("hsa_amd_memory_async_copy_on_engine (ingress) failed");
      if (split) {
        hsa_signal_store_relaxed(ing_sig2_[is], 1);
        if (hsa_amd_memory_async_copy_on_engine(ingress_slot_[is] + h1, gpu_agent_, (const void*)(src + h1), cpu_agent_,
                                                len - h1, 0, nullptr, ing_sig2_[is], ing_engine2_,
                                                true) != HSA_STATUS_SUCCESS)
          throw std::runtime_error("hsa_amd_memory_async_copy_on_engine (ingress, second half) failed");
      }
      ing_hsa_[is] = true;
      ing_split_[is] = split;
      return;
    }
    if (step >= INGRESS_SLOTS && ing_slot_issued_[is] && hipEventQuery(ev_ing_slot_[is]) != hipSuccess)
      HIPCHECK(hipStreamWaitEvent(ps, ev_ing_slot_[is], 0));
    HIPCHECK(hipMemcpyAsync((void*)ingress_slot_[is], (const void*)ptr, len,
                            sdma_ ? hipMemcpyDeviceToDeviceNoCU : hipMemcpyHostToDevice, ps));
    ing_hsa_[is] = false;
    ing_split_[is] = false;
  }
  hipEvent_t ev_h2d_[NPAR_MAX], ev_done_[NPAR_MAX], ev_d2h_[EGRESS_SLOTS];
  bool inflight_[NPAR_MAX] = {};
  bool staged_[NPAR_MAX] = {};   // submitted with defer, kernels not launched yet
  bool d2h_issued_[EGRESS_SLOTS] = {};
  u64 seq_ = 0;
};

static py::array alloc_pinned(size_t bytes) {
  void* p = nullptr;
  HIPCHECK(hipHostMalloc(&p, bytes, hipHostMallocPortable));
  return py::array(py::dtype("uint8"), {(py::ssize_t)bytes}, {(py::ssize_t)1}, p,
                   py::capsule(p, [](void* q) { (void)hipHostFree(q); }));
}

static u64 create_stream(int device) {
  HIPCHECK(hipSetDevice(device));
  hipStream_t st;
  HIPCHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  return (u64)st;
}

static int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

PYBIND11_MODULE(_dataplane, m) {
  m.doc() = "MI355X (gfx950) AMQP data-plane kernels + native step runtime";
  m.def("alloc_pinned", &alloc_pinned, "page-locked host buffer (numpy uint8)");
  m.def("roctx_push", [](const std::string& n) { roctxRangePushA(n.c_str()); });
  m.def("roctx_pop", []() { roctxRangePop(); });
  m.def("roctx_mark", [](const std::string& n) { roctxMarkA(n.c_str()); });
  m.def("device_count", &device_count);
  m.def("create_stream", &create_stream, py::arg("device") = 0);
  m.attr("CAND_MAX") = CAND_MAX;
  m.attr("TOPIC_K") = TOPIC_K;
  m.attr("TOPIC_WORDS") = TOPIC_WORDS;
  m.attr("LAT_BINS") = LAT_BINS;
  py::class_<Engine>(m, "Engine")
      .def(py::init<py::dict>())
      .def("info", &Engine::info)
      .def("fill", &Engine::fill)
      .def("upload", &Engine::upload, py::arg("name"), py::arg("data"), py::arg("offset") = 0)
      .def("download", &Engine::download, py::arg("name"), py::arg("offset") = 0, py::arg("n") = 0)
      .def("host_view", &Engine::host_view)
      .def("submit", &Engine::submit, py::arg("segs"), py::arg("payload_ptr"), py::arg("payload_len"),
           py::arg("now_ms"), py::arg("step"), py::arg("id_ms"), py::arg("worker"), py::arg("defer") = false,
           py::arg("flags") = 0)
      .def("launch", &Engine::launch)
      .def("prefetch", &Engine::prefetch, py::arg("payload_ptr"), py::arg("payload_len"))
      .def("persist_slot", &Engine::persist_slot)
      .def("stage_unpause", &Engine::stage_unpause)
      .def("stage_gets", [](Engine& e, py::buffer b) {
             py::buffer_info bi = b.request();
             const size_t nb = (size_t)bi.size * bi.itemsize;
             if (nb % sizeof(GetReq)) throw std::runtime_error("stage_gets: GetReq[] (u32 conn, chslot, q, noack)");
             e.stage_gets((const GetReq*)bi.ptr, (u32)(nb / sizeof(GetReq)));
           })
      .def("get_out", &Engine::get_out_py)
      .def("send_counts", &Engine::send_counts)
      .def("submit_b", &Engine::submit_b, py::arg("parity"), py::arg("recv"), py::arg("stream") = 0)
      .def("set_xfer_buffers", &Engine::set_xfer_buffers)
      .def("set_xfer_parity", &Engine::set_xfer_parity)
      .def("set_import", &Engine::set_import, py::arg("recv"), py::arg("stream") = 0)
      .def("restore", &Engine::restore, py::arg("desc"), py::arg("payload"), py::arg("now_ms"))
      .def("spill", &Engine::spill, py::arg("lim"), py::arg("hot"), py::call_guard<py::gil_scoped_release>())
      .def("cold_pick", &Engine::cold_pick, py::arg("hot"), py::arg("lim"), py::arg("max_n"), py::arg("max_bytes"))
      .def("cold_commit", &Engine::cold_commit)
      .def("cold_scan", &Engine::cold_scan, py::arg("window"), py::arg("max_n"))
      .def("cold_in", &Engine::cold_in)
      .def("side_cold_pick", &Engine::side_cold_pick, py::arg("hot"), py::arg("lim"), py::arg("min_used"),
           py::arg("max_n"), py::arg("max_bytes"))
      .def("side_cold_commit", &Engine::side_cold_commit)
      .def("side_cold_scan", &Engine::side_cold_scan, py::arg("window"), py::arg("max_n"))
      .def("side_cold_in", &Engine::side_cold_in)
      .def("side_cold_live", &Engine::side_cold_live)
      .def("side_wait", &Engine::side_wait, py::arg("timeout_s"))
      .def("side_pending", &Engine::side_pending)
      .def("basic_get", &Engine::basic_get, py::arg("q"), py::arg("chslot"), py::arg("noack"), py::arg("now_ms"))
      .def("wait_results", &Engine::wait_results)
      .def("egress_copy", &Engine::egress_copy)
      .def("egress_wait", &Engine::egress_wait)
      .def("egress_slot", &Engine::egress_slot)
      .def("set_egress_ref", &Engine::set_egress_ref)
      .def("set_deliver_cap_bytes", [](Engine& e, u32 n) { e.dcap_bytes_ = n; })
      .def("egress_wait_slot", &Engine::egress_wait_slot)
      .def("egress_done_slot", &Engine::egress_done_slot)
      .def("step_done", &Engine::step_done)
      .def("sync", &Engine::sync)
      .def("c_api", &Engine::c_api)
      .def("xchg_setup", &Engine::xchg_setup, py::arg("kind"), py::arg("arg"), py::arg("members"),
           py::arg("timeout_ms") = 10000, py::arg("failover") = false, py::arg("counts_shm") = "",
           py::arg("async_x") = false,
           py::call_guard<py::gil_scoped_release>())
      .def_static("xchg_unique_id", &Engine::xchg_unique_id)
      .def("exchange", [](Engine& e, int q, u32 flags) {
             u32 orf = 0;
             int rc;
             {
               py::gil_scoped_release nogil;
               rc = e.exchange(q, flags, &orf);
             }
             return py::make_tuple(rc, orf);
           }, py::arg("parity"), py::arg("flags") = 0)
      .def("drop_exchange", &Engine::drop_exchange, py::arg("q"), py::arg("collect") = false)
      .def("launch_b", &Engine::launch_b)
      .def("counters", &Engine::counters)
      .def("host_times", &Engine::host_times, py::arg("reset") = false)
      .def("egress_stats", &Engine::egress_stats)
      .def("inject_gate_fault", &Engine::inject_gate_fault)
      .def("inject_h2d_fault", &Engine::inject_h2d_fault)
      .def("wait_failed", &Engine::wait_failed)
      .def("stage_write", &Engine::stage_write_buf, py::arg("name"), py::arg("data"), py::arg("offset") = 0)
      .def("stage_mark_dirty", &Engine::stage_mark_dirty)
      .def("stage_begin", &Engine::stage_begin)
      .def("dl_state", &Engine::dl_state)
      .def("stage_end", &Engine::stage_end)
      .def("stage_spill", &Engine::stage_spill)
      .def("deltas_pending", &Engine::deltas_pending)
      .def("flush_deltas", &Engine::flush_deltas, py::call_guard<py::gil_scoped_release>());
}

// pybind11 module `_core`: the native broker, store and codec for Python.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <condition_variable>

#include "broker.hpp"
#include "codec.hpp"
#include "frontend.hpp"
#include "persist.hpp"
#include "tls_proxy.hpp"
#include "gateway.hpp"
#include "loadgen.hpp"
#include "store.hpp"
#include "../kernels/xchg_host.h"

namespace py = pybind11;
using namespace cmq;

static BrokerConfig config_from(py::dict d) {
  BrokerConfig c;
#define S(k, f) if (d.contains(k)) c.f = d[k].cast<decltype(c.f)>()
  S("host", host); S("port", port); S("amqp_enable", amqp_enable); S("tls_port", tls_port);
  S("tls_enable", tls_enable); S("tls_cert", tls_cert); S("tls_key", tls_key); S("tls_p12", tls_p12);
  S("tls_p12_password", tls_p12_password); S("channel_max", channel_max); S("frame_max", frame_max);
  S("frame_min", frame_min); S("heartbeat", heartbeat); S("default_vhost", default_vhost);
  S("data_dir", data_dir); S("fsync", fsync); S("worker_id", worker_id);
  S("mem_high_watermark", mem_high_watermark); S("mem_low_watermark", mem_low_watermark);
  S("flow_channel", flow_channel); S("max_connections", max_connections); S("hash_wildcard", hash_wildcard);
#undef S
  return c;
}

static py::tuple decode(py::bytes payload) {
  std::string s = payload;
  Method m = decode_method((const u8*)s.data(), s.size());
  py::list args;
  for (size_t k = 0; k < m.spec->fields.size(); ++k) {
    switch (m.spec->fields[k].second) {
      case A_SHORTSTR: args.append(py::bytes(m.args[k].s)); break;
      case A_LONGSTR: args.append(py::bytes(m.args[k].s)); break;
      case A_TABLE: {
        py::dict t;
        for (auto& kv : m.args[k].t) t[py::str(kv.first)] = py::str(kv.second.tag == 'S' ? kv.second.s : std::to_string(kv.second.i));
        args.append(t);
        break;
      }
      default: args.append(m.args[k].i);
    }
  }
  return py::make_tuple(m.cls(), m.mid(), std::string(m.spec->name), args);
}

static py::bytes reencode(py::bytes payload) {
  std::string s = payload;
  Method m = decode_method((const u8*)s.data(), s.size());
  return py::bytes(encode_method_payload(m));
}

PYBIND11_MODULE(_core, m) {
  m.doc() = "chanamq native broker core (C++): AMQP codec, control plane, CPU data path, store";
  py::class_<Broker>(m, "Broker")
      .def(py::init([](py::dict d) { return new Broker(config_from(d)); }))
      .def("start", &Broker::start, py::call_guard<py::gil_scoped_release>())
      .def("stop", &Broker::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("port", &Broker::listen_port)
      .def_property_readonly("tls_port", &Broker::listen_tls_port)
      .def_property_readonly("running", &Broker::running)
      .def("create_vhost", &Broker::create_vhost, py::call_guard<py::gil_scoped_release>())
      .def("delete_vhost", &Broker::delete_vhost, py::call_guard<py::gil_scoped_release>())
      .def("stats_json", &Broker::stats_json, py::call_guard<py::gil_scoped_release>())
      .def("queues_json", &Broker::queues_json, py::call_guard<py::gil_scoped_release>());

  py::class_<Store>(m, "Store")
      .def(py::init<>())
      .def("open", &Store::open, py::arg("dir"), py::arg("fsync") = true)
      .def("close", &Store::close, py::call_guard<py::gil_scoped_release>())
      .def("sync", &Store::sync, py::call_guard<py::gil_scoped_release>())
      .def("compact", &Store::compact, py::call_guard<py::gil_scoped_release>())
      .def("set_auto_compact", &Store::set_auto_compact, py::arg("ratio"), py::arg("min_bytes"))
      .def("set_quota", &Store::set_quota, py::arg("bytes"))
      .def("wait_compaction", &Store::wait_compaction, py::call_guard<py::gil_scoped_release>())
      .def("wal_bytes", &Store::walBytes)
      .def("live_estimate", &Store::liveEstimate)
      .def("compact_stats", [](Store& s) {
             CompactStats c = s.compactStats();
             py::dict d;
             d["runs"] = c.runs; d["last_before"] = c.last_before; d["last_after"] = c.last_after;
             d["tail_bytes"] = c.tail_bytes; d["last_s"] = c.last_s; d["max_lock_s"] = c.max_lock_s;
             d["failures"] = c.failures; d["last_error"] = c.last_error;
             return d;
           })
      .def("configure_body_log", &Store::configureBodyLog, py::arg("stripes"), py::arg("seg_bytes"))
      .def("has_body_log", &Store::hasBodyLog)
      .def("body_stats", [](Store& s) {
             BodyLog::Stats b = s.bodyStats();
             py::dict d;
             d["written"] = b.written; d["records"] = b.records; d["live_bytes"] = b.live_bytes;
             d["live_records"] = b.live_records; d["disk_bytes"] = b.disk_bytes; d["segments"] = b.segments;
             d["reclaimed"] = b.reclaimed; d["bad_reads"] = b.bad_reads; d["write_s"] = b.write_s; d["sync_s"] = b.sync_s;
             return d;
           })
      .def("deleted_queue_ids", &Store::deletedQueueIds)
      .def("select_deleted_queue", [](Store& s, std::string q) -> py::object {
             QueueMetaDeletedRow meta;
             std::vector<QueueMsgRow> msgs, unacks;
             bool has = s.selectDeletedQueue(q, &meta, &msgs, &unacks);
             py::list ml, ul;
             for (auto& r : msgs) ml.append(py::make_tuple(r.offset, r.msgid, r.size));
             for (auto& r : unacks) ul.append(py::make_tuple(r.offset, r.msgid, r.size));
             py::object m = has ? (py::object)py::make_tuple(meta.lconsumed, meta.nconsumer, meta.durable) : py::none();
             return py::make_tuple(m, ml, ul);
           })
      .def("insert_deleted_queue_meta", &Store::insertDeletedQueueMeta)
      .def("insert_deleted_queue_msg", &Store::insertDeletedQueueMsg)
      .def("insert_deleted_queue_unack", &Store::insertDeletedQueueUnack)
      .def("row_count", &Store::rowCount)
      .def("queue_ids", &Store::queueIds)
      .def("message_ids", &Store::messageIds)
      .def("exchange_ids", &Store::exchangeIds)
      .def("vhost_ids", &Store::vhostIds)
      .def("insert_vhost", &Store::insertVhost)
      .def("delete_vhost", &Store::deleteVhost)
      .def("insert_message", [](Store& s, int64_t id, int64_t tstamp, py::bytes header, py::bytes body,
                                std::string ex, std::string rk, bool durable, int32_t refer, int64_t ttl_ms) {
             MsgRow r;
             r.id = id; r.tstamp = tstamp; r.header = header; r.body = body; r.exchange = ex; r.routing = rk;
             r.durable = durable; r.refer = refer;
             s.insertMessage(r, ttl_ms);
           })
      .def("select_message", [](Store& s, int64_t id) -> py::object {
             MsgRow r;
             if (!s.selectMessage(id, &r)) return py::none();
             return py::make_tuple(r.id, r.tstamp, py::bytes(r.header), py::bytes(r.body), r.exchange, r.routing,
                                   r.durable, r.refer);
           })
      .def("delete_message", &Store::deleteMessage)
      .def("update_message_refer_count", &Store::updateMessageReferCount)
      .def("insert_queue_meta", &Store::insertQueueMeta)
      .def("insert_queue_msg", &Store::insertQueueMsg)
      .def("insert_last_consumed", &Store::insertLastConsumed)
      .def("consumed_queue_messages", [](Store& s, std::string q, int64_t l, std::vector<std::tuple<int64_t, int64_t, int32_t>> u) {
             std::vector<QueueMsgRow> rows;
             for (auto& t : u) { QueueMsgRow r; r.offset = std::get<0>(t); r.msgid = std::get<1>(t); r.size = std::get<2>(t); rows.push_back(r); }
             s.consumedQueueMessages(q, l, rows);
           })
      .def("select_queue", [](Store& s, std::string q) -> py::object {
             QueueMetaRow meta;
             std::vector<QueueMsgRow> msgs, unacks;
             if (!s.selectQueue(q, &meta, &msgs, &unacks)) return py::none();
             py::list ml, ul;
             for (auto& r : msgs) ml.append(py::make_tuple(r.offset, r.msgid, r.size));
             for (auto& r : unacks) ul.append(py::make_tuple(r.offset, r.msgid, r.size));
             return py::make_tuple(py::make_tuple(meta.lconsumed, meta.consumers, meta.durable, meta.ttl), ml, ul);
           })
      .def("force_delete_queue", &Store::forceDeleteQueue)
      .def("pending_delete_queue", &Store::pendingDeleteQueue)
      .def("delete_consumed_queue_msgs", &Store::deleteConsumedQueueMsgs)
      .def("insert_queue_unack", &Store::insertQueueUnack)
      .def("delete_queue_unack", &Store::deleteQueueUnack)
      .def("delete_queue_msg", &Store::deleteQueueMsg)
      .def("insert_exchange", [](Store& s, std::string id, std::string tpe, bool durable, bool autodel, bool internal,
                                 std::map<std::string, std::string> args) {
             ExchangeRow x; x.tpe = tpe; x.durable = durable; x.autodel = autodel; x.internal = internal; x.args = args;
             s.insertExchange(id, x);
           })
      .def("insert_bind", &Store::insertBind)
      .def("select_exchange", [](Store& s, std::string id) -> py::object {
             ExchangeRow x;
             std::vector<BindRow> b;
             if (!s.selectExchange(id, &x, &b)) return py::none();
             py::list bl;
             for (auto& r : b) bl.append(py::make_tuple(r.queue, r.key, r.args));
             return py::make_tuple(py::make_tuple(x.tpe, x.durable, x.autodel, x.internal, x.args), bl);
           })
      .def("delete_bind", &Store::deleteBind)
      .def("delete_binds_of_queue", &Store::deleteBindsOfQueue)
      .def("delete_exchange", &Store::deleteExchange)
      .def("select_vhost", [](Store& s, std::string id) -> py::object {
             bool a;
             if (!s.selectVhost(id, &a)) return py::none();
             return py::bool_(a);
           })
      // change feed of the live Cassandra mirror (store/cassandra_live.py)
      .def("set_mirror", &Store::setMirror)
      .def("mirror_pending", &Store::mirrorPending)
      .def("mirror_take", [](Store& s, size_t max_keys) {
             Store::MirrorKeys k = s.mirrorTake(max_keys);
             py::dict d;
             d["msgs"] = k.msgs; d["qmsgs"] = k.qmsgs; d["qunacks"] = k.qunacks; d["qmetas"] = k.qmetas;
             d["qparts"] = k.qparts; d["xs"] = k.xs; d["vhosts"] = k.vhosts; d["deleted"] = k.deleted;
             return d;
           }, py::arg("max_keys") = 4096)
      .def("select_queue_msg", [](Store& s, std::string q, int64_t off) -> py::object {
             QueueMsgRow r;
             if (!s.selectQueueMsg(q, off, &r)) return py::none();
             return py::make_tuple(r.offset, r.msgid, r.size);
           })
      .def("select_queue_unack", [](Store& s, std::string q, int64_t mid) -> py::object {
             QueueMsgRow r;
             if (!s.selectQueueUnack(q, mid, &r)) return py::none();
             return py::make_tuple(r.offset, r.msgid, r.size);
           })
      .def("select_queue_meta", [](Store& s, std::string q) -> py::object {
             QueueMetaRow m;
             if (!s.selectQueueMeta(q, &m)) return py::none();
             return py::make_tuple(m.lconsumed, m.consumers, m.durable, m.ttl);
           });

  py::class_<Gateway>(m, "Gateway")
      .def(py::init<const std::string&, int, uint32_t, bool>(), py::arg("host") = "127.0.0.1", py::arg("port") = 0,
           py::arg("max_conns") = 1024, py::arg("reuseport") = false)
      .def_property_readonly("port", &Gateway::port)
      .def_readonly("rx_bytes", &Gateway::rx_bytes)
      .def_readonly("tx_bytes", &Gateway::tx_bytes)
      .def("poll", [](Gateway& g, int timeout_ms, py::buffer buf, uint64_t offset, uint64_t per_conn_cap) {
             py::buffer_info bi = buf.request(true);
             uint64_t cap = (uint64_t)bi.size * bi.itemsize;
             if (offset > cap) throw std::runtime_error("offset beyond buffer");
             GwPoll r;
             {
               py::gil_scoped_release nogil;
               r = g.poll(timeout_ms, (uint8_t*)bi.ptr + offset, cap - offset, per_conn_cap);
             }
             for (auto& s : r.segs) s.src += offset;
             py::bytes segs((const char*)r.segs.data(), r.segs.size() * sizeof(GwSeg));
             py::list hs;
             for (auto& h : r.handshake) hs.append(py::make_tuple(h.first, py::bytes(h.second)));
             return py::make_tuple(segs, r.used + offset, hs, r.opened, r.closed);
           }, py::arg("timeout_ms"), py::arg("buf"), py::arg("offset") = 0, py::arg("per_conn_cap") = 1 << 20)
      .def("send", [](Gateway& g, uint32_t conn, py::bytes b) {
             std::string s = b;
             g.send(conn, s.data(), s.size());
           })
      .def("send_egress", [](Gateway& g, py::buffer egress, py::buffer conn_out, uint32_t n_slots) {
             py::buffer_info e = egress.request(), c = conn_out.request();
             if ((uint64_t)c.size * c.itemsize < 8ull * n_slots) throw std::runtime_error("conn_out too small");
             py::gil_scoped_release nogil;
             return g.send_egress((const uint8_t*)e.ptr, (const uint32_t*)c.ptr, n_slots);
           })
      .def("flush", &Gateway::flush, py::call_guard<py::gil_scoped_release>())
      .def("set_data_mode", &Gateway::set_data_mode)
      .def("set_read_paused", &Gateway::set_read_paused)
      .def("close", &Gateway::close)
      .def("pending_bytes", &Gateway::pending_bytes);

  py::class_<Frontend>(m, "Frontend")
      .def(py::init([](uint64_t api, py::dict d) {
             FrontendCfg c;
#define S(k, f) if (d.contains(k)) c.f = d[k].cast<decltype(c.f)>()
             S("host", host); S("port", port); S("io_threads", io_threads); S("per_conn_read", per_conn_read);
             S("idle_step_ms", idle_step_ms); S("sweep_ms", sweep_ms); S("worker", worker); S("max_slot", max_slot); S("reuseport", reuseport);
             S("sndbuf", sndbuf); S("rcvbuf", rcvbuf); S("wblock_high", wblock_high); S("wblock_low", wblock_low);
             S("async_scatter", async_scatter); S("egress_ref", egress_ref); S("egress_ref_min", egress_ref_min); S("egress_ref_step_min", egress_ref_step_min);
#undef S
             return new Frontend(c, (const CmqEngineApi*)api);
           }), py::arg("engine_api"), py::arg("cfg") = py::dict())
      .def_property_readonly("port", &Frontend::port)
      .def("start", &Frontend::start, py::call_guard<py::gil_scoped_release>())
      .def("stop", &Frontend::stop, py::call_guard<py::gil_scoped_release>())
      .def("poll_events", [](Frontend& f, int timeout_ms) {
             std::vector<FeEvent> evs;
             {
               py::gil_scoped_release nogil;
               evs = f.poll_events(timeout_ms);
             }
             py::list out;
             for (auto& e : evs)
               out.append(py::make_tuple(e.kind, e.conn, e.a, e.b, py::bytes(e.data), py::bytes(e.data2)));
             return out;
           }, py::arg("timeout_ms") = 100)
      .def("take", [](Frontend& f, uint32_t conn) { return py::bytes(f.take(conn)); })
      .def("send", [](Frontend& f, uint32_t conn, py::bytes b) {
             std::string s = b;
             py::gil_scoped_release nogil;
             f.send(conn, s.data(), s.size());
           })
      .def("send_after", [](Frontend& f, uint32_t conn, py::bytes b) {
             std::string s = b;
             py::gil_scoped_release nogil;
             f.send_after(conn, s.data(), s.size());
           })
      .def("wake", &Frontend::wake)
      .def("flush_ctl", &Frontend::flush_ctl, py::call_guard<py::gil_scoped_release>())
      .def("ctl_state", &Frontend::ctl_state)
      .def("send_egress", [](Frontend& f, py::buffer egress, py::buffer conn_out, uint32_t n_slots) {
             py::buffer_info e = egress.request(), c = conn_out.request();
             if ((uint64_t)c.size * c.itemsize < 8ull * n_slots) throw std::runtime_error("conn_out too small");
             py::gil_scoped_release nogil;
             f.send_egress((const u8*)e.ptr, (const ConnOut*)c.ptr, n_slots);
           })
      .def("set_data_mode", [](Frontend& f, uint32_t conn, py::bytes leftover) {
             std::string s = leftover;
             f.set_data_mode(conn, s);
           }, py::arg("conn"), py::arg("leftover") = py::bytes(""))
      .def("set_host_mode", &Frontend::set_host_mode)
      .def("set_heartbeat", &Frontend::set_heartbeat)
      .def("set_read_cap", &Frontend::set_read_cap)
      .def("close", &Frontend::close, py::arg("conn"), py::arg("gen") = -1)
      .def("kick", &Frontend::kick)
      .def("pause", &Frontend::pause, py::call_guard<py::gil_scoped_release>())
      .def("resume", &Frontend::resume, py::call_guard<py::gil_scoped_release>())
      .def("release", &Frontend::release)
      .def("attach_persist", &Frontend::attach_persist, py::keep_alive<1, 2>())
      .def("pending_out", &Frontend::pending_out)
      .def("request_sync", &Frontend::request_sync)
      .def("inject", [](Frontend& f, uint32_t conn, py::bytes b) { f.inject(conn, std::string(b)); })
      .def("queue_get", &Frontend::queue_get, py::arg("conn"), py::arg("chslot"), py::arg("q"), py::arg("noack"),
           py::arg("id"))
      .def("cancel_gets", &Frontend::cancel_gets)
      .def("sync_done", &Frontend::sync_done)
      .def("healthy", &Frontend::healthy, py::arg("stuck_s") = 5.0)
      .def("inject_fault", &Frontend::inject_fault, py::arg("kind"), py::arg("steps") = 0)
      .def("stats", [](Frontend& f) {
             FeStats s = f.stats();
             py::dict o;
             o["steps"] = s.steps; o["published"] = s.published; o["delivered"] = s.delivered;
             o["spill_moved"] = s.spill_moved;
             o["rx_bytes"] = s.rx_bytes; o["tx_bytes"] = s.tx_bytes; o["egress_bytes"] = s.egress_bytes;
             o["store_fail_nacks"] = s.store_fail_nacks;
             o["held_steps"] = s.held_steps; o["idle_steps"] = s.idle_steps; o["gather_segs"] = s.gather_segs;
             o["live_bytes"] = s.live_bytes; o["live_msgs"] = s.live_msgs; o["io_phase_s"] = s.io_phase_s;
             o["dropped_nomem"] = s.dropped_nomem; o["ring_full"] = s.ring_full; o["unroutable"] = s.unroutable;
             o["routed"] = s.routed; o["expired"] = s.expired; o["ctrl"] = s.ctrl; o["log_used"] = s.log_used;
             o["wait_s"] = s.wait_s;
             o["submit_s"] = s.submit_s;
             o["xchg_s"] = s.xchg_s; o["xchg_steps"] = s.xchg_steps; o["syncs"] = s.syncs;
             o["xfails"] = s.xfails; o["flush_steps"] = s.flush_steps;
             o["lat_hist"] = std::vector<u64>(s.lat_hist, s.lat_hist + 32);
             o["h_period_us_log2"] = std::vector<u64>(s.h_period, s.h_period + 32);
             o["h_io_us_log2"] = std::vector<u64>(s.h_io, s.h_io + 32);
             o["h_submit_us_log2"] = std::vector<u64>(s.h_submit, s.h_submit + 32);
             o["h_wait_us_log2"] = std::vector<u64>(s.h_wait, s.h_wait + 32);
             o["max_period_s"] = s.max_period_s; o["max_io_s"] = s.max_io_s; o["max_wait_s"] = s.max_wait_s;
             return o;
           });
  py::class_<PersistWorker>(m, "PersistWorker")
      .def(py::init<Store*>(), py::keep_alive<1, 2>())
      .def("start", &PersistWorker::start)
      .def("stop", &PersistWorker::stop, py::call_guard<py::gil_scoped_release>())
      .def("set_queue", &PersistWorker::set_queue)
      .def("seed_row", &PersistWorker::seed_row)
      .def("submit", [](PersistWorker& w, u64 step, py::bytes persist, py::bytes consumed) {
             w.submit(step, std::string(persist), std::string(consumed));
           })
      .def("drain", &PersistWorker::drain, py::call_guard<py::gil_scoped_release>())
      .def("set_group_delay", &PersistWorker::set_group_delay)
      .def("stats", [](PersistWorker& w) {
             py::dict o;
             o["rows"] = w.rows(); o["commits"] = w.commits(); o["body_bytes"] = w.bytes(); o["busy_s"] = w.busy_s();
             o["apply_s"] = w.apply_s(); o["flush_s"] = w.flush_s(); o["sync_s"] = w.sync_s();
             o["failed"] = w.failed(); o["error"] = w.error();
             return o;
           });
  py::class_<TlsProxy>(m, "TlsProxy")
      .def(py::init([](py::dict d) {
             TlsProxyCfg c;
#define S(k, f) if (d.contains(k)) c.f = d[k].cast<decltype(c.f)>()
             S("host", host); S("port", port); S("upstream_host", upstream_host); S("upstream_port", upstream_port);
             S("cert", cert); S("key", key); S("p12", p12); S("p12_password", p12_password); S("buffer", buffer);
#undef S
             return new TlsProxy(c);
           }))
      .def_property_readonly("port", &TlsProxy::port)
      .def("start", &TlsProxy::start)
      .def("stop", &TlsProxy::stop, py::call_guard<py::gil_scoped_release>())
      .def("connections", &TlsProxy::connections);
  py::class_<EchoEngine>(m, "EchoEngine")
      .def(py::init<u32, u32, u64, u32, u32, u32>(), py::arg("c_max"), py::arg("seg_max"), py::arg("ingress_cap"),
           py::arg("carry_cap"), py::arg("world") = 1, py::arg("rank") = 0)
      .def("c_api", &EchoEngine::c_api)
      .def("unpause", &EchoEngine::unpause)
      .def("xchg_setup", &EchoEngine::xchg_setup, py::arg("name"), py::arg("members"), py::arg("timeout_ms") = 5000,
           py::arg("async_x") = false)
      .def_readonly("imported", &EchoEngine::imported)
      .def_readonly("steps", &EchoEngine::steps);

  // the shared-memory exchange's barrier alone (tests of its failure semantics)
  py::class_<cmqx::ShmXchg>(m, "ShmXchg")
      .def(py::init<const std::string&, const std::vector<int>&, int, size_t, int>(), py::arg("name"),
           py::arg("members"), py::arg("me"), py::arg("box_bytes") = 4096, py::arg("timeout_ms") = 1000)
      .def("barrier", &cmqx::ShmXchg::barrier, py::call_guard<py::gil_scoped_release>());

  m.def("run_load", [](py::dict d) {
    LoadSpec s;
#define S(k, f) if (d.contains(k)) s.f = d[k].cast<decltype(s.f)>()
    S("host", host); S("port", port); S("vhost", vhost); S("producers", producers); S("consumers", consumers);
    S("msg_size", msg_size); S("seconds", seconds); S("exchange", exchange); S("exchange_type", exchange_type);
    S("consumer_port", consumer_port); S("producer_port", producer_port);
    S("routing_key", routing_key); S("queue", queue); S("queues", queues); S("auto_ack", auto_ack);
    S("prefetch", prefetch); S("persistent", persistent); S("durable", durable); S("confirm", confirm);
    S("rate", rate); S("threads", threads); S("warmup", warmup); S("confirm_window", confirm_window);
    S("consumer_threads", consumer_threads); S("nack_every", nack_every);
#undef S
    LoadResult r;
    {
      py::gil_scoped_release nogil;
      r = run_load(s);
    }
    py::dict o;
    o["sent"] = r.sent; o["received"] = r.received; o["elapsed"] = r.elapsed; o["p50_us"] = r.p50_us;
    o["p95_us"] = r.p95_us; o["p99_us"] = r.p99_us; o["error"] = r.error;
    o["confirmed"] = r.confirmed; o["nacked"] = r.nacked; o["threads"] = r.threads;
    o["cpu_consumers_s"] = r.cpu_consumers_s; o["cpu_producers_s"] = r.cpu_producers_s;
    o["redelivered"] = r.redelivered; o["requeued"] = r.requeued; o["flow_off"] = r.flow_off;
    return o;
  });
  m.def("decode_method", &decode);
  m.def("reencode_method", &reencode);
  m.def("method_table", [] {
    py::list out;
    for (auto& s : method_table()) {
      py::list f;
      for (auto& x : s.fields) f.append(py::make_tuple(std::string(x.first), (int)x.second));
      out.append(py::make_tuple(s.cls, s.mid, std::string(s.name), f, s.content));
    }
    return out;
  });
}

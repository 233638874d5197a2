// AMQP 0-9-1 codec (see codec.hpp).  Golden model: chanamq_amd/protocol/codec.py.
#include "codec.hpp"

namespace cmq {

const char HEARTBEAT_FRAME[8] = {8, 0, 0, 0, 0, 0, 0, (char)0xCE};

const Value* table_get(const Table& t, const std::string& k) {
  for (auto& kv : t)
    if (kv.first == k) return &kv.second;
  return nullptr;
}

bool value_as_int(const Value& v, i64* out) {
  switch (v.tag) {
    case 'b': case 'B': case 's': case 'u': case 'I': case 'i': case 'l': case 'T': case 't':
      *out = v.i; return true;
    case 'S': {
      if (v.s.empty()) return false;
      i64 x = 0;
      for (char c : v.s) { if (c < '0' || c > '9') return false; x = x * 10 + (c - '0'); }
      *out = x; return true;
    }
    default: return false;
  }
}

// ------------------------------------------------------------------ reader
bool Reader::bit() {
  if (nbits == 0) { need(1); bits = p[pos++]; nbits = 8; }
  bool v = bits & 1;
  bits >>= 1;
  --nbits;
  return v;
}

Table Reader::table() {
  u32 len = lng();
  need(len);
  Reader sub(p + pos, len);
  Table t;
  while (sub.pos < sub.n) {
    std::string k = sub.shortstr();
    Value v = sub.value();
    if (!table_get(t, k)) t.emplace_back(std::move(k), std::move(v));  // first duplicate wins
  }
  pos += len;
  return t;
}

Value Reader::value() {
  Value v;
  v.tag = (char)octet();
  switch (v.tag) {
    case 'S': v.s = longstr(); break;
    case 'x': v.s = longstr(); break;
    case 'I': v.i = (int32_t)lng(); break;
    case 'i': v.i = lng(); break;
    case 'l': v.i = (i64)llng(); break;
    case 'T': v.i = (i64)llng(); break;
    case 's': v.i = (int16_t)shrt(); break;
    case 'u': v.i = shrt(); break;
    case 'b': v.i = (int8_t)octet(); break;
    case 'B': v.i = octet(); break;
    case 't': v.i = octet() != 0; break;
    case 'd': { u64 x = llng(); memcpy(&v.d, &x, 8); break; }
    case 'f': { u32 x = lng(); float f; memcpy(&f, &x, 4); v.d = f; break; }
    case 'D': v.scale = octet(); v.i = (int32_t)lng(); break;
    case 'F': v.t = std::make_shared<Table>(table()); break;
    case 'A': {
      u32 len = lng();
      need(len);
      Reader sub(p + pos, len);
      v.a = std::make_shared<Array>();
      while (sub.pos < sub.n) v.a->push_back(sub.value());
      pos += len;
      break;
    }
    case 'V': break;
    default: throw AmqpError(SYNTAX_ERROR, std::string("unknown field tag ") + v.tag, true);
  }
  return v;
}

// ------------------------------------------------------------------ writer
void Writer::table(const Table& t) {
  flush_bits();
  Writer inner;
  for (auto& kv : t) {
    inner.shortstr(kv.first);
    inner.value(kv.second);
  }
  longstr(inner.done());
}

void Writer::value(const Value& v) {
  octet((u8)v.tag);
  switch (v.tag) {
    case 'S': case 'x': longstr(v.s); break;
    case 'I': lng((u32)(int32_t)v.i); break;
    case 'i': lng((u32)v.i); break;
    case 'l': case 'T': llng((u64)v.i); break;
    case 's': case 'u': shrt((u16)v.i); break;
    case 'b': case 'B': octet((u8)v.i); break;
    case 't': octet(v.i ? 1 : 0); break;
    case 'd': { u64 x; memcpy(&x, &v.d, 8); llng(x); break; }
    case 'f': { float f = (float)v.d; u32 x; memcpy(&x, &f, 4); lng(x); break; }
    case 'D': octet(v.scale); lng((u32)(int32_t)v.i); break;
    case 'F': table(v.t ? *v.t : Table{}); break;
    case 'A': {
      Writer inner;
      if (v.a)
        for (auto& x : *v.a) inner.value(x);
      longstr(inner.done());
      break;
    }
    case 'V': break;
    default: throw AmqpError(SYNTAX_ERROR, "cannot encode field tag", true);
  }
}

// ------------------------------------------------------------------ method table
// same order/fields as chanamq_amd/protocol/methods.py (tests/test_core_codec.py checks)
static std::vector<MethodSpec> build_table() {
  using F = std::vector<std::pair<const char*, ArgType>>;
  std::vector<MethodSpec> T;
  auto m = [&](u16 c, u16 i, const char* n, F f = {}, bool content = false) {
    T.push_back(MethodSpec{c, i, n, std::move(f), content});
  };
  m(10, 10, "connection.start", {{"version_major", A_OCTET}, {"version_minor", A_OCTET},
                                 {"server_properties", A_TABLE}, {"mechanisms", A_LONGSTR}, {"locales", A_LONGSTR}});
  m(10, 11, "connection.start_ok", {{"client_properties", A_TABLE}, {"mechanism", A_SHORTSTR},
                                    {"response", A_LONGSTR}, {"locale", A_SHORTSTR}});
  m(10, 20, "connection.secure", {{"challenge", A_LONGSTR}});
  m(10, 21, "connection.secure_ok", {{"response", A_LONGSTR}});
  m(10, 30, "connection.tune", {{"channel_max", A_SHORT}, {"frame_max", A_LONG}, {"heartbeat", A_SHORT}});
  m(10, 31, "connection.tune_ok", {{"channel_max", A_SHORT}, {"frame_max", A_LONG}, {"heartbeat", A_SHORT}});
  m(10, 40, "connection.open", {{"virtual_host", A_SHORTSTR}, {"capabilities", A_SHORTSTR}, {"insist", A_BIT}});
  m(10, 41, "connection.open_ok", {{"known_hosts", A_SHORTSTR}});
  m(10, 50, "connection.close", {{"reply_code", A_SHORT}, {"reply_text", A_SHORTSTR}, {"class_id", A_SHORT},
                                 {"method_id", A_SHORT}});
  m(10, 51, "connection.close_ok");
  m(10, 60, "connection.blocked", {{"reason", A_SHORTSTR}});
  m(10, 61, "connection.unblocked");
  m(20, 10, "channel.open", {{"out_of_band", A_SHORTSTR}});
  m(20, 11, "channel.open_ok", {{"channel_id", A_LONGSTR}});
  m(20, 20, "channel.flow", {{"active", A_BIT}});
  m(20, 21, "channel.flow_ok", {{"active", A_BIT}});
  m(20, 40, "channel.close", {{"reply_code", A_SHORT}, {"reply_text", A_SHORTSTR}, {"class_id", A_SHORT},
                              {"method_id", A_SHORT}});
  m(20, 41, "channel.close_ok");
  m(30, 10, "access.request", {{"realm", A_SHORTSTR}, {"exclusive", A_BIT}, {"passive", A_BIT}, {"active", A_BIT},
                               {"write", A_BIT}, {"read", A_BIT}});
  m(30, 11, "access.request_ok", {{"ticket", A_SHORT}});
  m(40, 10, "exchange.declare", {{"ticket", A_SHORT}, {"exchange", A_SHORTSTR}, {"type", A_SHORTSTR},
                                 {"passive", A_BIT}, {"durable", A_BIT}, {"auto_delete", A_BIT}, {"internal", A_BIT},
                                 {"nowait", A_BIT}, {"arguments", A_TABLE}});
  m(40, 11, "exchange.declare_ok");
  m(40, 20, "exchange.delete", {{"ticket", A_SHORT}, {"exchange", A_SHORTSTR}, {"if_unused", A_BIT},
                                {"nowait", A_BIT}});
  m(40, 21, "exchange.delete_ok");
  m(40, 30, "exchange.bind", {{"ticket", A_SHORT}, {"destination", A_SHORTSTR}, {"source", A_SHORTSTR},
                              {"routing_key", A_SHORTSTR}, {"nowait", A_BIT}, {"arguments", A_TABLE}});
  m(40, 31, "exchange.bind_ok");
  m(40, 40, "exchange.unbind", {{"ticket", A_SHORT}, {"destination", A_SHORTSTR}, {"source", A_SHORTSTR},
                                {"routing_key", A_SHORTSTR}, {"nowait", A_BIT}, {"arguments", A_TABLE}});
  m(40, 51, "exchange.unbind_ok");
  m(50, 10, "queue.declare", {{"ticket", A_SHORT}, {"queue", A_SHORTSTR}, {"passive", A_BIT}, {"durable", A_BIT},
                              {"exclusive", A_BIT}, {"auto_delete", A_BIT}, {"nowait", A_BIT},
                              {"arguments", A_TABLE}});
  m(50, 11, "queue.declare_ok", {{"queue", A_SHORTSTR}, {"message_count", A_LONG}, {"consumer_count", A_LONG}});
  m(50, 20, "queue.bind", {{"ticket", A_SHORT}, {"queue", A_SHORTSTR}, {"exchange", A_SHORTSTR},
                           {"routing_key", A_SHORTSTR}, {"nowait", A_BIT}, {"arguments", A_TABLE}});
  m(50, 21, "queue.bind_ok");
  m(50, 30, "queue.purge", {{"ticket", A_SHORT}, {"queue", A_SHORTSTR}, {"nowait", A_BIT}});
  m(50, 31, "queue.purge_ok", {{"message_count", A_LONG}});
  m(50, 40, "queue.delete", {{"ticket", A_SHORT}, {"queue", A_SHORTSTR}, {"if_unused", A_BIT},
                             {"if_empty", A_BIT}, {"nowait", A_BIT}});
  m(50, 41, "queue.delete_ok", {{"message_count", A_LONG}});
  m(50, 50, "queue.unbind", {{"ticket", A_SHORT}, {"queue", A_SHORTSTR}, {"exchange", A_SHORTSTR},
                             {"routing_key", A_SHORTSTR}, {"arguments", A_TABLE}});
  m(50, 51, "queue.unbind_ok");
  m(60, 10, "basic.qos", {{"prefetch_size", A_LONG}, {"prefetch_count", A_SHORT}, {"global_", A_BIT}});
  m(60, 11, "basic.qos_ok");
  m(60, 20, "basic.consume", {{"ticket", A_SHORT}, {"queue", A_SHORTSTR}, {"consumer_tag", A_SHORTSTR},
                              {"no_local", A_BIT}, {"no_ack", A_BIT}, {"exclusive", A_BIT}, {"nowait", A_BIT},
                              {"arguments", A_TABLE}});
  m(60, 21, "basic.consume_ok", {{"consumer_tag", A_SHORTSTR}});
  m(60, 30, "basic.cancel", {{"consumer_tag", A_SHORTSTR}, {"nowait", A_BIT}});
  m(60, 31, "basic.cancel_ok", {{"consumer_tag", A_SHORTSTR}});
  m(60, 40, "basic.publish", {{"ticket", A_SHORT}, {"exchange", A_SHORTSTR}, {"routing_key", A_SHORTSTR},
                              {"mandatory", A_BIT}, {"immediate", A_BIT}}, true);
  m(60, 50, "basic.return", {{"reply_code", A_SHORT}, {"reply_text", A_SHORTSTR}, {"exchange", A_SHORTSTR},
                             {"routing_key", A_SHORTSTR}}, true);
  m(60, 60, "basic.deliver", {{"consumer_tag", A_SHORTSTR}, {"delivery_tag", A_LONGLONG}, {"redelivered", A_BIT},
                              {"exchange", A_SHORTSTR}, {"routing_key", A_SHORTSTR}}, true);
  m(60, 70, "basic.get", {{"ticket", A_SHORT}, {"queue", A_SHORTSTR}, {"no_ack", A_BIT}});
  m(60, 71, "basic.get_ok", {{"delivery_tag", A_LONGLONG}, {"redelivered", A_BIT}, {"exchange", A_SHORTSTR},
                             {"routing_key", A_SHORTSTR}, {"message_count", A_LONG}}, true);
  m(60, 72, "basic.get_empty", {{"cluster_id", A_SHORTSTR}});
  m(60, 80, "basic.ack", {{"delivery_tag", A_LONGLONG}, {"multiple", A_BIT}});
  m(60, 90, "basic.reject", {{"delivery_tag", A_LONGLONG}, {"requeue", A_BIT}});
  m(60, 100, "basic.recover_async", {{"requeue", A_BIT}});
  m(60, 110, "basic.recover", {{"requeue", A_BIT}});
  m(60, 111, "basic.recover_ok");
  m(60, 120, "basic.nack", {{"delivery_tag", A_LONGLONG}, {"multiple", A_BIT}, {"requeue", A_BIT}});
  m(85, 10, "confirm.select", {{"nowait", A_BIT}});
  m(85, 11, "confirm.select_ok");
  m(90, 10, "tx.select");
  m(90, 11, "tx.select_ok");
  m(90, 20, "tx.commit");
  m(90, 21, "tx.commit_ok");
  m(90, 30, "tx.rollback");
  m(90, 31, "tx.rollback_ok");
  return T;
}

const std::vector<MethodSpec>& method_table() {
  static const std::vector<MethodSpec> T = build_table();
  return T;
}

const MethodSpec* find_method(u16 cls, u16 mid) {
  static std::map<u32, const MethodSpec*> idx = [] {
    std::map<u32, const MethodSpec*> m;
    for (auto& s : method_table()) m[(u32(s.cls) << 16) | s.mid] = &s;
    return m;
  }();
  auto it = idx.find((u32(cls) << 16) | mid);
  return it == idx.end() ? nullptr : it->second;
}

Method decode_method(const u8* p, size_t n) {
  Reader r(p, n);
  u16 cls = r.shrt(), mid = r.shrt();
  const MethodSpec* spec = find_method(cls, mid);
  if (!spec) throw AmqpError(COMMAND_INVALID, "unknown class/method " + std::to_string(cls) + "/" +
                             std::to_string(mid), true, cls, mid);
  Method m;
  m.spec = spec;
  m.args.resize(spec->fields.size());
  for (size_t k = 0; k < spec->fields.size(); ++k) {
    Arg& a = m.args[k];
    switch (spec->fields[k].second) {
      case A_BIT: a.i = r.bit(); break;
      case A_OCTET: a.i = r.octet(); break;
      case A_SHORT: a.i = r.shrt(); break;
      case A_LONG: a.i = r.lng(); break;
      case A_LONGLONG: case A_TIMESTAMP: a.i = (i64)r.llng(); break;
      case A_SHORTSTR: a.s = r.shortstr(); break;
      case A_LONGSTR: a.s = r.longstr(); break;
      case A_TABLE: a.t = r.table(); break;
    }
  }
  return m;
}

Method make_method(u16 cls, u16 mid) {
  Method m;
  m.spec = find_method(cls, mid);
  if (!m.spec) throw std::runtime_error("make_method: unknown method");
  m.args.resize(m.spec->fields.size());
  return m;
}

std::string encode_method_payload(const Method& m) {
  Writer w;
  w.shrt(m.cls());
  w.shrt(m.mid());
  for (size_t k = 0; k < m.spec->fields.size(); ++k) {
    const Arg& a = m.args[k];
    switch (m.spec->fields[k].second) {
      case A_BIT: w.bit(a.i != 0); break;
      case A_OCTET: w.octet((u8)a.i); break;
      case A_SHORT: w.shrt((u16)a.i); break;
      case A_LONG: w.lng((u32)a.i); break;
      case A_LONGLONG: case A_TIMESTAMP: w.llng((u64)a.i); break;
      case A_SHORTSTR: w.shortstr(a.s); break;
      case A_LONGSTR: w.longstr(a.s); break;
      case A_TABLE: w.table(a.t); break;
    }
  }
  return w.done();
}

// ------------------------------------------------------------------ frames
void append_frame(std::string& out, u8 type, u16 ch, const char* payload, size_t n) {
  char h[7] = {(char)type, (char)(ch >> 8), (char)ch, (char)(n >> 24), (char)(n >> 16), (char)(n >> 8), (char)n};
  out.append(h, 7);
  out.append(payload, n);
  out.push_back((char)FRAME_END);
}

void append_method_frame(std::string& out, u16 ch, const Method& m) {
  std::string p = encode_method_payload(m);
  append_frame(out, FRAME_METHOD, ch, p.data(), p.size());
}

void append_content(std::string& out, u16 ch, u16 cls, const std::string& props, const std::string& body,
                    u32 frame_max) {
  char h[12] = {(char)(cls >> 8), (char)cls, 0, 0};
  u64 bs = body.size();
  for (int i = 0; i < 8; ++i) h[4 + i] = (char)(bs >> (56 - 8 * i));
  size_t n = 12 + props.size();
  char fh[7] = {(char)FRAME_HEADER, (char)(ch >> 8), (char)ch, (char)(n >> 24), (char)(n >> 16), (char)(n >> 8), (char)n};
  out.append(fh, 7);
  out.append(h, 12);
  out += props;
  out.push_back((char)FRAME_END);
  size_t step = frame_max ? frame_max - 8 : body.size();
  if (step == 0) step = body.size();
  for (size_t o = 0; o < body.size(); o += step) {
    size_t k = std::min(step, body.size() - o);
    append_frame(out, FRAME_BODY, ch, body.data() + o, k);
  }
}

Props parse_props(const std::string& raw) {
  Props pr;
  Reader r((const u8*)raw.data(), raw.size());
  std::vector<bool> present;
  while (true) {
    u16 f = r.shrt();
    for (int b = 15; b >= 1; --b) present.push_back((f >> b) & 1);
    if (!(f & 1)) break;
  }
  present.resize(std::max<size_t>(present.size(), 14));
  // order: ctype, cenc, headers, dmode, prio, corr, replyto, expiration, msgid, timestamp, type, user, app, cluster
  if (present[0]) r.shortstr();
  if (present[1]) r.shortstr();
  if (present[2]) { pr.headers = r.table(); pr.has_headers = true; }
  if (present[3]) pr.delivery_mode = r.octet();
  if (present[4]) pr.priority = r.octet();
  if (present[5]) r.shortstr();
  if (present[6]) r.shortstr();
  if (present[7]) {
    std::string e = r.shortstr();
    i64 v = 0;
    bool ok = !e.empty() && e.size() <= 18;
    for (char c : e) { if (c < '0' || c > '9') { ok = false; break; } v = v * 10 + (c - '0'); }
    if (ok) { pr.has_expiration = true; pr.expiration_ms = v; }
  }
  if (present[8]) r.shortstr();
  if (present[9]) { pr.has_timestamp = true; pr.timestamp = r.llng(); }
  return pr;
}

std::string encode_props_simple(int delivery_mode, const std::string& content_type) {
  Writer w;
  u16 flags = 0;
  if (!content_type.empty()) flags |= 1u << 15;
  if (delivery_mode) flags |= 1u << 12;
  w.shrt(flags);
  if (!content_type.empty()) w.shortstr(content_type);
  if (delivery_mode) w.octet((u8)delivery_mode);
  return w.done();
}

bool FrameParser::next(const std::string& buf, size_t& pos, Frame& out) {
  if (buf.size() - pos < 7) return false;
  const u8* p = (const u8*)buf.data() + pos;
  u8 type = p[0];
  u16 ch = (u16(p[1]) << 8) | p[2];
  u32 size = (u32(p[3]) << 24) | (u32(p[4]) << 16) | (u32(p[5]) << 8) | p[6];
  if (type != FRAME_METHOD && type != FRAME_HEADER && type != FRAME_BODY && type != FRAME_HEARTBEAT)
    throw AmqpError(FRAME_ERROR, "bad frame type " + std::to_string(type), true);
  if (frame_max_ && (u64)size + 8 > frame_max_)
    throw AmqpError(FRAME_ERROR, "frame larger than negotiated frame-max", true);
  if (buf.size() - pos < (size_t)size + 8) return false;
  if (p[7 + size] != FRAME_END) throw AmqpError(FRAME_ERROR, "bad frame end marker", true);
  out.type = type;
  out.ch = ch;
  out.payload.assign((const char*)p + 7, size);
  pos += size + 8;
  return true;
}

}  // namespace cmq

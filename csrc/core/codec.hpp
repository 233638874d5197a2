// AMQP 0-9-1 codec for the native broker (host control plane + CPU data path).
//
// Mirrors chanamq_amd/protocol (the golden Python codec): method table in the same
// order as methods.py, field tables with tags S I D T F A b d f l s t x V (+ B u i),
// LSB-first bit packing, 14 basic properties with a u16 flag chain.
// Reference behaviour: chana-mq-base/.../method/*.scala, model/Value{Reader,Writer}.scala,
// model/BasicProperties.scala, model/Frame.scala.
#pragma once
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace cmq {

using u8 = uint8_t;
using u16 = uint16_t;
using u32 = uint32_t;
using u64 = uint64_t;
using i64 = int64_t;

enum FrameType : u8 { FRAME_METHOD = 1, FRAME_HEADER = 2, FRAME_BODY = 3, FRAME_HEARTBEAT = 8 };
constexpr u8 FRAME_END = 0xCE;
static const char PROTOCOL_HEADER[8] = {'A', 'M', 'Q', 'P', 0, 0, 9, 1};

enum Reply : u16 {
  REPLY_SUCCESS = 200, CONTENT_TOO_LARGE = 311, NO_ROUTE = 312, NO_CONSUMERS = 313, CONNECTION_FORCED = 320,
  INVALID_PATH = 402, ACCESS_REFUSED = 403, NOT_FOUND = 404, RESOURCE_LOCKED = 405, PRECONDITION_FAILED = 406,
  FRAME_ERROR = 501, SYNTAX_ERROR = 502, COMMAND_INVALID = 503, CHANNEL_ERROR = 504, UNEXPECTED_FRAME = 505,
  RESOURCE_ERROR = 506, NOT_ALLOWED = 530, NOT_IMPLEMENTED = 540, INTERNAL_ERROR = 541
};

struct AmqpError : std::runtime_error {
  u16 code;
  bool connection;  // connection-level (true) or channel-level (false)
  u16 cls, mid;
  AmqpError(u16 c, const std::string& t, bool conn, u16 cl = 0, u16 m = 0)
      : std::runtime_error(t), code(c), connection(conn), cls(cl), mid(m) {}
};

// ------------------------------------------------------------------ field values
struct Value;
using Table = std::vector<std::pair<std::string, Value>>;  // insertion-ordered, first key wins
using Array = std::vector<Value>;

struct Value {
  char tag = 'V';
  i64 i = 0;            // integer tags, bool, timestamp
  double d = 0;         // 'd' 'f'
  u8 scale = 0;         // 'D'
  std::string s;        // 'S' 'x'
  std::shared_ptr<Table> t;
  std::shared_ptr<Array> a;
  static Value str(const std::string& v) { Value x; x.tag = 'S'; x.s = v; return x; }
  static Value boolean(bool v) { Value x; x.tag = 't'; x.i = v; return x; }
  static Value i32(i64 v) { Value x; x.tag = 'I'; x.i = v; return x; }
  static Value table(const Table& v) { Value x; x.tag = 'F'; x.t = std::make_shared<Table>(v); return x; }
};

const Value* table_get(const Table& t, const std::string& k);
bool value_as_int(const Value& v, i64* out);

// ------------------------------------------------------------------ byte io
struct Reader {
  const u8* p;
  size_t n, pos = 0;
  u8 bits = 0, nbits = 0;
  Reader(const u8* data, size_t len) : p(data), n(len) {}
  void need(size_t k) {
    if (pos + k > n) throw AmqpError(FRAME_ERROR, "truncated frame payload", true);
  }
  void clear_bits() { nbits = 0; }
  bool bit();
  u8 octet() { clear_bits(); need(1); return p[pos++]; }
  u16 shrt() { clear_bits(); need(2); u16 v = (u16(p[pos]) << 8) | p[pos + 1]; pos += 2; return v; }
  u32 lng() { clear_bits(); need(4); u32 v = (u32(p[pos]) << 24) | (u32(p[pos + 1]) << 16) | (u32(p[pos + 2]) << 8) | p[pos + 3]; pos += 4; return v; }
  u64 llng() { u64 hi = lng(); return (hi << 32) | lng(); }
  std::string shortstr() { u8 k = octet(); need(k); std::string s((const char*)p + pos, k); pos += k; return s; }
  std::string longstr() { u32 k = lng(); need(k); std::string s((const char*)p + pos, k); pos += k; return s; }
  Table table();
  Value value();
};

struct Writer {
  std::string b;
  u8 bits = 0, nbits = 0;
  void flush_bits() { if (nbits) { b.push_back((char)bits); bits = 0; nbits = 0; } }
  void bit(bool v) { if (nbits == 8) flush_bits(); if (v) bits |= (u8)(1u << nbits); ++nbits; }
  void octet(u8 v) { flush_bits(); b.push_back((char)v); }
  void shrt(u16 v) { flush_bits(); b.push_back((char)(v >> 8)); b.push_back((char)v); }
  void lng(u32 v) { flush_bits(); for (int s = 24; s >= 0; s -= 8) b.push_back((char)(v >> s)); }
  void llng(u64 v) { lng((u32)(v >> 32)); lng((u32)v); }
  void shortstr(const std::string& s) {
    if (s.size() > 255) throw AmqpError(SYNTAX_ERROR, "shortstr longer than 255 bytes", true);
    octet((u8)s.size()); b += s;
  }
  void longstr(const std::string& s) { lng((u32)s.size()); b += s; }
  void table(const Table& t);
  void value(const Value& v);
  std::string& done() { flush_bits(); return b; }
};

// ------------------------------------------------------------------ methods
enum ArgType : u8 { A_BIT, A_OCTET, A_SHORT, A_LONG, A_LONGLONG, A_SHORTSTR, A_LONGSTR, A_TABLE, A_TIMESTAMP };

struct MethodSpec {
  u16 cls, mid;
  const char* name;
  std::vector<std::pair<const char*, ArgType>> fields;
  bool content;
};

struct Arg {
  i64 i = 0;
  std::string s;
  Table t;
};

struct Method {
  const MethodSpec* spec = nullptr;
  std::vector<Arg> args;
  u16 cls() const { return spec->cls; }
  u16 mid() const { return spec->mid; }
  i64 i(size_t k) const { return args[k].i; }
  bool b(size_t k) const { return args[k].i != 0; }
  const std::string& s(size_t k) const { return args[k].s; }
  const Table& t(size_t k) const { return args[k].t; }
};

const MethodSpec* find_method(u16 cls, u16 mid);
const std::vector<MethodSpec>& method_table();
Method decode_method(const u8* p, size_t n);

// builder: Method m = make_method(60, 60); m.args[0].s = ...
Method make_method(u16 cls, u16 mid);
std::string encode_method_payload(const Method& m);

// ------------------------------------------------------------------ frames / content
void append_frame(std::string& out, u8 type, u16 ch, const char* payload, size_t n);
void append_method_frame(std::string& out, u16 ch, const Method& m);
// content header payload = class u16 | weight 0 | body size u64 | props (flags + values, verbatim)
void append_content(std::string& out, u16 ch, u16 cls, const std::string& props, const std::string& body,
                    u32 frame_max);
extern const char HEARTBEAT_FRAME[8];

struct Props {        // the fields the broker acts on; the raw bytes are re-emitted verbatim
  int delivery_mode = 0;
  int priority = -1;
  bool has_expiration = false;
  i64 expiration_ms = 0;
  bool has_timestamp = false;
  u64 timestamp = 0;  // seconds (wire)
  bool has_headers = false;
  Table headers;
};
Props parse_props(const std::string& raw);   // throws on malformed
std::string encode_props_simple(int delivery_mode, const std::string& content_type = "");

// streaming frame splitter with carry-over (FrameParser.scala:67-157)
struct Frame {
  u8 type;
  u16 ch;
  std::string payload;
};
class FrameParser {
 public:
  explicit FrameParser(u32 frame_max = 0) : frame_max_(frame_max) {}
  void set_frame_max(u32 fm) { frame_max_ = fm; }
  // parses as many complete frames as possible from buf[pos..]; returns false when
  // more bytes are needed. Throws AmqpError(FRAME_ERROR) on malformed input.
  bool next(const std::string& buf, size_t& pos, Frame& out);
 private:
  u32 frame_max_;
};

}  // namespace cmq

// Host-side process compiler: BPMN 2.0 XML -> flat CSR transition tables.
//
// Restates the deploy-time transformation of the reference
// (engine/src/main/java/io/camunda/zeebe/engine/processing/deployment/model/transformation/
// BpmnTransformer.java:109-127) for the supported element subset:
//  - FlowElementInstantiationTransformer.java:37-60: one executable element per flow node/flow;
//  - ModelWalker.walk (bpmn-model/.../traversal/ModelWalker.java:60-81) pushes siblings with
//    addFirst, so SequenceFlowTransformer.connectWithFlowNodes runs over the flows in REVERSE
//    document order: that fixes every getOutgoing()/getIncoming() order;
//  - SequenceFlowTransformer.parseCondition runs before connect, so ExecutableExclusiveGateway
//    .addOutgoing sees the condition (outgoingWithCondition keeps outgoing order);
//  - ExclusiveGatewayTransformer: default flow;
//  - StartEventTransformer.java:40 / EndEventTransformer.java:37: event type NONE.
// FEEL conditions (`=`-prefixed, FeelExpressionLanguage.parseExpression) are lowered to the
// postfix bytecode of include/zbhip.h; anything outside the typed comparison subset is rejected
// at deploy time (ZBHIP_EUNSUPP) rather than evaluated differently on the device.
#include <algorithm>
#include <cctype>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/zbhip.h"

namespace zbc {

// ---------------------------------------------------------------------------
// XML: a compact pull tokenizer building an element tree (prefixes dropped).
// ---------------------------------------------------------------------------
struct Elem {
  std::string tag;
  std::vector<std::pair<std::string, std::string>> attrs;
  std::string text;
  std::vector<Elem> children;
  const std::string* get(const char* name) const {
    for (auto& a : attrs)
      if (a.first == name) return &a.second;
    return nullptr;
  }
  const Elem* first(const char* tag_name) const {
    for (auto& c : children)
      if (c.tag == tag_name) return &c;
    return nullptr;
  }
};

class Xml {
 public:
  Xml(const char* s, size_t n) : p_(s), end_(s + n) {}
  bool parse(Elem& root, std::string& err) {
    skip_prolog();
    if (!element(root)) {
      err = err_.empty() ? "malformed XML" : err_;
      return false;
    }
    return true;
  }

 private:
  const char* p_;
  const char* end_;
  std::string err_;

  static std::string local(const std::string& q) {
    size_t c = q.rfind(':');
    return c == std::string::npos ? q : q.substr(c + 1);
  }
  bool starts(const char* lit) const {
    size_t n = strlen(lit);
    return (size_t)(end_ - p_) >= n && memcmp(p_, lit, n) == 0;
  }
  bool skip_to(const char* lit) {
    size_t n = strlen(lit);
    while (p_ + n <= end_) {
      if (memcmp(p_, lit, n) == 0) {
        p_ += n;
        return true;
      }
      ++p_;
    }
    return false;
  }
  void ws() {
    while (p_ < end_ && isspace((unsigned char)*p_)) ++p_;
  }
  void skip_prolog() {
    for (;;) {
      ws();
      if (starts("<?")) { skip_to("?>"); continue; }
      if (starts("<!--")) { skip_to("-->"); continue; }
      if (starts("<!")) { skip_to(">"); continue; }
      return;
    }
  }
  static void decode_into(std::string& out, const char* b, const char* e) {
    while (b < e) {
      if (*b != '&') { out += *b++; continue; }
      const char* semi = (const char*)memchr(b, ';', e - b);
      if (!semi) { out += *b++; continue; }
      std::string ent(b + 1, semi);
      if (ent == "lt") out += '<';
      else if (ent == "gt") out += '>';
      else if (ent == "amp") out += '&';
      else if (ent == "quot") out += '"';
      else if (ent == "apos") out += '\'';
      else if (ent.size() > 1 && ent[0] == '#') {
        long v = ent[1] == 'x' ? strtol(ent.c_str() + 2, nullptr, 16) : strtol(ent.c_str() + 1, nullptr, 10);
        if (v > 0 && v < 128) out += (char)v;
      }
      b = semi + 1;
    }
  }
  bool element(Elem& el) {
    if (p_ >= end_ || *p_ != '<') { err_ = "expected '<'"; return false; }
    ++p_;
    const char* s = p_;
    while (p_ < end_ && !isspace((unsigned char)*p_) && *p_ != '>' && *p_ != '/') ++p_;
    el.tag = local(std::string(s, p_));
    for (;;) {
      ws();
      if (p_ >= end_) { err_ = "unterminated tag"; return false; }
      if (*p_ == '/') {
        if (p_ + 1 >= end_ || p_[1] != '>') { err_ = "bad empty tag"; return false; }
        p_ += 2;
        return true;
      }
      if (*p_ == '>') { ++p_; break; }
      const char* an = p_;
      while (p_ < end_ && *p_ != '=' && !isspace((unsigned char)*p_)) ++p_;
      std::string name = local(std::string(an, p_));
      ws();
      if (p_ >= end_ || *p_ != '=') { err_ = "attribute without value"; return false; }
      ++p_;
      ws();
      if (p_ >= end_ || (*p_ != '"' && *p_ != '\'')) { err_ = "unquoted attribute"; return false; }
      char q = *p_++;
      const char* vb = p_;
      while (p_ < end_ && *p_ != q) ++p_;
      if (p_ >= end_) { err_ = "unterminated attribute"; return false; }
      std::string v;
      decode_into(v, vb, p_);
      ++p_;
      el.attrs.emplace_back(std::move(name), std::move(v));
    }
    for (;;) {
      if (p_ >= end_) { err_ = "unterminated element <" + el.tag + ">"; return false; }
      if (starts("</")) {
        if (!skip_to(">")) { err_ = "unterminated end tag"; return false; }
        return true;
      }
      if (starts("<![CDATA[")) {
        p_ += 9;
        const char* b = p_;
        if (!skip_to("]]>")) { err_ = "unterminated CDATA"; return false; }
        el.text.append(b, p_ - 3);
        continue;
      }
      if (starts("<!--")) { skip_to("-->"); continue; }
      if (starts("<?")) { skip_to("?>"); continue; }
      if (*p_ == '<') {
        el.children.emplace_back();
        if (!element(el.children.back())) return false;
        continue;
      }
      const char* b = p_;
      while (p_ < end_ && *p_ != '<') ++p_;
      decode_into(el.text, b, p_);
    }
  }
};

// ---------------------------------------------------------------------------
// FEEL subset -> postfix bytecode
// ---------------------------------------------------------------------------
class FeelCompiler {
 public:
  FeelCompiler(const std::string& src, std::vector<zbhip_insn>& code,
               std::function<uint32_t(const std::string&)> name_of)
      : s_(src), code_(code), name_of_(std::move(name_of)) {}

  bool compile(std::string& err) {
    if (!disj()) { err = "FEEL outside the supported subset: " + s_; return false; }
    ws();
    if (i_ != s_.size()) { err = "FEEL outside the supported subset (trailing input): " + s_; return false; }
    emit(ZBHIP_OP_END, 0, 0);
    return true;
  }

 private:
  const std::string& s_;
  size_t i_ = 0;
  std::vector<zbhip_insn>& code_;
  std::function<uint32_t(const std::string&)> name_of_;

  void emit(uint8_t op, uint32_t arg, int64_t lit) {
    zbhip_insn in{};
    in.op = op;
    in.arg = arg;
    in.literal = lit;
    code_.push_back(in);
  }
  void ws() { while (i_ < s_.size() && isspace((unsigned char)s_[i_])) ++i_; }
  static bool ident_char(char c) { return isalnum((unsigned char)c) || c == '_'; }
  bool keyword(const char* w) {
    ws();
    size_t n = strlen(w);
    if (s_.compare(i_, n, w) != 0) return false;
    if (i_ + n < s_.size() && ident_char(s_[i_ + n])) return false;
    i_ += n;
    return true;
  }
  bool disj() {
    if (!conj()) return false;
    while (keyword("or")) {
      if (!conj()) return false;
      emit(ZBHIP_OP_OR, 0, 0);
    }
    return true;
  }
  bool conj() {
    if (!comparison()) return false;
    while (keyword("and")) {
      if (!comparison()) return false;
      emit(ZBHIP_OP_AND, 0, 0);
    }
    return true;
  }
  bool comparison() {
    if (!operand()) return false;
    ws();
    struct { const char* t; uint8_t op; } ops[] = {{"<=", ZBHIP_OP_LE}, {">=", ZBHIP_OP_GE}, {"!=", ZBHIP_OP_NE},
                                                   {"<", ZBHIP_OP_LT}, {">", ZBHIP_OP_GT}, {"=", ZBHIP_OP_EQ}};
    for (auto& o : ops) {
      size_t n = strlen(o.t);
      if (s_.compare(i_, n, o.t) == 0) {
        i_ += n;
        if (!operand()) return false;
        emit(o.op, 0, 0);
        return true;
      }
    }
    return true;
  }
  bool operand() {
    ws();
    if (i_ >= s_.size()) return false;
    if (s_[i_] == '(') {
      ++i_;
      if (!disj()) return false;
      ws();
      if (i_ >= s_.size() || s_[i_] != ')') return false;
      ++i_;
      return true;
    }
    if (keyword("not")) {
      ws();
      if (i_ >= s_.size() || s_[i_] != '(') return false;
      ++i_;
      if (!disj()) return false;
      ws();
      if (i_ >= s_.size() || s_[i_] != ')') return false;
      ++i_;
      emit(ZBHIP_OP_NOT, 0, 0);
      return true;
    }
    if (keyword("true")) { emit(ZBHIP_OP_PUSH_BOOL, 1, 0); return true; }
    if (keyword("false")) { emit(ZBHIP_OP_PUSH_BOOL, 0, 0); return true; }
    if (keyword("null")) { emit(ZBHIP_OP_PUSH_NULL, 0, 0); return true; }
    bool neg = false;
    if (s_[i_] == '-') { neg = true; ++i_; }
    if (i_ < s_.size() && (isdigit((unsigned char)s_[i_]) || s_[i_] == '.')) {
      // exact decimal literal, scaled by 10^ZBHIP_DEC_SCALE
      __int128 v = 0;
      int frac = -1;
      for (; i_ < s_.size() && (isdigit((unsigned char)s_[i_]) || s_[i_] == '.'); ++i_) {
        if (s_[i_] == '.') {
          if (frac >= 0) return false;
          frac = 0;
          continue;
        }
        if (frac >= 0 && ++frac > ZBHIP_DEC_SCALE) return false;  // not exactly representable
        v = v * 10 + (s_[i_] - '0');
        if (v > ((__int128)1 << 62)) return false;
      }
      for (int k = frac < 0 ? 0 : frac; k < ZBHIP_DEC_SCALE; ++k) v *= 10;
      if (v > (__int128)INT64_MAX) return false;
      emit(ZBHIP_OP_PUSH_NUM, 0, neg ? -(int64_t)v : (int64_t)v);
      return true;
    }
    if (neg) return false;
    if (isalpha((unsigned char)s_[i_]) || s_[i_] == '_') {
      size_t b = i_;
      while (i_ < s_.size() && ident_char(s_[i_])) ++i_;
      std::string name = s_.substr(b, i_ - b);
      ws();
      if (i_ < s_.size() && (s_[i_] == '.' || s_[i_] == '[' || s_[i_] == '(')) return false;  // paths, calls
      emit(ZBHIP_OP_PUSH_VAR, name_of_(name), 0);
      return true;
    }
    return false;
  }
};

// ---------------------------------------------------------------------------
// The compiled process (owns the storage the CSR view points into)
// ---------------------------------------------------------------------------
struct Compiled {
  zbhip_process_csr csr{};
  std::vector<zbhip_element> elements;
  std::vector<uint16_t> out_flow;
  std::vector<uint32_t> cond_begin;
  std::vector<std::string> cond_texts;
  std::vector<const char*> cond_ptrs;
  std::vector<zbhip_insn> code;
  std::vector<zbhip_mapping> mappings;
  std::vector<std::string> headers;  // per element: its customHeaders msgpack map ("" = NO_HEADERS)
  std::vector<uint32_t> header_begin;
  std::vector<uint8_t> header_bytes;
  std::vector<std::string> strings;
  std::vector<const char*> string_ptrs;
  std::unordered_map<std::string, uint16_t> string_ids;

  uint16_t str(const std::string& s) {
    auto it = string_ids.find(s);
    if (it != string_ids.end()) return it->second;
    uint16_t id = (uint16_t)strings.size();
    strings.push_back(s);
    string_ids.emplace(s, id);
    return id;
  }
  void finish() {
    string_ptrs.clear();
    for (auto& s : strings) string_ptrs.push_back(s.c_str());
    csr.n_elements = (uint32_t)elements.size();
    csr.elements = elements.data();
    csr.n_out = (uint32_t)out_flow.size();
    csr.out_flow = out_flow.data();
    csr.n_conditions = cond_begin.empty() ? 0 : (uint32_t)cond_begin.size() - 1;
    csr.cond_begin = cond_begin.data();
    cond_ptrs.clear();
    for (auto& t : cond_texts) cond_ptrs.push_back(t.c_str());
    csr.n_mappings = (uint32_t)mappings.size();
    csr.mappings = mappings.data();
    csr.cond_text = cond_ptrs.data();
    csr.n_code = (uint32_t)code.size();
    csr.code = code.data();
    csr.n_strings = (uint32_t)strings.size();
    csr.strings = string_ptrs.data();
    header_begin.clear();
    header_bytes.clear();
    headers.resize(elements.size());
    bool any = false;
    for (auto& h : headers) any |= !h.empty();
    if (any) {
      for (auto& h : headers) {
        header_begin.push_back((uint32_t)header_bytes.size());
        header_bytes.insert(header_bytes.end(), h.begin(), h.end());
      }
      header_begin.push_back((uint32_t)header_bytes.size());
    }
    csr.header_begin = any ? header_begin.data() : nullptr;
    csr.header_bytes = any ? header_bytes.data() : nullptr;
  }
};

// String.hashCode (java.lang.String): s[0]*31^(n-1) + ... over the UTF-16 code units of the UTF-8 text
static int32_t java_string_hash(const std::string& s) {
  uint32_t h = 0;
  auto unit = [&h](uint32_t u) { h = 31u * h + u; };
  for (size_t i = 0; i < s.size();) {
    const unsigned char c = (unsigned char)s[i];
    uint32_t cp;
    int n;
    if (c < 0x80) { cp = c; n = 1; }
    else if ((c >> 5) == 6) { cp = c & 0x1F; n = 2; }
    else if ((c >> 4) == 14) { cp = c & 0x0F; n = 3; }
    else { cp = c & 0x07; n = 4; }
    for (int k = 1; k < n && i + k < s.size(); ++k) cp = (cp << 6) | ((unsigned char)s[i + k] & 0x3F);
    i += n;
    if (cp >= 0x10000) {  // a surrogate pair
      cp -= 0x10000;
      unit(0xD800 + (cp >> 10));
      unit(0xDC00 + (cp & 0x3FF));
    } else {
      unit(cp);
    }
  }
  return (int32_t)h;
}

// MsgPackWriter.writeString / writeMapHeader (msgpack-core/.../MsgPackWriter.java): fixstr / str8 / str16 /
// str32, fixmap / map16 / map32, big-endian lengths
static void mp_header(std::string& o, uint32_t n, uint8_t fix, uint32_t fix_max, uint8_t b8, uint8_t b16, uint8_t b32) {
  if (n <= fix_max) { o += (char)(fix | n); return; }
  if (b8 && n <= 0xFF) { o += (char)b8; o += (char)n; return; }
  if (n <= 0xFFFF) { o += (char)b16; o += (char)(n >> 8); o += (char)n; return; }
  o += (char)b32;
  for (int k = 3; k >= 0; --k) o += (char)(n >> (8 * k));
}

// zeebe:taskHeaders -> the customHeaders of the job worker's jobs.  TaskHeadersTransformer (deployment/
// model/transformer/zeebe/TaskHeadersTransformer.java:24-58) keeps the headers with a non-empty key and value
// (Collectors.toMap: a duplicate key fails the deployment -- refused here); BpmnJobBehavior.encodeHeaders
// copies them into a HashMap (:219-248) and HeaderEncoder.encode (:365-399) collects them into another,
// whose iteration order is written.  A java.util.HashMap iterates its buckets in index order and a bucket's
// entries in insertion order (a resize splits a bucket keeping it), the bucket being (h ^ h >>> 16) &
// (capacity - 1): the two default-constructed maps grow alike (16, doubled past 3/4 load), the pre-sized copy
// (JDK 21 HashMap(Map): tableSizeFor(ceil(size / 0.75))) has a capacity dividing theirs, so every map keeps
// ties in document order and the entries come out in document order stably sorted by the final bucket.  A
// bucket of 9 entries would turn into a tree (or force an extra resize): outside the subset.
static int encode_task_headers(const Elem& th, std::string& out, std::string& err) {
  std::vector<std::pair<std::string, std::string>> hs;
  for (auto& h : th.children) {
    if (h.tag != "header") continue;
    const std::string* k = h.get("key");
    const std::string* v = h.get("value");
    if (!k || !v || k->empty() || v->empty()) continue;  // isValidHeader
    for (auto& e : hs)
      if (e.first == *k) { err = "duplicate task header key '" + *k + "'"; return ZBHIP_EPARSE; }
    hs.push_back({*k, *v});
  }
  out.clear();
  if (hs.empty()) return ZBHIP_OK;  // no valid header: NO_HEADERS
  uint32_t cap = 16;
  while (hs.size() > cap / 4 * 3) cap *= 2;
  std::vector<std::pair<uint32_t, size_t>> order;
  uint32_t in16[16] = {};
  for (size_t i = 0; i < hs.size(); ++i) {
    const uint32_t h = (uint32_t)java_string_hash(hs[i].first);
    const uint32_t spread = h ^ (h >> 16);
    order.push_back({spread & (cap - 1), i});
    if (++in16[spread & 15] > 8) { err = "task headers that a HashMap would treeify"; return ZBHIP_EUNSUPP; }
  }
  std::stable_sort(order.begin(), order.end(), [](auto& a, auto& b) { return a.first < b.first; });
  mp_header(out, (uint32_t)hs.size(), 0x80, 15, 0, 0xDE, 0xDF);
  for (auto& [b, i] : order) {
    for (const std::string* t : {&hs[i].first, &hs[i].second}) {
      mp_header(out, (uint32_t)t->size(), 0xA0, 31, 0xD9, 0xDA, 0xDB);
      out += *t;
    }
  }
  return ZBHIP_OK;
}

// Interval.parse (bpmn-model/.../util/time/Interval.java) of a static duration
// "P[0D][T[nH][nM][n[.f]S]]": a Duration, so due = now + a fixed number of ms.  Days (a Period, which
// Interval.toEpochMilli adds in the broker's system zone), years, months, weeks, negative parts and
// `=` expressions: -1 (outside the subset).
static int64_t duration_ms(const std::string& text, bool days_exact = false) {
  size_t a = text.find_first_not_of(" \t\r\n"), b = text.find_last_not_of(" \t\r\n");
  if (a == std::string::npos) return -1;
  const std::string t = text.substr(a, b - a + 1);
  if (t.size() < 3 || t[0] != 'P') return -1;
  int64_t ms = 0;
  bool in_time = false, any = false;
  for (size_t i = 1; i < t.size();) {
    if (t[i] == 'T') {
      if (in_time) return -1;
      in_time = true;
      ++i;
      continue;
    }
    const size_t s = i;
    int64_t whole = 0, frac = 0;
    int digits = 0;
    while (i < t.size() && isdigit((unsigned char)t[i])) {
      whole = whole * 10 + (t[i++] - '0');
      if (whole > (1LL << 40)) return -1;
    }
    if (i < t.size() && t[i] == '.') {
      ++i;
      while (i < t.size() && isdigit((unsigned char)t[i])) {
        if (digits < 3) { frac = frac * 10 + (t[i] - '0'); ++digits; }
        ++i;
      }
      for (; digits < 3; ++digits) frac *= 10;
    }
    if (i == s || i >= t.size()) return -1;
    const char u = t[i++];
    any = true;
    // days make the interval calendar-based (Interval.isCalendarBased): ZonedDateTime.plus in the
    // broker's system zone, so a DST change moves the due date by an hour -- outside the subset
    // (days_exact: a FEEL day-time duration, java.time.Duration -- a day is 24 h)
    if (!in_time && u == 'D' && !frac && (whole == 0 || days_exact)) ms += whole * 86400000LL;
    else if (in_time && u == 'H' && !frac) ms += whole * 3600000LL;
    else if (in_time && u == 'M' && !frac) ms += whole * 60000LL;
    else if (in_time && u == 'S') ms += whole * 1000LL + frac;
    else return -1;
  }
  return any ? ms : -1;
}

// A timer's timeDuration / timeCycle text -> (milliseconds, repetitions): the static forms, and the
// constant FEEL expressions ExpressionProcessor.evaluateIntervalExpression (processing/common/
// ExpressionProcessor.java:142-175) turns into the same Interval -- `=duration("d")` (a FEEL day-time
// duration: new Interval(Duration), days of 24 h), `="d"` (a string: Interval.parse, as the static
// form) -- and for a cycle the strings FeelFunctionProvider.cycle builds (feel/.../
// FeelFunctionProvider.scala:23-47): `=cycle(duration("d"))` = "R/d", `=cycle(n, duration("d"))` =
// "Rn/d".  reps: 1 for a duration, 255 for an infinite cycle.  Expressions naming variables, year-month
// durations and calendar days stay outside the subset (-1).
static std::string trim(const std::string& t) {
  const size_t a = t.find_first_not_of(" \t\r\n"), b = t.find_last_not_of(" \t\r\n");
  return a == std::string::npos ? std::string() : t.substr(a, b - a + 1);
}
// `name(args)` -> args, or false
static bool call_args(const std::string& t, const char* name, std::string& args) {
  const size_t n = strlen(name);
  if (t.compare(0, n, name) != 0) return false;
  const std::string r = trim(t.substr(n));
  if (r.size() < 2 || r.front() != '(' || r.back() != ')') return false;
  args = trim(r.substr(1, r.size() - 2));
  return true;
}
static bool string_literal(const std::string& t, std::string& v) {
  if (t.size() < 2 || t.front() != '"' || t.back() != '"') return false;
  v = t.substr(1, t.size() - 2);
  return v.find_first_of("\"\\") == std::string::npos;
}
static int64_t feel_interval_ms(const std::string& e) {  // a FEEL expression (after the `=`)
  std::string a, v;
  if (call_args(e, "duration", a) && string_literal(a, v)) return duration_ms(v, true);
  if (string_literal(e, v)) return duration_ms(v);
  return -1;
}
static int64_t parse_repetitions(const std::string& n) {  // RepeatingInterval.parse's "Rn"
  if (n.empty()) return 255;
  if (n.size() > 3 || n.find_first_not_of("0123456789") != std::string::npos) return -1;
  const int r = atoi(n.c_str());
  return r >= 1 && r <= 254 ? r : -1;
}
static int64_t timer_ms(const std::string& text, bool cycle, uint32_t& reps) {
  const std::string t = trim(text);
  reps = 1;
  if (!cycle) return t.size() > 1 && t[0] == '=' ? feel_interval_ms(trim(t.substr(1))) : duration_ms(t);
  std::string r = t;
  if (t.size() > 1 && t[0] == '=') {
    const std::string e = trim(t.substr(1));
    std::string args, v;
    if (string_literal(e, v)) {
      r = v;
    } else if (call_args(e, "cycle", args)) {
      const size_t comma = args.find(',');
      const std::string n = comma == std::string::npos ? std::string() : trim(args.substr(0, comma));
      const int64_t rp = parse_repetitions(n);
      if (rp < 0) return -1;
      reps = (uint32_t)rp;
      return feel_interval_ms(trim(comma == std::string::npos ? args : args.substr(comma + 1)));
    } else {
      return -1;
    }
  }
  const size_t slash = r.find('/');
  if (r.size() < 3 || r[0] != 'R' || slash == std::string::npos || r.find('/', slash + 1) != std::string::npos)
    return -1;
  const int64_t rp = parse_repetitions(r.substr(1, slash - 1));
  if (rp < 0) return -1;
  reps = (uint32_t)rp;
  return duration_ms(r.substr(slash + 1));
}

// `= name`: a FEEL variable reference (no path, no call, no literal) -> name, else ""
static std::string feel_variable(const std::string& t) {
  size_t i = t.find_first_not_of(" \t\r\n");
  if (i == std::string::npos || t[i] != '=') return "";
  ++i;
  while (i < t.size() && isspace((unsigned char)t[i])) ++i;
  const size_t s0 = i;
  if (i >= t.size() || !(isalpha((unsigned char)t[i]) || t[i] == '_')) return "";
  while (i < t.size() && (isalnum((unsigned char)t[i]) || t[i] == '_')) ++i;
  const std::string v = t.substr(s0, i - s0);
  while (i < t.size() && isspace((unsigned char)t[i])) ++i;
  if (i != t.size() || v == "true" || v == "false" || v == "null" || v == "not") return "";
  return v;
}

// A multi-instance activity's loop characteristics (MultiInstanceActivityTransformer
// .transformLoopCharacteristics, deployment/model/transformer/MultiInstanceActivityTransformer.java:
// 80-122) in the subset: the inputCollection a static FEEL list literal of integer, string, boolean and
// null items (FeelToMessagePackTransformer writes a whole number as a msgpack integer) or a list
// variable (`= items`: coll_var), an optional inputElement, an outputCollection with an outputElement
// naming a variable (`= result`), and a completionCondition of the FEEL subset (its text after '=').
struct MiItem { uint8_t type; int64_t value; std::string text; };
struct MiLoop {
  bool seq = false;
  std::string input, coll_var, out_coll, out_elem, cond;
  std::vector<MiItem> items;
};
static bool parse_loop(const Elem& mil, MiLoop& L, std::string& err) {
  const std::string* sq = mil.get("isSequential");
  L.seq = sq && *sq == "true";
  bool& seq = L.seq;
  (void)seq;
  std::string& input = L.input;
  std::vector<MiItem>& items = L.items;
  if (const Elem* cc = mil.first("completionCondition")) {
    const size_t a = cc->text.find_first_not_of(" \t\r\n");
    if (a != std::string::npos) {
      const size_t b = cc->text.find_last_not_of(" \t\r\n");
      if (cc->text[a] != '=') { err = "static (non-FEEL) completionCondition outside the subset"; return false; }
      L.cond = cc->text.substr(a + 1, b - a);
    }
  }
  const Elem* ext = mil.first("extensionElements");
  const Elem* lc = ext ? ext->first("loopCharacteristics") : nullptr;
  if (!lc) { err = "multi-instance without zeebe:loopCharacteristics"; return false; }
  const std::string* oc = lc->get("outputCollection");
  const std::string* oe = lc->get("outputElement");
  if ((oc && !oc->empty()) || (oe && !oe->empty())) {
    L.out_elem = oe ? feel_variable(*oe) : "";
    if (!oc || oc->empty() || L.out_elem.empty()) {
      err = "multi-instance outputCollection / outputElement outside the supported subset (a variable)";
      return false;
    }
    L.out_coll = *oc;
  }
  const std::string* ie = lc->get("inputElement");
  input = ie ? *ie : "";
  const std::string* ic = lc->get("inputCollection");
  const std::string t = ic ? *ic : "";
  L.coll_var = feel_variable(t);
  if (!L.coll_var.empty()) return true;
  auto bad = [&]() { err = "multi-instance inputCollection outside the supported subset (a static list or a variable): " + t; return false; };
  size_t i = t.find_first_not_of(" \t\r\n");
  auto ws = [&]() { while (i < t.size() && isspace((unsigned char)t[i])) ++i; };
  if (i == std::string::npos || t[i] != '=') return bad();
  ++i;
  ws();
  if (i >= t.size() || t[i] != '[') return bad();
  ++i;
  ws();
  if (i < t.size() && t[i] == ']') {
    ++i;
  } else {
    for (;;) {
      ws();
      if (i >= t.size()) return bad();
      MiItem it{ZBHIP_DOC_INT, 0, ""};
      if (t[i] == '"') {
        const size_t e = t.find('"', i + 1);
        if (e == std::string::npos) return bad();
        it.type = ZBHIP_DOC_STR;
        it.text = t.substr(i + 1, e - i - 1);
        if (it.text.find('\\') != std::string::npos) return bad();
        i = e + 1;
      } else if (t.compare(i, 4, "true") == 0 || t.compare(i, 4, "null") == 0 || t.compare(i, 5, "false") == 0) {
        it.type = t[i] == 'n' ? ZBHIP_DOC_NIL : ZBHIP_DOC_BOOL;
        it.value = t[i] == 't';
        i += t[i] == 'f' ? 5 : 4;
      } else {
        const bool neg = t[i] == '-';
        if (neg) ++i;
        const size_t s0 = i;
        unsigned long long v = 0;
        for (; i < t.size() && isdigit((unsigned char)t[i]); ++i) {
          if (v > 922337203685477580ULL) return bad();
          v = v * 10 + (unsigned)(t[i] - '0');
        }
        if (i == s0 || v > 9223372036854775807ULL || (i < t.size() && (t[i] == '.' || isalpha((unsigned char)t[i]))))
          return bad();
        it.value = neg ? -(int64_t)v : (int64_t)v;
      }
      items.push_back(it);
      ws();
      if (i < t.size() && t[i] == ',') { ++i; continue; }
      if (i < t.size() && t[i] == ']') { ++i; break; }
      return bad();
    }
  }
  ws();
  if (i != t.size() || items.size() > 65535) return bad();
  return true;
}

// zeebe:ioMapping (VariableMappingTransformer.java:73-200) in the device subset (zbhip.h
// zbhip_mapping): one input and one output mapping at most, a plain target, a variable reference or a
// literal source (a source without '=' is a static string: StaticExpression, quoted at :176-180).
static int parse_mappings(const Elem* ext, uint16_t elem, Compiled& C, std::string& err) {
  const Elem* io = ext ? ext->first("ioMapping") : nullptr;
  if (!io) return ZBHIP_OK;
  auto trim = [](const std::string& t) {
    const size_t a = t.find_first_not_of(" \t\r\n"), b = t.find_last_not_of(" \t\r\n");
    return a == std::string::npos ? std::string() : t.substr(a, b - a + 1);
  };
  auto ident = [](const std::string& v) {
    bool ok = !v.empty() && (isalpha((unsigned char)v[0]) || v[0] == '_');
    for (char ch : v) ok = ok && (isalnum((unsigned char)ch) || ch == '_');
    return ok && v != "true" && v != "false" && v != "null";
  };
  bool seen[2] = {false, false};
  for (auto& m : io->children) {
    if (m.tag != "input" && m.tag != "output") continue;
    const int out = m.tag == "output";
    if (seen[out]) { err = "more than one " + m.tag + " mapping outside the supported subset (document order unpinned)"; return ZBHIP_EUNSUPP; }
    seen[out] = true;
    const std::string* tp = m.get("target");
    const std::string* sp = m.get("source");
    const std::string target = tp ? trim(*tp) : "";
    const std::string src = sp ? *sp : "";
    if (!ident(target)) { err = "io mapping target outside the supported subset: " + target; return ZBHIP_EUNSUPP; }
    zbhip_mapping M{};
    M.element = elem;
    M.output = (uint8_t)out;
    M.target = C.str(target);
    if (src.empty() || src[0] != '=') {
      M.source_type = ZBHIP_DOC_STR;
      M.source = C.str(src);
    } else {
      const std::string x = trim(src.substr(1));
      if (ident(x)) {
        M.source_type = ZBHIP_MAP_VARIABLE;
        M.source = C.str(x);
      } else if (x == "true" || x == "false") {
        M.source_type = ZBHIP_DOC_BOOL;
        M.literal = x == "true";
      } else if (x == "null") {
        M.source_type = ZBHIP_DOC_NIL;
      } else if (x.size() >= 2 && x.front() == '"' && x.back() == '"' && x.find('"', 1) == x.size() - 1 &&
                 x.find('\\') == std::string::npos) {
        M.source_type = ZBHIP_DOC_STR;
        M.source = C.str(x.substr(1, x.size() - 2));
      } else {
        size_t i = x.size() && x[0] == '-' ? 1 : 0;
        unsigned long long v = 0;
        bool ok = i < x.size();
        for (; ok && i < x.size(); ++i) {
          ok = isdigit((unsigned char)x[i]) && v <= 922337203685477580ULL;
          if (ok) v = v * 10 + (unsigned)(x[i] - '0');
        }
        if (!ok || v > 9223372036854775807ULL) { err = "io mapping source outside the supported subset: " + src; return ZBHIP_EUNSUPP; }
        M.source_type = ZBHIP_DOC_INT;
        M.literal = x[0] == '-' ? -(int64_t)v : (int64_t)v;
      }
    }
    C.mappings.push_back(M);
  }
  return ZBHIP_OK;
}

static zbhip_element blank(uint8_t type, uint16_t id) {
  zbhip_element e{};
  e.element_type = type;
  e.event_type = ZBHIP_EV_UNSPECIFIED;
  e.flow_source = e.flow_target = e.condition = e.default_flow = ZBHIP_NONE16;
  e.job_type = e.join_slot = ZBHIP_NONE16;
  e.flow_scope = 0;
  e.start_event = ZBHIP_NONE16;
  e.duration_ms = 0;
  e.message_name = e.correlation_var = ZBHIP_NONE16;
  e.job_retries = 0;
  e.id = id;
  return e;
}

static int compile(const char* xml, size_t len, int64_t def_key, int32_t version, Compiled& C,
                   std::string& err) {
  Elem root;
  Xml parser(xml, len);
  if (!parser.parse(root, err)) return ZBHIP_EPARSE;
  const Elem* proc = nullptr;
  for (auto& c : root.children) {
    if (c.tag != "process") continue;
    const std::string* ex = c.get("isExecutable");
    if (ex && *ex == "false") continue;
    proc = &c;
    break;
  }
  if (!proc || !proc->get("id")) { err = "no executable process"; return ZBHIP_EPARSE; }
  const std::string pid = *proc->get("id");
  // <message> elements of the definitions (MessageTransformer.java:30-60): static names and
  // `= variable` correlation keys only
  struct Msg { std::string name, corr; bool ok; std::string why; };
  std::unordered_map<std::string, Msg> messages;
  for (auto& c : root.children) {
    if (c.tag != "message" || !c.get("id")) continue;
    Msg m{"", "", true, ""};
    const std::string* nm = c.get("name");
    if (!nm || nm->empty() || (*nm)[0] == '=') { m.ok = false; m.why = "message name expression outside the subset"; }
    else m.name = *nm;
    const Elem* ext = c.first("extensionElements");
    const Elem* sub = ext ? ext->first("subscription") : nullptr;
    const std::string* ck = sub ? sub->get("correlationKey") : nullptr;
    std::string t = ck ? *ck : "";
    size_t a = t.find_first_not_of(" \t\r\n"), b = t.find_last_not_of(" \t\r\n");
    t = a == std::string::npos ? "" : t.substr(a, b - a + 1);
    if (t.size() < 2 || t[0] != '=') { m.ok = false; m.why = "correlation key must be a `= variable` expression"; }
    else {
      std::string v = t.substr(1);
      size_t va = v.find_first_not_of(" \t\r\n"), vb = v.find_last_not_of(" \t\r\n");
      v = va == std::string::npos ? "" : v.substr(va, vb - va + 1);
      bool ident = !v.empty() && (isalpha((unsigned char)v[0]) || v[0] == '_');
      for (char ch : v) ident = ident && (isalnum((unsigned char)ch) || ch == '_');
      if (!ident) { m.ok = false; m.why = "correlation key expression outside the subset (`= variable` only)"; }
      m.corr = v;
    }
    messages[*c.get("id")] = m;
  }
  // <error> elements of the definitions (ErrorTransformer): static error codes
  std::unordered_map<std::string, std::string> errors;
  for (auto& c : root.children)
    if (c.tag == "error" && c.get("id")) errors[*c.get("id")] = c.get("errorCode") ? *c.get("errorCode") : "";
  C.csr.bpmn_process_id = C.str(pid);
  C.elements.push_back(blank(ZBHIP_EL_PROCESS, C.csr.bpmn_process_id));
  C.elements[0].flow_scope = 0;
  std::unordered_map<std::string, uint16_t> index{{pid, 0}};
  std::vector<const Elem*> flows;
  std::vector<std::vector<uint16_t>> out_lists, in_lists;
  std::vector<const Elem*> xgws;
  std::vector<std::pair<uint16_t, std::string>> boundaries;  // (boundary event, attachedToRef)
  std::vector<std::pair<uint16_t, MiLoop>> collections;  // (multi-instance body, its loop characteristics)

  // Elements in document pre-order: an embedded sub-process, then its children, then its next
  // sibling (the oracle numbers them the same way).  Every sequence flow connects two nodes of one
  // container, so the flows' reverse document order per container is the walker's order.
  std::function<int(const Elem&, uint16_t)> container = [&](const Elem& parent, uint16_t scope) -> int {
    for (auto& c : parent.children) {
      uint8_t type;
      if (c.tag == "startEvent") type = ZBHIP_EL_START_EVENT;
      else if (c.tag == "endEvent") type = ZBHIP_EL_END_EVENT;
      else if (c.tag == "serviceTask") type = ZBHIP_EL_SERVICE_TASK;
      else if (c.tag == "sendTask") type = ZBHIP_EL_SEND_TASK;
      else if (c.tag == "scriptTask") type = ZBHIP_EL_SCRIPT_TASK;
      else if (c.tag == "businessRuleTask") type = ZBHIP_EL_BUSINESS_RULE_TASK;
      else if (c.tag == "exclusiveGateway") type = ZBHIP_EL_EXCLUSIVE_GATEWAY;
      else if (c.tag == "parallelGateway") type = ZBHIP_EL_PARALLEL_GATEWAY;
      else if (c.tag == "sequenceFlow") type = ZBHIP_EL_SEQUENCE_FLOW;
      else if (c.tag == "intermediateCatchEvent") type = ZBHIP_EL_INTERMEDIATE_CATCH_EVENT;
      else if (c.tag == "intermediateThrowEvent") type = ZBHIP_EL_INTERMEDIATE_THROW_EVENT;
      else if (c.tag == "task") type = ZBHIP_EL_TASK;
      else if (c.tag == "manualTask") type = ZBHIP_EL_MANUAL_TASK;
      else if (c.tag == "subProcess") {
        const std::string* tbe = c.get("triggeredByEvent");
        type = tbe && *tbe == "true" ? ZBHIP_EL_EVENT_SUB_PROCESS : ZBHIP_EL_SUB_PROCESS;
      }
      else if (c.tag == "boundaryEvent") type = ZBHIP_EL_BOUNDARY_EVENT;
      else if (c.tag == "extensionElements" || c.tag == "documentation" || c.tag == "textAnnotation" ||
               c.tag == "association" || c.tag == "incoming" || c.tag == "outgoing")
        continue;
      else { err = "element <" + c.tag + "> outside the supported subset"; return ZBHIP_EUNSUPP; }
      const std::string* id = c.get("id");
      if (!id || id->empty()) { err = "element without id"; return ZBHIP_EPARSE; }
      if (C.elements.size() >= 0xFF0) { err = "too many elements"; return ZBHIP_EUNSUPP; }
      zbhip_element e = blank(type, C.str(*id));
      e.flow_scope = scope;
      const bool esp_start = type == ZBHIP_EL_START_EVENT && C.elements[scope].element_type == ZBHIP_EL_EVENT_SUB_PROCESS;
      if (esp_start) {
        // the error start event of an event sub-process (CatchEventTransformer.java:166): a static
        // errorCode ("" catches every code) in message_name, interrupting (isInterrupting, default true)
        // in job_retries bit 0; the device never activates it -- a JOB:THROW_ERROR hands the instance off
        const Elem* eed = c.first("errorEventDefinition");
        for (auto& d : c.children)
          if (&d != eed && d.tag.size() > 15 && d.tag.compare(d.tag.size() - 15, 15, "EventDefinition") == 0) {
            err = "event definition <" + d.tag + "> of an event sub-process outside the supported subset";
            return ZBHIP_EUNSUPP;
          }
        const std::string* ii = c.get("isInterrupting");
        if (!eed || (ii && *ii == "false")) {
          err = "event sub-process start event outside the supported subset (interrupting error start events)";
          return ZBHIP_EUNSUPP;
        }
        std::string code;
        if (const std::string* ref = eed->get("errorRef")) {
          auto ei = errors.find(*ref);
          if (ei == errors.end()) { err = "unknown error " + *ref; return ZBHIP_EPARSE; }
          code = ei->second;
          if (!code.empty() && code[0] == '=') { err = "error code expressions outside the supported subset"; return ZBHIP_EUNSUPP; }
        }
        if (const Elem* ext = c.first("extensionElements"))
          if (ext->first("ioMapping")) { err = "io mappings outside the supported subset"; return ZBHIP_EUNSUPP; }
        e.event_type = ZBHIP_EV_ERROR;
        e.message_name = C.str(code);
        e.job_retries = 1;
      } else if (type == ZBHIP_EL_END_EVENT && c.first("errorEventDefinition")) {
        // an error end event (EndEventTransformer.java:70-83): a static errorCode in message_name; the
        // device never activates it (the command reaching it hands the instance to the engine)
        const Elem* eed = c.first("errorEventDefinition");
        for (auto& d : c.children)
          if (&d != eed && d.tag.size() > 15 && d.tag.compare(d.tag.size() - 15, 15, "EventDefinition") == 0) {
            err = "event definition <" + d.tag + "> outside the supported subset";
            return ZBHIP_EUNSUPP;
          }
        const std::string* ref = eed->get("errorRef");
        auto ei = ref ? errors.find(*ref) : errors.end();
        if (ei == errors.end() || ei->second.empty() || ei->second[0] == '=') {
          err = "error end event outside the supported subset (a static errorCode)";
          return ZBHIP_EUNSUPP;
        }
        if (const Elem* ext = c.first("extensionElements"))
          if (ext->first("ioMapping")) { err = "io mappings outside the supported subset"; return ZBHIP_EUNSUPP; }
        e.event_type = ZBHIP_EV_ERROR;
        e.message_name = C.str(ei->second);
      } else if (type == ZBHIP_EL_START_EVENT || type == ZBHIP_EL_END_EVENT) {
        for (auto& d : c.children)
          if (d.tag.size() > 15 && d.tag.compare(d.tag.size() - 15, 15, "EventDefinition") == 0) {
            err = "event definition <" + d.tag + "> outside the supported subset";
            return ZBHIP_EUNSUPP;
          }
        e.event_type = ZBHIP_EV_NONE;
      }
      if (type == ZBHIP_EL_EVENT_SUB_PROCESS) {
        // an event sub-process (SubProcessTransformer.transformEventSubprocess :36-60), attached to the
        // process or an embedded sub-process; its start event is its start_event
        if (c.first("multiInstanceLoopCharacteristics") || c.first("standardLoopCharacteristics") ||
            (c.first("extensionElements") && c.first("extensionElements")->first("ioMapping")) ||
            (scope != 0 && C.elements[scope].element_type != ZBHIP_EL_SUB_PROCESS)) {
          err = "event sub-process outside the supported subset";
          return ZBHIP_EUNSUPP;
        }
      }
      if (type == ZBHIP_EL_INTERMEDIATE_THROW_EVENT || type == ZBHIP_EL_TASK || type == ZBHIP_EL_MANUAL_TASK) {
        // activities / events without behaviour (UndefinedTaskProcessor, ManualTaskProcessor,
        // IntermediateThrowEventProcessor.NoneIntermediateThrowEventBehavior): none events only
        for (auto& d : c.children)
          if (d.tag.size() > 15 && d.tag.compare(d.tag.size() - 15, 15, "EventDefinition") == 0) {
            err = "event definition <" + d.tag + "> outside the supported subset";
            return ZBHIP_EUNSUPP;
          }
        if (const Elem* ext = c.first("extensionElements"))
          if (ext->first("ioMapping")) { err = "io mappings outside the supported subset"; return ZBHIP_EUNSUPP; }
        if (type == ZBHIP_EL_INTERMEDIATE_THROW_EVENT) e.event_type = ZBHIP_EV_NONE;
      }
      if (type == ZBHIP_EL_SUB_PROCESS) {
        // embedded sub-process (SubProcessTransformer / SubProcessProcessor): no multi-instance
        if (c.first("multiInstanceLoopCharacteristics") || c.first("standardLoopCharacteristics")) {
          err = "multi-instance sub-process outside the supported subset";
          return ZBHIP_EUNSUPP;
        }
        if (int rc = parse_mappings(c.first("extensionElements"), (uint16_t)C.elements.size(), C, err)) return rc;
      }
      if (type == ZBHIP_EL_BOUNDARY_EVENT && c.first("errorEventDefinition")) {
        // an error boundary event on a job worker task (BoundaryEventTransformer, ErrorTransformer):
        // interrupting, a static errorCode ("" -- no errorRef, or an <error> without a code -- catches every
        // code); nothing to subscribe: JOB:THROW_ERROR finds it (CatchEventAnalyzer), and the adapter hands
        // the instance to the engine for that command
        const Elem* eed = c.first("errorEventDefinition");
        for (auto& d : c.children)
          if (&d != eed && d.tag.size() > 15 && d.tag.compare(d.tag.size() - 15, 15, "EventDefinition") == 0) {
            err = "event definition <" + d.tag + "> outside the supported subset";
            return ZBHIP_EUNSUPP;
          }
        const std::string* ca = c.get("cancelActivity");
        if (ca && *ca == "false") { err = "a non-interrupting error boundary event"; return ZBHIP_EPARSE; }
        std::string code;
        if (const std::string* ref = eed->get("errorRef")) {
          auto ei = errors.find(*ref);
          if (ei == errors.end()) { err = "unknown error " + *ref; return ZBHIP_EPARSE; }
          code = ei->second;
          if (!code.empty() && code[0] == '=') { err = "error code expressions outside the supported subset"; return ZBHIP_EUNSUPP; }
        }
        if (const Elem* ext = c.first("extensionElements"))
          if (ext->first("ioMapping")) { err = "io mappings outside the supported subset"; return ZBHIP_EUNSUPP; }
        const std::string* at = c.get("attachedToRef");
        if (!at) { err = "boundary event without attachedToRef"; return ZBHIP_EPARSE; }
        e.event_type = ZBHIP_EV_ERROR;
        e.message_name = C.str(code);
        e.job_retries = 1;  // interrupting
        boundaries.push_back({(uint16_t)C.elements.size(), *at});
      } else if (type == ZBHIP_EL_BOUNDARY_EVENT && c.first("messageEventDefinition")) {
        // BoundaryEventTransformer + CatchEventTransformer.transformMessageEventDefinition: a message
        // boundary event on a job worker task, interrupting or not (static name, `= variable`
        // correlation key, evaluated in the task's flow scope); attached after the walk
        const std::string* ca = c.get("cancelActivity");
        const Elem* med = c.first("messageEventDefinition");
        for (auto& d : c.children)
          if (&d != med && d.tag.size() > 15 && d.tag.compare(d.tag.size() - 15, 15, "EventDefinition") == 0) {
            err = "event definition <" + d.tag + "> outside the supported subset";
            return ZBHIP_EUNSUPP;
          }
        if (!med->get("messageRef")) { err = "boundary event without a message"; return ZBHIP_EUNSUPP; }
        auto mi = messages.find(*med->get("messageRef"));
        if (mi == messages.end()) { err = "unknown message " + *med->get("messageRef"); return ZBHIP_EPARSE; }
        if (!mi->second.ok) { err = mi->second.why; return ZBHIP_EUNSUPP; }
        if (const Elem* ext = c.first("extensionElements"))
          if (ext->first("ioMapping")) { err = "io mappings outside the supported subset"; return ZBHIP_EUNSUPP; }
        const std::string* at = c.get("attachedToRef");
        if (!at) { err = "boundary event without attachedToRef"; return ZBHIP_EPARSE; }
        e.event_type = ZBHIP_EV_MESSAGE;
        e.message_name = C.str(mi->second.name);
        e.correlation_var = C.str(mi->second.corr);
        e.job_retries = ca && *ca == "false" ? 0 : 1;  // cancelActivity (BoundaryEvent default: interrupting)
        boundaries.push_back({(uint16_t)C.elements.size(), *at});
      } else if (type == ZBHIP_EL_BOUNDARY_EVENT) {
        // BoundaryEventTransformer: timer boundary events (a static timeDuration; interrupting or not)
        // on job worker tasks; attached after the walk
        const std::string* ca = c.get("cancelActivity");  // BoundaryEvent default: interrupting
        const bool interrupting = !(ca && *ca == "false");
        const Elem* ted = c.first("timerEventDefinition");
        const Elem* td = ted ? ted->first("timeDuration") : nullptr;
        const Elem* tc = ted && !td ? ted->first("timeCycle") : nullptr;
        for (auto& d : c.children)
          if (&d != ted && d.tag.size() > 15 && d.tag.compare(d.tag.size() - 15, 15, "EventDefinition") == 0) td = tc = nullptr;
        // a timeCycle (RepeatingInterval.parse "R[n]/duration", or its constant FEEL form): repetitions n
        // (1..254) or infinite (255); a duration: 1
        uint32_t reps = 1;
        if (!td && !tc) {
          err = "boundary event outside the supported subset (timer timeDuration or timeCycle)";
          return ZBHIP_EUNSUPP;
        }
        const std::string dtext = td ? td->text : tc->text;
        const int64_t ms = timer_ms(dtext, !td, reps);
        e.job_retries = (uint16_t)((interrupting ? 1u : 0u) | (reps << 8));
        if (ms < 0 || ms > 0xFFFFFFFFLL) { err = "timer outside the supported subset: " + dtext; return ZBHIP_EUNSUPP; }
        if (const Elem* ext = c.first("extensionElements"))
          if (ext->first("ioMapping")) { err = "io mappings outside the supported subset"; return ZBHIP_EUNSUPP; }
        const std::string* at = c.get("attachedToRef");
        if (!at) { err = "boundary event without attachedToRef"; return ZBHIP_EPARSE; }
        e.event_type = ZBHIP_EV_TIMER;
        e.duration_ms = (uint32_t)ms;
        boundaries.push_back({(uint16_t)C.elements.size(), *at});
      }
      if (type == ZBHIP_EL_INTERMEDIATE_CATCH_EVENT && c.first("timerEventDefinition")) {
        // CatchEventTransformer.transformTimerEventDefinition: a static timeDuration only
        const Elem* ted = c.first("timerEventDefinition");
        const Elem* td = ted->first("timeDuration");
        if (!td || c.first("messageEventDefinition") || c.first("signalEventDefinition")) {
          err = "timer catch event outside the supported subset (timeDuration only)";
          return ZBHIP_EUNSUPP;
        }
        uint32_t reps = 1;
        const int64_t ms = timer_ms(td->text, false, reps);
        if (ms < 0 || ms > 0xFFFFFFFFLL) { err = "timer duration outside the supported subset: " + td->text; return ZBHIP_EUNSUPP; }
        if (const Elem* ext = c.first("extensionElements"))
          if (ext->first("ioMapping")) { err = "io mappings outside the supported subset"; return ZBHIP_EUNSUPP; }
        e.event_type = ZBHIP_EV_TIMER;
        e.duration_ms = (uint32_t)ms;
      } else if (type == ZBHIP_EL_INTERMEDIATE_CATCH_EVENT) {
        // CatchEventTransformer.transformMessageEventDefinition: message catch events only
        const Elem* med = c.first("messageEventDefinition");
        for (auto& d : c.children)
          if (&d != med && d.tag.size() > 15 && d.tag.compare(d.tag.size() - 15, 15, "EventDefinition") == 0) {
            err = "event definition <" + d.tag + "> outside the supported subset";
            return ZBHIP_EUNSUPP;
          }
        if (!med || !med->get("messageRef")) { err = "intermediate catch event without a message"; return ZBHIP_EUNSUPP; }
        auto mi = messages.find(*med->get("messageRef"));
        if (mi == messages.end()) { err = "unknown message " + *med->get("messageRef"); return ZBHIP_EPARSE; }
        if (!mi->second.ok) { err = mi->second.why; return ZBHIP_EUNSUPP; }
        if (const Elem* ext = c.first("extensionElements"))
          if (ext->first("ioMapping")) { err = "io mappings outside the supported subset"; return ZBHIP_EUNSUPP; }
        e.event_type = ZBHIP_EV_MESSAGE;
        e.message_name = C.str(mi->second.name);
        e.correlation_var = C.str(mi->second.corr);
      }
      if (ZBHIP_IS_JOB_WORKER(type)) {
        // job worker tasks: a zeebe:taskDefinition (a zeebe:script / zeebe:calledDecision is
        // ScriptTaskProcessor's / BusinessRuleTaskProcessor's non-job behaviour: outside the subset)
        const Elem* ext = c.first("extensionElements");
        if (ext && (ext->first("script") || ext->first("calledDecision"))) {
          err = "script / decision tasks without a job outside the supported subset";
          return ZBHIP_EUNSUPP;
        }
        const Elem* td = ext ? ext->first("taskDefinition") : nullptr;
        const std::string* jt = td ? td->get("type") : nullptr;
        if (!jt || jt->empty()) { err = "service task '" + *id + "' without a job type"; return ZBHIP_EPARSE; }
        const std::string* rt = td->get("retries");
        std::string retries = rt ? *rt : "3";
        if ((*jt)[0] == '=' || retries.empty() || retries[0] == '=') {
          err = "job type/retries expressions outside the supported subset";
          return ZBHIP_EUNSUPP;
        }
        if (const Elem* th = ext->first("taskHeaders")) {
          C.headers.resize(C.elements.size() + 1);
          if (int rc = encode_task_headers(*th, C.headers[C.elements.size()], err)) return rc;
        }
        if (int rc = parse_mappings(ext, (uint16_t)C.elements.size(), C, err)) return rc;
        e.job_type = C.str(*jt);
        e.job_retries = (uint16_t)atoi(retries.c_str());
      }
      if (type == ZBHIP_EL_SEQUENCE_FLOW) flows.push_back(&c);
      if (type == ZBHIP_EL_EXCLUSIVE_GATEWAY) xgws.push_back(&c);
      if (index.count(*id)) { err = "duplicate element id " + *id; return ZBHIP_EPARSE; }
      if (c.first("standardLoopCharacteristics")) { err = "standard loops outside the supported subset"; return ZBHIP_EUNSUPP; }
      if (const Elem* mil = c.first("multiInstanceLoopCharacteristics")) {
        // MultiInstanceActivityTransformer.transform (:35-78): the body takes the activity's id, flow
        // scope and sequence flows (its index answers the id); the inner activity follows it, its flow
        // scope the body
        if (!ZBHIP_IS_JOB_WORKER(type) && type != ZBHIP_EL_TASK && type != ZBHIP_EL_MANUAL_TASK) {
          err = "multi-instance <" + c.tag + "> outside the supported subset (job worker and undefined tasks)";
          return ZBHIP_EUNSUPP;
        }
        if (!C.mappings.empty() && C.mappings.back().element == C.elements.size()) {
          err = "io mappings of a multi-instance activity outside the supported subset";
          return ZBHIP_EUNSUPP;
        }
        MiLoop loop;
        if (!parse_loop(*mil, loop, err)) return ZBHIP_EUNSUPP;
        zbhip_element b = blank(ZBHIP_EL_MULTI_INSTANCE_BODY, e.id);
        b.flow_scope = scope;
        b.job_retries = loop.seq ? 1 : 0;
        b.message_name = loop.input.empty() ? ZBHIP_NONE16 : C.str(loop.input);
        const uint16_t bi = (uint16_t)C.elements.size();
        b.start_event = (uint16_t)(bi + 1);
        if (C.headers.size() > bi) {  // the task headers belong to the inner activity, after the body
          std::string h = std::move(C.headers[bi]);
          C.headers.resize(bi + 2);
          C.headers[bi + 1] = std::move(h);
        }
        index[*id] = bi;
        C.elements.push_back(b);
        collections.push_back({bi, std::move(loop)});
        e.flow_scope = bi;
        C.elements.push_back(e);
        continue;
      }
      const uint16_t self = (uint16_t)C.elements.size();
      index[*id] = self;
      C.elements.push_back(e);
      if (type == ZBHIP_EL_SUB_PROCESS) {
        if (int rc = container(c, self)) return rc;
      } else if (type == ZBHIP_EL_EVENT_SUB_PROCESS) {
        if (int rc = container(c, self)) return rc;
        const uint16_t st = C.elements[self].start_event;
        if (st == ZBHIP_NONE16 || C.elements[st].event_type != ZBHIP_EV_ERROR) {
          err = "event sub-process without an error start event";
          return ZBHIP_EUNSUPP;
        }
      } else if (type == ZBHIP_EL_START_EVENT) {
        // getNoneStartEvent of the container (the last none start event in document order)
        C.elements[scope].start_event = self;
      }
    }
    return ZBHIP_OK;
  };
  if (int rc = container(*proc, 0)) return rc;
  // ExecutableActivity.attach (ExecutableActivity.java:28-38): one boundary event per job worker
  // task of the same container
  for (auto& [b, ref] : boundaries) {
    auto it = index.find(ref);
    if (it == index.end()) { err = "boundary event attached to an unknown element " + ref; return ZBHIP_EPARSE; }
    zbhip_element& A = C.elements[it->second];
    // job worker tasks; embedded sub-processes with a timer or an error boundary event (the sub-process
    // keeps it in default_flow: its start_event is its none start event)
    const bool on_sub = A.element_type == ZBHIP_EL_SUB_PROCESS && (C.elements[b].event_type == ZBHIP_EV_TIMER ||
                                                                   C.elements[b].event_type == ZBHIP_EV_ERROR);
    // (an error boundary event of a multi-instance activity: attached to its body, which keeps no slot for
    // it -- the runtime finds it by flow_source)
    if (A.element_type == ZBHIP_EL_MULTI_INSTANCE_BODY && C.elements[b].event_type == ZBHIP_EV_ERROR &&
        A.flow_scope == C.elements[b].flow_scope) {
      C.elements[b].flow_source = it->second;
      continue;
    }
    if ((!ZBHIP_IS_JOB_WORKER(A.element_type) && !on_sub) || A.flow_scope != C.elements[b].flow_scope) {
      err = "boundary event on an element outside the supported subset (job worker tasks, timers on sub-processes)";
      return ZBHIP_EUNSUPP;
    }
    // the slot holds the activity's timer / message boundary event, else its first error one; further
    // error boundary events need no device state (the runtime finds them by flow_source)
    uint16_t& slot = on_sub ? A.default_flow : A.start_event;
    const bool err_b = C.elements[b].event_type == ZBHIP_EV_ERROR;
    if (slot != ZBHIP_NONE16) {
      if (!err_b && C.elements[slot].event_type != ZBHIP_EV_ERROR) {
        err = "more than one timer / message boundary event on an activity outside the supported subset";
        return ZBHIP_EUNSUPP;
      }
      if (!err_b) slot = b;
    } else {
      slot = b;
    }
    C.elements[b].flow_source = it->second;
  }
  for (size_t e = 1; e < C.elements.size(); ++e)
    if (C.elements[e].element_type == ZBHIP_EL_SUB_PROCESS && C.elements[e].start_event == ZBHIP_NONE16) {
      err = "sub-process without a none start event";
      return ZBHIP_EUNSUPP;
    }
  out_lists.resize(C.elements.size());
  in_lists.resize(C.elements.size());

  for (const Elem* c : xgws) {
    if (const std::string* d = c->get("default")) {
      auto it = index.find(*d);
      if (it == index.end()) { err = "unknown default flow " + *d; return ZBHIP_EPARSE; }
      C.elements[index[*c->get("id")]].default_flow = it->second;
    }
  }

  C.cond_begin.push_back(0);
  auto name_of = [&C](const std::string& n) -> uint32_t { return C.str(n); };
  // Reverse document order: ModelWalker.java:75-79
  for (auto it = flows.rbegin(); it != flows.rend(); ++it) {
    const Elem& f = **it;
    uint16_t fi = index[*f.get("id")];
    const std::string* sr = f.get("sourceRef");
    const std::string* tr = f.get("targetRef");
    auto s = sr ? index.find(*sr) : index.end();
    auto t = tr ? index.find(*tr) : index.end();
    if (s == index.end() || t == index.end()) { err = "sequence flow with unknown source/target"; return ZBHIP_EPARSE; }
    zbhip_element& fe = C.elements[fi];
    if (C.elements[s->second].flow_scope != fe.flow_scope || C.elements[t->second].flow_scope != fe.flow_scope) {
      err = "sequence flow crossing a sub-process boundary";
      return ZBHIP_EPARSE;
    }
    fe.flow_source = s->second;
    fe.flow_target = t->second;
    if (const Elem* ce = f.first("conditionExpression")) {
      size_t a = ce->text.find_first_not_of(" \t\r\n");
      size_t b = ce->text.find_last_not_of(" \t\r\n");
      std::string txt = a == std::string::npos ? "" : ce->text.substr(a, b - a + 1);
      if (txt.empty() || txt[0] != '=') { err = "static (non-FEEL) condition outside the subset"; return ZBHIP_EUNSUPP; }
      std::string body = txt.substr(1);
      FeelCompiler fc(body, C.code, name_of);
      if (!fc.compile(err)) return ZBHIP_EUNSUPP;
      fe.condition = (uint16_t)(C.cond_begin.size() - 1);
      C.cond_begin.push_back((uint32_t)C.code.size());
      C.cond_texts.push_back(body);  // FeelExpressionLanguage.parseExpression: group(1) of "\\=(.+)"
    }
    out_lists[fe.flow_source].push_back(fi);
    in_lists[fe.flow_target].push_back(fi);
  }
  // the bodies' inputCollections after the flows' conditions (condition indices of flows unchanged):
  // the static items (ZBHIP_OP_ITEM) or the collection variable (ZBHIP_OP_COLLECTION), then the
  // outputCollection (ZBHIP_OP_OUTPUT); a completionCondition is a condition of its own, its index in
  // the body's default_flow
  for (auto& [b, loop] : collections) {
    C.elements[b].condition = (uint16_t)(C.cond_begin.size() - 1);
    if (!loop.coll_var.empty()) {
      zbhip_insn in{};
      in.op = ZBHIP_OP_COLLECTION;
      in.arg = C.str(loop.coll_var);
      C.code.push_back(in);
    }
    for (const MiItem& it : loop.items) {
      zbhip_insn in{};
      in.op = ZBHIP_OP_ITEM;
      in.arg = it.type;
      in.literal = it.type == ZBHIP_DOC_STR ? (int64_t)C.str(it.text) : it.value;
      C.code.push_back(in);
    }
    if (!loop.out_coll.empty()) {
      zbhip_insn in{};
      in.op = ZBHIP_OP_OUTPUT;
      in.arg = C.str(loop.out_coll);
      in.literal = C.str(loop.out_elem);
      C.code.push_back(in);
    }
    zbhip_insn end{};
    end.op = ZBHIP_OP_END;
    C.code.push_back(end);
    C.cond_begin.push_back((uint32_t)C.code.size());
    C.cond_texts.emplace_back();
    if (!loop.cond.empty()) {
      FeelCompiler fc(loop.cond, C.code, name_of);
      if (!fc.compile(err)) { err = "completionCondition: " + err; return ZBHIP_EUNSUPP; }
      C.elements[b].default_flow = (uint16_t)(C.cond_begin.size() - 1);
      C.cond_begin.push_back((uint32_t)C.code.size());
      C.cond_texts.push_back(loop.cond);
    }
  }
  // CSR of outgoing lists
  for (size_t e = 0; e < C.elements.size(); ++e) {
    C.elements[e].out_begin = (uint16_t)C.out_flow.size();
    C.elements[e].out_count = (uint16_t)out_lists[e].size();
    C.elements[e].in_count = (uint16_t)in_lists[e].size();
    for (uint16_t f : out_lists[e]) C.out_flow.push_back(f);
  }
  // join counters (NUMBER_OF_TAKEN_SEQUENCE_FLOWS[flowScope, gateway, flow]): the incoming flows of
  // each parallel gateway get consecutive per-instance counter slots; the gateway's join_slot is the
  // base of its range, so canActivateParallelGateway counts slots [base, base + in_count).
  uint16_t slots = 0;
  for (size_t g = 0; g < C.elements.size(); ++g) {
    if (C.elements[g].element_type != ZBHIP_EL_PARALLEL_GATEWAY) continue;
    C.elements[g].join_slot = slots;
    for (uint16_t f : in_lists[g]) C.elements[f].join_slot = slots++;
  }
  C.csr.n_join_slots = slots;
  C.csr.none_start = C.elements[0].start_event;
  C.csr.process_definition_key = def_key;
  C.csr.version = version;
  C.finish();
  return ZBHIP_OK;
}

}  // namespace zbc

extern "C" int zbhip_compile_bpmn(const char* xml, size_t len, int64_t process_definition_key, int32_t version,
                                  zbhip_process_csr** out, char* err, size_t err_cap) {
  if (!xml || !out) return ZBHIP_EINVAL;
  auto* c = new zbc::Compiled();
  std::string e;
  int rc = zbc::compile(xml, len, process_definition_key, version, *c, e);
  if (rc != ZBHIP_OK) {
    if (err && err_cap) snprintf(err, err_cap, "%s", e.c_str());
    delete c;
    *out = nullptr;
    return rc;
  }
  *out = &c->csr;  // csr is the first member: zbhip_free_csr recovers the owner
  return ZBHIP_OK;
}

extern "C" void zbhip_free_csr(zbhip_process_csr* csr) {
  delete reinterpret_cast<zbc::Compiled*>(reinterpret_cast<char*>(csr));
}

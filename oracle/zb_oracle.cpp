// ============================================================================
// zb_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of Zeebe's BPMN element-lifecycle hot path (reference:
// honlyc/zeebe 8.4.0-SNAPSHOT, read-only at /root/reference).  It is the checker
// the GPU executor is parity-tested against and the "port" CPU baseline timed by
// bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
// may load it; the product (zeebe_amd/, libzbhip.so) never links or calls it.
//
// Parity pinning: the reference is Java 21 + Maven and cannot be built or run in
// this image (no JDK); the oracle is pinned against golden vectors transcribed
// from the reference's own tests and code-derived sequences,
// see tests/golden/ and tests/test_oracle_golden.py.
//
// Every function cites the reference file:line it restates.  Paths are relative
// to /root/reference/engine/src/main/java/io/camunda/zeebe/engine/ unless they
// start with another module name.
// ============================================================================
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "../include/zbhip.h"

namespace {

// ---------------------------------------------------------------------------
// Minimal XML reader (enough for BPMN 2.0 files written by the modeler or the
// fluent builder).  Namespace prefixes are stripped.
// ---------------------------------------------------------------------------
struct XNode {
  std::string name;
  std::map<std::string, std::string> attrs;
  std::string text;
  std::vector<std::unique_ptr<XNode>> kids;
  const XNode* child(const std::string& n) const {
    for (auto& k : kids)
      if (k->name == n) return k.get();
    return nullptr;
  }
  std::string attr(const std::string& n, const std::string& dflt = "") const {
    auto it = attrs.find(n);
    return it == attrs.end() ? dflt : it->second;
  }
};

static std::string strip_ns(const std::string& s) {
  auto p = s.find(':');
  return p == std::string::npos ? s : s.substr(p + 1);
}

static std::string xml_unescape(const std::string& s) {
  std::string o;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '&') {
      auto e = s.find(';', i);
      if (e == std::string::npos) { o += s[i]; continue; }
      std::string ent = s.substr(i + 1, e - i - 1);
      if (ent == "lt") o += '<';
      else if (ent == "gt") o += '>';
      else if (ent == "amp") o += '&';
      else if (ent == "quot") o += '"';
      else if (ent == "apos") o += '\'';
      else if (!ent.empty() && ent[0] == '#') {
        long cp = ent.size() > 1 && ent[1] == 'x' ? strtol(ent.c_str() + 2, nullptr, 16)
                                                  : strtol(ent.c_str() + 1, nullptr, 10);
        if (cp < 128) o += (char)cp;
      }
      i = e;
    } else {
      o += s[i];
    }
  }
  return o;
}

struct XmlParser {
  const std::string& s;
  size_t i = 0;
  std::string err;
  explicit XmlParser(const std::string& src) : s(src) {}
  void skip_ws() { while (i < s.size() && isspace((unsigned char)s[i])) ++i; }
  bool parse_misc() {  // comments, PIs, doctype
    for (;;) {
      skip_ws();
      if (s.compare(i, 4, "<!--") == 0) {
        auto e = s.find("-->", i);
        if (e == std::string::npos) return false;
        i = e + 3;
      } else if (s.compare(i, 2, "<?") == 0) {
        auto e = s.find("?>", i);
        if (e == std::string::npos) return false;
        i = e + 2;
      } else if (s.compare(i, 2, "<!") == 0) {
        auto e = s.find('>', i);
        if (e == std::string::npos) return false;
        i = e + 1;
      } else {
        return true;
      }
    }
  }
  std::unique_ptr<XNode> parse_element() {
    if (!parse_misc() || i >= s.size() || s[i] != '<') { err = "expected element"; return nullptr; }
    ++i;
    auto n = std::make_unique<XNode>();
    size_t st = i;
    while (i < s.size() && !isspace((unsigned char)s[i]) && s[i] != '>' && s[i] != '/') ++i;
    n->name = strip_ns(s.substr(st, i - st));
    for (;;) {
      skip_ws();
      if (i >= s.size()) { err = "eof in tag"; return nullptr; }
      if (s[i] == '/') {
        if (s.compare(i, 2, "/>") != 0) { err = "bad tag end"; return nullptr; }
        i += 2;
        return n;
      }
      if (s[i] == '>') { ++i; break; }
      size_t as = i;
      while (i < s.size() && s[i] != '=' && !isspace((unsigned char)s[i])) ++i;
      std::string an = s.substr(as, i - as);
      skip_ws();
      if (i >= s.size() || s[i] != '=') { err = "bad attribute"; return nullptr; }
      ++i;
      skip_ws();
      char q = s[i];
      if (q != '"' && q != '\'') { err = "bad attribute quote"; return nullptr; }
      auto e = s.find(q, i + 1);
      if (e == std::string::npos) { err = "eof in attribute"; return nullptr; }
      n->attrs[strip_ns(an)] = xml_unescape(s.substr(i + 1, e - i - 1));
      i = e + 1;
    }
    // content
    for (;;) {
      if (i >= s.size()) { err = "eof in content"; return nullptr; }
      if (s.compare(i, 2, "</") == 0) {
        auto e = s.find('>', i);
        if (e == std::string::npos) { err = "eof in end tag"; return nullptr; }
        i = e + 1;
        return n;
      }
      if (s.compare(i, 9, "<![CDATA[") == 0) {
        auto e = s.find("]]>", i);
        if (e == std::string::npos) { err = "eof in cdata"; return nullptr; }
        n->text += s.substr(i + 9, e - i - 9);
        i = e + 3;
        continue;
      }
      if (s.compare(i, 4, "<!--") == 0 || s.compare(i, 2, "<?") == 0) {
        if (!parse_misc()) { err = "bad misc"; return nullptr; }
        continue;
      }
      if (s[i] == '<') {
        auto k = parse_element();
        if (!k) return nullptr;
        n->kids.push_back(std::move(k));
        continue;
      }
      auto e = s.find('<', i);
      if (e == std::string::npos) e = s.size();
      n->text += xml_unescape(s.substr(i, e - i));
      i = e;
    }
  }
};

// ---------------------------------------------------------------------------
// FEEL subset: boolean conditions over numbers/booleans/null
// (feel-scala 1.17.0 is a third-party dependency absent from the tree:
// parent/pom.xml:93,925-927).  Numbers are exact decimals (BigDecimal in
// feel-scala, feel/.../MessagePackValueMapper.scala:41-71); held here as
// __int128 scaled by 10^18.
// ---------------------------------------------------------------------------
enum VKind { V_NULL, V_BOOL, V_NUM, V_ERR, V_STR };
struct FVal {
  VKind k = V_NULL;
  __int128 n = 0;
  bool b = false;
};
static const __int128 kScale18 = (__int128)1000000000000000000LL;

struct FExpr {
  enum Op { NUM, BOOL, NUL, VAR, CMP, AND, OR, NOT } op;
  std::string cmp;  // "<" "<=" ">" ">=" "=" "!="
  __int128 num = 0;
  bool b = false;
  std::string var;
  std::unique_ptr<FExpr> l, r;
};

struct FeelParser {
  std::string s;
  size_t i = 0;
  bool ok = true;
  explicit FeelParser(std::string src) : s(std::move(src)) {}
  void ws() { while (i < s.size() && isspace((unsigned char)s[i])) ++i; }
  bool kw(const char* w) {
    ws();
    size_t n = strlen(w);
    if (s.compare(i, n, w) == 0 && (i + n >= s.size() || !(isalnum((unsigned char)s[i + n]) || s[i + n] == '_'))) {
      i += n;
      return true;
    }
    return false;
  }
  std::unique_ptr<FExpr> parse_or() {
    auto l = parse_and();
    while (ok && kw("or")) {
      auto e = std::make_unique<FExpr>();
      e->op = FExpr::OR;
      e->l = std::move(l);
      e->r = parse_and();
      l = std::move(e);
    }
    return l;
  }
  std::unique_ptr<FExpr> parse_and() {
    auto l = parse_cmp();
    while (ok && kw("and")) {
      auto e = std::make_unique<FExpr>();
      e->op = FExpr::AND;
      e->l = std::move(l);
      e->r = parse_cmp();
      l = std::move(e);
    }
    return l;
  }
  std::unique_ptr<FExpr> parse_cmp() {
    auto l = parse_atom();
    ws();
    static const char* ops[] = {"<=", ">=", "!=", "<", ">", "="};
    for (auto o : ops) {
      size_t n = strlen(o);
      if (s.compare(i, n, o) == 0) {
        i += n;
        auto e = std::make_unique<FExpr>();
        e->op = FExpr::CMP;
        e->cmp = o;
        e->l = std::move(l);
        e->r = parse_atom();
        return e;
      }
    }
    return l;
  }
  std::unique_ptr<FExpr> parse_atom() {
    ws();
    auto e = std::make_unique<FExpr>();
    if (i >= s.size()) { ok = false; return e; }
    if (s[i] == '(') {
      ++i;
      auto in = parse_or();
      ws();
      if (i >= s.size() || s[i] != ')') ok = false;
      else ++i;
      return in;
    }
    if (kw("not")) {
      ws();
      if (i >= s.size() || s[i] != '(') { ok = false; return e; }
      ++i;
      e->op = FExpr::NOT;
      e->l = parse_or();
      ws();
      if (i >= s.size() || s[i] != ')') ok = false;
      else ++i;
      return e;
    }
    if (kw("true")) { e->op = FExpr::BOOL; e->b = true; return e; }
    if (kw("false")) { e->op = FExpr::BOOL; e->b = false; return e; }
    if (kw("null")) { e->op = FExpr::NUL; return e; }
    bool neg = false;
    if (s[i] == '-') { neg = true; ++i; }
    if (i < s.size() && (isdigit((unsigned char)s[i]) || s[i] == '.')) {
      __int128 ip = 0, fp = 0, fs = 1;
      while (i < s.size() && isdigit((unsigned char)s[i])) ip = ip * 10 + (s[i++] - '0');
      if (i < s.size() && s[i] == '.') {
        ++i;
        int digits = 0;
        while (i < s.size() && isdigit((unsigned char)s[i])) {
          if (digits < 18) { fp = fp * 10 + (s[i] - '0'); fs *= 10; }
          ++digits;
          ++i;
        }
        if (digits > 18) ok = false;
      }
      e->op = FExpr::NUM;
      e->num = ip * kScale18 + fp * (kScale18 / fs);
      if (neg) e->num = -e->num;
      return e;
    }
    if (neg) { ok = false; return e; }
    if (isalpha((unsigned char)s[i]) || s[i] == '_') {
      size_t st = i;
      while (i < s.size() && (isalnum((unsigned char)s[i]) || s[i] == '_')) ++i;
      e->op = FExpr::VAR;
      e->var = s.substr(st, i - st);
      ws();
      if (i < s.size() && (s[i] == '.' || s[i] == '[' || s[i] == '(')) ok = false;  // paths/calls: outside subset
      return e;
    }
    ok = false;
    return e;
  }
};

// ---------------------------------------------------------------------------
// Process model (ExecutableProcess / ExecutableFlowNode / ExecutableSequenceFlow)
// ---------------------------------------------------------------------------
struct OEl {
  std::string id;
  int type = ZBHIP_EL_UNSPECIFIED;
  int event = ZBHIP_EV_UNSPECIFIED;
  std::vector<int> out, in, out_with_cond;
  int src = -1, tgt = -1;
  bool has_cond = false;
  std::unique_ptr<FExpr> cond;
  std::string cond_text;           // the FEEL expression's text after '=' (ParsedExpression.text)
  int default_flow = -1;
  std::string job_type;
  int retries = 3;
  std::string msg_name, corr_var;  // message catch event (MessageTransformer.java:30-60)
  int64_t timer_ms = -1;           // timer catch event: the static timeDuration in ms (TimerTransformer)
  int scope = 0;                   // flow scope element (ExecutableFlowElement.getFlowScope): 0 = process
  int start = -1;                  // process / sub-process: getNoneStartEvent
  int attached = -1;               // boundary event: the activity it is attached to (attachedToRef)
  int boundary = -1;               // activity: its timer / message boundary event, else its first error one
  std::vector<int> boundaries;     // every boundary event, in attach order (ExecutableActivity.attach)
  std::vector<int> esps;           // a container's event sub-processes, in attach order (SubProcessTransformer)
  bool interrupting = true;        // boundary event: cancelActivity (ExecutableBoundaryEvent.interrupting)
  int reps = 1;                    // timer: repetitions (RepeatingInterval; 1 a duration, -1 infinite)
  // multi-instance body (ExecutableMultiInstanceBody / ExecutableLoopCharacteristics): its inner
  // activity (the next element, same id, flow scope = the body), isSequential, the static
  // inputCollection's items (zbhip_doc_type, value; strings as text until deploy interns them) and the
  // inputElement variable name ("" none)
  int inner = -1;
  bool mi_seq = false;
  std::vector<std::pair<uint8_t, int64_t>> mi_items;
  std::vector<std::string> mi_item_text;
  std::string mi_input;
  int mi_input_id = -1, mi_loop_id = -1;
  // inputCollection `= name` (a list variable, evaluateArrayExpression), outputCollection with its
  // outputElement `= name`, and a completionCondition (a FEEL boolean of the subset)
  std::string mi_coll_name, mi_out_coll, mi_out_elem;
  int mi_coll_id = -1, mi_out_coll_id = -1, mi_out_elem_id = -1;
  std::unique_ptr<FExpr> mi_cond;
  std::string mi_cond_text;
  // zeebe:ioMapping (VariableMappingTransformer, deployment/model/transformer/VariableMappingTransformer.java:
  // 73-200) in the subset: at most one input and one output mapping, a plain target name, a source that
  // is a variable reference (`= x`), a literal (`= 5`, `= true`, `= null`, `= "s"`) or a static string
  struct Mapping {
    bool present = false;
    bool var = false;         // the source is a variable reference
    std::string source;       // the variable name, or the string literal's text
    uint8_t type = 0;         // zbhip_doc_type of a literal
    int64_t value = 0;
    std::string target;
    int source_id = -1, target_id = -1;  // name ids (deploy); a string literal: its value-dictionary id
  };
  Mapping in_map, out_map;
  // an error boundary event: the errorCode of its <error> ("" = a catch-all errorEventDefinition)
  std::string error_code;
  // zeebe:taskHeaders of a job worker (document order) and the customHeaders its jobs carry
  std::vector<std::pair<std::string, std::string>> headers;
  std::string header_bytes;
};

struct OProc {
  std::string bpmn_id;
  int64_t def_key = 0;
  int version = 1;
  std::vector<OEl> els;  // [0] = process
  int none_start = -1;
  std::vector<int> msg_starts;  // message start events of the process (ExecutableProcess.getStartEvents)
  int bpmn_name = -1;           // the bpmnProcessId in the name dictionary (message start events)
};

// BpmnTransformer.transformDefinitions (deployment/model/transformation/BpmnTransformer.java:109-127)
// with ModelWalker.walk (bpmn-model/.../traversal/ModelWalker.java:60-81): siblings are
// pushed with addFirst, so sequence flows are connected in reverse document order
// (SequenceFlowTransformer.connectWithFlowNodes), which fixes getOutgoing() order.
using MessageDefs = std::unordered_map<std::string, std::pair<std::string, std::string>>;  // id -> (name, corr var)

// Interval.parse (bpmn-model/.../util/time/Interval.java) for static durations: "P[0D][T[nH][nM][n[.f]S]]"
// -- a Duration, so the due date is now + a fixed number of ms.  Days (a Period: calendar-based in the
// system zone), years / months / weeks, negative parts and expressions (`=`) are outside the subset: -1.
static int64_t parse_duration_ms(std::string t) {
  size_t a = t.find_first_not_of(" \t\r\n"), b = t.find_last_not_of(" \t\r\n");
  if (a == std::string::npos) return -1;
  t = t.substr(a, b - a + 1);
  if (t.size() < 3 || t[0] != 'P') return -1;
  int64_t ms = 0;
  bool time = false, any = false;
  size_t i = 1;
  while (i < t.size()) {
    if (t[i] == 'T') { if (time) return -1; time = true; ++i; continue; }
    int64_t whole = 0, frac = 0, fdig = 0;
    size_t s = i;
    while (i < t.size() && isdigit((unsigned char)t[i])) { whole = whole * 10 + (t[i] - '0'); if (whole > (1LL << 40)) return -1; ++i; }
    if (i < t.size() && t[i] == '.') {
      ++i;
      while (i < t.size() && isdigit((unsigned char)t[i])) { if (fdig < 3) { frac = frac * 10 + (t[i] - '0'); ++fdig; } ++i; }
      while (fdig < 3) { frac *= 10; ++fdig; }
    }
    if (i == s || i >= t.size()) return -1;
    const char u = t[i++];
    any = true;
    // a non-zero day count makes the interval calendar-based (Interval.isCalendarBased,
    // Interval.java:77-93: ZonedDateTime.plus in the system zone): outside the subset
    if (!time && u == 'D' && !frac && whole == 0) continue;
    else if (time && u == 'H' && !frac) ms += whole * 3600000LL;
    else if (time && u == 'M' && !frac) ms += whole * 60000LL;
    else if (time && u == 'S') ms += whole * 1000LL + frac;
    else return -1;
  }
  return any ? ms : -1;
}

// The timer expressions of the subset, evaluated as ExpressionProcessor.evaluateIntervalExpression
// (processing/common/ExpressionProcessor.java:142-175) does: a static text is a string; `=` starts a FEEL
// expression whose constant value is a string ("..."), a day-time duration (duration("...") -- a
// java.time.Duration, days of 24 h, turned into new Interval(duration)) or, for cycles, the string
// FeelFunctionProvider.cycle (feel/.../FeelFunctionProvider.scala:23-47) builds, "R[n]/" + duration.
// A string goes through Interval.parse (timeDuration) or RepeatingInterval.parse (timeCycle).
struct TimerValue {
  bool ok = false;
  int64_t ms = -1;  // DURATION / the cycle's interval
  int reps = 1;     // timeCycle: RepeatingInterval repetitions (-1 infinite)
};
static std::string strip(const std::string& t) {
  size_t a = t.find_first_not_of(" \t\r\n"), b = t.find_last_not_of(" \t\r\n");
  return a == std::string::npos ? "" : t.substr(a, b - a + 1);
}
static int64_t parse_feel_daytime_ms(const std::string& t) {  // FEEL duration("P[nD][T[nH][nM][n[.f]S]]")
  size_t d = t.find('D');
  if (t.size() < 3 || t[0] != 'P' || t.find_first_of("YMW") < t.find('T')) return -1;
  int64_t days = 0;
  std::string rest = t;
  if (d != std::string::npos && d < t.find('T')) {
    const std::string n = t.substr(1, d - 1);
    if (n.empty() || n.size() > 6 || n.find_first_not_of("0123456789") != std::string::npos) return -1;
    days = atoll(n.c_str());
    rest = "P" + t.substr(d + 1);
    if (rest == "P") return days * 86400000LL;
  }
  const int64_t ms = parse_duration_ms(rest);
  return ms < 0 ? -1 : ms + days * 86400000LL;
}
static bool feel_string(const std::string& e, std::string& v) {
  if (e.size() < 2 || e.front() != '"' || e.back() != '"') return false;
  v = e.substr(1, e.size() - 2);
  return v.find('"') == std::string::npos && v.find('\\') == std::string::npos;
}
static bool feel_call(const std::string& e, const std::string& fn, std::vector<std::string>& args) {
  if (e.compare(0, fn.size(), fn) != 0) return false;
  const std::string r = strip(e.substr(fn.size()));
  if (r.size() < 2 || r.front() != '(' || r.back() != ')') return false;
  args.clear();
  std::string cur;
  int depth = 0;
  for (char ch : r.substr(1, r.size() - 2)) {
    if (ch == '(') ++depth;
    if (ch == ')') --depth;
    if (ch == ',' && depth == 0) { args.push_back(strip(cur)); cur.clear(); continue; }
    cur += ch;
  }
  args.push_back(strip(cur));
  return true;
}
static int repeating_reps(const std::string& n) {  // RepeatingInterval.parse: "R" [n] "/"
  if (n.empty()) return -1;                         // INFINITE
  if (n.size() > 3 || n.find_first_not_of("0123456789") != std::string::npos) return 0;
  const int r = atoi(n.c_str());
  return r >= 1 && r <= 254 ? r : 0;
}
static TimerValue timer_value(const std::string& text, bool cycle) {
  TimerValue v;
  std::string t = strip(text), str;
  bool is_string = true;
  if (!t.empty() && t[0] == '=') {
    const std::string e = strip(t.substr(1));
    std::vector<std::string> a;
    if (feel_string(e, str)) {
      t = str;
    } else if (!cycle && feel_call(e, "duration", a) && a.size() == 1 && feel_string(a[0], str)) {
      v.ms = parse_feel_daytime_ms(str);
      is_string = false;
    } else if (cycle && feel_call(e, "cycle", a) && (a.size() == 1 || a.size() == 2)) {
      std::vector<std::string> d;
      if (!feel_call(a.back(), "duration", d) || d.size() != 1 || !feel_string(d[0], str)) return v;
      v.ms = parse_feel_daytime_ms(str);
      v.reps = a.size() == 2 ? repeating_reps(a[0]) : -1;
      v.ok = v.ms >= 0 && v.reps != 0;
      return v;
    } else {
      return v;  // variables, other functions: outside the subset
    }
  }
  if (is_string) {
    if (cycle) {
      const size_t slash = t.find('/');
      if (t.size() < 3 || t[0] != 'R' || slash == std::string::npos || t.find('/', slash + 1) != std::string::npos) return v;
      v.reps = repeating_reps(t.substr(1, slash - 1));
      if (v.reps == 0) return v;
      t = t.substr(slash + 1);
    }
    v.ms = parse_duration_ms(t);
  }
  v.ok = v.ms >= 0;
  return v;
}

// `= name`: a FEEL variable reference (no path, no call) -> name, else ""
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

// MultiInstanceActivityTransformer.transformLoopCharacteristics
// (deployment/model/transformer/MultiInstanceActivityTransformer.java:80-122) for the subset: the
// inputCollection a static FEEL list literal (`= [10, 20, 30]`, `= ["a", "b"]`: integer, string,
// boolean and null items -- FeelToMessagePackTransformer writes a whole number as a msgpack integer)
// or a list variable (`= items`), an optional inputElement, an outputCollection with an outputElement
// that names a variable (`= result`), and a completionCondition of the FEEL subset (`= x`, `= item = 20`,
// comparisons over numberOfInstances / numberOfActiveInstances / numberOfCompletedInstances /
// numberOfTerminatedInstances and variables).
static bool parse_multi_instance(const XNode& mil, OEl& body, std::string& err) {
  body.mi_seq = mil.attr("isSequential") == "true";
  const XNode* cc = mil.child("completionCondition");
  if (cc && cc->text.find_first_not_of(" \t\r\n") != std::string::npos) {
    const size_t a = cc->text.find_first_not_of(" \t\r\n");
    if (cc->text[a] != '=') { err = "static (non-FEEL) completionCondition outside the subset"; return false; }
    FeelParser fp(cc->text.substr(a + 1));
    body.mi_cond = fp.parse_or();
    fp.ws();
    if (!fp.ok || fp.i != fp.s.size()) { err = "completionCondition outside the FEEL subset: " + cc->text; return false; }
    const size_t b = cc->text.find_first_not_of(" \t\r\n", a + 1);
    body.mi_cond_text = b == std::string::npos ? "" : cc->text.substr(b);
  }
  const XNode* ext = mil.child("extensionElements");
  const XNode* lc = ext ? ext->child("loopCharacteristics") : nullptr;
  if (!lc) { err = "multi-instance without zeebe:loopCharacteristics"; return false; }
  const std::string oc = lc->attr("outputCollection"), oe = lc->attr("outputElement");
  if (!oc.empty() || !oe.empty()) {
    body.mi_out_elem = feel_variable(oe);
    if (oc.empty() || body.mi_out_elem.empty()) {
      err = "multi-instance outputCollection / outputElement outside the supported subset (a variable)";
      return false;
    }
    body.mi_out_coll = oc;
  }
  body.mi_input = lc->attr("inputElement");
  std::string t = lc->attr("inputCollection");
  body.mi_coll_name = feel_variable(t);
  if (!body.mi_coll_name.empty()) return true;
  size_t i = t.find_first_not_of(" \t\r\n");
  auto bad = [&err, &t]() { err = "multi-instance inputCollection outside the supported subset (a static list or a variable): " + t; return false; };
  if (i == std::string::npos || t[i] != '=') return bad();
  auto ws = [&]() { while (i < t.size() && isspace((unsigned char)t[i])) ++i; };
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
      if (t[i] == '"') {
        size_t e = t.find('"', i + 1);
        if (e == std::string::npos) return bad();
        const std::string v = t.substr(i + 1, e - i - 1);
        if (v.find('\\') != std::string::npos) return bad();
        body.mi_items.push_back({ZBHIP_DOC_STR, 0});
        body.mi_item_text.push_back(v);
        i = e + 1;
      } else if (t.compare(i, 4, "true") == 0 || t.compare(i, 5, "false") == 0 || t.compare(i, 4, "null") == 0) {
        const bool n = t[i] == 'n', tr = t[i] == 't';
        body.mi_items.push_back({n ? ZBHIP_DOC_NIL : ZBHIP_DOC_BOOL, tr ? 1 : 0});
        body.mi_item_text.emplace_back();
        i += t[i] == 'f' ? 5 : 4;
      } else {
        const bool neg = t[i] == '-';
        if (neg) ++i;
        const size_t s0 = i;
        unsigned long long v = 0;
        while (i < t.size() && isdigit((unsigned char)t[i])) {
          if (v > 922337203685477580ULL) return bad();
          v = v * 10 + (unsigned)(t[i] - '0');
          ++i;
        }
        if (i == s0 || v > 9223372036854775807ULL || (i < t.size() && (t[i] == '.' || isalpha((unsigned char)t[i]))))
          return bad();
        body.mi_items.push_back({ZBHIP_DOC_INT, neg ? -(int64_t)v : (int64_t)v});
        body.mi_item_text.emplace_back();
      }
      ws();
      if (i < t.size() && t[i] == ',') { ++i; continue; }
      if (i < t.size() && t[i] == ']') { ++i; break; }
      return bad();
    }
  }
  ws();
  if (i != t.size() || body.mi_items.size() > 65535) return bad();
  return true;
}

// zeebe:ioMapping of a job worker task or an embedded sub-process (the subset above); false + err
// outside it.  A source without a leading '=' is a static string (StaticExpression:
// VariableMappingTransformer.java:176-180 quotes it).  Several mappings of one kind produce a
// multi-entry document, iterated in agrona Int2IntHashMap order (IndexedDocument.java:44-63):
// parity unpinned, so they are outside the subset.
static bool parse_mappings(const XNode* ext, OEl& e, std::string& err) {
  const XNode* io = ext ? ext->child("ioMapping") : nullptr;
  if (!io) return true;
  auto trim = [](const std::string& t) {
    const size_t a = t.find_first_not_of(" \t\r\n"), b = t.find_last_not_of(" \t\r\n");
    return a == std::string::npos ? std::string() : t.substr(a, b - a + 1);
  };
  auto ident = [](const std::string& v) {
    bool ok = !v.empty() && (isalpha((unsigned char)v[0]) || v[0] == '_');
    for (char ch : v) ok = ok && (isalnum((unsigned char)ch) || ch == '_');
    return ok && v != "true" && v != "false" && v != "null";
  };
  for (auto& m : io->kids) {
    if (m->name != "input" && m->name != "output") continue;
    OEl::Mapping& M = m->name == "input" ? e.in_map : e.out_map;
    if (M.present) { err = "more than one " + m->name + " mapping (document order unpinned)"; return false; }
    M.present = true;
    M.target = trim(m->attr("target"));
    if (!ident(M.target)) { err = "io mapping target outside the subset: " + M.target; return false; }
    const std::string src = m->attr("source");
    if (src.empty() || src[0] != '=') {  // a static string
      M.type = ZBHIP_DOC_STR;
      M.source = src;
      continue;
    }
    const std::string x = trim(src.substr(1));
    if (ident(x)) { M.var = true; M.source = x; continue; }
    if (x == "true" || x == "false") { M.type = ZBHIP_DOC_BOOL; M.value = x == "true"; continue; }
    if (x == "null") { M.type = ZBHIP_DOC_NIL; continue; }
    if (x.size() >= 2 && x.front() == '"' && x.back() == '"' && x.find('"', 1) == x.size() - 1 &&
        x.find('\\') == std::string::npos) {
      M.type = ZBHIP_DOC_STR;
      M.source = x.substr(1, x.size() - 2);
      continue;
    }
    size_t i = x[0] == '-' ? 1 : 0;
    unsigned long long v = 0;
    bool ok = i < x.size();
    for (; ok && i < x.size(); ++i) {
      ok = isdigit((unsigned char)x[i]) && v <= 922337203685477580ULL;
      if (ok) v = v * 10 + (unsigned)(x[i] - '0');
    }
    if (!ok || v > 9223372036854775807ULL) { err = "io mapping source outside the subset: " + src; return false; }
    M.type = ZBHIP_DOC_INT;
    M.value = x[0] == '-' ? -(int64_t)v : (int64_t)v;
  }
  return true;
}

using ErrorDefs = std::unordered_map<std::string, std::string>;  // <error> id -> errorCode

static bool build_process(const XNode& proc, const MessageDefs& msgs, const ErrorDefs& errors, OProc& P,
                          std::string& err) {
  P.bpmn_id = proc.attr("id");
  P.els.clear();
  OEl pe;
  pe.id = P.bpmn_id;
  pe.type = ZBHIP_EL_PROCESS;
  P.els.push_back(std::move(pe));
  std::unordered_map<std::string, int> idx;
  idx[P.bpmn_id] = 0;
  std::vector<const XNode*> flows, xgws;
  std::vector<std::pair<int, std::string>> boundaries;  // (boundary event, attachedToRef)
  // FlowElementInstantiationTransformer over every container (the process and its embedded
  // sub-processes, SubProcessTransformer): elements numbered in document pre-order
  std::function<bool(const XNode&, int)> walk = [&](const XNode& parent, int scope) -> bool {
  for (auto& k : parent.kids) {
    const std::string& n = k->name;
    OEl e;
    e.id = k->attr("id");
    e.scope = scope;
    if (n == "startEvent" && k->child("errorEventDefinition") && P.els[scope].type == ZBHIP_EL_EVENT_SUB_PROCESS) {
      // the error start event of an event sub-process (CatchEventTransformer.java:166: ERROR; its errorCode
      // as an error boundary event's; interrupting -- isInterrupting, default true -- as an error start
      // event must be)
      e.type = ZBHIP_EL_START_EVENT;
      e.event = ZBHIP_EV_ERROR;
      e.interrupting = k->attr("isInterrupting") != "false";
      if (!e.interrupting || k->child("messageEventDefinition") || k->child("timerEventDefinition") ||
          k->child("signalEventDefinition")) {
        err = "error start event outside the supported subset";
        return false;
      }
      const std::string ref = k->child("errorEventDefinition")->attr("errorRef");
      if (!ref.empty()) {
        auto it = errors.find(ref);
        if (it == errors.end()) { err = "error start event with an unknown errorRef"; return false; }
        if (!it->second.empty() && it->second[0] == '=') { err = "error code expression outside the supported subset"; return false; }
        e.error_code = it->second;
      }
      const XNode* ext = k->child("extensionElements");
      if (ext && ext->child("ioMapping")) { err = "io mappings outside the supported subset"; return false; }
    } else if (n == "startEvent") {
      e.type = ZBHIP_EL_START_EVENT;
      // StartEventTransformer.java:40 — event type from the event definition
      const XNode* med = k->child("messageEventDefinition");
      if ((med && scope != 0) || k->child("timerEventDefinition") ||
          k->child("signalEventDefinition") || k->child("errorEventDefinition") ||
          k->child("escalationEventDefinition") || k->child("conditionalEventDefinition")) {
        err = "start event with event definition outside the supported subset";
        return false;
      }
      e.event = ZBHIP_EV_NONE;
      if (med) {
        // a message start event of the process (CatchEventTransformer.transformMessageEventDefinition:
        // a static message name, no correlation key), opened as a MessageStartEventSubscription at deploy
        auto mi = msgs.find(med->attr("messageRef"));
        if (mi == msgs.end() || mi->second.first.empty()) {
          err = "message start event outside the supported subset (static name)";
          return false;
        }
        const XNode* ext = k->child("extensionElements");
        if (ext && ext->child("ioMapping")) { err = "io mappings outside the supported subset"; return false; }
        e.event = ZBHIP_EV_MESSAGE;
        e.msg_name = mi->second.first;
      }
    } else if (n == "endEvent" && k->child("errorEventDefinition")) {
      // an error end event (EndEventTransformer.java:70-83: ERROR): a static errorCode (ErrorTransformer)
      e.type = ZBHIP_EL_END_EVENT;
      e.event = ZBHIP_EV_ERROR;
      const std::string ref = k->child("errorEventDefinition")->attr("errorRef");
      auto it = errors.find(ref);
      if (ref.empty() || it == errors.end() || it->second.empty() || it->second[0] == '=' ||
          k->child("messageEventDefinition") || k->child("terminateEventDefinition")) {
        err = "error end event outside the supported subset (a static errorCode)";
        return false;
      }
      e.error_code = it->second;
      const XNode* ext = k->child("extensionElements");
      if (ext && ext->child("ioMapping")) { err = "io mappings outside the supported subset"; return false; }
    } else if (n == "endEvent") {
      e.type = ZBHIP_EL_END_EVENT;
      if (k->child("terminateEventDefinition") || k->child("errorEventDefinition") ||
          k->child("messageEventDefinition") || k->child("escalationEventDefinition") ||
          k->child("signalEventDefinition")) {
        err = "end event with event definition outside the supported subset";
        return false;
      }
      e.event = ZBHIP_EV_NONE;  // EndEventTransformer.java:37
    } else if (n == "serviceTask" || n == "sendTask" || n == "scriptTask" || n == "businessRuleTask") {
      // job worker tasks (BpmnElementProcessors.java:46-60): JobWorkerTaskProcessor, or the job
      // behaviour of ScriptTaskProcessor / BusinessRuleTaskProcessor (a zeebe:taskDefinition)
      e.type = n == "serviceTask" ? ZBHIP_EL_SERVICE_TASK : n == "sendTask" ? ZBHIP_EL_SEND_TASK
               : n == "scriptTask" ? ZBHIP_EL_SCRIPT_TASK : ZBHIP_EL_BUSINESS_RULE_TASK;
      const XNode* ext = k->child("extensionElements");
      if (ext && (ext->child("script") || ext->child("calledDecision"))) {
        err = "script / decision task without a job outside the supported subset";
        return false;
      }
      const XNode* td = ext ? ext->child("taskDefinition") : nullptr;
      if (!td) { err = "service task without zeebe:taskDefinition"; return false; }
      e.job_type = td->attr("type");
      std::string r = td->attr("retries", "3");
      if (e.job_type.empty() || e.job_type[0] == '=' || r.empty() || r[0] == '=') {
        err = "job type/retries expressions outside the supported subset";
        return false;
      }
      e.retries = atoi(r.c_str());
      if (const XNode* th = ext ? ext->child("taskHeaders") : nullptr) {
        // TaskHeadersTransformer (deployment/model/transformer/zeebe/TaskHeadersTransformer.java:24-58):
        // the headers with a non-empty key and value, in document order (Collectors.toMap: a duplicate
        // key fails the deployment)
        for (auto& h : th->kids) {
          if (h->name != "header") continue;
          const std::string hk = h->attr("key"), hv = h->attr("value");
          if (hk.empty() || hv.empty()) continue;
          for (auto& x : e.headers)
            if (x.first == hk) { err = "duplicate task header key"; return false; }
          e.headers.push_back({hk, hv});
        }
      }
      if (!parse_mappings(ext, e, err)) return false;
    } else if (n == "intermediateCatchEvent" && k->child("timerEventDefinition")) {
      // CatchEventTransformer.transformTimerEventDefinition: timeDuration (a static ISO-8601
      // duration, Interval.parse) only; timeDate / timeCycle / expressions outside the subset
      e.type = ZBHIP_EL_INTERMEDIATE_CATCH_EVENT;
      const XNode* ted = k->child("timerEventDefinition");
      const XNode* td = ted->child("timeDuration");
      if (!td || k->child("messageEventDefinition") || k->child("signalEventDefinition")) {
        err = "timer catch event outside the supported subset (timeDuration only)";
        return false;
      }
      const TimerValue tv = timer_value(td->text, false);
      e.timer_ms = tv.ok ? tv.ms : -1;
      if (e.timer_ms < 0 || e.timer_ms > 0xFFFFFFFFLL) { err = "timer duration outside the supported subset: " + td->text; return false; }
      const XNode* ext = k->child("extensionElements");
      if (ext && ext->child("ioMapping")) { err = "io mappings outside the supported subset"; return false; }
      e.event = ZBHIP_EV_TIMER;
    } else if (n == "boundaryEvent" && k->child("errorEventDefinition")) {
      // an error boundary event (BoundaryEventTransformer, ErrorTransformer): interrupting; the errorCode of
      // its <error> (a static code; no errorRef: a catch-all, errorCode "") -- looked up when a job throws
      // an error (CatchEventAnalyzer.findErrorCatchEvent)
      e.type = ZBHIP_EL_BOUNDARY_EVENT;
      e.interrupting = true;
      const XNode* ed = k->child("errorEventDefinition");
      if (k->attr("cancelActivity") == "false" || k->child("timerEventDefinition") || k->child("messageEventDefinition") ||
          k->child("signalEventDefinition") || k->child("escalationEventDefinition")) {
        err = "error boundary event outside the supported subset";
        return false;
      }
      const std::string ref = ed->attr("errorRef");
      if (!ref.empty()) {
        auto it = errors.find(ref);
        if (it == errors.end() || (!it->second.empty() && it->second[0] == '=')) {
          err = "error outside the supported subset (a static errorCode)";
          return false;
        }
        e.error_code = it->second;
      }
      const XNode* ext = k->child("extensionElements");
      if (ext && ext->child("ioMapping")) { err = "io mappings outside the supported subset"; return false; }
      e.event = ZBHIP_EV_ERROR;
      boundaries.push_back({(int)P.els.size(), k->attr("attachedToRef")});
    } else if (n == "boundaryEvent" && k->child("messageEventDefinition")) {
      // a message boundary event, interrupting or not (BoundaryEventTransformer, CatchEventTransformer
      // .transformMessageEventDefinition): static name, `= variable` correlation key -- evaluated in the
      // activity's flow scope (CatchEventBehavior.evaluateCorrelationKey, common/CatchEventBehavior.java:187-205)
      e.type = ZBHIP_EL_BOUNDARY_EVENT;
      e.interrupting = k->attr("cancelActivity") != "false";
      if (k->child("timerEventDefinition") || k->child("errorEventDefinition") || k->child("signalEventDefinition") ||
          k->child("escalationEventDefinition") || k->child("conditionalEventDefinition")) {
        err = "message boundary event outside the supported subset";
        return false;
      }
      auto mi = msgs.find(k->child("messageEventDefinition")->attr("messageRef"));
      if (mi == msgs.end() || mi->second.first.empty() || mi->second.second.empty()) {
        err = "message outside the supported subset (static name, `= variable` correlation key)";
        return false;
      }
      const XNode* ext = k->child("extensionElements");
      if (ext && ext->child("ioMapping")) { err = "io mappings outside the supported subset"; return false; }
      e.event = ZBHIP_EV_MESSAGE;
      e.msg_name = mi->second.first;
      e.corr_var = mi->second.second;
      boundaries.push_back({(int)P.els.size(), k->attr("attachedToRef")});
    } else if (n == "boundaryEvent") {
      // BoundaryEventTransformer (deployment/model/transformer/BoundaryEventTransformer.java):
      // timer boundary events (interrupting or not) with a static timeDuration on job worker tasks only
      e.type = ZBHIP_EL_BOUNDARY_EVENT;
      e.interrupting = k->attr("cancelActivity") != "false";
      const XNode* ted = k->child("timerEventDefinition");
      const XNode* td = ted ? ted->child("timeDuration") : nullptr;
      const XNode* tc = ted && !td ? ted->child("timeCycle") : nullptr;
      if ((!td && !tc) || k->child("messageEventDefinition") || k->child("errorEventDefinition") ||
          k->child("signalEventDefinition") || k->child("escalationEventDefinition") ||
          k->child("compensateEventDefinition") || k->child("conditionalEventDefinition")) {
        err = "boundary event outside the supported subset (timer timeDuration or timeCycle)";
        return false;
      }
      const TimerValue tv = timer_value(td ? td->text : tc->text, tc != nullptr);
      e.reps = tc ? tv.reps : 1;
      e.timer_ms = tv.ok ? tv.ms : -1;
      if (e.timer_ms < 0 || e.timer_ms > 0xFFFFFFFFLL) {
        err = "timer outside the supported subset: " + (td ? td->text : tc->text);
        return false;
      }
      const XNode* ext = k->child("extensionElements");
      if (ext && ext->child("ioMapping")) { err = "io mappings outside the supported subset"; return false; }
      e.event = ZBHIP_EV_TIMER;
      boundaries.push_back({(int)P.els.size(), k->attr("attachedToRef")});
    } else if (n == "intermediateCatchEvent") {
      // CatchEventTransformer.transformMessageEventDefinition (transformer/CatchEventTransformer.java:88-100)
      e.type = ZBHIP_EL_INTERMEDIATE_CATCH_EVENT;
      const XNode* med = k->child("messageEventDefinition");
      if (!med || k->child("timerEventDefinition") || k->child("signalEventDefinition") ||
          k->child("linkEventDefinition") || k->child("conditionalEventDefinition")) {
        err = "intermediate catch event outside the supported subset (message only)";
        return false;
      }
      auto mi = msgs.find(med->attr("messageRef"));
      if (mi == msgs.end() || mi->second.first.empty() || mi->second.second.empty()) {
        err = "message outside the supported subset (static name, `= variable` correlation key)";
        return false;
      }
      e.event = ZBHIP_EV_MESSAGE;
      e.msg_name = mi->second.first;
      e.corr_var = mi->second.second;
    } else if (n == "task" || n == "manualTask") {
      // undefined / manual tasks (BpmnElementProcessors.java:65-68 -> UndefinedTaskProcessor):
      // activities without behaviour, event type UNSPECIFIED
      e.type = n == "task" ? ZBHIP_EL_TASK : ZBHIP_EL_MANUAL_TASK;
      const XNode* ext = k->child("extensionElements");
      if (ext && ext->child("ioMapping")) { err = "io mappings outside the supported subset"; return false; }
    } else if (n == "intermediateThrowEvent") {
      // IntermediateThrowEventProcessor.NoneIntermediateThrowEventBehavior (:113-138): none events only
      e.type = ZBHIP_EL_INTERMEDIATE_THROW_EVENT;
      for (auto& d : k->kids)
        if (d->name.size() > 15 && d->name.compare(d->name.size() - 15, 15, "EventDefinition") == 0) {
          err = "intermediate throw event with event definition outside the supported subset";
          return false;
        }
      const XNode* ext = k->child("extensionElements");
      if (ext && ext->child("ioMapping")) { err = "io mappings outside the supported subset"; return false; }
      e.event = ZBHIP_EV_NONE;
    } else if (n == "subProcess" && k->attr("triggeredByEvent") == "true") {
      // an event sub-process (SubProcessTransformer.transformEventSubprocess :36-60): EVENT_SUB_PROCESS,
      // attached to its container -- the process or an embedded sub-process; one error start event
      e.type = ZBHIP_EL_EVENT_SUB_PROCESS;
      const XNode* ext = k->child("extensionElements");
      if ((ext && ext->child("ioMapping")) || k->child("multiInstanceLoopCharacteristics") ||
          k->child("standardLoopCharacteristics") ||
          (P.els[scope].type != ZBHIP_EL_PROCESS && P.els[scope].type != ZBHIP_EL_SUB_PROCESS)) {
        err = "event sub-process outside the supported subset";
        return false;
      }
    } else if (n == "subProcess") {
      // embedded sub-process (SubProcessProcessor): no loop
      e.type = ZBHIP_EL_SUB_PROCESS;
      if (k->child("multiInstanceLoopCharacteristics") || k->child("standardLoopCharacteristics")) {
        err = "multi-instance outside the supported subset";
        return false;
      }
      if (!parse_mappings(k->child("extensionElements"), e, err)) return false;
    } else if (n == "exclusiveGateway") {
      e.type = ZBHIP_EL_EXCLUSIVE_GATEWAY;
      xgws.push_back(k.get());
    } else if (n == "parallelGateway") {
      e.type = ZBHIP_EL_PARALLEL_GATEWAY;
    } else if (n == "sequenceFlow") {
      e.type = ZBHIP_EL_SEQUENCE_FLOW;
      flows.push_back(k.get());
    } else if (n == "extensionElements" || n == "documentation" || n == "textAnnotation" ||
               n == "association" || n == "incoming" || n == "outgoing") {
      continue;
    } else {
      err = "element <" + n + "> outside the supported subset";
      return false;
    }
    if (e.id.empty()) { err = "element without id"; return false; }
    if (k->child("standardLoopCharacteristics")) { err = "standard loop outside the supported subset"; return false; }
    if (const XNode* mil = k->child("multiInstanceLoopCharacteristics")) {
      // MultiInstanceActivityTransformer.transform (:35-78): the body takes the activity's id, flow
      // scope and sequence flows; the inner activity's flow scope is the body
      if (!ZBHIP_IS_JOB_WORKER(e.type) && e.type != ZBHIP_EL_TASK && e.type != ZBHIP_EL_MANUAL_TASK) {
        err = "multi-instance " + n + " outside the supported subset (job worker and undefined tasks)";
        return false;
      }
      if (e.in_map.present || e.out_map.present) {
        // an inner multi-instance activity maps in its own scope (getVariableScopeKey): outside the subset
        err = "io mappings of a multi-instance activity outside the supported subset";
        return false;
      }
      OEl b;
      b.id = e.id;
      b.type = ZBHIP_EL_MULTI_INSTANCE_BODY;
      b.scope = scope;
      if (!parse_multi_instance(*mil, b, err)) return false;
      const int bi = (int)P.els.size();
      b.inner = bi + 1;
      idx[e.id] = bi;
      P.els.push_back(std::move(b));
      e.scope = bi;
      P.els.push_back(std::move(e));
      continue;
    }
    const int self = (int)P.els.size();
    const int type = e.type, event = e.event;
    idx[e.id] = self;
    P.els.push_back(std::move(e));
    if (type == ZBHIP_EL_SUB_PROCESS) {
      if (!walk(*k, self)) return false;
      if (P.els[self].start < 0) { err = "sub-process without a none start event"; return false; }
    } else if (type == ZBHIP_EL_EVENT_SUB_PROCESS) {
      if (!walk(*k, self)) return false;
      if (P.els[self].start < 0) { err = "event sub-process without an error start event"; return false; }
      P.els[scope].esps.push_back(self);  // ExecutableActivity.attach(eventSubprocess)
    } else if (type == ZBHIP_EL_START_EVENT && P.els[scope].type == ZBHIP_EL_EVENT_SUB_PROCESS) {
      if (event != ZBHIP_EV_ERROR || P.els[scope].start >= 0) {
        err = "event sub-process start event outside the supported subset";
        return false;
      }
      P.els[scope].start = self;
    } else if (type == ZBHIP_EL_START_EVENT && event == ZBHIP_EV_NONE) {
      P.els[scope].start = self;
    } else if (type == ZBHIP_EL_START_EVENT) {
      P.msg_starts.push_back(self);
    }
  }
  return true;
  };
  if (!walk(proc, 0)) return false;
  // BoundaryEventTransformer: attach to the activity (ExecutableActivity.attach, ExecutableActivity.java:28-38)
  for (auto& [b, ref] : boundaries) {
    auto it = idx.find(ref);
    if (it == idx.end()) { err = "boundary event attached to an unknown element"; return false; }
    OEl& a = P.els[it->second];
    // job worker tasks; embedded sub-processes with a timer boundary event (subscribed when their start
    // event completes, StartEventProcessor.onComplete :52-67) or an error boundary event (found by
    // CatchEventAnalyzer's walk through the flow scopes of a job's task)
    const bool sub_ok = a.type == ZBHIP_EL_SUB_PROCESS &&
                        (P.els[b].event == ZBHIP_EV_TIMER || P.els[b].event == ZBHIP_EV_ERROR);
    // (an error boundary event of a multi-instance activity attaches to its body, MultiInstanceActivity
    // Transformer: the body takes the activity's id)
    const bool body_ok = a.type == ZBHIP_EL_MULTI_INSTANCE_BODY && P.els[b].event == ZBHIP_EV_ERROR;
    if ((!ZBHIP_IS_JOB_WORKER(a.type) && !sub_ok && !body_ok) || a.scope != P.els[b].scope) {
      err = "boundary event on an element outside the supported subset (job worker tasks, timers on sub-processes)";
      return false;
    }
    // several error boundary events beside at most one timer / message boundary event
    if (a.boundary >= 0) {
      if (P.els[a.boundary].event != ZBHIP_EV_ERROR && P.els[b].event != ZBHIP_EV_ERROR) {
        err = "more than one timer / message boundary event on an activity outside the supported subset";
        return false;
      }
      if (P.els[b].event != ZBHIP_EV_ERROR) a.boundary = b;
    } else {
      a.boundary = b;
    }
    a.boundaries.push_back(b);
    P.els[b].attached = it->second;
  }
  // gateway default flows (ExclusiveGatewayTransformer.transformDefaultFlow)
  for (const XNode* k : xgws) {
    if (!k->attr("default").empty()) {
      auto it = idx.find(k->attr("default"));
      if (it == idx.end()) { err = "unknown default flow"; return false; }
      P.els[idx[k->attr("id")]].default_flow = it->second;
    }
  }
  // step 2 walk: reverse document order (ModelWalker.java:75-79)
  for (auto it = flows.rbegin(); it != flows.rend(); ++it) {
    const XNode* f = *it;
    int fi = idx[f->attr("id")];
    auto s = idx.find(f->attr("sourceRef"));
    auto t = idx.find(f->attr("targetRef"));
    if (s == idx.end() || t == idx.end()) { err = "flow with unknown source/target"; return false; }
    OEl& fe = P.els[fi];
    if (P.els[s->second].scope != fe.scope || P.els[t->second].scope != fe.scope) {
      err = "sequence flow crossing a sub-process boundary";
      return false;
    }
    fe.src = s->second;
    fe.tgt = t->second;
    // SequenceFlowTransformer.parseCondition: runs before connectWithFlowNodes
    if (const XNode* c = f->child("conditionExpression")) {
      std::string txt = c->text;
      size_t a = txt.find_first_not_of(" \t\r\n");
      size_t b = txt.find_last_not_of(" \t\r\n");
      txt = a == std::string::npos ? "" : txt.substr(a, b - a + 1);
      fe.has_cond = true;
      if (txt.empty() || txt[0] != '=') { err = "static (non-FEEL) condition outside the subset"; return false; }
      fe.cond_text = txt.substr(1);
      FeelParser fp(txt.substr(1));
      fe.cond = fp.parse_or();
      fp.ws();
      if (!fp.ok || fp.i != fp.s.size()) { err = "FEEL condition outside the subset: " + txt; return false; }
    }
    P.els[fe.src].out.push_back(fi);  // ExecutableFlowNode.addOutgoing
    if (P.els[fe.src].type == ZBHIP_EL_EXCLUSIVE_GATEWAY && fe.has_cond)
      P.els[fe.src].out_with_cond.push_back(fi);  // ExecutableExclusiveGateway.addOutgoing
    P.els[fe.tgt].in.push_back(fi);
  }
  P.none_start = P.els[0].start;
  return true;
}

// ---------------------------------------------------------------------------
// Engine state (zb-db column families, protocol/.../ZbColumnFamilies.java)
// ---------------------------------------------------------------------------
struct PiValue {  // ProcessInstanceRecord (protocol-impl/.../ProcessInstanceRecord.java:36-72)
  int proc = -1;
  int elem = -1;
  int64_t flowScopeKey = -1;
  int64_t piKey = -1;
};

struct ElementInstance {  // state/instance/ElementInstance.java:23-54
  int64_t key = -1;
  int64_t parentKey = -1;
  int childCount = 0;
  int64_t jobKey = 0;
  int state = 0;
  PiValue value;
  int activeSequenceFlows = 0;
  int childActivated = 0, childCompleted = 0, childTerminated = 0, loopCounter = 0;  // multi-instance (ElementInstance.java:25-33)
  int interrupting_elem = -1;  // interruptingElementId: the interrupting event sub-process (EventSubProcessInterruptionMarker)
};

struct Doc {  // a variable document (msgpack map) as a list of entries
  uint32_t begin = 0;
  uint32_t count = 0;
};

struct JobRow {  // JobRecord without variables (DbJobState.createJobRecord)
  PiValue pi;
  int64_t elementInstanceKey = -1;
  std::string type;
  int retries = 3;
  bool activated = false;  // JOB_STATES ACTIVATED (DbJobState.activate :118-133)
  bool failed = false;     // JOB_STATES FAILED (DbJobState.fail :191-203)
  int64_t deadline = -1;
  std::string worker;
  // JobFailProcessor.failJob (:103-125) stored them: the record's retries / errorMessage /
  // retryBackoff / recurringTime differ from JOB:CREATED's from then on
  bool fail_fields = false;
  std::string error_message;
  int64_t retry_backoff = 0, recurring_time = -1;
  // JobThrowErrorProcessor with no catch event (DbJobState.throwError): ERROR_THROWN, the stored record's
  // errorCode, and its elementId the NO_CATCH_EVENT_FOUND marker
  bool error_thrown = false, no_catch = false;
  std::string error_code;
};

// java.lang.String.hashCode over the UTF-16 code units of UTF-8 text
static int32_t jstring_hash(const std::string& s) {
  uint32_t h = 0;
  size_t i = 0;
  while (i < s.size()) {
    const unsigned char c = (unsigned char)s[i];
    const int n = c < 0x80 ? 1 : c < 0xE0 ? 2 : c < 0xF0 ? 3 : 4;
    uint32_t cp = n == 1 ? c : n == 2 ? (c & 0x1Fu) : n == 3 ? (c & 0x0Fu) : (c & 0x07u);
    for (int k = 1; k < n; ++k) cp = (cp << 6) | (i + k < s.size() ? ((unsigned char)s[i + k] & 0x3Fu) : 0u);
    i += (size_t)n;
    if (cp > 0xFFFF) {
      h = 31u * h + (0xD800u + ((cp - 0x10000u) >> 10));
      h = 31u * h + (0xDC00u + ((cp - 0x10000u) & 0x3FFu));
    } else {
      h = 31u * h + cp;
    }
  }
  return (int32_t)h;
}

// java.util.HashMap<String, String> (JDK 21) as far as its iteration order goes: a power-of-two table of
// insertion-ordered chains, hash (h ^ h >>> 16) & (n - 1), resize at size > 3/4 capacity (chains split in
// order), first table 16 -- or, pre-sized by HashMap(Map) (putMapEntries), tableSizeFor(ceil(s / 0.75)).
// A chain reaching TREEIFY_THRESHOLD would turn into a tree (or resize early): outside the restatement.
struct JHashMap {
  std::vector<std::vector<std::pair<std::string, std::string>>> tab;
  size_t size = 0, threshold = 0;
  static uint32_t spread(const std::string& k) {
    const uint32_t h = (uint32_t)jstring_hash(k);
    return h ^ (h >> 16);
  }
  void resize() {
    const size_t cap = tab.empty() ? (threshold ? threshold : 16) : tab.size() * 2;
    std::vector<std::vector<std::pair<std::string, std::string>>> t(cap);
    for (auto& b : tab)
      for (auto& e : b) t[spread(e.first) & (cap - 1)].push_back(e);
    tab.swap(t);
    threshold = cap / 4 * 3;
  }
  void presize(size_t s) {  // HashMap(Map m) -> putMapEntries (table == null)
    if (!s) return;
    const size_t t = (size_t)std::ceil((double)s / 0.75);
    size_t c = 1;
    while (c < t) c <<= 1;
    threshold = c;
  }
  bool put(const std::string& k, const std::string& v) {
    if (tab.empty()) resize();
    auto& b = tab[spread(k) & (tab.size() - 1)];
    for (auto& e : b)
      if (e.first == k) { e.second = v; return true; }
    if (b.size() >= 8) return false;
    b.push_back({k, v});
    if (++size > threshold) resize();
    return true;
  }
  std::vector<std::pair<std::string, std::string>> entries() const {
    std::vector<std::pair<std::string, std::string>> o;
    for (auto& b : tab) o.insert(o.end(), b.begin(), b.end());
    return o;
  }
};

// msgpack (MsgPackWriter.writeMapHeader / writeString): fix / 8 / 16 / 32-bit forms, big-endian lengths
static void mp_len(std::string& o, uint32_t n, uint8_t fix, uint32_t fix_max, uint8_t b8, uint8_t b16, uint8_t b32) {
  if (n <= fix_max) { o += (char)(fix | n); return; }
  if (b8 && n <= 0xFF) { o += (char)b8; o += (char)n; return; }
  if (n <= 0xFFFF) { o += (char)b16; o += (char)(n >> 8); o += (char)n; return; }
  o += (char)b32;
  for (int k = 3; k >= 0; --k) o += (char)(n >> (8 * k));
}

// BpmnJobBehavior.writeJobCreatedEvent -> encodeHeaders (processing/bpmn/behavior/BpmnJobBehavior.java:194-248):
// the transformer's map (Collectors.toMap over the document-ordered headers), copied with new HashMap<>(m),
// then HeaderEncoder.encode (:365-399) collects the valid entries into a third HashMap (Collectors.toMap)
// and writes its entries in iteration order; no headers: JobRecord.NO_HEADERS (an empty map)
static bool encode_headers(const std::vector<std::pair<std::string, std::string>>& hs, std::string& out) {
  out.clear();
  if (hs.empty()) return true;
  JHashMap h1, h2, h3;
  for (auto& [k, v] : hs)
    if (!h1.put(k, v)) return false;
  h2.presize(h1.size);
  for (auto& [k, v] : h1.entries())
    if (!h2.put(k, v)) return false;
  for (auto& [k, v] : h2.entries())
    if (!k.empty() && !v.empty() && !h3.put(k, v)) return false;
  mp_len(out, (uint32_t)h3.size, 0x80, 15, 0, 0xDE, 0xDF);
  for (auto& [k, v] : h3.entries()) {
    mp_len(out, (uint32_t)k.size(), 0xA0, 31, 0xD9, 0xDA, 0xDB);
    out += k;
    mp_len(out, (uint32_t)v.size(), 0xA0, 31, 0xD9, 0xDA, 0xDB);
    out += v;
  }
  return true;
}

// hex of a string in a state row (error messages may hold ',' and '|')
static std::string hex_of(const std::string& v) {
  static const char* d = "0123456789abcdef";
  std::string o;
  for (unsigned char c : v) { o += d[c >> 4]; o += d[c & 15]; }
  return o;
}
static std::string unhex(const std::string& h) {
  std::string o;
  for (size_t i = 0; i + 1 < h.size(); i += 2) o += (char)std::stoi(h.substr(i, 2), nullptr, 16);
  return o;
}

struct EventTrigger {  // state/instance/EventTrigger.java
  int elem = -1;
  int proc = -1;
  Doc vars;
  int64_t piKey = -1;
};

struct VarRow {
  int64_t key;
  uint8_t type;
  int64_t value;
  uint32_t doc_index;
};

// Message values (MessageSubscriptionRecord / ProcessMessageSubscriptionRecord / MessageRecord,
// protocol-impl/.../record/value/message/*.java) in compact form, plus the routing handle of the
// subscribing element instance (instance slot, key ordinal) that the cross-partition commands carry.
struct MsgVal {
  int64_t pik = -1, eik = -1, msg_key = -1;
  uint32_t corr = ZBHIP_NO_STRING;
  uint16_t name = 0xFFFF, bpmn = 0xFFFF;
  int32_t partition = 0;
  uint8_t interrupting = 0;
  int proc = -1, elem = -1;  // PMS records that carry the elementId
  uint32_t inst = 0;
  uint16_t eord = 0;
  // MESSAGE:PUBLISH (MessageRecord.java:37-43): timeToLive, messageId (string id), the command's timestamp
  int64_t ttl = 0, timestamp = 0;
  uint32_t message_id = ZBHIP_NO_STRING;
};

// A command or event in flight (TypedRecord)
struct ORecord {
  zbhip_record r;
  MsgVal m;
  PiValue pi;          // for PI records
  Doc doc;             // variables carried (CREATE/JOB_COMPLETE/ VARIABLE entry)
  std::string reason;  // rejection reason
  uint32_t instance = 0;
  int32_t job_ord = -1;
  bool slot = false;   // subject is the correlation slot `instance` (MESSAGE / MESSAGE_SUBSCRIPTION commands)
};

static void fill_msg(ORecord& rec, const MsgVal& m) {
  rec.m = m;
  rec.r.scope_key = m.eik;
  rec.r.process_instance_key = m.pik;
  rec.r.message_key = m.msg_key;
  rec.r.correlation_key = m.corr;
  rec.r.message_name = m.name;
  rec.r.bpmn_process_id = m.bpmn;
  rec.r.partition = m.partition;
  rec.r.interrupting = m.interrupting;
  rec.r.process_idx = m.proc;
  rec.r.element_idx = m.elem;
}

static void xpart_kind(int kind, int& vt, int& intent) {
  switch (kind) {
    case ZBHIP_CMD_MSG_SUB_CREATE: vt = ZBHIP_VT_MESSAGE_SUBSCRIPTION; intent = ZBHIP_MS_CREATE; return;
    case ZBHIP_CMD_MSG_SUB_CORRELATE: vt = ZBHIP_VT_MESSAGE_SUBSCRIPTION; intent = ZBHIP_MS_CORRELATE; return;
    case ZBHIP_CMD_PMS_CREATE: vt = ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION; intent = ZBHIP_PMS_CREATE; return;
    case ZBHIP_CMD_MSG_SUB_DELETE: vt = ZBHIP_VT_MESSAGE_SUBSCRIPTION; intent = ZBHIP_MS_DELETE; return;
    case ZBHIP_CMD_PMS_DELETE: vt = ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION; intent = ZBHIP_PMS_DELETE; return;
    default: vt = ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION; intent = ZBHIP_PMS_CORRELATE; return;
  }
}

// The record value each SubscriptionCommandSender method writes (SubscriptionCommandSender.java:54-338):
// openMessageSubscription: pik, eik, bpmnProcessId, messageKey -1, name, correlationKey, interrupting;
// openProcessMessageSubscription: subscriptionPartitionId = sender, pik, eik, messageKey -1, name, interrupting;
// correlateProcessMessageSubscription: subscriptionPartitionId = sender, pik, eik, bpmnProcessId, messageKey,
//   name, variables, correlationKey;  correlateMessageSubscription: pik, eik, bpmnProcessId, messageKey -1, name;
// closeMessageSubscription: pik, eik, messageKey -1, name (:220-236); closeProcessMessageSubscription:
//   subscriptionPartitionId = sender, pik, eik, messageKey -1, name (:267-283).
// Properties not set keep their declared defaults: interrupting = true (MessageSubscriptionRecord.java:33,
// ProcessMessageSubscriptionRecord.java:37), strings "", messageKey -1.
static MsgVal command_value(int kind, const MsgVal& in, int sender) {
  MsgVal m;
  m.pik = in.pik;
  m.eik = in.eik;
  m.name = in.name;
  m.inst = in.inst;
  m.eord = in.eord;
  switch (kind) {
    case ZBHIP_CMD_MSG_SUB_CREATE:
      m.bpmn = in.bpmn; m.corr = in.corr; m.interrupting = in.interrupting; break;
    case ZBHIP_CMD_PMS_CREATE:
      m.partition = sender; m.interrupting = in.interrupting; break;
    case ZBHIP_CMD_PMS_CORRELATE:  // interrupting keeps its default (true)
      m.partition = sender; m.bpmn = in.bpmn; m.msg_key = in.msg_key; m.corr = in.corr; m.interrupting = 1; break;
    case ZBHIP_CMD_MSG_SUB_DELETE:
      m.interrupting = 1; break;
    case ZBHIP_CMD_PMS_DELETE:
      m.partition = sender; m.interrupting = 1; break;
    default:  // MSG_SUB_CORRELATE; interrupting keeps its default (true)
      m.bpmn = in.bpmn; m.interrupting = 1; break;
  }
  return m;
}

// SubscriptionUtil.getSubscriptionHashCode / getSubscriptionPartitionId
// (protocol-impl/.../SubscriptionUtil.java:22-44): String#hashCode over SIGNED bytes, Java int
// overflow, then abs(hash % partitionCount) + START_PARTITION_ID.
static int32_t java_hash(const std::string& b) {
  uint32_t h = 0;
  for (char c : b) h = 31u * h + (uint32_t)(int32_t)(int8_t)c;
  return (int32_t)h;
}
static int subscription_partition(const std::string& b, int partition_count) {
  int32_t h = java_hash(b);
  int32_t r = h % partition_count;
  return (r < 0 ? -r : r) + 1;
}

// StringUtil.limitString(message, maxLength) (util/.../StringUtil.java:50-56) on the UTF-8 bytes of a Java
// String: the length counts UTF-16 code units (a character beyond the BMP is two); a cut inside a
// surrogate pair keeps the lone high surrogate, which String.getBytes(UTF_8) writes as '?'
static std::string limit_java_string(const std::string& s, size_t max_units) {
  size_t units = 0, i = 0;
  while (i < s.size()) {
    const unsigned char c = (unsigned char)s[i];
    const size_t len = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : 4;
    const size_t u = len == 4 ? 2 : 1;
    if (units + u > max_units) return s.substr(0, i) + (units < max_units ? "?" : "") + "...";
    units += u;
    i += len;
  }
  return s;
}

struct Unsupported {
  std::string what;
};

// org.agrona.collections.Int2IntHashMap (third-party agrona 1.19.2, parent/pom.xml:38; not in the
// reference tree), as IndexedDocument (state/variable/IndexedDocument.java:20-63) uses it: missingValue -1,
// entries = int[2 * capacity] of (key, value) pairs, capacity 8 at first, resizeThreshold = (int)(capacity
// * 0.65f).  put: index = Hashing.evenHash(key, mask) = ((key << 1) - (key << 8)) & mask over the pair
// array (mask = entries.length - 1), probing index + 2 until a free value slot; past the threshold
// rehash(doubled) re-puts the old pairs in array order.  Iteration (AbstractIterator.reset / findNext):
// from the top pair down, or, when the top pair is taken, from just below the first free pair, once
// around.  Iterator.remove frees the pair and compactChain(deleteIndex) pulls later chain members back.
// Published algorithm, restated; the reference's tests do not pin a multi-entry document's order.
struct AgronaIntMap {
  std::vector<int32_t> e;
  int size = 0, threshold = 0;
  AgronaIntMap() { capacity(8); }
  void capacity(int c) {
    threshold = (int)((float)c * 0.65f);
    e.assign((size_t)2 * c, -1);
  }
  int mask() const { return (int)e.size() - 1; }
  static int even_hash(int32_t v, int m) { return (int)(((uint32_t)v << 1) - ((uint32_t)v << 8)) & m; }
  void put(int32_t key, int32_t value) {
    int i = even_hash(key, mask());
    while (e[i + 1] != -1) {
      if (e[i] == key) { e[i + 1] = value; return; }
      i = (i + 2) & mask();
    }
    ++size;
    e[i] = key;
    e[i + 1] = value;
    if (size > threshold) {  // increaseCapacity -> rehash(entries.length)
      const std::vector<int32_t> old = e;
      capacity((int)old.size());
      for (size_t k = 0; k < old.size(); k += 2) {
        if (old[k + 1] == -1) continue;
        int j = even_hash(old[k], mask());
        while (e[j + 1] != -1) j = (j + 2) & mask();
        e[j] = old[k];
        e[j + 1] = old[k + 1];
      }
    }
  }
  struct Iter {
    int remaining = 0, position = 0, stop = 0;
    bool valid = false;
  };
  Iter iterator() const {
    Iter it;
    it.remaining = size;
    const int cap = (int)e.size();
    int i = cap;
    if (e[cap - 1] != -1)
      for (i = 0; i < cap; i += 2)
        if (e[i + 1] == -1) break;
    it.stop = i;
    it.position = i + cap;
    return it;
  }
  // the key of the next entry, false at the end
  bool next(Iter& it, int32_t& key) const {
    if (it.remaining <= 0) return false;
    for (int i = it.position - 2; i >= it.stop; i -= 2) {
      const int idx = i & mask();
      if (e[idx + 1] != -1) {
        it.valid = true;
        it.position = i;
        --it.remaining;
        key = e[idx];
        return true;
      }
    }
    throw Unsupported{"agrona iterator past its entries"};
  }
  void remove(Iter& it) {
    int del = it.position & mask();
    e[del + 1] = -1;
    --size;
    for (int i = del;;) {  // compactChain
      i = (i + 2) & mask();
      if (e[i + 1] == -1) break;
      const int h = even_hash(e[i], mask());
      if ((i < h && (h <= del || del <= i)) || (h <= del && del <= i)) {
        e[del] = e[i];
        e[del + 1] = e[i + 1];
        e[i + 1] = -1;
        del = i;
      }
    }
    it.valid = false;
  }
};

class Oracle {
 public:
  Oracle(int partition, int partition_count, int max_cmds, int64_t initial_key)
      : partition_(partition), partition_count_(partition_count), max_cmds_(max_cmds) {
    key_counter_ = initial_key;
  }

  std::vector<OProc> procs;
  std::vector<std::string> names;
  std::unordered_map<std::string, int> name_ids;
  std::vector<zbhip_doc_entry> docs;  // all submitted document entries (global index)
  std::vector<zbhip_xpart_cmd> xdocs;  // all received cross-partition commands (global index)
  std::vector<zbhip_xpart_cmd> outbox;  // sent cross-partition commands (post-commit side effects)
  std::vector<std::string> notified;    // job types of publishWork's notifyJobAvailable side effects
  bool track_notified = false;          // (kept only when a caller takes them: zbo_take_notified)
  std::string last_error;

  // value dictionary (zbhip_intern_string)
  std::vector<std::string> strs;
  std::unordered_map<std::string, uint32_t> str_ids;
  const std::vector<std::string>* shared_strs = nullptr;  // bench: one dictionary for all partitions
  const std::string& str(uint32_t id) const { return shared_strs ? shared_strs->at(id) : strs.at(id); }
  uint32_t intern_string(const std::string& v) {
    auto it = str_ids.find(v);
    if (it != str_ids.end()) return it->second;
    uint32_t id = (uint32_t)strs.size();
    strs.push_back(v);
    str_ids.emplace(v, id);
    return id;
  }

  // the list dictionary (ZBHIP_DOC_LIST values: a list of scalar items, each (zbhip_doc_type, value))
  using Items = std::vector<std::pair<uint8_t, int64_t>>;
  std::vector<Items> lists;
  std::map<Items, int> list_ids;
  int64_t intern_list(const Items& items) {
    auto it = list_ids.find(items);
    if (it != list_ids.end()) return it->second;
    const int id = (int)lists.size();
    lists.push_back(items);
    list_ids.emplace(items, id);
    return id;
  }
  static std::string list_text(const Items& items) {
    std::string o;
    for (size_t i = 0; i < items.size(); ++i) {
      if (i) o += ';';
      o += std::to_string((int)items[i].first) + ":" + std::to_string((long long)items[i].second);
    }
    return o;
  }
  static Items parse_list_text(const std::string& t) {
    Items items;
    size_t a = 0;
    while (a < t.size()) {
      size_t b = t.find(';', a);
      if (b == std::string::npos) b = t.size();
      const std::string it = t.substr(a, b - a);
      const size_t c = it.find(':');
      items.push_back({(uint8_t)std::stoi(it.substr(0, c)), (int64_t)std::stoll(it.substr(c + 1))});
      a = b + 1;
    }
    return items;
  }

  int intern(const std::string& n) {
    auto it = name_ids.find(n);
    if (it != name_ids.end()) return it->second;
    int id = (int)names.size();
    names.push_back(n);
    name_ids[n] = id;
    return id;
  }

  int deploy(const std::string& xml, int64_t def_key, int version) {
    XmlParser xp(xml);
    auto root = xp.parse_element();
    if (!root) { last_error = "xml: " + xp.err; return ZBHIP_EPARSE; }
    const XNode* proc = nullptr;
    for (auto& k : root->kids)
      if (k->name == "process" && k->attr("isExecutable", "true") != "false") { proc = k.get(); break; }
    if (!proc) { last_error = "no executable process"; return ZBHIP_EPARSE; }
    // <message> definitions: static name, correlation key `= variable` (MessageTransformer.java:30-60)
    MessageDefs msgs;
    for (auto& k : root->kids) {
      if (k->name != "message") continue;
      std::string nm = k->attr("name"), ck;
      const XNode* ext = k->child("extensionElements");
      const XNode* sub = ext ? ext->child("subscription") : nullptr;
      if (sub) ck = sub->attr("correlationKey");
      auto trim = [](std::string t) {
        size_t a = t.find_first_not_of(" \t\r\n"), b = t.find_last_not_of(" \t\r\n");
        return a == std::string::npos ? std::string() : t.substr(a, b - a + 1);
      };
      ck = trim(ck);
      std::string var;
      if (ck.size() >= 2 && ck[0] == '=') {
        var = trim(ck.substr(1));
        bool ident = !var.empty() && (isalpha((unsigned char)var[0]) || var[0] == '_');
        for (char ch : var) ident = ident && (isalnum((unsigned char)ch) || ch == '_');
        if (!ident) var.clear();
      }
      if (!nm.empty() && nm[0] == '=') nm.clear();
      msgs[k->attr("id")] = {nm, var};
    }
    ErrorDefs errors;  // <error> elements of the definitions (ErrorTransformer: errorCode)
    for (auto& k : root->kids)
      if (k->name == "error") errors[k->attr("id")] = k->attr("errorCode");
    OProc P;
    if (!build_process(*proc, msgs, errors, P, last_error)) return ZBHIP_EUNSUPP;
    P.def_key = def_key;
    P.version = version;
    // intern condition variable names now so ids match the product's deploy order
    for (auto& e : P.els) intern_vars(e.cond.get());
    // message names, correlation variables and the bpmnProcessId of processes with message catch
    // events go into the same name dictionary (the product's zbhip_deploy interns in this order)
    bool has_msg = false;
    for (auto& e : P.els)
      if ((e.type == ZBHIP_EL_INTERMEDIATE_CATCH_EVENT || e.type == ZBHIP_EL_BOUNDARY_EVENT) && e.event == ZBHIP_EV_MESSAGE) {
        intern(e.msg_name);
        intern(e.corr_var);
        has_msg = true;
      }
    if (has_msg) intern(P.bpmn_id);
    // multi-instance bodies, in element order: the inputElement and loopCounter names, then the string
    // items into the value dictionary (the product's zbhip_deploy interns in this order)
    for (auto& e : P.els) {
      if (e.type != ZBHIP_EL_MULTI_INSTANCE_BODY) continue;
      if (!e.mi_input.empty()) e.mi_input_id = intern(e.mi_input);
      e.mi_loop_id = intern("loopCounter");
      for (size_t j = 0; j < e.mi_items.size(); ++j)
        if (e.mi_items[j].first == ZBHIP_DOC_STR) e.mi_items[j].second = intern_string(e.mi_item_text[j]);
      // then the collection variable, the outputCollection and outputElement names, the completion
      // condition's variables
      if (!e.mi_coll_name.empty()) e.mi_coll_id = intern(e.mi_coll_name);
      if (!e.mi_out_coll.empty()) {
        e.mi_out_coll_id = intern(e.mi_out_coll);
        e.mi_out_elem_id = intern(e.mi_out_elem);
      }
      intern_vars(e.mi_cond.get());
    }
    // io mappings, in element order: the input's source variable and target, then the output's (the
    // product's zbhip_deploy interns in this order); string literals into the value dictionary
    for (auto& e : P.els)
      for (OEl::Mapping* M : {&e.in_map, &e.out_map}) {
        if (!M->present) continue;
        if (M->var) M->source_id = intern(M->source);
        else if (M->type == ZBHIP_DOC_STR) M->value = intern_string(M->source);
        M->target_id = intern(M->target);
      }
    for (auto& e : P.els)
      if (!encode_headers(e.headers, e.header_bytes)) {
        last_error = "task headers a HashMap would treeify";
        return ZBHIP_EUNSUPP;
      }
    std::set<std::string> start_names;
    for (int s : P.msg_starts) {
      if (!start_names.insert(P.els[s].msg_name).second) {
        last_error = "two message start events with one message name";
        return ZBHIP_EUNSUPP;
      }
      intern(P.els[s].msg_name);
    }
    if (!P.msg_starts.empty()) P.bpmn_name = intern(P.bpmn_id);
    procs.push_back(std::move(P));
    open_start_event_subscriptions((int)procs.size() - 1);
    return (int)procs.size() - 1;
  }

  // StartEventSubscriptionManager.tryReOpenStartEventSubscription (processing/deployment/
  // StartEventSubscriptionManager.java:46-140) for a deployed process that is the latest version of its
  // bpmnProcessId: the previous versions' message start event subscriptions closed, its own opened
  // (MessageStartEventSubscriptionCreatedApplier / DeletedApplier: DbMessageStartEventSubscriptionState
  // .put / remove).  Deployment runs outside the processing loop here, so no CREATED / DELETED records
  // are written, and a subscription's key stands at its process definition key.
  void open_start_event_subscriptions(int proc) {
    const OProc& p = procs[proc];
    for (size_t i = 0; i < procs.size(); ++i)
      if ((int)i != proc && procs[i].bpmn_id == p.bpmn_id && procs[i].version > p.version) return;
    for (auto it = msg_start_subs_.begin(); it != msg_start_subs_.end();)
      it = procs[it->second.proc].bpmn_id == p.bpmn_id ? msg_start_subs_.erase(it) : std::next(it);
    for (int s : p.msg_starts)
      msg_start_subs_[{intern(p.els[s].msg_name), p.def_key}] = MsgStartSub{proc, s, p.def_key};
  }

  void intern_vars(const FExpr* e) {
    if (!e) return;
    if (e->op == FExpr::VAR) intern(e->var);
    intern_vars(e->l.get());
    intern_vars(e->r.get());
  }

  // Writes external commands to the log (the client side of EngineRule).
  void submit(const zbhip_command* cmds, size_t n, const zbhip_doc_entry* d, size_t nd,
              const zbhip_xpart_cmd* xp = nullptr, size_t nx = 0) {
    uint32_t doc_base = (uint32_t)docs.size();
    docs.insert(docs.end(), d, d + nd);
    uint32_t x_base = (uint32_t)xdocs.size();
    if (nx) xdocs.insert(xdocs.end(), xp, xp + nx);
    for (size_t i = 0; i < n; ++i) {
      const zbhip_command& c = cmds[i];
      ORecord rec{};
      std::memset(&rec.r, 0, sizeof(rec.r));
      rec.r.record_type = ZBHIP_RT_COMMAND;
      rec.r.rejection_type = ZBHIP_REJ_NONE;
      rec.instance = c.instance;
      rec.doc = Doc{doc_base + c.doc_begin, c.doc_count};
      rec.r.process_idx = -1;
      rec.r.element_idx = -1;
      rec.r.scope_key = -1;
      rec.r.process_instance_key = -1;
      rec.r.aux = c.doc_count ? (int64_t)(doc_base + c.doc_begin) : -1;
      rec.r.message_key = -1;
      rec.r.correlation_key = ZBHIP_NO_STRING;
      rec.r.message_name = 0xFFFF;
      rec.r.bpmn_process_id = 0xFFFF;
      if (c.kind == ZBHIP_CMD_CREATE) {
        rec.r.process_idx = c.ref;
        rec.r.value_type = ZBHIP_VT_PROCESS_INSTANCE_CREATION;
        rec.r.intent = ZBHIP_PIC_CREATE;
        rec.r.key = -1;
      } else if (c.kind == ZBHIP_CMD_PUBLISH) {
        // MessageRecord: name, correlationKey, timeToLive 0, no variables, no messageId
        rec.doc = Doc{0, 0};
        rec.r.aux = -1;
        rec.r.value_type = ZBHIP_VT_MESSAGE;
        rec.r.intent = ZBHIP_MSG_PUBLISH;
        rec.r.key = -1;
        rec.m.corr = c.instance;
        rec.m.name = c.ref;
        fill_msg(rec, rec.m);
        rec.slot = true;
      } else if ((c.kind >= ZBHIP_CMD_MSG_SUB_CREATE && c.kind <= ZBHIP_CMD_MSG_SUB_CORRELATE) ||
                 c.kind == ZBHIP_CMD_MSG_SUB_DELETE || c.kind == ZBHIP_CMD_PMS_DELETE) {
        const zbhip_xpart_cmd& x = xdocs[x_base + c.doc_begin];
        rec.doc = Doc{0, 0};
        rec.r.aux = -1;
        rec.r.key = -1;
        MsgVal m;
        m.eik = x.element_instance_key;
        m.pik = x.process_instance_key;
        m.msg_key = x.message_key;
        m.corr = x.correlation_key;
        m.name = x.message_name;
        m.bpmn = x.bpmn_process_id;
        m.interrupting = x.interrupting;
        m.inst = x.instance;
        m.eord = x.element_ord;
        int vt, it;
        xpart_kind(c.kind, vt, it);
        rec.r.value_type = (uint8_t)vt;
        rec.r.intent = (uint8_t)it;
        rec.m = command_value(c.kind, m, x.source_partition);
        fill_msg(rec, rec.m);
        rec.slot = c.kind == ZBHIP_CMD_MSG_SUB_CREATE || c.kind == ZBHIP_CMD_MSG_SUB_CORRELATE ||
                   c.kind == ZBHIP_CMD_MSG_SUB_DELETE;
      } else if (c.kind == ZBHIP_CMD_TIMER_TRIGGER) {
        rec.doc = Doc{0, 0};
        rec.r.aux = (int64_t)((uint64_t)c.doc_begin | ((uint64_t)c.pad << 32));  // the command's dueDate
        rec.r.value_type = ZBHIP_VT_TIMER;
        rec.r.intent = ZBHIP_TIMER_TRIGGER;
        rec.r.key = -1;
        rec.job_ord = (int32_t)c.ref;
      } else {
        rec.r.value_type = ZBHIP_VT_JOB;
        rec.r.intent = ZBHIP_JOB_COMPLETE;
        rec.r.key = -1;  // resolved when processed: the job may be created earlier in this window
        rec.job_ord = (int32_t)c.ref;
      }
      rec.r.source_index = next_source_++;
      log_.push_back(std::move(rec));
    }
  }

  // StreamProcessor / ProcessingStateMachine: read the log and process each command as a batch.
  int run() {
    int processed = 0;
    while (!log_.empty()) {
      ORecord cmd = std::move(log_.front());
      log_.pop_front();
      try {
        batch_processing(cmd);
      } catch (const Unsupported& u) {
        last_error = "unsupported at source " + std::to_string(cmd.r.source_index) + ": " + u.what;
        fallback_.push_back(cmd.instance);
        return ZBHIP_EUNSUPP;
      }
      ++processed;
    }
    return processed;
  }

  std::vector<ORecord> out;  // every follow-up record, in log order
  std::vector<uint32_t> fallback_;

  // key ordinal lookup: per instance slot, every key generated in its batches
  std::unordered_map<uint32_t, std::vector<int64_t>> inst_keys;
  std::unordered_map<uint32_t, std::vector<int64_t>> slot_keys;  // keys generated by correlation slots

  int64_t resolve(uint32_t inst, uint32_t ord) {
    auto it = inst_keys.find(inst);
    if (it == inst_keys.end() || ord >= it->second.size()) return -1;
    return it->second[ord];
  }

  std::string dump_state() const;

  // ---- one command at a time (tests/psm.py restates ProcessingStateMachine around this) ----------
  // Engine.process (Engine.java:99-131) for exactly one command: its records are appended to `out`
  // (ordinals from first_ordinal, source index `source`) and nothing else runs -- the caller's batch
  // FIFO feeds the follow-up commands back.  The command comes as a record: value type, intent, key
  // (JOB:COMPLETE: the job key; TIMER:TRIGGER: the timer key, dueDate in aux; PROCESS_INSTANCE
  // commands: the element instance key or -1), process / element indices, flowScopeKey (scope_key),
  // processInstanceKey; `instance` is its subject slot (key bookkeeping), `d` its variable document.
  int process_one(const zbhip_record& r, uint32_t instance, const zbhip_doc_entry* d, size_t nd, int64_t source,
                  int first_ordinal) {
    ORecord rec{};
    rec.r = r;
    rec.r.record_type = ZBHIP_RT_COMMAND;
    rec.r.unprocessed = 0;
    rec.instance = instance;
    rec.job_ord = -1;
    const uint32_t base = (uint32_t)docs.size();
    docs.insert(docs.end(), d, d + nd);
    rec.doc = Doc{base, (uint32_t)nd};
    rec.r.aux = r.value_type == ZBHIP_VT_TIMER ? r.aux : nd ? (int64_t)base : -1;
    rec.pi.proc = r.process_idx;
    rec.pi.elem = r.element_idx;
    rec.pi.flowScopeKey = r.scope_key;
    rec.pi.piKey = r.process_instance_key;
    const bool msg = (r.value_type == ZBHIP_VT_MESSAGE && (r.intent == ZBHIP_MSG_PUBLISH || r.intent == ZBHIP_MSG_EXPIRE)) ||
                     (r.value_type == ZBHIP_VT_MESSAGE_SUBSCRIPTION &&
                      (r.intent == ZBHIP_MS_CREATE || r.intent == ZBHIP_MS_CORRELATE || r.intent == ZBHIP_MS_DELETE)) ||
                     (r.value_type == ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION &&
                      (r.intent == ZBHIP_PMS_CREATE || r.intent == ZBHIP_PMS_CORRELATE || r.intent == ZBHIP_PMS_DELETE));
    const bool known = (r.value_type == ZBHIP_VT_PROCESS_INSTANCE_CREATION && r.intent == ZBHIP_PIC_CREATE) ||
                       (r.value_type == ZBHIP_VT_JOB && (r.intent == ZBHIP_JOB_COMPLETE || r.intent == ZBHIP_JOB_TIME_OUT ||
                                                          r.intent == ZBHIP_JOB_FAIL || r.intent == ZBHIP_JOB_THROW_ERROR)) ||
                       (r.value_type == ZBHIP_VT_TIMER && r.intent == ZBHIP_TIMER_TRIGGER) ||
                       (r.value_type == ZBHIP_VT_PROCESS_INSTANCE && r.intent >= ZBHIP_PI_ACTIVATE_ELEMENT) ||
                       (r.value_type == ZBHIP_VT_PROCESS_INSTANCE_BATCH &&
                        (r.intent == ZBHIP_PIB_ACTIVATE || r.intent == ZBHIP_PIB_TERMINATE)) || msg;
    if (!known) { last_error = "process_one: command outside the restated subset"; return ZBHIP_EUNSUPP; }
    if (msg) {
      // the command's record value as the log holds it (MessageRecord / MessageSubscriptionRecord /
      // ProcessMessageSubscriptionRecord): the subject is the correlation slot `instance` for MESSAGE
      // and MESSAGE_SUBSCRIPTION commands, the process instance slot for PROCESS_MESSAGE_SUBSCRIPTION
      MsgVal m;
      m.eik = r.scope_key;
      m.pik = r.process_instance_key;
      m.msg_key = r.message_key;
      m.corr = r.correlation_key;
      m.name = r.message_name;
      m.bpmn = r.bpmn_process_id;
      m.partition = r.partition;
      m.interrupting = r.interrupting;
      m.inst = instance;
      if (r.value_type == ZBHIP_VT_MESSAGE) {
        // a PUBLISH carries timeToLive in aux, the command's timestamp in scope_key and the messageId's
        // string id in process_instance_key (-1: none); an EXPIRE its message key as the key
        m.ttl = r.aux;
        m.timestamp = r.scope_key;
        m.message_id = r.process_instance_key < 0 ? ZBHIP_NO_STRING : (uint32_t)r.process_instance_key;
        m.eik = m.pik = -1;
      }
      rec.doc = Doc{0, 0};
      rec.r.aux = -1;
      fill_msg(rec, m);
      rec.slot = r.value_type != ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION;
    }
    if (r.value_type == ZBHIP_VT_PROCESS_INSTANCE || r.value_type == ZBHIP_VT_PROCESS_INSTANCE_CREATION)
      if (r.process_idx < 0 || r.process_idx >= (int)procs.size() ||
          (r.value_type == ZBHIP_VT_PROCESS_INSTANCE &&
           (r.element_idx < 0 || r.element_idx >= (int)procs[r.process_idx].els.size()))) {
        last_error = "process_one: unknown process or element";
        return ZBHIP_EINVAL;
      }
    std::vector<ORecord> batch;
    batch_ = &batch;
    cur_instance_ = instance;
    cur_slot_ = rec.slot;
    cur_source_ = source;
    try {
      process(rec);
    } catch (const Unsupported& u) {
      batch_ = nullptr;
      last_error = "unsupported: " + u.what;
      return ZBHIP_EUNSUPP;
    }
    ++commands_processed;
    batch_ = nullptr;
    for (auto& x : batch) {
      x.r.ordinal = (uint16_t)(x.r.ordinal + first_ordinal);
      out.push_back(std::move(x));
    }
    return (int)batch.size();
  }

  // The zb-db rows of a hand-off (the device's zbhip_export_instances text, the dump_state format) into
  // this engine's column families: what the host adapter's RawDbWriter puts into RocksDB before the
  // CPU engine processes the instance's commands (fallback hand-off).  Returns the
  // number of rows read, or < 0 (last_error) for a row outside the restated families.
  int import_rows(const std::string& text) {
    std::vector<std::vector<std::string>> rows;
    size_t a = 0;
    while (a < text.size()) {
      size_t b = text.find('\n', a);
      if (b == std::string::npos) b = text.size();
      if (b > a) {
        std::vector<std::string> parts;
        size_t s = a;
        for (size_t i = a; i <= b; ++i)
          if (i == b || text[i] == '|') { parts.push_back(text.substr(s, i - s)); s = i + 1; }
        rows.push_back(std::move(parts));
      }
      a = b + 1;
    }
    auto fields = [](const std::string& f) {
      std::map<std::string, std::string> m;
      size_t s = 0;
      while (s <= f.size()) {
        size_t e = f.find(',', s);
        if (e == std::string::npos) e = f.size();
        const std::string kv = f.substr(s, e - s);
        const size_t q = kv.find('=');
        if (q != std::string::npos) m[kv.substr(0, q)] = kv.substr(q + 1);
        s = e + 1;
      }
      return m;
    };
    auto L = [](const std::string& v) { return (int64_t)std::stoll(v); };
    // (by id and, where given, element type -- -2: a job worker: a multi-instance body and its inner
    // activity share the id)
    auto find_proc = [this](int64_t def_key, const std::string& elem_id, int& proc, int& elem, int type = -1) {
      for (size_t p = 0; p < procs.size(); ++p) {
        if (procs[p].def_key != def_key) continue;
        for (size_t e = 0; e < procs[p].els.size(); ++e)
          if (procs[p].els[e].id == elem_id &&
              (type == -1 || procs[p].els[e].type == type || (type == -2 && ZBHIP_IS_JOB_WORKER(procs[p].els[e].type)))) {
            proc = (int)p;
            elem = (int)e;
            return true;
          }
      }
      return false;
    };
    int n = 0;
    try {
      // element instances first (the other families find their process through them), job states
      // last (after their JOBS rows)
      for (int pass = 0; pass < 3; ++pass)
        for (auto& r : rows) {
          const std::string& cf = r[0];
          const bool first = cf == "ELEMENT_INSTANCE_KEY";
          if ((first ? 0 : cf == "JOB_STATES" ? 2 : 1) != pass) continue;
          ++n;
          if (cf == "KEY" || cf == "TIMER_DUE_DATES" || cf == "JOB_ACTIVATABLE" || cf == "JOB_DEADLINES" ||
              cf == "JOB_BACKOFF")
            continue;
          if (first) {
            auto f = fields(r.at(2));
            ElementInstance ei;
            ei.key = L(r.at(1));
            ei.parentKey = L(f.at("parentKey"));
            ei.childCount = (int)L(f.at("childCount"));
            ei.jobKey = L(f.at("jobKey"));
            ei.state = (int)L(f.at("state"));
            ei.activeSequenceFlows = (int)L(f.at("activeSequenceFlows"));
            ei.childActivated = (int)L(f.at("childActivatedCount"));
            ei.childCompleted = (int)L(f.at("childCompletedCount"));
            ei.loopCounter = (int)L(f.at("multiInstanceLoopCounter"));
            ei.childTerminated = (int)L(f.at("childTerminatedCount"));
            ei.value.flowScopeKey = L(f.at("flowScopeKey"));
            ei.value.piKey = L(f.at("processInstanceKey"));
            if (!find_proc(L(f.at("processDefinitionKey")), f.at("elementId"), ei.value.proc, ei.value.elem,
                           (int)L(f.at("bpmnElementType"))))
              throw Unsupported{"element " + f.at("elementId")};
            ei_[ei.key] = ei;
          } else if (cf == "ELEMENT_INSTANCE_PARENT_CHILD") {
            parent_child_.insert({L(r.at(1)), L(r.at(2))});
          } else if (cf == "ELEMENT_INSTANCE_CHILD_PARENT") {
            child_parent_[L(r.at(1))] = L(r.at(2));
          } else if (cf == "NUMBER_OF_TAKEN_SEQUENCE_FLOWS") {
            const int64_t scope = L(r.at(1));
            const OProc& pr = procs[ei_.at(scope).value.proc];
            int gw = -1, fl = -1;
            for (size_t e = 0; e < pr.els.size(); ++e) {
              if (pr.els[e].id == r.at(2)) gw = (int)e;
              if (pr.els[e].id == r.at(3)) fl = (int)e;
            }
            if (gw < 0 || fl < 0) throw Unsupported{"taken flow " + r.at(2) + "/" + r.at(3)};
            taken_[{scope, gw, fl}] = (int)L(r.at(4));
          } else if (cf == "PROCESS_INSTANCE_KEY_BY_DEFINITION_KEY") {
            pi_by_def_.insert({L(r.at(1)), L(r.at(2))});
          } else if (cf == "VARIABLES") {
            auto f = fields(r.at(3));
            const uint8_t type = (uint8_t)L(f.at("type"));
            const int64_t value = type == ZBHIP_DOC_LIST ? intern_list(parse_list_text(f.at("value"))) : L(f.at("value"));
            vars_[{L(r.at(1)), intern(r.at(2))}] = VarRow{L(f.at("key")), type, value, 0};
          } else if (cf == "EVENT_SCOPE") {
            auto f = fields(r.at(2));
            const int64_t k = L(r.at(1));
            event_scope_.insert(k);
            if (f.at("accepting") == "0") es_closed_.insert(k);
            if (f.at("interrupted") == "1") es_interrupted_.insert(k);
          } else if (cf == "TIMERS") {
            auto f = fields(r.at(3));
            TimerRow t;
            const int64_t eik = L(r.at(1));
            if (!find_proc(L(f.at("processDefinitionKey")), f.at("handlerNodeId"), t.pi.proc, t.pi.elem))
              throw Unsupported{"timer handler " + f.at("handlerNodeId")};
            t.pi.piKey = L(f.at("processInstanceKey"));
            auto eit = ei_.find(eik);
            if (eit != ei_.end()) t.pi.flowScopeKey = eit->second.value.flowScopeKey;
            t.dueDate = L(f.at("dueDate"));
            t.reps = (int)L(f.at("repetitions"));
            timers_[{eik, L(r.at(2))}] = t;
          } else if (cf == "JOBS") {
            auto f = fields(r.at(2));
            JobRow j;
            if (!find_proc(L(f.at("processDefinitionKey")), f.at("elementId"), j.pi.proc, j.pi.elem, -2))
              throw Unsupported{"job element " + f.at("elementId")};
            j.pi.piKey = L(f.at("processInstanceKey"));
            j.elementInstanceKey = L(f.at("elementInstanceKey"));
            auto eit = ei_.find(j.elementInstanceKey);
            if (eit != ei_.end()) j.pi.flowScopeKey = eit->second.value.flowScopeKey;
            j.type = f.at("type");
            j.retries = (int)L(f.at("retries"));
            j.deadline = L(f.at("deadline"));
            j.worker = f.at("worker");
            if (f.count("errorMessageHex")) {  // a failed job's stored fields
              j.fail_fields = true;
              j.error_message = unhex(f.at("errorMessageHex"));
              j.retry_backoff = L(f.at("retryBackoff"));
              j.recurring_time = L(f.at("recurringTime"));
            } else if (j.retries != procs[j.pi.proc].els[j.pi.elem].retries) {
              // a failure that left errorMessage, retryBackoff and recurringTime at their defaults (a state
              // read back from zb-db rows, where they do not show): its retries alone
              j.fail_fields = true;
              j.recurring_time = -1;
            }
            jobs_[L(r.at(1))] = j;
          } else if (cf == "JOB_STATES") {
            const int64_t k = L(r.at(1));
            JobRow& j = jobs_.at(k);
            j.activated = r.at(2) == "ACTIVATED";
            j.failed = r.at(2) == "FAILED";
            if (!j.activated && !j.failed) activatable_.insert({j.type, "<default>", k});
          } else if (cf == "INCIDENTS") {
            auto f = fields(r.at(2));
            IncidentRow in;
            if (!find_proc(L(f.at("processDefinitionKey")), f.at("elementId"), in.pi.proc, in.pi.elem))
              throw Unsupported{"incident element " + f.at("elementId")};
            in.pi.piKey = L(f.at("processInstanceKey"));
            in.eik = L(f.at("elementInstanceKey"));
            in.error_type = (int)L(f.at("errorType"));
            in.flow = (int)L(f.at("flow"));
            in.result = (int)L(f.at("result"));
            if (f.count("jobKey")) {
              in.job_key = L(f.at("jobKey"));
              in.message = unhex(f.at("messageHex"));
            }
            incidents_[L(r.at(1))] = in;
          } else if (cf == "INCIDENT_PROCESS_INSTANCES") {
            incident_pi_[L(r.at(1))] = L(r.at(2));
          } else if (cf == "INCIDENT_JOBS") {
            incident_jobs_[L(r.at(1))] = L(r.at(2));
          } else if (cf == "PROCESS_SUBSCRIPTION_BY_KEY") {
            // a handed-off instance's process message subscription [elementInstanceKey, messageName]
            auto f = fields(r.at(3));
            MsgVal m;
            m.eik = L(r.at(1));
            m.name = (uint16_t)intern(r.at(2));
            m.pik = L(f.at("processInstanceKey"));
            m.partition = (int32_t)L(f.at("subscriptionPartitionId"));
            m.bpmn = (uint16_t)intern(f.at("bpmnProcessId"));
            m.msg_key = L(f.at("messageKey"));
            m.corr = (uint32_t)intern_string(f.at("correlationKey"));
            m.interrupting = (uint8_t)L(f.at("interrupting"));
            const ElementInstance& owner = ei_.at(m.eik);
            if (!find_proc(procs[owner.value.proc].def_key, f.at("elementId"), m.proc, m.elem))
              throw Unsupported{"subscription element " + f.at("elementId")};
            m.inst = 0xFFFFFFFFu;  // (no instance slot of this engine's: routing handles are the device's)
            PmsRow row{L(f.at("key")), f.at("state") == "OPENED", m};
            row.closing = f.at("state") == "CLOSING";
            pms_[{m.eik, (int)m.name}] = row;
            ++pms_inst_[m.inst];
          } else if (cf == "MESSAGE_SUBSCRIPTION_BY_KEY") {
            // a message partition's subscriptions moved from the device (its correlation key's message
            // state goes to the engine): [elementInstanceKey, messageName] -> MessageSubscription
            auto f = fields(r.at(3));
            MsgVal m;
            m.eik = L(r.at(1));
            m.name = (uint16_t)intern(r.at(2));
            m.pik = L(f.at("processInstanceKey"));
            m.bpmn = (uint16_t)intern(f.at("bpmnProcessId"));
            m.msg_key = L(f.at("messageKey"));
            m.corr = (uint32_t)intern_string(f.at("correlationKey"));
            m.interrupting = (uint8_t)L(f.at("interrupting"));
            msub_[{m.eik, (int)m.name}] = MsgSub{L(f.at("key")), f.at("correlating") == "1", m};
            msub_by_corr_.insert({(int)m.name, m.corr, m.eik});
          } else if (cf == "MESSAGE_SUBSCRIPTION_BY_NAME_AND_CORRELATION_KEY") {
            continue;  // (the index of the BY_KEY rows)
          } else {
            throw Unsupported{"column family " + cf};
          }
        }
    } catch (const Unsupported& u) {
      last_error = "import: " + u.what;
      return ZBHIP_EUNSUPP;
    } catch (const std::exception& e) {
      last_error = std::string("import: malformed row (") + e.what() + ")";
      return ZBHIP_EINVAL;
    }
    return n;
  }
  // JOB_BATCH:ACTIVATE (processing/job/JobBatchActivateProcessor.java:60-143, JobBatchCollector.java
  // :67-123): jobs of `type` in JOB_ACTIVATABLE order ([[type, jobKey], tenant]), deadline, worker,
  // variables (JobVariablesCollector -> DbVariableState.getVariablesAsDocument :193-247: the element
  // scope, then its flow scope; names in DbString key order (length, bytes), each once), then
  // JobBatchActivatedApplier -> DbJobState.activate.  Returns the rejection reason (0 accepted).
  struct Activated {
    int64_t key, eik, pik, deadline;
    int proc, elem, retries;
    std::vector<std::pair<int, VarRow>> vars;  // (name id, row)
  };
  int activate_jobs(const std::string& type, const std::string& worker, int64_t timeout, int max_jobs,
                    int64_t timestamp, const std::vector<std::string>& requested, std::vector<Activated>& out,
                    int64_t& batch_key) {
    out.clear();
    batch_key = -1;
    if (max_jobs < 1) return 1;
    if (timeout < 1) return 2;
    if (type.empty()) return 3;
    if (!worker.empty()) intern_string(worker);  // (the value dictionary: JOB records name it)
    batch_key = ((int64_t)partition_ << 51) + ++key_counter_;  // keyGenerator.nextKey, no instance's
    std::vector<int64_t> keys;
    for (auto it = activatable_.lower_bound({type, "<default>", INT64_MIN});
         it != activatable_.end() && std::get<0>(*it) == type && std::get<1>(*it) == "<default>" &&
         (int)keys.size() < max_jobs;
         ++it)
      keys.push_back(std::get<2>(*it));
    for (int64_t k : keys) {
      JobRow& j = jobs_.at(k);
      Activated a;
      a.key = k;
      a.eik = j.elementInstanceKey;
      a.pik = j.pi.piKey;
      a.deadline = timestamp + timeout;
      a.proc = j.pi.proc;
      a.elem = j.pi.elem;
      a.retries = j.retries;
      collect_variables(j, requested, a);
      j.activated = true;
      j.deadline = a.deadline;
      j.worker = worker;
      activatable_.erase({j.type, "<default>", k});
      out.push_back(std::move(a));
    }
    return 0;
  }

  // JobVariablesCollector.setJobVariables: the element scope, then every scope above it (a multi-instance
  // inner activity: its loop variables, the body, the process instance); names in DbString key order
  // (4-byte big-endian length, then the bytes), each once, `requested` only if any
  void collect_variables(const JobRow& j, const std::vector<std::string>& requested, Activated& a) {
    auto name_less = [this](int x_, int y_) {
      const std::string& x = names[x_];
      const std::string& y = names[y_];
      return x.size() != y.size() ? x.size() < y.size() : x < y;
    };
    std::vector<int64_t> scopes{j.elementInstanceKey};
    for (auto pit = child_parent_.find(j.elementInstanceKey); pit != child_parent_.end() && pit->second > 0;
         pit = child_parent_.find(pit->second))
      scopes.push_back(pit->second);
    std::set<int> seen;
    for (int64_t scope : scopes) {
      std::vector<int> local;
      for (auto& [sk, row] : vars_)
        if (sk.first == scope) local.push_back(sk.second);
      std::sort(local.begin(), local.end(), name_less);
      for (int nid : local) {
        if (seen.count(nid)) continue;
        if (!requested.empty() && std::find(requested.begin(), requested.end(), names[nid]) == requested.end()) continue;
        seen.insert(nid);
        a.vars.push_back({nid, vars_.at({scope, nid})});
      }
    }
  }
  // the push side effect's ActivatedJob (BpmnJobActivationBehavior.publishWork :83-97): the job as stored
  // now, with the stream's fetchVariables; false for no such job
  bool job_variables(int64_t key, const std::vector<std::string>& requested, Activated& a) {
    auto it = jobs_.find(key);
    if (it == jobs_.end()) return false;
    const JobRow& j = it->second;
    a = Activated{};
    a.key = key;
    a.eik = j.elementInstanceKey;
    a.pik = j.pi.piKey;
    a.deadline = j.activated ? j.deadline : -1;
    a.proc = j.pi.proc;
    a.elem = j.pi.elem;
    a.retries = j.retries;
    collect_variables(j, requested, a);
    return true;
  }

  // DbKeyGenerator's current value (the CPU engine of a fallback hand-off is set to the device's)
  int64_t key_counter() const { return key_counter_; }
  void set_key_counter(int64_t v) { key_counter_ = v; }
  uint64_t transitions = 0, completed_instances = 0, commands_processed = 0;

 private:
  int partition_, partition_count_, max_cmds_;
  int64_t key_counter_ = 0;
  int64_t next_source_ = 0;
  std::deque<ORecord> log_;

  // --- state (zb-db column families) ---
  std::map<int64_t, ElementInstance> ei_;                       // ELEMENT_INSTANCE_KEY
  std::set<std::pair<int64_t, int64_t>> parent_child_;          // ELEMENT_INSTANCE_PARENT_CHILD
  std::map<int64_t, int64_t> child_parent_;                     // ELEMENT_INSTANCE_CHILD_PARENT
  std::map<std::tuple<int64_t, int, int>, int> taken_;          // NUMBER_OF_TAKEN_SEQUENCE_FLOWS (proc-local ids)
  std::set<std::pair<int64_t, int64_t>> pi_by_def_;             // PROCESS_INSTANCE_KEY_BY_DEFINITION_KEY
  std::map<std::pair<int64_t, int>, VarRow> vars_;              // VARIABLES (scope, name id)
  std::set<int64_t> event_scope_;                               // EVENT_SCOPE
  std::set<int64_t> es_interrupted_, es_closed_;                // EventScopeInstance.interrupted / !accepting
  std::map<std::pair<int64_t, int64_t>, EventTrigger> triggers_;// EVENT_TRIGGER
  struct TimerRow {  // TimerInstance (state/instance/TimerInstance.java:23-44)
    PiValue pi;      // process, handler element, process instance key
    int64_t dueDate = 0;
    int reps = 1;    // repetitions (-1 infinite)
  };
  std::map<std::pair<int64_t, int64_t>, TimerRow> timers_;     // TIMERS [elementInstanceKey, timerKey]
 public:
  int64_t now_ms = 0;  // ActorClock.currentTimeMillis() of the window's processing (zbo_set_clock)
  std::map<std::string, std::pair<std::string, int64_t>> streams;  // job streams: type -> (worker, timeout)
 private:
  std::map<int64_t, JobRow> jobs_;                              // JOBS (+ JOB_STATES = ACTIVATABLE)
  struct IncidentRow {  // IncidentRecord (protocol-impl/.../incident/IncidentRecord.java:20-48)
    PiValue pi;         // process, element, process instance key
    int64_t eik = -1;   // elementInstanceKey (= variableScopeKey unless variable_scope says otherwise)
    int64_t variable_scope = -1;
    int error_type = 0, flow = -1, result = 0;  // the message: zbhip_incident_message
    int64_t job_key = -1;       // a job's incident (JOB_NO_RETRIES): INCIDENT_JOBS, its errorMessage
    std::string message;
    bool no_catch = false;      // UNHANDLED_ERROR_EVENT: elementId NO_CATCH_EVENT_FOUND (the job's record)
  };
  std::map<int64_t, int64_t> incident_jobs_;                    // INCIDENT_JOBS [jobKey -> incident]
  std::map<int64_t, IncidentRow> incidents_;                    // INCIDENTS
  std::map<int64_t, int64_t> incident_pi_;                      // INCIDENT_PROCESS_INSTANCES [eik -> incident]
  std::set<std::tuple<std::string, std::string, int64_t>> activatable_;  // JOB_ACTIVATABLE

  // --- message state (ZbColumnFamilies PROCESS_SUBSCRIPTION_BY_KEY, MESSAGE_SUBSCRIPTION_BY_KEY,
  // MESSAGE_SUBSCRIPTION_BY_NAME_AND_CORRELATION_KEY, MESSAGE_STATS) ---
  struct PmsRow { int64_t key; bool opened; MsgVal rec; bool closing = false; };
  struct MsgSub { int64_t key; bool correlating; MsgVal rec; };
  std::map<std::pair<int64_t, int>, PmsRow> pms_;                        // [eik, name]
  std::unordered_map<uint32_t, int> pms_inst_;                           // open subscriptions per instance slot
  std::map<std::pair<int64_t, int>, MsgSub> msub_;                       // [eik, name]
  std::set<std::tuple<int, uint32_t, int64_t>> msub_by_corr_;           // [name, corr, eik]
  bool msg_stats_ = false;                                               // messagesDeadlineCount row
  // buffered messages (DbMessageState.java:133-213): MESSAGE_KEY, MESSAGES [[tenant, name, correlationKey],
  // key], MESSAGE_DEADLINES [deadline, key], MESSAGE_IDS [[tenant, name, correlationKey], messageId],
  // MESSAGE_CORRELATED [key, bpmnProcessId] and the messagesDeadlineCount of MESSAGE_STATS
  struct StoredMessage { uint16_t name; uint32_t corr; int64_t ttl, deadline; uint32_t message_id; };
  std::map<int64_t, StoredMessage> messages_;
  std::set<std::tuple<int, uint32_t, int64_t>> msg_by_corr_;
  std::set<std::pair<int64_t, int64_t>> msg_deadlines_;
  std::set<std::tuple<int, uint32_t, uint32_t>> msg_ids_;
  std::set<std::pair<int64_t, int>> msg_correlated_;
  int64_t msg_deadline_count_ = 0;
  // message start events (DbMessageStartEventSubscriptionState: MESSAGE_START_EVENT_SUBSCRIPTION_BY_NAME_AND_KEY
  // [[tenant, messageName], processDefinitionKey]) and the process-correlation-key locks of DbMessageState
  // (MESSAGE_PROCESSES_ACTIVE_BY_CORRELATION_KEY [[bpmnProcessId, correlationKey]],
  // MESSAGE_PROCESS_INSTANCE_CORRELATION_KEYS [processInstanceKey -> correlationKey])
  struct MsgStartSub { int proc; int elem; int64_t key; };
  std::map<std::pair<int, int64_t>, MsgStartSub> msg_start_subs_;
  std::set<std::pair<int, uint32_t>> active_by_corr_;
  std::map<int64_t, uint32_t> pi_corr_keys_;

  // --- batch context ---
  std::vector<ORecord>* batch_ = nullptr;
  uint32_t cur_instance_ = 0;
  bool cur_slot_ = false;   // keys of the batch so far belong to the correlation slot cur_instance_
  int64_t cur_source_ = 0;

  // DbKeyGenerator.nextKey (stream-platform/.../state/DbKeyGenerator.java:39-42) with
  // Protocol.encodePartitionId (protocol/.../Protocol.java:98-100)
  int64_t next_key() {
    ++key_counter_;
    int64_t k = ((int64_t)partition_ << 51) + key_counter_;
    (cur_slot_ ? slot_keys : inst_keys)[cur_instance_].push_back(k);
    return k;
  }
  // key ordinal of `key` within the instance slot `inst` (routing handle of the xpart commands)
  uint16_t ord_of(uint32_t inst, int64_t key) {
    auto& v = inst_keys[inst];
    for (size_t i = v.size(); i-- > 0;)
      if (v[i] == key) return (uint16_t)i;
    throw Unsupported{"routing handle of an unknown key"};
  }
  // switches the batch to the subject instance `inst` (a PI command inside a message batch)
  void enter_instance(uint32_t inst) {
    cur_slot_ = false;
    cur_instance_ = inst;
  }

  const OProc& P(int proc) const { return procs[proc]; }
  const OEl& E(const PiValue& v) const { return procs[v.proc].els[v.elem]; }

  ORecord& append(int rt, int vt, int intent, int64_t key) {
    ORecord rec{};
    std::memset(&rec.r, 0, sizeof(rec.r));
    rec.r.record_type = (uint8_t)rt;
    rec.r.value_type = (uint8_t)vt;
    rec.r.intent = (uint8_t)intent;
    rec.r.key = key;
    rec.r.rejection_type = ZBHIP_REJ_NONE;
    rec.r.source_index = cur_source_;
    rec.r.ordinal = (uint16_t)batch_->size();
    rec.r.aux = -1;
    rec.r.process_idx = -1;
    rec.r.element_idx = -1;
    rec.r.scope_key = -1;
    rec.r.process_instance_key = -1;
    rec.r.message_key = -1;
    rec.r.correlation_key = ZBHIP_NO_STRING;
    rec.r.message_name = 0xFFFF;
    rec.r.bpmn_process_id = 0xFFFF;
    rec.instance = cur_instance_;
    rec.slot = cur_slot_;
    batch_->push_back(std::move(rec));
    return batch_->back();
  }

  void fill_pi(ORecord& rec, const PiValue& v) {
    rec.pi = v;
    rec.r.process_idx = v.proc;
    rec.r.element_idx = v.elem;
    rec.r.scope_key = v.flowScopeKey;
    rec.r.process_instance_key = v.piKey;
  }

  // ResultBuilderBackedEventApplyingStateWriter.appendFollowUpEvent
  // (processing/streamprocessor/writers/ResultBuilderBackedEventApplyingStateWriter.java:45-57):
  // append the record, then apply it immediately.
  void pi_event(int64_t key, int intent, const PiValue& v) {
    ORecord& rec = append(ZBHIP_RT_EVENT, ZBHIP_VT_PROCESS_INSTANCE, intent, key);
    fill_pi(rec, v);
    ++transitions;
    if (intent == ZBHIP_PI_ELEMENT_COMPLETED && P(v.proc).els[v.elem].type == ZBHIP_EL_PROCESS)
      ++completed_instances;
    apply_pi(key, intent, v);
  }

  // ResultBuilderBackedTypedCommandWriter.appendFollowUpCommand
  void pi_command(int64_t key, int intent, const PiValue& v) {
    ORecord& rec = append(ZBHIP_RT_COMMAND, ZBHIP_VT_PROCESS_INSTANCE, intent, key);
    fill_pi(rec, v);
  }

  // TypedRejectionWriter.appendRejection: key and value of the command
  void reject(const ORecord& cmd, int type, const std::string& reason) {
    ORecord& rec = append(ZBHIP_RT_REJECTION, cmd.r.value_type, cmd.r.intent, cmd.r.key);
    rec.r.rejection_type = (uint8_t)type;
    rec.r.process_idx = cmd.r.process_idx;
    rec.r.element_idx = cmd.r.element_idx;
    rec.r.scope_key = cmd.r.scope_key;
    rec.r.process_instance_key = cmd.r.process_instance_key;
    rec.r.aux = cmd.r.aux;
    rec.r.message_key = cmd.r.message_key;
    rec.r.correlation_key = cmd.r.correlation_key;
    rec.r.message_name = cmd.r.message_name;
    rec.r.bpmn_process_id = cmd.r.bpmn_process_id;
    rec.r.partition = cmd.r.partition;
    rec.r.interrupting = cmd.r.interrupting;
    rec.m = cmd.m;
    rec.pi = cmd.pi;
    rec.doc = cmd.doc;
    rec.reason = reason;
  }

  // ---------------------------------------------------------------------
  // ProcessingStateMachine.batchProcessing / collectBatchProcessingStepResult
  // (stream-platform/.../stream/impl/ProcessingStateMachine.java:328-417)
  // ---------------------------------------------------------------------
  void batch_processing(ORecord& initial) {
    std::vector<ORecord> batch;
    batch_ = &batch;
    cur_instance_ = initial.instance;
    cur_slot_ = initial.slot;
    cur_source_ = initial.r.source_index;
    std::deque<ORecord> pending;
    pending.push_back(initial);
    int processed = 0;
    size_t last_size = 0;
    while (!pending.empty() && processed < max_cmds_) {
      ORecord cmd = std::move(pending.front());
      pending.pop_front();
      process(cmd);
      ++commands_processed;
      int current_batch_size = (int)pending.size() + processed + 1;
      int to_process = 0;
      for (size_t i = last_size; i < batch.size(); ++i) {
        if (batch[i].r.record_type == ZBHIP_RT_COMMAND) {
          if (current_batch_size + to_process < max_cmds_) {
            pending.push_back(batch[i]);
            ++to_process;
          } else {
            // written to the log unprocessed: processed later as its own batch
            batch[i].r.unprocessed = 1;
            ORecord later = batch[i];
            later.r.unprocessed = 0;
            later.r.source_index = next_source_++;
            log_.push_back(later);
          }
        }
      }
      last_size = batch.size();
      ++processed;
    }
    for (auto& r : batch) out.push_back(std::move(r));
    batch_ = nullptr;
  }

  // Engine.process (Engine.java:99-131) -> RecordProcessorMap dispatch
  void process(ORecord& cmd) {
    if (cmd.r.value_type == ZBHIP_VT_PROCESS_INSTANCE_CREATION)
      create_process_instance(cmd);
    else if (cmd.r.value_type == ZBHIP_VT_JOB && cmd.r.intent == ZBHIP_JOB_TIME_OUT)
      time_out_job(cmd);
    else if (cmd.r.value_type == ZBHIP_VT_JOB && cmd.r.intent == ZBHIP_JOB_FAIL)
      fail_job(cmd);
    else if (cmd.r.value_type == ZBHIP_VT_JOB && cmd.r.intent == ZBHIP_JOB_THROW_ERROR)
      throw_error(cmd);
    else if (cmd.r.value_type == ZBHIP_VT_JOB)
      complete_job(cmd);
    else if (cmd.r.value_type == ZBHIP_VT_TIMER && cmd.r.intent == ZBHIP_TIMER_TRIGGER)
      trigger_timer(cmd);
    else if (cmd.r.value_type == ZBHIP_VT_PROCESS_INSTANCE)
      bpmn_process_record(cmd);
    else if (cmd.r.value_type == ZBHIP_VT_PROCESS_INSTANCE_BATCH && cmd.r.intent == ZBHIP_PIB_TERMINATE)
      terminate_batch(cmd);
    else if (cmd.r.value_type == ZBHIP_VT_PROCESS_INSTANCE_BATCH && cmd.r.intent == ZBHIP_PIB_ACTIVATE)
      activate_batch(cmd);
    else if (cmd.r.value_type == ZBHIP_VT_MESSAGE && cmd.r.intent == ZBHIP_MSG_PUBLISH)
      publish_message(cmd);
    else if (cmd.r.value_type == ZBHIP_VT_MESSAGE && cmd.r.intent == ZBHIP_MSG_EXPIRE)
      expire_message(cmd);
    else if (cmd.r.value_type == ZBHIP_VT_MESSAGE_SUBSCRIPTION && cmd.r.intent == ZBHIP_MS_CREATE)
      message_subscription_create(cmd);
    else if (cmd.r.value_type == ZBHIP_VT_MESSAGE_SUBSCRIPTION && cmd.r.intent == ZBHIP_MS_CORRELATE)
      message_subscription_correlate(cmd);
    else if (cmd.r.value_type == ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION && cmd.r.intent == ZBHIP_PMS_CREATE)
      process_message_subscription_create(cmd);
    else if (cmd.r.value_type == ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION && cmd.r.intent == ZBHIP_PMS_CORRELATE)
      process_message_subscription_correlate(cmd);
    else if (cmd.r.value_type == ZBHIP_VT_MESSAGE_SUBSCRIPTION && cmd.r.intent == ZBHIP_MS_DELETE)
      message_subscription_delete(cmd);
    else if (cmd.r.value_type == ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION && cmd.r.intent == ZBHIP_PMS_DELETE)
      process_message_subscription_delete(cmd);
    else
      throw Unsupported{"value type"};
  }

  // =====================================================================
  // Message correlation
  // =====================================================================
  ORecord& msg_record(int rt, int vt, int intent, int64_t key, const MsgVal& m) {
    ORecord& r = append(rt, vt, intent, key);
    fill_msg(r, m);
    return r;
  }

  // SubscriptionCommandSender.handleFollowUpCommandBasedOnPartition (:304-320): the receiver's own
  // partition -> a follow-up command in this batch (key -1); another partition -> a post-commit side
  // effect (InterPartitionCommandSender.sendCommand), collected in the outbox in batch order.
  void send_command(int target, int kind, const MsgVal& in) {
    MsgVal v = command_value(kind, in, partition_);
    int vt, it;
    xpart_kind(kind, vt, it);
    if (target == partition_) {
      ORecord& r = msg_record(ZBHIP_RT_COMMAND, vt, it, -1, v);
      r.slot = false;
      return;
    }
    zbhip_xpart_cmd x{};
    x.element_instance_key = in.eik;
    x.process_instance_key = in.pik;
    x.message_key = v.msg_key;
    x.correlation_key = in.corr;  // routing: the correlation slot on the message partition
    x.instance = in.inst;
    x.element_ord = in.eord;
    x.message_name = in.name;
    x.bpmn_process_id = in.bpmn;
    x.kind = (uint8_t)kind;
    x.interrupting = in.interrupting;
    x.source_partition = (int16_t)partition_;
    x.target_partition = (int16_t)target;
    outbox.push_back(x);
  }

  static int partition_of_key(int64_t key) { return (int)(key >> 51); }  // Protocol.decodePartitionId

  // CatchEventBehavior.subscribeToEvents -> subscribeToMessageEvent (processing/common/CatchEventBehavior.java:111-125,248-283)
  // CatchEventBehavior.subscribeToTimerEvent (processing/common/CatchEventBehavior.java:303-330):
  // dueDate = now + duration, TIMER:CREATED (+key); TimerCreatedApplier stores the TimerInstance
  void subscribe_to_timer(const OEl& el, int64_t key, const PiValue& v) { subscribe_timer_at(key, v, now_ms + el.timer_ms, el.reps); }
  void subscribe_timer_at(int64_t key, const PiValue& v, int64_t due, int reps) {
    const int64_t tk = next_key();
    ORecord& rec = append(ZBHIP_RT_EVENT, ZBHIP_VT_TIMER, ZBHIP_TIMER_CREATED, tk);
    rec.r.process_idx = v.proc;
    rec.r.element_idx = v.elem;
    rec.r.scope_key = key;
    rec.r.process_instance_key = v.piKey;
    rec.r.aux = due;
    rec.r.partition = reps;  // TimerRecord.repetitions
    TimerRow t;
    t.pi = v;
    t.dueDate = due;
    t.reps = reps;
    timers_[{key, tk}] = t;
  }

  // TriggerTimerProcessor.processRecord (processing/timer/TriggerTimerProcessor.java:81-114) for a
  // timer of an intermediate catch event: TIMER:TRIGGERED (the command's key and value), then
  // EventHandle.activateElement (EventHandle.java:104-131): PROCESS_EVENT:TRIGGERING (+key, no
  // variables) and COMPLETE_ELEMENT for the catch event
  void trigger_timer(ORecord& cmd) {
    if (cmd.job_ord >= 0) cmd.r.key = resolve(cmd.instance, (uint32_t)cmd.job_ord);
    const int64_t tk = cmd.r.key;
    auto it = timers_.begin();
    for (; it != timers_.end(); ++it)
      if (it->first.second == tk) break;
    if (it == timers_.end()) {
      reject(cmd, ZBHIP_REJ_NOT_FOUND,
             "Expected to trigger timer with key '" + std::to_string(tk) + "', but no such timer was found");
      return;
    }
    const int64_t eik = it->first.first;
    const TimerRow t = it->second;
    auto eit = ei_.find(eik);
    if (eit == ei_.end() || eit->second.state != ZBHIP_PI_ELEMENT_ACTIVATED || !can_trigger(eik, t.pi.elem, t.pi.proc)) {
      reject(cmd, ZBHIP_REJ_INVALID_STATE,
             "Expected to trigger a timer with key '" + std::to_string(tk) + "', but the timer is not active anymore");
      return;
    }
    ORecord& rec = append(ZBHIP_RT_EVENT, ZBHIP_VT_TIMER, ZBHIP_TIMER_TRIGGERED, tk);
    rec.r.process_idx = t.pi.proc;
    rec.r.element_idx = t.pi.elem;
    rec.r.scope_key = eik;
    rec.r.process_instance_key = t.pi.piKey;
    rec.r.aux = t.dueDate;
    rec.r.partition = t.reps;
    timers_.erase(it);  // TimerTriggeredApplier
    const int64_t eventKey = next_key();
    ORecord& pe = append(ZBHIP_RT_EVENT, ZBHIP_VT_PROCESS_EVENT, ZBHIP_PE_TRIGGERING, eventKey);
    pe.r.process_idx = t.pi.proc;
    pe.r.element_idx = t.pi.elem;
    pe.r.scope_key = eik;
    pe.r.process_instance_key = t.pi.piKey;
    pe.r.aux = -1;
    trigger_event(eik, eventKey, t.pi.elem, t.pi.proc, Doc{0, 0}, t.pi.piKey);
    const OEl& target = E(t.pi);
    if (target.type == ZBHIP_EL_BOUNDARY_EVENT && target.interrupting)  // terminate the activity first
      pi_command(eik, ZBHIP_PI_TERMINATE_ELEMENT, eit->second.value);
    else if (target.type == ZBHIP_EL_BOUNDARY_EVENT)  // non-interrupting: activateTriggeredEvent now
      activate_triggered_event(eventKey, t.pi.elem, eik, eit->second.value.flowScopeKey, eit->second.value);
    else                                              // isElementActivated (catch event)
      pi_command(eik, ZBHIP_PI_COMPLETE_ELEMENT, eit->second.value);
    // shouldReschedule / rescheduleTimer (TriggerTimerProcessor.java:116-160): a cycle's next timer
    // from the last dueDate (refreshTimer: Interval.withStart(dueDate) starts at dueDate + interval),
    // one repetition fewer; subscribeToTimerEvent takes timer.getDueDate(now) = Interval.toEpochMilli
    // (Interval.java:77-93): that start, or now + interval when the start is not after now
    if (t.reps == -1 || t.reps > 1) {
      const int64_t start = t.dueDate + target.timer_ms;
      subscribe_timer_at(eik, t.pi, start <= now_ms ? now_ms + target.timer_ms : start, t.reps == -1 ? -1 : t.reps - 1);
    }
  }

  // DbEventScopeInstanceState.canTriggerEvent (state/instance/DbEventScopeInstanceState.java:178-182):
  // accepting, and not interrupted unless the element is one of the scope's boundary events
  bool can_trigger(int64_t scope, int elem, int proc) const {
    if (!event_scope_.count(scope) || es_closed_.count(scope)) return false;
    if (!es_interrupted_.count(scope)) return true;
    const OEl& e = procs[proc].els[elem];
    return e.type == ZBHIP_EL_BOUNDARY_EVENT;
  }

  // DbEventScopeInstanceState.triggerEvent (:100-124): an interrupting element id interrupts the
  // scope, an interrupting boundary event also closes it; then the EVENT_TRIGGER row
  void trigger_event(int64_t scope, int64_t eventKey, int elem, int proc, Doc vars, int64_t piKey) {
    if (!can_trigger(scope, elem, proc)) return;
    auto sit = ei_.find(scope);
    if (sit != ei_.end()) {
      const OEl& owner = procs[sit->second.value.proc].els[sit->second.value.elem];
      const bool attached = std::find(owner.boundaries.begin(), owner.boundaries.end(), elem) != owner.boundaries.end();
      const OEl& te = procs[proc].els[elem];
      const bool esp_start = te.type == ZBHIP_EL_START_EVENT && te.scope > 0 &&
                             std::find(owner.esps.begin(), owner.esps.end(), te.scope) != owner.esps.end();
      const bool interrupting = owner.id == te.id ? owner.type == ZBHIP_EL_INTERMEDIATE_CATCH_EVENT ||
                                                        owner.type == ZBHIP_EL_BOUNDARY_EVENT
                                                  : (attached || esp_start) && te.interrupting;
      if (interrupting) es_interrupted_.insert(scope);
      if (interrupting && attached) es_closed_.insert(scope);
      // EventSubProcessInterruptionMarker.markInstanceIfInterrupted (:36-63)
      if (esp_start && te.interrupting) sit->second.interrupting_elem = te.scope;
    }
    triggers_[{scope, eventKey}] = EventTrigger{elem, proc, vars, piKey};
  }

  // CatchEventBehavior.unsubscribeFromTimerEvents (processing/common/CatchEventBehavior.java:369-392):
  // TIMER:CANCELED (the timer's key and stored value) per timer of the element instance; TimerCancelledApplier
  void unsubscribe_timers(int64_t eik) {
    for (auto it = timers_.lower_bound({eik, INT64_MIN}); it != timers_.end() && it->first.first == eik;) {
      const TimerRow& t = it->second;
      ORecord& rec = append(ZBHIP_RT_EVENT, ZBHIP_VT_TIMER, ZBHIP_TIMER_CANCELED, it->first.second);
      rec.r.process_idx = t.pi.proc;
      rec.r.element_idx = t.pi.elem;
      rec.r.scope_key = eik;
      rec.r.process_instance_key = t.pi.piKey;
      rec.r.aux = t.dueDate;
      rec.r.partition = t.reps;
      it = timers_.erase(it);
    }
  }

  // `scope`: where the correlation key is evaluated -- the element itself, or for a boundary event
  // the activity's flow scope (CatchEventBehavior.evaluateCorrelationKey, common/CatchEventBehavior.java:187-205)
  // Returns false after the EXTRACT_VALUE_ERROR incident of a correlation key that is neither a string
  // nor a number (ExpressionProcessor.typeCheckCorrelationKey, :317-331; the failure's variableScopeKey
  // is `scope`): the element is left ACTIVATING, its caller writes nothing more (incidentBehavior
  // .createIncident(failure, context), JobWorkerTaskProcessor.onActivate :50-61).  `incident` is the
  // element instance the incident is raised on (the task for a boundary event) and its value.
  bool subscribe_to_message(const OEl& el, int64_t key, const PiValue& v, int64_t scope, int64_t incident_key,
                            const PiValue& incident_v) {
    // evaluateCorrelationKey (:155-178) -> ExpressionProcessor.evaluateMessageCorrelationKeyExpression
    // (processing/common/ExpressionProcessor.java:309-337): STRING or NUMBER, else incident
    auto nit = name_ids.find(el.corr_var);
    const VarRow* vr = nit == name_ids.end() ? nullptr : lookup_var(scope, nit->second);
    if (!vr || vr->type == ZBHIP_DOC_NIL || vr->type == ZBHIP_DOC_BOOL) {
      FlowFailure f;
      f.error_type = ZBHIP_ERR_EXTRACT_VALUE_ERROR;
      f.flow = kCorrelationKeyFailure;
      f.result = vr && vr->type == ZBHIP_DOC_BOOL ? kFeelBoolean : ZBHIP_FEEL_NULL;
      create_incident(f, incident_key, incident_v);
      incidents_.rbegin()->second.variable_scope = scope;
      batch_->back().r.message_key = scope;  // (the record's variableScopeKey; INCIDENT records only here)
      return false;
    }
    if (vr->type != ZBHIP_DOC_STR) throw Unsupported{"correlation key is a NUMBER (outside the subset)"};
    MsgVal m;
    m.corr = (uint32_t)vr->value;
    m.name = (uint16_t)intern(el.msg_name);
    m.bpmn = (uint16_t)intern(P(v.proc).bpmn_id);
    m.pik = v.piKey;
    m.eik = key;
    m.partition = subscription_partition(str(m.corr), partition_count_);
    // intermediate catch events interrupt (ExecutableCatchEvent.java:36-38); a boundary event as its
    // cancelActivity says (ExecutableBoundaryEvent.interrupting)
    m.interrupting = el.type == ZBHIP_EL_BOUNDARY_EVENT ? (el.interrupting ? 1 : 0) : 1;
    m.proc = v.proc;
    m.elem = v.elem;
    m.inst = cur_instance_;
    m.eord = ord_of(cur_instance_, key);
    if (pms_inst_[cur_instance_] > 0) throw Unsupported{"second open message subscription of an instance"};
    int64_t subKey = next_key();
    msg_record(ZBHIP_RT_EVENT, ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION, ZBHIP_PMS_CREATING, subKey, m);
    pms_[{key, (int)m.name}] = PmsRow{subKey, false, m};  // ProcessMessageSubscriptionCreatingApplier
    ++pms_inst_[cur_instance_];
    send_command(m.partition, ZBHIP_CMD_MSG_SUB_CREATE, m);
    return true;
  }

  // MessageSubscriptionCreateProcessor.processRecord (processing/message/MessageSubscriptionCreateProcessor.java:66-104)
  void message_subscription_create(ORecord& cmd) {
    const MsgVal c = cmd.m;
    MsgVal ack = c;
    if (msub_.count({c.eik, (int)c.name})) {
      send_command(partition_of_key(c.pik), ZBHIP_CMD_PMS_CREATE, ack);
      reject(cmd, ZBHIP_REJ_INVALID_STATE,
             "Expected to open a new message subscription for element with key '" + std::to_string(c.eik) +
                 "' and message name '" + names.at(c.name) +
                 "', but there is already a message subscription for that element key and message name opened");
      return;
    }
    int64_t k = next_key();
    msg_record(ZBHIP_RT_EVENT, ZBHIP_VT_MESSAGE_SUBSCRIPTION, ZBHIP_MS_CREATED, k, c);
    msub_[{c.eik, (int)c.name}] = MsgSub{k, false, c};  // MessageSubscriptionCreatedApplier
    msub_by_corr_.insert({(int)c.name, c.corr, c.eik});
    // MessageCorrelator.correlateNextMessage (processing/message/MessageCorrelator.java:41-96): the first
    // buffered message of [tenant, name, correlationKey] (key order) whose deadline is after now and that
    // no instance of this process got yet -> MESSAGE_SUBSCRIPTION:CORRELATING (the subscription key, the
    // command's record with the message key) and PROCESS_MESSAGE_SUBSCRIPTION:CORRELATE instead of the
    // acknowledgement
    for (auto it = msg_by_corr_.lower_bound({(int)c.name, c.corr, INT64_MIN});
         it != msg_by_corr_.end() && std::get<0>(*it) == (int)c.name && std::get<1>(*it) == c.corr; ++it) {
      const int64_t mk = std::get<2>(*it);
      if (!(messages_.at(mk).deadline > now_ms) || msg_correlated_.count({mk, (int)c.bpmn})) continue;
      MsgSub& sub = msub_.at({c.eik, (int)c.name});
      sub.rec.msg_key = mk;
      msg_record(ZBHIP_RT_EVENT, ZBHIP_VT_MESSAGE_SUBSCRIPTION, ZBHIP_MS_CORRELATING, k, sub.rec);
      sub.correlating = true;  // MessageSubscriptionCorrelatingApplier: updateToCorrelatingState,
      msg_correlated_.insert({mk, (int)c.bpmn});  // putMessageCorrelation
      send_command(partition_of_key(c.pik), ZBHIP_CMD_PMS_CORRELATE, sub.rec);
      return;
    }
    send_command(partition_of_key(c.pik), ZBHIP_CMD_PMS_CREATE, ack);
  }

  // ProcessMessageSubscriptionCreateProcessor.processRecord
  void process_message_subscription_create(ORecord& cmd) {
    if (cmd.r.record_type == ZBHIP_RT_COMMAND && cur_slot_) enter_instance(cmd.m.inst);
    const MsgVal c = cmd.m;
    auto it = pms_.find({c.eik, (int)c.name});
    if (it != pms_.end() && !it->second.opened) {
      msg_record(ZBHIP_RT_EVENT, ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION, ZBHIP_PMS_CREATED, it->second.key, it->second.rec);
      it->second.opened = true;  // ProcessMessageSubscriptionCreatedApplier.updateToOpenedState
      return;
    }
    const std::string base = "Expected to create process message subscription with element key '" +
                             std::to_string(c.eik) + "' and message name '" + names.at(c.name) + "', but ";
    if (it == pms_.end()) reject(cmd, ZBHIP_REJ_NOT_FOUND, base + "no such subscription was found");
    else reject(cmd, ZBHIP_REJ_INVALID_STATE, base + (it->second.closing ? "it is already closing" : "it is already opened"));
  }

  // CatchEventBehavior.unsubscribeFromMessageEvents / unsubscribeFromMessageEvent
  // (processing/common/CatchEventBehavior.java:394-432): per process message subscription of the
  // element instance, PROCESS_MESSAGE_SUBSCRIPTION:DELETING (its key and stored record;
  // ProcessMessageSubscriptionDeletingApplier -> updateToClosingState) and MESSAGE_SUBSCRIPTION:DELETE
  // to the subscription partition (SubscriptionCommandSender.closeMessageSubscription, :220-236)
  void unsubscribe_messages(int64_t eik) {
    for (auto it = pms_.lower_bound({eik, INT32_MIN}); it != pms_.end() && it->first.first == eik; ++it) {
      PmsRow& row = it->second;
      msg_record(ZBHIP_RT_EVENT, ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION, ZBHIP_PMS_DELETING, row.key, row.rec);
      row.closing = true;
      // closeMessageSubscription (SubscriptionCommandSender.java:220-236): a fresh record -- its
      // interrupting flag keeps the default (true)
      MsgVal del = row.rec;
      del.interrupting = 1;
      send_command(row.rec.partition, ZBHIP_CMD_MSG_SUB_DELETE, del);
    }
  }

  // MessageSubscriptionDeleteProcessor.processRecord (processing/message/MessageSubscriptionDeleteProcessor.java:50-68):
  // MESSAGE_SUBSCRIPTION:DELETED (the stored subscription; MessageSubscriptionDeletedApplier removes it),
  // then the acknowledgement PROCESS_MESSAGE_SUBSCRIPTION:DELETE (closeProcessMessageSubscription, :267-283)
  void message_subscription_delete(ORecord& cmd) {
    const MsgVal c = cmd.m;
    auto it = msub_.find({c.eik, (int)c.name});
    if (it == msub_.end()) throw Unsupported{"MESSAGE_SUBSCRIPTION:DELETE of no subscription (NOT_FOUND rejection)"};
    const MsgSub sub = it->second;
    msg_record(ZBHIP_RT_EVENT, ZBHIP_VT_MESSAGE_SUBSCRIPTION, ZBHIP_MS_DELETED, sub.key, sub.rec);
    msub_by_corr_.erase({(int)sub.rec.name, sub.rec.corr, sub.rec.eik});
    msub_.erase(it);
    send_command(partition_of_key(c.pik), ZBHIP_CMD_PMS_DELETE, c);
  }

  // ProcessMessageSubscriptionDeleteProcessor.processRecord (processing/message/
  // ProcessMessageSubscriptionDeleteProcessor.java:39-56): PROCESS_MESSAGE_SUBSCRIPTION:DELETED (the stored
  // subscription; ProcessMessageSubscriptionDeletedApplier removes it)
  void process_message_subscription_delete(ORecord& cmd) {
    if (cmd.r.record_type == ZBHIP_RT_COMMAND && cur_slot_) enter_instance(cmd.m.inst);
    const MsgVal c = cmd.m;
    auto it = pms_.find({c.eik, (int)c.name});
    if (it == pms_.end()) throw Unsupported{"PROCESS_MESSAGE_SUBSCRIPTION:DELETE of no subscription (NOT_FOUND rejection)"};
    msg_record(ZBHIP_RT_EVENT, ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION, ZBHIP_PMS_DELETED, it->second.key, it->second.rec);
    --pms_inst_[it->second.rec.inst];
    pms_.erase(it);
  }

  // the MESSAGE record of a message (MessageRecord.java:37-43): name, correlationKey, timeToLive, messageId,
  // deadline -- zbhip_record.reason_arg bit 1 marks them set: aux = timeToLive, scope_key = deadline,
  // partition = the messageId's string id (-1 none); without it (TTL 0, no id: the records the device
  // writes too) a reader takes TTL 0 / deadline = the command's timestamp
  void message_record(int intent, int64_t key, const StoredMessage& sm) {
    MsgVal mv;
    mv.name = sm.name;
    mv.corr = sm.corr;
    ORecord& r = msg_record(ZBHIP_RT_EVENT, ZBHIP_VT_MESSAGE, intent, key, mv);
    if (sm.ttl == 0 && sm.message_id == ZBHIP_NO_STRING) return;  // (the device's form: TTL 0, no id)
    r.r.reason_arg = 2;
    r.r.aux = sm.ttl;
    r.r.scope_key = sm.deadline;
    r.r.partition = sm.message_id == ZBHIP_NO_STRING ? -1 : (int32_t)sm.message_id;
  }

  // MessagePublishedApplier -> DbMessageState.put (:225-249)
  void put_message(int64_t key, const StoredMessage& sm) {
    messages_[key] = sm;
    msg_by_corr_.insert({(int)sm.name, sm.corr, key});
    msg_deadlines_.insert({sm.deadline, key});
    ++msg_deadline_count_;
    msg_stats_ = true;
    if (sm.message_id != ZBHIP_NO_STRING) msg_ids_.insert({(int)sm.name, sm.corr, sm.message_id});
  }

  // MessageExpiredApplier -> DbMessageState.remove (:313-349): the message, its index rows and its
  // MESSAGE_CORRELATED rows (a key no longer stored: nothing)
  void remove_message(int64_t key) {
    auto it = messages_.find(key);
    if (it == messages_.end()) return;
    const StoredMessage sm = it->second;
    messages_.erase(it);
    msg_by_corr_.erase({(int)sm.name, sm.corr, key});
    if (sm.message_id != ZBHIP_NO_STRING) msg_ids_.erase({(int)sm.name, sm.corr, sm.message_id});
    msg_deadlines_.erase({sm.deadline, key});
    --msg_deadline_count_;
    for (auto c = msg_correlated_.lower_bound({key, INT32_MIN}); c != msg_correlated_.end() && c->first == key;)
      c = msg_correlated_.erase(c);
  }

  // MessagePublishProcessor.processRecord / handleNewMessage (processing/message/MessagePublishProcessor.java
  // :83-124): a messageId already buffered for [name, correlationKey] -> ALREADY_EXISTS; else PUBLISHED
  // (deadline = the command's timestamp + timeToLive), correlateToSubscriptions, the correlate commands,
  // and with timeToLive <= 0 EXPIRED in the same batch.  (No message start events: their processes are
  // outside the oracle's deployments.)
  void publish_message(ORecord& cmd) {
    const MsgVal c = cmd.m;  // name, correlationKey, timeToLive, messageId (no variables)
    if (c.message_id != ZBHIP_NO_STRING && msg_ids_.count({(int)c.name, c.corr, c.message_id})) {
      reject(cmd, ZBHIP_REJ_ALREADY_EXISTS,
             "Expected to publish a new message with id '" + str(c.message_id) +
                 "', but a message with that id was already published");
      return;
    }
    int64_t msgKey = next_key();
    const StoredMessage sm{c.name, c.corr, c.ttl, c.timestamp + c.ttl, c.message_id};
    message_record(ZBHIP_MSG_PUBLISHED, msgKey, sm);
    put_message(msgKey, sm);
    // correlateToSubscriptions: visit [tenant, name, correlationKey, *] in element-instance-key order
    std::vector<MsgVal> correlating;
    std::set<int> bpmn_seen;
    for (auto it = msub_by_corr_.lower_bound({(int)c.name, c.corr, INT64_MIN}); it != msub_by_corr_.end(); ++it) {
      if (std::get<0>(*it) != (int)c.name || std::get<1>(*it) != c.corr) break;
      MsgSub& sub = msub_.at({std::get<2>(*it), (int)c.name});
      if (sub.correlating || bpmn_seen.count(sub.rec.bpmn)) continue;
      sub.rec.msg_key = msgKey;
      msg_record(ZBHIP_RT_EVENT, ZBHIP_VT_MESSAGE_SUBSCRIPTION, ZBHIP_MS_CORRELATING, sub.key, sub.rec);
      sub.correlating = true;  // MessageSubscriptionCorrelatingApplier
      msg_correlated_.insert({msgKey, (int)sub.rec.bpmn});
      bpmn_seen.insert(sub.rec.bpmn);
      correlating.push_back(sub.rec);
    }
    // correlateToMessageStartEvents (:157-180): the start event subscriptions of the name in process
    // definition key order; one instance per process, and per correlation key while an instance the key
    // created is active (an empty correlation key creates one every time)
    const bool no_key = c.corr == ZBHIP_NO_STRING || str(c.corr).empty();
    for (auto it = msg_start_subs_.lower_bound({(int)c.name, INT64_MIN});
         it != msg_start_subs_.end() && it->first.first == (int)c.name; ++it) {
      const MsgStartSub s = it->second;
      const int bpmn = P(s.proc).bpmn_name;
      if (bpmn_seen.count(bpmn) || (!no_key && active_by_corr_.count({bpmn, c.corr}))) continue;
      bpmn_seen.insert(bpmn);
      trigger_message_start_event(s, msgKey, c.name, c.corr);
    }
    // sendCorrelateCommand: correlateProcessMessageSubscription with the message's name and key
    for (MsgVal m : correlating) {
      m.msg_key = msgKey;
      m.name = c.name;
      m.corr = c.corr;
      send_command(partition_of_key(m.pik), ZBHIP_CMD_PMS_CORRELATE, m);
    }
    if (c.ttl <= 0) {  // EXPIRED in the same batch: MessageExpiredApplier removes it and its correlations
      message_record(ZBHIP_MSG_EXPIRED, msgKey, sm);
      remove_message(msgKey);
    }
  }

  // MESSAGE_BATCH:EXPIRE of the MessageTimeToLiveChecker, one message key at a time (MessageBatchExpire
  // Processor.java:33-52): MESSAGE:EXPIRED with an empty MessageRecord (name "", correlationKey "",
  // timeToLive -1, deadline -1), then MessageExpiredApplier.  tests/psm.py feeds the batch's keys.
  void expire_message(ORecord& cmd) {
    const StoredMessage empty{0xFFFF, ZBHIP_NO_STRING, -1, -1, ZBHIP_NO_STRING};
    message_record(ZBHIP_MSG_EXPIRED, cmd.r.key, empty);
    remove_message(cmd.r.key);
  }

  // EventHandle.triggerMessageStartEvent (processing/common/EventHandle.java:176-235): a new process
  // instance key; MESSAGE_START_EVENT_SUBSCRIPTION:CORRELATED (MessageStartEventSubscriptionCorrelatedApplier
  // .java:27-39: putMessageCorrelation, and with a correlation key the lock [bpmnProcessId, correlationKey]
  // and the instance's correlation key); PROCESS_EVENT:TRIGGERING of the start event in the process
  // definition's event scope (ProcessEventTriggeringApplier -> triggerStartEvent); then
  // PROCESS_INSTANCE:ACTIVATE_ELEMENT of the process (activateProcessInstanceForStartEvent)
  void trigger_message_start_event(const MsgStartSub& s, int64_t msgKey, uint16_t name, uint32_t corr) {
    const OProc& p = P(s.proc);
    const int64_t piKey = next_key();
    ORecord& r = append(ZBHIP_RT_EVENT, ZBHIP_VT_MESSAGE_START_EVENT_SUBSCRIPTION, ZBHIP_MSES_CORRELATED, s.key);
    r.r.process_idx = s.proc;
    r.r.element_idx = s.elem;
    r.r.process_instance_key = piKey;
    r.r.message_key = msgKey;
    r.r.correlation_key = corr;
    r.r.message_name = name;
    r.r.bpmn_process_id = (uint16_t)p.bpmn_name;
    msg_correlated_.insert({msgKey, p.bpmn_name});
    if (corr != ZBHIP_NO_STRING && !str(corr).empty()) {
      active_by_corr_.insert({p.bpmn_name, corr});
      pi_corr_keys_[piKey] = corr;
    }
    const int64_t eventKey = next_key();
    ORecord& pe = append(ZBHIP_RT_EVENT, ZBHIP_VT_PROCESS_EVENT, ZBHIP_PE_TRIGGERING, eventKey);
    pe.r.process_idx = s.proc;
    pe.r.element_idx = s.elem;
    pe.r.scope_key = p.def_key;
    pe.r.process_instance_key = piKey;
    triggers_[{p.def_key, eventKey}] = EventTrigger{s.elem, s.proc, Doc{0, 0}, piKey};
    PiValue v;
    v.proc = s.proc;
    v.elem = 0;
    v.flowScopeKey = -1;
    v.piKey = piKey;
    pi_command(piKey, ZBHIP_PI_ACTIVATE_ELEMENT, v);
  }

  // ProcessProcessor's post-transition action of a process with message start events (ProcessProcessor
  // .java:196-206) -> BpmnBufferedMessageStartEventBehavior.correlateMessage (:56-120): after an instance a
  // message created with a correlation key ended (its lock released by the applier), the first buffered
  // message of that key for the latest version's start events -- by message key over the subscriptions,
  // visited in message-name order -- that is not expired and not yet correlated to the process starts the
  // next instance
  void correlate_buffered_start_message(int proc, uint32_t corr) {
    int latest = proc;
    for (size_t i = 0; i < procs.size(); ++i)
      if (procs[i].bpmn_id == P(proc).bpmn_id && procs[i].version > P(latest).version) latest = (int)i;
    const OProc& p = P(latest);
    std::vector<std::pair<std::string, MsgStartSub>> subs;  // [processDefinitionKey, [tenant, messageName]] order
    for (auto& [k, s] : msg_start_subs_)
      if (s.proc == latest) subs.push_back({names.at(k.first), s});
    std::sort(subs.begin(), subs.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    int64_t best = INT64_MAX;
    const MsgStartSub* chosen = nullptr;
    uint16_t chosen_name = 0;
    for (auto& [nm, s] : subs) {
      const int name = (int)name_ids.at(nm);
      for (auto it = msg_by_corr_.lower_bound({name, corr, INT64_MIN});
           it != msg_by_corr_.end() && std::get<0>(*it) == name && std::get<1>(*it) == corr; ++it) {
        const int64_t mk = std::get<2>(*it);
        if (messages_.at(mk).deadline > now_ms && !msg_correlated_.count({mk, p.bpmn_name})) {
          if (mk < best) {
            best = mk;
            chosen = &s;
            chosen_name = (uint16_t)name;
          }
          break;
        }
      }
    }
    if (chosen) trigger_message_start_event(*chosen, best, chosen_name, corr);
  }

  // ProcessMessageSubscriptionCorrelateProcessor.processRecord
  void process_message_subscription_correlate(ORecord& cmd) {
    if (cur_slot_) enter_instance(cmd.m.inst);
    const MsgVal c = cmd.m;
    auto it = pms_.find({c.eik, (int)c.name});
    if (it == pms_.end()) throw Unsupported{"PMS correlate rejection (MESSAGE_SUBSCRIPTION:REJECT outside the subset)"};
    if (it->second.closing) throw Unsupported{"PMS correlate of a closing subscription (MESSAGE_SUBSCRIPTION:REJECT)"};
    auto eit = ei_.find(c.eik);
    // EventHandle.canTriggerElement: active instance, event scope accepting, flow scope not interrupted
    if (eit == ei_.end() || eit->second.state != ZBHIP_PI_ELEMENT_ACTIVATED || !event_scope_.count(c.eik))
      throw Unsupported{"PMS correlate rejection (no event occurred)"};
    MsgVal m = c;  // record.setElementId(subscription elementId).setInterrupting(...)
    m.interrupting = it->second.rec.interrupting;
    m.proc = it->second.rec.proc;
    m.elem = it->second.rec.elem;
    const int64_t subKey = it->second.key;
    const bool interrupting = it->second.rec.interrupting;
    msg_record(ZBHIP_RT_EVENT, ZBHIP_VT_PROCESS_MESSAGE_SUBSCRIPTION, ZBHIP_PMS_CORRELATED, subKey, m);
    if (interrupting) {  // ProcessMessageSubscriptionCorrelatedApplier (:27-37): removed ...
      --pms_inst_[it->second.rec.inst];
      pms_.erase(it);
    } else {  // ... or, non-interrupting, updateToOpenedState(record): the stored record is the CORRELATED one
      MsgVal& row = it->second.rec;
      const MsgVal keep = row;
      row = m;
      row.inst = keep.inst;
      row.eord = keep.eord;
      it->second.opened = true;
    }
    // EventHandle.activateElement (processing/common/EventHandle.java:109-150)
    const ElementInstance inst = eit->second;
    int64_t eventKey = next_key();
    ORecord& pe = append(ZBHIP_RT_EVENT, ZBHIP_VT_PROCESS_EVENT, ZBHIP_PE_TRIGGERING, eventKey);
    pe.r.process_idx = inst.value.proc;
    pe.r.element_idx = m.elem;  // ProcessEventRecord.targetElementId: the catch event (a boundary event's own id)
    pe.r.scope_key = c.eik;
    pe.r.process_instance_key = inst.value.piKey;
    if (P(m.proc).els[m.elem].type == ZBHIP_EL_BOUNDARY_EVENT) {
      // a boundary event of the activity: the trigger (ProcessEventTriggeringApplier, interrupting the
      // event scope), then TERMINATE_ELEMENT of the activity -- its onTerminate activates the event; a
      // non-interrupting one is activated right away (EventTriggerBehavior.activateTriggeredEvent)
      trigger_event(c.eik, eventKey, m.elem, m.proc, Doc{0, 0}, inst.value.piKey);
      if (interrupting)
        pi_command(c.eik, ZBHIP_PI_TERMINATE_ELEMENT, inst.value);
      else
        activate_triggered_event(eventKey, m.elem, c.eik, inst.value.flowScopeKey, inst.value);
    } else {
      if (event_scope_.count(c.eik))  // ProcessEventTriggeringApplier: trigger with the message variables (none)
        triggers_[{c.eik, eventKey}] = EventTrigger{inst.value.elem, inst.value.proc, Doc{0, 0}, inst.value.piKey};
      pi_command(c.eik, ZBHIP_PI_COMPLETE_ELEMENT, inst.value);  // isElementActivated: intermediate catch
    }
    // sendAcknowledgeCommand -> correlateMessageSubscription(record.subscriptionPartitionId, ...)
    MsgVal ack = c;
    ack.corr = it == pms_.end() ? c.corr : c.corr;
    send_command(c.partition, ZBHIP_CMD_MSG_SUB_CORRELATE, ack);
  }

  // MessageSubscriptionCorrelateProcessor.processRecord
  void message_subscription_correlate(ORecord& cmd) {
    const MsgVal c = cmd.m;
    auto it = msub_.find({c.eik, (int)c.name});
    if (it == msub_.end()) {
      reject(cmd, ZBHIP_REJ_NOT_FOUND,
             "Expected to correlate subscription for element with key '" + std::to_string(c.eik) +
                 "' and message name '" + names.at(c.name) + "', but no such message subscription exists");
      return;
    }
    const MsgSub sub = it->second;
    msg_record(ZBHIP_RT_EVENT, ZBHIP_VT_MESSAGE_SUBSCRIPTION, ZBHIP_MS_CORRELATED, sub.key, sub.rec);
    // MessageSubscriptionCorrelatedApplier (:26-37): removed, or (non-interrupting) open again for the
    // next message -- updateToCorrelatedState: not correlating, the last message key kept
    if (!sub.rec.interrupting) {
      it->second.correlating = false;
      return;
    }
    msub_by_corr_.erase({(int)sub.rec.name, sub.rec.corr, sub.rec.eik});
    msub_.erase(it);
  }

  // ---------------------------------------------------------------------
  // CreateProcessInstanceProcessor (processing/processinstance/CreateProcessInstanceProcessor.java:100-158,319-330)
  // wrapped by CommandProcessorImpl.processRecord (processing/streamprocessor/CommandProcessorImpl.java:65-103)
  // ---------------------------------------------------------------------
  void create_process_instance(ORecord& cmd) {
    int proc = cmd.r.process_idx;
    if (proc < 0 || proc >= (int)procs.size()) {
      reject(cmd, ZBHIP_REJ_NOT_FOUND, "Expected to find process definition with key '" +
                                           std::to_string(proc) + "', but none found");
      return;
    }
    const OProc& p = P(proc);
    if (p.none_start < 0) {
      reject(cmd, ZBHIP_REJ_INVALID_STATE,
             "Expected to create instance of process with none start event, but there is no such event");
      return;
    }
    int64_t piKey = next_key();
    // setVariablesFromDocument -> VariableBehavior.mergeLocalDocument (processing/variable/VariableBehavior.java:60-82)
    merge_local_document(piKey, proc, piKey, cmd.doc);
    PiValue v;  // initProcessInstanceRecord
    v.proc = proc;
    v.elem = 0;
    v.flowScopeKey = -1;
    v.piKey = piKey;
    pi_command(piKey, ZBHIP_PI_ACTIVATE_ELEMENT, v);
    // controller.accept(CREATED) -> entityKey = nextKey (command key is -1)
    int64_t createdKey = next_key();
    ORecord& rec = append(ZBHIP_RT_EVENT, ZBHIP_VT_PROCESS_INSTANCE_CREATION, ZBHIP_PIC_CREATED, createdKey);
    rec.r.process_idx = proc;
    rec.r.element_idx = 0;
    rec.r.scope_key = piKey;
    rec.r.process_instance_key = piKey;
    rec.r.aux = cmd.doc.count ? (int64_t)cmd.doc.begin : -1;
    rec.doc = cmd.doc;
  }

  // The byte size of a value / string as the log writes it (MsgPackWriter: the smallest integer form,
  // float64 decimals, fixstr / str8 / str16 / str32, fixarray / array16 / array32 of scalars)
  static size_t mp_str_size(size_t n) { return n + (n < 32 ? 1 : n < 256 ? 2 : n < 65536 ? 3 : 5); }
  size_t mp_value_size(uint8_t type, int64_t v) const {
    switch (type) {
      case ZBHIP_DOC_NIL:
      case ZBHIP_DOC_BOOL: return 1;
      case ZBHIP_DOC_INT:
        if (v < -(1LL << 5)) return v < -(1LL << 31) ? 9 : v < -(1LL << 15) ? 5 : v < -(1LL << 7) ? 3 : 2;
        return v < (1LL << 7) ? 1 : v < (1LL << 8) ? 2 : v < (1LL << 16) ? 3 : v < (1LL << 32) ? 5 : 9;
      case ZBHIP_DOC_DEC: return 9;
      case ZBHIP_DOC_STR: return mp_str_size(str((uint32_t)v).size());
      case ZBHIP_DOC_LIST: {
        const Items& items = lists.at((size_t)v);
        size_t n = items.size() < 16 ? 1 : items.size() < 65536 ? 3 : 5;
        for (const auto& it : items) n += mp_value_size(it.first, it.second);
        return n;
      }
      default: throw Unsupported{"a document value of unknown encoded size"};
    }
  }

  // IndexedDocument.index (IndexedDocument.java:44-56): key offset -> value offset of every entry of
  // the document's msgpack map, into the agrona map; keys[offset] = the entry
  AgronaIntMap index_document(const Doc& d, std::map<int32_t, uint32_t>& keys) const {
    AgronaIntMap m;
    size_t at = d.count < 16 ? 1 : d.count < 65536 ? 3 : 5;
    for (uint32_t j = 0; j < d.count; ++j) {
      const zbhip_doc_entry& de = docs[d.begin + j];
      const size_t name = mp_str_size(names.at(de.name_id).size());
      m.put((int32_t)at, (int32_t)(at + name));
      keys[(int32_t)at] = d.begin + j;
      at += name + mp_value_size(de.type, de.value);
    }
    return m;
  }

  // VariableBehavior.mergeLocalDocument + setLocalVariable (VariableBehavior.java:60-82,191-200): every
  // entry in the IndexedDocument's iteration order
  void merge_local_document(int64_t scopeKey, int proc, int64_t piKey, const Doc& d) {
    if (d.count == 0) return;
    std::map<int32_t, uint32_t> keys;
    AgronaIntMap m = index_document(d, keys);
    AgronaIntMap::Iter it = m.iterator();
    for (int32_t k; m.next(it, k);) set_local_variable(scopeKey, proc, piKey, keys.at(k));
  }

  void set_local_variable(int64_t scopeKey, int proc, int64_t piKey, uint32_t entry) {
    const zbhip_doc_entry& de = docs[entry];
    auto it = vars_.find({scopeKey, (int)de.name_id});
    if (it == vars_.end()) {
      int64_t key = next_key();
      var_event(key, ZBHIP_VAR_CREATED, scopeKey, proc, piKey, entry);
    } else if (!(it->second.type == de.type && it->second.value == de.value)) {
      var_event(it->second.key, ZBHIP_VAR_UPDATED, scopeKey, proc, piKey, entry);
    }
  }

  void var_event(int64_t key, int intent, int64_t scopeKey, int proc, int64_t piKey, uint32_t entry) {
    ORecord& rec = append(ZBHIP_RT_EVENT, ZBHIP_VT_VARIABLE, intent, key);
    rec.r.process_idx = proc;
    rec.r.element_idx = (int32_t)docs[entry].name_id;
    rec.r.scope_key = scopeKey;
    rec.r.process_instance_key = piKey;
    rec.r.aux = entry;
    // VariableApplier.applyState -> DbVariableState.setVariableLocal
    vars_[{scopeKey, (int)docs[entry].name_id}] = VarRow{key, docs[entry].type, docs[entry].value, entry};
  }

  // VariableBehavior.mergeDocument (VariableBehavior.java:105-150): every scope below the process
  // instance's iterates the entries left, updating (and removing) those it holds with another value; the
  // process instance's scope sets the rest, in the iteration order of what is left
  void merge_document(int64_t scopeKey, int proc, int64_t piKey, const Doc& d) {
    if (d.count == 0) return;
    std::map<int32_t, uint32_t> keys;
    AgronaIntMap m = index_document(d, keys);
    int64_t current = scopeKey;
    for (;;) {
      auto pit = child_parent_.find(current);
      int64_t parent = pit == child_parent_.end() ? -1 : pit->second;
      if (parent <= 0) break;
      AgronaIntMap::Iter it = m.iterator();
      for (int32_t k; m.next(it, k);) {
        const uint32_t e = keys.at(k);
        const zbhip_doc_entry& de = docs[e];
        auto vit = vars_.find({current, (int)de.name_id});
        if (vit != vars_.end() && !(vit->second.type == de.type && vit->second.value == de.value)) {
          var_event(vit->second.key, ZBHIP_VAR_UPDATED, current, proc, piKey, e);
          m.remove(it);
        }
      }
      current = parent;
    }
    AgronaIntMap::Iter it = m.iterator();
    for (int32_t k; m.next(it, k);) set_local_variable(current, proc, piKey, keys.at(k));
  }

  // ---------------------------------------------------------------------
  // JobCompleteProcessor (processing/job/JobCompleteProcessor.java:47-92) with
  // DefaultJobCommandPreconditionGuard (processing/job/DefaultJobCommandPreconditionGuard.java:26-46)
  // ---------------------------------------------------------------------
  void complete_job(ORecord& cmd) {
    if (cmd.job_ord >= 0) cmd.r.key = resolve(cmd.instance, (uint32_t)cmd.job_ord);
    int64_t jobKey = cmd.r.key;
    auto jit = jobs_.find(jobKey);
    if (jit == jobs_.end()) {
      // JobCommandPreconditionChecker.check: NOT_FOUND
      reject(cmd, ZBHIP_REJ_NOT_FOUND,
             "Expected to complete job with key '" + std::to_string(jobKey) + "', but no such job was found");
      return;
    }
    if (jit->second.failed || jit->second.error_thrown) {  // DefaultJobCommandPreconditionGuard: ACTIVATABLE or ACTIVATED only
      reject(cmd, ZBHIP_REJ_INVALID_STATE, "Expected to complete job with key '" + std::to_string(jobKey) +
                                               "', but it is in state '" +
                                               (jit->second.error_thrown ? "ERROR_THROWN" : "FAILED") + "'");
      return;
    }
    JobRow job = jit->second;
    // accept(COMPLETED, job with command variables) -> event, JobCompletedApplier
    ORecord& rec = append(ZBHIP_RT_EVENT, ZBHIP_VT_JOB, ZBHIP_JOB_COMPLETED, jobKey);
    rec.r.process_idx = job.pi.proc;
    rec.r.element_idx = job.pi.elem;
    rec.r.scope_key = job.elementInstanceKey;
    rec.r.process_instance_key = job.pi.piKey;
    rec.r.aux = cmd.doc.count ? (int64_t)cmd.doc.begin : -1;
    rec.doc = cmd.doc;
    job_activation_fields(rec, job);
    apply_job_completed(jobKey, job);
    // afterAccept
    auto sit = ei_.find(job.elementInstanceKey);
    if (sit != ei_.end()) {
      ElementInstance task = sit->second;
      auto fit = ei_.find(task.value.flowScopeKey);
      if (fit != ei_.end() && fit->second.state == ZBHIP_PI_ELEMENT_ACTIVATED) {
        // EventHandle.triggeringProcessEvent(JobRecord) (processing/common/EventHandle.java:151-158)
        // -> EventTriggerBehavior.triggeringProcessEvent (processing/common/EventTriggerBehavior.java:148-166)
        int64_t eventKey = next_key();
        ORecord& pe = append(ZBHIP_RT_EVENT, ZBHIP_VT_PROCESS_EVENT, ZBHIP_PE_TRIGGERING, eventKey);
        pe.r.process_idx = job.pi.proc;
        pe.r.element_idx = job.pi.elem;
        pe.r.scope_key = job.elementInstanceKey;
        pe.r.process_instance_key = job.pi.piKey;
        pe.r.aux = cmd.doc.count ? (int64_t)cmd.doc.begin : -1;
        pe.doc = cmd.doc;
        // ProcessEventTriggeringApplier (state/appliers/ProcessEventTriggeringApplier.java:35-56)
        // -> DbEventScopeInstanceState.triggerEvent (only if the scope accepts)
        trigger_event(job.elementInstanceKey, eventKey, job.pi.elem, job.pi.proc, cmd.doc, job.pi.piKey);
        pi_command(job.elementInstanceKey, ZBHIP_PI_COMPLETE_ELEMENT, task.value);
      }
    }
  }

  // JobTimeOutProcessor.processRecord (processing/job/JobTimeOutProcessor.java:46-73): an ACTIVATED job
  // whose deadline passed (deadline < ActorClock.currentTimeMillis()) -> JOB:TIMED_OUT with the stored
  // job; JobTimedOutApplier -> DbJobState.timeout (:142-150): ACTIVATABLE again, the record (deadline,
  // worker) kept, out of JOB_DEADLINES.  Else NOT_FOUND "Expected to time out activated job with key
  // '%d', but %s".  (publishWork's notification / push is a side effect; no stream: no records.)
  void time_out_job(ORecord& cmd) {
    if (cmd.job_ord >= 0) cmd.r.key = resolve(cmd.instance, (uint32_t)cmd.job_ord);
    const int64_t jobKey = cmd.r.key;
    auto jit = jobs_.find(jobKey);
    const char* why = jit == jobs_.end() ? "no such job was found"
                      : jit->second.failed ? "it is marked as failed and is not activated"
                      : jit->second.error_thrown ? "it has thrown an error and is not activated"
                      : !jit->second.activated ? "it must be activated first"
                      : !(jit->second.deadline < now_ms) ? "it has not timed out" : nullptr;
    if (why) {
      reject(cmd, ZBHIP_REJ_NOT_FOUND,
             "Expected to time out activated job with key '" + std::to_string(jobKey) + "', but " + why);
      return;
    }
    JobRow& job = jit->second;
    ORecord& rec = append(ZBHIP_RT_EVENT, ZBHIP_VT_JOB, ZBHIP_JOB_TIMED_OUT, jobKey);
    rec.r.process_idx = job.pi.proc;
    rec.r.element_idx = job.pi.elem;
    rec.r.scope_key = job.elementInstanceKey;
    rec.r.process_instance_key = job.pi.piKey;
    job_activation_fields(rec, job);
    job.activated = false;
    activatable_.insert({job.type, "<default>", jobKey});
    publish_work(jobKey);
  }

  // JobFailProcessor.processRecord / failJob (processing/job/JobFailProcessor.java:79-162): the job
  // must be ACTIVATABLE or ACTIVATED (else NOT_FOUND / INVALID_STATE); JOB:FAILED with the stored job and
  // the command's retries, errorMessage (limitString, 10000), retryBackoff and variables (recurringTime =
  // timestamp + backoff when it retries later), the variables merged into the job's element instance
  // (setFailedVariables), no retries left -> INCIDENT:CREATED (JOB_NO_RETRIES, "No more retries left."
  // unless the job says otherwise; key = nextKey, jobKey, variableScopeKey = the element instance).
  // JobFailedApplier -> DbJobState.fail (:191-203).  The command: retries in `partition`, retryBackoff in
  // `message_key`, errorMessage's string id in `correlation_key`, its document in `aux`; timestamp = now.
  void fail_job(ORecord& cmd) {
    if (cmd.job_ord >= 0) cmd.r.key = resolve(cmd.instance, (uint32_t)cmd.job_ord);
    const int64_t jobKey = cmd.r.key;
    auto jit = jobs_.find(jobKey);
    if (jit == jobs_.end()) {
      reject(cmd, ZBHIP_REJ_NOT_FOUND, "Expected to fail job with key '" + std::to_string(jobKey) + "', but no such job was found");
      return;
    }
    if (jit->second.failed || jit->second.error_thrown) {
      reject(cmd, ZBHIP_REJ_INVALID_STATE, "Expected to fail job with key '" + std::to_string(jobKey) +
                                               "', but it is in state '" +
                                               (jit->second.error_thrown ? "ERROR_THROWN" : "FAILED") + "'");
      return;
    }
    JobRow& job = jit->second;
    const int retries = cmd.r.partition;
    const int64_t backoff = cmd.r.message_key;
    std::string msg = cmd.r.correlation_key < strs.size() ? strs[cmd.r.correlation_key] : std::string();
    msg = limit_java_string(msg, 10000);
    job.retries = retries;
    job.error_message = msg;
    job.retry_backoff = backoff;
    job.fail_fields = true;
    if (retries > 0 && backoff > 0) job.recurring_time = now_ms + backoff;
    ORecord& rec = append(ZBHIP_RT_EVENT, ZBHIP_VT_JOB, ZBHIP_JOB_FAILED, jobKey);
    rec.r.process_idx = job.pi.proc;
    rec.r.element_idx = job.pi.elem;
    rec.r.scope_key = job.elementInstanceKey;
    rec.r.process_instance_key = job.pi.piKey;
    rec.r.aux = cmd.doc.count ? (int64_t)cmd.doc.begin : -1;
    rec.doc = cmd.doc;
    job_activation_fields(rec, job);
    // JobFailedApplier -> DbJobState.fail: updateJob(retries > 0: backoff ? FAILED : ACTIVATABLE; else FAILED)
    job.activated = false;
    job.failed = !(retries > 0 && backoff <= 0);
    if (!job.failed) activatable_.insert({job.type, "<default>", jobKey});
    else activatable_.erase({job.type, "<default>", jobKey});
    // setFailedVariables: mergeLocalDocument into the job's element instance
    merge_local_document(job.elementInstanceKey, job.pi.proc, job.pi.piKey, cmd.doc);
    if (retries > 0 && backoff <= 0) publish_work(jobKey);  // retryImmediately
    if (retries <= 0) {  // raiseIncident (:139-162)
      const int64_t key = next_key();
      ORecord& in = append(ZBHIP_RT_EVENT, ZBHIP_VT_INCIDENT, ZBHIP_INCIDENT_CREATED, key);
      in.r.process_idx = job.pi.proc;
      in.r.element_idx = job.pi.elem;
      in.r.scope_key = job.elementInstanceKey;
      in.r.process_instance_key = job.pi.piKey;
      in.r.partition = ZBHIP_ERR_JOB_NO_RETRIES;
      in.r.aux = jobKey;
      const std::string text = msg.empty() ? "No more retries left." : msg;
      in.r.correlation_key = intern_string(text);
      IncidentRow row;
      row.pi = job.pi;
      row.eik = job.elementInstanceKey;
      row.error_type = ZBHIP_ERR_JOB_NO_RETRIES;
      row.job_key = jobKey;
      row.message = text;
      incidents_[key] = row;
      incident_jobs_[jobKey] = key;
    }
  }

  // JobThrowErrorProcessor (processing/job/JobThrowErrorProcessor.java:84-176) with CatchEventAnalyzer
  // .findErrorCatchEvent (processing/common/CatchEventAnalyzer.java:55-160): the job must be ACTIVATABLE or
  // ACTIVATED (JobCommandPreconditionChecker: NOT_FOUND / INVALID_STATE); the job takes the command's errorCode,
  // errorMessage (limitString, 10 000) and variables; the catch event is looked up from the job's element
  // instance up through its flow scopes, per scope the element's error events code-specific before a catch-all
  // (the codes seen are the "available" ones).  Caught: JOB:ERROR_THROWN (JobErrorThrownApplier: throwError,
  // then the task's job reference removed and the job deleted), then BpmnEventPublicationBehavior
  // .throwErrorEvent -> EventHandle.activateElement: PROCESS_EVENT:TRIGGERING (the command's variables) and,
  // an error boundary event interrupting, TERMINATE_ELEMENT of the task.  Not caught: the job's elementId
  // becomes NO_CATCH_EVENT_FOUND, JOB:ERROR_THROWN (the job stays, ERROR_THROWN) and INCIDENT:CREATED
  // (UNHANDLED_ERROR_EVENT, the analyzer's message; elementId the marker, jobKey, variableScopeKey = the
  // element instance).  The command: errorCode's string id in `partition`, errorMessage's in
  // `correlation_key`, its document in `aux`.
  void throw_error(ORecord& cmd) {
    if (cmd.job_ord >= 0) cmd.r.key = resolve(cmd.instance, (uint32_t)cmd.job_ord);
    const int64_t jobKey = cmd.r.key;
    auto jit = jobs_.find(jobKey);
    const std::string pre = "Expected to throw an error for job with key '" + std::to_string(jobKey) + "', but ";
    if (jit == jobs_.end()) { reject(cmd, ZBHIP_REJ_NOT_FOUND, pre + "no such job was found"); return; }
    if (jit->second.failed || jit->second.error_thrown) {
      reject(cmd, ZBHIP_REJ_INVALID_STATE,
             pre + "it is in state '" + (jit->second.error_thrown ? "ERROR_THROWN" : "FAILED") + "'");
      return;
    }
    JobRow& job = jit->second;
    const std::string code = cmd.r.partition >= 0 && (uint32_t)cmd.r.partition < strs.size() ? strs[cmd.r.partition] : "";
    const std::string msg =
        limit_java_string(cmd.r.correlation_key < strs.size() ? strs[cmd.r.correlation_key] : std::string(), 10000);
    // findErrorCatchEvent: from the job's element instance through its active, not interrupted flow scopes
    std::vector<std::string> avail;
    int catch_elem = -1;
    int64_t scope = job.elementInstanceKey;
    find_error_catch_event(code, scope, avail, catch_elem);
    auto put = [&](const char* elem_marker) {  // JOB:ERROR_THROWN with the stored job + the command's fields
      ORecord& rec = append(ZBHIP_RT_EVENT, ZBHIP_VT_JOB, ZBHIP_JOB_ERROR_THROWN, jobKey);
      rec.r.process_idx = job.pi.proc;
      rec.r.element_idx = job.pi.elem;
      rec.r.scope_key = job.elementInstanceKey;
      rec.r.process_instance_key = job.pi.piKey;
      rec.r.aux = cmd.doc.count ? (int64_t)cmd.doc.begin : -1;
      rec.doc = cmd.doc;
      JobRow shown = job;
      shown.fail_fields = true;  // (the errorMessage travels as a failed job's does)
      shown.error_message = msg;
      job_activation_fields(rec, shown);
      // errorCode's string id: reason_arg bit 2, in interrupting | pad[0] << 8 | pad[1] << 16
      const uint32_t cid = intern_string(code);
      rec.r.reason_arg |= 4 | (elem_marker ? 8 : 0);  // (bit 3: elementId NO_CATCH_EVENT_FOUND)
      rec.r.interrupting = (uint8_t)cid;
      rec.r.pad[0] = (uint8_t)(cid >> 8);
      rec.r.pad[1] = (uint8_t)(cid >> 16);
    };
    if (catch_elem < 0) {
      job.no_catch = true;
      put("NO_CATCH_EVENT_FOUND");
      // DbJobState.throwError: the record (errorCode, errorMessage, the marker) stored, ERROR_THROWN, not
      // activatable, out of JOB_DEADLINES
      job.error_thrown = true;
      job.error_code = code;
      job.error_message = msg;
      job.fail_fields = true;
      job.activated = false;
      activatable_.erase({job.type, "<default>", jobKey});
      std::string text = "Expected to throw an error event with the code '" + code + "'" +
                         (msg.empty() ? std::string() : " with message '" + msg + "'") + ", but it was not caught.";
      if (avail.empty()) {
        text += " No error events are available in the scope.";
      } else {
        text += " Available error events are [";
        for (size_t i = 0; i < avail.size(); ++i) text += (i ? ", " : "") + avail[i];
        text += "]";
      }
      const int64_t key = next_key();
      ORecord& in = append(ZBHIP_RT_EVENT, ZBHIP_VT_INCIDENT, ZBHIP_INCIDENT_CREATED, key);
      in.r.process_idx = job.pi.proc;
      in.r.element_idx = job.pi.elem;
      in.r.reason_arg = 8;  // elementId NO_CATCH_EVENT_FOUND
      in.r.scope_key = job.elementInstanceKey;
      in.r.process_instance_key = job.pi.piKey;
      in.r.partition = ZBHIP_ERR_UNHANDLED_ERROR_EVENT;
      in.r.aux = jobKey;
      in.r.correlation_key = intern_string(text);
      IncidentRow row;
      row.pi = job.pi;
      row.eik = job.elementInstanceKey;
      row.error_type = ZBHIP_ERR_UNHANDLED_ERROR_EVENT;
      row.job_key = jobKey;
      row.message = text;
      row.no_catch = true;
      incidents_[key] = row;
      incident_jobs_[jobKey] = key;
      return;
    }
    // (the task not active / its event scope not accepting: rejections naming ElementInstance.toString --
    // outside the restatement)
    if (!can_trigger(scope, catch_elem, job.pi.proc)) throw Unsupported{"THROW_ERROR into a scope not accepting events"};
    put(nullptr);
    // JobErrorThrownApplier: the task's job reference removed, the job deleted
    const JobRow gone = job;
    ei_.at(job.elementInstanceKey).jobKey = -1;
    activatable_.erase({gone.type, "<default>", jobKey});
    jobs_.erase(jit);
    // throwErrorEvent -> EventHandle.activateElement (common/EventHandle.java:104-150)
    const ElementInstance task = ei_.at(scope);
    const int64_t eventKey = next_key();
    ORecord& pe = append(ZBHIP_RT_EVENT, ZBHIP_VT_PROCESS_EVENT, ZBHIP_PE_TRIGGERING, eventKey);
    pe.r.process_idx = task.value.proc;
    pe.r.element_idx = catch_elem;
    pe.r.scope_key = scope;
    pe.r.process_instance_key = task.value.piKey;
    pe.r.aux = cmd.doc.count ? (int64_t)cmd.doc.begin : -1;
    pe.doc = cmd.doc;
    trigger_event(scope, eventKey, catch_elem, task.value.proc, cmd.doc, task.value.piKey);
    if (P(task.value.proc).els[catch_elem].type == ZBHIP_EL_START_EVENT) {
      trigger_event_sub_process(catch_elem, scope);  // an event sub-process's start event
      return;
    }
    pi_command(scope, ZBHIP_PI_TERMINATE_ELEMENT, task.value);
  }

  // CatchEventAnalyzer.findErrorCatchEvent (:55-160): from the instance `scope` through its active flow
  // scopes not interrupted by an event sub-process (ElementInstance.isInterrupted); every error code visited
  // joins `avail`; on a match `catch_elem` is the catch event and `scope` the instance it belongs to
  void find_error_catch_event(const std::string& code, int64_t& scope, std::vector<std::string>& avail,
                              int& catch_elem) {
    catch_elem = -1;
    for (auto it = ei_.find(scope); it != ei_.end() && catch_elem < 0;) {
      const ElementInstance& inst = it->second;
      if (!(inst.state == ZBHIP_PI_ELEMENT_ACTIVATING || inst.state == ZBHIP_PI_ELEMENT_ACTIVATED) ||
          inst.interrupting_elem >= 0)
        break;

      const OEl& el = E(inst.value);
      // findErrorCatchEventInScope: the element's error catch events ordered by errorCode, descending
      // (ERROR_CODE_COMPARATOR: DirectBuffer.compareTo -- signed bytes, then length -- reversed; a
      // stable sort), each visited code joining the available ones until the first match
      // (getEvents: the event sub-processes' start events -- each attached at index 0, so the last one
      // first -- then the boundary events)
      std::vector<int> errs;
      for (auto e = el.esps.rbegin(); e != el.esps.rend(); ++e)
        if (P(inst.value.proc).els[P(inst.value.proc).els[*e].start].event == ZBHIP_EV_ERROR)
          errs.push_back(P(inst.value.proc).els[*e].start);
      for (int b : el.boundaries)
        if (P(inst.value.proc).els[b].event == ZBHIP_EV_ERROR) errs.push_back(b);
      auto signed_less = [](const std::string& x, const std::string& y) {
        for (size_t i = 0; i < x.size() && i < y.size(); ++i)
          if ((int8_t)x[i] != (int8_t)y[i]) return (int8_t)x[i] < (int8_t)y[i];
        return x.size() < y.size();
      };
      std::stable_sort(errs.begin(), errs.end(), [&](int x, int y) {
        return signed_less(P(inst.value.proc).els[y].error_code, P(inst.value.proc).els[x].error_code);
      });
      for (int b : errs) {
        const std::string& bc = P(inst.value.proc).els[b].error_code;
        avail.push_back(bc);
        if (bc.empty() || bc == code) {
          catch_elem = b;
          scope = inst.key;
          break;
        }
      }
      if (catch_elem >= 0) break;
      it = ei_.find(inst.parentKey);
    }
  }

  // EndEventProcessor.ErrorEndEventBehavior.onActivate (:143-158): the catch event from the end event's
  // flow scope up (BpmnEventPublicationBehavior.findErrorCatchEvent) -> ACTIVATED, then throwErrorEvent
  // (canTriggerElement -> EventHandle.activateElement without variables: PROCESS_EVENT:TRIGGERING, then the
  // event sub-process's trigger or TERMINATE_ELEMENT of the boundary event's activity); none -> an
  // UNHANDLED_ERROR_EVENT incident on the end event (ACTIVATING), its message without an error message
  void throw_error_end_event(const OEl& el, int64_t key, const PiValue& v) {
    std::vector<std::string> avail;
    int catch_elem = -1;
    int64_t scope = v.flowScopeKey;
    find_error_catch_event(el.error_code, scope, avail, catch_elem);
    if (catch_elem < 0) {
      std::string text = "Expected to throw an error event with the code '" + el.error_code + "', but it was not caught.";
      if (avail.empty()) {
        text += " No error events are available in the scope.";
      } else {
        text += " Available error events are [";
        for (size_t i = 0; i < avail.size(); ++i) text += (i ? ", " : "") + avail[i];
        text += "]";
      }
      const int64_t ik = next_key();
      ORecord& in = append(ZBHIP_RT_EVENT, ZBHIP_VT_INCIDENT, ZBHIP_INCIDENT_CREATED, ik);
      in.r.process_idx = v.proc;
      in.r.element_idx = v.elem;
      in.r.scope_key = key;
      in.r.process_instance_key = v.piKey;
      in.r.partition = ZBHIP_ERR_UNHANDLED_ERROR_EVENT;
      in.r.aux = -1;  // jobKey
      in.r.correlation_key = intern_string(text);
      IncidentRow row;
      row.pi = v;
      row.eik = key;
      row.error_type = ZBHIP_ERR_UNHANDLED_ERROR_EVENT;
      row.message = text;
      incidents_[ik] = row;
      incident_pi_[key] = ik;
      return;
    }
    pi_event(key, ZBHIP_PI_ELEMENT_ACTIVATED, v);
    if (!can_trigger(scope, catch_elem, v.proc)) return;
    const ElementInstance target = ei_.at(scope);
    const int64_t eventKey = next_key();
    ORecord& pe = append(ZBHIP_RT_EVENT, ZBHIP_VT_PROCESS_EVENT, ZBHIP_PE_TRIGGERING, eventKey);
    pe.r.process_idx = target.value.proc;
    pe.r.element_idx = catch_elem;
    pe.r.scope_key = scope;
    pe.r.process_instance_key = target.value.piKey;
    pe.r.aux = -1;
    trigger_event(scope, eventKey, catch_elem, target.value.proc, Doc{}, target.value.piKey);
    if (P(target.value.proc).els[catch_elem].type == ZBHIP_EL_START_EVENT) {
      trigger_event_sub_process(catch_elem, scope);
      return;
    }
    pi_command(scope, ZBHIP_PI_TERMINATE_ELEMENT, target.value);
  }

  // EventTriggerBehavior.triggerEventSubProcess (common/EventTriggerBehavior.java:74-118): discarded when
  // the flow scope is interrupted by another event sub-process or holds no trigger; an interrupting one
  // terminates the flow scope's children (a TERMINATE_ELEMENT each, key order, those that can terminate)
  // and activates the event sub-process once none is active -- at once when there was none, else from
  // the flow scope's onChildTerminated
  void trigger_event_sub_process(int start, int64_t scope) {
    ElementInstance& fs = ei_.at(scope);
    const OEl& st = P(fs.value.proc).els[start];
    if (fs.interrupting_elem >= 0 && fs.interrupting_elem != st.scope) return;
    auto tit = triggers_.lower_bound({scope, INT64_MIN});
    if (tit == triggers_.end() || tit->first.first != scope) return;
    if (st.interrupting) {
      std::vector<int64_t> children;  // unsubscribeEventSubprocesses: error start events hold none
      for (auto it = parent_child_.lower_bound({scope, INT64_MIN}); it != parent_child_.end() && it->first == scope; ++it)
        children.push_back(it->second);
      for (int64_t c : children) {
        const ElementInstance& ci = ei_.at(c);
        if (ci.state == ZBHIP_PI_ELEMENT_ACTIVATING || ci.state == ZBHIP_PI_ELEMENT_ACTIVATED ||
            ci.state == ZBHIP_PI_ELEMENT_COMPLETING)
          pi_command(c, ZBHIP_PI_TERMINATE_ELEMENT, ci.value);
      }
      if (ei_.at(scope).childCount != 0) return;
    }
    activate_event_sub_process(scope);
  }

  // BpmnEventSubscriptionBehavior.activateTriggeredEvent -> EventTriggerBehavior.activateTriggeredEvent
  // (:191-244) for an event sub-process's start event: activateEventSubProcess (:258-264) --
  // ACTIVATE_ELEMENT of the event sub-process as a new command (key -1; the start event's trigger stays
  // for its output mappings: no PROCESS_EVENT:TRIGGERED)
  void activate_event_sub_process(int64_t scope) {
    auto tit = triggers_.lower_bound({scope, INT64_MIN});
    if (tit == triggers_.end() || tit->first.first != scope) return;
    PiValue c = ei_.at(scope).value;
    c.elem = P(c.proc).els[tit->second.elem].scope;
    c.flowScopeKey = scope;
    pi_command(-1, ZBHIP_PI_ACTIVATE_ELEMENT, c);
  }

  // BpmnStateBehavior.isInterrupted (:205-212): no active child, interrupted by an event sub-process, active
  bool esp_interrupted(const ElementInstance& fs) const {
    return fs.childCount == 0 && fs.interrupting_elem >= 0 && fs.state == ZBHIP_PI_ELEMENT_ACTIVATED;
  }

  // BpmnJobActivationBehavior.publishWork (processing/bpmn/behavior/BpmnJobActivationBehavior.java:61-100):
  // with a job stream for the job's type, JOB_BATCH:ACTIVATED (key = nextKey) of that one job -- deadline
  // = now + the stream's timeout, its worker -- applied at once (JobBatchActivatedApplier ->
  // DbJobState.activate); the push itself is a side effect.  No stream: a notification (no record).
  // The record: aux = the job key, the job's fields as a JOB record's (scope_key = its element instance,
  // message_key = the deadline, correlation_key = the worker's string id, a failed job's fields); the
  // batch's timeout is the stream's.
  void publish_work(int64_t jobKey) {
    JobRow& job = jobs_.at(jobKey);
    auto st = streams.find(job.type);
    if (st == streams.end()) {  // notifyJobAvailable (:103-111): JobStreamer.notifyWorkAvailable(type)
      if (track_notified) notified.push_back(job.type);
      return;
    }
    const int64_t key = next_key();
    job.activated = true;
    job.deadline = now_ms + st->second.second;
    job.worker = st->second.first;
    activatable_.erase({job.type, "<default>", jobKey});
    ORecord& rec = append(ZBHIP_RT_EVENT, ZBHIP_VT_JOB_BATCH, ZBHIP_JOB_BATCH_ACTIVATED, key);
    rec.r.process_idx = job.pi.proc;
    rec.r.element_idx = job.pi.elem;
    rec.r.scope_key = job.elementInstanceKey;
    rec.r.process_instance_key = job.pi.piKey;
    rec.r.aux = jobKey;
    job_activation_fields(rec, job);  // the job as activated: deadline, worker (+ a failed job's fields)
  }

  // the stored job's deadline and worker (DbJobState.activate wrote them; a timed-out job keeps
  // them): the zbhip_record fields message_key / correlation_key of a JOB record; a failed job's
  // retries and errorMessage (reason_arg bit 0: partition = retries, message_name | bpmn_process_id
  // << 16 = the errorMessage's string id)
  void job_activation_fields(ORecord& rec, const JobRow& job) {
    if (job.fail_fields) {
      rec.r.reason_arg = 1;
      rec.r.partition = job.retries;
      const uint32_t id = job.error_message.empty() ? ZBHIP_NO_STRING : intern_string(job.error_message);
      rec.r.message_name = (uint16_t)(id & 0xFFFF);
      rec.r.bpmn_process_id = (uint16_t)(id >> 16);
    }
    if (job.deadline == -1 && job.worker.empty()) return;
    rec.r.message_key = job.deadline;
    rec.r.correlation_key = job.worker.empty() ? ZBHIP_NO_STRING : intern_string(job.worker);
  }

  // JobCreatedApplier (state/appliers/JobCreatedApplier.java:28-41) / DbJobState.create
  void apply_job_created(int64_t jobKey, const JobRow& job) {
    jobs_[jobKey] = job;
    activatable_.insert({job.type, "<default>", jobKey});
    auto it = ei_.find(job.elementInstanceKey);
    if (it != ei_.end()) it->second.jobKey = jobKey;
  }

  // JobCompletedApplier (state/appliers/JobCompletedApplier.java:28-45) / DbJobState.delete (:175-188)
  void apply_job_completed(int64_t jobKey, const JobRow& job) {
    jobs_.erase(jobKey);
    activatable_.erase({job.type, "<default>", jobKey});
    auto it = ei_.find(job.elementInstanceKey);
    if (it != ei_.end()) {
      auto fit = ei_.find(it->second.value.flowScopeKey);
      if (fit != ei_.end() && fit->second.state == ZBHIP_PI_ELEMENT_ACTIVATED) it->second.jobKey = -1;
    }
  }

  // JobCanceledApplier (state/appliers/JobCanceledApplier.java:28-30) -> DbJobState.cancel -> delete
  void apply_job_canceled(int64_t jobKey, const JobRow& job) {
    jobs_.erase(jobKey);
    activatable_.erase({job.type, "<default>", jobKey});
  }

  // ActivateProcessInstanceBatchProcessor.processRecord (processing/processinstance/
  // ActivateProcessInstanceBatchProcessor.java:44-60): `index` ACTIVATE_ELEMENT commands of the inner
  // activity, each with a new key, the body's record value with flow scope = the body
  // (createChildInstanceRecord :62-84).  The size-based split into a follow-up batch command
  // (canWriteCommands, ~4 MB batches) never happens at these record sizes.
  void activate_batch(ORecord& cmd) {
    auto it = ei_.find(cmd.r.scope_key);
    if (it == ei_.end()) throw Unsupported{"batch activation without its body instance"};
    PiValue c = it->second.value;
    c.flowScopeKey = it->second.key;
    c.elem = E(it->second.value).inner;
    for (int32_t n = cmd.r.partition; n > 0; --n) pi_command(next_key(), ZBHIP_PI_ACTIVATE_ELEMENT, c);
  }

  // MultiInstanceBodyProcessor.onChildActivating (:129-158) -> setLoopVariables (:270-305): the item at
  // loopCounter - 1 as the inputElement (if any), then loopCounter, local to the inner instance
  // (the outputElement variable, nil-initialized unless it is the inputElement or loopCounter, between them)
  void on_child_activating(const OEl& body, int64_t key, const PiValue& v) {
    const int loop = ei_.at(key).loopCounter;
    const Items items = input_collection(body, key);
    if (loop < 1 || loop > (int)items.size()) throw Unsupported{"loop counter past the input collection (incident)"};
    const auto& item = items[loop - 1];
    if (body.mi_input_id >= 0) set_local_inline(key, v.proc, v.piKey, body.mi_input_id, item.first, item.second);
    if (body.mi_out_elem_id >= 0 && body.mi_out_elem != body.mi_input && body.mi_out_elem != "loopCounter")
      set_local_inline(key, v.proc, v.piKey, body.mi_out_elem_id, ZBHIP_DOC_NIL, 0);
    set_local_inline(key, v.proc, v.piKey, body.mi_loop_id, ZBHIP_DOC_INT, loop);
  }

  // readInputCollectionVariable (MultiInstanceBodyProcessor.java:362-367 -> evaluateArrayExpression):
  // the static list, or the list variable seen from `scope` (anything else is an EXTRACT_VALUE_ERROR
  // incident: outside the subset)
  Items input_collection(const OEl& b, int64_t scope) {
    if (b.mi_coll_id < 0) return b.mi_items;
    const VarRow* vr = lookup_var(scope, b.mi_coll_id);
    if (!vr || vr->type != ZBHIP_DOC_LIST) throw Unsupported{"input collection is not a list (incident)"};
    return lists.at((size_t)vr->value);
  }

  // MultiInstanceBodyProcessor.beforeExecutionPathCompleted (:160-191) of the inner instance `child`:
  // updateOutputCollection (MultiInstanceOutputCollectionBehavior.java:57-141: the outputElement's value
  // at loopCounter - 1 of the body's local collection, setLocalVariable), then the completion condition
  // (satisfiesCompletionCondition :380-394, the numberOf* variables from the body first), then for a
  // sequential body the input collection read again.  Returns whether the condition is satisfied.
  bool mi_before_completed(const OEl& b, ElementInstance& body, int64_t child) {
    if (b.mi_out_coll_id >= 0) {
      const int loop = ei_.at(child).loopCounter;
      const VarRow* ev = lookup_var(child, b.mi_out_elem_id);
      if (!ev) throw Unsupported{"output element variable missing (null: unpinned)"};
      if (ev->type == ZBHIP_DOC_LIST) throw Unsupported{"a list as output element"};
      const uint8_t et = ev->type;
      const int64_t evv = ev->value;
      auto cit = vars_.find({body.key, b.mi_out_coll_id});
      if (cit == vars_.end() || cit->second.type != ZBHIP_DOC_LIST) throw Unsupported{"output collection not a list (incident)"};
      Items items = lists.at((size_t)cit->second.value);
      if (loop < 1 || loop > (int)items.size()) throw Unsupported{"output collection too small (incident)"};
      items[loop - 1] = {et, evv};
      set_local_inline(body.key, body.value.proc, body.value.piKey, b.mi_out_coll_id, ZBHIP_DOC_LIST, intern_list(items));
    }
    bool sat = false;
    if (b.mi_cond) {
      cond_body_ = &body;
      FVal r;
      try {
        r = eval(b.mi_cond.get(), child);
      } catch (...) {
        cond_body_ = nullptr;
        throw;
      }
      cond_body_ = nullptr;
      if (r.k != V_BOOL) throw Unsupported{"completion condition not a boolean (incident)"};
      sat = r.b;
    }
    if (b.mi_seq) (void)input_collection(b, body.key);
    return sat;
  }
  const ElementInstance* cond_body_ = nullptr;  // the body whose completion condition is evaluated

  // TerminateProcessInstanceBatchProcessor.processRecord (processing/processinstance/
  // TerminateProcessInstanceBatchProcessor.java:38-85): TERMINATE_ELEMENT of every child of the body
  // that can terminate (ACTIVATING / ACTIVATED / COMPLETING), in ELEMENT_INSTANCE_PARENT_CHILD order
  void terminate_batch(ORecord& cmd) {
    const int64_t body = cmd.r.scope_key;
    if (cmd.r.partition != -1) throw Unsupported{"a continued termination batch"};
    std::vector<int64_t> kids;
    for (auto it = parent_child_.lower_bound({body, INT64_MIN}); it != parent_child_.end() && it->first == body; ++it)
      kids.push_back(it->second);
    for (int64_t c : kids) {
      const ElementInstance& ci = ei_.at(c);
      if (ci.state == ZBHIP_PI_ELEMENT_ACTIVATING || ci.state == ZBHIP_PI_ELEMENT_ACTIVATED ||
          ci.state == ZBHIP_PI_ELEMENT_COMPLETING)
        pi_command(c, ZBHIP_PI_TERMINATE_ELEMENT, ci.value);
    }
  }

  // VariableBehavior.setLocalVariable (VariableBehavior.java:191-200) of a value the engine computed
  // (not a command document entry): the record carries it inline (zbhip_record.aux = ZBHIP_AUX_INLINE)
  void set_local_inline(int64_t scopeKey, int proc, int64_t piKey, int name, uint8_t type, int64_t value) {
    auto it = vars_.find({scopeKey, name});
    int64_t key;
    int intent;
    if (it == vars_.end()) {
      key = next_key();
      intent = ZBHIP_VAR_CREATED;
    } else if (!(it->second.type == type && it->second.value == value)) {
      key = it->second.key;
      intent = ZBHIP_VAR_UPDATED;
    } else {
      return;
    }
    ORecord& rec = append(ZBHIP_RT_EVENT, ZBHIP_VT_VARIABLE, intent, key);
    rec.r.process_idx = proc;
    rec.r.element_idx = name;
    rec.r.scope_key = scopeKey;
    rec.r.process_instance_key = piKey;
    rec.r.aux = ZBHIP_AUX_INLINE;
    rec.r.message_key = value;
    rec.r.partition = type;
    vars_[{scopeKey, name}] = VarRow{key, type, value, UINT32_MAX};
  }

  // ExpressionProcessor.evaluateVariableMappingExpression of a one-entry mapping context in `scope`
  // (DbVariableState.getVariable walks the scope chain).  FeelToMessagePackTransformer writes a whole
  // number as an integer (FeelToMessagePackTransformer.scala:35-39): a whole decimal becomes an INT.  A
  // missing source variable is outside the subset (feel-scala 1.17's null for it is unpinned here).
  void eval_mapping(const OEl::Mapping& M, int64_t scope, uint8_t& type, int64_t& value) {
    if (!M.var) {
      type = M.type;
      value = M.value;
      return;
    }
    const VarRow* vr = lookup_var(scope, M.source_id);
    if (!vr) throw Unsupported{"io mapping source variable missing"};
    if (vr->type != ZBHIP_DOC_NIL && vr->type != ZBHIP_DOC_BOOL && vr->type != ZBHIP_DOC_INT &&
        vr->type != ZBHIP_DOC_DEC && vr->type != ZBHIP_DOC_STR)
      throw Unsupported{"io mapping source outside the value subset"};
    type = vr->type;
    value = vr->value;
    if (type == ZBHIP_DOC_DEC && value % 1000000 == 0) {
      type = ZBHIP_DOC_INT;
      value /= 1000000;
    }
  }

  // BpmnVariableMappingBehavior.applyInputMappings (behavior/BpmnVariableMappingBehavior.java:53-77):
  // the mapping evaluated in the element's scope, mergeLocalDocument into it
  void apply_input_mappings(const OEl& el, int64_t key, const PiValue& v) {
    if (!el.in_map.present) return;
    uint8_t type;
    int64_t value;
    eval_mapping(el.in_map, key, type, value);
    set_local_inline(key, v.proc, v.piKey, el.in_map.target_id, type, value);
  }

  // VariableBehavior.mergeDocument (VariableBehavior.java:105-150) of a one-entry document computed by
  // the engine: updated in the first scope of the chain that holds it with another value, else set
  // locally in the root scope
  void merge_document_value(int64_t scopeKey, int proc, int64_t piKey, int name, uint8_t type, int64_t value) {
    int64_t current = scopeKey;
    for (;;) {
      auto pit = child_parent_.find(current);
      const int64_t parent = pit == child_parent_.end() ? -1 : pit->second;
      if (parent <= 0) break;
      auto vit = vars_.find({current, name});
      if (vit != vars_.end() && !(vit->second.type == type && vit->second.value == value)) {
        set_local_inline(current, proc, piKey, name, type, value);
        return;
      }
      current = parent;
    }
    set_local_inline(current, proc, piKey, name, type, value);
  }

  // ---------------------------------------------------------------------
  // BpmnStreamProcessor.processRecord (processing/bpmn/BpmnStreamProcessor.java:74-162)
  // ---------------------------------------------------------------------
  void bpmn_process_record(ORecord& cmd) {
    std::string violation;
    if (!check_state_transition(cmd, violation)) {
      reject(cmd, ZBHIP_REJ_INVALID_STATE, violation);
      return;
    }
    const OEl& el = E(cmd.pi);
    if (cmd.r.intent == ZBHIP_PI_ACTIVATE_ELEMENT) {
      // BpmnStateTransitionBehavior.transitionToActivating (behavior/BpmnStateTransitionBehavior.java:72-100)
      if (ei_.count(cmd.r.key)) throw Unsupported{"re-activation (incident resolution)"};
      int64_t key = cmd.r.key == -1 ? next_key() : cmd.r.key;
      pi_event(key, ZBHIP_PI_ELEMENT_ACTIVATING, cmd.pi);
      // onElementActivating -> container.onChildActivating: ProcessProcessor / SubProcessProcessor
      // default (right); a multi-instance body sets the inner instance's loop variables
      if (el.scope > 0 && P(cmd.pi.proc).els[el.scope].type == ZBHIP_EL_MULTI_INSTANCE_BODY)
        on_child_activating(P(cmd.pi.proc).els[el.scope], key, cmd.pi);
      on_activate(el, key, cmd.pi);
    } else if (cmd.r.intent == ZBHIP_PI_COMPLETE_ELEMENT) {
      // transitionToCompleting (:116-130)
      if (ei_.at(cmd.r.key).state == ZBHIP_PI_ELEMENT_COMPLETING) throw Unsupported{"re-completion (incident resolution)"};
      pi_event(cmd.r.key, ZBHIP_PI_ELEMENT_COMPLETING, cmd.pi);
      on_complete(el, cmd.r.key, cmd.pi);
    } else {
      // TERMINATE_ELEMENT: transitionToTerminating, then the processor's onTerminate (:151-154)
      pi_event(cmd.r.key, ZBHIP_PI_ELEMENT_TERMINATING, cmd.pi);
      on_terminate(el, cmd.r.key, cmd.pi);
    }
  }

  // ProcessInstanceStateTransitionGuard.checkStateTransition (processing/bpmn/ProcessInstanceStateTransitionGuard.java:47-186)
  static const char* state_name(int s) {
    switch (s) {
      case ZBHIP_PI_ELEMENT_ACTIVATING: return "ELEMENT_ACTIVATING";
      case ZBHIP_PI_ELEMENT_ACTIVATED: return "ELEMENT_ACTIVATED";
      case ZBHIP_PI_ELEMENT_COMPLETING: return "ELEMENT_COMPLETING";
      case ZBHIP_PI_ELEMENT_COMPLETED: return "ELEMENT_COMPLETED";
      case ZBHIP_PI_ELEMENT_TERMINATING: return "ELEMENT_TERMINATING";
      case ZBHIP_PI_ELEMENT_TERMINATED: return "ELEMENT_TERMINATED";
      default: return "?";
    }
  }

  bool has_active_flow_scope(const ORecord& cmd, std::string& v) {
    const OEl& el = E(cmd.pi);
    if (el.type == ZBHIP_EL_PROCESS) return true;
    auto it = ei_.find(cmd.pi.flowScopeKey);
    if (it == ei_.end()) {
      v = "Expected flow scope instance with key '" + std::to_string(cmd.pi.flowScopeKey) +
          "' to be present in state but not found.";
      return false;
    }
    if (it->second.state != ZBHIP_PI_ELEMENT_ACTIVATED) {
      v = std::string("Expected flow scope instance to be in state 'ELEMENT_ACTIVATED' but was '") +
          state_name(it->second.state) + "'.";
      return false;
    }
    // hasNonInterruptedFlowScope (:160-174): only the interrupting event sub-process itself
    const int ie = it->second.interrupting_elem;
    if (ie >= 0 && ie != cmd.pi.elem) {
      v = "Expected flow scope instance to be not interrupted but was interrupted by an event with id '" +
          P(cmd.pi.proc).els[ie].id + "'.";
      return false;
    }
    return true;
  }

  bool check_state_transition(const ORecord& cmd, std::string& v) {
    if (cmd.r.intent == ZBHIP_PI_ACTIVATE_ELEMENT) {
      if (!has_active_flow_scope(cmd, v)) return false;
      const OEl& el = E(cmd.pi);
      if (el.type == ZBHIP_EL_PARALLEL_GATEWAY) {  // canActivateParallelGateway (:169-186)
        int taken = number_of_taken_flows(cmd.pi.flowScopeKey, cmd.pi.proc, cmd.pi.elem);
        if (taken < (int)el.in.size()) {
          v = "Expected to be able to activate parallel gateway '" + el.id +
              "', but not all sequence flows have been taken.";
          return false;
        }
      }
      return true;
    }
    if (cmd.r.intent == ZBHIP_PI_COMPLETE_ELEMENT) {
      auto it = ei_.find(cmd.r.key);
      if (it == ei_.end()) {
        v = "Expected element instance with key '" + std::to_string(cmd.r.key) +
            "' to be present in state but not found.";
        return false;
      }
      int s = it->second.state;
      if (s != ZBHIP_PI_ELEMENT_ACTIVATED && s != ZBHIP_PI_ELEMENT_COMPLETING) {
        v = std::string("Expected element instance to be in state 'ELEMENT_ACTIVATED' or one of "
                        "'[ELEMENT_COMPLETING]' but was '") + state_name(s) + "'.";
        return false;
      }
      return has_active_flow_scope(cmd, v);
    }
    if (cmd.r.intent == ZBHIP_PI_TERMINATE_ELEMENT) {  // hasElementInstanceWithState (:60-64)
      auto it = ei_.find(cmd.r.key);
      if (it == ei_.end()) {
        v = "Expected element instance with key '" + std::to_string(cmd.r.key) +
            "' to be present in state but not found.";
        return false;
      }
      int s = it->second.state;
      if (s != ZBHIP_PI_ELEMENT_ACTIVATING && s != ZBHIP_PI_ELEMENT_ACTIVATED && s != ZBHIP_PI_ELEMENT_COMPLETING) {
        v = std::string("Expected element instance to be in state 'ELEMENT_ACTIVATING' or one of "
                        "'[ELEMENT_ACTIVATED, ELEMENT_COMPLETING]' but was '") + state_name(s) + "'.";
        return false;
      }
      return true;
    }
    throw Unsupported{"intent"};
  }

  // DbElementInstanceState.getNumberOfTakenSequenceFlows (state/instance/DbElementInstanceState.java:330-344):
  // counts DISTINCT flows with a counter row under (flowScopeKey, gatewayId)
  int number_of_taken_flows(int64_t fs, int proc, int gw) {
    int n = 0;
    for (auto it = taken_.lower_bound({fs, gw, -1}); it != taken_.end(); ++it) {
      if (std::get<0>(it->first) != fs || std::get<1>(it->first) != gw) break;
      ++n;
    }
    (void)proc;
    return n;
  }

  // ---------------------------------------------------------------------
  // element processors: onActivate / onComplete
  // ---------------------------------------------------------------------
  void on_activate(const OEl& el, int64_t key, const PiValue& v) {
    switch (el.type) {
      case ZBHIP_EL_PROCESS: {  // ProcessProcessor.onActivate (processing/bpmn/container/ProcessProcessor.java:55-61,119-128)
        pi_event(key, ZBHIP_PI_ELEMENT_ACTIVATED, v);
        const OProc& p = P(v.proc);
        if (!p.msg_starts.empty()) {
          // activateStartEvent (:98-114): the process definition's first event trigger, if it is this
          // instance's, activates its start event (BpmnEventSubscriptionBehavior.activateTriggeredStartEvent)
          auto tit = triggers_.lower_bound({p.def_key, INT64_MIN});
          if (tit != triggers_.end() && tit->first.first == p.def_key &&
              (tit->second.piKey == v.piKey || tit->second.piKey == -1)) {
            activate_triggered_event(tit->first.second, tit->second.elem, p.def_key, key, v);
            break;
          }
        }
        if (p.none_start < 0) throw Unsupported{"process without a none start event activated without a trigger"};
        PiValue c = v;  // activateChildInstance (BpmnStateTransitionBehavior.java:279-290)
        c.flowScopeKey = key;
        c.elem = p.none_start;
        pi_command(-1, ZBHIP_PI_ACTIVATE_ELEMENT, c);
        break;
      }
      case ZBHIP_EL_EVENT_SUB_PROCESS:  // EventSubProcessProcessor.onActivate (container/EventSubProcessProcessor.java:41-54)
      case ZBHIP_EL_SUB_PROCESS: {  // SubProcessProcessor.onActivate (processing/bpmn/container/SubProcessProcessor.java:49-66)
        // applyInputMappings, transitionToActivated, activateChildInstance(none start)
        apply_input_mappings(el, key, v);
        pi_event(key, ZBHIP_PI_ELEMENT_ACTIVATED, v);
        PiValue c = v;
        c.flowScopeKey = key;
        c.elem = el.start;
        pi_command(-1, ZBHIP_PI_ACTIVATE_ELEMENT, c);
        break;
      }
      case ZBHIP_EL_MULTI_INSTANCE_BODY: {
        // MultiInstanceBodyProcessor.onActivate (processing/bpmn/container/MultiInstanceBodyProcessor.java:83-98):
        // the static inputCollection always evaluates, no event subscriptions; activate (:229-252):
        // ACTIVATED, then an empty collection completes the body, a sequential body activates its
        // first inner instance (activateChildInstanceWithKey, BpmnStateTransitionBehavior.java:292-307),
        // a parallel one writes PROCESS_INSTANCE_BATCH:ACTIVATE (activateChildInstancesInBatches :315-324)
        const Items items = input_collection(el, key);
        pi_event(key, ZBHIP_PI_ELEMENT_ACTIVATED, v);
        if (el.mi_out_coll_id >= 0)  // initializeOutputCollection (:43-55): [nil] * size, local to the body
          set_local_inline(key, v.proc, v.piKey, el.mi_out_coll_id, ZBHIP_DOC_LIST,
                           intern_list(Items(items.size(), {(uint8_t)ZBHIP_DOC_NIL, 0})));
        if (items.empty()) {
          pi_command(key, ZBHIP_PI_COMPLETE_ELEMENT, v);
          break;
        }
        PiValue c = v;
        c.flowScopeKey = key;
        c.elem = el.inner;
        if (el.mi_seq) {
          pi_command(next_key(), ZBHIP_PI_ACTIVATE_ELEMENT, c);
        } else {
          const int64_t bk = next_key();
          ORecord& rec = append(ZBHIP_RT_COMMAND, ZBHIP_VT_PROCESS_INSTANCE_BATCH, ZBHIP_PIB_ACTIVATE, bk);
          rec.r.process_idx = v.proc;
          rec.r.element_idx = v.elem;
          rec.r.scope_key = key;  // batchElementInstanceKey
          rec.r.process_instance_key = v.piKey;
          rec.r.partition = (int32_t)items.size();  // index: the children to activate
          rec.pi = v;
        }
        break;
      }
      case ZBHIP_EL_START_EVENT:  // StartEventProcessor.onActivate (processing/bpmn/event/StartEventProcessor.java:45-50)
      case ZBHIP_EL_TASK:         // UndefinedTaskProcessor.onActivate (processing/bpmn/task/UndefinedTaskProcessor.java:37-42)
      case ZBHIP_EL_MANUAL_TASK:  // ManualTaskProcessor extends UndefinedTaskProcessor
      case ZBHIP_EL_INTERMEDIATE_THROW_EVENT:  // NoneIntermediateThrowEventBehavior.onActivate (:120-126)
        pi_event(key, ZBHIP_PI_ELEMENT_ACTIVATED, v);
        pi_command(key, ZBHIP_PI_COMPLETE_ELEMENT, v);
        break;
      case ZBHIP_EL_END_EVENT:  // EndEventProcessor.NoneEndEventBehavior.onActivate (processing/bpmn/event/EndEventProcessor.java:110-134)
        if (el.event == ZBHIP_EV_ERROR) {
          throw_error_end_event(el, key, v);
          break;
        }
        pi_event(key, ZBHIP_PI_ELEMENT_ACTIVATED, v);
        pi_event(key, ZBHIP_PI_ELEMENT_COMPLETING, v);
        complete_and_take(el, key, v, /*output_mappings=*/true);
        break;
      case ZBHIP_EL_SERVICE_TASK:  // JobWorkerTaskProcessor.onActivate (processing/bpmn/task/JobWorkerTaskProcessor.java:49-61)
      case ZBHIP_EL_SEND_TASK:
      case ZBHIP_EL_SCRIPT_TASK:
      case ZBHIP_EL_BUSINESS_RULE_TASK: {
        // applyInputMappings, then eventSubscriptionBehavior.subscribeToEvents: the attached boundary
        // event's message subscription or timer, then the job
        apply_input_mappings(el, key, v);
        if (el.boundary >= 0) {
          PiValue bv = v;
          bv.elem = el.boundary;
          const OEl& b = P(v.proc).els[el.boundary];
          if (b.event == ZBHIP_EV_MESSAGE) {
            if (!subscribe_to_message(b, key, bv, v.flowScopeKey, key, v)) break;  // incident on the task
          } else if (b.event == ZBHIP_EV_TIMER) {
            subscribe_to_timer(b, key, bv);
          }  // (an error boundary event subscribes to nothing: JOB:THROW_ERROR looks it up)
        }
        // BpmnJobBehavior.createNewJob -> writeJobCreatedEvent (behavior/BpmnJobBehavior.java:113-119,194-218)
        JobRow job;
        job.pi = v;
        job.elementInstanceKey = key;
        job.type = el.job_type;
        job.retries = el.retries;
        int64_t jobKey = next_key();
        ORecord& rec = append(ZBHIP_RT_EVENT, ZBHIP_VT_JOB, ZBHIP_JOB_CREATED, jobKey);
        rec.r.process_idx = v.proc;
        rec.r.element_idx = v.elem;
        rec.r.scope_key = key;
        rec.r.process_instance_key = v.piKey;
        apply_job_created(jobKey, job);
        publish_work(jobKey);
        pi_event(key, ZBHIP_PI_ELEMENT_ACTIVATED, v);
        break;
      }
      case ZBHIP_EL_EXCLUSIVE_GATEWAY: {  // ExclusiveGatewayProcessor.onActivate (processing/bpmn/gateway/ExclusiveGatewayProcessor.java:47-66)
        FlowFailure fail;
        int flow = find_sequence_flow_to_take(el, key, v.proc, fail);
        if (flow == -2) {  // incidentBehavior.createIncident(failure, activating)
          create_incident(fail, key, v);
          break;
        }
        pi_event(key, ZBHIP_PI_ELEMENT_ACTIVATED, v);
        pi_event(key, ZBHIP_PI_ELEMENT_COMPLETING, v);
        transition_to_completed(el, key, v);
        if (flow >= 0) take_sequence_flow(key, v, flow);
        break;
      }
      case ZBHIP_EL_INTERMEDIATE_CATCH_EVENT:
        // IntermediateCatchEventProcessor.DefaultIntermediateCatchEventBehavior.onActivate
        // (processing/bpmn/event/IntermediateCatchEventProcessor.java): subscribeToEvents, then ACTIVATED
        if (el.event == ZBHIP_EV_TIMER) subscribe_to_timer(el, key, v);
        else if (!subscribe_to_message(el, key, v, key, key, v)) break;  // incident: stays ACTIVATING
        pi_event(key, ZBHIP_PI_ELEMENT_ACTIVATED, v);
        break;
      case ZBHIP_EL_PARALLEL_GATEWAY:  // ParallelGatewayProcessor.onActivate (processing/bpmn/gateway/ParallelGatewayProcessor.java:34-50)
        pi_event(key, ZBHIP_PI_ELEMENT_ACTIVATED, v);
        pi_event(key, ZBHIP_PI_ELEMENT_COMPLETING, v);
        transition_to_completed(el, key, v);
        for (int f : el.out) take_sequence_flow(key, v, f);
        break;
      default:
        throw Unsupported{"element type"};
    }
  }

  void on_complete(const OEl& el, int64_t key, const PiValue& v) {
    switch (el.type) {
      case ZBHIP_EL_PROCESS: {  // ProcessProcessor.onComplete (:63-76): never end of path
        // getPostTransitionAction (:186-206): the correlation key read before the transition (the
        // applier releases the lock), the next buffered message correlated after it
        auto cit = P(v.proc).msg_starts.empty() ? pi_corr_keys_.end() : pi_corr_keys_.find(v.piKey);
        const bool by_message = cit != pi_corr_keys_.end();
        const uint32_t corr = by_message ? cit->second : ZBHIP_NO_STRING;
        pi_event(key, ZBHIP_PI_ELEMENT_COMPLETED, v);
        if (by_message) correlate_buffered_start_message(v.proc, corr);
        break;
      }
      case ZBHIP_EL_START_EVENT:  // StartEventProcessor.onComplete (:52-67): applyOutputMappings,
        // subscribeToEvents of the flow scope (a sub-process's boundary timer), transitionToCompleted
        complete_and_take(el, key, v, true, false, /*subscribe_scope=*/true);
        break;
      case ZBHIP_EL_SUB_PROCESS:  // SubProcessProcessor.onComplete (:68-82): applyOutputMappings,
        // unsubscribeFromEvents (its boundary timer: TIMER:CANCELED), transitionToCompleted, take flows
        complete_and_take(el, key, v, true, /*unsubscribe=*/true);
        break;
      case ZBHIP_EL_EVENT_SUB_PROCESS:  // EventSubProcessProcessor.onComplete (:58-66): applyOutputMappings,
        // transitionToCompleted (no outgoing flows: the flow scope's afterExecutionPathCompleted)
        complete_and_take(el, key, v, true);
        break;
      case ZBHIP_EL_SERVICE_TASK:  // JobWorkerTaskProcessor.onComplete (:63-75)
      case ZBHIP_EL_SEND_TASK:
      case ZBHIP_EL_SCRIPT_TASK:
      case ZBHIP_EL_BUSINESS_RULE_TASK:
        // applyOutputMappings, unsubscribeFromEvents (the boundary event's timer: TIMER:CANCELED),
        // transitionToCompleted, takeOutgoingSequenceFlows
        complete_and_take(el, key, v, true, /*unsubscribe=*/true);
        break;
      case ZBHIP_EL_BOUNDARY_EVENT:  // BoundaryEventProcessor.onComplete (processing/bpmn/event/BoundaryEventProcessor.java:47-56)
      case ZBHIP_EL_INTERMEDIATE_THROW_EVENT:  // NoneIntermediateThrowEventBehavior.onComplete (:128-137)
        complete_and_take(el, key, v, true);
        break;
      case ZBHIP_EL_TASK:  // UndefinedTaskProcessor.onComplete (:44-51): no output mappings
      case ZBHIP_EL_MANUAL_TASK:
        complete_and_take(el, key, v, false);
        break;
      case ZBHIP_EL_MULTI_INSTANCE_BODY:
        // MultiInstanceBodyProcessor.onComplete (:100-114): unsubscribeFromEvents (none), the output
        // collection propagated (BpmnStateBehavior.propagateVariable :163-178: the variable seen from the
        // body merged into its flow scope), transitionToCompleted, takeOutgoingSequenceFlows
        if (el.mi_out_coll_id >= 0) {
          const VarRow* vr = lookup_var(key, el.mi_out_coll_id);
          if (vr) {
            const uint8_t t = vr->type;
            const int64_t val = vr->value;
            merge_document_value(v.flowScopeKey, v.proc, v.piKey, el.mi_out_coll_id, t, val);
          }
        }
        complete_and_take(el, key, v, false);
        break;
      case ZBHIP_EL_INTERMEDIATE_CATCH_EVENT: {
        // IntermediateCatchEventProcessor.onComplete: applyOutputMappings, unsubscribeFromEvents
        // (CatchEventBehavior.unsubscribeFromMessageEvents visits the element's remaining process
        // message subscriptions: none after an interrupting correlation), transitionToCompleted
        auto pit = pms_.lower_bound({key, INT32_MIN});
        if (pit != pms_.end() && pit->first.first == key)
          throw Unsupported{"unsubscribe (PROCESS_MESSAGE_SUBSCRIPTION:DELETING)"};
        auto tit = timers_.lower_bound({key, INT64_MIN});  // unsubscribeFromTimerEvents: TIMER:CANCELED
        if (tit != timers_.end() && tit->first.first == key) throw Unsupported{"unsubscribe (TIMER:CANCEL)"};
        complete_and_take(el, key, v, true);
        break;
      }
      default:
        throw Unsupported{"complete of element without wait state"};
    }
  }

  // JobWorkerTaskProcessor.onTerminate (processing/bpmn/task/JobWorkerTaskProcessor.java:77-104)
  // the processors' onTerminate (processing/bpmn/**: JobWorkerTaskProcessor :77-104, IntermediateCatch
  // EventProcessor, SubProcessProcessor :84-95): job workers cancel their job, catch events and
  // containers unsubscribe; a container terminates its children first (terminateChildInstances,
  // BpmnStateTransitionBehavior.java:348-363: PROCESS_INSTANCE_BATCH:TERMINATE) and finishes in
  // onChildTerminated once none is active
  void on_terminate(const OEl& el, int64_t key, const PiValue& v) {
    if (el.type == ZBHIP_EL_MULTI_INSTANCE_BODY) {
      // MultiInstanceBodyProcessor.onTerminate (:116-125): unsubscribeFromEvents, terminateChildInstances,
      // terminate at once when no inner instance is active
      unsubscribe_timers(key);
      unsubscribe_messages(key);
      if (ei_.at(key).childCount == 0) {
        mi_terminate(key);
      } else {
        ORecord& rec = append(ZBHIP_RT_COMMAND, ZBHIP_VT_PROCESS_INSTANCE_BATCH, ZBHIP_PIB_TERMINATE, next_key());
        rec.r.process_idx = v.proc;
        rec.r.element_idx = v.elem;
        rec.r.scope_key = key;  // batchElementInstanceKey
        rec.r.process_instance_key = v.piKey;
        rec.r.partition = -1;
        rec.pi = v;
      }
      return;
    }
    if (el.type == ZBHIP_EL_SUB_PROCESS || el.type == ZBHIP_EL_EVENT_SUB_PROCESS) {
      // (EventSubProcessProcessor.onTerminate :68-77: terminateChildInstances, no subscriptions)
      unsubscribe_timers(key);  // unsubscribeFromEvents
      unsubscribe_messages(key);
      const ElementInstance& sub = ei_.at(key);
      if (sub.childCount == 0) {
        container_child_terminated(key);
      } else {
        ORecord& rec = append(ZBHIP_RT_COMMAND, ZBHIP_VT_PROCESS_INSTANCE_BATCH, ZBHIP_PIB_TERMINATE, next_key());
        rec.r.process_idx = v.proc;
        rec.r.element_idx = v.elem;
        rec.r.scope_key = key;  // batchElementInstanceKey
        rec.r.process_instance_key = v.piKey;
        rec.r.partition = -1;   // index: from the first child
        rec.pi = v;
      }
      return;
    }
    if (el.type == ZBHIP_EL_END_EVENT) {
      // EndEventProcessor.onTerminate (:92-101): an error end event that threw (ACTIVATED) -- resolveIncidents
      // (none: an uncaught one stays ACTIVATING with its incident, outside this restatement),
      // transitionToTerminated, onElementTerminated
      if (incident_pi_.count(key)) throw Unsupported{"terminating an end event with an incident"};
      pi_event(key, ZBHIP_PI_ELEMENT_TERMINATED, v);
      child_terminated(v);
      return;
    }
    if (el.type == ZBHIP_EL_INTERMEDIATE_CATCH_EVENT) {
      // IntermediateCatchEventProcessor.onTerminate: unsubscribeFromEvents, resolveIncidents (none),
      // transitionToTerminated, onElementTerminated
      unsubscribe_timers(key);
      unsubscribe_messages(key);
      pi_event(key, ZBHIP_PI_ELEMENT_TERMINATED, v);
      child_terminated(v);
      return;
    }
    if (!ZBHIP_IS_JOB_WORKER(el.type)) throw Unsupported{"terminate of an element outside the subset"};
    // jobBehavior.cancelJob (behavior/BpmnJobBehavior.java:251-274): JOB:CANCELED with the stored job
    const int64_t jobKey = ei_.at(key).jobKey;
    auto jit = jobKey > 0 ? jobs_.find(jobKey) : jobs_.end();
    if (jit != jobs_.end()) {
      const JobRow job = jit->second;
      ORecord& rec = append(ZBHIP_RT_EVENT, ZBHIP_VT_JOB, ZBHIP_JOB_CANCELED, jobKey);
      rec.r.process_idx = job.pi.proc;
      rec.r.element_idx = job.pi.elem;
      rec.r.scope_key = job.elementInstanceKey;
      rec.r.process_instance_key = job.pi.piKey;
      job_activation_fields(rec, job);
      apply_job_canceled(jobKey, job);
    }
    unsubscribe_timers(key);  // unsubscribeFromEvents: timers, then message subscriptions
    unsubscribe_messages(key);
    // findEventTrigger (BpmnEventSubscriptionBehavior.java:63-70): the scope's first trigger, unless
    // it is the element's own -- taken only while the flow scope is active and not interrupted
    auto tit = triggers_.lower_bound({key, INT64_MIN});
    const bool found = tit != triggers_.end() && tit->first.first == key && tit->second.elem != v.elem;
    auto fit = ei_.find(v.flowScopeKey);
    const bool fs_active = v.flowScopeKey == v.piKey ? fit != ei_.end() && fit->second.state == ZBHIP_PI_ELEMENT_ACTIVATED
                                                      : fit != ei_.end() && fit->second.state == ZBHIP_PI_ELEMENT_ACTIVATED;
    if (found && fs_active && !es_interrupted_.count(v.flowScopeKey)) {
      const int64_t eventKey = tit->first.second;
      const int target = tit->second.elem;
      const Doc vars = tit->second.vars;  // (the event trigger read before the scope's removal)
      pi_event(key, ZBHIP_PI_ELEMENT_TERMINATED, v);  // transitionToTerminated
      activate_triggered_event(eventKey, target, key, v.flowScopeKey, v, &vars);
      return;
    }
    // no event trigger: transitionToTerminated, onElementTerminated
    pi_event(key, ZBHIP_PI_ELEMENT_TERMINATED, v);
    child_terminated(v);
  }

  // BpmnStateTransitionBehavior.onElementTerminated (:419-441): the flow scope's onChildTerminated --
  // a multi-instance body (MultiInstanceBodyProcessor.onChildTerminated :232-247: one that is not
  // terminating completes once no child is active: its completion condition was met), a sub-process
  // (SubProcessProcessor.onChildTerminated :108-160)
  void child_terminated(const PiValue& child) {
    auto fit = ei_.find(child.flowScopeKey);
    if (fit == ei_.end()) throw Unsupported{"terminated child without its flow scope"};
    const OEl& fe = E(fit->second.value);
    if (fe.type == ZBHIP_EL_MULTI_INSTANCE_BODY) {
      const ElementInstance& body = fit->second;
      if (body.state == ZBHIP_PI_ELEMENT_TERMINATING) {
        // (:244-246) canBeTerminated: no inner instance is active
        if (body.childCount == 0) mi_terminate(body.key);
        return;
      }
      if ((int64_t)body.childCount + body.activeSequenceFlows == 0)
        pi_command(body.key, ZBHIP_PI_COMPLETE_ELEMENT, body.value);
      return;
    }
    if (fe.type == ZBHIP_EL_SUB_PROCESS || fe.type == ZBHIP_EL_EVENT_SUB_PROCESS) {
      // canBeTerminated(child): no active child of the sub-process is left
      if (fit->second.childCount == 0) container_child_terminated(fit->first);
      return;
    }
    // ProcessProcessor.onChildTerminated (:143-180): interrupted by an event sub-process, its trigger
    // activates it; an active process with an active child left (the boundary event a terminated
    // multi-instance body's trigger activated) does nothing
    if (esp_interrupted(fit->second)) {
      activate_event_sub_process(fit->first);
      return;
    }
    if (fit->second.state == ZBHIP_PI_ELEMENT_ACTIVATED && fit->second.childCount > 0) return;
    throw Unsupported{"terminated child of the process (cancel)"};
  }

  // MultiInstanceBodyProcessor.terminate (:282-315): resolveIncidents (none), then with the body's
  // boundary event trigger (its flow scope active and not interrupted) transitionToTerminated,
  // activateTriggeredEvent and onElementTerminated; otherwise transitionToTerminated and
  // onElementTerminated
  void mi_terminate(int64_t key) {
    const ElementInstance body = ei_.at(key);
    const PiValue v = body.value;
    auto tit = triggers_.lower_bound({key, INT64_MIN});
    const bool found = tit != triggers_.end() && tit->first.first == key;
    auto fit = ei_.find(v.flowScopeKey);
    const bool fs_active = fit != ei_.end() && fit->second.state == ZBHIP_PI_ELEMENT_ACTIVATED;
    // (the trigger read before the TERMINATED applier removes the event scope)
    const Doc vars = found ? tit->second.vars : Doc();
    const int64_t eventKey = found ? tit->first.second : -1;
    const int target = found ? tit->second.elem : -1;
    pi_event(key, ZBHIP_PI_ELEMENT_TERMINATED, v);
    if (found && fs_active && !es_interrupted_.count(v.flowScopeKey))
      activate_triggered_event(eventKey, target, key, v.flowScopeKey, v, &vars);
    child_terminated(v);
  }

  // SubProcessProcessor.onChildTerminated (:108-160) with no active child left: its boundary event's
  // trigger (the flow scope active and not interrupted) -> transitionToTerminated and
  // activateTriggeredEvent; else, terminated by its own flow scope -> transitionToTerminated and
  // onElementTerminated
  void container_child_terminated(int64_t key) {
    const ElementInstance sub = ei_.at(key);
    const PiValue v = sub.value;
    if (esp_interrupted(sub)) {  // an interrupting event sub-process was triggered (SubProcessProcessor :114-125)
      activate_event_sub_process(key);
      return;
    }
    auto tit = triggers_.lower_bound({key, INT64_MIN});
    const bool found = tit != triggers_.end() && tit->first.first == key;
    auto fit = ei_.find(v.flowScopeKey);
    const bool fs_active = fit != ei_.end() && fit->second.state == ZBHIP_PI_ELEMENT_ACTIVATED;
    if (found && fs_active && !es_interrupted_.count(v.flowScopeKey)) {
      const int64_t eventKey = tit->first.second;
      const int target = tit->second.elem;
      const Doc vars = tit->second.vars;  // (an error's variables: local to the boundary event)
      pi_event(key, ZBHIP_PI_ELEMENT_TERMINATED, v);
      activate_triggered_event(eventKey, target, key, v.flowScopeKey, v, &vars);
      return;
    }
    if (sub.state == ZBHIP_PI_ELEMENT_TERMINATING) {
      pi_event(key, ZBHIP_PI_ELEMENT_TERMINATED, v);
      child_terminated(v);
    }
  }

  // EventTriggerBehavior.activateTriggeredEvent (processing/common/EventTriggerBehavior.java:191-244):
  // PROCESS_EVENT:TRIGGERED (the trigger's key), ACTIVATING + ACTIVATED of the triggered event
  // (+key, flow scope = the given one), COMPLETE_ELEMENT
  void activate_triggered_event(int64_t eventKey, int target, int64_t scope, int64_t flowScopeKey, const PiValue& v,
                                const Doc* trigger_vars = nullptr) {
    ORecord& pe = append(ZBHIP_RT_EVENT, ZBHIP_VT_PROCESS_EVENT, ZBHIP_PE_TRIGGERED, eventKey);
    pe.r.process_idx = v.proc;
    pe.r.element_idx = target;
    pe.r.scope_key = scope;
    pe.r.process_instance_key = v.piKey;
    pe.r.aux = -1;
    auto tr = triggers_.find({scope, eventKey});
    const Doc vars = trigger_vars ? *trigger_vars : tr != triggers_.end() ? tr->second.vars : Doc{0, 0};
    triggers_.erase({scope, eventKey});  // ProcessEventTriggeredApplier: deleteTrigger (if it exists)
    PiValue bv = v;
    bv.elem = target;
    bv.flowScopeKey = flowScopeKey;
    const int64_t bk = next_key();
    pi_event(bk, ZBHIP_PI_ELEMENT_ACTIVATING, bv);
    pi_event(bk, ZBHIP_PI_ELEMENT_ACTIVATED, bv);
    // the event's variables become local variables of the event instance (for its output mappings)
    if (vars.count > 0) merge_local_document(bk, v.proc, v.piKey, vars);
    pi_command(bk, ZBHIP_PI_COMPLETE_ELEMENT, bv);
  }

  // applyOutputMappings (behavior/BpmnVariableMappingBehavior.java:86-156) ->
  // transitionToCompleted -> takeOutgoingSequenceFlows (BpmnStateTransitionBehavior.java:365-369)
  void complete_and_take(const OEl& el, int64_t key, const PiValue& v, bool output_mappings, bool unsubscribe = false,
                         bool subscribe_scope = false) {
    if (output_mappings) {
      const EventTrigger* trig = nullptr;  // peekEventTrigger(elementInstanceKey)
      auto it = triggers_.lower_bound({key, INT64_MIN});
      if (it != triggers_.end() && it->first.first == key) trig = &it->second;
      if (el.out_map.present) {
        // the event's variables become local, then the mapping is evaluated in the element's scope
        // and merged into its flow scope (getVariableScopeKey; no multi-instance inner activities)
        if (trig && trig->vars.count > 0) merge_local_document(key, v.proc, v.piKey, trig->vars);
        uint8_t type;
        int64_t value;
        eval_mapping(el.out_map, key, type, value);
        merge_document_value(v.flowScopeKey, v.proc, v.piKey, el.out_map.target_id, type, value);
      } else if (trig && trig->vars.count > 0) {
        merge_document(key, v.proc, v.piKey, trig->vars);
      }
      // START_EVENT without trigger: local variables of the start event are empty.
    }
    if (unsubscribe) {  // unsubscribeFromEvents (CatchEventBehavior.java:126-138): timers, then messages
      unsubscribe_timers(key);
      unsubscribe_messages(key);
    }
    if (subscribe_scope) {  // a start event: subscribeToEvents(flowScope) -- the sub-process's boundary timer
      auto fit = ei_.find(v.flowScopeKey);
      if (fit != ei_.end()) {
        const OEl& fe = E(fit->second.value);
        if (fe.type == ZBHIP_EL_SUB_PROCESS && fe.boundary >= 0 &&
            P(fit->second.value.proc).els[fe.boundary].event == ZBHIP_EV_TIMER) {
          PiValue bv = fit->second.value;
          bv.elem = fe.boundary;
          subscribe_to_timer(P(bv.proc).els[fe.boundary], fit->first, bv);
        }
      }
    }
    transition_to_completed(el, key, v);
    for (int f : el.out) take_sequence_flow(key, v, f);
  }

  // BpmnStateTransitionBehavior.transitionToCompleted (:158-191) and afterExecutionPathCompleted (:404-417)
  void transition_to_completed(const OEl& el, int64_t key, const PiValue& v) {
    bool end_of_path = el.type != ZBHIP_EL_PROCESS && el.out.empty();
    // beforeExecutionPathCompleted (BpmnStateTransitionBehavior.java:158-191): the container's check
    // before the COMPLETED record (a multi-instance body: output collection, completion condition)
    bool satisfies = false;
    if (end_of_path) {
      auto bit = ei_.find(v.flowScopeKey);
      if (bit != ei_.end() && E(bit->second.value).type == ZBHIP_EL_MULTI_INSTANCE_BODY)
        satisfies = mi_before_completed(E(bit->second.value), bit->second, key);
    }
    pi_event(key, ZBHIP_PI_ELEMENT_COMPLETED, v);
    if (end_of_path) {
      // ProcessProcessor.afterExecutionPathCompleted (:130-140) -> BpmnStateBehavior.canBeCompleted (behavior/BpmnStateBehavior.java:76-95)
      auto fit = ei_.find(v.flowScopeKey);
      if (fit != ei_.end() && E(fit->second.value).type == ZBHIP_EL_MULTI_INSTANCE_BODY) {
        // MultiInstanceBodyProcessor.afterExecutionPathCompleted (:193-230): a satisfied completion
        // condition terminates the remaining children (terminateChildInstances, BpmnStateTransitionBehavior
        // .java:348-363: PROCESS_INSTANCE_BATCH:TERMINATE) and completes the body once none is active (a
        // sequential body at once); else a sequential body creates its next inner instance while items
        // are left, and the body completes once no child is active
        const ElementInstance& body = fit->second;
        const OEl& b = E(body.value);
        if (satisfies) {
          const bool none = body.childCount == 0;
          if (!none) {
            ORecord& rec = append(ZBHIP_RT_COMMAND, ZBHIP_VT_PROCESS_INSTANCE_BATCH, ZBHIP_PIB_TERMINATE, next_key());
            rec.r.process_idx = body.value.proc;
            rec.r.element_idx = body.value.elem;
            rec.r.scope_key = body.key;  // batchElementInstanceKey
            rec.r.process_instance_key = body.value.piKey;
            rec.r.partition = -1;  // index: from the first child
            rec.pi = body.value;
          }
          if (none || b.mi_seq) pi_command(body.key, ZBHIP_PI_COMPLETE_ELEMENT, body.value);
        } else if (b.mi_seq && body.loopCounter < (int)input_collection(b, body.key).size()) {
          PiValue c = body.value;
          c.flowScopeKey = body.key;
          c.elem = b.inner;
          pi_command(next_key(), ZBHIP_PI_ACTIVATE_ELEMENT, c);
        } else if ((int64_t)body.childCount + body.activeSequenceFlows == 0) {
          pi_command(body.key, ZBHIP_PI_COMPLETE_ELEMENT, body.value);
        }
      } else if (fit != ei_.end()) {
        const ElementInstance& fs = fit->second;
        if ((int64_t)fs.childCount + fs.activeSequenceFlows == 0) {
          pi_command(fs.key, ZBHIP_PI_COMPLETE_ELEMENT, fs.value);
        }
      }
    }
  }

  // takeSequenceFlow (:243-263) + activateElementInstanceInFlowScope (:326-339)
  void take_sequence_flow(int64_t /*from*/, const PiValue& v, int flow) {
    const OEl& f = P(v.proc).els[flow];
    PiValue sv = v;
    sv.elem = flow;
    int64_t sfKey = next_key();
    pi_event(sfKey, ZBHIP_PI_SEQUENCE_FLOW_TAKEN, sv);
    PiValue tv = v;
    tv.elem = f.tgt;
    int64_t k = next_key();
    pi_command(k, ZBHIP_PI_ACTIVATE_ELEMENT, tv);
  }

  // ExclusiveGatewayProcessor.findSequenceFlowToTake (:86-126)
  // A failure (Either.left) is returned as -2 with `fail`: the error type, the flow whose condition
  // did not evaluate to a boolean (-1: none chosen) and that result's type.
  struct FlowFailure { int error_type = 0, flow = -1, result = 0; };
  // an incident's `flow` marking a message correlation key that is neither a string nor a number, and
  // that key's BOOLEAN result type (beside ZBHIP_FEEL_NULL / NUMBER / STRING)
  static constexpr int kCorrelationKeyFailure = -3, kFeelBoolean = 3;
  int find_sequence_flow_to_take(const OEl& el, int64_t gwKey, int proc, FlowFailure& fail) {
    const OProc& p = P(proc);
    if (el.out.empty()) return -1;  // implicit end of the flow scope
    if (el.out.size() == 1 && !p.els[el.out[0]].has_cond) return el.out[0];
    for (int f : el.out_with_cond) {
      if (el.default_flow == f) continue;  // the default flow's condition is never evaluated
      // ExpressionProcessor.evaluateBooleanExpression (processing/common/ExpressionProcessor.java:126-131,356-368):
      // typeCheck -> EXTRACT_VALUE_ERROR "Expected result of the expression '%s' to be 'BOOLEAN', but was '%s'."
      FVal r = eval(p.els[f].cond.get(), gwKey);
      if (r.k != V_BOOL) {
        if (r.k == V_ERR) throw Unsupported{"condition value outside the subset"};
        fail.error_type = ZBHIP_ERR_EXTRACT_VALUE_ERROR;
        fail.flow = f;
        fail.result = r.k == V_NULL ? ZBHIP_FEEL_NULL : r.k == V_NUM ? ZBHIP_FEEL_NUMBER : ZBHIP_FEEL_STRING;
        return -2;
      }
      if (r.b) return f;
    }
    if (el.default_flow >= 0) return el.default_flow;
    // (:121-125) NO_OUTGOING_FLOW_CHOSEN_ERROR, CONDITION_ERROR
    fail.error_type = ZBHIP_ERR_CONDITION_ERROR;
    return -2;
  }

  // BpmnIncidentBehavior.createIncident (processing/bpmn/behavior/BpmnIncidentBehavior.java:51-71):
  // INCIDENT:CREATED (key = nextKey) for the element instance, variable scope = the element instance
  // (the failure's scope key is the gateway's); IncidentCreatedApplier -> DbIncidentState.createIncident
  // (INCIDENTS, INCIDENT_PROCESS_INSTANCES).  The element instance stays where the failure left it.
  void create_incident(const FlowFailure& f, int64_t eik, const PiValue& v) {
    const int64_t key = next_key();
    ORecord& rec = append(ZBHIP_RT_EVENT, ZBHIP_VT_INCIDENT, ZBHIP_INCIDENT_CREATED, key);
    rec.r.process_idx = v.proc;
    rec.r.element_idx = v.elem;
    rec.r.scope_key = eik;
    rec.r.process_instance_key = v.piKey;
    rec.r.partition = f.error_type;
    rec.r.aux = f.flow;
    rec.r.reason_arg = (uint8_t)f.result;
    IncidentRow row;
    row.pi = v;
    row.eik = eik;
    row.error_type = f.error_type;
    row.flow = f.flow;
    row.result = f.result;
    incidents_[key] = row;
    incident_pi_[eik] = key;
  }

  // DbVariableState.getVariable walks the scope chain (state/variable/DbVariableState.java:174-200)
  const VarRow* lookup_var(int64_t scope, int name) {
    int64_t s = scope;
    while (s > 0) {
      auto it = vars_.find({s, name});
      if (it != vars_.end()) return &it->second;
      auto pit = child_parent_.find(s);
      if (pit == child_parent_.end()) break;
      s = pit->second;
    }
    return nullptr;
  }

  FVal eval(const FExpr* e, int64_t scope) {
    FVal r;
    switch (e->op) {
      case FExpr::NUM: r.k = V_NUM; r.n = e->num; return r;
      case FExpr::BOOL: r.k = V_BOOL; r.b = e->b; return r;
      case FExpr::NUL: r.k = V_NULL; return r;
      case FExpr::VAR: {
        if (cond_body_) {  // the completion condition's primary context (MultiInstanceBodyProcessor :396-460)
          const ElementInstance& b = *cond_body_;
          const std::string& n = e->var;
          int64_t x = 0;
          bool hit = true;
          if (n == "numberOfInstances") x = b.childActivated;
          else if (n == "numberOfActiveInstances") x = b.childCount - 1;
          else if (n == "numberOfCompletedInstances") x = b.childCompleted + 1;
          else if (n == "numberOfTerminatedInstances") x = b.childTerminated;
          else hit = false;
          if (hit) { r.k = V_NUM; r.n = (__int128)x * kScale18; return r; }
        }
        auto it = name_ids.find(e->var);
        const VarRow* vr = it == name_ids.end() ? nullptr : lookup_var(scope, it->second);
        if (!vr || vr->type == ZBHIP_DOC_NIL) { r.k = V_NULL; return r; }
        if (vr->type == ZBHIP_DOC_BOOL) { r.k = V_BOOL; r.b = vr->value != 0; return r; }
        if (vr->type == ZBHIP_DOC_INT) { r.k = V_NUM; r.n = (__int128)vr->value * kScale18; return r; }
        if (vr->type == ZBHIP_DOC_DEC) { r.k = V_NUM; r.n = (__int128)vr->value * (kScale18 / 1000000); return r; }
        if (vr->type == ZBHIP_DOC_STR) { r.k = V_STR; return r; }  // (the text is never compared)
        r.k = V_ERR;
        return r;
      }
      case FExpr::NOT: {
        FVal a = eval(e->l.get(), scope);
        if (a.k != V_BOOL) throw Unsupported{"not() of non-boolean"};
        r.k = V_BOOL; r.b = !a.b; return r;
      }
      case FExpr::AND:
      case FExpr::OR: {
        FVal a = eval(e->l.get(), scope), b = eval(e->r.get(), scope);
        if (a.k != V_BOOL || b.k != V_BOOL) throw Unsupported{"and/or over non-booleans"};
        r.k = V_BOOL;
        r.b = e->op == FExpr::AND ? (a.b && b.b) : (a.b || b.b);
        return r;
      }
      case FExpr::CMP: {
        FVal a = eval(e->l.get(), scope), b = eval(e->r.get(), scope);
        if (a.k == V_ERR || b.k == V_ERR) throw Unsupported{"value type outside the subset"};
        const std::string& c = e->cmp;
        if (c == "=" || c == "!=") {
          bool eq;
          if (a.k == V_STR || b.k == V_STR) throw Unsupported{"string equality"};
          if (a.k == V_NULL || b.k == V_NULL) eq = a.k == b.k;
          else if (a.k != b.k) throw Unsupported{"comparison of mixed types"};
          else eq = a.k == V_NUM ? a.n == b.n : a.b == b.b;
          r.k = V_BOOL;
          r.b = c == "=" ? eq : !eq;
          return r;
        }
        // feel-scala 1.17: an ordering comparison with null, or of a string with a number, is null
        // (ConditionIncidentTest.shouldCreateIncidentIfConditionFailsToEvaluate: `foo > 10` with
        // foo = "bar" was 'NULL')
        if (a.k == V_NULL || b.k == V_NULL || (a.k == V_STR && b.k == V_NUM) || (a.k == V_NUM && b.k == V_STR)) {
          r.k = V_NULL;
          return r;
        }
        if (a.k != V_NUM || b.k != V_NUM) throw Unsupported{"ordering comparison with non-number"};
        r.k = V_BOOL;
        if (c == "<") r.b = a.n < b.n;
        else if (c == "<=") r.b = a.n <= b.n;
        else if (c == ">") r.b = a.n > b.n;
        else r.b = a.n >= b.n;
        return r;
      }
    }
    throw Unsupported{"expr"};
  }

  // ---------------------------------------------------------------------
  // event appliers for PROCESS_INSTANCE (state/appliers/EventAppliers.java:121-157)
  // ---------------------------------------------------------------------
  void apply_pi(int64_t key, int intent, const PiValue& v) {
    const OEl& el = E(v);
    switch (intent) {
      case ZBHIP_PI_ELEMENT_ACTIVATING: {  // ProcessInstanceElementActivatingApplier.applyState (:48-77)
        // createEventScope (:255-289): job worker elements get an event scope
        // (a sub-process only with events: its boundary event)
        if (ZBHIP_IS_JOB_WORKER(el.type) || el.type == ZBHIP_EL_INTERMEDIATE_CATCH_EVENT ||
            el.type == ZBHIP_EL_BOUNDARY_EVENT ||
            ((el.type == ZBHIP_EL_SUB_PROCESS || el.type == ZBHIP_EL_MULTI_INSTANCE_BODY) && el.boundary >= 0) ||
            ((el.type == ZBHIP_EL_PROCESS || el.type == ZBHIP_EL_SUB_PROCESS) && !el.esps.empty()))
          event_scope_.insert(key);
        // cleanupSequenceFlowsTaken (:79-98): Tetris decrement of (flowScope, gateway)
        if (el.type == ZBHIP_EL_PARALLEL_GATEWAY) {
          for (auto it = taken_.lower_bound({v.flowScopeKey, v.elem, -1}); it != taken_.end();) {
            if (std::get<0>(it->first) != v.flowScopeKey || std::get<1>(it->first) != v.elem) break;
            if (--it->second > 0) ++it;
            else it = taken_.erase(it);
          }
        }
        auto fit = ei_.find(v.flowScopeKey);
        // DbElementInstanceState.newInstance/createInstance (state/instance/DbElementInstanceState.java:141-210)
        ElementInstance inst;
        inst.key = key;
        inst.state = ZBHIP_PI_ELEMENT_ACTIVATING;
        inst.value = v;
        if (fit != ei_.end()) {
          inst.parentKey = fit->second.key;
          fit->second.childCount += 1;
        }
        if (fit != ei_.end() && E(fit->second.value).type == ZBHIP_EL_MULTI_INSTANCE_BODY) {
          // manageMultiInstance (:237-253): the body's loop counter and childActivatedCount, the
          // inner instance's loop counter
          fit->second.loopCounter += 1;
          fit->second.childActivated += 1;
          inst.loopCounter = fit->second.loopCounter;
        }
        ei_[key] = inst;
        parent_child_.insert({inst.parentKey, key});
        child_parent_[key] = inst.parentKey;  // DbVariableState.createScope
        if (el.type == ZBHIP_EL_PROCESS) pi_by_def_.insert({P(v.proc).def_key, key});
        if (fit == ei_.end()) return;  // root process (applyRootProcessState: no parent)
        // decrementActiveSequenceFlow (:130-204); decrementActiveSequenceFlows clamps at 0 (ElementInstance.java:203-213)
        ElementInstance& fs = fit->second;
        auto dec = [&fs]() { if (fs.activeSequenceFlows > 0) fs.activeSequenceFlows--; };
        switch (el.type) {
          case ZBHIP_EL_START_EVENT:
          case ZBHIP_EL_BOUNDARY_EVENT:
            break;
          case ZBHIP_EL_PARALLEL_GATEWAY:
            for (size_t i = 0; i < el.in.size(); ++i) dec();
            break;
          case ZBHIP_EL_EVENT_SUB_PROCESS:  // decrementEventSubProcessSequenceFlow (:206-218): interrupting -> reset
            if (P(v.proc).els[el.start].interrupting) fs.activeSequenceFlows = 0;
            break;
          default:
            dec();
        }
        if (el.type == ZBHIP_EL_START_EVENT && E(fs.value).type == ZBHIP_EL_EVENT_SUB_PROCESS) {
          // moveVariablesToNewEventScope (:102-116): the event sub-process's flow scope's (first) event
          // trigger moves to the start event's instance, whose output mappings read its variables
          auto tit = triggers_.lower_bound({fs.parentKey, INT64_MIN});
          if (tit != triggers_.end() && tit->first.first == fs.parentKey) {
            EventTrigger t = tit->second;
            const int64_t eventKey = tit->first.second;
            triggers_.erase(tit);
            triggers_[{key, eventKey}] = t;
          }
        }
        break;
      }
      case ZBHIP_PI_ELEMENT_ACTIVATED:  // ProcessInstanceElementActivatedApplier
        ei_.at(key).state = ZBHIP_PI_ELEMENT_ACTIVATED;
        break;
      case ZBHIP_PI_ELEMENT_COMPLETING:  // ProcessInstanceElementCompletingApplier
        ei_.at(key).state = ZBHIP_PI_ELEMENT_COMPLETING;
        break;
      case ZBHIP_PI_ELEMENT_TERMINATING:  // ProcessInstanceElementTerminatingApplier
        ei_.at(key).state = ZBHIP_PI_ELEMENT_TERMINATING;
        break;
      case ZBHIP_PI_ELEMENT_TERMINATED:  // ProcessInstanceElementTerminatedApplier (:38-55): the same removal
      case ZBHIP_PI_ELEMENT_COMPLETED: {  // ProcessInstanceElementCompletedApplier (:45-73)
        // eventScopeInstanceState.deleteInstance: triggers then the scope
        for (auto it = triggers_.lower_bound({key, INT64_MIN}); it != triggers_.end() && it->first.first == key;)
          it = triggers_.erase(it);
        event_scope_.erase(key);
        es_interrupted_.erase(key);
        es_closed_.erase(key);
        // DbElementInstanceState.removeInstance (:160-193)
        auto it = ei_.find(key);
        if (it == ei_.end()) break;
        int64_t parent = it->second.parentKey;
        parent_child_.erase({parent, key});
        ei_.erase(it);
        // variableState.removeScope: variables of the scope + child->parent row
        for (auto vit = vars_.lower_bound({key, INT32_MIN}); vit != vars_.end() && vit->first.first == key;)
          vit = vars_.erase(vit);
        child_parent_.erase(key);
        for (auto tit = taken_.lower_bound({key, INT32_MIN, INT32_MIN}); tit != taken_.end() && std::get<0>(tit->first) == key;)
          tit = taken_.erase(tit);
        if (el.type == ZBHIP_EL_PROCESS) pi_by_def_.erase({P(v.proc).def_key, key});
        if (el.type == ZBHIP_EL_PROCESS && !P(v.proc).msg_starts.empty()) {
          // BufferedStartMessageEventStateApplier.removeMessageLock (:36-66)
          auto cit = pi_corr_keys_.find(v.piKey);
          if (cit != pi_corr_keys_.end()) {
            active_by_corr_.erase({P(v.proc).bpmn_name, cit->second});
            pi_corr_keys_.erase(cit);
          }
        }
        if (parent > 0) {
          ElementInstance& pe = ei_.at(parent);
          pe.childCount -= 1;
          if (E(pe.value).type == ZBHIP_EL_MULTI_INSTANCE_BODY) {  // manageMultiInstance (Completed :104-110,
            if (intent == ZBHIP_PI_ELEMENT_TERMINATED) pe.childTerminated += 1;  // Terminated :53-58)
            else pe.childCompleted += 1;
          }
        }
        break;
      }
      case ZBHIP_PI_SEQUENCE_FLOW_TAKEN: {  // ProcessInstanceSequenceFlowTakenApplier (:32-69)
        ElementInstance& fs = ei_.at(v.flowScopeKey);
        fs.activeSequenceFlows += 1;
        const OEl& tgt = P(v.proc).els[el.tgt];
        if (tgt.type == ZBHIP_EL_PARALLEL_GATEWAY) taken_[{v.flowScopeKey, el.tgt, v.elem}] += 1;
        break;
      }
      default:
        break;
    }
  }
};

std::string Oracle::dump_state() const {
  std::vector<std::string> rows;
  char buf[512];
  auto pid = [this](const PiValue& v, int e) -> const std::string& { return procs[v.proc].els[e].id; };
  snprintf(buf, sizeof buf, "KEY|latestKey|%lld", (long long)(((int64_t)partition_ << 51) + key_counter_));
  rows.push_back(buf);
  for (auto& [k, e] : ei_) {
    const OEl& el = procs[e.value.proc].els[e.value.elem];
    snprintf(buf, sizeof buf,
             "ELEMENT_INSTANCE_KEY|%lld|parentKey=%lld,childCount=%d,childActivatedCount=%d,childCompletedCount=%d,"
             "childTerminatedCount=%d,jobKey=%lld,multiInstanceLoopCounter=%d,interruptingElementId=%s,"
             "calledChildInstanceKey=-1,state=%d,elementId=%s,bpmnElementType=%d,bpmnEventType=%d,flowScopeKey=%lld,"
             "processInstanceKey=%lld,processDefinitionKey=%lld,activeSequenceFlows=%d",
             (long long)k, (long long)e.parentKey, e.childCount, e.childActivated, e.childCompleted,
             e.childTerminated, (long long)e.jobKey, e.loopCounter,
             e.interrupting_elem >= 0 ? procs[e.value.proc].els[e.interrupting_elem].id.c_str() : "", e.state, el.id.c_str(), el.type,
             el.event, (long long)e.value.flowScopeKey, (long long)e.value.piKey,
             (long long)procs[e.value.proc].def_key, e.activeSequenceFlows);
    rows.push_back(buf);
  }
  for (auto& [p, c] : parent_child_) {
    snprintf(buf, sizeof buf, "ELEMENT_INSTANCE_PARENT_CHILD|%lld|%lld", (long long)p, (long long)c);
    rows.push_back(buf);
  }
  for (auto& [c, p] : child_parent_) {
    snprintf(buf, sizeof buf, "ELEMENT_INSTANCE_CHILD_PARENT|%lld|%lld", (long long)c, (long long)p);
    rows.push_back(buf);
  }
  for (auto& [k, n] : taken_) {
    // gateway/flow ids need the process: find it via any element instance is not possible here;
    // ids are process-local indices resolved through the first process that has them
    int gw = std::get<1>(k), fl = std::get<2>(k);
    const OProc* proc = nullptr;
    auto eit = ei_.find(std::get<0>(k));
    if (eit != ei_.end()) proc = &procs[eit->second.value.proc];
    snprintf(buf, sizeof buf, "NUMBER_OF_TAKEN_SEQUENCE_FLOWS|%lld|%s|%s|%d", (long long)std::get<0>(k),
             proc ? proc->els[gw].id.c_str() : "?", proc ? proc->els[fl].id.c_str() : "?", n);
    rows.push_back(buf);
  }
  for (auto& [d, p] : pi_by_def_) {
    snprintf(buf, sizeof buf, "PROCESS_INSTANCE_KEY_BY_DEFINITION_KEY|%lld|%lld", (long long)d, (long long)p);
    rows.push_back(buf);
  }
  for (auto& [k, vr] : vars_) {
    if (vr.type == ZBHIP_DOC_LIST) {  // a list: its items (type:value, ';'-separated)
      snprintf(buf, sizeof buf, "VARIABLES|%lld|%s|key=%lld,type=%d,value=", (long long)k.first, names[k.second].c_str(),
               (long long)vr.key, vr.type);
      rows.push_back(std::string(buf) + list_text(lists.at((size_t)vr.value)));
      continue;
    }
    snprintf(buf, sizeof buf, "VARIABLES|%lld|%s|key=%lld,type=%d,value=%lld", (long long)k.first,
             names[k.second].c_str(), (long long)vr.key, vr.type, (long long)vr.value);
    rows.push_back(buf);
  }
  for (auto k : event_scope_) {
    // EventScopeInstance (state/instance/EventScopeInstance.java:25-35): the interrupting ids of a
    // catch / boundary event are its own id (ExecutableCatchEventElement.java:124-132), an activity's
    // those of its interrupting boundary events, which are also its boundaryElementIds
    // (ExecutableActivity.java:28-38)
    auto eit = ei_.find(k);
    const OProc* op = eit == ei_.end() ? nullptr : &procs[eit->second.value.proc];
    const OEl* el = op ? &op->els[eit->second.value.elem] : nullptr;
    std::string intr, bnd;
    if (el && (el->type == ZBHIP_EL_INTERMEDIATE_CATCH_EVENT || el->type == ZBHIP_EL_BOUNDARY_EVENT)) intr = el->id;
    if (el && (el->boundary >= 0 || !el->esps.empty())) {  // interruptingIds only for cancelActivity boundary events
      for (int b : el->boundaries) {
        bnd += (bnd.empty() ? "" : ";") + op->els[b].id;
        if (op->els[b].interrupting) intr += (intr.empty() ? "" : ";") + op->els[b].id;
      }
      // then the interrupting event sub-processes' start events (attached in a later transformation step)
      for (int esp : el->esps) {
        const OEl& st = op->els[op->els[esp].start];
        if (st.interrupting) intr += (intr.empty() ? "" : ";") + st.id;
      }
    }
    snprintf(buf, sizeof buf, "EVENT_SCOPE|%lld|accepting=%d,interrupted=%d,interrupting=%s,boundaryElementIds=%s",
             (long long)k, es_closed_.count(k) ? 0 : 1, es_interrupted_.count(k) ? 1 : 0, intr.c_str(), bnd.c_str());
    rows.push_back(buf);
  }
  for (auto& [k, t] : triggers_) {
    PiValue pv;
    pv.proc = t.proc;
    snprintf(buf, sizeof buf, "EVENT_TRIGGER|%lld|%lld|elementId=%s,processInstanceKey=%lld,vars=%u:%u",
             (long long)k.first, (long long)k.second, pid(pv, t.elem).c_str(), (long long)t.piKey, t.vars.begin,
             t.vars.count);
    rows.push_back(buf);
  }
  for (auto& [k, t] : timers_) {
    const OProc& p = procs[t.pi.proc];
    snprintf(buf, sizeof buf,
             "TIMERS|%lld|%lld|handlerNodeId=%s,processDefinitionKey=%lld,key=%lld,elementInstanceKey=%lld,"
             "processInstanceKey=%lld,dueDate=%lld,repetitions=%d,tenantId=<default>",
             (long long)k.first, (long long)k.second, p.els[t.pi.elem].id.c_str(), (long long)p.def_key,
             (long long)k.second, (long long)k.first, (long long)t.pi.piKey, (long long)t.dueDate, t.reps);
    rows.push_back(buf);
    snprintf(buf, sizeof buf, "TIMER_DUE_DATES|%lld|%lld|%lld", (long long)t.dueDate, (long long)k.first,
             (long long)k.second);
    rows.push_back(buf);
  }
  for (auto& [k, j] : jobs_) {
    const OProc& p = procs[j.pi.proc];
    snprintf(buf, sizeof buf,
             "JOBS|%lld|type=%s,retries=%d,elementId=%s,elementInstanceKey=%lld,processInstanceKey=%lld,"
             "bpmnProcessId=%s,processDefinitionKey=%lld,processDefinitionVersion=%d,tenantId=<default>,"
             "deadline=%lld,worker=",
             (long long)k, j.type.c_str(), j.retries, j.no_catch ? "NO_CATCH_EVENT_FOUND" : p.els[j.pi.elem].id.c_str(),
             (long long)j.elementInstanceKey, (long long)j.pi.piKey, p.bpmn_id.c_str(), (long long)p.def_key, p.version,
             (long long)j.deadline);
    // (worker and errorMessage appended unbounded: a message holds up to 10 000 characters)
    rows.push_back(std::string(buf) + j.worker +
                   (j.fail_fields ? ",errorMessageHex=" + hex_of(j.error_message) + ",retryBackoff=" +
                                        std::to_string(j.retry_backoff) + ",recurringTime=" + std::to_string(j.recurring_time)
                                  : std::string()) +
                   (j.error_thrown ? ",errorCodeHex=" + hex_of(j.error_code) : std::string()));
    snprintf(buf, sizeof buf, "JOB_STATES|%lld|%s", (long long)k,
             j.error_thrown ? "ERROR_THROWN" : j.failed ? "FAILED" : j.activated ? "ACTIVATED" : "ACTIVATABLE");
    rows.push_back(buf);
    if (j.failed && j.retries > 0 && j.retry_backoff > 0) {  // JOB_BACKOFF [recurringTime, jobKey] -> DbNil
      snprintf(buf, sizeof buf, "JOB_BACKOFF|%lld|%lld", (long long)j.recurring_time, (long long)k);
      rows.push_back(buf);
    }
    if (j.activated) {  // JOB_DEADLINES [deadline, jobKey] -> DbNil
      snprintf(buf, sizeof buf, "JOB_DEADLINES|%lld|%lld", (long long)j.deadline, (long long)k);
      rows.push_back(buf);
    }
  }
  for (auto& [k, in] : incidents_) {  // INCIDENTS (DbIncidentState.createIncident)
    const OProc& p = procs[in.pi.proc];
    snprintf(buf, sizeof buf,
             "INCIDENTS|%lld|errorType=%d,flow=%d,result=%d,processDefinitionKey=%lld,processInstanceKey=%lld,"
             "elementId=%s,elementInstanceKey=%lld",
             (long long)k, in.error_type, in.flow, in.result, (long long)p.def_key, (long long)in.pi.piKey,
             in.no_catch ? "NO_CATCH_EVENT_FOUND" : p.els[in.pi.elem].id.c_str(), (long long)in.eik);
    rows.push_back(std::string(buf) +
                   (in.job_key >= 0 ? ",jobKey=" + std::to_string(in.job_key) + ",messageHex=" + hex_of(in.message) : ""));
  }
  for (auto& [j, k] : incident_jobs_) {  // INCIDENT_JOBS [jobKey] -> incident key (a job's incident)
    snprintf(buf, sizeof buf, "INCIDENT_JOBS|%lld|%lld", (long long)j, (long long)k);
    rows.push_back(buf);
  }
  for (auto& [e, k] : incident_pi_) {
    snprintf(buf, sizeof buf, "INCIDENT_PROCESS_INSTANCES|%lld|%lld", (long long)e, (long long)k);
    rows.push_back(buf);
  }
  for (auto& [t, ten, k] : activatable_) {
    snprintf(buf, sizeof buf, "JOB_ACTIVATABLE|%s|%s|%lld", t.c_str(), ten.c_str(), (long long)k);
    rows.push_back(buf);
  }
  auto nm = [this](int id) -> const char* { return id >= 0 && id < (int)names.size() ? names[id].c_str() : ""; };
  auto sv = [this](uint32_t id) -> const char* { return id < strs.size() ? strs[id].c_str() : ""; };
  for (auto& [k, row] : pms_) {
    const MsgVal& m = row.rec;
    snprintf(buf, sizeof buf,
             "PROCESS_SUBSCRIPTION_BY_KEY|%lld|%s|key=%lld,state=%s,subscriptionPartitionId=%d,processInstanceKey=%lld,"
             "bpmnProcessId=%s,messageKey=%lld,correlationKey=%s,elementId=%s,interrupting=%d",
             (long long)k.first, nm(k.second), (long long)row.key, row.closing ? "CLOSING" : row.opened ? "OPENED" : "OPENING", m.partition,
             (long long)m.pik, nm(m.bpmn), (long long)m.msg_key, sv(m.corr), procs[m.proc].els[m.elem].id.c_str(),
             m.interrupting);
    rows.push_back(buf);
  }
  for (auto& [k, sub] : msub_) {
    const MsgVal& m = sub.rec;
    snprintf(buf, sizeof buf,
             "MESSAGE_SUBSCRIPTION_BY_KEY|%lld|%s|key=%lld,correlating=%d,processInstanceKey=%lld,bpmnProcessId=%s,"
             "messageKey=%lld,correlationKey=%s,interrupting=%d",
             (long long)k.first, nm(k.second), (long long)sub.key, sub.correlating ? 1 : 0, (long long)m.pik,
             nm(m.bpmn), (long long)m.msg_key, sv(m.corr), m.interrupting);
    rows.push_back(buf);
  }
  for (auto& [n, c, e] : msub_by_corr_) {
    snprintf(buf, sizeof buf, "MESSAGE_SUBSCRIPTION_BY_NAME_AND_CORRELATION_KEY|<default>|%s|%s|%lld", nm(n), sv(c),
             (long long)e);
    rows.push_back(buf);
  }
  for (auto& [k, m] : messages_) {
    rows.push_back("MESSAGE_KEY|" + std::to_string(k) + "|name=" + nm(m.name) + ",correlationKey=" + sv(m.corr) +
                   ",timeToLive=" + std::to_string(m.ttl) + ",deadline=" + std::to_string(m.deadline) +
                   ",messageId=" + (m.message_id == ZBHIP_NO_STRING ? std::string() : sv(m.message_id)));
    rows.push_back("MESSAGES|<default>|" + std::string(nm(m.name)) + "|" + sv(m.corr) + "|" + std::to_string(k));
    if (m.message_id != ZBHIP_NO_STRING)
      rows.push_back("MESSAGE_IDS|<default>|" + std::string(nm(m.name)) + "|" + sv(m.corr) + "|" + sv(m.message_id));
  }
  for (auto& [d, k] : msg_deadlines_) rows.push_back("MESSAGE_DEADLINES|" + std::to_string(d) + "|" + std::to_string(k));
  for (auto& [k, b] : msg_correlated_) rows.push_back("MESSAGE_CORRELATED|" + std::to_string(k) + "|" + nm(b));
  for (auto& [k, s] : msg_start_subs_) {  // DbMessageStartEventSubscriptionState's two column families
    const OProc& p = procs[s.proc];
    rows.push_back("MESSAGE_START_EVENT_SUBSCRIPTION_BY_NAME_AND_KEY|<default>|" + std::string(nm(k.first)) + "|" +
                   std::to_string(k.second) + "|key=" + std::to_string(s.key) + ",bpmnProcessId=" + p.bpmn_id +
                   ",startEventId=" + p.els[s.elem].id);
    rows.push_back("MESSAGE_START_EVENT_SUBSCRIPTION_BY_KEY_AND_NAME|" + std::to_string(k.second) + "|<default>|" +
                   nm(k.first));
  }
  for (auto& [b, c] : active_by_corr_)
    rows.push_back("MESSAGE_PROCESSES_ACTIVE_BY_CORRELATION_KEY|" + std::string(nm(b)) + "|" + sv(c));
  for (auto& [pk, c] : pi_corr_keys_)
    rows.push_back("MESSAGE_PROCESS_INSTANCE_CORRELATION_KEYS|" + std::to_string(pk) + "|" + sv(c));
  if (msg_stats_) rows.push_back("MESSAGE_STATS|messagesDeadlineCount|" + std::to_string(msg_deadline_count_));
  std::sort(rows.begin(), rows.end());
  std::string s;
  for (auto& r : rows) { s += r; s += '\n'; }
  return s;
}

}  // namespace

// ============================================================================
// C API (ctypes) — test infrastructure only
// ============================================================================
extern "C" {

void* zbo_new(int partition_id, int partition_count, int max_commands_in_batch, int64_t initial_key) {
  return new Oracle(partition_id, partition_count, max_commands_in_batch, initial_key);
}
void zbo_free(void* o) { delete static_cast<Oracle*>(o); }
const char* zbo_last_error(void* o) { return static_cast<Oracle*>(o)->last_error.c_str(); }

int zbo_deploy_xml(void* o, const char* xml, int64_t def_key, int version) {
  return static_cast<Oracle*>(o)->deploy(std::string(xml), def_key, version);
}
int zbo_intern(void* o, const char* name) { return static_cast<Oracle*>(o)->intern(name); }
const char* zbo_name(void* o, int id) {
  auto* O = static_cast<Oracle*>(o);
  return id >= 0 && id < (int)O->names.size() ? O->names[id].c_str() : "";
}
int zbo_n_elements(void* o, int proc) { return (int)static_cast<Oracle*>(o)->procs.at(proc).els.size(); }
const char* zbo_element_id(void* o, int proc, int elem) {
  return static_cast<Oracle*>(o)->procs.at(proc).els.at(elem).id.c_str();
}

// deployment tables for the log-serialisation checker (oracle/logserial.py)
int zbo_element_info(void* o, int proc, int elem, int* type, int* event, int* retries) {
  const OEl& e = static_cast<Oracle*>(o)->procs.at(proc).els.at(elem);
  *type = e.type;
  *event = e.event;
  *retries = e.retries;
  return 0;
}
const char* zbo_element_cond_text(void* o, int proc, int elem) {
  auto* z = static_cast<Oracle*>(o);
  if (proc < 0 || (size_t)proc >= z->procs.size() || elem < 0 || (size_t)elem >= z->procs[proc].els.size()) return "";
  return z->procs[proc].els[elem].cond_text.c_str();
}

const char* zbo_element_job_type(void* o, int proc, int elem) {
  return static_cast<Oracle*>(o)->procs.at(proc).els.at(elem).job_type.c_str();
}
// the customHeaders msgpack map of a job worker's jobs (empty: NO_HEADERS); returns its length
int zbo_element_headers(void* o, int proc, int elem, char* buf, int cap) {
  const std::string& h = static_cast<Oracle*>(o)->procs.at(proc).els.at(elem).header_bytes;
  if (buf && cap > 0) memcpy(buf, h.data(), std::min<size_t>((size_t)cap, h.size()));
  return (int)h.size();
}
const char* zbo_process_info(void* o, int proc, int64_t* def_key, int* version) {
  const OProc& P = static_cast<Oracle*>(o)->procs.at(proc);
  *def_key = P.def_key;
  *version = P.version;
  return P.bpmn_id.c_str();
}
const char* zbo_string_value(void* o, int id, size_t* len) {
  const std::string& v = static_cast<Oracle*>(o)->str((uint32_t)id);
  *len = v.size();
  return v.data();
}
int zbo_n_strings(void* o) { return (int)static_cast<Oracle*>(o)->strs.size(); }
int zbo_n_names(void* o) { return (int)static_cast<Oracle*>(o)->names.size(); }
int zbo_n_processes(void* o) { return (int)static_cast<Oracle*>(o)->procs.size(); }

int zbo_submit(void* o, const zbhip_command* cmds, size_t n, const zbhip_doc_entry* docs, size_t nd) {
  static_cast<Oracle*>(o)->submit(cmds, n, docs, nd);
  return 0;
}
int zbo_submit_ex(void* o, const zbhip_command* cmds, size_t n, const zbhip_doc_entry* docs, size_t nd,
                  const zbhip_xpart_cmd* xp, size_t nx) {
  static_cast<Oracle*>(o)->submit(cmds, n, docs, nd, xp, nx);
  return 0;
}
int64_t zbo_intern_string(void* o, const char* b, size_t len) {
  return static_cast<Oracle*>(o)->intern_string(std::string(b, len));
}
// the list dictionary (ZBHIP_DOC_LIST values): items as zbhip_doc_entry rows (type, value; name unused)
int64_t zbo_intern_list(void* o, const zbhip_doc_entry* items, size_t n) {
  Oracle::Items v;
  for (size_t i = 0; i < n; ++i) v.push_back({items[i].type, items[i].value});
  return static_cast<Oracle*>(o)->intern_list(v);
}
size_t zbo_list_items(void* o, int64_t id, zbhip_doc_entry* out, size_t cap) {
  auto* O = static_cast<Oracle*>(o);
  if (id < 0 || (size_t)id >= O->lists.size()) return 0;
  const auto& v = O->lists[(size_t)id];
  for (size_t i = 0; i < v.size() && i < cap; ++i) {
    memset(&out[i], 0, sizeof out[i]);
    out[i].type = v[i].first;
    out[i].value = v[i].second;
  }
  return v.size();
}
size_t zbo_outbox(void* o, zbhip_xpart_cmd* out, size_t cap) {
  auto* O = static_cast<Oracle*>(o);
  size_t n = std::min(cap, O->outbox.size());
  for (size_t i = 0; i < n; ++i) out[i] = O->outbox[i];
  return O->outbox.size();
}
void zbo_clear_outbox(void* o) { static_cast<Oracle*>(o)->outbox.clear(); }
// the job types notified since the last call (notifyWorkAvailable side effects), '\n'-separated; cleared
size_t zbo_take_notified(void* o, char* buf, size_t cap) {
  auto* O = static_cast<Oracle*>(o);
  O->track_notified = true;
  std::string s;
  for (const auto& t : O->notified) s += t + "\n";
  if (buf && cap >= s.size()) {
    std::memcpy(buf, s.data(), s.size());
    O->notified.clear();
  }
  return s.size();
}
int zbo_subscription_partition(const char* b, size_t len, int partition_count) {
  return subscription_partition(std::string(b, len), partition_count);
}
int32_t zbo_java_hash(const char* b, size_t len) { return java_hash(std::string(b, len)); }
int zbo_run(void* o) { return static_cast<Oracle*>(o)->run(); }
int64_t zbo_key_counter(void* o) { return static_cast<Oracle*>(o)->key_counter(); }
// names: requested variable names, NUL-separated (n of them)
// a job stream for `type` (JobStreamer.streamFor: the gateway's StreamActivatedJobs), or none (on = 0)
void zbo_set_job_stream(void* o, const char* type, const char* worker, int64_t timeout, int on) {
  auto& e = *static_cast<Oracle*>(o);
  if (on) e.streams[type] = {worker, timeout};
  else e.streams.erase(type);
}

int zbo_activate_jobs(void* o, const char* type, const char* worker, int64_t timeout, int max_jobs, int64_t timestamp,
                      const char* names, size_t n_names, zbhip_activated_job* out, size_t cap, size_t* n_out,
                      int64_t* batch_key) {
  auto* O = static_cast<Oracle*>(o);
  std::vector<std::string> req;
  for (size_t i = 0; i < n_names; ++i) {
    req.emplace_back(names);
    names += req.back().size() + 1;
  }
  std::vector<Oracle::Activated> got;
  const int reason = O->activate_jobs(type, worker, timeout, max_jobs, timestamp, req, got, *batch_key);
  *n_out = got.size();
  for (size_t i = 0; i < got.size() && i < cap; ++i) {
    zbhip_activated_job& j = out[i];
    memset(&j, 0, sizeof j);
    j.key = got[i].key;
    j.element_instance_key = got[i].eik;
    j.process_instance_key = got[i].pik;
    j.deadline = got[i].deadline;
    j.process_idx = got[i].proc;
    j.element_idx = got[i].elem;
    j.retries = (uint16_t)got[i].retries;
    j.n_variables = (uint16_t)got[i].vars.size();
    for (size_t v = 0; v < got[i].vars.size() && v < 6; ++v) {
      j.variables[v].name_id = (uint32_t)got[i].vars[v].first;
      j.variables[v].type = got[i].vars[v].second.type;
      j.variables[v].value = got[i].vars[v].second.value;
    }
  }
  return reason;
}
// zbhip_job_variables' restatement: key -1 for a key that is no job
int zbo_job_variables(void* o, const int64_t* keys, size_t n, const char* names, size_t n_names,
                      zbhip_activated_job* out) {
  auto* O = static_cast<Oracle*>(o);
  std::vector<std::string> req;
  for (size_t i = 0; i < n_names; ++i) {
    req.emplace_back(names);
    names += req.back().size() + 1;
  }
  for (size_t i = 0; i < n; ++i) {
    zbhip_activated_job& j = out[i];
    memset(&j, 0, sizeof j);
    j.key = -1;
    Oracle::Activated a;
    if (!O->job_variables(keys[i], req, a)) continue;
    j.key = a.key;
    j.element_instance_key = a.eik;
    j.process_instance_key = a.pik;
    j.deadline = a.deadline;
    j.process_idx = a.proc;
    j.element_idx = a.elem;
    j.retries = (uint16_t)a.retries;
    j.n_variables = (uint16_t)std::min<size_t>(a.vars.size(), 6);
    for (size_t v = 0; v < a.vars.size() && v < 6; ++v) {
      j.variables[v].name_id = (uint32_t)a.vars[v].first;
      j.variables[v].type = a.vars[v].second.type;
      j.variables[v].value = a.vars[v].second.value;
    }
  }
  return 0;
}
void zbo_set_key_counter(void* o, int64_t v) { static_cast<Oracle*>(o)->set_key_counter(v); }

size_t zbo_n_records(void* o) { return static_cast<Oracle*>(o)->out.size(); }
int zbo_process_one(void* o, const zbhip_record* r, uint32_t instance, const zbhip_doc_entry* docs, size_t nd,
                    int64_t source, int first_ordinal) {
  return static_cast<Oracle*>(o)->process_one(*r, instance, docs, nd, source, first_ordinal);
}
int64_t zbo_ordinal_of(void* o, uint32_t instance, int64_t key) {
  auto& m = static_cast<Oracle*>(o)->inst_keys;
  auto it = m.find(instance);
  if (it == m.end()) return -1;
  for (size_t i = 0; i < it->second.size(); ++i)
    if (it->second[i] == key) return (int64_t)i;
  return -1;
}
int zbo_import_rows(void* o, const char* text, size_t len) {
  return static_cast<Oracle*>(o)->import_rows(std::string(text, len));
}
size_t zbo_records(void* o, zbhip_record* out, size_t cap) {
  auto* O = static_cast<Oracle*>(o);
  size_t n = std::min(cap, O->out.size());
  for (size_t i = 0; i < n; ++i) out[i] = O->out[i].r;
  return O->out.size();
}
int zbo_reason(void* o, size_t idx, char* buf, size_t cap) {
  auto* O = static_cast<Oracle*>(o);
  if (idx >= O->out.size()) return -1;
  snprintf(buf, cap, "%s", O->out[idx].reason.c_str());
  return (int)O->out[idx].reason.size();
}
void zbo_clear_records(void* o) { static_cast<Oracle*>(o)->out.clear(); }
void zbo_set_clock(void* o, int64_t now_ms) { static_cast<Oracle*>(o)->now_ms = now_ms; }
int64_t zbo_resolve(void* o, uint32_t instance, uint32_t ord) { return static_cast<Oracle*>(o)->resolve(instance, ord); }

size_t zbo_state(void* o, char* buf, size_t cap) {
  std::string s = static_cast<Oracle*>(o)->dump_state();
  if (buf && cap) snprintf(buf, cap, "%s", s.c_str());
  return s.size() + 1;
}
size_t zbo_fallback(void* o, uint32_t* out, size_t cap) {
  auto* O = static_cast<Oracle*>(o);
  size_t n = std::min(cap, O->fallback_.size());
  for (size_t i = 0; i < n; ++i) out[i] = O->fallback_[i];
  return O->fallback_.size();
}
void zbo_counters(void* o, uint64_t* transitions, uint64_t* completed, uint64_t* commands) {
  auto* O = static_cast<Oracle*>(o);
  *transitions = O->transitions;
  *completed = O->completed_instances;
  *commands = O->commands_processed;
}

// CPU baseline: `threads` independent partitions (one per host core, as Zeebe runs one
// actor per partition), each processing `n_instances` CREATE commands and then `phases`
// windows of JOB:COMPLETE (one per instance, completing the job created in the previous
// phase).  Returns wall seconds of the processing loop; process compilation excluded.
// CPU baseline of config 5: P partitions (one thread each) run the message-correlation protocol
// on n instances each; the exchange between the phases (route by target partition, sources in
// partition order) runs on the calling thread.  Returns wall seconds of processing + exchange.
double zbo_bench_msg(const char* xml, int P, int n, uint64_t* transitions_out, uint64_t* completed_out) {
  std::vector<std::string> dict;
  dict.reserve((size_t)P * n);
  for (int p = 1; p <= P; ++p)
    for (int i = 0; i < n; ++i) dict.push_back("k-" + std::to_string(p) + "-" + std::to_string(i));
  std::vector<std::unique_ptr<Oracle>> os;
  for (int p = 1; p <= P; ++p) {
    os.emplace_back(new Oracle(p, P, 100, 0));
    if (os.back()->deploy(xml, 2251799813685249LL, 1) < 0) return -1.0;
    os.back()->shared_strs = &dict;
  }
  const int var = os[0]->intern("key"), name = os[0]->intern("msg");
  std::vector<std::vector<zbhip_command>> cmd(P), pub(P);
  std::vector<std::vector<zbhip_doc_entry>> docs(P);
  for (int p = 0; p < P; ++p)
    for (int i = 0; i < n; ++i) {
      zbhip_command c{};
      c.instance = (uint32_t)i;
      c.kind = ZBHIP_CMD_CREATE;
      c.doc_count = 1;
      c.doc_begin = (uint32_t)i;
      cmd[p].push_back(c);
      zbhip_doc_entry d{};
      d.name_id = (uint32_t)var;
      d.type = ZBHIP_DOC_STR;
      d.value = (int64_t)p * n + i;
      docs[p].push_back(d);
    }
  for (uint32_t id = 0; id < (uint32_t)dict.size(); ++id) {
    zbhip_command c{};
    c.instance = id;
    c.kind = ZBHIP_CMD_PUBLISH;
    c.ref = (uint16_t)name;
    pub[subscription_partition(dict[id], P) - 1].push_back(c);
  }
  auto parallel = [&](auto fn) {
    std::vector<std::thread> th;
    for (int p = 0; p < P; ++p) th.emplace_back([&, p]() { fn(p); });
    for (auto& t : th) t.join();
  };
  auto exchange = [&]() {
    for (int round = 0; round < 8; ++round) {
      std::vector<std::vector<zbhip_xpart_cmd>> inbox(P);
      size_t total = 0;
      for (int s = 0; s < P; ++s) {
        for (auto& x : os[s]->outbox) inbox[x.target_partition - 1].push_back(x);
        total += os[s]->outbox.size();
        os[s]->outbox.clear();
      }
      if (!total) return;
      parallel([&](int t) {
        std::vector<zbhip_command> cs(inbox[t].size());
        for (size_t i = 0; i < inbox[t].size(); ++i) {
          const zbhip_xpart_cmd& x = inbox[t][i];
          const bool pms = x.kind == ZBHIP_CMD_PMS_CREATE || x.kind == ZBHIP_CMD_PMS_CORRELATE ||
                           x.kind == ZBHIP_CMD_PMS_DELETE;
          cs[i] = zbhip_command{};
          cs[i].instance = pms ? x.instance : x.correlation_key;
          cs[i].kind = x.kind;
          cs[i].doc_begin = (uint32_t)i;
        }
        os[t]->submit(cs.data(), cs.size(), nullptr, 0, inbox[t].data(), inbox[t].size());
        os[t]->run();
        os[t]->out.clear();
      });
    }
  };
  auto t0 = std::chrono::steady_clock::now();
  parallel([&](int p) {
    os[p]->submit(cmd[p].data(), cmd[p].size(), docs[p].data(), docs[p].size());
    os[p]->run();
    os[p]->out.clear();
  });
  exchange();
  parallel([&](int p) {
    os[p]->submit(pub[p].data(), pub[p].size(), nullptr, 0);
    os[p]->run();
    os[p]->out.clear();
  });
  exchange();
  double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  uint64_t tr = 0, cp = 0;
  for (auto& o : os) { tr += o->transitions; cp += o->completed_instances; }
  *transitions_out = tr;
  *completed_out = cp;
  return sec;
}

static double bench_impl(const char* xml, int threads, int n_instances, int phases, int var_name_kind, uint64_t seed,
                         const uint16_t* job_ords, int n_ords, uint64_t* transitions_out, uint64_t* completed_out);

double zbo_bench(const char* xml, int threads, int n_instances, int phases, int var_name_kind,
                 uint64_t seed, uint64_t* transitions_out, uint64_t* completed_out) {
  return bench_impl(xml, threads, n_instances, phases, var_name_kind, seed, nullptr, 0, transitions_out, completed_out);
}

// Variant 4b: every instance waits on n_ords jobs at once (their key ordinals in the
// CREATE batch) and completes them in its own random order, one per phase.
double zbo_bench_jobs(const char* xml, int threads, int n_instances, const uint16_t* job_ords, int n_ords,
                      uint64_t seed, uint64_t* transitions_out, uint64_t* completed_out) {
  return bench_impl(xml, threads, n_instances, n_ords, 0, seed, job_ords, n_ords, transitions_out, completed_out);
}

static double bench_impl(const char* xml, int threads, int n_instances, int phases, int var_name_kind, uint64_t seed,
                         const uint16_t* job_ords, int n_ords, uint64_t* transitions_out, uint64_t* completed_out) {
  std::vector<std::unique_ptr<Oracle>> os;
  std::vector<std::vector<zbhip_command>> creates(threads);
  std::vector<std::vector<zbhip_doc_entry>> docs(threads);
  for (int t = 0; t < threads; ++t) {
    os.emplace_back(new Oracle(t + 1, threads, 100, 0));
    if (os.back()->deploy(xml, 2251799813685249LL, 1) < 0) return -1.0;
    int name = os.back()->intern("amount");
    uint64_t s = seed + (uint64_t)t * 0x9E3779B97F4A7C15ULL;
    for (int i = 0; i < n_instances; ++i) {
      zbhip_command c{};
      c.instance = (uint32_t)i;
      c.kind = ZBHIP_CMD_CREATE;
      c.ref = 0;
      if (var_name_kind) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        zbhip_doc_entry d{};
        d.name_id = (uint32_t)name;
        d.type = ZBHIP_DOC_INT;
        d.value = (int64_t)(s % 2001);
        c.doc_begin = (uint32_t)docs[t].size();
        c.doc_count = 1;
        docs[t].push_back(d);
      }
      creates[t].push_back(c);
    }
  }
  // per instance a random order of its jobs (variant 4b)
  std::vector<std::vector<uint16_t>> order(threads);
  if (job_ords)
    for (int t = 0; t < threads; ++t) {
      uint64_t s = seed * 0x2545F4914F6CDD1DULL + (uint64_t)t + 1;
      order[t].resize((size_t)n_instances * n_ords);
      for (int i = 0; i < n_instances; ++i) {
        uint16_t* o = &order[t][(size_t)i * n_ords];
        for (int k = 0; k < n_ords; ++k) o[k] = (uint16_t)k;
        for (int k = n_ords - 1; k > 0; --k) {
          s ^= s << 13; s ^= s >> 7; s ^= s << 17;
          std::swap(o[k], o[s % (uint64_t)(k + 1)]);
        }
      }
    }
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t) {
    th.emplace_back([&, t]() {
      Oracle& O = *os[t];
      O.submit(creates[t].data(), creates[t].size(), docs[t].data(), docs[t].size());
      O.run();
      O.out.clear();
      for (int ph = 0; ph < phases; ++ph) {
        // complete the job each instance is waiting on (the last JOB:CREATED of the instance)
        std::vector<zbhip_command> cs;
        cs.reserve(n_instances);
        for (int i = 0; i < n_instances; ++i) {
          auto& ks = O.inst_keys[(uint32_t)i];
          zbhip_command c{};
          c.instance = (uint32_t)i;
          c.kind = ZBHIP_CMD_JOB_COMPLETE;
          c.ref = (uint16_t)(ks.size() - 1);  // the job key is the last key of the activating batch
          if (job_ords) c.ref = job_ords[order[t][(size_t)i * n_ords + ph]];
          cs.push_back(c);
        }
        O.submit(cs.data(), cs.size(), nullptr, 0);
        O.run();
        O.out.clear();
      }
    });
  }
  for (auto& x : th) x.join();
  double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  uint64_t tr = 0, cp = 0;
  for (auto& o : os) { tr += o->transitions; cp += o->completed_instances; }
  *transitions_out = tr;
  *completed_out = cp;
  return sec;
}

}  // extern "C"

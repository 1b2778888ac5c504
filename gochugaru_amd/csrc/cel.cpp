// cel.cpp — CEL subset with partial evaluation, and JSON caveat contexts (cel.hpp).
//
// Grammar (lowest to highest precedence): c ? a : b | || | && | == != < <= > >= in | + - |
// * / % | ! - (unary) | member access .f and index [k] | literals, identifiers, (e), [list].
// Values follow the JSON data model (null, bool, int, double, string, list, map). Partial
// evaluation: an identifier bound in neither context is UNKNOWN; && is false if either side is
// false and || true if either side is true, whatever the other side; ?: with an unknown
// condition is known only when both branches agree; every other operator with an unknown
// operand is unknown. Semantics are those of the test oracle's restatement
// (oracle/spicedb_ref.py cel_eval), which pins this file (tests/test_cel.py).
#include "cel.hpp"

#include <cctype>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include <arpa/inet.h>

#include "engine.hpp"

namespace gck {
namespace cel {

namespace {

[[noreturn]] void bad_json(const std::string& m) { throw Error(GCK_E_INVALID_ARGUMENT, "caveat context: " + m); }
[[noreturn]] void eval_error(const std::string& m) { throw Error(GCK_E_INVALID_ARGUMENT, "caveat evaluation: " + m); }

Value mk_bool(bool b) {
  Value v;
  v.k = Value::BOOL;
  v.b = b;
  return v;
}
Value mk_int(int64_t i) {
  Value v;
  v.k = Value::INT;
  v.i = i;
  return v;
}
Value mk_dbl(double d) {
  Value v;
  v.k = Value::DBL;
  v.d = d;
  return v;
}
Value mk_str(std::string s) {
  Value v;
  v.k = Value::STR;
  v.s = std::move(s);
  return v;
}

void put_utf8(std::string& out, uint32_t cp) {
  if (cp < 0x80) {
    out += (char)cp;
  } else if (cp < 0x800) {
    out += (char)(0xC0 | (cp >> 6));
    out += (char)(0x80 | (cp & 0x3F));
  } else if (cp < 0x10000) {
    out += (char)(0xE0 | (cp >> 12));
    out += (char)(0x80 | ((cp >> 6) & 0x3F));
    out += (char)(0x80 | (cp & 0x3F));
  } else {
    out += (char)(0xF0 | (cp >> 18));
    out += (char)(0x80 | ((cp >> 12) & 0x3F));
    out += (char)(0x80 | ((cp >> 6) & 0x3F));
    out += (char)(0x80 | (cp & 0x3F));
  }
}

// ---- JSON -------------------------------------------------------------------------------------
struct Json {
  const std::string& s;
  size_t i = 0;
  void ws() {
    while (i < s.size() && std::isspace((unsigned char)s[i])) ++i;
  }
  bool lit(const char* w) {
    size_t n = std::strlen(w);
    if (s.compare(i, n, w) == 0) {
      i += n;
      return true;
    }
    return false;
  }
  uint32_t hex4() {
    if (i + 4 > s.size()) bad_json("truncated \\u escape");
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = s[i++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else bad_json("bad \\u escape");
    }
    return v;
  }
  std::string str() {
    if (i >= s.size() || s[i] != '"') bad_json("expected a string");
    ++i;
    std::string out;
    for (;;) {
      if (i >= s.size()) bad_json("unterminated string");
      char c = s[i++];
      if (c == '"') return out;
      if (c != '\\') {
        out += c;
        continue;
      }
      if (i >= s.size()) bad_json("unterminated escape");
      char e = s[i++];
      switch (e) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && i + 6 <= s.size() && s[i] == '\\' && s[i + 1] == 'u') {
            i += 2;
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(out, cp);
          break;
        }
        default: bad_json(std::string("bad escape \\") + e);
      }
    }
  }
  Value value() {
    ws();
    if (i >= s.size()) bad_json("unexpected end");
    char c = s[i];
    if (c == '{') {
      ++i;
      auto m = std::make_shared<Object>();
      ws();
      if (i < s.size() && s[i] == '}') {
        ++i;
      } else {
        for (;;) {
          ws();
          std::string k = str();
          ws();
          if (i >= s.size() || s[i] != ':') bad_json("expected ':'");
          ++i;
          (*m)[k] = value();  // a repeated key keeps the last value (Python json.loads)
          ws();
          if (i < s.size() && s[i] == ',') {
            ++i;
            continue;
          }
          if (i < s.size() && s[i] == '}') {
            ++i;
            break;
          }
          bad_json("expected ',' or '}'");
        }
      }
      Value v;
      v.k = Value::MAP;
      v.m = m;
      return v;
    }
    if (c == '[') {
      ++i;
      auto l = std::make_shared<std::vector<Value>>();
      ws();
      if (i < s.size() && s[i] == ']') {
        ++i;
      } else {
        for (;;) {
          l->push_back(value());
          ws();
          if (i < s.size() && s[i] == ',') {
            ++i;
            continue;
          }
          if (i < s.size() && s[i] == ']') {
            ++i;
            break;
          }
          bad_json("expected ',' or ']'");
        }
      }
      Value v;
      v.k = Value::LIST;
      v.l = l;
      return v;
    }
    if (c == '"') return mk_str(str());
    if (lit("true")) return mk_bool(true);
    if (lit("false")) return mk_bool(false);
    if (lit("null")) {
      Value v;
      v.k = Value::NUL;
      return v;
    }
    if (c == '-' || std::isdigit((unsigned char)c)) {
      size_t b = i;
      bool is_float = false;
      if (s[i] == '-') ++i;
      while (i < s.size() && std::isdigit((unsigned char)s[i])) ++i;
      if (i < s.size() && s[i] == '.') {
        is_float = true;
        ++i;
        while (i < s.size() && std::isdigit((unsigned char)s[i])) ++i;
      }
      if (i < s.size() && (s[i] == 'e' || s[i] == 'E')) {
        is_float = true;
        ++i;
        if (i < s.size() && (s[i] == '+' || s[i] == '-')) ++i;
        while (i < s.size() && std::isdigit((unsigned char)s[i])) ++i;
      }
      std::string t = s.substr(b, i - b);
      if (t == "-" || t.empty()) bad_json("bad number");
      if (!is_float) {
        errno = 0;
        long long v = std::strtoll(t.c_str(), nullptr, 10);
        if (errno == 0) return mk_int(v);
      }
      return mk_dbl(std::strtod(t.c_str(), nullptr));
    }
    bad_json(std::string("unexpected character '") + c + "'");
  }
};

// ---- CEL lexer / parser -----------------------------------------------------------------------
struct Tok {
  enum K { IDENT, OP, STR, NUM, END } k;
  std::string v;
};

std::vector<Tok> lex(const std::string& s) {
  std::vector<Tok> out;
  size_t i = 0, n = s.size();
  while (i < n) {
    char c = s[i];
    if (std::isspace((unsigned char)c)) {
      ++i;
      continue;
    }
    if (std::isalpha((unsigned char)c) || c == '_') {
      size_t b = i;
      while (i < n && (std::isalnum((unsigned char)s[i]) || s[i] == '_')) ++i;
      out.push_back({Tok::IDENT, s.substr(b, i - b)});
      continue;
    }
    if (std::isdigit((unsigned char)c)) {
      size_t b = i;
      while (i < n && std::isdigit((unsigned char)s[i])) ++i;
      if (i + 1 < n && s[i] == '.' && std::isdigit((unsigned char)s[i + 1])) {
        ++i;
        while (i < n && std::isdigit((unsigned char)s[i])) ++i;
      }
      out.push_back({Tok::NUM, s.substr(b, i - b)});
      continue;
    }
    if (c == '"' || c == '\'') {
      size_t b = i++;
      while (i < n && s[i] != c) i += (s[i] == '\\') ? 2 : 1;
      if (i >= n) throw Error(GCK_E_SCHEMA, "caveat: unterminated string literal");
      ++i;
      out.push_back({Tok::STR, s.substr(b, i - b)});
      continue;
    }
    static const char* two[] = {"==", "!=", "<=", ">=", "&&", "||"};
    bool done = false;
    for (const char* t : two) {
      if (s.compare(i, 2, t) == 0) {
        out.push_back({Tok::OP, t});
        i += 2;
        done = true;
        break;
      }
    }
    if (done) continue;
    if (std::strchr("()[]:+-*/%<>!.,?", c)) {
      out.push_back({Tok::OP, std::string(1, c)});
      ++i;
      continue;
    }
    throw Error(GCK_E_SCHEMA, std::string("caveat: unexpected character '") + c + "'");
  }
  out.push_back({Tok::END, ""});
  return out;
}

// String literal body -> bytes (the common escapes; \xHH and \uXXXX as code points).
std::string unquote(const std::string& t) {
  std::string out;
  const std::string b = t.substr(1, t.size() - 2);
  for (size_t i = 0; i < b.size(); ++i) {
    if (b[i] != '\\' || i + 1 >= b.size()) {
      out += b[i];
      continue;
    }
    char e = b[++i];
    auto hexn = [&](int n) {
      uint32_t v = 0;
      for (int k = 0; k < n && i + 1 < b.size(); ++k) {
        char c = b[++i];
        v = v * 16 + (std::isdigit((unsigned char)c) ? c - '0' : (std::tolower(c) - 'a' + 10));
      }
      return v;
    };
    switch (e) {
      case 'n': out += '\n'; break;
      case 't': out += '\t'; break;
      case 'r': out += '\r'; break;
      case '\\': out += '\\'; break;
      case '\'': out += '\''; break;
      case '"': out += '"'; break;
      case 'x': put_utf8(out, hexn(2)); break;
      case 'u': put_utf8(out, hexn(4)); break;
      default:
        out += '\\';
        out += e;
    }
  }
  return out;
}

}  // namespace

struct Node {
  enum Op { LIT, VAR, LIST, AND, OR, COND, NOT, NEG, FIELD, INDEX, EQ, NE, LT, LE, GT, GE, IN, ADD, SUB, MUL, DIV, MOD,
            CALL, HAS };
  Op op = LIT;
  Value lit;
  std::string name;  // VAR / FIELD / CALL (function or method name) / HAS (field)
  std::vector<std::shared_ptr<const Node>> kids;  // CALL: [receiver,] arguments
  bool method = false;                             // CALL: receiver.name(args)
  Value::Kind conv = Value::UNKNOWN;               // VAR: declared timestamp / duration / ipaddress
};

namespace {

using NodeP = std::shared_ptr<const Node>;

NodeP mk(Node::Op op, std::vector<NodeP> kids, std::string name = "") {
  auto n = std::make_shared<Node>();
  n->op = op;
  n->kids = std::move(kids);
  n->name = std::move(name);
  return n;
}

class Parser {
 public:
  Parser(const std::string& body, const std::vector<std::pair<std::string, std::string>>& params) : t_(lex(body)) {
    for (const auto& p : params) {
      if (p.second == "timestamp") conv_[p.first] = Value::TS;
      if (p.second == "duration") conv_[p.first] = Value::DUR;
      if (p.second == "ipaddress") conv_[p.first] = Value::IP;
    }
  }
  NodeP parse() {
    NodeP e = ternary();
    if (peek().k != Tok::END) fail("trailing tokens: '" + peek().v + "'");
    return e;
  }

 private:
  std::vector<Tok> t_;
  size_t i_ = 0;
  std::map<std::string, Value::Kind> conv_;
  std::vector<NodeP> args() {  // after '(' up to and including ')'
    std::vector<NodeP> out;
    while (!is_op(")")) {
      if (peek().k == Tok::END) fail("unterminated argument list");
      out.push_back(ternary());
      if (is_op(",")) ++i_;
      else if (!is_op(")")) fail("expected ',' or ')'");
    }
    ++i_;
    return out;
  }
  const Tok& peek() const { return t_[std::min(i_, t_.size() - 1)]; }
  bool is_op(const char* v) const { return peek().k == Tok::OP && peek().v == v; }
  [[noreturn]] void fail(const std::string& m) const { throw Error(GCK_E_SCHEMA, "caveat expression: " + m); }
  void expect(const char* v) {
    if (!is_op(v)) fail(std::string("expected '") + v + "'");
    ++i_;
  }

  NodeP ternary() {
    NodeP c = lor();
    if (is_op("?")) {
      ++i_;
      NodeP a = ternary();
      expect(":");
      NodeP b = ternary();
      return mk(Node::COND, {c, a, b});
    }
    return c;
  }
  NodeP lor() {
    NodeP e = land();
    while (is_op("||")) {
      ++i_;
      e = mk(Node::OR, {e, land()});
    }
    return e;
  }
  NodeP land() {
    NodeP e = rel();
    while (is_op("&&")) {
      ++i_;
      e = mk(Node::AND, {e, rel()});
    }
    return e;
  }
  NodeP rel() {
    NodeP e = add();
    for (;;) {
      static const std::pair<const char*, Node::Op> ops[] = {{"==", Node::EQ}, {"!=", Node::NE}, {"<", Node::LT},
                                                             {"<=", Node::LE}, {">", Node::GT}, {">=", Node::GE}};
      Node::Op op = Node::LIT;
      for (auto& o : ops)
        if (is_op(o.first)) op = o.second;
      if (op == Node::LIT && peek().k == Tok::IDENT && peek().v == "in") op = Node::IN;
      if (op == Node::LIT) return e;
      ++i_;
      e = mk(op, {e, add()});
    }
  }
  NodeP add() {
    NodeP e = mul();
    while (is_op("+") || is_op("-")) {
      Node::Op op = is_op("+") ? Node::ADD : Node::SUB;
      ++i_;
      e = mk(op, {e, mul()});
    }
    return e;
  }
  NodeP mul() {
    NodeP e = unary();
    while (is_op("*") || is_op("/") || is_op("%")) {
      Node::Op op = is_op("*") ? Node::MUL : is_op("/") ? Node::DIV : Node::MOD;
      ++i_;
      e = mk(op, {e, unary()});
    }
    return e;
  }
  NodeP unary() {
    if (is_op("!")) {
      ++i_;
      return mk(Node::NOT, {unary()});
    }
    if (is_op("-")) {
      ++i_;
      return mk(Node::NEG, {unary()});
    }
    return member();
  }
  NodeP member() {
    NodeP e = primary();
    for (;;) {
      if (is_op(".")) {
        ++i_;
        if (peek().k != Tok::IDENT) fail("expected a field name");
        const std::string f = t_[i_++].v;
        if (is_op("(")) {  // method call
          ++i_;
          std::vector<NodeP> kids{e};
          for (NodeP& a : args()) kids.push_back(std::move(a));
          auto n = std::make_shared<Node>();
          n->op = Node::CALL;
          n->name = f;
          n->kids = std::move(kids);
          n->method = true;
          e = n;
        } else {
          e = mk(Node::FIELD, {e}, f);
        }
      } else if (is_op("[")) {
        ++i_;
        NodeP k = ternary();
        expect("]");
        e = mk(Node::INDEX, {e, k});
      } else {
        return e;
      }
    }
  }
  NodeP primary() {
    const Tok t = peek();
    ++i_;
    auto lit = [](Value v) {
      auto n = std::make_shared<Node>();
      n->op = Node::LIT;
      n->lit = std::move(v);
      return NodeP(n);
    };
    if (t.k == Tok::NUM) {
      if (t.v.find('.') != std::string::npos) return lit(mk_dbl(std::strtod(t.v.c_str(), nullptr)));
      return lit(mk_int(std::strtoll(t.v.c_str(), nullptr, 10)));
    }
    if (t.k == Tok::STR) return lit(mk_str(unquote(t.v)));
    if (t.k == Tok::IDENT) {
      if (t.v == "true") return lit(mk_bool(true));
      if (t.v == "false") return lit(mk_bool(false));
      if (t.v == "null") {
        Value v;
        v.k = Value::NUL;
        return lit(v);
      }
      if (is_op("(")) {  // global function, or the has() macro
        ++i_;
        std::vector<NodeP> a = args();
        if (t.v == "has") {
          if (a.size() != 1 || a[0]->op != Node::FIELD) fail("has() takes one field selection");
          return mk(Node::HAS, {a[0]->kids[0]}, a[0]->name);
        }
        return mk(Node::CALL, std::move(a), t.v);
      }
      auto n = std::make_shared<Node>();
      n->op = Node::VAR;
      n->name = t.v;
      auto c = conv_.find(t.v);
      if (c != conv_.end()) n->conv = c->second;
      return NodeP(n);
    }
    if (t.k == Tok::OP && t.v == "(") {
      NodeP e = ternary();
      expect(")");
      return e;
    }
    if (t.k == Tok::OP && t.v == "[") {
      std::vector<NodeP> items;
      while (!is_op("]")) {
        if (peek().k == Tok::END) fail("unterminated list");
        items.push_back(ternary());
        if (is_op(",")) ++i_;
      }
      ++i_;
      return mk(Node::LIST, std::move(items));
    }
    fail("unexpected token '" + t.v + "'");
  }
};

// ---- evaluation ---------------------------------------------------------------------------------
bool numeric(const Value& v) { return v.k == Value::BOOL || v.k == Value::INT || v.k == Value::DBL; }
bool integral(const Value& v) { return v.k == Value::BOOL || v.k == Value::INT; }
int64_t as_int(const Value& v) { return v.k == Value::BOOL ? (v.b ? 1 : 0) : v.i; }
double as_dbl(const Value& v) { return v.k == Value::DBL ? v.d : (double)as_int(v); }

bool truthy(const Value& v) {
  switch (v.k) {
    case Value::NUL: return false;
    case Value::BOOL: return v.b;
    case Value::INT: return v.i != 0;
    case Value::DBL: return v.d != 0;
    case Value::STR: return !v.s.empty();
    case Value::LIST: return !v.l->empty();
    case Value::MAP: return !v.m->empty();
    case Value::TS:
    case Value::DUR:
    case Value::IP: return true;
    default: return false;
  }
}

bool equal(const Value& a, const Value& b) {
  if (numeric(a) && numeric(b)) {
    if (integral(a) && integral(b)) return as_int(a) == as_int(b);
    return as_dbl(a) == as_dbl(b);
  }
  if (a.k != b.k) return false;
  switch (a.k) {
    case Value::NUL: return true;
    case Value::STR:
    case Value::IP: return a.s == b.s;
    case Value::TS:
    case Value::DUR: return a.i == b.i;
    case Value::LIST: {
      if (a.l->size() != b.l->size()) return false;
      for (size_t k = 0; k < a.l->size(); ++k)
        if (!equal((*a.l)[k], (*b.l)[k])) return false;
      return true;
    }
    case Value::MAP: {
      if (a.m->size() != b.m->size()) return false;
      for (const auto& kv : *a.m) {
        auto it = b.m->find(kv.first);
        if (it == b.m->end() || !equal(kv.second, it->second)) return false;
      }
      return true;
    }
    default: return false;
  }
}

// -1 / 0 / 1; numbers, strings and lists (lexicographic) are ordered, anything else is an error
int compare(const Value& a, const Value& b) {
  if (numeric(a) && numeric(b)) {
    if (integral(a) && integral(b)) return as_int(a) < as_int(b) ? -1 : as_int(a) > as_int(b);
    const double x = as_dbl(a), y = as_dbl(b);
    return x < y ? -1 : x > y;
  }
  if (a.k == Value::STR && b.k == Value::STR) return a.s < b.s ? -1 : a.s > b.s;
  if ((a.k == Value::TS || a.k == Value::DUR) && a.k == b.k) return a.i < b.i ? -1 : a.i > b.i;
  if (a.k == Value::LIST && b.k == Value::LIST) {
    const size_t n = std::min(a.l->size(), b.l->size());
    for (size_t k = 0; k < n; ++k) {
      if (equal((*a.l)[k], (*b.l)[k])) continue;
      return compare((*a.l)[k], (*b.l)[k]);
    }
    return a.l->size() < b.l->size() ? -1 : a.l->size() > b.l->size();
  }
  eval_error("ordering is not defined between these values");
}

int64_t floor_div(int64_t a, int64_t b) {
  int64_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  return q;
}

// ---- timestamps, durations, IP addresses (CEL standard functions + SpiceDB's ipaddress) -----
constexpr int64_t kUsPerSec = 1000000;

int64_t days_from_civil(int64_t y, int64_t m, int64_t d) {  // proleptic Gregorian
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const int64_t yoe = y - era * 400;
  const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  return era * 146097 + yoe * 365 + yoe / 4 - yoe / 100 + doy - 719468;
}

void civil_from_days(int64_t z, int64_t& y, int64_t& m, int64_t& d) {
  z += 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const int64_t doe = z - era * 146097;
  const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const int64_t mp = (5 * doy + 2) / 153;
  d = doy - (153 * mp + 2) / 5 + 1;
  m = mp < 10 ? mp + 3 : mp - 9;
  y = yoe + era * 400 + (m <= 2);
}

// RFC 3339: YYYY-MM-DDTHH:MM:SS[.frac](Z|+HH:MM|-HH:MM); fractions below 1 µs are truncated
bool parse_rfc3339(const std::string& t, int64_t& us) {
  auto dig = [&](size_t at, size_t n, int64_t& v) {
    if (at + n > t.size()) return false;
    v = 0;
    for (size_t k = at; k < at + n; ++k) {
      if (!std::isdigit((unsigned char)t[k])) return false;
      v = v * 10 + (t[k] - '0');
    }
    return true;
  };
  int64_t Y, M, D, h, mi, se;
  if (!dig(0, 4, Y) || t.size() < 20 || t[4] != '-' || !dig(5, 2, M) || t[7] != '-' || !dig(8, 2, D) ||
      (t[10] != 'T' && t[10] != 't') || !dig(11, 2, h) || t[13] != ':' || !dig(14, 2, mi) || t[16] != ':' ||
      !dig(17, 2, se))
    return false;
  static const int mdays[] = {31, 29, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  const bool leap = (Y % 4 == 0 && Y % 100 != 0) || Y % 400 == 0;
  if (Y < 1 || M < 1 || M > 12 || D < 1 || D > mdays[M - 1] || (M == 2 && D == 29 && !leap) || h > 23 || mi > 59 || se > 59)
    return false;
  size_t i = 19;
  int64_t frac = 0;
  if (i < t.size() && t[i] == '.') {
    ++i;
    size_t nd = 0;
    while (i < t.size() && std::isdigit((unsigned char)t[i])) {
      if (nd < 6) frac = frac * 10 + (t[i] - '0');
      ++nd;
      ++i;
    }
    if (nd == 0) return false;
    for (size_t k = nd; k < 6; ++k) frac *= 10;
  }
  int64_t off = 0;
  if (i < t.size() && (t[i] == 'Z' || t[i] == 'z')) {
    ++i;
  } else if (i < t.size() && (t[i] == '+' || t[i] == '-')) {
    int64_t oh, om;
    if (!dig(i + 1, 2, oh) || i + 3 >= t.size() || t[i + 3] != ':' || !dig(i + 4, 2, om) || oh > 23 || om > 59)
      return false;
    off = (t[i] == '-' ? -1 : 1) * (oh * 3600 + om * 60);
    i += 6;
  } else {
    return false;
  }
  if (i != t.size()) return false;
  us = ((days_from_civil(Y, M, D) * 86400 + h * 3600 + mi * 60 + se) - off) * kUsPerSec + frac;
  return true;
}

// Go duration syntax ("1h30m", "-1.5s", "300ms", "0"): units ns us µs ms s m h; the value is
// truncated toward zero to whole microseconds
bool parse_duration(const std::string& t, int64_t& us) {
  size_t i = 0;
  bool neg = false;
  if (i < t.size() && (t[i] == '-' || t[i] == '+')) neg = t[i++] == '-';
  if (t.substr(i) == "0") {
    us = 0;
    return true;
  }
  if (i == t.size()) return false;
  __int128 ns = 0;
  while (i < t.size()) {
    __int128 whole = 0, frac = 0, scale = 1;
    size_t nd = 0;
    while (i < t.size() && std::isdigit((unsigned char)t[i])) {
      whole = whole * 10 + (t[i++] - '0');
      ++nd;
      if (whole > ((__int128)1 << 80)) return false;
    }
    if (i < t.size() && t[i] == '.') {
      ++i;
      while (i < t.size() && std::isdigit((unsigned char)t[i])) {
        if (scale < (__int128)1000000000000000000ll) {
          frac = frac * 10 + (t[i] - '0');
          scale *= 10;
        }
        ++i;
        ++nd;
      }
    }
    if (nd == 0) return false;
    static const std::pair<const char*, int64_t> units[] = {
        {"ns", 1}, {"us", 1000}, {"\xC2\xB5s", 1000}, {"ms", 1000000}, {"s", 1000000000ll},
        {"m", 60000000000ll}, {"h", 3600000000000ll}};
    int64_t unit = 0;
    size_t ul = 0;
    for (const auto& u : units) {
      const size_t l = std::strlen(u.first);
      if (t.compare(i, l, u.first) == 0 && l > ul && !(l == 1 && u.first[0] == 'm' && t.compare(i, 2, "ms") == 0)) {
        unit = u.second;
        ul = l;
      }
    }
    if (!unit) return false;
    i += ul;
    ns += whole * unit + frac * unit / scale;
    if (ns > ((__int128)1 << 100)) return false;
  }
  const __int128 v = ns / 1000;
  if (v > (__int128)INT64_MAX / 2) return false;
  us = neg ? -(int64_t)v : (int64_t)v;
  return true;
}

bool parse_ip(const std::string& t, std::string& out) {
  unsigned char b[16];
  if (t.find(':') == std::string::npos) {
    // dotted quad, decimal octets without leading zeros
    int64_t parts[4];
    size_t i = 0;
    for (int k = 0; k < 4; ++k) {
      if (k && (i >= t.size() || t[i++] != '.')) return false;
      const size_t b0 = i;
      int64_t v = 0;
      while (i < t.size() && std::isdigit((unsigned char)t[i]) && i - b0 < 4) v = v * 10 + (t[i++] - '0');
      if (i == b0 || v > 255 || (i - b0 > 1 && t[b0] == '0')) return false;
      parts[k] = v;
    }
    if (i != t.size()) return false;
    out.assign(4, '\0');
    for (int k = 0; k < 4; ++k) out[k] = (char)parts[k];
    return true;
  }
  if (inet_pton(AF_INET6, t.c_str(), b) != 1) return false;
  out.assign(reinterpret_cast<const char*>(b), 16);
  return true;
}

bool in_cidr(const std::string& ip, const std::string& cidr) {
  const size_t slash = cidr.find('/');
  std::string net;
  if (slash == std::string::npos || !parse_ip(cidr.substr(0, slash), net)) eval_error("invalid CIDR '" + cidr + "'");
  const std::string bits = cidr.substr(slash + 1);
  if (bits.empty() || bits.size() > 3 || bits.find_first_not_of("0123456789") != std::string::npos)
    eval_error("invalid CIDR '" + cidr + "'");
  const int n = std::atoi(bits.c_str());
  if (n > (int)net.size() * 8) eval_error("invalid CIDR '" + cidr + "'");
  if (ip.size() != net.size()) return false;
  for (int k = 0; k < n; ++k) {
    const int byte = k / 8, bit = 7 - k % 8;
    if (((ip[byte] >> bit) & 1) != ((net[byte] >> bit) & 1)) return false;
  }
  return true;
}

Value mk_kind(Value::Kind k, int64_t i) {
  Value v;
  v.k = k;
  v.i = i;
  return v;
}

struct Env {
  const Object* stored;
  const Object* check;
  Value lookup(const std::string& n) const {
    if (stored) {
      auto it = stored->find(n);
      if (it != stored->end()) return it->second;
    }
    if (check) {
      auto it = check->find(n);
      if (it != check->end()) return it->second;
    }
    return Value{};
  }
};

Value call(const Node& e, const Env& env);

Value eval(const Node& e, const Env& env) {
  using V = Value;
  switch (e.op) {
    case Node::LIT: return e.lit;
    case Node::VAR: {
      V v = env.lookup(e.name);
      if (e.conv == V::UNKNOWN || v.k == V::UNKNOWN || v.k == e.conv) return v;
      if (v.k != V::STR) eval_error("parameter '" + e.name + "' has the wrong type");
      V out;
      out.k = e.conv;
      const bool ok = e.conv == V::TS ? parse_rfc3339(v.s, out.i)
                      : e.conv == V::DUR ? parse_duration(v.s, out.i)
                                         : parse_ip(v.s, out.s);
      if (!ok) eval_error("parameter '" + e.name + "': cannot convert '" + v.s + "'");
      return out;
    }
    case Node::HAS: {
      const V a = eval(*e.kids[0], env);
      if (a.k == V::UNKNOWN) return V{};
      if (a.k != V::MAP) eval_error("has() on a non-map");
      return mk_bool(a.m->count(e.name) > 0);
    }
    case Node::CALL: return call(e, env);
    case Node::LIST: {
      auto l = std::make_shared<std::vector<Value>>();
      bool unk = false;
      for (const NodeP& k : e.kids) {
        l->push_back(eval(*k, env));
        unk |= l->back().k == V::UNKNOWN;
      }
      if (unk) return V{};
      V v;
      v.k = V::LIST;
      v.l = l;
      return v;
    }
    case Node::AND:
    case Node::OR: {
      const V a = eval(*e.kids[0], env), b = eval(*e.kids[1], env);  // no short circuit
      const bool dom = e.op == Node::OR;  // the value that decides regardless of the other side
      if ((a.k == V::BOOL && a.b == dom) || (b.k == V::BOOL && b.b == dom)) return mk_bool(dom);
      if (a.k == V::UNKNOWN || b.k == V::UNKNOWN) return V{};
      return mk_bool(e.op == Node::OR ? (truthy(a) || truthy(b)) : (truthy(a) && truthy(b)));
    }
    case Node::COND: {
      const V c = eval(*e.kids[0], env);
      if (c.k == V::UNKNOWN) {
        const V a = eval(*e.kids[1], env), b = eval(*e.kids[2], env);
        return (a.k != V::UNKNOWN && b.k != V::UNKNOWN && equal(a, b)) ? a : V{};
      }
      return eval(*e.kids[truthy(c) ? 1 : 2], env);
    }
    case Node::NOT: {
      const V a = eval(*e.kids[0], env);
      return a.k == V::UNKNOWN ? V{} : mk_bool(!truthy(a));
    }
    case Node::NEG: {
      const V a = eval(*e.kids[0], env);
      if (a.k == V::UNKNOWN) return V{};
      if (integral(a)) return mk_int(-as_int(a));
      if (a.k == V::DBL) return mk_dbl(-a.d);
      eval_error("unary '-' on a non-number");
    }
    case Node::FIELD: {
      const V a = eval(*e.kids[0], env);
      if (a.k != V::MAP) return V{};
      auto it = a.m->find(e.name);
      return it == a.m->end() ? V{} : it->second;
    }
    default: break;
  }
  const V a = eval(*e.kids[0], env), b = eval(*e.kids[1], env);
  if (a.k == V::UNKNOWN || b.k == V::UNKNOWN) return V{};
  switch (e.op) {
    case Node::INDEX:
      if (a.k == V::LIST && integral(b)) {
        int64_t k = as_int(b), n = (int64_t)a.l->size();
        if (k < 0) k += n;
        if (k < 0 || k >= n) eval_error("list index out of range");
        return (*a.l)[(size_t)k];
      }
      if (a.k == V::MAP && b.k == V::STR) {
        auto it = a.m->find(b.s);
        if (it == a.m->end()) eval_error("no such key '" + b.s + "'");
        return it->second;
      }
      if (a.k == V::STR && integral(b)) {
        int64_t k = as_int(b), n = (int64_t)a.s.size();
        if (k < 0) k += n;
        if (k < 0 || k >= n) eval_error("string index out of range");
        return mk_str(a.s.substr((size_t)k, 1));
      }
      eval_error("invalid index operation");
    case Node::EQ: return mk_bool(equal(a, b));
    case Node::NE: return mk_bool(!equal(a, b));
    case Node::LT: return mk_bool(compare(a, b) < 0);
    case Node::LE: return mk_bool(compare(a, b) <= 0);
    case Node::GT: return mk_bool(compare(a, b) > 0);
    case Node::GE: return mk_bool(compare(a, b) >= 0);
    case Node::IN:
      if (b.k == V::LIST) {
        for (const V& x : *b.l)
          if (equal(a, x)) return mk_bool(true);
        return mk_bool(false);
      }
      if (b.k == V::MAP) return mk_bool(a.k == V::STR && b.m->count(a.s) > 0);
      if (b.k == V::STR && a.k == V::STR) return mk_bool(b.s.find(a.s) != std::string::npos);
      eval_error("'in' needs a list, map or string");
    case Node::ADD:
      if (a.k == V::DUR && b.k == V::DUR) return mk_kind(V::DUR, a.i + b.i);
      if (a.k == V::TS && b.k == V::DUR) return mk_kind(V::TS, a.i + b.i);
      if (a.k == V::DUR && b.k == V::TS) return mk_kind(V::TS, a.i + b.i);
      if (integral(a) && integral(b)) return mk_int(as_int(a) + as_int(b));
      if (numeric(a) && numeric(b)) return mk_dbl(as_dbl(a) + as_dbl(b));
      if (a.k == V::STR && b.k == V::STR) return mk_str(a.s + b.s);
      if (a.k == V::LIST && b.k == V::LIST) {
        auto l = std::make_shared<std::vector<Value>>(*a.l);
        l->insert(l->end(), b.l->begin(), b.l->end());
        V v;
        v.k = V::LIST;
        v.l = l;
        return v;
      }
      eval_error("'+' on incompatible values");
    case Node::SUB:
      if (a.k == V::TS && b.k == V::TS) return mk_kind(V::DUR, a.i - b.i);
      if (a.k == V::TS && b.k == V::DUR) return mk_kind(V::TS, a.i - b.i);
      if (a.k == V::DUR && b.k == V::DUR) return mk_kind(V::DUR, a.i - b.i);
      [[fallthrough]];
    case Node::MUL:
      if (!numeric(a) || !numeric(b)) eval_error("arithmetic on a non-number");
      if (integral(a) && integral(b))
        return mk_int(e.op == Node::SUB ? as_int(a) - as_int(b) : as_int(a) * as_int(b));
      return mk_dbl(e.op == Node::SUB ? as_dbl(a) - as_dbl(b) : as_dbl(a) * as_dbl(b));
    case Node::DIV:
      if (!numeric(a) || !numeric(b)) eval_error("arithmetic on a non-number");
      if (integral(a) && integral(b)) {
        if (as_int(b) == 0) eval_error("division by zero");
        return mk_int(floor_div(as_int(a), as_int(b)));
      }
      if (as_dbl(b) == 0) eval_error("division by zero");
      return mk_dbl(as_dbl(a) / as_dbl(b));
    case Node::MOD:
      if (!numeric(a) || !numeric(b)) eval_error("arithmetic on a non-number");
      if (integral(a) && integral(b)) {
        if (as_int(b) == 0) eval_error("modulo by zero");
        return mk_int(as_int(a) - floor_div(as_int(a), as_int(b)) * as_int(b));
      } else {
        const double x = as_dbl(a), y = as_dbl(b);
        if (y == 0) eval_error("modulo by zero");
        double r = std::fmod(x, y);
        if (r != 0 && ((r < 0) != (y < 0))) r += y;
        return mk_dbl(r);
      }
    default: eval_error("unsupported operator");
  }
}

size_t utf8_len(const std::string& s) {
  size_t n = 0;
  for (unsigned char c : s) n += (c & 0xC0) != 0x80;
  return n;
}

// Function and method calls: size, startsWith / endsWith / contains, int / double / string,
// timestamp / duration and their UTC accessors, ipaddress / in_cidr. An unknown argument or
// receiver makes the call unknown.
Value call(const Node& e, const Env& env) {
  using V = Value;
  std::vector<V> a;
  for (const NodeP& k : e.kids) {
    a.push_back(eval(*k, env));
    if (a.back().k == V::UNKNOWN) return V{};
  }
  const std::string& f = e.name;
  auto want = [&](size_t n) {
    if (a.size() != n) eval_error(f + "(): wrong number of arguments");
  };
  if (f == "size") {
    want(1);
    const V& x = a[0];
    if (x.k == V::STR) return mk_int((int64_t)utf8_len(x.s));
    if (x.k == V::LIST) return mk_int((int64_t)x.l->size());
    if (x.k == V::MAP) return mk_int((int64_t)x.m->size());
    eval_error("size() of a value without a size");
  }
  if (e.method && (f == "startsWith" || f == "endsWith" || f == "contains")) {
    want(2);
    if (a[0].k != V::STR || a[1].k != V::STR) eval_error(f + "() needs strings");
    const std::string &x = a[0].s, &y = a[1].s;
    if (f == "contains") return mk_bool(x.find(y) != std::string::npos);
    if (y.size() > x.size()) return mk_bool(false);
    return mk_bool(f == "startsWith" ? x.compare(0, y.size(), y) == 0 : x.compare(x.size() - y.size(), y.size(), y) == 0);
  }
  if (!e.method && f == "timestamp") {
    want(1);
    if (a[0].k == V::TS) return a[0];
    int64_t us;
    if (a[0].k != V::STR || !parse_rfc3339(a[0].s, us)) eval_error("timestamp(): not an RFC 3339 string");
    return mk_kind(V::TS, us);
  }
  if (!e.method && f == "duration") {
    want(1);
    if (a[0].k == V::DUR) return a[0];
    int64_t us;
    if (a[0].k != V::STR || !parse_duration(a[0].s, us)) eval_error("duration(): not a duration string");
    return mk_kind(V::DUR, us);
  }
  if (!e.method && f == "ipaddress") {
    want(1);
    V v;
    v.k = V::IP;
    if (a[0].k != V::STR || !parse_ip(a[0].s, v.s)) eval_error("ipaddress(): not an IP address");
    return v;
  }
  if (e.method && f == "in_cidr") {
    want(2);
    if (a[0].k != V::IP || a[1].k != V::STR) eval_error("in_cidr() needs an ipaddress and a string");
    return mk_bool(in_cidr(a[0].s, a[1].s));
  }
  if (!e.method && f == "int") {
    want(1);
    const V& x = a[0];
    if (x.k == V::INT) return x;
    if (x.k == V::DBL) {
      if (!(x.d > -9.2e18 && x.d < 9.2e18)) eval_error("int(): out of range");
      return mk_int((int64_t)x.d);  // toward zero
    }
    if (x.k == V::STR) {
      const std::string& t = x.s;
      size_t i = (!t.empty() && (t[0] == '-' || t[0] == '+')) ? 1 : 0;
      if (i == t.size() || t.size() - i > 18 || t.find_first_not_of("0123456789", i) != std::string::npos)
        eval_error("int(): not an integer string");
      return mk_int(std::strtoll(t.c_str(), nullptr, 10));
    }
    if (x.k == V::TS) return mk_int(floor_div(x.i, kUsPerSec));
    eval_error("int(): unsupported argument");
  }
  if (!e.method && f == "double") {
    want(1);
    const V& x = a[0];
    if (x.k == V::DBL) return x;
    if (x.k == V::INT) return mk_dbl((double)x.i);
    eval_error("double(): unsupported argument");
  }
  if (!e.method && f == "string") {
    want(1);
    const V& x = a[0];
    if (x.k == V::STR) return x;
    if (x.k == V::INT) return mk_str(std::to_string(x.i));
    if (x.k == V::BOOL) return mk_str(x.b ? "true" : "false");
    eval_error("string(): unsupported argument");
  }
  if (e.method && a[0].k == V::TS && a.size() == 1) {
    const int64_t secs = floor_div(a[0].i, kUsPerSec), days = floor_div(secs, 86400), sod = secs - days * 86400;
    int64_t y, m, d;
    civil_from_days(days, y, m, d);
    if (f == "getFullYear") return mk_int(y);
    if (f == "getMonth") return mk_int(m - 1);
    if (f == "getDate") return mk_int(d);
    if (f == "getDayOfMonth") return mk_int(d - 1);
    if (f == "getDayOfWeek") return mk_int(((days % 7) + 11) % 7);  // 1970-01-01 was a Thursday
    if (f == "getDayOfYear") return mk_int(days - days_from_civil(y, 1, 1));
    if (f == "getHours") return mk_int(sod / 3600);
    if (f == "getMinutes") return mk_int(sod / 60 % 60);
    if (f == "getSeconds") return mk_int(sod % 60);
    if (f == "getMilliseconds") return mk_int((a[0].i - secs * kUsPerSec) / 1000);
  }
  if (e.method && a[0].k == V::DUR && a.size() == 1) {  // totals, truncated toward zero
    const int64_t us = a[0].i;
    if (f == "getHours") return mk_int(us / (3600 * kUsPerSec));
    if (f == "getMinutes") return mk_int(us / (60 * kUsPerSec));
    if (f == "getSeconds") return mk_int(us / kUsPerSec);
    if (f == "getMilliseconds") return mk_int(us / 1000);
  }
  eval_error("unknown function '" + f + "'");
}

}  // namespace

Object parse_context(const std::string& json) {
  Json p{json};
  p.ws();
  if (p.i == json.size()) return Object{};
  Value v = p.value();
  p.ws();
  if (p.i != json.size()) bad_json("trailing characters");
  if (v.k != Value::MAP) bad_json("not a JSON object");
  return *v.m;
}

std::shared_ptr<const Node> compile(const std::string& body,
                                    const std::vector<std::pair<std::string, std::string>>& params) {
  return Parser(body, params).parse();
}

Outcome evaluate(const Node& expr, const Object* stored, const Object* check) {
  const Value v = eval(expr, Env{stored, check});
  if (v.k == Value::UNKNOWN) return PARTIAL;
  return (v.k == Value::BOOL && v.b) ? TRUE : FALSE;
}

}  // namespace cel
}  // namespace gck

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
  enum Op { LIT, VAR, LIST, AND, OR, COND, NOT, NEG, FIELD, INDEX, EQ, NE, LT, LE, GT, GE, IN, ADD, SUB, MUL, DIV, MOD };
  Op op = LIT;
  Value lit;
  std::string name;  // VAR / FIELD
  std::vector<std::shared_ptr<const Node>> kids;
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
  explicit Parser(const std::string& body) : t_(lex(body)) {}
  NodeP parse() {
    NodeP e = ternary();
    if (peek().k != Tok::END) fail("trailing tokens: '" + peek().v + "'");
    return e;
  }

 private:
  std::vector<Tok> t_;
  size_t i_ = 0;
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
        if (peek().k == Tok::END) fail("expected a field name");
        e = mk(Node::FIELD, {e}, t_[i_++].v);
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
      return mk(Node::VAR, {}, t.v);
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
    case Value::STR: return a.s == b.s;
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

Value eval(const Node& e, const Env& env) {
  using V = Value;
  switch (e.op) {
    case Node::LIT: return e.lit;
    case Node::VAR: return env.lookup(e.name);
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

std::shared_ptr<const Node> compile(const std::string& body) { return Parser(body).parse(); }

Outcome evaluate(const Node& expr, const Object* stored, const Object* check) {
  const Value v = eval(expr, Env{stored, check});
  if (v.k == Value::UNKNOWN) return PARTIAL;
  return (v.k == Value::BOOL && v.b) ? TRUE : FALSE;
}

}  // namespace cel
}  // namespace gck

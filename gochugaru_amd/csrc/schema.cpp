// schema.cpp — SpiceDB schema DSL -> node program compiler (host side).
//
// Consumes the schema text that Client.ReadSchema returns (client/client.go:416-422) and
// produces the node program the check kernels interpret (gck_internal.hpp). Grammar subset:
//   definition T { relation r: A | B#rel | C:* | D with cav | E with expiration ...
//                  permission p = <expr> }
//   caveat name(param type, ...) { <CEL> }        use expiration
//   expr: '-' loosest, '&', '+' tightest, left-assoc; primary: (expr) | nil | a->b |
//         a.any(b) | a.all(b) | name
// Rewrite semantics follow SURVEY.md §5.1 items 3-6.
#include <cctype>
#include <functional>
#include <set>
#include <sstream>

#include "engine.hpp"

namespace gck {
namespace {

struct Tok {
  enum K { IDENT, OP, STR, NUM, END } k;
  std::string v;
  size_t pos;
};

std::vector<Tok> lex(const std::string& s) {
  std::vector<Tok> out;
  size_t i = 0, n = s.size();
  auto is_id0 = [](char c) { return std::isalpha((unsigned char)c) || c == '_'; };
  auto is_id = [](char c) { return std::isalnum((unsigned char)c) || c == '_'; };
  while (i < n) {
    char c = s[i];
    if (std::isspace((unsigned char)c)) { ++i; continue; }
    if (c == '/' && i + 1 < n && s[i + 1] == '/') {
      while (i < n && s[i] != '\n') ++i;
      continue;
    }
    if (c == '/' && i + 1 < n && s[i + 1] == '*') {
      size_t e = s.find("*/", i + 2);
      if (e == std::string::npos) throw Error(GCK_E_SCHEMA, "unterminated block comment");
      i = e + 2;
      continue;
    }
    if (is_id0(c)) {
      size_t b = i;
      while (i < n && is_id(s[i])) ++i;
      // prefixed type names: org/user
      while (i + 1 < n && s[i] == '/' && is_id0(s[i + 1])) {
        ++i;
        while (i < n && is_id(s[i])) ++i;
      }
      out.push_back({Tok::IDENT, s.substr(b, i - b), b});
      continue;
    }
    if (std::isdigit((unsigned char)c)) {
      size_t b = i;
      while (i < n && (std::isdigit((unsigned char)s[i]) || s[i] == '.')) ++i;
      out.push_back({Tok::NUM, s.substr(b, i - b), b});
      continue;
    }
    if (c == '"' || c == '\'') {
      size_t b = i++;
      while (i < n && s[i] != c) i += (s[i] == '\\') ? 2 : 1;
      if (i >= n) throw Error(GCK_E_SCHEMA, "unterminated string literal");
      ++i;
      out.push_back({Tok::STR, s.substr(b, i - b), b});
      continue;
    }
    static const char* two[] = {"->", "==", "!=", "<=", ">=", "&&", "||"};
    bool done = false;
    for (const char* t : two) {
      if (s.compare(i, 2, t) == 0) {
        out.push_back({Tok::OP, t, i});
        i += 2;
        done = true;
        break;
      }
    }
    if (done) continue;
    if (std::string("{}()[]:#|=+-&.,*<>!;/%?").find(c) != std::string::npos) {
      out.push_back({Tok::OP, std::string(1, c), i});
      ++i;
      continue;
    }
    std::ostringstream m;
    m << "unexpected character '" << c << "' at offset " << i;
    throw Error(GCK_E_SCHEMA, m.str());
  }
  out.push_back({Tok::END, "", n});
  return out;
}

struct RawAllowed {
  std::string type, rel, caveat;
  bool wildcard = false, expiration = false;
};
struct RawRel {
  std::string name;
  bool perm = false;
  std::vector<RawAllowed> allowed;
  Expr expr;
};
struct RawDef {
  std::string name;
  std::vector<RawRel> rels;
};

class Parser {
 public:
  explicit Parser(const std::string& text) : t_(lex(text)) {}

  void parse(std::vector<RawDef>& defs, Schema& sc) {
    while (peek().k != Tok::END) {
      std::string kw = ident();
      if (kw == "definition") {
        defs.push_back(definition());
      } else if (kw == "caveat") {
        caveat(sc);
      } else if (kw == "use") {
        std::string what = ident();
        if (what == "expiration") sc.use_expiration = true;
      } else {
        fail("unexpected keyword '" + kw + "'");
      }
    }
  }

 private:
  std::vector<Tok> t_;
  size_t i_ = 0;

  const Tok& peek(size_t k = 0) const { return t_[std::min(i_ + k, t_.size() - 1)]; }
  [[noreturn]] void fail(const std::string& m) const {
    std::ostringstream o;
    o << m << " (at offset " << peek().pos << ")";
    throw Error(GCK_E_SCHEMA, o.str());
  }
  std::string ident() {
    if (peek().k != Tok::IDENT) fail("expected identifier, got '" + peek().v + "'");
    return t_[i_++].v;
  }
  bool accept(const char* op) {
    if (peek().k == Tok::OP && peek().v == op) {
      ++i_;
      return true;
    }
    return false;
  }
  void expect(const char* op) {
    if (!accept(op)) fail(std::string("expected '") + op + "', got '" + peek().v + "'");
  }

  RawDef definition() {
    RawDef d;
    d.name = ident();
    expect("{");
    while (!accept("}")) {
      std::string kw = ident();
      RawRel r;
      r.name = ident();
      if (kw == "relation") {
        expect(":");
        r.allowed.push_back(allowed());
        while (accept("|")) r.allowed.push_back(allowed());
      } else if (kw == "permission") {
        r.perm = true;
        expect("=");
        r.expr = expr(0);
      } else {
        fail("expected 'relation' or 'permission', got '" + kw + "'");
      }
      accept(";");
      d.rels.push_back(std::move(r));
    }
    return d;
  }

  RawAllowed allowed() {
    RawAllowed a;
    a.type = ident();
    if (accept(":")) {
      expect("*");
      a.wildcard = true;
    } else if (accept("#")) {
      a.rel = ident();
    }
    if (peek().k == Tok::IDENT && peek().v == "with") {
      ++i_;
      std::string w = ident();
      if (w == "expiration") {
        a.expiration = true;
      } else {
        a.caveat = w;
        if (peek().k == Tok::IDENT && peek().v == "and") {
          ++i_;
          if (ident() != "expiration") fail("expected 'expiration' after 'and'");
          a.expiration = true;
        }
      }
    }
    return a;
  }

  // level 0: '-' (exclusion), 1: '&' (intersection), 2: '+' (union), 3: primary
  Expr expr(int level) {
    if (level == 3) return primary();
    static const char* sym[] = {"-", "&", "+"};
    static const Expr::Op ops[] = {Expr::EXCLUDE, Expr::INTERSECT, Expr::UNION};
    Expr left = expr(level + 1);
    while (peek().k == Tok::OP && peek().v == sym[level]) {
      ++i_;
      Expr right = expr(level + 1);
      if (left.op == ops[level] && !left.kids.empty()) {
        left.kids.push_back(std::move(right));
      } else {
        Expr e;
        e.op = ops[level];
        e.kids.push_back(std::move(left));
        e.kids.push_back(std::move(right));
        left = std::move(e);
      }
    }
    return left;
  }

  Expr primary() {
    Expr e;
    if (accept("(")) {
      e = expr(0);
      expect(")");
      return e;
    }
    std::string name = ident();
    if (name == "nil") {
      e.op = Expr::NIL;
      return e;
    }
    if (accept("->")) {
      e.op = Expr::ARROW;
      e.tupleset = name;
      e.name = ident();
      return e;
    }
    if (accept(".")) {
      std::string fn = ident();
      if (fn != "any" && fn != "all") fail("unknown arrow function '" + fn + "'");
      expect("(");
      e.op = Expr::ARROW;
      e.tupleset = name;
      e.name = ident();
      e.all = (fn == "all");
      expect(")");
      return e;
    }
    e.op = Expr::COMPUTED;
    e.name = name;
    return e;
  }

  void caveat(Schema& sc) {
    CaveatDef c;
    c.name = ident();
    expect("(");
    while (!accept(")")) {
      std::string p = ident();
      std::string ty = ident();
      if (accept("<")) {
        ty += "<" + ident() + ">";
        expect(">");
      }
      c.params.emplace_back(p, ty);
      accept(",");
    }
    expect("{");
    int depth = 1;
    std::string body;
    while (depth) {
      if (peek().k == Tok::END) fail("unterminated caveat body");
      const Tok& t = t_[i_++];
      if (t.k == Tok::OP && t.v == "{") ++depth;
      if (t.k == Tok::OP && t.v == "}" && --depth == 0) break;
      if (!body.empty()) body += ' ';
      body += t.v;
    }
    c.body = body;
    c.expr = cel::compile(body, c.params);
    if (sc.caveats.count(c.name)) fail("duplicate caveat '" + c.name + "'");
    sc.caveats[c.name] = std::move(c);
  }
};

// ---- program compilation ------------------------------------------------------------------
class Compiler {
 public:
  explicit Compiler(Schema& s) : s_(s) {}

  void run() {
    const size_t R = s_.rels.size();
    s_.nodes.assign(R, DevNode{});
    // relations first so every node id < R is a schema relation
    for (size_t r = 0; r < R; ++r) {
      const RelDef& rd = s_.rels[r];
      DevNode& n = s_.nodes[r];
      n.type = rd.type;
      n.flags = NF_REAL;
      if (!rd.is_perm) {
        n.kind = NK_RELATION;
        n.first = (uint32_t)s_.items.size();
        std::set<std::pair<uint16_t, uint16_t>> seen;
        for (const Allowed& a : rd.allowed) {
          if (!seen.insert({a.stype, a.srel}).second) continue;
          DevItem it{};
          it.kind = IT_KIND;
          it.stype = a.stype;
          it.srel = a.srel;
          it.target = a.srel == kEllipsis ? kNoNode : a.srel;
          it.csr_plain = it.csr_ext = kNone;
          push_item(it, (uint16_t)r);
        }
        s_.nodes[r].count = (uint32_t)s_.items.size() - s_.nodes[r].first;
      }
    }
    for (size_t r = 0; r < R; ++r) {
      const RelDef& rd = s_.rels[r];
      if (rd.is_perm) build(rd.type, rd.expr, (int)r);
    }
    if (s_.nodes.size() >= kNoNode) throw Error(GCK_E_SCHEMA, "schema too large (node ids)");
  }

 private:
  Schema& s_;

  void push_item(const DevItem& it, uint16_t rel) {
    s_.items.push_back(it);
    s_.item_rel.push_back(rel);
  }

  uint16_t new_node(uint16_t type, uint8_t kind) {
    DevNode n{};
    n.type = type;
    n.kind = kind;
    s_.nodes.push_back(n);
    return (uint16_t)(s_.nodes.size() - 1);
  }

  // Arrow items: one per distinct subject kind of the tupleset relation.
  void arrow_items(uint16_t type, const Expr& e, std::vector<std::pair<DevItem, uint16_t>>& out) {
    int ts = s_.find_rel(type, e.tupleset);
    const RelDef& tr = s_.rels[ts];
    std::set<std::pair<uint16_t, uint16_t>> seen;
    for (const Allowed& a : tr.allowed) {
      if (!seen.insert({a.stype, a.srel}).second) continue;
      int tgt = s_.find_rel(a.stype, e.name);
      if (tgt < 0 && !e.all) continue;  // subject type lacks the target: contributes NO
      DevItem it{};
      it.kind = IT_ARROW;
      it.stype = a.stype;
      it.srel = a.srel;
      it.target = tgt < 0 ? kNoNode : (uint16_t)tgt;
      it.csr_plain = it.csr_ext = kNone;
      out.push_back({it, (uint16_t)ts});
    }
  }

  // Build the node for expression `e` on `type`. If `real` >= 0 the node is that schema
  // relation's node; otherwise a synthetic node is created. Returns the node id.
  uint16_t build(uint16_t type, const Expr& e, int real) {
    std::vector<std::pair<DevItem, uint16_t>> its;
    uint8_t kind;
    switch (e.op) {
      case Expr::NIL:
        kind = NK_NIL;
        break;
      case Expr::COMPUTED:
      case Expr::UNION:
        kind = NK_UNION;
        union_items(type, e, its);
        break;
      case Expr::ARROW:
        if (e.all) {
          kind = NK_ARROW_ALL;
          arrow_items(type, e, its);
        } else {
          kind = NK_UNION;
          arrow_items(type, e, its);
        }
        break;
      case Expr::INTERSECT:
      case Expr::EXCLUDE: {
        kind = e.op == Expr::INTERSECT ? NK_INTERSECT : NK_EXCLUDE;
        for (const Expr& k : e.kids) {
          DevItem it{};
          it.kind = IT_OPERAND;
          it.csr_plain = it.csr_ext = kNone;
          if (k.op == Expr::COMPUTED) {
            it.target = (uint16_t)s_.find_rel(type, k.name);
            it.dispatch = 1;
          } else {
            it.target = build(type, k, -1);
            it.dispatch = 0;
          }
          its.push_back({it, kNoNode});
        }
        break;
      }
      default:
        throw Error(GCK_E_SCHEMA, "internal: bad expression");
    }
    uint16_t id = real >= 0 ? (uint16_t)real : new_node(type, kind);
    // children may have appended nodes; re-fetch by index
    s_.nodes[id].type = type;
    s_.nodes[id].kind = kind;
    s_.nodes[id].flags = real >= 0 ? NF_REAL : 0;
    s_.nodes[id].first = (uint32_t)s_.items.size();
    for (auto& p : its) push_item(p.first, p.second);
    s_.nodes[id].count = (uint32_t)its.size();
    return id;
  }

  void union_items(uint16_t type, const Expr& e, std::vector<std::pair<DevItem, uint16_t>>& out) {
    if (e.op == Expr::UNION) {
      for (const Expr& k : e.kids) union_items(type, k, out);
      return;
    }
    DevItem it{};
    it.csr_plain = it.csr_ext = kNone;
    switch (e.op) {
      case Expr::NIL:
        return;
      case Expr::COMPUTED:
        it.kind = IT_COMPUTED;
        it.target = (uint16_t)s_.find_rel(type, e.name);
        out.push_back({it, kNoNode});
        return;
      case Expr::ARROW:
        if (!e.all) {
          arrow_items(type, e, out);
          return;
        }
        [[fallthrough]];
      default:
        it.kind = IT_SUB;
        it.target = build(type, e, -1);
        out.push_back({it, kNoNode});
        return;
    }
  }
};

void validate_expr(const Schema& s, uint16_t type, const Expr& e, const std::string& where) {
  switch (e.op) {
    case Expr::COMPUTED:
      if (s.find_rel(type, e.name) < 0)
        throw Error(GCK_E_SCHEMA, where + ": unknown relation or permission '" + e.name + "'");
      break;
    case Expr::ARROW: {
      int ts = s.find_rel(type, e.tupleset);
      if (ts < 0 || s.rels[ts].is_perm)
        throw Error(GCK_E_SCHEMA, where + ": arrow tupleset '" + e.tupleset + "' must be a relation");
      bool any = false;
      for (const Allowed& a : s.rels[ts].allowed) {
        if (a.wildcard)
          throw Error(GCK_E_SCHEMA, where + ": arrow tupleset '" + e.tupleset + "' allows a wildcard");
        if (s.find_rel(a.stype, e.name) >= 0) any = true;
      }
      if (!any)
        throw Error(GCK_E_SCHEMA, where + ": arrow target '" + e.name + "' exists on no subject type");
      break;
    }
    default:
      break;
  }
  for (const Expr& k : e.kids) validate_expr(s, type, k, where);
}

}  // namespace

std::unique_ptr<Schema> compile_schema(const std::string& text) {
  auto sc = std::make_unique<Schema>();
  std::vector<RawDef> defs;
  Parser(text).parse(defs, *sc);
  // types
  for (const RawDef& d : defs) {
    if (sc->type_ids.count(d.name)) throw Error(GCK_E_SCHEMA, "duplicate definition '" + d.name + "'");
    if (sc->types.size() >= 0xFFF0) throw Error(GCK_E_SCHEMA, "too many types");
    sc->type_ids[d.name] = (uint16_t)sc->types.size();
    TypeDef t;
    t.name = d.name;
    sc->types.push_back(std::move(t));
  }
  // relation ids (definition order)
  for (size_t ti = 0; ti < defs.size(); ++ti) {
    for (const RawRel& r : defs[ti].rels) {
      if (sc->types[ti].rels.count(r.name))
        throw Error(GCK_E_SCHEMA, "duplicate relation '" + defs[ti].name + "#" + r.name + "'");
      if (sc->rels.size() >= 0xFF00) throw Error(GCK_E_SCHEMA, "too many relations");
      sc->types[ti].rels[r.name] = (uint16_t)sc->rels.size();
      RelDef rd;
      rd.name = r.name;
      rd.type = (uint16_t)ti;
      rd.is_perm = r.perm;
      rd.expr = r.expr;
      sc->rels.push_back(std::move(rd));
    }
  }
  // resolve allowed subject types
  for (size_t ti = 0; ti < defs.size(); ++ti) {
    for (const RawRel& r : defs[ti].rels) {
      RelDef& rd = sc->rels[sc->types[ti].rels[r.name]];
      std::string where = defs[ti].name + "#" + r.name;
      for (const RawAllowed& a : r.allowed) {
        int st = sc->find_type(a.type);
        if (st < 0) throw Error(GCK_E_SCHEMA, where + ": unknown type '" + a.type + "'");
        Allowed al;
        al.stype = (uint16_t)st;
        al.wildcard = a.wildcard;
        al.expiration = a.expiration;
        al.caveat = a.caveat;
        if (!a.rel.empty()) {
          int sr = sc->find_rel((uint16_t)st, a.rel);
          if (sr < 0) throw Error(GCK_E_SCHEMA, where + ": unknown relation '" + a.type + "#" + a.rel + "'");
          al.srel = (uint16_t)sr;
        }
        if (!a.caveat.empty() && !sc->caveats.count(a.caveat))
          throw Error(GCK_E_SCHEMA, where + ": unknown caveat '" + a.caveat + "'");
        rd.allowed.push_back(al);
      }
    }
  }
  for (const RelDef& rd : sc->rels)
    if (rd.is_perm) validate_expr(*sc, rd.type, rd.expr, sc->types[rd.type].name + "#" + rd.name);
  Compiler(*sc).run();
  return sc;
}

}  // namespace gck

// snapshot.cpp — host-side ingest: canonical relationship text -> interned tuples -> CSR.
//
// Ingest record = rel.Relationship (rel/relationship.go:28-38) as streamed by
// Client.ExportRelationships (client/client.go:472-499); text form = Relationship.String
// (rel/relationship.go:51-90). The builder groups tuples per (relation, subject kind) and
// splits plain edges from caveated/expiring ones (separate "ext" CSR with caveat ids and
// expiry times), sorts every row ascending (wildcard id 0xFFFFFFFF sorts last) and keeps the
// last write of a duplicate relationship (TOUCH semantics).
#include <algorithm>
#include <atomic>
#include <cstring>
#include <numeric>
#include <thread>

#include "engine.hpp"

namespace gck {
namespace {

// days since 1970-01-01 for a proleptic Gregorian date (H. Hinnant's algorithm)
int64_t days_from_civil(int64_t y, unsigned m, unsigned d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const unsigned yoe = (unsigned)(y - era * 400);
  const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + (int64_t)doe - 719468;
}

bool parse_num(const std::string& s, size_t& i, int digits, int64_t& out) {
  out = 0;
  for (int k = 0; k < digits; ++k, ++i) {
    if (i >= s.size() || !isdigit((unsigned char)s[i])) return false;
    out = out * 10 + (s[i] - '0');
  }
  return true;
}

// RFC 3339 timestamp -> unix microseconds
int64_t parse_rfc3339(const std::string& s) {
  size_t i = 0;
  int64_t Y, M, D, h, m, sec;
  auto bad = [&]() -> Error { return Error(GCK_E_INVALID_ARGUMENT, "bad expiration timestamp '" + s + "'"); };
  if (!parse_num(s, i, 4, Y) || s[i++] != '-' || !parse_num(s, i, 2, M) || s[i++] != '-' ||
      !parse_num(s, i, 2, D) || (s[i] != 'T' && s[i] != 't') || !parse_num(s, ++i, 2, h) ||
      s[i++] != ':' || !parse_num(s, i, 2, m) || s[i++] != ':' || !parse_num(s, i, 2, sec))
    throw bad();
  int64_t frac_us = 0;
  if (i < s.size() && s[i] == '.') {
    ++i;
    int64_t scale = 100000;
    while (i < s.size() && isdigit((unsigned char)s[i])) {
      frac_us += (s[i] - '0') * scale;
      scale /= 10;
      ++i;
    }
  }
  int64_t off_s = 0;
  if (i < s.size() && (s[i] == 'Z' || s[i] == 'z')) {
    ++i;
  } else if (i < s.size() && (s[i] == '+' || s[i] == '-')) {
    int sign = s[i++] == '-' ? -1 : 1;
    int64_t oh, om;
    if (!parse_num(s, i, 2, oh) || s[i++] != ':' || !parse_num(s, i, 2, om)) throw bad();
    off_s = sign * (oh * 3600 + om * 60);
  } else {
    throw bad();
  }
  if (i != s.size()) throw bad();
  int64_t days = days_from_civil(Y, (unsigned)M, (unsigned)D);
  return ((days * 86400 + h * 3600 + m * 60 + sec) - off_s) * 1000000 + frac_us;
}

uint32_t intern_one(Engine& e, uint16_t type, const std::string& id) {
  if (id == "*") return kWildcard;
  TypeInterner& ti = e.interner[type];
  auto it = ti.ids.find(id);
  if (it != ti.ids.end()) return it->second;
  if (e.part_world > 1)  // (an id here would not be the one the name's owner gives it)
    throw Error(GCK_E_STATE, "a partitioned engine interns a new name through its owner rank "
                             "(gck_part_intern_with, gck_part_add_tuples_text_with): '" + id + "'");
  if (ti.count >= kAbsent) throw Error(GCK_E_CAPACITY, "too many objects of one type");
  uint32_t nid = ti.count++;
  ti.ids.emplace(id, nid);
  if (ti.names.size() < ti.count) ti.names.resize(ti.count);
  ti.names[nid] = id;
  return nid;
}

// Finds the end of a JSON value starting at s[i] ('{'), honouring strings and nesting.
size_t json_end(const std::string& s, size_t i) {
  int depth = 0;
  bool str = false;
  for (; i < s.size(); ++i) {
    char c = s[i];
    if (str) {
      if (c == '\\') ++i;
      else if (c == '"') str = false;
      continue;
    }
    if (c == '"') str = true;
    else if (c == '{' || c == '[') ++depth;
    else if (c == '}' || c == ']') {
      if (--depth == 0) return i + 1;
    }
  }
  throw Error(GCK_E_INVALID_ARGUMENT, "unterminated caveat context");
}

}  // namespace

uint32_t add_caveat_instance(Engine& e, const std::string& name, const std::string& json);

// Schema and interner validation of one relationship (WriteRelationships would reject it).
void validate_tuple(const Engine& e, const gck_tuple& t) {
  const Schema& sc = *e.schema;
  if (t.resource_type >= sc.types.size() || t.subject_type >= sc.types.size())
    throw Error(GCK_E_INVALID_ARGUMENT, "tuple references an unknown type");
  if (t.relation >= sc.rels.size() || sc.rels[t.relation].type != t.resource_type)
    throw Error(GCK_E_INVALID_ARGUMENT, "tuple relation is not defined on its resource type");
  const RelDef& rd = sc.rels[t.relation];
  if (rd.is_perm)
    throw Error(GCK_E_INVALID_ARGUMENT, "cannot write a relationship to permission '" + rd.name + "'");
  bool ok = false;
  for (const Allowed& a : rd.allowed) {
    if (a.stype != t.subject_type) continue;
    if (t.subject_id == kWildcard) {
      if (a.wildcard && t.subject_relation == kEllipsis) ok = true;
    } else if (!a.wildcard && a.srel == t.subject_relation) {
      ok = true;
    }
  }
  if (!ok)
    throw Error(GCK_E_INVALID_ARGUMENT, "subject type/relation not allowed on '" +
                                            sc.types[rd.type].name + "#" + rd.name + "'");
  if (t.resource_id >= e.interner[t.resource_type].count ||
      (t.subject_id != kWildcard && t.subject_id >= e.interner[t.subject_type].count))
    throw Error(GCK_E_INVALID_ARGUMENT, "tuple references an object id that was never interned");
  if (t.caveat >= e.caveat_instances.size())
    throw Error(GCK_E_INVALID_ARGUMENT, "unknown caveat instance id");
}

void stage_tuple(Engine& e, const gck_tuple& t) {
  validate_tuple(e, t);
  if (!part_keep(e, t.relation, t.resource_id, t.subject_id, t.subject_relation)) return;  // another rank's
  StagedTuple s{};
  s.rel = t.relation;
  s.stype = t.subject_type;
  s.srel = t.subject_relation;
  s.obj = t.resource_id;
  s.sid = t.subject_id;
  s.cav = t.caveat;
  s.exp_us = t.expires_at_us;
  s.seq = e.seq++;
  e.staged.push_back(s);
}

// A page of interned tuples (an ExportRelationships page, client/client.go:472-499): validated
// and staged by up to 16 threads; on an invalid tuple nothing of the page is staged and the
// error of the first invalid tuple is raised.
void stage_tuples(Engine& e, const gck_tuple* t, size_t n) {
  const size_t base = e.staged.size();
  e.staged.resize(base + n);
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const size_t chunk = std::max<size_t>(1 << 16, (n + hw - 1) / hw);
  const size_t n_chunks = (n + chunk - 1) / chunk;
  std::vector<std::string> err(n_chunks);
  std::vector<int> code(n_chunks, 0);
  auto work = [&](size_t c) {
    const size_t lo = c * chunk, hi = std::min(n, lo + chunk);
    try {
      for (size_t i = lo; i < hi; ++i) {
        validate_tuple(e, t[i]);
        StagedTuple& s = e.staged[base + i];
        s = StagedTuple{};
        s.rel = t[i].relation;
        s.stype = t[i].subject_type;
        s.srel = t[i].subject_relation;
        s.obj = t[i].resource_id;
        s.sid = t[i].subject_id;
        s.cav = t[i].caveat;
        s.exp_us = t[i].expires_at_us;
        s.seq = e.seq + i;
      }
    } catch (const Error& x) {
      code[c] = x.code;
      err[c] = x.what();
    }
  };
  if (n_chunks <= 1) {
    if (n) work(0);
  } else {
    std::vector<std::thread> pool;
    for (size_t c = 0; c < n_chunks; ++c) pool.emplace_back(work, c);
    for (std::thread& th : pool) th.join();
  }
  for (size_t c = 0; c < n_chunks; ++c)
    if (code[c]) {
      e.staged.resize(base);
      throw Error(code[c], err[c]);
    }
  e.seq += n;
  if (e.part_world > 1)  // a partitioned graph: what this rank keeps (part_keep), the page validated whole
    e.staged.erase(std::remove_if(e.staged.begin() + base, e.staged.end(),
                                  [&](const StagedTuple& s) { return !part_keep(e, s.rel, s.obj, s.sid, s.srel); }),
                   e.staged.end());
}

namespace {

// Splits text into trimmed lines, skipping blank lines and comments ('#', '//').
template <class F>
void for_each_line(const char* text, size_t len, F&& f) {
  size_t pos = 0;
  while (pos < len) {
    size_t nl = pos;
    while (nl < len && text[nl] != '\n') ++nl;
    std::string line(text + pos, nl - pos);
    pos = nl + 1;
    while (!line.empty() && (line.back() == '\r' || line.back() == ' ' || line.back() == '\t')) line.pop_back();
    size_t st = 0;
    while (st < line.size() && (line[st] == ' ' || line[st] == '\t')) ++st;
    line = line.substr(st);
    if (line.empty() || line[0] == '#' || line.compare(0, 2, "//") == 0) continue;
    f(line);
  }
}

}  // namespace

// One canonical line: type:id#rel@type:id[#rel][caveat[:{json}]][expiration:T], by name:
// the types, relations and caveat instance resolved (the instance registered), the object ids
// left as text (interned by the caller: locally, or by their owners on a partitioned graph).
TupleNames parse_tuple_names(Engine& e, const std::string& line) {
  const Schema& sc = *e.schema;
  {
    auto bad = [&](const char* why) {
      return Error(GCK_E_INVALID_ARGUMENT, std::string(why) + ": '" + line + "'");
    };
    size_t at = line.find('@');
    if (at == std::string::npos) throw bad("invalid subject");
    std::string res = line.substr(0, at);
    size_t hash = res.find('#');
    if (hash == std::string::npos || hash + 1 == res.size()) throw bad("invalid relation");
    std::string rname = res.substr(hash + 1);
    res = res.substr(0, hash);
    size_t colon = res.find(':');
    if (colon == std::string::npos) throw bad("invalid resource");
    std::string rtype = res.substr(0, colon), rid = res.substr(colon + 1);
    // subject ends at the first '['
    std::string rest = line.substr(at + 1);
    size_t br = rest.find('[');
    std::string subj = br == std::string::npos ? rest : rest.substr(0, br);
    std::string tail = br == std::string::npos ? std::string() : rest.substr(br);
    std::string srel_name;
    size_t sh = subj.find('#');
    if (sh != std::string::npos) {
      srel_name = subj.substr(sh + 1);
      subj = subj.substr(0, sh);
    }
    size_t sc_ = subj.find(':');
    if (sc_ == std::string::npos) throw bad("invalid subject");
    std::string stype = subj.substr(0, sc_), sid = subj.substr(sc_ + 1);
    // optional [caveat[:{json}]] then optional [expiration:T]
    std::string cav_name, cav_json;
    int64_t exp_us = 0;
    size_t i = 0;
    while (i < tail.size()) {
      if (tail[i] != '[') throw bad("malformed trailer");
      size_t j = i + 1;
      while (j < tail.size() && tail[j] != ':' && tail[j] != ']') ++j;
      if (j >= tail.size()) throw bad("malformed trailer");
      std::string name = tail.substr(i + 1, j - i - 1);
      if (name == "expiration") {
        size_t k = tail.find(']', j);
        if (k == std::string::npos) throw bad("malformed expiration");
        exp_us = parse_rfc3339(tail.substr(j + 1, k - j - 1));
        if (exp_us == 0) exp_us = 1;  // 0 is the "never" sentinel
        i = k + 1;
      } else {
        cav_name = name;
        if (tail[j] == ':') {
          size_t k = json_end(tail, j + 1);
          cav_json = tail.substr(j + 1, k - j - 1);
          j = k;
        }
        if (j >= tail.size() || tail[j] != ']') throw bad("malformed caveat");
        i = j + 1;
      }
    }
    int rt = sc.find_type(rtype), stt = sc.find_type(stype);
    if (rt < 0 || stt < 0) throw bad("unknown type");
    int rr = sc.find_rel((uint16_t)rt, rname);
    if (rr < 0) throw bad("unknown relation");
    uint16_t srel = kEllipsis;
    if (!srel_name.empty() && srel_name != "...") {
      int x = sc.find_rel((uint16_t)stt, srel_name);
      if (x < 0) throw bad("unknown subject relation");
      srel = (uint16_t)x;
    }
    TupleNames t;
    t.rt = (uint16_t)rt;
    t.rel = (uint16_t)rr;
    t.rid = std::move(rid);
    t.st = (uint16_t)stt;
    t.srel = srel;
    t.sid = std::move(sid);
    t.cav = cav_name.empty() ? 0 : add_caveat_instance(e, cav_name, cav_json);
    t.exp = exp_us;
    return t;
  }
}

namespace {

// The same, its ids interned here (creating them).
gck_tuple parse_tuple_line(Engine& e, const std::string& line) {
  TupleNames p = parse_tuple_names(e, line);
  gck_tuple t{};
  t.resource_type = p.rt;
  t.relation = p.rel;
  t.resource_id = intern_one(e, p.rt, p.rid);
  t.subject_type = p.st;
  t.subject_relation = p.srel;
  t.subject_id = intern_one(e, p.st, p.sid);
  t.caveat = p.cav;
  t.expires_at_us = p.exp;
  return t;
}

}  // namespace

std::vector<TupleNames> parse_tuples_text(Engine& e, const char* text, size_t len) {
  std::vector<TupleNames> out;
  for_each_line(text, len, [&](const std::string& line) { out.push_back(parse_tuple_names(e, line)); });
  return out;
}

void add_tuples_text(Engine& e, const char* text, size_t len) {
  for_each_line(text, len, [&](const std::string& line) { stage_tuple(e, parse_tuple_line(e, line)); });
}

// Watch updates as text, one per line: "<OP> <relationship>", OP = CREATE | TOUCH | DELETE
// (rel.UpdateType, rel/relationship.go:267-274; the OPERATION_ prefix of the v1 proto enum is
// accepted too).
void parse_updates_text(Engine& e, const char* text, size_t len, std::vector<gck_update>& out) {
  for_each_line(text, len, [&](const std::string& line) {
    size_t sp = line.find_first_of(" \t");
    if (sp == std::string::npos) throw Error(GCK_E_INVALID_ARGUMENT, "update without a relationship: '" + line + "'");
    std::string op = line.substr(0, sp);
    if (op.compare(0, 10, "OPERATION_") == 0) op = op.substr(10);
    gck_update u{};
    if (op == "CREATE") u.op = GCK_UPDATE_CREATE;
    else if (op == "TOUCH") u.op = GCK_UPDATE_TOUCH;
    else if (op == "DELETE") u.op = GCK_UPDATE_DELETE;
    else throw Error(GCK_E_INVALID_ARGUMENT, "unknown update operation '" + op + "'");
    size_t st = line.find_first_not_of(" \t", sp);
    u.tuple = parse_tuple_line(e, line.substr(st));
    out.push_back(u);
  });
}

// The validation group_updates does, alone: a partitioned engine validates the whole batch before
// it keeps its own updates (part_keep), so that an update only one rank keeps — an unknown
// relation, a subject the schema disallows, an id never interned — is refused by every rank and
// no rank moves to the new revision without the others. One schema check per (resource type,
// kind, wildcard) combination, as group_updates makes them.
void validate_updates(const Engine& e, const gck_update* ups, size_t n) {
  std::vector<uint64_t> seen;
  for (size_t i = 0; i < n; ++i) {
    const gck_update& u = ups[i];
    if (u.op != GCK_UPDATE_CREATE && u.op != GCK_UPDATE_TOUCH && u.op != GCK_UPDATE_DELETE)
      throw Error(GCK_E_INVALID_ARGUMENT, "unknown update operation " + std::to_string(u.op));
    const gck_tuple& t = u.tuple;
    const uint64_t combo = ((uint64_t)(t.resource_type & 0x7FFF) << 48) | ((uint64_t)t.relation << 32) |
                           ((uint64_t)t.subject_type << 16) | t.subject_relation |
                           (t.subject_id == kWildcard ? (1ull << 63) : 0ull);
    if (std::find(seen.begin(), seen.end(), combo) == seen.end()) {
      validate_tuple(e, t);
      seen.push_back(combo);
    } else if (t.resource_id >= e.interner[t.resource_type].count ||
               (t.subject_id != kWildcard && t.subject_id >= e.interner[t.subject_type].count) ||
               t.caveat >= e.caveat_instances.size()) {
      validate_tuple(e, t);  // (raises the error)
    }
  }
}

// Validates the updates and groups them per (relation, subject type, subject relation); within a
// group the last write per (object, subject) wins (the order of the Watch stream). Groups come
// out in ascending (relation, subject type, subject relation) order, keys ascending.
//
// One pass over the batch validates and stages each update into its kind's record array: a
// direct-mapped cache of the (resource type, kind, wildcard) combinations whose schema checks
// passed holds the kind and the object counts the id checks need, so the per-update work is a
// hash, one well-predicted compare and the bounds checks (a linear search of the combinations
// mispredicted its exit on every update of a mixed batch). Per kind a stable counting pass on
// the key's top bits into ~one bucket per update, then an insertion sort of each bucket (a bucket
// that a skewed batch fills is merge-sorted). Everything lives in Engine::group_buf and is reused
// batch after batch (fresh vectors cost a 10K-update batch its allocations and page faults).
const std::vector<UpdateGroup>& group_updates(const Engine& e, GroupBuffers& B, const gck_update* ups, size_t n,
                                              std::shared_mutex* schema_mu) {
  PhaseClock pc("group");
  if (n >= (1ull << 30)) throw Error(GCK_E_CAPACITY, "a Watch batch holds at most 2^30 updates");
  // (a staged batch reads the schema and the interner under the engine lock, shared and briefly:
  // once per new combination and for an update that fails its bounds)
  auto locked = [&](auto&& f) {
    if (!schema_mu) return f();
    std::shared_lock<std::shared_mutex> sl(*schema_mu);
    return f();
  };
  struct KI {
    uint64_t k;  // (object << 32) | subject
    uint64_t i;  // update index << 34 | upsert << 33 | has expiration << 32 | caveat
  };
  static_assert(sizeof(KI) == 16, "group record");
  constexpr uint32_t kSlots = 64;
  struct Slot {
    uint64_t combo;
    uint32_t kind, rows, subs, used;
  } cache[kSlots];
  for (Slot& sl : cache) sl.used = 0;
  std::vector<uint64_t>& kinds = B.kinds;  // distinct (relation, subject type, subject relation)
  kinds.clear();
  std::vector<uint32_t>& cnt = B.cnt;
  cnt.clear();
  auto recs = [&](uint32_t k) -> KI* {  // the kind's record array (capacity n)
    std::vector<uint64_t>& v = B.recs[k];
    if (v.size() < 2 * n) v.resize(2 * n);
    return reinterpret_cast<KI*>(v.data());
  };
  std::vector<KI*> arr;
  const uint32_t n_cav = locked([&] { return (uint32_t)std::min<size_t>(e.caveat_instances.size(), 0xFFFFFFFFu); });
  for (size_t i = 0; i < n; ++i) {
    const gck_update& u = ups[i];
    if (u.op != GCK_UPDATE_CREATE && u.op != GCK_UPDATE_TOUCH && u.op != GCK_UPDATE_DELETE)
      throw Error(GCK_E_INVALID_ARGUMENT, "unknown update operation " + std::to_string(u.op));
    const gck_tuple& t = u.tuple;
    const bool wild = t.subject_id == kWildcard;
    const uint64_t combo = ((uint64_t)(t.resource_type & 0x7FFF) << 48) | ((uint64_t)t.relation << 32) |
                           ((uint64_t)t.subject_type << 16) | t.subject_relation | (wild ? (1ull << 63) : 0ull);
    Slot& sl = cache[(combo * 0x9E3779B97F4A7C15ull) >> 58];
    if (sl.used && sl.combo == combo) {
      if (t.resource_id >= sl.rows || (!wild && t.subject_id >= sl.subs) || t.caveat >= n_cav)
        locked([&] { validate_tuple(e, t); });  // (raises the error)
    } else {
      uint32_t rows = 0, subs = 0;
      locked([&] {
        validate_tuple(e, t);
        rows = e.interner[t.resource_type].count;
        subs = e.interner[t.subject_type].count;
      });
      const uint64_t gk = combo & 0xFFFFFFFFFFFFull;
      uint32_t k = 0;
      while (k < kinds.size() && kinds[k] != gk) ++k;
      if (k == kinds.size()) {
        kinds.push_back(gk);
        cnt.push_back(0);
        if (B.recs.size() <= k) B.recs.resize(k + 1);
        arr.push_back(recs(k));
      }
      sl = Slot{combo, k, rows, subs, 1u};
    }
    const uint32_t k = sl.kind;
    const uint64_t up = u.op != GCK_UPDATE_DELETE ? 1 : 0;
    arr[k][cnt[k]++] = {((uint64_t)t.resource_id << 32) | t.subject_id,
                        ((uint64_t)i << 34) | (up << 33) | ((t.expires_at_us != 0 ? 1ull : 0ull) << 32) | t.caveat};
  }
  pc.mark("validate");
  const size_t G = kinds.size();
  std::vector<uint32_t> by_kind(G);
  for (size_t j = 0; j < G; ++j) by_kind[j] = (uint32_t)j;
  std::sort(by_kind.begin(), by_kind.end(), [&](uint32_t x, uint32_t y) { return kinds[x] < kinds[y]; });
  std::vector<UpdateGroup>& out = B.out;
  out.resize(G);
  if (B.tmp.size() < 2 * n) B.tmp.resize(2 * n);
  KI* b = reinterpret_cast<KI*>(B.tmp.data());
  std::vector<uint32_t>& bucket = B.bucket;
  for (size_t gi = 0; gi < G; ++gi) {
    const uint32_t kk = by_kind[gi];
    KI* a = arr[kk];
    const size_t m = cnt[kk];
    // stable sort by key (a later write of a key stays after the earlier ones): one counting pass
    // on the key's top bits into ~one bucket per update, then an insertion sort of each bucket
    uint64_t kmin = ~0ull, kmax = 0;
    for (size_t i = 0; i < m; ++i) {
      kmin = std::min(kmin, a[i].k);
      kmax = std::max(kmax, a[i].k);
    }
    KI* src = a;
    if (m > 1 && kmax != kmin) {
      int lb = 1;
      while (lb < 16 && ((size_t)1 << lb) < m) ++lb;
      const int bits = 64 - __builtin_clzll(kmax - kmin);
      const int sh = bits > lb ? bits - lb : 0;
      const size_t nb = ((kmax - kmin) >> sh) + 1;
      bucket.assign(nb + 1, 0u);
      for (size_t i = 0; i < m; ++i) ++bucket[((a[i].k - kmin) >> sh) + 1];
      for (size_t j = 0; j < nb; ++j) bucket[j + 1] += bucket[j];
      for (size_t i = 0; i < m; ++i) b[bucket[(a[i].k - kmin) >> sh]++] = a[i];
      src = b;
      // (bucket[j] is now the end of bucket j)
      size_t s0 = 0;
      for (size_t j = 0; j < nb; ++j) {
        const size_t s1 = bucket[j];
        if (s1 - s0 > 32) {
          std::stable_sort(b + s0, b + s1, [](const KI& x, const KI& y) { return x.k < y.k; });
        } else {
          for (size_t i = s0 + 1; i < s1; ++i) {
            const KI v = b[i];
            size_t p = i;
            while (p > s0 && b[p - 1].k > v.k) {
              b[p] = b[p - 1];
              --p;
            }
            b[p] = v;
          }
        }
        s0 = s1;
      }
    }
    const uint64_t kind = kinds[kk];
    UpdateGroup& g = out[gi];
    g.rel = (uint16_t)(kind >> 32);
    g.stype = (uint16_t)(kind >> 16);
    g.srel = (uint16_t)kind;
    g.keys.resize(m);
    g.upsert.resize(m);
    g.is_ext.resize(m);
    g.cav.resize(m);
    g.exp_us.resize(m);
    size_t w = 0;
    for (size_t i = 0; i < m; ++i) {
      if (i + 1 < m && src[i + 1].k == src[i].k) continue;  // a later write of the same relationship follows
      const uint64_t v = src[i].i;
      const bool up = (v >> 33) & 1, has_exp = (v >> 32) & 1;
      const uint32_t cav = (uint32_t)v;
      g.keys[w] = src[i].k;
      g.upsert[w] = up ? 1 : 0;
      g.is_ext[w] = up && (cav != 0 || has_exp) ? 1 : 0;
      g.cav[w] = up ? cav : 0;
      g.exp_us[w] = up && has_exp ? ups[v >> 34].tuple.expires_at_us : 0;
      ++w;
    }
    g.keys.resize(w);
    g.upsert.resize(w);
    g.is_ext.resize(w);
    g.cav.resize(w);
    g.exp_us.resize(w);
  }
  pc.mark("sort");
  // the merge's upload image (delta.inc device_apply_build copies it to the device whole): per
  // group its keys, the insert flags of its plain and its caveated class, caveats, expirations —
  // made here, so that a staged batch's is made on the staging thread, beside the previous apply
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  size_t bytes = 0;
  for (const UpdateGroup& g : out) {
    const size_t m = g.keys.size();
    bytes += al(8 * m) + 2 * al(m) + al(4 * m) + al(8 * m);
  }
  if (B.img_cap < bytes) {
    if (B.img) pinned_free(B.img);
    B.img = nullptr;
    B.img_cap = 0;
    const size_t cap = std::max(bytes + bytes / 2, (size_t)1 << 20);
    B.img = static_cast<unsigned char*>(pinned_alloc(cap));
    if (!B.img) throw Error(GCK_E_DEVICE, "pinned allocation of a Watch upload image failed");
    B.img_cap = cap;
  }
  B.img_bytes = bytes;
  size_t at = 0;
  for (UpdateGroup& g : out) {
    const size_t m = g.keys.size();
    g.img = B.img;
    g.o_keys = at, at += al(8 * m);
    g.o_ins[0] = at, at += al(m);
    g.o_ins[1] = at, at += al(m);
    g.o_cav = at, at += al(4 * m);
    g.o_exp = at, at += al(8 * m);
    std::memcpy(B.img + g.o_keys, g.keys.data(), 8 * m);
    std::memcpy(B.img + g.o_cav, g.cav.data(), 4 * m);
    std::memcpy(B.img + g.o_exp, g.exp_us.data(), 8 * m);
    uint8_t* i0 = B.img + g.o_ins[0];
    uint8_t* i1 = B.img + g.o_ins[1];
    // (branch-free: the upsert / caveat mix of a Watch batch is random)
    uint32_t nc0 = 0, nc1 = 0, mr0 = 0, mr1 = 0, w0 = 0, w1 = 0, wa = 0;
    for (size_t d = 0; d < m; ++d) {
      const uint32_t up = g.upsert[d] != 0, x = g.is_ext[d] != 0;
      const uint32_t in1 = up & x, in0 = up & (x ^ 1u);
      const uint32_t row1 = (uint32_t)(g.keys[d] >> 32) + 1, w = (uint32_t)g.keys[d] == kWildcard;
      i0[d] = (uint8_t)in0;
      i1[d] = (uint8_t)in1;
      nc0 += in0;
      nc1 += in1;
      mr0 = std::max(mr0, in0 ? row1 : 0u);
      mr1 = std::max(mr1, in1 ? row1 : 0u);
      w0 |= in0 & w;
      w1 |= in1 & w;
      wa |= w;
    }
    g.n_cand[0] = nc0, g.n_cand[1] = nc1;
    g.max_row[0] = mr0, g.max_row[1] = mr1;
    g.wild_ins[0] = (uint8_t)w0, g.wild_ins[1] = (uint8_t)w1, g.wild_any = (uint8_t)wa;
  }
  pc.mark("image");
  return out;
}

// Orders the staged tuples by (relation, subject type, subject relation, object, subject) with
// equal relationships in arrival order — the order a comparison sort on (..., seq) gives — by
// a stable counting sort into (relation, subject kind) groups followed, per group, by a stable
// LSD radix sort of the 64-bit (object << 32 | subject) keys in 16-bit digits (digits constant
// over the group are skipped). Groups sort in parallel. Staged tuples are in arrival order.
static void sort_staged(std::vector<StagedTuple>& v) {
  const size_t n = v.size();
  if (n < 2) return;
  auto gkey = [](const StagedTuple& t) {
    return ((uint64_t)t.rel << 32) | ((uint64_t)t.stype << 16) | t.srel;
  };
  std::vector<uint64_t> gkeys;
  for (const StagedTuple& t : v) {
    const uint64_t k = gkey(t);
    if (gkeys.empty() || gkeys.back() != k) gkeys.push_back(k);
  }
  std::sort(gkeys.begin(), gkeys.end());
  gkeys.erase(std::unique(gkeys.begin(), gkeys.end()), gkeys.end());
  auto group_of = [&](const StagedTuple& t) {
    return (size_t)(std::lower_bound(gkeys.begin(), gkeys.end(), gkey(t)) - gkeys.begin());
  };
  const size_t G = gkeys.size();
  std::vector<size_t> start(G + 1, 0);
  std::vector<uint32_t> g_of(n);
  for (size_t i = 0; i < n; ++i) {
    g_of[i] = (uint32_t)group_of(v[i]);
    ++start[g_of[i] + 1];
  }
  for (size_t g = 0; g < G; ++g) start[g + 1] += start[g];
  std::vector<StagedTuple> out(n);
  {
    std::vector<size_t> pos(start.begin(), start.end() - 1);
    for (size_t i = 0; i < n; ++i) out[pos[g_of[i]]++] = v[i];
  }
  std::vector<uint32_t>().swap(g_of);
  auto sort_group = [&](size_t g) {
    const size_t b = start[g], m = start[g + 1] - b;
    if (m < 2) return;
    struct KI {
      uint64_t k;
      uint64_t i;
    };
    std::vector<KI> a(m), t(m);
    uint64_t orv = 0, andv = ~0ull;
    for (size_t i = 0; i < m; ++i) {
      const StagedTuple& x = out[b + i];
      a[i] = {((uint64_t)x.obj << 32) | x.sid, i};
      orv |= a[i].k;
      andv &= a[i].k;
    }
    std::vector<size_t> cnt(65537);
    for (int d = 0; d < 4; ++d) {
      const int sh = 16 * d;
      if ((((orv ^ andv) >> sh) & 0xFFFF) == 0) continue;  // constant digit
      std::fill(cnt.begin(), cnt.end(), 0);
      for (size_t i = 0; i < m; ++i) ++cnt[((a[i].k >> sh) & 0xFFFF) + 1];
      for (size_t j = 0; j < 65536; ++j) cnt[j + 1] += cnt[j];
      for (size_t i = 0; i < m; ++i) t[cnt[(a[i].k >> sh) & 0xFFFF]++] = a[i];
      a.swap(t);
    }
    for (size_t i = 0; i < m; ++i) v[b + i] = out[b + a[i].i];
  };
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<std::thread> pool;
  std::atomic<size_t> next{0};
  for (unsigned k = 0; k < std::min<size_t>(hw, G); ++k)
    pool.emplace_back([&] {
      for (size_t g; (g = next.fetch_add(1)) < G;) sort_group(g);
    });
  for (std::thread& th : pool) th.join();
  for (size_t g = 0; g < G; ++g)  // groups of one tuple were not copied back
    if (start[g + 1] - start[g] == 1) v[start[g]] = out[start[g]];
}

std::vector<HostCSR> build_csrs(Engine& e) {
  const Schema& sc = *e.schema;
  std::vector<StagedTuple>& v = e.staged;
  sort_staged(v);
  // keep the last write per (rel, stype, srel, obj, sid)
  size_t w = 0;
  for (size_t i = 0; i < v.size(); ++i) {
    if (i + 1 < v.size() && v[i + 1].rel == v[i].rel && v[i + 1].stype == v[i].stype &&
        v[i + 1].srel == v[i].srel && v[i + 1].obj == v[i].obj && v[i + 1].sid == v[i].sid)
      continue;
    v[w++] = v[i];
  }
  v.resize(w);
  e.n_tuples = w;

  std::vector<HostCSR> out;
  size_t i = 0;
  while (i < v.size()) {
    size_t j = i;
    while (j < v.size() && v[j].rel == v[i].rel && v[j].stype == v[i].stype && v[j].srel == v[i].srel) ++j;
    const uint32_t n_rows = e.interner[sc.rels[v[i].rel].type].count;
    for (int ext = 0; ext < 2; ++ext) {
      HostCSR h;
      h.rel = v[i].rel;
      h.stype = v[i].stype;
      h.srel = v[i].srel;
      h.ext = ext == 1;
      h.n_rows = n_rows;
      h.off.assign((size_t)n_rows + 1, 0);
      for (size_t k = i; k < j; ++k) {
        bool is_ext = v[k].cav != 0 || v[k].exp_us != 0;
        if (is_ext == h.ext) h.off[v[k].obj + 1]++;
      }
      std::partial_sum(h.off.begin(), h.off.end(), h.off.begin());
      if (h.off.back() == 0) continue;
      h.nbr.reserve(h.off.back());
      for (size_t k = i; k < j; ++k) {  // already sorted by (obj, sid)
        bool is_ext = v[k].cav != 0 || v[k].exp_us != 0;
        if (is_ext != h.ext) continue;
        h.nbr.push_back(v[k].sid);
        if (h.ext) {
          h.cav.push_back(v[k].cav);
          h.exp_us.push_back(v[k].exp_us);
        }
      }
      out.push_back(std::move(h));
    }
    i = j;
  }
  // prebuilt CSRs (gck_load_csr)
  for (HostCSR& p : e.prebuilt) {
    for (const HostCSR& h : out)
      if (h.rel == p.rel && h.stype == p.stype && h.srel == p.srel && !h.ext)
        throw Error(GCK_E_INVALID_ARGUMENT, "a CSR was loaded for a subject kind that also has staged tuples");
    if (p.n_rows != e.interner[sc.rels[p.rel].type].count)
      throw Error(GCK_E_INVALID_ARGUMENT, "prebuilt CSR row count does not match the type's object count");
    e.n_tuples += p.dev_off ? p.n_edges : p.nbr.size();
    out.push_back(std::move(p));
  }
  e.prebuilt.clear();
  return out;
}

}  // namespace gck

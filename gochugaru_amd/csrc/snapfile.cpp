// snapfile.cpp — on-disk snapshot cache: the committed snapshot of an engine,
// keyed by its schema text and revision, written once and loaded by later processes instead of
// re-running ExportRelationships (client/client.go:472-499) + interning + CSR construction.
//
// What is stored is exactly what a commit starts from: the interner (named ids per type and the
// id count, anonymous reserved ids included), the caveat instances (name + stored context, in
// id order), and every base CSR (offsets, neighbours, and for caveated / expiring edges the
// caveat instance and expiration per edge). Derived device structures (membership indexes,
// transposed CSRs, ancestor closures, heights) are rebuilt on load by the same device_upload a
// commit uses, so a loaded engine is indistinguishable from the one that saved it.
//
// Layout (native little-endian): "GCKSNAP" 0x01, u64 schema length + schema text, u64 revision,
// u64 tuple count, u32 types { u32 count, u32 named { u32 id, u32 len, bytes } }, u32 caveat
// instances (excluding the "none" instance 0) { u32 len, name, u32 len, json }, u32 CSRs { u16
// relation, u16 subject type, u16 subject relation, u8 ext, u8 0, u32 rows, u64 edges, u32
// off[rows+1], u32 nbr[edges], ext: u32 cav[edges], i64 expires_at_us[edges] }, u64 end marker.
#include <cstdio>
#include <cstring>

#include "engine.hpp"

namespace gck {

namespace {

constexpr char kMagic[8] = {'G', 'C', 'K', 'S', 'N', 'A', 'P', 0x01};
constexpr uint64_t kEnd = 0x444E455041534B43ull;  // "CKSAPEND"

struct File {
  FILE* f = nullptr;
  std::string path;
  File(const std::string& p, const char* mode) : path(p) {
    f = fopen(p.c_str(), mode);
    if (!f) throw Error(GCK_E_INVALID_ARGUMENT, "cannot open snapshot file '" + p + "'");
  }
  ~File() {
    if (f) fclose(f);
  }
  void put(const void* p, size_t n) {
    if (n && fwrite(p, 1, n, f) != n) throw Error(GCK_E_INVALID_ARGUMENT, "short write to '" + path + "'");
  }
  void get(void* p, size_t n) {
    if (n && fread(p, 1, n, f) != n) throw Error(GCK_E_INVALID_ARGUMENT, "truncated snapshot file '" + path + "'");
  }
  template <class T> void put_v(T v) { put(&v, sizeof(T)); }
  template <class T> T get_v() {
    T v;
    get(&v, sizeof(T));
    return v;
  }
  void put_s(const std::string& s) {
    put_v<uint32_t>((uint32_t)s.size());
    put(s.data(), s.size());
  }
  std::string get_s(size_t limit) {
    const uint32_t n = get_v<uint32_t>();
    if (n > limit) throw Error(GCK_E_INVALID_ARGUMENT, "corrupt snapshot file '" + path + "'");
    std::string s(n, '\0');
    get(&s[0], n);
    return s;
  }
};

}  // namespace

void save_snapshot_file(Engine& e, const std::string& path) {
  if (!e.committed || !e.dev) throw Error(GCK_E_STATE, "no committed snapshot to save");
  if (e.part_world > 1) throw Error(GCK_E_STATE, "a partitioned engine holds only its rank's rows");
  std::vector<HostCSR> csrs;
  device_export(e, csrs);
  const std::string tmp = path + ".tmp";
  {
    File f(tmp, "wb");
    f.put(kMagic, sizeof(kMagic));
    f.put_v<uint64_t>(e.schema_text.size());
    f.put(e.schema_text.data(), e.schema_text.size());
    f.put_v<uint64_t>(e.revision);
    f.put_v<uint64_t>(e.n_tuples);
    f.put_v<uint32_t>((uint32_t)e.interner.size());
    for (const TypeInterner& ti : e.interner) {
      f.put_v<uint32_t>(ti.count);
      uint32_t named = 0;
      for (const std::string& s : ti.names) named += !s.empty();
      f.put_v<uint32_t>(named);
      for (uint32_t id = 0; id < ti.names.size(); ++id) {
        if (ti.names[id].empty()) continue;
        f.put_v<uint32_t>(id);
        f.put_s(ti.names[id]);
      }
    }
    f.put_v<uint32_t>((uint32_t)e.caveat_instances.size() - 1);
    for (size_t k = 1; k < e.caveat_instances.size(); ++k) {
      f.put_s(e.caveat_instances[k].first);
      f.put_s(e.caveat_instances[k].second);
    }
    f.put_v<uint32_t>((uint32_t)csrs.size());
    for (const HostCSR& h : csrs) {
      f.put_v<uint16_t>(h.rel);
      f.put_v<uint16_t>(h.stype);
      f.put_v<uint16_t>(h.srel);
      f.put_v<uint8_t>(h.ext ? 1 : 0);
      f.put_v<uint8_t>(0);
      f.put_v<uint32_t>(h.n_rows);
      f.put_v<uint64_t>(h.nbr.size());
      f.put(h.off.data(), h.off.size() * 4);
      f.put(h.nbr.data(), h.nbr.size() * 4);
      if (h.ext) {
        f.put(h.cav.data(), h.cav.size() * 4);
        f.put(h.exp_us.data(), h.exp_us.size() * 8);
      }
    }
    f.put_v<uint64_t>(kEnd);
    if (fflush(f.f) != 0) throw Error(GCK_E_INVALID_ARGUMENT, "short write to '" + tmp + "'");
  }
  if (rename(tmp.c_str(), path.c_str()) != 0)  // readers never see a partial file
    throw Error(GCK_E_INVALID_ARGUMENT, "cannot rename '" + tmp + "' to '" + path + "'");
}

void load_snapshot_file(Engine& e, const std::string& path) {
  if (!e.schema) throw Error(GCK_E_STATE, "gck_load_schema first");
  if (e.staging) throw Error(GCK_E_STATE, "a snapshot is being staged");
  if (e.part_world > 1) throw Error(GCK_E_STATE, "a partitioned engine holds only its rank's rows");
  File f(path, "rb");
  char magic[8];
  f.get(magic, sizeof(magic));
  if (memcmp(magic, kMagic, sizeof(kMagic)) != 0)
    throw Error(GCK_E_INVALID_ARGUMENT, "'" + path + "' is not a gck snapshot file");
  const uint64_t slen = f.get_v<uint64_t>();
  if (slen != e.schema_text.size()) throw Error(GCK_E_SCHEMA, "snapshot file was saved under another schema");
  std::string stext(slen, '\0');
  f.get(&stext[0], slen);
  if (stext != e.schema_text) throw Error(GCK_E_SCHEMA, "snapshot file was saved under another schema");
  const Schema& sc = *e.schema;
  const uint64_t revision = f.get_v<uint64_t>();
  const uint64_t n_tuples = f.get_v<uint64_t>();
  const uint32_t n_types = f.get_v<uint32_t>();
  if (n_types != sc.types.size()) throw Error(GCK_E_INVALID_ARGUMENT, "corrupt snapshot file (types)");
  std::vector<TypeInterner> interner(n_types);
  for (TypeInterner& ti : interner) {
    ti.count = f.get_v<uint32_t>();
    const uint32_t named = f.get_v<uint32_t>();
    if (named > ti.count || ti.count >= GCK_ID_ABSENT) throw Error(GCK_E_INVALID_ARGUMENT, "corrupt snapshot file (ids)");
    for (uint32_t k = 0; k < named; ++k) {
      const uint32_t id = f.get_v<uint32_t>();
      if (id >= ti.count) throw Error(GCK_E_INVALID_ARGUMENT, "corrupt snapshot file (ids)");
      std::string name = f.get_s(1u << 20);
      if (ti.names.size() <= id) ti.names.resize((size_t)id + 1);
      ti.ids.emplace(name, id);
      ti.names[id] = std::move(name);
    }
  }
  const uint32_t n_cav = f.get_v<uint32_t>();
  std::vector<std::pair<std::string, std::string>> cavs(n_cav);
  for (auto& c : cavs) {
    c.first = f.get_s(1u << 16);
    c.second = f.get_s(1u << 26);
  }
  const uint32_t n_csrs = f.get_v<uint32_t>();
  std::vector<HostCSR> csrs(n_csrs);
  uint64_t total = 0;
  for (HostCSR& h : csrs) {
    h.rel = f.get_v<uint16_t>();
    h.stype = f.get_v<uint16_t>();
    h.srel = f.get_v<uint16_t>();
    h.ext = f.get_v<uint8_t>() != 0;
    (void)f.get_v<uint8_t>();
    h.n_rows = f.get_v<uint32_t>();
    const uint64_t ne = f.get_v<uint64_t>();
    // the kind must be one the schema allows, with one row per object of the relation's type and
    // neighbours that are objects of the subject type (or the wildcard, where allowed), each row
    // strictly ascending: what build_csrs produces and device_upload's kernels index by
    bool allowed = false, wildcard = false;
    if (h.rel < sc.rels.size() && !sc.rels[h.rel].is_perm) {
      for (const Allowed& a : sc.rels[h.rel].allowed) {
        allowed |= a.stype == h.stype && a.srel == h.srel;
        wildcard |= a.wildcard && a.stype == h.stype && h.srel == kEllipsis;
      }
    }
    if (!allowed || ne >= 0xFFFFFFFFull || h.stype >= n_types)
      throw Error(GCK_E_INVALID_ARGUMENT, "corrupt snapshot file (CSR)");
    // (a CSR no Watch batch touched since objects were added has fewer rows than the count:
    // kernels test obj < n_rows before reading a row)
    if (h.n_rows > interner[sc.rels[h.rel].type].count)
      throw Error(GCK_E_INVALID_ARGUMENT, "corrupt snapshot file (CSR rows exceed the object count)");
    h.off.resize((size_t)h.n_rows + 1);
    f.get(h.off.data(), h.off.size() * 4);
    if (h.off[0] != 0 || h.off.back() != ne) throw Error(GCK_E_INVALID_ARGUMENT, "corrupt snapshot file (offsets)");
    for (uint32_t r = 0; r < h.n_rows; ++r)
      if (h.off[r] > h.off[r + 1]) throw Error(GCK_E_INVALID_ARGUMENT, "corrupt snapshot file (offsets)");
    h.nbr.resize(ne);
    f.get(h.nbr.data(), ne * 4);
    const uint32_t n_subjects = interner[h.stype].count;
    for (uint32_t r = 0; r < h.n_rows; ++r)
      for (uint32_t k = h.off[r]; k < h.off[r + 1]; ++k) {
        const uint32_t v = h.nbr[k];
        if (!(v < n_subjects || (v == GCK_ID_WILDCARD && wildcard)) || (k > h.off[r] && h.nbr[k - 1] >= v))
          throw Error(GCK_E_INVALID_ARGUMENT, "corrupt snapshot file (neighbours)");
      }
    if (h.ext) {
      h.cav.resize(ne);
      h.exp_us.resize(ne);
      f.get(h.cav.data(), ne * 4);
      f.get(h.exp_us.data(), ne * 8);
      for (uint32_t c : h.cav)
        if (c > n_cav) throw Error(GCK_E_INVALID_ARGUMENT, "corrupt snapshot file (caveat instance)");
    }
    total += ne;
  }
  if (f.get_v<uint64_t>() != kEnd) throw Error(GCK_E_INVALID_ARGUMENT, "corrupt snapshot file (end marker)");
  if (total != n_tuples) throw Error(GCK_E_INVALID_ARGUMENT, "corrupt snapshot file (tuple count)");
  // install: caveat instances keep their ids (the CSRs refer to them), then the device upload;
  // on any failure the engine keeps its previous interner, caveat tables and device snapshot
  auto cav_instances = e.caveat_instances;
  auto cav_ids = e.caveat_ids;
  auto cav_expr = e.caveat_expr;
  auto cav_ctx = e.caveat_ctx;
  auto cav_static = e.caveat_static;
  auto cav_row = e.caveat_row;
  auto cav_partial = e.caveat_partial;
  std::swap(e.interner, interner);
  try {
    reset_caveats(e);
    for (uint32_t k = 0; k < n_cav; ++k)
      if (add_caveat_instance(e, cavs[k].first, cavs[k].second) != k + 1)
        throw Error(GCK_E_INVALID_ARGUMENT, "corrupt snapshot file (duplicate caveat instance)");
    device_upload(e, csrs);
  } catch (...) {
    std::swap(e.interner, interner);
    e.caveat_instances = std::move(cav_instances);
    e.caveat_ids = std::move(cav_ids);
    e.caveat_expr = std::move(cav_expr);
    e.caveat_ctx = std::move(cav_ctx);
    e.caveat_static = std::move(cav_static);
    e.caveat_row = std::move(cav_row);
    e.caveat_partial = std::move(cav_partial);
    throw;
  }
  e.prebuilt.clear();
  e.staged.clear();
  e.n_tuples = n_tuples;
  e.revision = revision;
  e.committed = true;
}

}  // namespace gck

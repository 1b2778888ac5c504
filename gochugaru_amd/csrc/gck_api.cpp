// gck_api.cpp — the extern "C" boundary (include/gck.h). Every entry point converts C++
// exceptions into a negative status plus a thread-local message (gck_last_error).
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <thread>

#include "engine.hpp"

namespace gck {

thread_local std::string g_last_error;

#define REQUIRE(cond, code, msg) \
  do {                           \
    if (!(cond)) throw Error(code, msg); \
  } while (0)

Engine::~Engine() {
  device_free(*this);
  host_free_all(*this);
}

void reset_caveats(Engine& e) {
  ++e.shape_gen;  // (with the schema and a snapshot file: the interner starts over too)
  e.caveat_instances.assign(1, {"", ""});
  e.caveat_ids.clear();
  e.caveat_expr.assign(1, nullptr);
  e.caveat_ctx.assign(1, cel::Object{});
  e.caveat_static.assign(1, (uint8_t)cel::TRUE);  // instance 0: no caveat
  e.caveat_row.assign(1, kNone);
  e.caveat_partial.clear();
}

// A caveat name + stored context (rel.Relationship.CaveatName/CaveatContext,
// rel/relationship.go:93-120). Identical pairs share one instance. The stored context is parsed
// and the expression evaluated over it alone once, here: a caveat it decides is a plain or an
// absent edge for every check; one left PARTIAL gets a row of the per-call outcome table.
uint32_t add_caveat_instance(Engine& e, const std::string& name, const std::string& json) {
  auto cd = e.schema->caveats.find(name);
  if (cd == e.schema->caveats.end()) throw Error(GCK_E_INVALID_ARGUMENT, "unknown caveat '" + name + "'");
  std::string key = name;
  key += '\0';
  key += json;
  auto hit = e.caveat_ids.find(key);
  if (hit != e.caveat_ids.end()) return hit->second;
  REQUIRE(e.caveat_instances.size() < 0xFFFFFFF0u, GCK_E_CAPACITY, "too many caveat instances");
  cel::Object ctx = cel::parse_context(json);
  const cel::Outcome o = cel::evaluate(*cd->second.expr, &ctx, nullptr);
  const uint32_t id = (uint32_t)e.caveat_instances.size();
  e.caveat_instances.emplace_back(name, json);
  e.caveat_expr.push_back(cd->second.expr);
  e.caveat_ctx.push_back(std::move(ctx));
  e.caveat_static.push_back((uint8_t)o);
  e.caveat_row.push_back(o == cel::PARTIAL ? (uint32_t)e.caveat_partial.size() : kNone);
  if (o == cel::PARTIAL) e.caveat_partial.push_back(id);
  e.caveat_ids.emplace(std::move(key), id);
  return id;
}

// The check-time caveat contexts of one call (engine.hpp CavCall). Each partial instance r
// (caveat_partial[r]) under context slot k + 1 (CheckBulkPermissionsRequestItem.Context,
// client/client.go:257) is evaluated with the instance's stored context taking precedence.
// While instances x contexts is small every pair is evaluated here into a dense table (identical
// context texts share their evaluations); beyond that the contexts are only copied, and the pairs
// a walk touches are parsed and evaluated on demand (engine.hip caveat_passes). An evaluation
// error is outcome 3: it fails only the checks whose walk meets it (GCK_ITEM_ERR_CAVEAT_EVAL).
constexpr size_t kDensePairs = 4096;  // evaluations done eagerly

static CavCall caveat_call(Engine& e, const char* const* ctxs, const size_t* lens, size_t n_ctx) {
  CavCall c;
  c.n_given = (uint32_t)std::min<size_t>(n_ctx, 0xFFFFFFFFu);
  const size_t rows = e.caveat_partial.size();
  if (n_ctx == 0 || rows == 0) return c;
  REQUIRE(n_ctx < (1ull << 31), GCK_E_INVALID_ARGUMENT, "too many check contexts");
  c.n_ctx = (uint32_t)n_ctx;
  if (!(e.cfg.flags & GCK_FLAG_LAZY_CAVEATS) && rows <= kDensePairs) {
    std::unordered_map<std::string_view, uint32_t> seen;
    seen.reserve(std::min<size_t>(n_ctx, 4 * kDensePairs));
    std::vector<std::string_view> dist;
    c.of_slot.resize(n_ctx);
    for (size_t k = 0; k < n_ctx && rows * dist.size() <= kDensePairs; ++k) {
      const std::string_view js(ctxs[k] ? ctxs[k] : "", ctxs[k] ? lens[k] : 0);
      auto it = seen.emplace(js, (uint32_t)dist.size()).first;
      if (it->second == dist.size()) dist.push_back(js);
      c.of_slot[k] = it->second;
    }
    if (rows * dist.size() <= kDensePairs) {
      const size_t nd = dist.size();
      c.n_dist = (uint32_t)nd;
      c.dense.resize(rows * nd);
      for (size_t k = 0; k < nd; ++k) {
        const cel::Object ctx = cel::parse_context(std::string(dist[k]));  // a malformed context fails the call
        for (size_t r = 0; r < rows; ++r) {
          const uint32_t id = e.caveat_partial[r];
          try {
            c.dense[r * nd + k] = (uint8_t)cel::evaluate(*e.caveat_expr[id], &e.caveat_ctx[id], &ctx);
          } catch (const Error&) {
            c.dense[r * nd + k] = 3;
          }
        }
      }
      return c;
    }
    c.of_slot.clear();
  }
  // lazy: one copy of the texts (a context is parsed when a walk first needs it; a malformed one
  // then fails the call)
  size_t total = 0;
  for (size_t k = 0; k < n_ctx; ++k) total += ctxs[k] ? lens[k] : 0;
  REQUIRE(total < (1ull << 32), GCK_E_INVALID_ARGUMENT, "check contexts above 4 GiB");
  auto text = std::make_shared<std::string>();
  auto off = std::make_shared<std::vector<uint32_t>>(n_ctx + 1);
  text->reserve(total);
  for (size_t k = 0; k < n_ctx; ++k) {
    (*off)[k] = (uint32_t)text->size();
    if (ctxs[k]) text->append(ctxs[k], lens[k]);
  }
  (*off)[n_ctx] = (uint32_t)text->size();
  c.text = std::move(text);
  c.off = std::move(off);
  return c;
}

void stage_tuple(Engine& e, const gck_tuple& t);
void stage_tuples(Engine& e, const gck_tuple* t, size_t n);

}  // namespace gck

using namespace gck;

// Watch batches staged ahead of their apply (gck_watch_stage): an engine-owned thread validates
// and groups batch k + 1 while batch k applies — a Watch consumer (client/client.go:370-413)
// receives the next batch while it applies the previous one. Each staged batch has its own
// grouping buffers; kSlots may be staged at once. The stager reads the schema and the interner
// under the engine lock held shared and briefly (group_updates' schema_mu), and records the
// engine's shape generation: a batch staged before a write that moved it is regrouped at apply.
struct WatchStager {
  static constexpr int kSlots = 4;
  struct Slot {
    const gck_update* ups = nullptr;
    size_t n = 0;
    uint64_t ticket = 0;  // 0: free
    int state = 0;        // 1 queued, 3 being grouped, 2 grouped (or failed)
    bool ok = false;
    uint64_t gen = 0;
    std::vector<gck_update> mine;  // (a partitioned rank's own updates)
    GroupBuffers buf;
    const std::vector<UpdateGroup>* groups = nullptr;
  } slots[kSlots];
  std::mutex m;
  std::condition_variable cv_job, cv_done;
  // two threads: a consumer holding the next two responses has both grouped beside its apply (the
  // grouping of one config-5 batch takes about as long as an apply, ~80-100 us)
  static constexpr int kThreads = 2;
  std::thread th[kThreads];
  bool stop = false;
  uint64_t next_ticket = 1;
  ~WatchStager() {
    {
      std::lock_guard<std::mutex> g(m);
      stop = true;
    }
    cv_job.notify_all();
    for (std::thread& t : th)
      if (t.joinable()) t.join();
  }
};

struct gck_engine {
  Engine impl;
  WatchStager stage;  // (destroyed first: its thread ends before the engine does)
};

template <class F>
static int guard(F&& f) {
  try {
    f();  // (a success leaves the message of the thread's last failure, as errno: a caller's loop that
          // drains its batches after an error still reads that error's message)
    return GCK_OK;
  } catch (const Error& ex) {
    g_last_error = ex.what();
    return ex.code;
  } catch (const std::bad_alloc&) {
    g_last_error = "host out of memory";
    return GCK_E_CAPACITY;
  } catch (const std::exception& ex) {
    g_last_error = ex.what();
    return GCK_E_INVALID_ARGUMENT;
  }
}

static Engine& need(gck_engine* e) {
  REQUIRE(e, GCK_E_INVALID_ARGUMENT, "null engine");
  return e->impl;
}

static Schema& need_schema(Engine& e) {
  REQUIRE(e.schema, GCK_E_STATE, "no schema loaded (gck_load_schema)");
  return *e.schema;
}

extern "C" {

// What changes the engine's state — schema, snapshot, Watch batches, caveat instances, partition
// — is serialised by Engine::writer_mu and holds the engine lock exclusively; a Watch batch takes
// the exclusive lock only to start and to publish its snapshot (apply_updates).
struct WriterLock {
  std::lock_guard<std::mutex> w;
  std::unique_lock<std::shared_mutex> lk;
  explicit WriterLock(Engine& e) : w(e.writer_mu), lk(e.mu) {}
};

static_assert(sizeof(gck_config) == 88, "gck_config layout (include/gck.h) changed: bump GCK_ABI_VERSION");
static_assert(sizeof(gck_stats) == 240, "gck_stats layout (include/gck.h) changed: bump GCK_ABI_VERSION");
static_assert(sizeof(gck_item) == 20 && sizeof(gck_tuple) == 32 && sizeof(gck_update) == 40, "item/tuple/update layout");

int gck_abi_version(void) { return GCK_ABI_VERSION; }

const char* gck_last_error(void) { return g_last_error.c_str(); }

int gck_create(const gck_config* cfg, gck_engine** out) {
  return guard([&] {
    REQUIRE(out, GCK_E_INVALID_ARGUMENT, "null out pointer");
    *out = nullptr;
    auto* e = new gck_engine();
    if (cfg) e->impl.cfg = *cfg;
    if (e->impl.cfg.device < 0) {
      delete e;
      throw Error(GCK_E_INVALID_ARGUMENT, "bad device ordinal");
    }
    if (e->impl.cfg.max_depth > 250) {  // frontier entries hold the depth in 8 bits
      delete e;
      throw Error(GCK_E_INVALID_ARGUMENT, "max_depth above 250");
    }
    reset_caveats(e->impl);
    *out = e;
  });
}

void gck_destroy(gck_engine* e) { delete e; }

int gck_load_schema(gck_engine* ge, const char* text, size_t len) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(text || !len, GCK_E_INVALID_ARGUMENT, "null schema text");
    auto sc = compile_schema(std::string(text ? text : "", len));
    WriterLock lk(e);
    drain_batches(e);
    e.schema = std::move(sc);
    partition_rules(e);
    e.schema_text.assign(text ? text : "", len);
    e.interner.assign(e.schema->types.size(), TypeInterner());
    reset_caveats(e);
    e.staged.clear();
    e.prebuilt.clear();
    e.staging = false;
    e.committed = false;
    device_free(e);
  });
}

int gck_type_id(gck_engine* ge, const char* name, size_t len, uint16_t* out) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(out && (name || !len), GCK_E_INVALID_ARGUMENT, "null argument");
    int t = need_schema(e).find_type(std::string(name, len));
    REQUIRE(t >= 0, GCK_E_NOT_FOUND, "unknown type '" + std::string(name, len) + "'");
    *out = (uint16_t)t;
  });
}

int gck_relation_id(gck_engine* ge, uint16_t type, const char* name, size_t len, uint16_t* out) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(out && (name || !len), GCK_E_INVALID_ARGUMENT, "null argument");
    int r = need_schema(e).find_rel(type, std::string(name, len));
    REQUIRE(r >= 0, GCK_E_NOT_FOUND, "unknown relation '" + std::string(name, len) + "'");
    *out = (uint16_t)r;
  });
}

int gck_type_count(gck_engine* ge, uint32_t* out) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(out, GCK_E_INVALID_ARGUMENT, "null out");
    *out = (uint32_t)need_schema(e).types.size();
  });
}

int gck_relation_count(gck_engine* ge, uint32_t* out) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(out, GCK_E_INVALID_ARGUMENT, "null out");
    *out = (uint32_t)need_schema(e).rels.size();
  });
}

int gck_intern(gck_engine* ge, uint16_t type, const char* const* ids, const uint32_t* lens, size_t n,
               uint32_t flags, uint32_t* out_ids) {
  return guard([&] {
    Engine& e = need(ge);
    Schema& sc = need_schema(e);
    REQUIRE(type < sc.types.size(), GCK_E_INVALID_ARGUMENT, "unknown type id");
    REQUIRE(n == 0 || (ids && lens && out_ids), GCK_E_INVALID_ARGUMENT, "null argument");
    const bool create = flags & GCK_INTERN_CREATE;
    // creating ids is a write of the interner: it takes the writer lock as every writer does, so
    // that no Watch batch is between its interner mark and its rollback meanwhile (a text batch
    // that fails truncates the interner to the counts it recorded, gck_apply_updates_text)
    std::unique_lock<std::mutex> wlk(e.writer_mu, std::defer_lock);
    std::unique_lock<std::shared_mutex> lk(e.mu, std::defer_lock);
    std::shared_lock<std::shared_mutex> slk(e.mu, std::defer_lock);
    if (create) {
      wlk.lock();
      lk.lock();
    } else {
      slk.lock();
    }
    TypeInterner& ti = e.interner[type];
    std::string key;
    for (size_t i = 0; i < n; ++i) {
      key.assign(ids[i], lens[i]);
      if (key == "*") {
        out_ids[i] = GCK_ID_WILDCARD;
        continue;
      }
      auto it = ti.ids.find(key);
      if (it != ti.ids.end()) {
        out_ids[i] = it->second;
      } else if (create) {
        // (a partitioned graph: only a name's owner gives it an id, gck_part_intern_with)
        REQUIRE(e.part_world <= 1, GCK_E_STATE, "a partitioned engine interns a new name through its owner rank "
                                                "(gck_part_intern_with): '" + key + "'");
        REQUIRE(ti.count < GCK_ID_ABSENT, GCK_E_CAPACITY, "too many objects of one type");
        uint32_t id = ti.count++;
        ti.ids.emplace(key, id);
        if (ti.names.size() < ti.count) ti.names.resize(ti.count);
        ti.names[id] = key;
        out_ids[i] = id;
      } else {
        out_ids[i] = GCK_ID_ABSENT;
      }
    }
  });
}

int gck_object_count(gck_engine* ge, uint16_t type, uint32_t* out) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(type < need_schema(e).types.size() && out, GCK_E_INVALID_ARGUMENT, "bad argument");
    *out = e.interner[type].count;
  });
}

int gck_reserve_objects(gck_engine* ge, uint16_t type, uint32_t n) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(type < need_schema(e).types.size(), GCK_E_INVALID_ARGUMENT, "bad type");
    REQUIRE(n < GCK_ID_ABSENT, GCK_E_CAPACITY, "too many objects");
    WriterLock lk(e);
    TypeInterner& ti = e.interner[type];
    if (n > ti.count) ti.count = n;
  });
}

int gck_object_name(gck_engine* ge, uint16_t type, uint32_t id, char* buf, size_t cap, size_t* out_len) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(type < need_schema(e).types.size(), GCK_E_INVALID_ARGUMENT, "bad type");
    TypeInterner& ti = e.interner[type];
    REQUIRE(id < ti.count, GCK_E_NOT_FOUND, "unknown object id");
    auto rv = ti.rev.find(id);
    std::string nm = id < ti.names.size() && !ti.names[id].empty() ? ti.names[id]
                     : rv != ti.rev.end()                           ? rv->second
                                                                    : std::to_string(id);
    if (out_len) *out_len = nm.size();
    if (buf && cap) {
      size_t k = std::min(cap - 1, nm.size());
      std::memcpy(buf, nm.data(), k);
      buf[k] = 0;
    }
  });
}

int gck_add_caveat_instance(gck_engine* ge, const char* name, size_t name_len, const char* json,
                            size_t json_len, uint32_t* out_id) {
  return guard([&] {
    Engine& e = need(ge);
    need_schema(e);
    REQUIRE(name && out_id, GCK_E_INVALID_ARGUMENT, "null argument");
    WriterLock lk(e);
    *out_id = add_caveat_instance(e, std::string(name, name_len), std::string(json ? json : "", json_len));
  });
}

int gck_evaluate_caveat(gck_engine* ge, const char* name, size_t name_len, const char* stored_json,
                        size_t stored_len, const char* context_json, size_t context_len, uint8_t* out) {
  return guard([&] {
    Engine& e = need(ge);
    Schema& sc = need_schema(e);
    REQUIRE(name && out, GCK_E_INVALID_ARGUMENT, "null argument");
    auto cd = sc.caveats.find(std::string(name, name_len));
    REQUIRE(cd != sc.caveats.end(), GCK_E_NOT_FOUND, "unknown caveat '" + std::string(name, name_len) + "'");
    const cel::Object st = cel::parse_context(std::string(stored_json ? stored_json : "", stored_json ? stored_len : 0));
    const cel::Object cx = cel::parse_context(std::string(context_json ? context_json : "", context_json ? context_len : 0));
    *out = (uint8_t)cel::evaluate(*cd->second.expr, &st, &cx);
  });
}

int gck_begin_snapshot(gck_engine* ge, uint64_t revision) {
  return guard([&] {
    Engine& e = need(ge);
    need_schema(e);
    WriterLock lk(e);
    e.staging = true;
    e.staged_revision = revision;
    e.staged.clear();
    e.prebuilt.clear();
    e.seq = 0;
  });
}

int gck_add_tuples(gck_engine* ge, const gck_tuple* tuples, size_t n) {
  return guard([&] {
    Engine& e = need(ge);
    need_schema(e);
    REQUIRE(e.staging, GCK_E_STATE, "gck_begin_snapshot first");
    REQUIRE(n == 0 || tuples, GCK_E_INVALID_ARGUMENT, "null tuples");
    WriterLock lk(e);
    stage_tuples(e, tuples, n);
  });
}

int gck_add_tuples_text(gck_engine* ge, const char* text, size_t len) {
  return guard([&] {
    Engine& e = need(ge);
    need_schema(e);
    REQUIRE(e.staging, GCK_E_STATE, "gck_begin_snapshot first");
    REQUIRE(text || !len, GCK_E_INVALID_ARGUMENT, "null text");
    WriterLock lk(e);
    add_tuples_text(e, text, len);
  });
}

int gck_load_csr(gck_engine* ge, uint16_t relation, uint16_t subject_type, uint16_t subject_relation,
                 uint32_t n_rows, const uint32_t* offsets, const uint32_t* neighbours, uint64_t n_edges,
                 uint32_t mem_flags) {
  return guard([&] {
    Engine& e = need(ge);
    Schema& sc = need_schema(e);
    REQUIRE(e.staging, GCK_E_STATE, "gck_begin_snapshot first");
    REQUIRE(relation < sc.rels.size() && !sc.rels[relation].is_perm, GCK_E_INVALID_ARGUMENT,
            "gck_load_csr: not a relation");
    REQUIRE(subject_type < sc.types.size(), GCK_E_INVALID_ARGUMENT, "gck_load_csr: bad subject type");
    bool allowed = false;
    for (const Allowed& a : sc.rels[relation].allowed)
      if (a.stype == subject_type && a.srel == subject_relation) allowed = true;
    REQUIRE(allowed, GCK_E_INVALID_ARGUMENT, "gck_load_csr: subject kind not allowed by the schema");
    REQUIRE(offsets && (neighbours || !n_edges), GCK_E_INVALID_ARGUMENT, "gck_load_csr: null arrays");
    REQUIRE(n_edges < 0xFFFFFFFFull, GCK_E_CAPACITY, "gck_load_csr: more than 2^32-1 edges in one CSR");
    WriterLock lk(e);
    HostCSR h;
    h.rel = relation;
    h.stype = subject_type;
    h.srel = subject_relation;
    h.ext = false;
    h.n_rows = n_rows;
    h.n_edges = n_edges;
    if (mem_flags & GCK_MEM_DEVICE) {  // (a partitioned engine copies only what it keeps: device_upload)
      h.dev_off = offsets;
      h.dev_nbr = neighbours;
    } else {
      REQUIRE(offsets[n_rows] == n_edges && offsets[0] == 0, GCK_E_INVALID_ARGUMENT,
              "gck_load_csr: offsets do not span the neighbour array");
      if (e.part_world > 1) {  // partitioned graph: the rows and subjects this rank keeps (part_keep)
        h.off.assign((size_t)n_rows + 1, 0);
        for (uint32_t r = 0; r < n_rows; ++r) {
          for (uint32_t k = offsets[r]; k < offsets[r + 1]; ++k)
            if (part_keep(e, relation, r, neighbours[k], subject_relation)) h.nbr.push_back(neighbours[k]);
          h.off[r + 1] = (uint32_t)h.nbr.size();
        }
        h.n_edges = h.nbr.size();
      } else {
        h.off.assign(offsets, offsets + (size_t)n_rows + 1);
        h.nbr.assign(neighbours, neighbours + n_edges);
      }
    }
    e.prebuilt.push_back(std::move(h));
  });
}

int gck_commit_snapshot(gck_engine* ge) {
  return guard([&] {
    Engine& e = need(ge);
    need_schema(e);
    REQUIRE(e.staging, GCK_E_STATE, "gck_begin_snapshot first");
    WriterLock lk(e);
    drain_batches(e);
    std::vector<HostCSR> csrs = build_csrs(e);
    device_upload(e, csrs);  // device-pointer CSRs are copied before the caller regains control
    ensure_pool(e);          // no check ever creates a workspace (engine.hip ensure_pool)
    e.staged.clear();
    e.staged.shrink_to_fit();
    e.staging = false;
    e.revision = e.staged_revision;
    e.committed = true;
  });
}

int gck_save_snapshot(gck_engine* ge, const char* path) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(path, GCK_E_INVALID_ARGUMENT, "null path");
    WriterLock lk(e);  // no Watch batch may move the snapshot meanwhile
    save_snapshot_file(e, path);
  });
}

int gck_load_snapshot_file(gck_engine* ge, const char* path) {
  return guard([&] {
    Engine& e = need(ge);
    need_schema(e);
    REQUIRE(path, GCK_E_INVALID_ARGUMENT, "null path");
    WriterLock lk(e);
    drain_batches(e);
    load_snapshot_file(e, path);
    ensure_pool(e);
  });
}

int gck_revision(gck_engine* ge, uint64_t* out) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(out, GCK_E_INVALID_ARGUMENT, "null out");
    std::shared_lock<std::shared_mutex> lk(e.mu);
    *out = e.revision;
  });
}

int gck_set_head_revision(gck_engine* ge, uint64_t revision) {
  return guard([&] {
    Engine& e = need(ge);
    WriterLock lk(e);
    if (revision > e.head_revision) e.head_revision = revision;  // the head only moves forward
  });
}

int gck_tuple_count(gck_engine* ge, uint64_t* out) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(out, GCK_E_INVALID_ARGUMENT, "null out");
    *out = e.n_tuples;
  });
}

int gck_device_bytes(gck_engine* ge, uint64_t* out) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(out, GCK_E_INVALID_ARGUMENT, "null out");
    *out = device_bytes(e);
  });
}

// Watch batch: validated and grouped on the host first (nothing is applied if any update is
// rejected), then merged on the device and the next snapshot derived from it (delta.inc) BESIDE
// the checks: the engine lock is held shared meanwhile, so checks keep running on the current
// snapshot; it is taken exclusively again only to finish the batches in flight, patch the
// membership indexes and swap the snapshot in (device_apply_publish). `lk` (exclusive, with
// writer_mu held) is released and re-acquired here. A device failure loses the snapshot.
// `staged`: the batch's groups, made ahead by the stager (gck_watch_apply_staged)
static void apply_updates(Engine& e, std::unique_lock<std::shared_mutex>& lk, uint64_t revision, const gck_update* ups,
                          size_t n, const std::vector<UpdateGroup>* staged = nullptr) {
  REQUIRE(e.committed, GCK_E_STATE, "no snapshot committed");
  REQUIRE(revision > e.revision || (n == 0 && revision == e.revision), GCK_E_REVISION,
          "update revision " + std::to_string(revision) + " is not newer than the snapshot's " +
              std::to_string(e.revision));
  PhaseClock pc("watch");
  std::vector<gck_update> mine;
  if (e.part_world > 1 && !staged) {  // partitioned graph: the updates of what this rank keeps (part_keep)
    // the whole batch validated first, as every rank validates it: an update another rank would
    // keep and reject fails the batch here too (every rank stays at the old revision)
    validate_updates(e, ups, n);
    for (size_t i = 0; i < n; ++i) {
      const gck_tuple& t = ups[i].tuple;
      if (part_keep(e, t.relation, t.resource_id, t.subject_id, t.subject_relation)) mine.push_back(ups[i]);
    }
    ups = mine.data();
    n = mine.size();
  }
  // validation and grouping read the interner and the schema, which only writers change (and
  // writer_mu holds them off): beside the checks too
  WatchBuild wb;
  lk.unlock();
  bool built = false;
  try {
    std::shared_lock<std::shared_mutex> sl(e.mu);  // (checks run on the current snapshot meanwhile)
    // (the engine's, until the next batch; or the staged batch's)
    const std::vector<UpdateGroup>& groups = staged ? *staged : group_updates(e, ups, n);
    pc.mark("group");
    if (!groups.empty()) device_apply_build(e, groups, wb);
    built = true;
  } catch (...) {
    lk.lock();
    if (!built && !wb.ds && wb.fresh.empty()) throw;  // rejected before anything was built: nothing lost
    device_apply_abort(e, wb);
    e.committed = false;
    throw;
  }
  pc.mark("build");
  lk.lock();
  try {
    device_apply_publish(e, wb);
    pc.mark("publish");
  } catch (...) {
    device_apply_abort(e, wb);
    e.committed = false;
    throw;
  }
  e.revision = revision;
}

int gck_apply_updates(gck_engine* ge, uint64_t revision, const gck_update* updates, size_t n) {
  return guard([&] {
    Engine& e = need(ge);
    need_schema(e);
    REQUIRE(n == 0 || updates, GCK_E_INVALID_ARGUMENT, "null updates");
    PhaseClock pc("watch_call");
    {
      WriterLock wl(e);
      pc.mark("lock");
      // (read in place: no copy of the batch)
      apply_updates(e, wl.lk, revision, updates, n);
      pc.mark("apply");
    }
    pc.mark("unlock");
  });
}

// The CPUs of a sysfs cpu list ("0-7,64-71").
static std::vector<int> cpu_list(const char* path) {
  std::vector<int> out;
  FILE* f = std::fopen(path, "r");
  if (!f) return out;
  char buf[4096];
  const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  buf[n] = 0;
  for (char* p = buf; *p;) {
    char* end;
    const long a = std::strtol(p, &end, 10);
    if (end == p) break;
    long b = a;
    if (*end == '-') b = std::strtol(end + 1, &end, 10);
    for (long c = a; c <= b && c < 65536; ++c) out.push_back((int)c);
    p = *end ? end + 1 : end;
  }
  return out;
}

// Places the stager on the applying thread's last-level cache (its L3 domain minus its own core):
// the applying thread reads every record the stager wrote, which then stays in that cache instead
// of crossing between core complexes (config 5: ~30 us of a 0.2 ms step). Left to the scheduler
// when the topology cannot be read.
static void stager_place(int caller_cpu) {
  if (caller_cpu < 0) return;
  char path[128];
  std::snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list", caller_cpu);
  std::vector<int> l3 = cpu_list(path);
  std::snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list", caller_cpu);
  const std::vector<int> sib = cpu_list(path);
  cpu_set_t allowed;
  if (l3.empty() || sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return;
  cpu_set_t set;
  CPU_ZERO(&set);
  int n = 0;
  for (int c : l3)
    if (c < CPU_SETSIZE && CPU_ISSET(c, &allowed) && std::find(sib.begin(), sib.end(), c) == sib.end()) {
      CPU_SET(c, &set);
      ++n;
    }
  if (n) (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
}

// The stager's thread: groups the queued batches in ticket order.
static void stager_loop(gck_engine* ge, int caller_cpu) {
  if (!debug_env("GCK_STAGER_ANYWHERE")) stager_place(caller_cpu);
  Engine& e = ge->impl;
  WatchStager& st = ge->stage;
  std::unique_lock<std::mutex> g(st.m);
  for (;;) {
    WatchStager::Slot* s = nullptr;
    for (;;) {
      for (WatchStager::Slot& x : st.slots)
        if (x.state == 1 && (!s || x.ticket < s->ticket)) s = &x;
      if (s || st.stop) break;
      st.cv_job.wait(g);
    }
    if (!s) return;
    s->state = 3;  // (the other thread takes the next queued one)
    const gck_update* ups = s->ups;
    size_t n = s->n;
    g.unlock();
    bool ok = false;
    uint64_t gen = 0;
    const std::vector<UpdateGroup>* groups = nullptr;
    try {
      bool part;
      {
        std::shared_lock<std::shared_mutex> sl(e.mu);
        gen = e.shape_gen;
        part = e.part_world > 1;
        if (part) {  // (as apply_updates: the whole batch validated, then this rank's updates kept)
          validate_updates(e, ups, n);
          s->mine.clear();
          for (size_t i = 0; i < n; ++i) {
            const gck_tuple& t = ups[i].tuple;
            if (part_keep(e, t.relation, t.resource_id, t.subject_id, t.subject_relation)) s->mine.push_back(ups[i]);
          }
        }
      }
      if (part) {
        ups = s->mine.data();
        n = s->mine.size();
      }
      groups = &group_updates(e, s->buf, ups, n, &e.mu);
      ok = true;
    } catch (...) {
      ok = false;  // (gck_watch_apply_staged regroups it under the writer lock and reports the error)
    }
    g.lock();
    s->ok = ok;
    s->gen = gen;
    s->groups = groups;
    s->state = 2;
    st.cv_done.notify_all();
  }
}

int gck_watch_stage(gck_engine* ge, const gck_update* updates, size_t n, uint64_t* ticket) {
  return guard([&] {
    Engine& e = need(ge);
    need_schema(e);
    REQUIRE(ticket && (n == 0 || updates), GCK_E_INVALID_ARGUMENT, "null argument");
    WatchStager& st = ge->stage;
    std::lock_guard<std::mutex> g(st.m);
    WatchStager::Slot* s = nullptr;
    for (WatchStager::Slot& x : st.slots)
      if (!x.ticket) {
        s = &x;
        break;
      }
    REQUIRE(s, GCK_E_CAPACITY, "every staging slot holds a batch: apply or discard one first");
    for (std::thread& t : st.th)
      if (!t.joinable()) t = std::thread(stager_loop, ge, sched_getcpu());
    s->ups = updates;
    s->n = n;
    s->ticket = st.next_ticket++;
    s->state = 1;
    s->ok = false;
    s->groups = nullptr;
    *ticket = s->ticket;
    st.cv_job.notify_all();
  });
}

// Waits for the staged batch and frees its slot afterwards (whatever happens)
struct StagedSlot {
  WatchStager& st;
  WatchStager::Slot* s = nullptr;
  StagedSlot(WatchStager& w, uint64_t ticket) : st(w) {
    std::unique_lock<std::mutex> g(st.m);
    for (WatchStager::Slot& x : st.slots)
      if (ticket && x.ticket == ticket) s = &x;
    if (!s) throw Error(GCK_E_INVALID_ARGUMENT, "no staged Watch batch with ticket " + std::to_string(ticket));
    st.cv_done.wait(g, [&] { return s->state == 2; });
  }
  ~StagedSlot() {
    std::lock_guard<std::mutex> g(st.m);
    s->ticket = 0;
    s->state = 0;
    s->groups = nullptr;
  }
};

int gck_watch_apply_staged(gck_engine* ge, uint64_t revision, uint64_t ticket) {
  return guard([&] {
    Engine& e = need(ge);
    need_schema(e);
    StagedSlot ss(ge->stage, ticket);
    PhaseClock pc("watch_call");
    WriterLock wl(e);
    pc.mark("lock");
    // grouped against the engine's current shape: applied as staged; else (a write moved the
    // shape since, or the staging failed) grouped again here, where any error is reported
    if (ss.s->ok && ss.s->gen == e.shape_gen)
      apply_updates(e, wl.lk, revision, ss.s->ups, ss.s->n, ss.s->groups);
    else
      apply_updates(e, wl.lk, revision, ss.s->ups, ss.s->n);
    pc.mark("apply");
  });
}

int gck_watch_discard(gck_engine* ge, uint64_t ticket) {
  return guard([&] {
    need(ge);
    StagedSlot ss(ge->stage, ticket);
  });
}

// What a text Watch batch may add before it is known to apply: new interned ids (CREATE of an
// unseen object) and new caveat instances. A rejected batch takes them back, so that nothing of
// it stays (interner counts are also the CSR row counts of the next batch).
struct InternMark {
  std::vector<uint32_t> counts;
  size_t n_cav = 0, n_partial = 0;
};

static InternMark intern_mark(const Engine& e) {
  InternMark m;
  for (const TypeInterner& ti : e.interner) m.counts.push_back(ti.count);
  m.n_cav = e.caveat_instances.size();
  m.n_partial = e.caveat_partial.size();
  return m;
}

static void intern_rollback(Engine& e, const InternMark& m) {
  ++e.shape_gen;
  for (size_t t = 0; t < m.counts.size() && t < e.interner.size(); ++t) {
    TypeInterner& ti = e.interner[t];
    for (uint32_t id = m.counts[t]; id < ti.names.size(); ++id)
      if (!ti.names[id].empty()) ti.ids.erase(ti.names[id]);
    if (ti.names.size() > m.counts[t]) ti.names.resize(m.counts[t]);
    ti.count = m.counts[t];
  }
  for (size_t id = m.n_cav; id < e.caveat_instances.size(); ++id) {
    std::string key = e.caveat_instances[id].first;  // add_caveat_instance's key
    key += '\0';
    key += e.caveat_instances[id].second;
    e.caveat_ids.erase(key);
  }
  e.caveat_instances.resize(m.n_cav);
  e.caveat_expr.resize(m.n_cav);
  e.caveat_ctx.resize(m.n_cav);
  e.caveat_static.resize(m.n_cav);
  e.caveat_row.resize(m.n_cav);
  e.caveat_partial.resize(m.n_partial);
}

int gck_apply_updates_text(gck_engine* ge, uint64_t revision, const char* text, size_t len) {
  return guard([&] {
    Engine& e = need(ge);
    need_schema(e);
    REQUIRE(text || !len, GCK_E_INVALID_ARGUMENT, "null text");
    WriterLock wl(e);
    REQUIRE(e.committed, GCK_E_STATE, "no snapshot committed");
    // the revision first: a stale batch is refused before its text is read
    REQUIRE(revision > e.revision || (len == 0 && revision == e.revision), GCK_E_REVISION,
            "update revision " + std::to_string(revision) + " is not newer than the snapshot's " +
                std::to_string(e.revision));
    drain_batches(e);
    const InternMark mark = intern_mark(e);
    try {
      std::vector<gck_update> ups;
      parse_updates_text(e, text, len, ups);
      apply_updates(e, wl.lk, revision, ups.data(), ups.size());
    } catch (...) {
      intern_rollback(e, mark);  // (apply_updates returns or throws with the lock held)
      throw;
    }
  });
}

// consistency.Strategy (consistency/consistency.go:15-77) against the applied revision. A
// requirement the snapshot has not reached yet is GCK_E_REVISION (gRPC Unavailable: the client
// retries, client/client.go:193-211, while the Watch stream catches up); a Snapshot revision the
// snapshot has moved past can never be served here (no MVCC on the device) and is permanent.
static void check_consistency(Engine& e, const gck_consistency* cs) {
  if (!cs) return;
  switch (cs->requirement) {
    case GCK_CONSISTENCY_MIN_LATENCY:
      return;
    case GCK_CONSISTENCY_FULL:
      REQUIRE(e.revision >= e.head_revision, GCK_E_REVISION,
              "snapshot revision " + std::to_string(e.revision) + " has not reached the head revision " +
                  std::to_string(e.head_revision));
      return;
    case GCK_CONSISTENCY_AT_LEAST:
      REQUIRE(e.revision >= cs->revision, GCK_E_REVISION,
              "snapshot revision " + std::to_string(e.revision) + " is older than the requested " +
                  std::to_string(cs->revision));
      return;
    case GCK_CONSISTENCY_SNAPSHOT:
      REQUIRE(e.revision <= cs->revision, GCK_E_REVISION_GONE,
              "snapshot revision " + std::to_string(cs->revision) + " is no longer available (the local snapshot is at " +
                  std::to_string(e.revision) + ")");
      REQUIRE(e.revision == cs->revision, GCK_E_REVISION,
              "snapshot revision " + std::to_string(e.revision) + " has not reached the requested " +
                  std::to_string(cs->revision));
      return;
    default:
      throw Error(GCK_E_INVALID_ARGUMENT, "unknown consistency requirement");
  }
}

// State errors before any workspace is taken (a workspace needs the device the first commit set
// up): no snapshot, or a partitioned engine.
static void precheck(Engine& e) {
  std::shared_lock<std::shared_mutex> lk(e.mu);
  REQUIRE(e.committed, GCK_E_STATE, "no snapshot committed");
  REQUIRE(e.part_world <= 1, GCK_E_STATE, "partitioned engine: use gck_part_* (every rank together)");
}

// The checks common to every check entry point (under the shared engine lock).
static void check_request(Engine& e, const gck_consistency* cs, const gck_item* items, size_t n, bool host_items,
                          const char* const* contexts, const size_t* context_lens, size_t n_contexts) {
  REQUIRE(e.committed, GCK_E_STATE, "no snapshot committed");
  REQUIRE(n_contexts == 0 || (contexts && context_lens), GCK_E_INVALID_ARGUMENT, "null contexts");
  REQUIRE(n_contexts < 0xFFFFFFFFull, GCK_E_INVALID_ARGUMENT, "too many contexts");
  REQUIRE(e.part_world <= 1, GCK_E_STATE, "partitioned engine: use gck_part_* (every rank together)");
  check_consistency(e, cs);
  // (a host item's context_slot is validated by its batch: the join of a zero-copy batch checks
  // every item it reads, the others are scanned before they are staged — engine.hip submit_batch;
  // a scan here read every host item once more on the submitting thread, ~27 us per 64K batch)
  (void)items;
  (void)n;
  (void)host_items;
}

int gck_check_bulk_at(gck_engine* ge, const gck_consistency* cs, const gck_item* items, size_t n,
                      const char* const* contexts, const size_t* context_lens, size_t n_contexts,
                      int64_t now_us, uint8_t* out_perm, int32_t* out_err, uint64_t* out_revision) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(n == 0 || (items && out_perm && out_err), GCK_E_INVALID_ARGUMENT, "null buffers");
    if (n == 0) {  // empty request -> empty response (client/client_test.go:203-207)
      std::shared_lock<std::shared_mutex> lk(e.mu);
      check_request(e, cs, items, 0, true, contexts, context_lens, n_contexts);
      if (out_revision) *out_revision = e.revision;
      return;
    }
    // workspaces first, then the engine lock (engine.hpp WsLease)
    precheck(e);
    // a request above max_batch alternates over two workspaces, taken in one step (never one
    // held while waiting for the other: acquire_ws_n)
    const size_t mb = e.cfg.max_batch ? e.cfg.max_batch : 65536;
    Workspace* ws[2] = {nullptr, nullptr};
    acquire_ws_n(e, n > mb ? 2 : 1, ws);
    struct Release {
      Engine& e;
      Workspace** ws;
      ~Release() {
        release_ws(e, ws[0]);
        if (ws[1] && ws[1] != ws[0]) release_ws(e, ws[1]);
      }
    } rel{e, ws};
    // (the shared lock is held until the results are written: no Watch batch publishes meanwhile,
    // so the revision read here is the one every chunk runs on)
    std::shared_lock<std::shared_mutex> lk(e.mu);
    check_request(e, cs, items, n, true, contexts, context_lens, n_contexts);
    const CavCall cav = caveat_call(e, contexts, context_lens, n_contexts);
    const uint64_t rev = e.revision;
    device_check_host(e, ws[0], ws[1], items, n, now_us, out_perm, out_err, cav);
    if (out_revision) *out_revision = rev;
  });
}

int gck_check_bulk_ctx(gck_engine* ge, const gck_consistency* cs, const gck_item* items, size_t n,
                       const char* const* contexts, const size_t* context_lens, size_t n_contexts,
                       int64_t now_us, uint8_t* out_perm, int32_t* out_err) {
  return gck_check_bulk_at(ge, cs, items, n, contexts, context_lens, n_contexts, now_us, out_perm, out_err, nullptr);
}

int gck_check_bulk(gck_engine* ge, const gck_consistency* cs, const gck_item* items, size_t n,
                   int64_t now_us, uint8_t* out_perm, int32_t* out_err) {
  return gck_check_bulk_at(ge, cs, items, n, nullptr, nullptr, 0, now_us, out_perm, out_err, nullptr);
}

// A uniform request's header against the call (include/gck.h gck_uniform): its context slot is
// every pair's, so it is checked once here.
static void check_uniform(const gck_uniform* h, size_t n_contexts) {
  REQUIRE(h, GCK_E_INVALID_ARGUMENT, "null header");
  REQUIRE(h->context_slot <= n_contexts, GCK_E_INVALID_ARGUMENT,
          "uniform header: context_slot " + std::to_string(h->context_slot) + " beyond the " +
              std::to_string(n_contexts) + " contexts given");
}

int gck_check_bulk_uniform(gck_engine* ge, const gck_consistency* cs, const gck_uniform* hdr, const uint32_t* pairs,
                           size_t n, const char* const* contexts, const size_t* context_lens, size_t n_contexts,
                           int64_t now_us, uint64_t* out_packed, gck_item_error* out_errs, size_t err_cap,
                           size_t* out_n_errs, uint64_t* out_revision) {
  return guard([&] {
    Engine& e = need(ge);
    check_uniform(hdr, n_contexts);
    REQUIRE(n == 0 || (pairs && out_packed), GCK_E_INVALID_ARGUMENT, "null buffers");
    REQUIRE(err_cap == 0 || out_errs, GCK_E_INVALID_ARGUMENT, "null error list");
    if (out_n_errs) *out_n_errs = 0;
    if (n == 0) {
      std::shared_lock<std::shared_mutex> lk(e.mu);
      check_request(e, cs, nullptr, 0, true, contexts, context_lens, n_contexts);
      if (out_revision) *out_revision = e.revision;
      return;
    }
    precheck(e);
    const size_t mb = e.cfg.max_batch ? e.cfg.max_batch : 65536;
    Workspace* ws[2] = {nullptr, nullptr};
    acquire_ws_n(e, n > (mb & ~(size_t)31) ? 2 : 1, ws);
    struct Release {
      Engine& e;
      Workspace** ws;
      ~Release() {
        release_ws(e, ws[0]);
        if (ws[1] && ws[1] != ws[0]) release_ws(e, ws[1]);
      }
    } rel{e, ws};
    std::shared_lock<std::shared_mutex> lk(e.mu);
    check_request(e, cs, nullptr, n, true, contexts, context_lens, n_contexts);
    const CavCall cav = caveat_call(e, contexts, context_lens, n_contexts);
    const uint64_t rev = e.revision;
    device_check_uniform(e, ws[0], ws[1], *hdr, pairs, n, now_us, out_packed, out_errs, err_cap, out_n_errs, cav);
    if (out_revision) *out_revision = rev;
  });
}

int gck_check_bulk_device_ctx(gck_engine* ge, const gck_item* d_items, size_t n, const char* const* contexts,
                              const size_t* context_lens, size_t n_contexts, int64_t now_us,
                              uint8_t* d_out_perm, int32_t* d_out_err, void* stream) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(n == 0 || (d_items && d_out_perm && d_out_err), GCK_E_INVALID_ARGUMENT, "null buffers");
    if (n == 0) {
      std::shared_lock<std::shared_mutex> lk(e.mu);
      check_request(e, nullptr, nullptr, 0, false, contexts, context_lens, n_contexts);
      return;
    }
    precheck(e);
    WsLease l0(e);
    std::shared_lock<std::shared_mutex> lk(e.mu);
    check_request(e, nullptr, nullptr, 0, false, contexts, context_lens, n_contexts);
    device_check(e, *l0.w, d_items, n, now_us, d_out_perm, d_out_err, stream,
                 caveat_call(e, contexts, context_lens, n_contexts));
  });
}

int gck_check_bulk_device(gck_engine* ge, const gck_item* d_items, size_t n, int64_t now_us,
                          uint8_t* d_out_perm, int32_t* d_out_err, void* stream) {
  return gck_check_bulk_device_ctx(ge, d_items, n, nullptr, nullptr, 0, now_us, d_out_perm, d_out_err, stream);
}

// A submitted batch: the workspace it holds (returned to the pool by the wait), or, for an empty
// batch, nothing to do.
struct gck_batch {
  Workspace* w = nullptr;
  uint64_t revision = 0;  // the snapshot's revision at submit: the one the batch runs on
};

int gck_check_submit(gck_engine* ge, const gck_consistency* cs, const gck_item* items, size_t n,
                     const char* const* contexts, const size_t* context_lens, size_t n_contexts, int64_t now_us,
                     uint8_t* out_perm, int32_t* out_err, uint32_t flags, void* stream, gck_batch** out) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(out, GCK_E_INVALID_ARGUMENT, "null out");
    *out = nullptr;
    REQUIRE(n == 0 || (items && out_perm && out_err), GCK_E_INVALID_ARGUMENT, "null buffers");
    const bool host = !(flags & GCK_SUBMIT_DEVICE);
    auto* b = new gck_batch();
    if (n == 0) {
      std::shared_lock<std::shared_mutex> lk(e.mu);
      try {
        check_request(e, cs, items, 0, host, contexts, context_lens, n_contexts);
        b->revision = e.revision;
      } catch (...) {
        delete b;
        throw;
      }
      *out = b;
      return;
    }
    precheck(e);
    Workspace* w = acquire_ws(e);  // before the engine lock (engine.hpp WsLease)
    try {
      std::shared_lock<std::shared_mutex> lk(e.mu);
      check_request(e, cs, items, n, host, contexts, context_lens, n_contexts);
      b->revision = e.revision;
      device_submit(e, w, items, n, now_us, out_perm, out_err, stream, host, !host && (flags & GCK_SUBMIT_ENGINE_STREAM),
                    caveat_call(e, contexts, context_lens, n_contexts));
    } catch (...) {
      release_ws(e, w);
      delete b;
      throw;
    }
    b->w = w;
    *out = b;
  });
}

int gck_check_submit_uniform(gck_engine* ge, const gck_consistency* cs, const gck_uniform* hdr, const uint32_t* pairs,
                             size_t n, const char* const* contexts, const size_t* context_lens, size_t n_contexts,
                             int64_t now_us, uint64_t* out_packed, gck_item_error* out_errs, size_t err_cap,
                             size_t* out_n_errs, gck_batch** out) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(out, GCK_E_INVALID_ARGUMENT, "null out");
    *out = nullptr;
    check_uniform(hdr, n_contexts);
    REQUIRE(n == 0 || (pairs && out_packed), GCK_E_INVALID_ARGUMENT, "null buffers");
    REQUIRE(err_cap == 0 || out_errs, GCK_E_INVALID_ARGUMENT, "null error list");
    if (out_n_errs) *out_n_errs = 0;
    auto* b = new gck_batch();
    if (n == 0) {
      std::shared_lock<std::shared_mutex> lk(e.mu);
      try {
        check_request(e, cs, nullptr, 0, true, contexts, context_lens, n_contexts);
        b->revision = e.revision;
      } catch (...) {
        delete b;
        throw;
      }
      *out = b;
      return;
    }
    precheck(e);
    Workspace* w = acquire_ws(e);
    try {
      std::shared_lock<std::shared_mutex> lk(e.mu);
      check_request(e, cs, nullptr, n, true, contexts, context_lens, n_contexts);
      b->revision = e.revision;
      device_submit_uniform(e, w, *hdr, pairs, n, now_us, out_packed, out_errs, err_cap, out_n_errs,
                            caveat_call(e, contexts, context_lens, n_contexts));
    } catch (...) {
      release_ws(e, w);
      delete b;
      throw;
    }
    b->w = w;
    *out = b;
  });
}

int gck_host_alloc(gck_engine* ge, size_t bytes, void** out) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(out, GCK_E_INVALID_ARGUMENT, "null out");
    *out = host_alloc(e, bytes);
  });
}

int gck_host_free(gck_engine* ge, void* p) {
  return guard([&] {
    Engine& e = need(ge);
    if (p) host_free(e, p);
  });
}

int gck_check_wait(gck_engine* ge, gck_batch* b) { return gck_check_wait_at(ge, b, nullptr); }

int gck_check_wait_at(gck_engine* ge, gck_batch* b, uint64_t* out_revision) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(b, GCK_E_INVALID_ARGUMENT, "null batch");
    std::unique_ptr<gck_batch> own(b);
    if (out_revision) *out_revision = b->revision;
    if (!b->w) return;
    Workspace* w = b->w;
    try {
      device_wait(e, w);
    } catch (...) {
      release_ws(e, w);
      throw;
    }
    release_ws(e, w);
  });
}

int gck_set_partition(gck_engine* ge, uint32_t rank, uint32_t world) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(world >= 1 && world <= 63 && rank < world, GCK_E_INVALID_ARGUMENT, "bad rank / world");
    WriterLock lk(e);
    REQUIRE(!e.committed && !e.dev && e.ws_pool.empty() && !e.part_ws && e.staged.empty() && e.prebuilt.empty(),
            GCK_E_STATE, "gck_set_partition must precede the first snapshot");
    e.part_rank = rank;
    e.part_world = world;
    e.part_set = true;
    ++e.shape_gen;
    partition_rules(e);
    // the bundles and the bidirectional search need the whole graph; the membership indexes serve
    // the bundles: a partitioned rank's checks are decided by the partitioned label join from the
    // slots, and its level loop (what the join leaves) finds a subject in a row by binary search —
    // at 1e9 tuples the index of the kept memberships alone would be 13 of a rank's 29 GB
    if (world > 1) e.cfg.flags |= GCK_FLAG_NO_BUNDLE | GCK_FLAG_NO_BIDIR | GCK_FLAG_NO_MHASH;
  });
}

uint32_t gck_partition_owner_name(uint16_t type, const char* name, size_t len, uint32_t world) {
  return part_owner_name(type, name ? name : "", name ? len : 0, world);
}

int gck_part_intern_with(gck_engine* ge, const gck_transport* t, const uint16_t* types, const char* const* names,
                         const uint32_t* lens, size_t n, uint32_t flags, uint32_t* out_ids) {
  return guard([&] {
    Engine& e = need(ge);
    need_schema(e);
    REQUIRE(t, GCK_E_INVALID_ARGUMENT, "null transport");
    REQUIRE(n == 0 || (types && names && lens && out_ids), GCK_E_INVALID_ARGUMENT, "null argument");
    WriterLock lk(e);  // (the interner changes; every rank's call blocks in the exchange together)
    part_intern(e, *t, types, names, lens, n, (flags & GCK_INTERN_CREATE) != 0, out_ids);
  });
}

int gck_part_add_tuples_text_with(gck_engine* ge, const gck_transport* t, const char* text, size_t len) {
  return guard([&] {
    Engine& e = need(ge);
    need_schema(e);
    REQUIRE(t, GCK_E_INVALID_ARGUMENT, "null transport");
    REQUIRE(text || !len, GCK_E_INVALID_ARGUMENT, "null text");
    WriterLock lk(e);
    REQUIRE(e.staging, GCK_E_STATE, "gck_begin_snapshot first");
    part_add_tuples_text(e, *t, text, len);
  });
}

int gck_interned_names(gck_engine* ge, uint16_t type, uint32_t* out) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(out, GCK_E_INVALID_ARGUMENT, "null out");
    REQUIRE(type < need_schema(e).types.size(), GCK_E_INVALID_ARGUMENT, "bad type");
    std::shared_lock<std::shared_mutex> lk(e.mu);
    *out = (uint32_t)e.interner[type].ids.size();
  });
}

uint32_t gck_partition_owner(uint32_t object_id, uint32_t world) {
  return world <= 1 ? 0u : part_owner(object_id, world);
}

int gck_part_unique_id(uint8_t* out) {
  return guard([&] {
    REQUIRE(out, GCK_E_INVALID_ARGUMENT, "null id buffer");
    part_unique_id(out);
  });
}

int gck_part_init(gck_engine* ge, const uint8_t* id) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(id, GCK_E_INVALID_ARGUMENT, "null id");
    WriterLock lk(e);
    part_init(e, id);
  });
}

int gck_part_check(gck_engine* ge, const gck_item* d_items, size_t n, int64_t now_us, uint8_t* d_out_perm,
                   int32_t* d_out_err, void* stream) {
  return guard([&] {
    Engine& e = need(ge);
    std::shared_lock<std::shared_mutex> lk(e.mu);
    REQUIRE(e.committed, GCK_E_STATE, "no snapshot committed");
    REQUIRE(n == 0 || (d_items && d_out_perm && d_out_err), GCK_E_INVALID_ARGUMENT, "null buffers");
    part_check(e, d_items, n, now_us, d_out_perm, d_out_err, stream);
  });
}

int gck_part_check_with(gck_engine* ge, const gck_transport* t, const gck_item* d_items, size_t n, int64_t now_us,
                        uint8_t* d_out_perm, int32_t* d_out_err, void* stream) {
  return guard([&] {
    Engine& e = need(ge);
    std::shared_lock<std::shared_mutex> lk(e.mu);
    REQUIRE(e.committed, GCK_E_STATE, "no snapshot committed");
    REQUIRE(t, GCK_E_INVALID_ARGUMENT, "null transport");
    REQUIRE(n == 0 || (d_items && d_out_perm && d_out_err), GCK_E_INVALID_ARGUMENT, "null buffers");
    part_check_with(e, *t, d_items, n, now_us, d_out_perm, d_out_err, stream);
  });
}

// The result of a lookup that did not fit the caller's buffer, kept per thread so that the retry
// with cap >= *out_n copies it out without a second sweep. It matches only a retry of the same
// request on the same snapshot (process-wide snapshot generation) at the same explicit now_us
// (now_us = 0, the wall clock, never matches), and is dropped once copied out.
struct LookupCache {
  uint64_t generation = 0;  // 0 = empty
  gck_item proto{};
  bool vary_res = false;
  int64_t now_us = 0;
  std::vector<uint32_t> ids;
  std::vector<uint8_t> perms;
};
thread_local LookupCache g_lookup;

static void lookup(gck_engine* ge, const gck_consistency* cs, const gck_item& proto, bool vary_res, int64_t now_us,
                   uint32_t* out_ids, uint8_t* out_perm, size_t cap, size_t* out_n) {
  Engine& e = need(ge);
  REQUIRE(out_n && (cap == 0 || (out_ids && out_perm)), GCK_E_INVALID_ARGUMENT, "null buffers");
  {
    std::shared_lock<std::shared_mutex> lk(e.mu);
    REQUIRE(e.committed, GCK_E_STATE, "no snapshot committed");
    REQUIRE(e.part_world <= 1, GCK_E_STATE, "lookups are not available on a partitioned engine");
  }
  WsLease lease(e);  // before the engine lock (engine.hpp WsLease)
  std::shared_lock<std::shared_mutex> lk(e.mu);
  REQUIRE(e.committed, GCK_E_STATE, "no snapshot committed");
  REQUIRE(e.part_world <= 1, GCK_E_STATE, "lookups are not available on a partitioned engine");
  check_consistency(e, cs);
  const Schema& sc = *e.schema;
  REQUIRE(proto.resource_type < sc.types.size() && proto.subject_type < sc.types.size(), GCK_E_NOT_FOUND,
          "object definition not found");
  REQUIRE(proto.permission < sc.rels.size() && sc.rels[proto.permission].type == proto.resource_type,
          GCK_E_NOT_FOUND, "relation/permission not found");
  REQUIRE(proto.subject_relation == GCK_ELLIPSIS ||
              (proto.subject_relation < sc.rels.size() && sc.rels[proto.subject_relation].type == proto.subject_type),
          GCK_E_NOT_FOUND, "subject relation not found");
  const bool hit = now_us != 0 && g_lookup.generation != 0 && g_lookup.generation == e.generation &&
                   g_lookup.vary_res == vary_res && g_lookup.now_us == now_us &&
                   std::memcmp(&g_lookup.proto, &proto, sizeof(gck_item)) == 0;
  if (!hit) {
    g_lookup.generation = 0;
    if (vary_res) {
      device_lookup(e, *lease.w, proto, true, e.interner[proto.resource_type].count, now_us, g_lookup.ids,
                    g_lookup.perms);
    } else {
      device_lookup_subjects(e, *lease.w, proto, now_us, g_lookup.ids, g_lookup.perms);
    }
    g_lookup.generation = e.generation;
    g_lookup.proto = proto;
    g_lookup.vary_res = vary_res;
    g_lookup.now_us = now_us;
  }
  *out_n = g_lookup.ids.size();
  REQUIRE(cap >= g_lookup.ids.size(), GCK_E_CAPACITY,
          "lookup result has " + std::to_string(g_lookup.ids.size()) + " ids: retry with that capacity");
  if (!g_lookup.ids.empty()) {
    std::memcpy(out_ids, g_lookup.ids.data(), g_lookup.ids.size() * 4);
    std::memcpy(out_perm, g_lookup.perms.data(), g_lookup.perms.size());
  }
  g_lookup.generation = 0;
  g_lookup.ids.clear();
  g_lookup.perms.clear();
}

int gck_lookup_resources(gck_engine* ge, const gck_consistency* cs, uint16_t resource_type, uint16_t permission,
                         uint16_t subject_type, uint16_t subject_relation, uint32_t subject_id, int64_t now_us,
                         uint32_t* out_ids, uint8_t* out_perm, size_t cap, size_t* out_n) {
  return guard([&] {
    REQUIRE(subject_id != GCK_ID_WILDCARD, GCK_E_INVALID_ARGUMENT, "cannot perform lookup on wildcard subject");
    gck_item proto{resource_type, permission, 0, subject_type, subject_relation, subject_id, 0};
    lookup(ge, cs, proto, true, now_us, out_ids, out_perm, cap, out_n);
  });
}

int gck_lookup_subjects(gck_engine* ge, const gck_consistency* cs, uint16_t resource_type, uint32_t resource_id,
                        uint16_t permission, uint16_t subject_type, uint16_t subject_relation, int64_t now_us,
                        uint32_t* out_ids, uint8_t* out_perm, size_t cap, size_t* out_n) {
  return guard([&] {
    gck_item proto{resource_type, permission, resource_id, subject_type, subject_relation, 0, 0};
    lookup(ge, cs, proto, false, now_us, out_ids, out_perm, cap, out_n);
  });
}

int gck_last_stats(gck_engine* ge, gck_stats* out) {
  return guard([&] {
    Engine& e = need(ge);
    REQUIRE(out, GCK_E_INVALID_ARGUMENT, "null out");
    *out = e.stats;
  });
}

int gck_set_profile(gck_engine* ge, uint32_t on) {
  return guard([&] {
    Engine& e = need(ge);
    std::unique_lock<std::shared_mutex> lk(e.mu);  // no batch is being submitted
    if (on) e.cfg.flags |= GCK_FLAG_PROFILE;
    else e.cfg.flags &= ~GCK_FLAG_PROFILE;
  });
}

int gck_reset_stats(gck_engine* ge) {
  return guard([&] {
    Engine& e = need(ge);
    e.stats = gck_stats{};
  });
}

}  // extern "C"

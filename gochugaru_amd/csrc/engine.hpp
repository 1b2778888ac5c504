// engine.hpp — host-side engine state: compiled schema, interner, snapshot staging and the
// device-resident snapshot + workspace. Everything behind the C ABI in include/gck.h.
#pragma once
#include <cstdint>
#include <cstdlib>
#include <map>
#include <memory>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "cel.hpp"
#include "gck.h"
#include "gck_internal.hpp"

namespace gck {

// Diagnostic switches (GCK_DEBUG_*, GCK_STAGER_ANYWHERE): read from the environment only in the
// debug build (make DEBUG=1 -> libgck_debug.so, -DGCK_DEBUG_KNOBS=1; load it with GCK_LIBRARY=...).
// The product library ignores them: none changes a result, and none may change its timing.
inline const char* debug_env(const char* name) {
#if GCK_DEBUG_KNOBS
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// ---- schema IR ------------------------------------------------------------------------------
struct Allowed {
  uint16_t stype = 0;
  uint16_t srel = kEllipsis;
  bool wildcard = false;
  bool expiration = false;
  std::string caveat;
};

struct Expr {
  enum Op { UNION, INTERSECT, EXCLUDE, NIL, COMPUTED, ARROW } op = NIL;
  std::vector<Expr> kids;
  std::string name;      // COMPUTED relation / ARROW target
  std::string tupleset;  // ARROW tupleset relation
  bool all = false;      // ARROW: .all()
};

struct RelDef {
  std::string name;
  uint16_t type = 0;
  bool is_perm = false;
  std::vector<Allowed> allowed;  // relation
  Expr expr;                     // permission
};

struct TypeDef {
  std::string name;
  std::unordered_map<std::string, uint16_t> rels;  // name -> global relation id
};

struct CaveatDef {
  std::string name;
  std::vector<std::pair<std::string, std::string>> params;
  std::string body;
  std::shared_ptr<const cel::Node> expr;  // compiled body (cel.hpp)
};

struct Schema {
  std::vector<TypeDef> types;
  std::unordered_map<std::string, uint16_t> type_ids;
  std::vector<RelDef> rels;
  std::unordered_map<std::string, CaveatDef> caveats;
  bool use_expiration = false;
  // compiled node program; DevItem csr fields are linked at snapshot commit
  std::vector<DevNode> nodes;
  std::vector<DevItem> items;
  std::vector<uint16_t> item_rel;  // relation whose CSR an IT_KIND/IT_ARROW item reads

  int find_type(const std::string& n) const {
    auto it = type_ids.find(n);
    return it == type_ids.end() ? -1 : it->second;
  }
  int find_rel(uint16_t t, const std::string& n) const {
    if (t >= types.size()) return -1;
    auto it = types[t].rels.find(n);
    return it == types[t].rels.end() ? -1 : it->second;
  }
};

// Parses and validates SpiceDB schema DSL text, then compiles the node program.
// Throws Error(GCK_E_SCHEMA, ...) on failure.
std::unique_ptr<Schema> compile_schema(const std::string& text);

// ---- interner -------------------------------------------------------------------------------
struct TypeInterner {
  std::unordered_map<std::string, uint32_t> ids;
  std::vector<std::string> names;  // names[id] ("" for anonymous reserved ids)
  uint32_t count = 0;              // ids [0, count) exist
  // a partitioned graph (partition.inc part_intern): the names this rank owns get ids
  // local * world + rank in order; the names of other ranks' objects it needs are kept with the
  // ids their owners gave, id -> name here (names[] would span the whole id space)
  uint32_t local = 0;
  std::unordered_map<uint32_t, std::string> rev;
};

// ---- snapshot staging -----------------------------------------------------------------------
struct StagedTuple {
  uint16_t rel, stype, srel, pad;
  uint32_t obj, sid, cav;
  int64_t exp_us;
  uint64_t seq;  // arrival order: the last write of a duplicate wins (TOUCH)
};

struct HostCSR {
  uint16_t rel, stype, srel;
  bool ext;
  uint32_t n_rows;
  std::vector<uint32_t> off, nbr, cav;
  std::vector<int64_t> exp_us;
  // prebuilt device-resident input (gck_load_csr with GCK_MEM_DEVICE)
  const uint32_t* dev_off = nullptr;
  const uint32_t* dev_nbr = nullptr;
  uint64_t n_edges = 0;
  // delta re-link (delta.inc): the snapshot takes these device arrays over without a copy
  bool adopt = false;
  const uint32_t* dev_cav = nullptr;
  const int64_t* dev_exp = nullptr;
  const unsigned long long* dev_mhash = nullptr;  // nullptr: build the index if the kind has one
  unsigned long long mmask = 0;
  uint8_t has_wild = 0;
  uint8_t wild_known = 0;  // has_wild holds without dev_mhash (engine.hip scan_wild's result, carried over)
  uint64_t mh_keys = 0;  // keys + tombstones in dev_mhash
};

// The updates of one (relation, subject type, subject relation), last write per key
// (snapshot.cpp group_updates).
struct UpdateGroup {
  uint16_t rel, stype, srel;
  std::vector<unsigned long long> keys;  // (object << 32) | subject, ascending, unique
  std::vector<uint8_t> upsert;           // 1 = CREATE / TOUCH, 0 = DELETE
  std::vector<uint8_t> is_ext;           // the upsert carries a caveat or an expiration
  std::vector<uint32_t> cav;             // caveat instance per key (0 = none)
  std::vector<int64_t> exp_us;           // expiration per key (0 = never)
  // the merge's upload image of the group, laid out by group_updates (on the staging thread for a
  // staged batch) in GroupBuffers::img: byte offsets of the keys, the insert flags of each class
  // (plain, caveated / expiring), the caveats and the expirations; and the classes' summaries
  const unsigned char* img = nullptr;
  size_t o_keys = 0, o_ins[2] = {0, 0}, o_cav = 0, o_exp = 0;
  uint32_t n_cand[2] = {0, 0}, max_row[2] = {0, 0};  // upserts into each class; 1 + their largest row
  uint8_t wild_ins[2] = {0, 0}, wild_any = 0;       // a wildcard upserted into each class; any wildcard key
};

// Pinned host memory for the Watch upload images (engine.hip; null on failure).
void* pinned_alloc(size_t bytes);
void pinned_free(void* p);

// snapshot.cpp group_updates' storage, reused batch after batch (a Watch batch holds it under the
// writer lock): per kind its records, the bucket pass's buffers, and the groups it returns.
struct GroupBuffers {
  std::vector<std::vector<uint64_t>> recs;
  std::vector<uint64_t> tmp, kinds;
  std::vector<uint32_t> cnt, bucket;
  std::vector<UpdateGroup> out;
  // the groups' upload image (pinned; the merge copies it to the device whole: delta.inc)
  unsigned char* img = nullptr;
  size_t img_cap = 0, img_bytes = 0;
  GroupBuffers() = default;
  GroupBuffers(const GroupBuffers&) = delete;
  GroupBuffers& operator=(const GroupBuffers&) = delete;
  ~GroupBuffers() {
    if (img) pinned_free(img);
  }
};

// The check-time caveat contexts of one call (CheckBulkPermissionsRequestItem.Context,
// client/client.go:257) and how their outcomes reach the device: a dense table of every partial
// caveat instance x context when that is small, otherwise lazily — the walk records the pairs it
// touches, the host parses and evaluates just those and the batch runs again (engine.hip
// caveat_passes).
struct CavCall {
  uint32_t n_ctx = 0;             // contexts of the call (0: none, or no partial instance)
  uint32_t n_given = 0;           // contexts the call gave (a host item's context_slot must not exceed it)
  // dense: rows x n_dist outcomes (0 false, 1 true, 2 partial, 3 error) over the distinct
  // context texts, and each slot's distinct text; empty with n_ctx > 0: lazy
  std::vector<uint8_t> dense;
  uint32_t n_dist = 0;
  std::vector<uint32_t> of_slot;
  // lazy: the contexts' JSON texts, concatenated (slot k + 1 = [off[k], off[k + 1]))
  std::shared_ptr<const std::string> text;
  std::shared_ptr<const std::vector<uint32_t>> off;
};

struct DeviceSnapshot;  // engine.hip
struct Workspace;       // engine.hip

struct Engine {
  gck_config cfg{};
  int device = 0;
  uint32_t part_rank = 0, part_world = 1;  // partitioned graph (gck_set_partition)
  bool part_set = false;                   // gck_set_partition was called (any world, one rank too)
  // the schema's hub nodes and the relations of their hierarchy (labels.inc partition_rules): what
  // a rank keeps beyond the rows it owns (part_keep)
  std::vector<char> part_hub_node, part_hub_rel;
  std::vector<uint8_t> part_sub_node;  // the hubs' nodes (partition.inc part_dest)
  bool device_ready = false;
  std::shared_mutex mu;  // shared: checks (and a Watch batch's build); exclusive: schema/snapshot
  std::mutex writer_mu;  // one writer at a time (gck_api.cpp WriterLock; a Watch batch holds it throughout)
  std::unique_ptr<Schema> schema;
  std::string schema_text;  // as loaded (the snapshot cache is keyed by it)
  std::vector<TypeInterner> interner;
  // caveat instances: a caveat name + stored context, deduplicated; [0] = none (gck_api.cpp)
  std::vector<std::pair<std::string, std::string>> caveat_instances;
  std::unordered_map<std::string, uint32_t> caveat_ids;       // name '\0' json -> instance
  std::vector<std::shared_ptr<const cel::Node>> caveat_expr;  // per instance (null for [0])
  std::vector<cel::Object> caveat_ctx;                        // per instance: stored context
  std::vector<uint8_t> caveat_static;   // per instance: cel::Outcome under the stored context alone
  std::vector<uint32_t> caveat_row;     // per instance: row of the per-call table (PARTIAL only)
  std::vector<uint32_t> caveat_partial; // row -> instance
  // staging
  bool staging = false;
  uint64_t staged_revision = 0;
  std::vector<StagedTuple> staged;
  std::vector<HostCSR> prebuilt;
  uint64_t seq = 0;
  // committed
  uint64_t revision = 0;
  uint64_t head_revision = 0;  // consistency.Full target (gck_set_head_revision; 0 = local head)
  uint64_t n_tuples = 0;
  bool committed = false;
  DeviceSnapshot* dev = nullptr;
  // check workspaces (engine.hip acquire_ws): one per batch in flight, at most
  // cfg.workspaces (0 = 4); ws_cv signals a released one
  std::mutex ws_mu;
  std::condition_variable ws_cv;
  std::vector<Workspace*> ws_pool;
  Workspace* part_ws = nullptr;   // the partitioned batch's own workspace (partition.inc)
  void* part_comm = nullptr;      // the RCCL communicator of gck_part_init (partition.inc RcclCtx)
  std::mutex stats_mu;            // stats are added by concurrent batches
  std::mutex host_mu;             // pinned host buffers handed out by gck_host_alloc (base -> bytes)
  std::map<uintptr_t, size_t> host_bufs;
  uint64_t generation = 0;        // bumped by every device snapshot (commit, Watch batch)
  void* delta_scratch = nullptr;  // device arena of Watch-batch application (delta.inc)
  void* free_stream = nullptr;    // hipStream_t: replaced snapshot arrays go back to the pool here
  void* delta_ev = nullptr;       // hipEvent_t: a Watch batch's merge totals are back (delta.inc)
  void* sync_ev = nullptr;        // hipEvent_t: the Watch path's polled waits (engine.hip spin_stream)
  void* patch_ev = nullptr;       // hipEvent_t: the last Watch publication's null-stream work, index patch included (make_ctx)
  void* build_ev = nullptr;       // hipEvent_t: the same publication's work before its index patch (the joins wait for it)
  uint64_t patch_seq = 0;         // publications recorded (0: none yet)
  struct ResState* res = nullptr;  // the resident closure join (resident.inc; GCK_FLAG_RESIDENT)
  bool res_tried = false;
  std::atomic<uint64_t> aql_patch_seen{0};  // the publication whose build the HSA-queue dispatches have waited for
  void* blob_host = nullptr;      // pinned: a Watch batch's program upload (device_build)
  size_t blob_host_cap = 0;
  size_t delta_scratch_cap = 0;
  void* delta_host = nullptr;     // pinned staging of the same (one upload, one small read back)
  size_t delta_host_cap = 0;
  void* delta_host_dev = nullptr; // (its device address: the prefix writes the batch's totals there)
  GroupBuffers group_buf;  // group_updates' records and groups, kept across Watch batches
  // bumped by every write that can invalidate a batch validated earlier (a schema, a snapshot file,
  // an interner rollback, a partition): a staged Watch batch (gck_watch_stage) is regrouped at
  // apply time when it moved
  uint64_t shape_gen = 0;
  // merged-CSR arrays of retired snapshots kept for the next Watch batch's merge (engine.hip
  // ralloc / retire_array): bytes -> array, and every array ralloc handed out -> its bytes
  std::multimap<size_t, void*> recycle;
  std::unordered_map<void*, size_t> recyclable;
  size_t recycle_bytes = 0;
  gck_stats stats{};
  // batches to come that chain the wave bundles behind the join in stage A (engine.hip
  // bundles_launch): reset to 16 by a batch whose join left kChainLeftovers or more, counted down by
  // one that left fewer
  std::atomic<int> defer_recent{0};
  // direct AQL dispatch of the join kernels (engine.hip aql.inc): the engine's HSA queue and the
  // kernels of libgck_kernels.co, set up at the first snapshot (null: launches go through HIP)
  struct AqlState* aql = nullptr;
  struct DeltaHint* delta_hint = nullptr;  // set while a Watch batch builds its snapshot (delta.inc)
  bool aql_tried = false;
  ~Engine();
};

// GCK_DEBUG_PHASES=1: wall time of the snapshot / Watch phases on stderr (engine.hip PhaseClock)
struct PhaseClock {
  const char* what;
  bool on;
  double t0, last;
  std::string line;
  explicit PhaseClock(const char* w);
  void mark(const char* phase);
  ~PhaseClock();
};

// Partitioned graphs: does rank e.part_rank keep the tuple rel(obj) <- (sid, srel)?
// Its own rows (part_owner(obj)); of a hub relation (partition_rules) instead every userset and
// wildcard tuple — the replicated hierarchy — and the direct tuples of the subjects it owns (their
// user slots, and what the level loop reads at a hub node, partition.inc part_dest). Every ingest path applies it (staging, gck_load_csr, Watch batches) after interning, so
// that ids and caveat instances stay the same on every rank.
inline bool part_keep(const Engine& e, uint16_t rel, uint32_t obj, uint32_t sid, uint16_t srel) {
  if (e.part_world <= 1) return true;
  if (rel >= e.part_hub_rel.size() || !e.part_hub_rel[rel]) return part_owner(obj, e.part_world) == e.part_rank;
  // a hub relation: the hierarchy everywhere, a direct tuple with its subject's owner only (the
  // level loop expands hub nodes there: partition.inc part_dest)
  return srel != kEllipsis || sid == kWildcard || part_owner(sid, e.part_world) == e.part_rank;
}
void partition_rules(Engine& e);  // labels.inc: e.part_hub_node / part_hub_rel from the schema

// snapshot.cpp
void add_tuples_text(Engine& e, const char* text, size_t len);
struct TupleNames {  // a relationship line with its object ids still names (parse_tuple_names)
  uint16_t rt = 0, rel = 0, st = 0, srel = kEllipsis;
  std::string rid, sid;
  uint32_t cav = 0;
  int64_t exp = 0;
};
TupleNames parse_tuple_names(Engine& e, const std::string& line);
std::vector<TupleNames> parse_tuples_text(Engine& e, const char* text, size_t len);
void stage_tuple(Engine& e, const gck_tuple& t);
// gck_api.cpp: caveat instances (a caveat name + stored context)
void reset_caveats(Engine& e);
uint32_t add_caveat_instance(Engine& e, const std::string& name, const std::string& json);
// snapfile.cpp: the on-disk snapshot cache
void save_snapshot_file(Engine& e, const std::string& path);
void load_snapshot_file(Engine& e, const std::string& path);
std::vector<HostCSR> build_csrs(Engine& e);
// Watch updates (rel.Update, rel/relationship.go:267-301): text lines "<OP> <relationship>"
void parse_updates_text(Engine& e, const char* text, size_t len, std::vector<gck_update>& out);
// `schema_mu`: held shared around each read of the schema and the interner (a batch staged on
// another thread, gck_watch_stage); null when the caller holds the engine lock
const std::vector<UpdateGroup>& group_updates(const Engine& e, GroupBuffers& B, const gck_update* ups, size_t n,
                                              std::shared_mutex* schema_mu = nullptr);
inline const std::vector<UpdateGroup>& group_updates(Engine& e, const gck_update* ups, size_t n) {
  return group_updates(e, e.group_buf, ups, n);
}
void validate_updates(const Engine& e, const gck_update* ups, size_t n);

// engine.hip
int device_init(Engine& e);
// delta: a Watch-batch re-link (delta.inc): derived structures of unchanged CSRs and the
// previous heights are taken over
void device_upload(Engine& e, std::vector<HostCSR>& csrs, bool delta = false);
// A Watch batch (delta.inc) in three steps: build the next snapshot beside the current one's
// checks (engine lock shared: the current snapshot is only read), then publish it (exclusive:
// batches in flight finished, membership indexes patched, snapshot swapped), or abort.
struct WatchBuild {
  DeviceSnapshot* ds = nullptr;
  std::vector<void*> adopted, fresh;
  int64_t tuple_delta = 0;
  const void* patch_jobs = nullptr;  // the deferred membership-index patch: its job table (device)
  int n_patch_jobs = 0;
  uint32_t patch_blocks = 0;
};
void device_apply_build(Engine& e, const std::vector<UpdateGroup>& groups, WatchBuild& wb);
void device_apply_publish(Engine& e, WatchBuild& wb);
void device_apply_abort(Engine& e, WatchBuild& wb);
// cav: the call's check-time caveat contexts (CavCall above)
// Pooled check workspaces (one per batch in flight, at most cfg.workspaces): acquire waits for
// a free one. Callers take their workspaces BEFORE the engine lock (the holders of busy ones
// may need the lock to finish their batches).
Workspace* acquire_ws(Engine& e);
void acquire_ws_n(Engine& e, int want, Workspace** out);  // 1 or 2 together (no hold-and-wait)
void release_ws(Engine& e, Workspace* w);
void ensure_pool(Engine& e);  // every workspace of the pool, created after a snapshot commit
struct WsLease {
  Engine& e;
  Workspace* w;
  explicit WsLease(Engine& en) : e(en), w(acquire_ws(en)) {}
  ~WsLease() { release_ws(e, w); }
  WsLease(const WsLease&) = delete;
  WsLease& operator=(const WsLease&) = delete;
};
void device_check(Engine& e, Workspace& w, const gck_item* d_items, size_t n, int64_t now_us,
                  uint8_t* d_perm, int32_t* d_err, void* stream, CavCall cav);
// Host buffers, chunks of max_batch alternating over w0 and w1 (w1 may be null or w0).
void device_check_host(Engine& e, Workspace* w0, Workspace* w1, const gck_item* items, size_t n, int64_t now_us,
                       uint8_t* perm, int32_t* err, const CavCall& cav);
// Asynchronous batches (gck_check_submit / gck_check_wait): submit starts one batch (n <=
// max_batch) on an acquired workspace; wait finishes it (later stages, results copied out) —
// the caller then releases the workspace. `items` etc. are device pointers on `stream`
// (host == false) or host buffers (host == true: the workspace's own stream).
void device_submit(Engine& e, Workspace* w, const gck_item* items, size_t n, int64_t now_us, uint8_t* perm,
                   int32_t* err, void* stream, bool host, bool engine_stream, CavCall cav);
void device_wait(Engine& e, Workspace* w);
// Uniform requests (gck_check_bulk_uniform / gck_check_submit_uniform): one header, id pairs, packed
// 2-bit results and the errored checks' (index, code) records in ascending order (the first `cap`
// written, their number in *n_errs). The submitted form's outputs are written by device_wait.
void device_check_uniform(Engine& e, Workspace* w0, Workspace* w1, const gck_uniform& h, const uint32_t* pairs,
                          size_t n, int64_t now_us, uint64_t* packed, gck_item_error* errs, size_t cap,
                          size_t* n_errs, const CavCall& cav);
void device_submit_uniform(Engine& e, Workspace* w, const gck_uniform& h, const uint32_t* pairs, size_t n,
                           int64_t now_us, uint64_t* packed, gck_item_error* errs, size_t cap, size_t* n_errs,
                           CavCall cav);
// Pinned host buffers (gck_host_alloc): a host batch whose items / results live in one is
// copied by DMA directly, without the workspace's staging copy.
void* host_alloc(Engine& e, size_t bytes);
void host_free(Engine& e, void* p);
void host_free_all(Engine& e);
// Finishes every batch in flight (a writer holding the engine exclusively calls this before
// it replaces the snapshot: the batches keep the results of the snapshot they started on).
void drain_batches(Engine& e);
uint64_t device_bytes(Engine& e);
void device_export(Engine& e, std::vector<HostCSR>& out);
// lookups (lookup.inc): candidates [0, n) of the varying id of `proto` (resource id when
// vary_res, else subject id); matching ids ascending with their permissionship
void device_lookup(Engine& e, Workspace& w, const gck_item& proto, bool vary_res, uint32_t n_candidates,
                   int64_t now_us, std::vector<uint32_t>& ids, std::vector<uint8_t>& perms);
void device_lookup_subjects(Engine& e, Workspace& w, const gck_item& proto, int64_t now_us, std::vector<uint32_t>& ids,
                            std::vector<uint8_t>& perms);
// partitioned checks (partition.inc): one batch over every rank, the exchange over RCCL inside
// libgck (part_check, after part_init) or the caller's transport (part_check_with)
void part_unique_id(uint8_t* out);
void part_init(Engine& e, const uint8_t* id);
void part_check(Engine& e, const gck_item* d_items, size_t n, int64_t now_us, uint8_t* d_perm, int32_t* d_err,
                void* stream);
void part_check_with(Engine& e, const gck_transport& t, const gck_item* d_items, size_t n, int64_t now_us,
                     uint8_t* d_perm, int32_t* d_err, void* stream);
uint32_t part_owner_name(uint16_t type, const char* s, size_t len, uint32_t world);
void part_intern(Engine& e, const gck_transport& t, const uint16_t* types, const char* const* names,
                 const uint32_t* lens, size_t n, bool create, uint32_t* out);
void part_add_tuples_text(Engine& e, const gck_transport& t, const char* text, size_t len);
void part_comm_free(Engine& e);
void device_free(Engine& e);

}  // namespace gck

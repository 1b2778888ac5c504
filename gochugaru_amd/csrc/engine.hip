// engine.hip — MI355X (gfx950) batched permission-check kernels and batch driver.
//
// Replaces SpiceDB's CheckBulkPermissions dispatch (the computation behind
// client/client.go:261-266; semantics SURVEY.md §5.1) with a level-synchronous, multi-query
// frontier expansion over HBM-resident CSR tuple tables:
//
//   level L frontier: Entry{query, object, node, depth, cond}
//     k_expand  : one lane per entry — identity filter, depth budget, direct-subject
//                 membership (binary search over the sorted CSR row, wildcard = last id),
//                 computed usersets pushed directly, userset/arrow rows emitted as segments,
//                 intersection/exclusion/all() nodes spawn a join of sub-queries
//     k_edges   : one lane per enumerated edge (load-balanced over the segments) — pushes
//                 the neighbour's (query, object, node) into the next frontier after a
//                 visited-hash dedupe (memoised per query, SURVEY §8d counting rule)
//     k_resolve : one lane per query — a query with a Y is decided; a query with no live
//                 entries and no pending joins is decided N/C/ERR; decisions cascade into
//                 joins (tri-state algebra) and up to the parent query
//   level L+1 ...
//
// Every frontier level is one dispatch wave of SpiceDB's recursion, so the depth budget
// (max_depth, default 50) is enforced per entry exactly as dispatch.CheckDepth does.
#include <cxxabi.h>
#include <dlfcn.h>
#include <hip/hip_ext.h>
#include <hipcub/hipcub.hpp>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <fstream>
#include <functional>
#include <sstream>
#include <string>
#include <thread>
#include <type_traits>

#include "engine.hpp"

namespace gck {

#define HIP_OK(x)                                                                         \
  do {                                                                                    \
    hipError_t err_ = (x);                                                                \
    if (err_ != hipSuccess)                                                               \
      throw Error(GCK_E_DEVICE, std::string(#x " failed: ") + hipGetErrorString(err_));   \
  } while (0)

constexpr int kBlock = 256;
constexpr unsigned long long kEmptyKey = ~0ull;
constexpr uint32_t kResErr = 0xF;

struct BaseCsr {  // a CSR of the snapshot itself: table[k] for k < base.size()
  uint16_t rel, stype, srel;
  bool ext;
  uint64_t n_edges;
  uint64_t mh_keys;  // keys + tombstones in its membership index (delta.inc)
};

struct Derived {  // a bidirectional structure and the base CSR it was built from (bidir.inc)
  uint8_t kind;   // 0 = transposed CSR, 1 = ancestor closure
  const uint32_t* src;
  uint64_t src_edges;
  DevCSR d;
  uint32_t* sig = nullptr;  // ancestor closure: 256-bit signature per row (closure.inc)
  uint32_t* lab = nullptr;      // ... tree labels per row: {pre | cover overflow << 31, end} (closure.inc)
  uint32_t* cov_off = nullptr;  // ... tree cover per row (preorder numbers), CSR
  uint32_t* cov_pre = nullptr;
};

// User slots of the snapshot (bidir.inc slots_for), found again by the next Watch batch, which
// recomputes only the slots of the users it touched when the hierarchy labels are unchanged.
struct SlotRec {
  const uint32_t* src_off;  // the transposed CSR the slots were built over
  const uint32_t* lab;      // the closure's labels and covers they were built from
  const uint32_t* cov_pre;
  uint32_t* slots;
  uint32_t* list;           // cover lists (null: none)
  uint64_t list_total;      // entries in `list`
  uint32_t n_rows;
  uint8_t kind;             // bidir.inc SlotKind (user / resource slots)
};

// Slots of some users, written into a slot array the snapshot shares with the current one when it
// is published (device_publish, after the batches in flight on the current one have finished).
struct SlotPatch {
  uint32_t* slots;
  const uint32_t* staged;  // kUSlotWords per user, in `ids` order
  const uint32_t* ids;
  uint32_t n;
};

struct DeviceSnapshot {
  std::vector<void*> allocs;
  std::vector<void*> hallocs;  // hipExtMallocWithFlags (physically contiguous) arrays: hipFree
  uint32_t slot_bits = 32;     // user-slot entry width (closure.inc): 24 when every hierarchy has <= 2^24 groups
  std::vector<BaseCsr> base;
  std::vector<DevCSR> table;     // host copy of the device CSR table (base, then derived)
  std::vector<Derived> derived;  // reused by the next snapshot when the source is unchanged
  // dispatch-graph heights per (forward node, object) (build_heights): hgt[n] = nullptr for a
  // node without successors (height 0); hmax[n] = their maximum; h_src = the row-edge CSRs
  // they were relaxed over (a Watch batch that changes none of them keeps them as they are)
  std::vector<uint32_t*> hgt;
  std::vector<uint32_t> hmax;
  std::vector<uint32_t> hcount;  // objects per hgt[n]
  std::vector<const uint32_t*> h_src;
  bool any_deep = false;         // some node is NF_DEEP: the grid-wide path keys entries by depth
  const unsigned long long* d_hgt = nullptr;  // device table of hgt[n] (in the program block)
  DevNode* nodes = nullptr;
  DevItem* items = nullptr;
  DevCSR* csrs = nullptr;
  uint32_t* type_counts = nullptr;
  uint32_t n_nodes = 0, n_items = 0, n_csrs = 0, n_types = 0, n_rels = 0;
  uint32_t n_fwd = 0;      // forward nodes; [n_fwd, n_nodes) is the reverse program (bidir.inc)
  bool has_bidir = false;  // some forward node is NF_BIDIR
  // closure-join stage (closure.inc): the flat table of eligible roots (in the program block)
  std::vector<unsigned char> cj_host;
  uint32_t cj_n_desc = 0, cj_o_meta = 0, cj_o_entries = 0;
  const unsigned char* d_cj = nullptr;
  // label-join stage (labels.inc): root table + LjMeta[] (in the program block), slot words
  std::vector<unsigned char> lj_host;
  uint32_t lj_o_meta = 0, lj_sw = 0, lj_bits = 24;
  bool lj_preferred = false;  // the labels cover every closure-join root and more: they take stage A
  bool lj_cav = false;        // some label root holds caveated pairs (labels.inc kLjCav)
  uint32_t n_cav = 0;         // caveat instances in cav_static / cav_row
  std::vector<uint64_t> lj_key;  // what the label tables were built from (labels.inc: reused while unchanged)
  std::vector<uint64_t> lj_dkey; // ... of it, the CSRs that feed only the resource slots' user lists
  std::vector<const uint32_t*> lj_hgt;  // the roots' heights arrays the tables were built against
  std::vector<void*> lj_ptrs;    // their arrays (in allocs or hallocs)
  // subjects a Watch batch changed a direct grant of since the tables were built (bit per subject;
  // null: none): their checks go to the wave bundles (labels.inc, lj_dirty_path)
  uint32_t* lj_dirty = nullptr;
  uint64_t lj_dirty_n = 0;       // changed grants marked (an upper bound of the dirty subjects)
  uint32_t lj_users = 0;
  // the arrow forest of the label roots' resources (labels.inc lj_forest: every object the
  // flattening of a resource visits is an ancestor of it): per vertex (pre, end), per type its
  // first vertex (kNone: not in the forest); null: no forest, a dirty subject's checks all defer
  uint32_t* lj_af = nullptr;
  // the forest's parent edges (labels.inc lj_chain_walk): tupleset CSR << 32 | the parent's forest
  // index (kNone: a root), per forest vertex; null: no chain programs
  unsigned long long* lj_afp = nullptr;
  uint32_t lj_afp_n = 0;
  uint32_t* lj_anc = nullptr;  // per forest vertex its ancestors, kAncWords each (labels.inc lj_chain_wave)
  std::vector<uint32_t> lj_af_base, lj_af_rows;
  std::vector<std::pair<uint32_t, uint16_t>> lj_dtype;  // direct-grant CSR -> the type of its rows
  // per dirty subject the forest intervals of the objects whose grants of it changed (kDovWords
  // each, labels.inc): its checks defer only when one holds the resource (shared like lj_dirty)
  uint32_t* lj_dov = nullptr;
  std::vector<void*> adopt_h;    // arrays of the current snapshot this one takes over at publish
                                 // (device_publish: contiguous ones move to hallocs, others to allocs)
  std::vector<SlotRec> slot_recs;
  std::vector<SlotPatch> slot_patches;  // applied by device_publish
  uint64_t lj_bytes = 0;
  const unsigned char* d_lj = nullptr;
  uint32_t node_bits = 1, q_bits = 1, q_bits_deep = 1;  // query-id bits of the visited keys (make_key)
  uint64_t bytes = 0;
  uint8_t* cav_static = nullptr;  // per caveat instance (Engine::caveat_static)
  uint32_t* cav_row = nullptr;    // per caveat instance (Engine::caveat_row)
};

struct PartState;  // partition.inc

// What a Watch batch being built (delta.inc device_apply_build) tells the snapshot build: the
// transposed CSRs it merged (taken over by build_bidir instead of transposing again), and per
// merged transpose the users whose memberships changed (slots_for recomputes only theirs).
struct DeltaHint {
  std::vector<Derived> derived;
  struct Fwd {  // a merged forward CSR class: its new neighbours and the batch's keys into it
    const uint32_t* nbr;
    const unsigned long long* keys;  // (object << 32 | subject), D of them
    const uint8_t* ins;              // after k_dj_prefix: inserted / removed (0 0: unchanged)
    const uint8_t* found;
    uint32_t D;
    bool wild;  // a wildcard subject among the keys
  };
  std::vector<Fwd> fwd;
  struct Users {
    const uint32_t* t_off;      // the merged transposed CSR
    const uint32_t* old_t_off;  // the current snapshot's, which it replaces
    const uint32_t* ids;        // users with a changed membership (device, ascending)
    uint32_t n;
  };
  std::vector<Users> users;
};

// One check workspace: the scratch of one batch in flight, on its own HIP stream. An engine
// keeps a pool of them (acquire_ws / release_ws), so concurrent callers — and the batches a
// caller submits without waiting (gck_check_submit) — run side by side on the device: the
// persistent bundle kernels of the next batch fill the tail of the previous one.
struct Workspace {
  PartState* part = nullptr;  // partitioned batch in progress (partition.inc; Engine::part_ws only)
  bool busy = false;          // taken from the pool (Engine::ws_mu)
  uint64_t bytes = 0;         // device scratch allocated for it (gck_device_bytes)
  size_t max_batch = 0, frontier_cap = 0, seg_cap = 0, query_cap = 0, join_cap = 0;
  uint64_t visited_cap = 0;
  // ---- the batch in flight (submit_batch .. finish_batch); guarded by `m` -----------------
  std::mutex m;
  int state = 0;              // 0 idle, 1 stage A submitted, 2 finished (results written)
  int fail_code = 0;          // a failure while a writer drained the batch (drain_batches)
  std::string fail_msg;
  hipStream_t b_st = nullptr; // the stream the batch runs on
  const gck_item* b_items = nullptr;
  uint32_t b_n = 0;
  int64_t b_now = 0;
  uint8_t* b_dperm = nullptr; // device results
  int32_t* b_derr = nullptr;
  uint8_t* b_hperm = nullptr; // host batch: the caller's result buffers (copied out by the wait)
  int32_t* b_herr = nullptr;
  uint8_t* b_copy_perm = nullptr;  // zero-copy batch over the pinned staging: the caller's result
  int32_t* b_copy_err = nullptr;   // buffers the wait copies the staging into
  uint8_t* b_xperm = nullptr; // host batch: where the results' D2H lands — the pinned staging, or
  int32_t* b_xerr = nullptr;  // the caller's buffers themselves when they are gck_host_alloc memory
  bool b_bundles = false;     // stage A is the bundle kernel (else the grid-wide path ran it all)
  bool b_label = false;       // ... and it was the label join
  bool b_closure = false;     // stage A began with the closure join: its leftovers are bundled in finish
  bool b_chained = false;     // ... or already in stage A, by bundles chained on the device
  bool b_timed = false;       // this batch's stage A is bracketed by ev0 / ev1 (GCK_FLAG_PROFILE, sampled)
  bool b_own_stream = false;  // a device batch on the workspace's stream (GCK_SUBMIT_ENGINE_STREAM)
  bool b_aql = false;         // ... whose join was dispatched into the engine's HSA queue (aql.inc)
  uint32_t b_sum_blocks = 0;  // ... in that many blocks, each with a summary slot (closure.inc block_summary)
  bool b_validate = false;    // host items read in place: the join checks their context slots
  bool b_res = false;         // ... posted to the resident join (resident.inc) instead
  uint32_t ws_index = 0;      // the workspace's place in the pool (its resident-join slot)
  uint32_t res_seq = 0;       // resident-join requests posted from it
  // ---- a uniform batch (gck_check_bulk_uniform / gck_check_submit_uniform) -----------------
  bool u_on = false;          // this batch is uniform: its wait packs the results (uniform_collect)
  bool u_join = false;        // ... and its join reads the pairs and writes the packed words in place
  uint32_t u_rp = 0, u_ss = 0, u_ctx = 0;       // the header (closure.inc CjArgs::u_rp ...)
  const uint32_t* u_pairs = nullptr;            // the pairs the join reads (caller's pinned buffer or staging)
  unsigned long long* u_packed = nullptr;       // the words the join writes (caller's pinned buffer or staging)
  unsigned long long* u_out = nullptr;          // the caller's words
  uint32_t u_ncj = 0;                           // checks the join left (answered into d_perm / d_err)
  std::vector<gck_item> u_items;                // otherwise: the request expanded to items ...
  std::vector<uint8_t> u_perm;                  // ... and its results
  std::vector<int32_t> u_err;
  gck_item_error* u_errs = nullptr;             // submit_uniform: the caller's error list
  size_t u_err_cap = 0;
  size_t* u_n_errs = nullptr;
  void* aql_kernarg = nullptr;  // aql.inc: kernarg block of the dispatched join (pinned host memory, or VRAM)
  bool aql_devargs = false;     // ... in VRAM (aql.inc AqlState::devargs)
  uint64_t aql_signal = 0;      // aql.inc: its completion signal (hsa_signal_t handle)
  void* aql_queue = nullptr;    // aql.inc: the engine queue this workspace dispatches into
  alignas(16) unsigned char aql_shadow[1024] = {};  // aql.inc: what the kernarg block holds now
  uint64_t n_batches = 0;     // batches run on this workspace (event sampling)
  unsigned b_seq = 0;         // publish sequence of stage A
  float b_ms = 0.f;
  // ---- grid-wide path (allocated on first use: ensure_wide) --------------------------------
  bool wide_ready = false;
  DevCheck* checks = nullptr;
  int32_t* item_err = nullptr;
  DevQuery* queries = nullptr;
  DevJoin* joins = nullptr;
  Entry* fr[2] = {nullptr, nullptr};
  Segment* segs = nullptr;
  unsigned long long* visited = nullptr;
  // ---- counters, publication, staging ------------------------------------------------------
  DevCounters* ctr = nullptr;
  DevCounters* h_ctr = nullptr;  // pinned, coherent (k_publish writes it)
  unsigned* h_seq = nullptr;     // after h_ctr + bundle counters: the last published batch
  unsigned pub_seq = 0;
  uint64_t patch_seen = 0;       // the engine's publication whose patch event this workspace's stream waited for
  void* patch_stream = nullptr;  // ... on this stream (make_ctx)
  uint64_t build_seen = 0;       // ... whose build event (the joins' wait)
  void* build_stream = nullptr;
  unsigned* d_hpub = nullptr;    // device address of h_ctr
  unsigned* h_slots = nullptr;   // pinned: {deferred, counters touched} per block of an AQL-dispatched join
  unsigned* d_slots = nullptr;   // (device address)
  uint32_t n_slots = 0;
  bool ctr_clean = false;        // ctr + b_ctrs are zero (k_publish left them so)
  gck_item* d_items = nullptr;   // staging for the host-buffer API
  uint8_t* d_perm = nullptr;
  int32_t* d_err = nullptr;
  gck_item* h_items = nullptr;   // pinned staging of a host batch: items in, results out
  uint8_t* h_perm = nullptr;
  int32_t* h_err = nullptr;
  hipStream_t stream = nullptr;  // the workspace's own stream (host batches, lookups)
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
  hipEvent_t pev[4] = {nullptr, nullptr, nullptr, nullptr};  // GCK_FLAG_PROFILE
  // ---- bundle path -------------------------------------------------------------------------
  uint32_t b_checks = 16, b_fc = 4096, b_vslots = 16384, b_blocks = 0;
  unsigned long long* b_fr = nullptr;  // packed frontier entries beyond the LDS part
  unsigned long long* b_vis = nullptr;
  uint32_t* b_vlog = nullptr;  // per slot: claimed visited slots (cleared by the bundle)
  uint32_t* b_deferred = nullptr;
  uint32_t* c_deferred = nullptr;  // checks the closure-join stage left to the bundles
  unsigned* b_ctrs = nullptr;      // kBCtrs words: [0] bundle ctr, [1] deferred, [2] giant bundle ctr,
                                   // [3] deferred2, [4] closure-join deferred (closure.inc)
  unsigned* h_bctrs = nullptr;     // pinned
  uint32_t b_budget = 1024;
  // giant-check stage: one 16-wave workgroup per bundle (allocated on first use: ensure_giant)
  bool giant_ready = false;
  uint32_t g_fc = 65536, g_vslots = 262144, g_slots = 0;
  unsigned long long* g_fr = nullptr;
  unsigned long long* g_vis = nullptr;
  uint32_t* g_vlog = nullptr;
  uint32_t* g_deferred = nullptr;
  gck_item* def_items = nullptr;
  uint8_t* def_perm = nullptr;
  int32_t* def_err = nullptr;
  // the current call's check-time caveat contexts (engine.hpp CavCall): its dense outcome table,
  // or the lazy evaluation's device map of the pairs evaluated so far (cav_keys / cav_vals, open
  // addressing, host-built) and the set / list of the unevaluated pairs a pass touched
  CavCall cav;
  bool cav_on = false;          // the call has contexts and the snapshot partial instances
  bool cav_lazy = false;
  uint8_t* cav_dyn = nullptr;
  size_t cav_dyn_cap = 0;
  uint32_t* cav_slot = nullptr;  // dense: each slot's distinct context (CavCall::of_slot)
  size_t cav_slot_cap = 0;
  std::vector<uint8_t> cav_dyn_up;    // what cav_dyn / cav_slot hold (a call with the same table
  std::vector<uint32_t> cav_slot_up;  // as the workspace's previous one uploads nothing)
  unsigned long long* cav_keys = nullptr;
  uint8_t* cav_vals = nullptr;
  size_t cav_map_cap = 0;       // slots of the device map (a power of two)
  size_t cav_map_alloc = 0;
  std::unordered_map<unsigned long long, uint8_t> cav_eval;  // host: the pairs evaluated for the call
  std::unordered_map<uint32_t, cel::Object> cav_parsed;       // host: the call's contexts parsed so far
  unsigned long long* req_set = nullptr;  // kReqSet slots
  unsigned long long* req_list = nullptr; // kReqCap pairs
  unsigned* req_cnt = nullptr;
  uint8_t* cav_flag = nullptr;  // per check of the batch: its walk touched a pair whose evaluation failed
  struct Ctx* d_ctx = nullptr;  // the batch's Ctx for the label join's caveated pairs (LjArgs::cx)
  struct Ctx* h_ctx = nullptr;  // (pinned: its upload is ordered on the batch's stream)
  uint32_t b_cav_req = 0, b_cav_err = 0;  // the published cav_requests / cav_errors of the batch's pass
  // lookups (lookup.inc): matching ids / permissionships of one candidate chunk, their count
  uint32_t* lk_ids = nullptr;
  uint8_t* lk_perm = nullptr;
  unsigned* lk_cnt = nullptr;
  // GCK_DEBUG_BUNDLE / GCK_DEBUG_TIMING buffers (per workspace: engines on several devices in
  // one process, and concurrent batches, never share one)
  uint32_t* dbg = nullptr;
  unsigned long long* timing = nullptr;
  size_t timing_cap = 0;
  std::vector<void*> allocs;
};

// ---- device helpers --------------------------------------------------------------------------

struct Ctx {
  const DevNode* nodes;
  const DevItem* items;
  const DevCSR* csrs;
  const uint32_t* type_counts;
  uint32_t n_types, n_rels;
  uint32_t n_nodes, n_items, n_csrs;
  uint32_t n_fwd;  // forward nodes (reverse-program nodes follow)
  DevCheck* checks;
  DevQuery* queries;
  DevJoin* joins;
  Entry* next;
  Segment* segs;
  unsigned long long* visited;
  uint64_t vmask;
  DevCounters* ctr;
  uint32_t frontier_cap, seg_cap, query_cap, join_cap;
  // visited key = q << q_shift | node << node_shift | (depth & depth_mask) << depth_shift |
  // tag << 32 | obj; the depth field exists only when the snapshot has deep roots (exact-depth
  // checks key their entries by depth), otherwise depth_mask = 0 and the tag is the cond bit
  uint32_t node_shift, q_shift, depth_shift, depth_mask;
  uint32_t level, max_depth;
  const unsigned long long* hgt;  // per forward node: its heights array (u32 per object) or 0
  int64_t now_us;
  // caveats (cel.hpp; gck_api.cpp caveat_call): per instance its outcome under the stored
  // context alone (0 false, 1 true, 2 partial) and, for partial ones, a row of the per-batch
  // table of outcomes under each check context (column slot - 1)
  const uint8_t* cav_static;
  const uint32_t* cav_row;
  const uint8_t* cav_dyn;
  const uint32_t* cav_slot;
  const gck_item* ck_items;  // the launch's items: check k's context slot
  uint32_t n_ctx, n_dist;
  // lazy evaluation (cav_keys non-null): the evaluated pairs, and where a pass records the rest
  const unsigned long long* cav_keys;
  const uint8_t* cav_vals;
  uint64_t cav_kmask;
  unsigned long long* req_set;
  unsigned long long* req_list;
  unsigned* req_cnt;
  // check k of the launch is check ck_map[k] (or ck_off + k) of the batch: its cav_flag byte
  uint8_t* cav_flag;
  const uint32_t* ck_map;
  uint32_t ck_off;
  // partitioned graphs (partition.inc): entries for objects another rank owns go to its outbox
  // region [d * out_cap, (d + 1) * out_cap) instead of the next frontier
  uint32_t rank, world;
  Entry* outbox;
  unsigned* out_cnt;
  uint32_t out_cap;
  // query / join ids this launch may allocate below (spawn_join): query_cap / join_cap, or on a
  // partitioned graph the end of this rank's own id range (partition.inc part_loop)
  uint32_t q_hi, j_hi;
  uint32_t force_exact;  // every root runs exact-depth (partitioned graphs: no global heights)
  // partitioned graphs: per node 1 for the nodes of a hub (group#member and the relations it
  // unions): their entries go to the owner of the check's subject, which holds the subject's
  // direct memberships and the replicated hierarchy (partition.inc part_dest); null: by object
  const uint8_t* part_sub;
};

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// ---- exact depth semantics -----------------------------------------------
// SpiceDB's dispatch(v, d) depends on the remaining depth d only through the depth error, and
// monotonically: once it is not ERR at some d it keeps that value for every larger d. A check
// whose every walk from its root stays below the budget (the root's dispatch-graph height,
// build_heights, is < max_depth) therefore has a depth-independent answer, which the memoised
// search (each (query, node, object) expanded once, at its minimal depth) computes. A check
// rooted higher runs in exact-depth mode instead: its entries are keyed by depth too, so every
// (vertex, depth) it can reach is expanded (at most max_depth + 1 per vertex, also on cyclic
// data), and each edge whose caveat is unresolved or false starts a single-operand and-query
// whose result goes through the oracle's and3 (a caveat-false edge still passes a depth error
// up; a HAS below an unresolved caveat no longer masks a sibling's error).
constexpr uint32_t kCondBit = 1u;   // Entry/Segment cond: reached through an unresolved caveat
constexpr uint32_t kExactBit = 2u;  // ... the check runs in exact-depth mode
constexpr uint32_t kTagNone = 0u, kTagCond = 1u, kTagFalse = 2u;  // DevQuery::operand >> 24

__device__ __forceinline__ uint32_t and_tag(uint32_t tag, uint32_t res) {
  if (tag == kTagNone || res == kResErr) return res;  // and3(_, ERR) = ERR
  if (tag == kTagFalse || res == GCK_PERM_NO) return GCK_PERM_NO;
  return GCK_PERM_CONDITIONAL;
}

__device__ __forceinline__ unsigned long long make_key(const Ctx& c, uint32_t q, uint32_t node, uint32_t tag,
                                                       uint32_t depth, uint32_t obj) {
  return ((unsigned long long)q << c.q_shift) | ((unsigned long long)node << c.node_shift) |
         ((unsigned long long)(depth & c.depth_mask) << c.depth_shift) | ((unsigned long long)(tag & 3u) << 32) |
         obj;
}

__device__ __forceinline__ bool vlookup(const Ctx& c, unsigned long long key) {
  uint64_t h = mix64(key) & c.vmask;
  for (int p = 0; p < 64; ++p) {
    unsigned long long v = __hip_atomic_load(&c.visited[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v == key) return true;
    if (v == kEmptyKey) return false;
    h = (h + 1) & c.vmask;
  }
  return false;
}

// 1 = inserted, 0 = already present, -1 = table overflow
__device__ __forceinline__ int vinsert(const Ctx& c, unsigned long long key) {
  uint64_t h = mix64(key) & c.vmask;
  for (int p = 0; p < 128; ++p) {
    unsigned long long v = __hip_atomic_load(&c.visited[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v == key) return 0;
    if (v == kEmptyKey) {
      unsigned long long prev = atomicCAS(&c.visited[h], kEmptyKey, key);
      if (prev == kEmptyKey) return 1;
      if (prev == key) return 0;
    }
    h = (h + 1) & c.vmask;
  }
  atomicOr(&c.ctr->overflow, 1u);
  return -1;
}

__device__ __forceinline__ uint32_t qflags(const DevQuery* q) {
  return __hip_atomic_load(&q->flags, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}
// A query's flags read only to skip work for a decided query (a stale value costs an expansion
// that the next level drops): no acquire, so no L1 invalidation (buffer_inv) per call.
__device__ __forceinline__ uint32_t qflags_hint(const DevQuery* q) {
  return __hip_atomic_load(&q->flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void set_found(const Ctx& c, uint32_t q, uint32_t cond) {
  atomicOr(&c.queries[q].flags, (cond & kCondBit) ? (uint32_t)QF_FOUND_C : (uint32_t)QF_FOUND_Y);
}

// The rank that expands an entry of a partitioned graph: the owner of its object's rows, or — at a
// hub's nodes, whose userset tuples every rank holds and whose direct tuples only the subject's
// owner does — the owner of the check's subject (engine.hpp part_keep).
__device__ __forceinline__ uint32_t part_dest(const Ctx& c, uint32_t q, uint32_t obj, uint16_t node) {
  if (c.part_sub && c.part_sub[node])
    return part_owner(c.ck_items[c.queries[q].check].subject_id, c.world);
  return part_owner(obj, c.world);
}

__device__ __forceinline__ void push_entry(const Ctx& c, uint32_t q, uint32_t obj, uint16_t node,
                                           uint32_t depth, uint32_t cond) {
  if (cond & kExactBit) {  // exact-depth: one entry per (vertex, depth); never a cond path
    if (vinsert(c, make_key(c, q, node, 0u, depth, obj)) <= 0) return;
  } else {
    if ((cond & kCondBit) && vlookup(c, make_key(c, q, node, 0u, 0u, obj))) return;  // unconditional visit exists
    if (vinsert(c, make_key(c, q, node, cond & kCondBit, 0u, obj)) <= 0) return;
  }
  Entry* dst = c.next;
  unsigned idx;
  if (c.world > 1 && part_dest(c, q, obj, node) != c.rank) {
    // another rank holds what the entry reads: exchanged after this level (the visited key
    // above also stops this rank from sending the same entry twice)
    const uint32_t d = part_dest(c, q, obj, node);
    idx = atomicAdd(&c.out_cnt[d], 1u);
    if (idx >= c.out_cap) {
      atomicOr(&c.ctr->overflow, 2u);
      return;
    }
    dst = c.outbox + (size_t)d * c.out_cap;
  } else {
    idx = atomicAdd(&c.ctr->next_size, 1u);
  }
  if (idx >= c.frontier_cap) {
    atomicOr(&c.ctr->overflow, 2u);
    return;
  }
  Entry e;
  e.q = q;
  e.obj = obj;
  e.node = node;
  e.depth = (uint8_t)(depth > 255 ? 255 : depth);
  e.cond = (uint8_t)cond;
  dst[idx] = e;
  c.queries[q].last_alive = c.level + 1;  // benign race: every writer stores the same value
}

// Device reads through the pointers a DevCSR holds. Those pointers are loaded from memory, so
// the compiler cannot tell they point at HBM and would emit flat instructions, whose waits also
// drain every outstanding LDS operation (and vice versa); the explicit global address space keeps
// them global_load_* (vmcnt only).
#define GCK_GLOBAL __attribute__((address_space(1)))
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

template <class T>
__device__ __forceinline__ const GCK_GLOBAL T* gptr(const T* p) {
  return (const GCK_GLOBAL T*)p;
}
template <class T>
__device__ __forceinline__ GCK_GLOBAL T* gptr_w(T* p) {
  return (GCK_GLOBAL T*)p;
}
// A result of a batch the join publishes before its kernel has ended, on a stream no reader is
// ordered after (GCK_SUBMIT_ENGINE_STREAM): an agent-scope store, written through the XCD's L2, so
// that once the wave's stores have completed (s_waitcnt) the value is visible to every XCD and
// to the copy engines — no end-of-kernel L2 write-back is needed before the publication.
template <class T>
__device__ __forceinline__ void store_result(T* p, T v, bool coherent) {
  if (coherent)
    __hip_atomic_store(gptr_w(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    *gptr_w(p) = v;
}
// A join's `coherent` word: kPubCoherent = results written through the L2 (above);
// kPubBySignal = the batch was dispatched into an engine HSA queue (aql.inc), whose packet's
// system-scope release fence and completion signal the host waits on: the last block's sequence
// word then needs no release of its own (a release there writes the L2s back mid-kernel, once
// more before the packet's own write-back, and waits for it: the dispatch span's tail)
constexpr uint32_t kPubCoherent = 1u, kPubBySignal = 2u;
__device__ __forceinline__ void pub_seq_store(unsigned* p, unsigned seq, uint32_t coherent) {
  if (coherent & kPubBySignal)
    __hip_atomic_store(p, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  else
    __hip_atomic_store(p, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t csr_off(const DevCSR& r, uint32_t i) { return gptr(r.off)[i]; }
__device__ __forceinline__ uint32_t csr_nbr(const DevCSR& r, uint32_t p) { return gptr(r.nbr)[p]; }
__device__ __forceinline__ uint32_t csr_cav(const DevCSR& r, uint32_t p) { return gptr(r.cav)[p]; }
__device__ __forceinline__ int64_t csr_exp(const DevCSR& r, uint32_t p) { return gptr(r.exp_us)[p]; }

// Is the check of permission node p on object obj an exact-depth check (its root can reach the
// depth budget)? obj must be a known object of the node's type.
__device__ __forceinline__ bool deep_root(const Ctx& c, const DevNode* nodes, uint32_t p, uint32_t obj) {
  if (c.force_exact) return true;
  if (!(nodes[p].flags & NF_DEEP) || !c.hgt) return false;
  const unsigned long long h = gptr(c.hgt)[p];
  return h != 0 && gptr(reinterpret_cast<const uint32_t*>(h))[obj] >= c.max_depth;
}

// lower_bound of `sid` in the CSR row of `obj`; returns the position or kNone.
__device__ __forceinline__ uint32_t row_find(const DevCSR& r, uint32_t obj, uint32_t sid,
                                             uint32_t& probes) {
  if (obj >= r.n_rows) return kNone;
  uint32_t lo = csr_off(r, obj), hi = csr_off(r, obj + 1);
  const uint32_t end = hi;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    ++probes;
    if (csr_nbr(r, mid) < sid) lo = mid + 1;
    else hi = mid;
  }
  if (lo < end) {
    if (hi == end) ++probes;  // the final equality read when the loop never touched lo
    if (csr_nbr(r, lo) == sid) return lo;
  }
  return kNone;
}

__device__ __forceinline__ bool visible(const DevCSR& r, uint32_t pos, int64_t now_us) {
  if (!r.is_ext) return true;
  int64_t x = csr_exp(r, pos);
  return x == 0 || x > now_us;
}

// Lazy caveat evaluation: the outcome of (partial instance row, context slot) from the map of
// pairs the host has evaluated, else 4 after recording the pair for the host (once per pass; a
// pass that overruns kReqCap leaves the rest to the next).
constexpr uint32_t kReqCap = 1u << 18;
constexpr uint32_t kReqSet = 1u << 20;

// (out of line — it is rare — with the Ctx fields it reads as arguments: a `const Ctx&` to an
// out-of-line callee makes every thread of the calling kernel copy the whole Ctx to scratch)
__device__ __noinline__ uint32_t cav_lazy(const unsigned long long* cav_keys, const uint8_t* cav_vals, uint64_t cav_kmask,
                                          unsigned long long* req_set, unsigned long long* req_list, unsigned* req_cnt,
                                          DevCounters* ctr, uint32_t row, uint32_t slot) {
  const unsigned long long key = ((unsigned long long)row << 32) | slot;
  uint64_t h = mix64(key) & cav_kmask;
  for (int p = 0; p < 64; ++p) {  // the host keeps the map at most half full
    const unsigned long long k = gptr(cav_keys)[h];
    if (k == key) return gptr(cav_vals)[h];
    if (k == kEmptyKey) break;
    h = (h + 1) & cav_kmask;
  }
  atomicAdd(&ctr->cav_requests, 1u);
  if (__hip_atomic_load(req_cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= kReqCap) return 4u;
  uint64_t s = mix64(key) & (kReqSet - 1);
  for (int p = 0; p < 128; ++p) {
    const unsigned long long v = __hip_atomic_load(&req_set[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v == key) return 4u;
    if (v == kEmptyKey) {
      const unsigned long long prev = atomicCAS(&req_set[s], kEmptyKey, key);
      if (prev == kEmptyKey) {
        const unsigned idx = atomicAdd(req_cnt, 1u);
        if (idx < kReqCap) gptr_w(req_list)[idx] = key;
        return 4u;
      }
      if (prev == key) return 4u;
    }
    s = (s + 1) & (kReqSet - 1);
  }
  return 4u;
}

// Caveat instance `cav` on a path of the check whose item is `item`: 0 = the caveat is false
// (the relationship does not count), 1 = true (a plain edge), 2 = unresolved (CONDITIONAL). A
// pair whose evaluation failed marks the check (it ends with GCK_ITEM_ERR_CAVEAT_EVAL) and a
// pair not evaluated yet reads as unresolved (the batch runs again once it is).
__device__ __forceinline__ uint32_t cav_state(const Ctx& c, uint32_t cav, uint32_t item) {
  const uint32_t s = gptr(c.cav_static)[cav];
  if (s != 2u || c.n_ctx == 0) return s;
  const uint32_t slot = gptr(c.ck_items)[item].context_slot;
  if (slot == 0 || slot > c.n_ctx) return 2u;
  const uint32_t row = gptr(c.cav_row)[cav];
  const uint32_t v = c.cav_keys ? cav_lazy(c.cav_keys, c.cav_vals, c.cav_kmask, c.req_set, c.req_list, c.req_cnt, c.ctr,
                                          row, slot)
                                : (uint32_t)gptr(c.cav_dyn)[(size_t)row * c.n_dist + gptr(c.cav_slot)[slot - 1]];
  if (v == 3u) {
    const uint32_t k = c.ck_map ? gptr(c.ck_map)[item] : c.ck_off + item;
    gptr_w(c.cav_flag)[k] = 1;
    atomicAdd(&c.ctr->cav_errors, 1u);
  }
  return v > 2u ? 2u : v;
}

__device__ __forceinline__ uint32_t ext_state(const Ctx& c, const DevCSR& r, uint32_t pos, uint32_t item) {
  if (!visible(r, pos, c.now_us)) return 0u;
  return cav_state(c, csr_cav(r, pos), item);
}

// Membership-index bucket scan: 1 = key present, 0 = absent (the bucket has an empty slot, so
// no key homed here overflowed), 2 = bucket full without the key (continue with the next one).
constexpr int kBucketKeys = 8;  // 8 x u64 = 64 B

__device__ __forceinline__ uint32_t bucket_probe(const unsigned long long* tab, uint32_t b,
                                                 unsigned long long key) {
  const GCK_GLOBAL u64x2* p = (const GCK_GLOBAL u64x2*)(tab + (size_t)b * kBucketKeys);
  const u64x2 a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
  const bool hit = a0.x == key || a0.y == key || a1.x == key || a1.y == key || a2.x == key ||
                   a2.y == key || a3.x == key || a3.y == key;
  const bool empty = a0.x == kEmptyKey || a0.y == kEmptyKey || a1.x == kEmptyKey || a1.y == kEmptyKey ||
                     a2.x == kEmptyKey || a2.y == kEmptyKey || a3.x == kEmptyKey || a3.y == kEmptyKey;
  return hit ? 1u : empty ? 0u : 2u;
}

__device__ __forceinline__ unsigned long long mkey(uint32_t obj, uint32_t sid) {
  return ((unsigned long long)obj << 32) | sid;
}

__device__ __forceinline__ uint32_t mbucket(const DevCSR& r, unsigned long long key) {
  return (uint32_t)(mix64(key) & r.mmask);
}

// Continue a lookup whose bucket b answered `v` (0/1/2, bucket_probe).
__device__ __forceinline__ bool mhash_finish(const DevCSR& r, uint32_t b, unsigned long long key, uint32_t v,
                                             uint32_t& probes) {
  while (v == 2u) {
    b = (uint32_t)((b + 1) & r.mmask);
    v = bucket_probe(r.mhash, b, key);
    ++probes;
  }
  return v == 1u;
}

// Is (obj, sid) in the membership index? One 64-byte bucket read in the common case.
__device__ __forceinline__ bool hash_member(const DevCSR& r, uint32_t obj, uint32_t sid, uint32_t& probes) {
  const unsigned long long key = mkey(obj, sid);
  const uint32_t b = mbucket(r, key);
  ++probes;
  return mhash_finish(r, b, key, bucket_probe(r.mhash, b, key), probes);
}

// checkDirect membership on one CSR: the subject itself (`direct`) and/or the wildcard
// (`wild`) for the check of `item`. Returns 0 = absent, 1 = present, 2 = present through a
// caveat that stays unresolved.
__device__ __forceinline__ uint32_t member_test(const Ctx& c, const DevCSR& r, uint32_t obj, uint32_t sid,
                                                bool direct, bool wild, uint32_t item, uint32_t& rows,
                                                uint32_t& probes) {
  if (obj >= r.n_rows) return 0;
  if (r.mhash) {  // plain direct CSR: hashed index, no row read
    if (direct && hash_member(r, obj, sid, probes)) return 1;
    if (wild && r.has_wild && hash_member(r, obj, kWildcard, probes)) return 1;
    return 0;
  }
  ++rows;
  uint32_t best = 0;
  if (direct) {
    const uint32_t p = row_find(r, obj, sid, probes);
    if (p != kNone) best = r.is_ext ? ext_state(c, r, p, item) : 1u;
  }
  if (wild && best != 1) {
    const uint32_t b = csr_off(r, obj), en = csr_off(r, obj + 1);
    ++probes;
    if (en > b && csr_nbr(r, en - 1) == kWildcard) {
      const uint32_t m = r.is_ext ? ext_state(c, r, en - 1, item) : 1u;
      if (m && (best == 0 || m == 1)) best = m;
    }
  }
  return best;
}

__device__ __forceinline__ void emit_segment(const Ctx& c, uint32_t csr, uint32_t obj, uint32_t q,
                                             uint16_t target, uint32_t depth, uint32_t cond,
                                             uint32_t& rows) {
  if (csr == kNone || target == kNoNode) return;
  const DevCSR& r = c.csrs[csr];
  if (obj >= r.n_rows) return;
  ++rows;
  uint32_t b = csr_off(r, obj), e = csr_off(r, obj + 1);
  if (e == b) return;
  unsigned long long packed =
      atomicAdd(&c.ctr->seg_ctr, (1ull << 40) | (unsigned long long)(e - b));
  uint32_t si = (uint32_t)(packed >> 40);
  if (si >= c.seg_cap) {
    atomicOr(&c.ctr->overflow, 4u);
    return;
  }
  Segment s;
  s.edge_start = packed & ((1ull << 40) - 1);
  s.q = q;
  s.begin = b;
  s.len = e - b;
  s.csr = csr;
  s.target = target;
  s.depth = (uint8_t)(depth > 255 ? 255 : depth);
  s.cond = (uint8_t)cond;
  s.pad = 0;
  c.segs[si] = s;
}

// Spawn a join (intersection / exclusion / all-arrow) for node `node` at `obj` on behalf of
// query `q`. Each operand becomes a child query with its own memoised frontier. `cond` carries
// the entry's bits: the cond bit conditions the join's result (non-exact checks), the exact bit
// passes on to the operands; an exact all() operand entered through a caveated tupleset edge is
// tagged with the caveat's outcome (and_tag) instead of a cond bit.
__device__ __forceinline__ void spawn_join(const Ctx& c, uint32_t q, uint32_t obj, uint16_t node, uint32_t depth,
                           uint32_t cond, uint32_t& rows) {
  const DevNode nd = c.nodes[node];
  const uint32_t check = c.queries[q].check;
  const uint32_t ex = cond & kExactBit;
  uint32_t n_ops = 0;
  if (nd.kind == NK_ARROW_ALL) {
    bool missing = false;
    for (uint32_t k = 0; k < nd.count; ++k) {
      const DevItem it = c.items[nd.first + k];
      for (int pass = 0; pass < 2; ++pass) {
        uint32_t ci = pass ? it.csr_ext : it.csr_plain;
        if (ci == kNone) continue;
        const DevCSR& r = c.csrs[ci];
        if (obj >= r.n_rows) continue;
        ++rows;
        uint32_t b = csr_off(r, obj), e = csr_off(r, obj + 1);
        for (uint32_t p = b; p < e; ++p) {
          if (!visible(r, p, c.now_us)) continue;
          // a subject lacking the target fails the all() (NO dominates every operand); so does
          // one whose caveat is false, unless the check is exact-depth (and3(false, ERR) = ERR)
          if (it.target == kNoNode || (!ex && r.is_ext && cav_state(c, csr_cav(r, p), check) == 0u)) missing = true;
          ++n_ops;
        }
      }
    }
    if (n_ops == 0 || missing) return;  // all() over nothing, or a subject lacking the target: NO
  } else if (nd.kind == NK_NIL) {
    return;
  } else {
    n_ops = nd.count;
  }
  unsigned j = atomicAdd(&c.ctr->n_joins, 1u);
  unsigned q0 = atomicAdd(&c.ctr->n_queries, n_ops);
  if (j >= c.j_hi) {
    atomicOr(&c.ctr->overflow, 16u);
    return;
  }
  if (q0 + n_ops > c.q_hi) {
    atomicOr(&c.ctr->overflow, 8u);
    return;
  }
  DevJoin J;
  J.parent_q = q;
  J.first_child = q0;
  J.n_ops = n_ops;
  J.op = nd.kind;
  J.cond = cond & kCondBit;
  J.remaining = (int32_t)n_ops;
  J.state = 0;
  J.pad = 0;
  c.joins[j] = J;
  for (uint32_t k = 0; k < n_ops; ++k) {
    DevQuery cq;
    cq.check = check;
    cq.parent_join = j;
    cq.flags = 0;
    cq.pending_joins = 0;
    cq.last_alive = c.level;  // raised to level+1 by push_entry
    cq.operand = k;
    c.queries[q0 + k] = cq;
  }
  __hip_atomic_fetch_add(&c.queries[q].pending_joins, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  if (nd.kind == NK_ARROW_ALL) {
    uint32_t k = 0;
    for (uint32_t t = 0; t < nd.count; ++t) {
      const DevItem it = c.items[nd.first + t];
      for (int pass = 0; pass < 2; ++pass) {
        uint32_t ci = pass ? it.csr_ext : it.csr_plain;
        if (ci == kNone) continue;
        const DevCSR& r = c.csrs[ci];
        if (obj >= r.n_rows) continue;
        uint32_t b = csr_off(r, obj), e = csr_off(r, obj + 1);
        for (uint32_t p = b; p < e; ++p) {
          if (!visible(r, p, c.now_us)) continue;
          const uint32_t st = r.is_ext ? cav_state(c, csr_cav(r, p), check) : 1u;
          if (ex) {
            c.queries[q0 + k].operand = k | ((st == 1u ? kTagNone : st == 2u ? kTagCond : kTagFalse) << 24);
            push_entry(c, q0 + k, csr_nbr(r, p), it.target, depth + 1, kExactBit);
          } else {
            push_entry(c, q0 + k, csr_nbr(r, p), it.target, depth + 1, st == 2u ? kCondBit : 0u);
          }
          ++k;
        }
      }
    }
  } else {
    for (uint32_t k = 0; k < n_ops; ++k) {
      const DevItem it = c.items[nd.first + k];
      push_entry(c, q0 + k, obj, it.target, depth + it.dispatch, ex);
    }
  }
}

// Exact-depth checks: the edge into (obj, node) has a caveat that is unresolved (kTagCond) or
// false (kTagFalse) for this check: a single-operand join whose operand query walks from
// (obj, node) and whose result reaches query q through and_tag. Deduplicated per (q, vertex,
// depth, tag).
__device__ __forceinline__ void spawn_and(const Ctx& c, uint32_t q, uint32_t obj, uint16_t node, uint32_t depth, uint32_t tag) {
  if (vinsert(c, make_key(c, q, node, tag, depth, obj)) <= 0) return;
  unsigned j = atomicAdd(&c.ctr->n_joins, 1u);
  unsigned q0 = atomicAdd(&c.ctr->n_queries, 1u);
  if (j >= c.j_hi) {
    atomicOr(&c.ctr->overflow, 16u);
    return;
  }
  if (q0 + 1 > c.q_hi) {
    atomicOr(&c.ctr->overflow, 8u);
    return;
  }
  DevJoin J;
  J.parent_q = q;
  J.first_child = q0;
  J.n_ops = 1;
  J.op = NK_INTERSECT;  // the intersection of one operand is the operand
  J.cond = 0;
  J.remaining = 1;
  J.state = 0;
  J.pad = 0;
  c.joins[j] = J;
  DevQuery cq;
  cq.check = c.queries[q].check;
  cq.parent_join = j;
  cq.flags = 0;
  cq.pending_joins = 0;
  cq.last_alive = c.level;
  cq.operand = tag << 24;
  c.queries[q0] = cq;
  __hip_atomic_fetch_add(&c.queries[q].pending_joins, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  push_entry(c, q0, obj, node, depth, kExactBit);
}

// ---- kernels -----------------------------------------------------------------------------

__device__ __forceinline__ void wave_add(unsigned long long* p, unsigned long long v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0 && v) atomicAdd(p, v);
}

__global__ void __launch_bounds__(kBlock) k_init(Ctx c, const gck_item* __restrict__ items,
                                                 uint32_t n, Entry* __restrict__ fr0,
                                                 int32_t* __restrict__ item_err) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const gck_item it = items[i];
  int32_t err = GCK_ITEM_OK;
  if (it.resource_type >= c.n_types || it.subject_type >= c.n_types) {
    err = GCK_ITEM_ERR_UNKNOWN_TYPE;
  } else if (it.permission >= c.n_rels || c.nodes[it.permission].type != it.resource_type) {
    err = GCK_ITEM_ERR_UNKNOWN_PERMISSION;
  } else if (it.subject_relation != kEllipsis &&
             (it.subject_relation >= c.n_rels ||
              c.nodes[it.subject_relation].type != it.subject_type)) {
    err = GCK_ITEM_ERR_UNKNOWN_SUBJECT_RELATION;
  } else if (it.subject_id == kWildcard) {
    err = GCK_ITEM_ERR_WILDCARD_SUBJECT;
  }
  item_err[i] = err;
  DevCheck ck;
  ck.sid = it.subject_id;
  ck.stype = it.subject_type;
  ck.srel = it.subject_relation;
  c.checks[i] = ck;
  DevQuery q;
  q.check = i;
  q.parent_join = kNone;
  q.pending_joins = 0;
  q.last_alive = 0;
  q.operand = 0;
  q.flags = 0;
  if (err != GCK_ITEM_OK) {
    q.flags = QF_DONE | (kResErr << QF_RES_SHIFT);
  } else if (it.resource_id >= c.type_counts[it.resource_type]) {
    // unknown object: no relationships (client/client_test.go:209-215) unless it is the
    // subject itself (identity filter)
    bool ident = it.resource_type == it.subject_type && it.permission == it.subject_relation &&
                 it.resource_id == it.subject_id && it.resource_id != kAbsent;
    q.flags = QF_DONE | ((ident ? GCK_PERM_HAS : GCK_PERM_NO) << QF_RES_SHIFT);
  }
  c.queries[i] = q;
  Entry e;
  e.q = i;
  e.obj = it.resource_id;
  e.node = it.permission;
  e.depth = 0;
  e.cond = (!(q.flags & QF_DONE) && deep_root(c, c.nodes, it.permission, it.resource_id)) ? kExactBit : 0u;
  fr0[i] = e;
}

__global__ void __launch_bounds__(kBlock) k_expand(Ctx c, const Entry* __restrict__ cur, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t rows = 0, probes = 0, expanded = 0;
  if (i < n) {
    const Entry e = cur[i];
    DevQuery* q = &c.queries[e.q];
    uint32_t qf = qflags_hint(q);
    if (!(qf & QF_DONE)) {
      ++expanded;
      const DevCheck s = c.checks[q->check];
      const DevNode nd = c.nodes[e.node];
      bool done = false;
      if ((nd.flags & NF_REAL) && e.node == s.srel && nd.type == s.stype && e.obj == s.sid) {
        set_found(c, e.q, e.cond);  // filterForFoundMemberResource
        done = true;
      } else if (e.depth >= c.max_depth) {
        atomicOr(&q->flags, (uint32_t)QF_ERR);  // dispatch.CheckDepth: max depth exceeded
        done = true;
      }
      if (!done) {
        switch (nd.kind) {
          case NK_RELATION: {
            // pass 1: direct subject + wildcard membership (checkDirect)
            for (uint32_t k = 0; k < nd.count && !done; ++k) {
              const DevItem it = c.items[nd.first + k];
              if (it.stype != s.stype) continue;
              const bool direct = it.srel == s.srel;
              const bool wild = it.srel == kEllipsis && s.srel == kEllipsis;
              if (!direct && !wild) continue;
              for (int pass = 0; pass < 2 && !done; ++pass) {
                uint32_t ci = pass ? it.csr_ext : it.csr_plain;
                if (ci == kNone) continue;
                const uint32_t m = member_test(c, c.csrs[ci], e.obj, s.sid, direct, wild, q->check, rows, probes);
                if (m) {
                  const uint32_t cond = (e.cond & kCondBit) | (m == 2);
                  set_found(c, e.q, cond);
                  if (!cond) done = true;
                }
              }
            }
            // pass 2: userset subjects are re-dispatched
            for (uint32_t k = 0; k < nd.count && !done; ++k) {
              const DevItem it = c.items[nd.first + k];
              if (it.srel == kEllipsis) continue;
              emit_segment(c, it.csr_plain, e.obj, e.q, it.target, e.depth + 1u, e.cond, rows);
              emit_segment(c, it.csr_ext, e.obj, e.q, it.target, e.depth + 1u, e.cond, rows);
            }
            break;
          }
          case NK_UNION: {
            for (uint32_t k = 0; k < nd.count; ++k) {
              const DevItem it = c.items[nd.first + k];
              if (it.kind == IT_COMPUTED) {
                push_entry(c, e.q, e.obj, it.target, e.depth + 1u, e.cond);
              } else if (it.kind == IT_ARROW) {
                emit_segment(c, it.csr_plain, e.obj, e.q, it.target, e.depth + 1u, e.cond, rows);
                emit_segment(c, it.csr_ext, e.obj, e.q, it.target, e.depth + 1u, e.cond, rows);
              } else if (it.kind == IT_SUB) {
                spawn_join(c, e.q, e.obj, it.target, e.depth, e.cond, rows);
              }
            }
            break;
          }
          case NK_INTERSECT:
          case NK_EXCLUDE:
          case NK_ARROW_ALL:
            spawn_join(c, e.q, e.obj, e.node, e.depth, e.cond, rows);
            break;
          default:
            break;
        }
      }
    }
  }
  wave_add(&c.ctr->row_lookups, rows);
  wave_add(&c.ctr->probes, probes);
  wave_add(&c.ctr->expanded, expanded);
}

// Load-balanced edge enumeration: edge e belongs to the last segment whose edge_start <= e.
__global__ void __launch_bounds__(kBlock) k_edges(Ctx c) {
  const unsigned long long packed = c.ctr->seg_ctr;
  const uint32_t nseg = (uint32_t)min((unsigned long long)(packed >> 40), (unsigned long long)c.seg_cap);
  const unsigned long long total = packed & ((1ull << 40) - 1);
  unsigned long long done_edges = 0, ext_edges = 0;
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long eid = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
       eid < total; eid += stride) {
    uint32_t lo = 0, hi = nseg;  // upper_bound
    while (lo < hi) {
      uint32_t mid = (lo + hi) >> 1;
      if (c.segs[mid].edge_start <= eid) lo = mid + 1;
      else hi = mid;
    }
    if (lo == 0) continue;
    const Segment s = c.segs[lo - 1];
    const unsigned long long off = eid - s.edge_start;
    if (off >= s.len) continue;  // a segment dropped on overflow
    if (qflags_hint(&c.queries[s.q]) & QF_DONE) continue;
    const DevCSR& r = c.csrs[s.csr];
    const uint32_t p = s.begin + (uint32_t)off;
    const uint32_t x = csr_nbr(r, p);
    ++done_edges;
    uint32_t cond = s.cond;
    if (r.is_ext) {
      ++ext_edges;
      if (!visible(r, p, c.now_us)) continue;
      const uint32_t st = cav_state(c, csr_cav(r, p), c.queries[s.q].check);
      if (cond & kExactBit) {
        if (st != 1u) {  // unresolved or false caveat: an and-query (and3 of the oracle)
          if (x != kWildcard) spawn_and(c, s.q, x, s.target, s.depth, st == 2u ? kTagCond : kTagFalse);
          continue;
        }
      } else {
        if (st == 0u) continue;
        cond |= (st == 2u);
      }
    }
    if (x == kWildcard) continue;
    push_entry(c, s.q, x, s.target, s.depth, cond);
  }
  wave_add(&c.ctr->edges, done_edges);
  wave_add(&c.ctr->ext_edges, ext_edges);
}

__device__ __forceinline__ uint32_t result_from_flags(uint32_t f) {
  if (f & QF_FOUND_Y) return GCK_PERM_HAS;
  if (f & QF_ERR) return kResErr;
  if (f & QF_FOUND_C) return GCK_PERM_CONDITIONAL;
  return GCK_PERM_NO;
}

__device__ __forceinline__ bool try_finalize(DevQuery* q, uint32_t res) {
  uint32_t f = qflags(q);
  while (!(f & QF_DONE)) {
    uint32_t nf = f | QF_DONE | (res << QF_RES_SHIFT);
    uint32_t prev = atomicCAS(&q->flags, f, nf);
    if (prev == f) return true;
    f = prev;
  }
  return false;
}

// Decide query `qi` with `res` and cascade the decision through its parent joins.
__device__ __forceinline__ void finalize(const Ctx& c, uint32_t qi, uint32_t res) {
  for (int guard = 0; guard < 1 << 20; ++guard) {
    DevQuery* q = &c.queries[qi];
    if (!try_finalize(q, res)) return;
    const uint32_t j = q->parent_join;
    if (j == kNone) return;
    DevJoin* J = &c.joins[j];
    const uint32_t op = J->op;
    const uint32_t opnd = q->operand;
    const uint32_t r = and_tag(opnd >> 24, res);  // the operand's contribution
    uint32_t bit;
    bool early;
    if (op == NK_EXCLUDE && (opnd & 0xFFFFFFu) == 0) {
      bit = r == GCK_PERM_HAS ? JS_BASE_Y : r == GCK_PERM_NO ? JS_BASE_N
            : r == GCK_PERM_CONDITIONAL ? JS_BASE_C : JS_BASE_ERR;
      early = r == GCK_PERM_NO;
    } else {
      bit = r == GCK_PERM_HAS ? JS_ANY_Y : r == GCK_PERM_NO ? JS_ANY_N
            : r == GCK_PERM_CONDITIONAL ? JS_ANY_C : JS_ANY_ERR;
      early = (op == NK_EXCLUDE) ? r == GCK_PERM_HAS : r == GCK_PERM_NO;
    }
    __hip_atomic_fetch_or(&J->state, bit, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    int rem = __hip_atomic_fetch_add(&J->remaining, -1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) - 1;
    if (!(rem == 0 || early)) return;
    uint32_t st = __hip_atomic_fetch_or(&J->state, (uint32_t)JS_RESOLVED, __ATOMIC_ACQ_REL,
                                        __HIP_MEMORY_SCOPE_AGENT);
    if (st & JS_RESOLVED) return;
    uint32_t jr;
    if (early) {
      jr = GCK_PERM_NO;
    } else if (op == NK_EXCLUDE) {
      jr = (st & (JS_BASE_N | JS_ANY_Y)) ? GCK_PERM_NO
           : (st & (JS_BASE_ERR | JS_ANY_ERR)) ? kResErr
           : (st & (JS_BASE_C | JS_ANY_C)) ? GCK_PERM_CONDITIONAL : GCK_PERM_HAS;
    } else {
      jr = (st & JS_ANY_N) ? GCK_PERM_NO : (st & JS_ANY_ERR) ? kResErr
           : (st & JS_ANY_C) ? GCK_PERM_CONDITIONAL : GCK_PERM_HAS;
    }
    if (rem > 0) {  // decided early: cancel the operands still running
      for (uint32_t k = 0; k < J->n_ops; ++k) {
        DevQuery* cq = &c.queries[J->first_child + k];
        uint32_t f = qflags(cq);
        while (!(f & QF_DONE)) {
          uint32_t prev = atomicCAS(&cq->flags, f, f | QF_DONE | QF_CANCELLED);
          if (prev == f) break;
          f = prev;
        }
      }
    }
    if (J->cond && jr == GCK_PERM_HAS) jr = GCK_PERM_CONDITIONAL;  // caveated edge AND result
    DevQuery* P = &c.queries[J->parent_q];
    uint32_t fbit = jr == GCK_PERM_HAS ? QF_FOUND_Y : jr == GCK_PERM_CONDITIONAL ? QF_FOUND_C
                    : jr == kResErr ? QF_ERR : 0u;
    if (fbit) __hip_atomic_fetch_or(&P->flags, fbit, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    int pend = __hip_atomic_fetch_add(&P->pending_joins, -1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) - 1;
    uint32_t pf = qflags(P);
    if (pf & QF_DONE) return;
    if (pf & QF_FOUND_Y) {
      qi = J->parent_q;
      res = GCK_PERM_HAS;
      continue;
    }
    if (pend == 0 && P->last_alive <= c.level) {
      qi = J->parent_q;
      res = result_from_flags(pf);
      continue;
    }
    return;
  }
}

__device__ __forceinline__ void resolve_query(const Ctx& c, uint32_t qi) {
  DevQuery* q = &c.queries[qi];
  uint32_t f = qflags(q);
  if (f & QF_DONE) return;
  if (f & QF_FOUND_Y) {
    finalize(c, qi, GCK_PERM_HAS);
    return;
  }
  if (q->last_alive > c.level) return;  // entries pushed for the next level
  int pend = __hip_atomic_load(&q->pending_joins, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
  if (pend != 0) return;
  f = qflags(q);
  finalize(c, qi, result_from_flags(f));
}

__global__ void __launch_bounds__(kBlock) k_resolve(Ctx c) {
  // after an overflow some allocated queries/joins were never written: the batch is re-run
  // split in half, so do not touch them
  if (__hip_atomic_load(&c.ctr->overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const uint32_t nq = min(__hip_atomic_load(&c.ctr->n_queries, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                          c.query_cap);
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t qi = blockIdx.x * blockDim.x + threadIdx.x; qi < nq; qi += stride) resolve_query(c, qi);
}

// Publish this level's counts and reset the per-level counters (one lane, after k_resolve).
__global__ void k_level_end(DevCounters* ctr) {
  unsigned long long packed = ctr->seg_ctr;
  ctr->segs_total += packed >> 40;
  ctr->last_next = ctr->next_size;
  ctr->next_size = 0;
  ctr->seg_ctr = 0;
}

// Publishes a finished bundle batch to the host without a copy engine or a stream
// synchronisation: the counter words go to coherent host memory, then the sequence word
// (system-scope release) that the host spins on; the device counters are zeroed on the way,
// so the next batch needs no memset.
__global__ void __launch_bounds__(64) k_publish(unsigned* ctr, uint32_t n_words, unsigned* h_out, unsigned* h_seq,
                                                unsigned seq) {
  for (uint32_t i = threadIdx.x; i < n_words; i += 64) {
    h_out[i] = ctr[i];
    ctr[i] = 0u;
  }
  __threadfence_system();
  if (threadIdx.x == 0) __hip_atomic_store(h_seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(kBlock) k_final(const DevQuery* __restrict__ queries, uint32_t n,
                                                  const int32_t* __restrict__ item_err,
                                                  uint8_t* __restrict__ out_perm,
                                                  int32_t* __restrict__ out_err,
                                                  DevCounters* ctr) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t f = queries[i].flags;
  uint32_t res = (f >> QF_RES_SHIFT) & 0xF;
  int32_t err = item_err[i];
  if (!(f & QF_DONE)) {
    atomicOr(&ctr->overflow, 32u);  // invariant violated: an undecided check
    res = kResErr;
  }
  if (err == GCK_ITEM_OK && res == kResErr) err = GCK_ITEM_ERR_MAX_DEPTH;
  out_perm[i] = (err != GCK_ITEM_OK) ? (uint8_t)GCK_PERM_UNSPECIFIED : (uint8_t)res;
  out_err[i] = err;
}

constexpr int kWaves = kBlock / 64;
constexpr uint32_t kBCtrs = 8;  // per-batch stage counters after DevCounters (Workspace::b_ctrs)
constexpr uint32_t kBDone = 5;  // b_ctrs[kBDone]: the closure join's finished blocks (closure.inc CjArgs::done)

#include "bundle.inc"

// Membership index build: one lane per edge of a plain direct-subject CSR. Each block owns 256
// consecutive edges; two lanes find the block's first and last rows, then every lane finds its
// row in that (usually 1-2 row) window. A key takes the first empty slot of its home bucket or,
// when that is full, of the next buckets in turn (the lookup rule in bucket_probe). Also flags
// whether any row holds the wildcard subject.
__global__ void __launch_bounds__(kBlock) k_build_mhash(const uint32_t* __restrict__ off,
                                                        const uint32_t* __restrict__ nbr, uint32_t n_rows,
                                                        unsigned long long n_edges,
                                                        unsigned long long* __restrict__ tab,
                                                        unsigned long long bmask, unsigned* has_wild) {
  __shared__ uint32_t rows[2];
  const unsigned long long e0 = (unsigned long long)blockIdx.x * kBlock;
  if (threadIdx.x < 2) {
    const unsigned long long t = threadIdx.x == 0 ? e0 : min(e0 + kBlock, n_edges) - 1;
    uint32_t lo = 0, hi = n_rows;  // last row r with off[r] <= t
    while (lo < hi) {
      uint32_t mid = (lo + hi + 1) >> 1;
      if (off[mid] <= t) lo = mid;
      else hi = mid - 1;
    }
    rows[threadIdx.x] = lo;
  }
  __syncthreads();
  const unsigned long long e = e0 + threadIdx.x;
  if (e >= n_edges) return;
  uint32_t lo = rows[0], hi = rows[1];
  while (lo < hi) {
    uint32_t mid = (lo + hi + 1) >> 1;
    if (off[mid] <= e) lo = mid;
    else hi = mid - 1;
  }
  const uint32_t sid = nbr[e];
  if (sid == kWildcard) atomicOr(has_wild, 1u);
  const unsigned long long key = mkey(lo, sid);
  unsigned long long b = mix64(key) & bmask;
  for (;;) {
    unsigned long long* bk = tab + b * kBucketKeys;
    for (int k = 0; k < kBucketKeys; ++k) {
      unsigned long long v = __hip_atomic_load(&bk[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v == key) return;
      if (v == kEmptyKey) {
        v = atomicCAS(&bk[k], kEmptyKey, key);
        if (v == kEmptyKey || v == key) return;
      }
    }
    b = (b + 1) & bmask;
  }
}

__global__ void __launch_bounds__(kBlock) k_gather(const gck_item* __restrict__ items,
                                                   const uint32_t* __restrict__ idx, uint32_t n,
                                                   gck_item* __restrict__ out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = items[idx[i]];
}

__global__ void __launch_bounds__(kBlock) k_scatter(const uint32_t* __restrict__ idx, uint32_t n,
                                                    const uint8_t* __restrict__ perm,
                                                    const int32_t* __restrict__ err,
                                                    uint8_t* __restrict__ out_perm,
                                                    int32_t* __restrict__ out_err) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    out_perm[idx[i]] = perm[i];
    out_err[idx[i]] = err[i];
  }
}

// ---- host side -----------------------------------------------------------------------------

static uint32_t ceil_log2(uint64_t x) {
  uint32_t b = 0;
  while ((1ull << b) < x) ++b;
  return b;
}

// Waits for `ev` by polling its status. hipEventSynchronize / hipStreamSynchronize wait actively
// only briefly and then sleep until the completion interrupt: a Watch batch's waits of a few
// dozen microseconds then pay the wake-up on top (config 5: the merge totals, the merged CSRs,
// the index patch). The host thread applying a Watch batch has nothing else to do meanwhile.
static void spin_event(hipEvent_t ev) {
  for (;;) {
    const hipError_t r = hipEventQuery(ev);
    if (r == hipSuccess) return;
    if (r != hipErrorNotReady) HIP_OK(r);
    __builtin_ia32_pause();
  }
}
// everything enqueued on `s` so far has completed (the engine's Watch event; one writer at a time)
static void spin_stream(Engine& e, hipStream_t s) {
  HIP_OK(hipEventRecord((hipEvent_t)e.sync_ev, s));
  spin_event((hipEvent_t)e.sync_ev);
}

template <class T>
static T* dalloc(std::vector<void*>& list, size_t count, uint64_t* bytes = nullptr) {
  void* p = nullptr;
  size_t sz = std::max<size_t>(count, 1) * sizeof(T);
  // stream-ordered pool (device_init keeps freed blocks cached): a Watch batch replaces a few
  // CSRs, and hipFree would synchronise the device once per array
  HIP_OK(hipMallocAsync(&p, sz, nullptr));
  list.push_back(p);
  if (bytes) *bytes += sz;
  return static_cast<T*>(p);
}

// Watch batches replace the same CSRs batch after batch: their merged arrays (delta.inc) are
// kept when a snapshot retires them and handed to a later batch's merge that fits them, instead
// of a pool free and a pool allocation per array (~4 us of host time each, ~20 per config-5
// batch). At most kRecycleMax bytes are kept; an array is reused for a request of at least 2/3
// of its size, and allocated with 1/8 of slack so that the next batch's (slightly larger) array
// fits it.
// (The largest CSRs of a 1e9-tuple graph — the group -> user memberships and their transpose, 4-5 GB
// each — are among them: a fresh allocation of that size costs tens of ms.)
constexpr size_t kRecycleMax = (size_t)24 << 30;

template <class T>
static T* ralloc(Engine& e, std::vector<void*>& list, size_t count) {
  const size_t need = std::max<size_t>(count, 1) * sizeof(T);
  auto it = e.recycle.lower_bound(need);
  if (it != e.recycle.end() && it->first <= need + need / 2) {
    void* p = it->second;
    e.recycle_bytes -= it->first;
    e.recycle.erase(it);
    list.push_back(p);
    return static_cast<T*>(p);
  }
  const size_t n = (need + need / 8 + 255) / sizeof(T);
  T* p = dalloc<T>(list, n);
  e.recyclable[p] = n * sizeof(T);
  return p;
}

// An array leaving a snapshot: kept for ralloc when ralloc made it and the bound allows, else
// returned to the pool on `st`.
static void retire_array(Engine& e, void* p, hipStream_t st) {
  auto it = e.recyclable.find(p);
  if (it != e.recyclable.end() && e.recycle_bytes + it->second <= kRecycleMax) {
    e.recycle.emplace(it->second, p);
    e.recycle_bytes += it->second;
    return;
  }
  if (it != e.recyclable.end()) e.recyclable.erase(it);
  (void)hipFreeAsync(p, st);
}

static void recycle_free(Engine& e) {
  for (auto& kv : e.recycle) (void)hipFreeAsync(kv.second, nullptr);
  e.recycle.clear();
  e.recyclable.clear();
  e.recycle_bytes = 0;
}

// Runs f(lo, hi) over [0, n) on up to 16 host threads (one below `grain` items); the first
// exception is rethrown.
template <class F>
static void host_parallel(size_t n, size_t grain, F&& f) {
  const size_t nt = std::min<size_t>({16, std::max(1u, std::thread::hardware_concurrency()), (n + grain - 1) / grain});
  if (nt <= 1) {
    if (n) f(0, n);
    return;
  }
  std::vector<std::thread> ts;
  std::vector<std::exception_ptr> ex(nt);
  for (size_t t = 0; t < nt; ++t)
    ts.emplace_back([&, t] {
      try {
        f(n * t / nt, n * (t + 1) / nt);
      } catch (...) {
        ex[t] = std::current_exception();
      }
    });
  for (auto& t : ts) t.join();
  for (auto& x : ex)
    if (x) std::rethrow_exception(x);
}

int device_init(Engine& e) {
  if (e.device_ready) return 0;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
    throw Error(GCK_E_NO_DEVICE, "no HIP device available (libgck requires an MI355X)");
  if (e.cfg.device < 0 || e.cfg.device >= n) throw Error(GCK_E_INVALID_ARGUMENT, "bad device ordinal");
  e.device = e.cfg.device;
  HIP_OK(hipSetDevice(e.device));
  hipMemPool_t pool;
  if (hipDeviceGetDefaultMemPool(&pool, e.device) == hipSuccess) {
    uint64_t keep = ~0ull;  // never hand freed blocks back to the driver between batches
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
  }
  hipStream_t fs = nullptr;
  HIP_OK(hipStreamCreateWithFlags(&fs, hipStreamNonBlocking));
  e.free_stream = fs;
  hipEvent_t dev = nullptr;
  HIP_OK(hipEventCreateWithFlags(&dev, hipEventDisableTiming));
  e.delta_ev = dev;
  hipEvent_t sev = nullptr;
  HIP_OK(hipEventCreateWithFlags(&sev, hipEventDisableTiming));
  e.sync_ev = sev;
  hipEvent_t pev = nullptr;
  HIP_OK(hipEventCreateWithFlags(&pev, hipEventDisableTiming));
  e.patch_ev = pev;
  hipEvent_t bev = nullptr;
  HIP_OK(hipEventCreateWithFlags(&bev, hipEventDisableTiming));
  e.build_ev = bev;
  e.device_ready = true;
  return 0;
}

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
PhaseClock::PhaseClock(const char* w) : what(w), on(debug_env("GCK_DEBUG_PHASES") != nullptr), t0(0), last(0) {
  if (on) t0 = last = now_s();
}
void PhaseClock::mark(const char* phase) {
  if (!on) return;
  const double t = now_s();
  char buf[96];
  snprintf(buf, sizeof(buf), " %s=%.1fus", phase, (t - last) * 1e6);
  line += buf;
  last = t;
}
PhaseClock::~PhaseClock() {
  if (on) fprintf(stderr, "[gck %s] total=%.1fus%s\n", what, (now_s() - t0) * 1e6, line.c_str());
}

static void free_list(std::vector<void*>& list) {
  for (void* p : list) (void)hipFreeAsync(p, nullptr);
  list.clear();
}

static void free_part(PartState* p);  // partition.inc
static void part_filter_device(const Engine& e, DeviceSnapshot& ds, const HostCSR& h, DevCSR& d, uint64_t& ne);

static void aql_workspace_free(Workspace& w);  // aql.inc

static void free_workspace(Workspace* w) {
  if (w->stream) (void)hipStreamSynchronize(w->stream);
  aql_workspace_free(*w);
  if (w->b_st && w->state == 1) (void)hipStreamSynchronize(w->b_st);  // a batch never waited for
  free_part(w->part);
  free_list(w->allocs);
  if (w->h_ctr) (void)hipHostFree(w->h_ctr);
  if (w->h_slots) (void)hipHostFree(w->h_slots);
  if (w->h_items) (void)hipHostFree(w->h_items);
  if (w->h_ctx) (void)hipHostFree(w->h_ctx);
  if (w->dbg) (void)hipFree(w->dbg);
  if (w->timing) (void)hipFree(w->timing);
  if (w->ev0) (void)hipEventDestroy(w->ev0);
  if (w->ev1) (void)hipEventDestroy(w->ev1);
  if (w->ev2) (void)hipEventDestroy(w->ev2);
  for (hipEvent_t ev : w->pev)
    if (ev) (void)hipEventDestroy(ev);
  if (w->stream) (void)hipStreamDestroy(w->stream);
  delete w;
}

static void aql_drain(Engine& e);  // aql.inc
static void aql_free(struct AqlState* st);
static void res_free(Engine& e);   // resident.inc
static uint32_t device_cus(int device);

void device_free(Engine& e) {
  res_free(e);   // (the resident join reads the snapshot and the workspaces: sealed, drained, freed)
  e.res_tried = false;
  aql_drain(e);  // (dispatched joins read the snapshot: none may run past here)
  part_comm_free(e);
  if (e.delta_scratch) {
    (void)hipSetDevice(e.device);
    (void)hipFree(e.delta_scratch);
    e.delta_scratch = nullptr;
    e.delta_scratch_cap = 0;
  }
  if (e.delta_host) {
    (void)hipHostFree(e.delta_host);
    e.delta_host = nullptr;
    e.delta_host_dev = nullptr;
    e.delta_host_cap = 0;
  }
  if (e.dev) {
    (void)hipSetDevice(e.device);
    free_list(e.dev->allocs);
    for (void* p : e.dev->hallocs) (void)hipFree(p);
    delete e.dev;
    e.dev = nullptr;
  }
  if (!e.recycle.empty() || !e.recyclable.empty()) {
    (void)hipSetDevice(e.device);
    recycle_free(e);
  }
  if (!e.ws_pool.empty() || e.part_ws) {
    (void)hipSetDevice(e.device);
    std::vector<Workspace*> all = e.ws_pool;
    if (e.part_ws) all.push_back(e.part_ws);
    for (Workspace* w : all) free_workspace(w);
    e.ws_pool.clear();
    e.part_ws = nullptr;
  }
  aql_free(e.aql);
  e.aql = nullptr;
  e.aql_tried = false;
  if (e.free_stream) {  // device_init makes a new one for the next snapshot
    (void)hipSetDevice(e.device);
    (void)hipStreamSynchronize((hipStream_t)e.free_stream);
    (void)hipStreamDestroy((hipStream_t)e.free_stream);
    e.free_stream = nullptr;
    if (e.delta_ev) (void)hipEventDestroy((hipEvent_t)e.delta_ev);
    e.delta_ev = nullptr;
    if (e.sync_ev) (void)hipEventDestroy((hipEvent_t)e.sync_ev);
    e.sync_ev = nullptr;
    if (e.patch_ev) (void)hipEventDestroy((hipEvent_t)e.patch_ev);
    e.patch_ev = nullptr;
    if (e.build_ev) (void)hipEventDestroy((hipEvent_t)e.build_ev);
    e.build_ev = nullptr;
    e.patch_seq = 0;
    if (e.blob_host) (void)hipHostFree(e.blob_host);
    e.blob_host = nullptr;
    e.blob_host_cap = 0;
    e.device_ready = false;
  }
}

// The snapshot plus every workspace's scratch (gck_device_bytes).
uint64_t device_bytes(Engine& e) {
  uint64_t b = e.dev ? e.dev->bytes : 0;
  std::lock_guard<std::mutex> lk(e.ws_mu);
  for (const Workspace* w : e.ws_pool) b += w->bytes;
  if (e.part_ws) b += e.part_ws->bytes;
  return b;
}

// Host copies of the committed snapshot's own CSRs (not the derived indexes, which a load
// rebuilds): the on-disk snapshot cache (snapfile.cpp) writes these.
void device_export(Engine& e, std::vector<HostCSR>& out) {
  if (!e.dev) throw Error(GCK_E_STATE, "no snapshot on the device");
  HIP_OK(hipSetDevice(e.device));
  HIP_OK(hipDeviceSynchronize());
  const DeviceSnapshot& ds = *e.dev;
  out.clear();
  out.reserve(ds.base.size());
  for (size_t k = 0; k < ds.base.size(); ++k) {
    const BaseCsr& b = ds.base[k];
    const DevCSR& d = ds.table[k];
    HostCSR h;
    h.rel = b.rel;
    h.stype = b.stype;
    h.srel = b.srel;
    h.ext = b.ext;
    h.n_rows = d.n_rows;
    h.off.resize((size_t)d.n_rows + 1);
    HIP_OK(hipMemcpy(h.off.data(), d.off, h.off.size() * 4, hipMemcpyDeviceToHost));
    const uint64_t ne = h.off.back();
    if (ne != b.n_edges) throw Error(GCK_E_DEVICE, "engine invariant violated: CSR edge count");
    h.nbr.resize(ne);
    if (ne) HIP_OK(hipMemcpy(h.nbr.data(), d.nbr, ne * 4, hipMemcpyDeviceToHost));
    if (b.ext) {
      h.cav.resize(ne);
      h.exp_us.resize(ne);
      if (ne) {
        HIP_OK(hipMemcpy(h.cav.data(), d.cav, ne * 4, hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(h.exp_us.data(), d.exp_us, ne * 8, hipMemcpyDeviceToHost));
      }
    }
    out.push_back(std::move(h));
  }
}

void* pinned_alloc(size_t bytes) {
  void* p = nullptr;
  return hipHostMalloc(&p, bytes, hipHostMallocDefault) == hipSuccess ? p : nullptr;
}
void pinned_free(void* p) { (void)hipHostFree(p); }

static uint64_t mhash_slots(uint64_t ne) { return 1ull << std::max<uint32_t>(10, ceil_log2(2 * ne)); }

// Whether a plain direct-subject CSR of `ne` edges gets a membership index. Above 4 GB of index
// (config 4's 1e9 group#member@user: 17.2 GB, a third of the snapshot) it is built only with
// GCK_FLAG_BIG_MHASH: the one-round joins never probe it, and a check they leave tests membership
// by a binary search of the row instead (member_test, the bundles' probes), as with
// GCK_FLAG_NO_MHASH.
static bool mhash_affordable(const Engine& e, uint64_t ne) {
  return mhash_slots(ne) * 8ull <= (4ull << 30) || (e.cfg.flags & GCK_FLAG_BIG_MHASH);
}
static bool want_mhash(const Engine& e, uint64_t ne) {
  if (ne == 0 || (e.cfg.flags & GCK_FLAG_NO_MHASH)) return false;
  return mhash_affordable(e, ne);
}
// DevCSR::pad bit: has_wild is known although the CSR has no index (scan_wild)
constexpr uint16_t kCsrWildKnown = 1;

// Membership index of a plain CSR (d.off / d.nbr on the device): sets d.mhash, d.mmask and
// d.has_wild.
static void build_mhash(DeviceSnapshot& ds, DevCSR& d, uint64_t ne) {
  const uint64_t slots = mhash_slots(ne);
  if (slots / kBucketKeys > (1ull << 32)) throw Error(GCK_E_CAPACITY, "membership index too large");
  unsigned long long* tab = dalloc<unsigned long long>(ds.allocs, slots, &ds.bytes);
  std::vector<void*> tmp;
  unsigned* wild_flag = dalloc<unsigned>(tmp, 1);
  unsigned hw = 0;
  try {
    HIP_OK(hipMemset(tab, 0xFF, slots * sizeof(unsigned long long)));
    HIP_OK(hipMemset(wild_flag, 0, sizeof(unsigned)));
    const uint64_t blocks = (ne + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_build_mhash, dim3((uint32_t)blocks), dim3(kBlock), 0, 0, d.off, d.nbr, d.n_rows,
                       (unsigned long long)ne, tab, (unsigned long long)(slots / kBucketKeys - 1), wild_flag);
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpy(&hw, wild_flag, sizeof(unsigned), hipMemcpyDeviceToHost));
  } catch (...) {
    free_list(tmp);
    throw;
  }
  free_list(tmp);
  d.mhash = tab;
  d.mmask = slots / kBucketKeys - 1;
  d.has_wild = hw ? 1 : 0;
}

__global__ void __launch_bounds__(kBlock) k_scan_wild(const uint32_t* __restrict__ nbr, unsigned long long n,
                                                      unsigned* __restrict__ flag) {
  const unsigned long long e = (unsigned long long)blockIdx.x * kBlock + threadIdx.x;
  if (e < n && nbr[e] == kWildcard) *flag = 1u;
}

// has_wild of a plain direct CSR that gets no index because of its size (want_mhash): the closure
// join's and the bidirectional search's planning read it (bidir.inc) as they read an index's.
static void scan_wild(const Engine& e, DevCSR& d, uint64_t ne) {
  if (ne == 0 || (e.cfg.flags & GCK_FLAG_NO_MHASH) || mhash_affordable(e, ne)) return;
  std::vector<void*> tmp;
  unsigned hw = 0;
  try {
    unsigned* flag = dalloc<unsigned>(tmp, 1);
    HIP_OK(hipMemsetAsync(flag, 0, 4, nullptr));
    hipLaunchKernelGGL(k_scan_wild, dim3((uint32_t)((ne + kBlock - 1) / kBlock)), dim3(kBlock), 0, 0, d.nbr,
                       (unsigned long long)ne, flag);
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpy(&hw, flag, 4, hipMemcpyDeviceToHost));
  } catch (...) {
    free_list(tmp);
    throw;
  }
  free_list(tmp);
  d.has_wild = hw ? 1 : 0;
  d.pad |= kCsrWildKnown;
}

#include "heights.inc"
#include "closure.inc"
#include "bidir.inc"
#include "labels.inc"
#include "aql.inc"
#include "resident.inc"

// Builds the device snapshot from `csrs` and replaces e.dev with it. A CSR with `adopt` set
// (delta re-link) is taken over without a copy, together with its index; bidir.inc reuses the
// derived structures of unchanged CSRs. Taken-over arrays join the new snapshot's allocation
// list only on success, so a failure frees nothing the previous snapshot still owns.
// device_upload in two steps (a Watch batch builds under the engine's shared lock, beside the
// checks of the current snapshot, and publishes under the exclusive one): device_build reads the
// current snapshot e.dev but never changes it — arrays it takes over are listed in `adopted`
// (pool arrays) and DeviceSnapshot::adopt_h (contiguous ones), and pass to the new snapshot only
// when device_publish swaps it in.
static DeviceSnapshot* device_build(Engine& e, std::vector<HostCSR>& csrs, bool delta, std::vector<void*>& adopted) {
  PhaseClock pc(delta ? "relink" : "upload");
  device_init(e);
  HIP_OK(hipSetDevice(e.device));
  pc.mark("init");
  Schema& sc = *e.schema;
  auto* ds = new DeviceSnapshot();
  try {
    std::vector<DevCSR> table;
    std::vector<CsrInfo> info;
    // (a partitioned engine's CSRs hold what this rank keeps — engine.hpp part_keep — already
    // filtered at ingest; a device CSR the caller loaded is filtered while it is copied)
    for (HostCSR& h : csrs) {
      DevCSR d{};
      d.n_rows = h.n_rows;
      d.is_ext = h.ext ? 1 : 0;
      uint64_t ne = h.dev_off ? h.n_edges : h.nbr.size();
      BaseCsr b{h.rel, h.stype, h.srel, h.ext, ne, 0};
      if (h.adopt) {
        d.off = h.dev_off;
        d.nbr = h.dev_nbr;
        d.cav = h.dev_cav;
        d.exp_us = h.dev_exp;
        for (const void* p : {(const void*)h.dev_off, (const void*)h.dev_nbr, (const void*)h.dev_cav,
                              (const void*)h.dev_exp})
          if (p) adopted.push_back(const_cast<void*>(p));
        ds->bytes += ((size_t)h.n_rows + 1) * 4 + ne * (h.ext ? 16 : 4);
        if (h.dev_mhash) {
          d.mhash = h.dev_mhash;
          d.mmask = h.mmask;
          d.has_wild = h.has_wild;
          b.mh_keys = h.mh_keys;
          adopted.push_back(const_cast<unsigned long long*>(h.dev_mhash));
          ds->bytes += (h.mmask + 1) * kBucketKeys * 8;
        } else if (!h.ext && h.srel == kEllipsis && want_mhash(e, ne)) {
          build_mhash(*ds, d, ne);
          b.mh_keys = ne;
        } else if (!h.ext && h.srel == kEllipsis && h.wild_known) {
          d.has_wild = h.has_wild;  // (an index-less CSR taken over or merged: its wildcard flag carried over)
          d.pad |= kCsrWildKnown;
        } else if (!h.ext && h.srel == kEllipsis) {
          scan_wild(e, d, ne);
        }
        table.push_back(d);
        info.push_back({ne, h.stype});
        ds->base.push_back(b);
        continue;
      }
      if (h.dev_off && e.part_world > 1) {  // partitioned graph: only the edges this rank keeps (partition.inc)
        const uint64_t loaded = ne;
        part_filter_device(e, *ds, h, d, ne);
        b.n_edges = ne;
        e.n_tuples -= std::min<uint64_t>(e.n_tuples, loaded - ne);  // (the engine counts what it holds)
        if (!h.ext && h.srel == kEllipsis && want_mhash(e, ne)) {
          build_mhash(*ds, d, ne);
          b.mh_keys = ne;
        } else if (!h.ext && h.srel == kEllipsis) {
          scan_wild(e, d, ne);
        }
        table.push_back(d);
        info.push_back({ne, h.stype});
        ds->base.push_back(b);
        continue;
      }
      uint32_t* off = dalloc<uint32_t>(ds->allocs, (size_t)h.n_rows + 1, &ds->bytes);
      uint32_t* nbr = dalloc<uint32_t>(ds->allocs, ne, &ds->bytes);
      if (h.dev_off) {
        HIP_OK(hipMemcpy(off, h.dev_off, ((size_t)h.n_rows + 1) * 4, hipMemcpyDeviceToDevice));
        if (ne) HIP_OK(hipMemcpy(nbr, h.dev_nbr, ne * 4, hipMemcpyDeviceToDevice));
      } else {
        HIP_OK(hipMemcpy(off, h.off.data(), h.off.size() * 4, hipMemcpyHostToDevice));
        if (ne) HIP_OK(hipMemcpy(nbr, h.nbr.data(), ne * 4, hipMemcpyHostToDevice));
      }
      d.off = off;
      d.nbr = nbr;
      if (h.ext) {
        uint32_t* cav = dalloc<uint32_t>(ds->allocs, ne, &ds->bytes);
        int64_t* ex = dalloc<int64_t>(ds->allocs, ne, &ds->bytes);
        if (ne) {
          HIP_OK(hipMemcpy(cav, h.cav.data(), ne * 4, hipMemcpyHostToDevice));
          HIP_OK(hipMemcpy(ex, h.exp_us.data(), ne * 8, hipMemcpyHostToDevice));
        }
        d.cav = cav;
        d.exp_us = ex;
      }
      // hashed membership index for plain direct-subject kinds (the check
      // "is this subject in the row" becomes one probe instead of a binary search)
      if (!h.ext && h.srel == kEllipsis && want_mhash(e, ne)) {
        build_mhash(*ds, d, ne);
        b.mh_keys = ne;
      } else if (!h.ext && h.srel == kEllipsis) {
        scan_wild(e, d, ne);
      }
      table.push_back(d);
      info.push_back({ne, h.stype});
      ds->base.push_back(b);
    }
    // the uploads, indexes and (a Watch batch) the merge are on the null stream: wait for those
    // only — a device-wide synchronisation would also wait for the check batches running on the
    // engine's non-blocking streams beside the build (config 5: ~55 us of a 0.29 ms Watch batch)
    pc.mark("csr_loop");
    // (a Watch batch does not wait here: what follows reads the merged arrays on the null stream
    // after the merge, or through a synchronous copy that waits for it; the publication waits for
    // the null stream before the snapshot is swapped in, device_apply_publish)
    static const bool dbg_csr_sync = debug_env("GCK_DEBUG_CSR_SYNC") != nullptr;
    if (!delta) HIP_OK(hipDeviceSynchronize());
    else if (dbg_csr_sync) spin_stream(e, nullptr);
    pc.mark("csr_sync");
    // link the node program to the CSR table
    std::vector<DevItem> items = sc.items;
    for (size_t i = 0; i < items.size(); ++i) {
      DevItem& it = items[i];
      if (it.kind != IT_KIND && it.kind != IT_ARROW) continue;
      uint16_t rel = sc.item_rel[i];
      for (size_t k = 0; k < csrs.size(); ++k) {
        const HostCSR& h = csrs[k];
        if (h.rel == rel && h.stype == it.stype && h.srel == it.srel) {
          (h.ext ? it.csr_ext : it.csr_plain) = (uint32_t)k;
        }
      }
    }
    std::vector<DevNode> nodes = sc.nodes;
    pc.mark("csrs");
    build_heights(e, *ds, nodes, items, table, info, adopted, delta);
    pc.mark("heights");
    build_bidir(e, *ds, nodes, items, table, info, adopted);
    pc.mark("bidir");
    build_labels(e, *ds, nodes, items, table, info);
    pc.mark("labels");
    for (size_t k = 0; k < ds->base.size(); ++k)  // indexes built for local probes (bidir.inc)
      if (table[k].mhash && !ds->base[k].mh_keys) ds->base[k].mh_keys = ds->base[k].n_edges;
    ds->table = table;
    ds->n_nodes = (uint32_t)nodes.size();
    ds->n_items = (uint32_t)items.size();
    ds->n_csrs = (uint32_t)table.size();
    ds->n_types = (uint32_t)sc.types.size();
    ds->n_rels = (uint32_t)sc.rels.size();
    // the program tables and the caveat-instance tables in one device block and one upload (a
    // synchronous copy each would cost a Watch batch ~20 us apiece)
    std::vector<uint32_t> counts(sc.types.size());
    for (size_t t = 0; t < counts.size(); ++t) counts[t] = e.interner[t].count;
    std::vector<uint8_t> cst(e.caveat_static);  // outcome under the stored context
    std::vector<uint32_t> crow(e.caveat_row);   // row of the per-call outcome table
    if (cst.empty()) {
      cst.push_back(1);
      crow.push_back(kNone);
    }
    std::vector<unsigned char> blob;
    auto put = [&](const void* src, size_t n) {
      const size_t o = (blob.size() + 255) & ~(size_t)255;
      blob.resize(o + std::max<size_t>(n, 1));
      if (n) std::memcpy(blob.data() + o, src, n);
      return o;
    };
    const size_t o_nodes = put(nodes.data(), nodes.size() * sizeof(DevNode));
    const size_t o_items = put(items.data(), items.size() * sizeof(DevItem));
    const size_t o_csrs = put(table.data(), table.size() * sizeof(DevCSR));
    const size_t o_counts = put(counts.data(), counts.size() * 4);
    const size_t o_cst = put(cst.data(), cst.size());
    const size_t o_crow = put(crow.data(), crow.size() * 4);
    const size_t o_cj = ds->cj_host.empty() ? 0 : put(ds->cj_host.data(), ds->cj_host.size());
    const size_t o_lj = ds->lj_host.empty() ? 0 : put(ds->lj_host.data(), ds->lj_host.size());
    std::vector<unsigned long long> hp(ds->hgt.size());  // heights array of each forward node
    for (size_t n = 0; n < hp.size(); ++n) hp[n] = (unsigned long long)(uintptr_t)ds->hgt[n];
    const size_t o_hgt = put(hp.data(), hp.size() * 8);
    unsigned char* d_blob = dalloc<unsigned char>(ds->allocs, blob.size(), &ds->bytes);
    if (delta) {
      // a Watch batch: from the engine's pinned blob buffer, on the null stream; complete before
      // the snapshot is published (device_apply_publish waits for the null stream)
      if (e.blob_host_cap < blob.size()) {
        if (e.blob_host) HIP_OK(hipHostFree(e.blob_host));
        e.blob_host = nullptr;
        e.blob_host_cap = 0;
        HIP_OK(hipHostMalloc(&e.blob_host, blob.size() * 2, hipHostMallocDefault));
        e.blob_host_cap = blob.size() * 2;
      }
      std::memcpy(e.blob_host, blob.data(), blob.size());
      HIP_OK(hipMemcpyAsync(d_blob, e.blob_host, blob.size(), hipMemcpyHostToDevice, nullptr));
    } else {
      HIP_OK(hipMemcpy(d_blob, blob.data(), blob.size(), hipMemcpyHostToDevice));
    }
    ds->nodes = reinterpret_cast<DevNode*>(d_blob + o_nodes);
    ds->items = reinterpret_cast<DevItem*>(d_blob + o_items);
    ds->csrs = reinterpret_cast<DevCSR*>(d_blob + o_csrs);
    ds->type_counts = reinterpret_cast<uint32_t*>(d_blob + o_counts);
    ds->cav_static = d_blob + o_cst;
    ds->n_cav = (uint32_t)cst.size();
    ds->cav_row = reinterpret_cast<uint32_t*>(d_blob + o_crow);
    ds->d_hgt = reinterpret_cast<const unsigned long long*>(d_blob + o_hgt);
    ds->d_cj = ds->cj_host.empty() ? nullptr : d_blob + o_cj;
    ds->d_lj = ds->lj_host.empty() ? nullptr : d_blob + o_lj;
    ds->node_bits = std::max<uint32_t>(1, ceil_log2(sc.nodes.size()));
    if (ds->node_bits > 12) throw Error(GCK_E_SCHEMA, "schema too large for the visited-key layout");
    ds->q_bits = 31 - ds->node_bits;
    // exact-depth layout (make_ctx): tag 2 bits, depth, node, query id below bit 63
    const uint32_t md = e.cfg.max_depth ? e.cfg.max_depth : 50;
    ds->q_bits_deep = 63 - (34 + ceil_log2((uint64_t)md + 1) + ds->node_bits);
    pc.mark("program");
  } catch (...) {
    free_list(ds->allocs);
    for (void* p : ds->hallocs) (void)hipFree(p);
    delete ds;
    throw;
  }
  return ds;
}

// sync_null false (a Watch publication, delta.inc device_apply_publish): the null stream's work is
// not waited for here — its readers are ordered behind the publication's event
static void device_publish(Engine& e, DeviceSnapshot* ds, std::vector<void*>& adopted, bool sync_null) {
  PhaseClock pc("publish");
  if (!ds->slot_patches.empty()) {  // (the batches in flight on the current snapshot have finished)
    for (const SlotPatch& sp : ds->slot_patches)
      if (sp.n)
        hipLaunchKernelGGL(k_slot_scatter, dim3(grid_for(sp.n)), dim3(kBlock), 0, 0, sp.slots, sp.staged, sp.ids, sp.n);
    HIP_OK(hipGetLastError());
    spin_stream(e, nullptr);
    ds->slot_patches.clear();
    pc.mark("slot_patch");
  }
  if (!ds->adopt_h.empty() && e.dev) {  // contiguous arrays taken over (label tables)
    auto& oh = e.dev->hallocs;
    for (void* q : ds->adopt_h) {
      auto it = std::find(oh.begin(), oh.end(), q);
      if (it != oh.end()) {
        oh.erase(it);
        ds->hallocs.push_back(q);
      } else {
        adopted.push_back(q);  // (a pool array)
      }
    }
    ds->adopt_h.clear();
  }
  if (!adopted.empty()) {
    std::sort(adopted.begin(), adopted.end());
    adopted.erase(std::unique(adopted.begin(), adopted.end()), adopted.end());
    if (e.dev) {  // the previous snapshot no longer owns what was taken over
      auto& old = e.dev->allocs;
      old.erase(std::remove_if(old.begin(), old.end(),
                               [&](void* p) { return std::binary_search(adopted.begin(), adopted.end(), p); }),
                old.end());
    }
    ds->allocs.insert(ds->allocs.end(), adopted.begin(), adopted.end());
  }
  if (e.dev) {
    // nothing uses the replaced arrays any more (checks and lookups are synchronous, and a
    // snapshot change holds the engine exclusively): return them to the pool on the engine's
    // own non-blocking stream, where a free costs a fraction of one on the legacy null stream,
    // which must order itself after every blocking stream
    const size_t n_free = e.dev->allocs.size();
    if (e.free_stream) {
      for (void* p : e.dev->allocs) retire_array(e, p, (hipStream_t)e.free_stream);
      e.dev->allocs.clear();
    } else {
      for (void* p : e.dev->allocs) e.recyclable.erase(p);
      free_list(e.dev->allocs);
    }
    pc.mark(n_free > 16 ? "free_many" : "free_few");
    if (!sync_null && !e.dev->hallocs.empty()) spin_stream(e, nullptr);  // (the build's kernels may read them)
    for (void* p : e.dev->hallocs) (void)hipFree(p);
    pc.mark(e.dev->hallocs.empty() ? "free_h0" : "free_h");
    delete e.dev;
  }
  pc.mark("retire");
  e.dev = ds;
  static std::atomic<uint64_t> g_generations{0};  // process-wide: a snapshot id never repeats
  e.generation = ++g_generations;
  if (sync_null) {
    HIP_OK(hipStreamSynchronize(nullptr));  // pool allocations are ordered on the null stream
    pc.mark("sync");
  }
}

void device_upload(Engine& e, std::vector<HostCSR>& csrs, bool delta) {
  std::vector<void*> adopted;
  DeviceSnapshot* ds = device_build(e, csrs, delta, adopted);
  device_publish(e, ds, adopted, true);
}

// ---- workspaces ------------------------------------------------------------------------------

static uint32_t device_cus(int device) {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    return (uint32_t)prop.multiProcessorCount;
  return 256;
}

// A workspace with its counters, staging and bundle scratch; the grid-wide and workgroup-bundle
// scratch follow on first use (ensure_wide / ensure_giant), since most batches never need them.
static Workspace* create_workspace(Engine& e) {
  HIP_OK(hipSetDevice(e.device));
  auto* w = new Workspace();
  try {
    const gck_config& cf = e.cfg;
    w->max_batch = cf.max_batch ? cf.max_batch : 65536;
    w->frontier_cap = cf.frontier_capacity ? cf.frontier_capacity : (size_t)16 << 20;
    w->seg_cap = cf.segment_capacity ? cf.segment_capacity : (size_t)8 << 20;
    w->query_cap = cf.query_capacity ? cf.query_capacity : std::max<size_t>((size_t)4 << 20, w->max_batch * 4);
    w->join_cap = std::max<size_t>(w->query_cap / 2, 1);
    uint64_t vc = cf.visited_capacity ? cf.visited_capacity : (1ull << 26);
    w->visited_cap = 1ull << ceil_log2(vc);
    w->frontier_cap = std::max(w->frontier_cap, w->max_batch);
    w->query_cap = std::max(w->query_cap, w->max_batch);
    if (w->frontier_cap > 0xFFFFFFF0ull || w->query_cap > 0x7FFFFFFFull)
      throw Error(GCK_E_INVALID_ARGUMENT, "workspace capacity too large");
    // the level / batch counters and the bundle counters share one buffer (one memset, one copy
    // back per batch)
    static_assert(sizeof(DevCounters) % 8 == 0, "bundle counters follow DevCounters");
    w->ctr = reinterpret_cast<DevCounters*>(dalloc<unsigned char>(w->allocs, sizeof(DevCounters) + kBCtrs * sizeof(unsigned), &w->bytes));
    w->b_ctrs = reinterpret_cast<unsigned*>(w->ctr + 1);
    w->d_items = dalloc<gck_item>(w->allocs, w->max_batch, &w->bytes);
    w->d_perm = dalloc<uint8_t>(w->allocs, w->max_batch, &w->bytes);
    w->d_err = dalloc<int32_t>(w->allocs, w->max_batch, &w->bytes);
    w->cav_flag = dalloc<uint8_t>(w->allocs, w->max_batch, &w->bytes);
    w->d_ctx = reinterpret_cast<Ctx*>(dalloc<unsigned char>(w->allocs, sizeof(Ctx), &w->bytes));
    HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&w->h_ctx), sizeof(Ctx), hipHostMallocDefault));
    HIP_OK(hipHostMalloc(&w->h_ctr, sizeof(DevCounters) + (kBCtrs + 4) * sizeof(unsigned),
                         hipHostMallocCoherent | hipHostMallocMapped));
    w->h_bctrs = reinterpret_cast<unsigned*>(w->h_ctr + 1);
    w->h_seq = w->h_bctrs + kBCtrs;
    *w->h_seq = 0;
    HIP_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&w->d_hpub), w->h_ctr, 0));
    // the block summaries of AQL-dispatched joins: one 8-B slot per block (>= 64 checks per block)
    w->n_slots = (uint32_t)(w->max_batch / 64 + 2);
    HIP_OK(hipHostMalloc(&w->h_slots, (size_t)w->n_slots * 8, hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(w->h_slots, 0, (size_t)w->n_slots * 8);
    HIP_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&w->d_slots), w->h_slots, 0));
    // pinned staging of host batches: 20 B of items in, 5 B of results out per check
    const size_t stage = w->max_batch * (sizeof(gck_item) + 1 + 4);
    void* hs = nullptr;
    HIP_OK(hipHostMalloc(&hs, stage, hipHostMallocDefault));
    w->h_items = static_cast<gck_item*>(hs);
    w->h_err = reinterpret_cast<int32_t*>(w->h_items + w->max_batch);
    w->h_perm = reinterpret_cast<uint8_t*>(w->h_err + w->max_batch);
    // bundle path scratch: per resident wavefront, a frontier pair and a visited table
    if (!(cf.flags & GCK_FLAG_NO_BUNDLE)) {
      const uint32_t cus = device_cus(e.device);
      // 8 resident bundle waves per CU with 32 checks each: the level latency of this gather-bound
      // loop grows with the requests in flight, so fewer, fuller waves finish a batch sooner
      // (config 4 sweep, profiles/r01/sweeps: 16 x 16 -> 250 M/s, 8 x 32 -> 323 M/s)
      const uint32_t wpc = cf.bundle_waves_per_cu ? cf.bundle_waves_per_cu : 8;
      w->b_checks = cf.bundle_checks ? std::min<uint32_t>(cf.bundle_checks, kBMax) : 32;
      w->b_fc = cf.bundle_frontier ? cf.bundle_frontier : 4096;
      w->b_vslots = 1u << ceil_log2(cf.bundle_visited ? cf.bundle_visited : 16384);
      w->b_blocks = std::max<uint32_t>(1, cus * wpc / kWaves);
      const size_t slots = (size_t)w->b_blocks * kWaves;
      w->b_fr = dalloc<unsigned long long>(w->allocs, slots * 2 * w->b_fc, &w->bytes);
      w->b_vis = dalloc<unsigned long long>(w->allocs, slots * w->b_vslots, &w->bytes);
      w->b_vlog = dalloc<uint32_t>(w->allocs, slots * w->b_vslots, &w->bytes);
      HIP_OK(hipMemsetAsync(w->b_vis, 0, slots * w->b_vslots * sizeof(unsigned long long), nullptr));
      w->b_deferred = dalloc<uint32_t>(w->allocs, w->max_batch, &w->bytes);
      w->c_deferred = dalloc<uint32_t>(w->allocs, w->max_batch, &w->bytes);
      w->b_budget = cf.bundle_budget ? cf.bundle_budget : 1024;
      w->g_fc = cf.giant_frontier ? cf.giant_frontier : 65536;
      w->g_vslots = 1u << ceil_log2(cf.giant_visited ? cf.giant_visited : 262144);
      w->g_slots = cf.giant_slots ? cf.giant_slots : cus;
      w->g_deferred = dalloc<uint32_t>(w->allocs, w->max_batch, &w->bytes);
      w->def_items = dalloc<gck_item>(w->allocs, w->max_batch, &w->bytes);
      w->def_perm = dalloc<uint8_t>(w->allocs, w->max_batch, &w->bytes);
      w->def_err = dalloc<int32_t>(w->allocs, w->max_batch, &w->bytes);
    }
    HIP_OK(hipMemsetAsync(w->ctr, 0, sizeof(DevCounters) + kBCtrs * sizeof(unsigned), nullptr));
    w->ctr_clean = true;
    HIP_OK(hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking));
    HIP_OK(hipEventCreate(&w->ev0));
    HIP_OK(hipEventCreate(&w->ev1));
    HIP_OK(hipEventCreate(&w->ev2));
    for (hipEvent_t& ev : w->pev) HIP_OK(hipEventCreate(&ev));
    HIP_OK(hipStreamSynchronize(nullptr));  // pool allocations are ordered on the null stream
  } catch (...) {
    free_workspace(w);
    throw;
  }
  return w;
}

// The grid-wide path's scratch (stage C, lookups' giant candidates, partitioned batches).
static void ensure_wide(Workspace& w) {
  if (w.wide_ready) return;
  w.checks = dalloc<DevCheck>(w.allocs, w.max_batch, &w.bytes);
  w.item_err = dalloc<int32_t>(w.allocs, w.max_batch, &w.bytes);
  w.queries = dalloc<DevQuery>(w.allocs, w.query_cap, &w.bytes);
  w.joins = dalloc<DevJoin>(w.allocs, w.join_cap, &w.bytes);
  w.fr[0] = dalloc<Entry>(w.allocs, w.frontier_cap, &w.bytes);
  w.fr[1] = dalloc<Entry>(w.allocs, w.frontier_cap, &w.bytes);
  w.segs = dalloc<Segment>(w.allocs, w.seg_cap, &w.bytes);
  w.visited = dalloc<unsigned long long>(w.allocs, w.visited_cap, &w.bytes);
  HIP_OK(hipStreamSynchronize(nullptr));  // pool allocations are ordered on the null stream
  w.wide_ready = true;
}

// The workgroup-bundle stage's scratch (stage B).
static void ensure_giant(Workspace& w) {
  if (w.giant_ready) return;
  w.g_fr = dalloc<unsigned long long>(w.allocs, (size_t)w.g_slots * 2 * w.g_fc, &w.bytes);
  w.g_vis = dalloc<unsigned long long>(w.allocs, (size_t)w.g_slots * w.g_vslots, &w.bytes);
  w.g_vlog = dalloc<uint32_t>(w.allocs, (size_t)w.g_slots * w.g_vslots, &w.bytes);
  HIP_OK(hipMemsetAsync(w.g_vis, 0, (size_t)w.g_slots * w.g_vslots * sizeof(unsigned long long), nullptr));
  HIP_OK(hipStreamSynchronize(nullptr));
  w.giant_ready = true;
}

// A free workspace of the pool (created while the pool holds fewer than cfg.workspaces;
// otherwise waits for one to be released). Call without holding the engine lock: the holders of
// busy workspaces may need it to finish their batches.
static size_t pool_cap(const Engine& e) { return e.cfg.workspaces ? e.cfg.workspaces : 4; }

// Every workspace of the pool, created up front (gck_commit_snapshot / gck_load_snapshot_file):
// a check never pays for creating one (~0.5 GB of scratch, pinned staging, a stream and its
// events, a synchronisation of the null stream) — the first `workspaces` concurrent batches
// would otherwise each pay it inside the caller's latency.
void ensure_pool(Engine& e) {
  if (e.part_world > 1) return;  // a partitioned engine runs on its own workspace (part_ws)
  std::lock_guard<std::mutex> lk(e.ws_mu);
  while (e.ws_pool.size() < pool_cap(e)) {
    Workspace* w = create_workspace(e);
    w->ws_index = (uint32_t)e.ws_pool.size();
    e.ws_pool.push_back(w);
  }
  if (!e.aql_tried) {
    e.aql_tried = true;
    e.aql = aql_init(e);
  }
  if (e.aql)
    for (Workspace* w : e.ws_pool) (void)aql_workspace(*e.aql, *w);  // (one without: its batches launch through HIP)
  if (!e.res_tried) {
    e.res_tried = true;
    e.res = res_init(e);
    res_start_keeper(e);
  }
}

// `want` (1 or 2) free workspaces of the pool, taken together: a caller never holds one while it
// waits for another (two callers each holding one and waiting for a second would deadlock a
// pool of two, and one caller would deadlock a pool of one). A pool of one serves `want` = 2
// with its single workspace (out[1] = out[0]). Workspaces missing from the pool (before
// ensure_pool) are created here. Call without holding the engine lock: the holders of busy
// workspaces may need it to finish their batches.
void acquire_ws_n(Engine& e, int want, Workspace** out) {
  const size_t cap = pool_cap(e);
  const size_t need = std::min<size_t>((size_t)want, cap);
  std::unique_lock<std::mutex> lk(e.ws_mu);
  for (;;) {
    std::vector<Workspace*> got;
    for (Workspace* w : e.ws_pool)
      if (!w->busy && got.size() < need) got.push_back(w);
    while (got.size() < need && e.ws_pool.size() < cap) {
      Workspace* w = create_workspace(e);
      w->ws_index = (uint32_t)e.ws_pool.size();
      e.ws_pool.push_back(w);
      got.push_back(w);
    }
    if (got.size() == need) {
      for (Workspace* w : got) w->busy = true;
      for (int k = 0; k < want; ++k) out[k] = got[std::min<size_t>((size_t)k, need - 1)];
      return;
    }
    e.ws_cv.wait(lk);
  }
}

Workspace* acquire_ws(Engine& e) {
  Workspace* w = nullptr;
  acquire_ws_n(e, 1, &w);
  return w;
}

void release_ws(Engine& e, Workspace* w) {
  {
    std::lock_guard<std::mutex> lk(e.ws_mu);
    w->busy = false;
  }
  e.ws_cv.notify_all();  // a two-workspace caller may be waiting beside one-workspace callers
}

// A Watch publication's null-stream work — the merge, the label tables, the membership-index
// patch — is not waited for (delta.inc device_apply_publish): every launch on the new snapshot is
// ordered after it on the GPU by its stream waiting for the publication's event (once per
// workspace, stream and publication). A join, which never probes the membership indexes, waits only
// for the work before the index patch (probes = false); the launches after it that may probe them
// wait for the patch too (wait_patch).
static void wait_patch(Engine& e, Workspace& w, hipStream_t st) {
  if (e.patch_seq && (w.patch_seen != e.patch_seq || w.patch_stream != (void*)st)) {
    HIP_OK(hipStreamWaitEvent(st, (hipEvent_t)e.patch_ev, 0));
    w.patch_seen = w.build_seen = e.patch_seq;
    w.patch_stream = w.build_stream = (void*)st;
  }
}
static Ctx make_ctx(Engine& e, Workspace& w, int64_t now_us, hipStream_t st, bool probes = true) {
  if (probes) {
    wait_patch(e, w, st);
  } else if (e.patch_seq && (w.build_seen != e.patch_seq || w.build_stream != (void*)st) &&
             (w.patch_seen != e.patch_seq || w.patch_stream != (void*)st)) {
    HIP_OK(hipStreamWaitEvent(st, (hipEvent_t)e.build_ev, 0));
    w.build_seen = e.patch_seq;
    w.build_stream = (void*)st;
  }
  DeviceSnapshot& ds = *e.dev;
  Ctx c{};
  c.nodes = ds.nodes;
  c.items = ds.items;
  c.csrs = ds.csrs;
  c.type_counts = ds.type_counts;
  c.n_types = ds.n_types;
  c.n_rels = ds.n_rels;
  c.n_nodes = ds.n_nodes;
  c.n_items = ds.n_items;
  c.n_csrs = ds.n_csrs;
  c.n_fwd = ds.n_fwd;
  c.checks = w.checks;
  c.queries = w.queries;
  c.joins = w.joins;
  c.segs = w.segs;
  c.visited = w.visited;
  c.vmask = w.visited_cap - 1;
  c.ctr = w.ctr;
  c.frontier_cap = (uint32_t)w.frontier_cap;
  c.seg_cap = (uint32_t)std::min<size_t>(w.seg_cap, (1u << 24) - 1);
  // a partitioned graph (world > 1) runs every check exact-depth (partition.inc): the deep layout
  const bool deep = ds.any_deep || e.part_world > 1;
  const uint32_t q_bits = deep ? ds.q_bits_deep : ds.q_bits;
  c.query_cap = (uint32_t)std::min<size_t>(w.query_cap, 1ull << q_bits);
  c.join_cap = (uint32_t)w.join_cap;
  c.q_hi = c.query_cap;
  c.j_hi = c.join_cap;
  c.force_exact = 0;
  c.part_sub = nullptr;
  c.max_depth = e.cfg.max_depth ? e.cfg.max_depth : 50;
  if (deep) {  // exact-depth checks key their entries by depth (make_key)
    const uint32_t db = ceil_log2((uint64_t)c.max_depth + 1);
    c.depth_shift = 34;
    c.depth_mask = (1u << db) - 1u;
    c.node_shift = 34 + db;
  } else {
    c.depth_shift = 0;
    c.depth_mask = 0;
    c.node_shift = 33;
  }
  c.q_shift = c.node_shift + ds.node_bits;
  c.hgt = ds.d_hgt;
  c.now_us = now_us;
  c.cav_static = ds.cav_static;
  c.cav_row = ds.cav_row;
  c.cav_dyn = w.cav_dyn;
  c.cav_slot = w.cav_slot;
  c.n_ctx = w.cav_on ? w.cav.n_ctx : 0u;
  c.n_dist = w.cav.n_dist;
  c.cav_keys = w.cav_lazy ? w.cav_keys : nullptr;
  c.cav_vals = w.cav_vals;
  c.cav_kmask = w.cav_map_cap ? w.cav_map_cap - 1 : 0;
  c.req_set = w.req_set;
  c.req_list = w.req_list;
  c.req_cnt = w.req_cnt;
  c.cav_flag = w.cav_flag;
  c.ck_map = nullptr;
  c.ck_off = 0;
  return c;
}

static void add_counters(Engine& e, Workspace& w, const DevCounters& h) {
  w.b_cav_req += h.cav_requests;
  w.b_cav_err += h.cav_errors;
  std::lock_guard<std::mutex> lk(e.stats_mu);
  e.stats.entries_expanded += h.expanded;
  e.stats.row_lookups += h.row_lookups;
  e.stats.membership_probes += h.probes;
  e.stats.edges_enumerated += h.edges;
  e.stats.ext_edges += h.ext_edges;
  e.stats.bidir_checks += h.bidir;
  e.stats.levels += h.bundle_levels;
  e.stats.bundles += h.bundles;
}

// Runs one batch (n <= max_batch) on the grid-wide path. Returns false on a workspace overflow
// (the caller splits the batch). Its check k is check map[k] (map null: pos + k) of the batch.
static bool run_batch(Engine& e, Workspace& w, const gck_item* d_items, uint32_t n, int64_t now_us,
                      uint8_t* d_perm, int32_t* d_err, hipStream_t st, float* ms_out, size_t pos,
                      const uint32_t* map) {
  ensure_wide(w);
  Ctx c = make_ctx(e, w, now_us, st);
  c.ck_items = d_items;
  c.ck_map = map;
  c.ck_off = map ? 0u : (uint32_t)pos;
  HIP_OK(hipEventRecord(w.ev0, st));
  w.ctr_clean = false;
  HIP_OK(hipMemsetAsync(w.ctr, 0, sizeof(DevCounters) + kBCtrs * sizeof(unsigned), st));
  HIP_OK(hipMemsetAsync(w.visited, 0xFF, w.visited_cap * sizeof(unsigned long long), st));
  DevCounters init{};
  init.n_queries = n;
  HIP_OK(hipMemcpyAsync(w.ctr, &init, sizeof(DevCounters), hipMemcpyHostToDevice, st));
  const uint32_t grid_n = (n + kBlock - 1) / kBlock;
  c.level = 0;
  hipLaunchKernelGGL(k_init, dim3(grid_n), dim3(kBlock), 0, st, c, d_items, n, w.fr[0], w.item_err);
  HIP_OK(hipGetLastError());

  const bool profile = (e.cfg.flags & GCK_FLAG_PROFILE) != 0;
  uint32_t n_cur = n;
  int cur = 0;
  const uint32_t level_cap = 64 * c.max_depth + 64;
  uint64_t levels = 0;
  for (uint32_t level = 0; n_cur > 0; ++level) {
    if (level > level_cap) throw Error(GCK_E_DEVICE, "level cap exceeded (engine invariant)");
    c.level = level;
    c.next = w.fr[cur ^ 1];
    if (profile) HIP_OK(hipEventRecord(w.pev[0], st));
    hipLaunchKernelGGL(k_expand, dim3((n_cur + kBlock - 1) / kBlock), dim3(kBlock), 0, st, c, w.fr[cur], n_cur);
    if (profile) HIP_OK(hipEventRecord(w.pev[1], st));
    hipLaunchKernelGGL(k_edges, dim3(2048), dim3(kBlock), 0, st, c);
    if (profile) HIP_OK(hipEventRecord(w.pev[2], st));
    hipLaunchKernelGGL(k_resolve, dim3(1024), dim3(kBlock), 0, st, c);
    if (profile) HIP_OK(hipEventRecord(w.pev[3], st));
    hipLaunchKernelGGL(k_level_end, dim3(1), dim3(1), 0, st, w.ctr);
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpyAsync(w.h_ctr, w.ctr, sizeof(DevCounters), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    if (profile) {
      float a = 0.f, b = 0.f, r = 0.f;
      HIP_OK(hipEventElapsedTime(&a, w.pev[0], w.pev[1]));
      HIP_OK(hipEventElapsedTime(&b, w.pev[1], w.pev[2]));
      HIP_OK(hipEventElapsedTime(&r, w.pev[2], w.pev[3]));
      std::lock_guard<std::mutex> lk(e.stats_mu);
      e.stats.expand_ms += a;
      e.stats.edges_ms += b;
      e.stats.resolve_ms += r;
      e.stats.expand_launches++;
      e.stats.edges_launches++;
    }
    if (w.h_ctr->overflow) return false;
    n_cur = w.h_ctr->last_next;
    cur ^= 1;
    ++levels;
  }
  hipLaunchKernelGGL(k_final, dim3(grid_n), dim3(kBlock), 0, st, w.queries, n, w.item_err, d_perm, d_err, w.ctr);
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(w.ev1, st));
  HIP_OK(hipMemcpyAsync(w.h_ctr, w.ctr, sizeof(DevCounters), hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  if (w.h_ctr->overflow & 31u) return false;
  if (w.h_ctr->overflow & 32u) throw Error(GCK_E_DEVICE, "engine invariant violated: undecided check");
  float ms = 0.f;
  HIP_OK(hipEventElapsedTime(&ms, w.ev0, w.ev1));
  *ms_out += ms;
  const DevCounters& h = *w.h_ctr;
  add_counters(e, w, h);
  std::lock_guard<std::mutex> lk(e.stats_mu);
  e.stats.levels += levels;
  e.stats.queries += h.n_queries;
  e.stats.joins += h.n_joins;
  e.stats.batches++;
  return true;
}

// map: the batch index of each of the n checks (null: they are the batch)
static void check_range_wide(Engine& e, Workspace& w, const gck_item* d_items, size_t n, int64_t now_us,
                             uint8_t* d_perm, int32_t* d_err, hipStream_t st, float* ms,
                             const uint32_t* map = nullptr) {
  size_t pos = 0;
  while (pos < n) {
    size_t len = std::min(n - pos, w.max_batch);
    while (!run_batch(e, w, d_items + pos, (uint32_t)len, now_us, d_perm + pos, d_err + pos, st, ms, pos,
                      map ? map + pos : nullptr)) {
      {
        std::lock_guard<std::mutex> lk(e.stats_mu);
        e.stats.retries++;
      }
      if (len == 1) throw Error(GCK_E_CAPACITY, "device workspace overflow on a single check");
      len = (len + 1) / 2;
    }
    pos += len;
  }
}

// Waits until k_publish has written batch `seq` to host memory: a spin on the coherent
// sequence word (no interrupt, no copy), with a periodic stream query so that a faulted or
// failed stream ends the wait with its error instead of spinning forever.
static void wait_published(Workspace& w, hipStream_t st, unsigned seq) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint64_t it = 1;; ++it) {
    if (__atomic_load_n(w.h_seq, __ATOMIC_ACQUIRE) == seq) return;
    // the stream is queried only once the batch has run for a millisecond (a query is a host
    // API call; a 64K batch takes ~0.15 ms)
    if ((it & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(1)) {
      const hipError_t q = hipStreamQuery(st);
      if (q == hipSuccess) {
        if (__atomic_load_n(w.h_seq, __ATOMIC_ACQUIRE) == seq) return;
        throw Error(GCK_E_DEVICE, "engine invariant violated: batch finished without publishing");
      }
      if (q != hipErrorNotReady) throw Error(GCK_E_DEVICE, std::string("HIP error: ") + hipGetErrorString(q));
    }
    __builtin_ia32_pause();
  }
}

// elapsed time of a published batch: its events are complete, though the runtime may not have
// marked them yet (synchronise only then)
static void elapsed_ms(float* out, hipEvent_t a, hipEvent_t b) {
  hipError_t r = hipEventElapsedTime(out, a, b);
  if (r == hipErrorNotReady) {
    HIP_OK(hipEventSynchronize(b));
    r = hipEventElapsedTime(out, a, b);
  }
  HIP_OK(r);
}

constexpr uint32_t kPubWords = (sizeof(DevCounters) + kBCtrs * sizeof(unsigned)) / 4;

static void publish_launch(Workspace& w, hipStream_t st) {
  const unsigned seq = ++w.pub_seq;
  hipLaunchKernelGGL(k_publish, dim3(1), dim3(64), 0, st, reinterpret_cast<unsigned*>(w.ctr), kPubWords, w.d_hpub,
                     w.d_hpub + kPubWords, seq);
  HIP_OK(hipGetLastError());
  w.b_seq = seq;
}

static BundleArgs bundle_args(Engine& e, Workspace& w, const gck_item* d_items, uint32_t n, uint8_t* d_perm,
                              int32_t* d_err) {
  BundleArgs a{};
  a.items = d_items;
  a.n = n;
  a.out_perm = d_perm;
  a.out_err = d_err;
  a.deferred = w.b_deferred;
  a.n_deferred = w.b_ctrs + 1;
  a.bundle_ctr = w.b_ctrs;
  a.B = w.b_checks;
  a.FC = w.b_fc;
  a.vmask = w.b_vslots - 1;
  a.fr_base = w.b_fr;
  a.vis_base = w.b_vis;
  a.vlog_base = w.b_vlog;
  static const bool dbg_on = debug_env("GCK_DEBUG_BUNDLE") != nullptr;
  if (dbg_on && !w.dbg) HIP_OK(hipMalloc(&w.dbg, (4 + kBQ * 6 + kBJ * 8) * 4));
  a.dbg = dbg_on ? w.dbg : nullptr;
  a.budget = w.b_budget;
  a.both = e.cfg.bidir_both ? e.cfg.bidir_both : 64;
  a.idx = nullptr;
  a.n_dev = nullptr;
  // GCK_DEBUG_TIMING=<file prefix>: per-bundle records (bundle.inc BundleArgs::timing) of both stages
  static const char* timing_env = debug_env("GCK_DEBUG_TIMING");
  // bundle records of stages A and B, then the closure join's per-wave records
  const size_t timing_words = (size_t)kTimingWords * (n + 1) * 2 +
                              std::max((size_t)kCjTimingWords * (n / 64 + 1), (size_t)kLjTimingWords * (n / 16 + 1));
  if (timing_env && w.timing_cap < timing_words) {
    if (w.timing) (void)hipFree(w.timing);
    w.timing = nullptr;
    HIP_OK(hipMalloc(&w.timing, timing_words * 8));
    w.timing_cap = timing_words;
  }
  a.timing = timing_env ? w.timing : nullptr;
  return a;
}

// The node program is staged in LDS when it fits (bundle.inc).
static bool program_in_lds(const Ctx& c) {
  const size_t prog_bytes = (size_t)c.n_csrs * sizeof(DevCSR) + (size_t)c.n_nodes * sizeof(DevNode) +
                            (size_t)c.n_items * sizeof(DevItem);
  return prog_bytes <= (size_t)kProgBytes;
}

static void launch_wave_bundles(Engine& e, Workspace& w, const Ctx& c, const BundleArgs& a, hipStream_t st) {
  const bool prog_lds = program_in_lds(c);
  // bidirectional instantiation only when the snapshot has an eligible permission (bidir.inc)
  const bool bd = e.dev->has_bidir;
  if (prog_lds && bd)
    hipLaunchKernelGGL((k_bundles<1, kLFWave, true, true>), dim3(w.b_blocks), dim3(bundle_block<1>()), 0, st, c, a);
  else if (prog_lds)
    hipLaunchKernelGGL((k_bundles<1, kLFWave, true, false>), dim3(w.b_blocks), dim3(bundle_block<1>()), 0, st, c, a);
  else if (bd)
    hipLaunchKernelGGL((k_bundles<1, kLFWave, false, true>), dim3(w.b_blocks), dim3(bundle_block<1>()), 0, st, c, a);
  else
    hipLaunchKernelGGL((k_bundles<1, kLFWave, false, false>), dim3(w.b_blocks), dim3(bundle_block<1>()), 0, st, c, a);
  HIP_OK(hipGetLastError());
}

// Stage A of a bundle batch (n <= max_batch): the persistent wave-bundle kernel over every
// check, then — for a host batch — the copy of the results into the pinned staging, and the
// publication the host spins on. Nothing waits here.
// The request check of host items that no join reads in place (include/gck.h: a context_slot
// beyond the call's contexts is GCK_E_INVALID_ARGUMENT).
static void slot_error(uint32_t i, uint32_t slot, uint32_t limit) {
  throw Error(GCK_E_INVALID_ARGUMENT, "item " + std::to_string(i) + ": context_slot " + std::to_string(slot) +
                                          " beyond the " + std::to_string(limit) + " contexts given");
}

static void validate_slots(const gck_item* items, uint32_t n, uint32_t limit) {
  for (uint32_t i = 0; i < n; ++i)
    if (items[i].context_slot > limit) slot_error(i, items[i].context_slot, limit);
}

// Stage A of a batch begins with the label join (labels.inc) rather than the closure join.
static bool label_join_on(const Engine& e) {
  const DeviceSnapshot& ds = *e.dev;
  return ds.d_lj && (!(ds.d_cj && !(e.cfg.flags & GCK_FLAG_NO_CLOSURE)) || ds.lj_preferred);
}

// An AQL-dispatched join reports through per-block summaries (closure.inc block_summary): its
// arguments point at the workspace's slots, and its deferred-list counter is one of two words that
// alternate per batch (b_ctrs[6 + (seq & 1)]; the join clears the other for the next batch).
static void aql_summaries(Workspace& w, uint32_t& coherent, unsigned*& h_out, unsigned*& clear, unsigned*& n_deferred,
                          uint32_t blocks) {
  if (blocks > w.n_slots) return;  // (kept on the last-block publication)
  const uint32_t e = w.pub_seq & 1u;
  coherent |= kPubBySignal;
  h_out = w.d_slots;
  n_deferred = w.b_ctrs + 6 + e;
  clear = w.b_ctrs + 6 + (e ^ 1u);
  w.b_sum_blocks = blocks;
}

// After the completion signal: the batch's counters from its blocks' summaries into the host copy
// the rest of the engine reads (*h_ctr, h_bctrs[4]); the device counters only when a block touched
// them (task rounds, probes, a bad context slot), read and cleared synchronously.
static void aql_collect(Workspace& w) {
  uint64_t* slot = reinterpret_cast<uint64_t*>(w.h_slots);
  uint32_t deferred = 0, touched = 0;
  for (uint32_t b = 0; b < w.b_sum_blocks; ++b) {
    const uint64_t v = slot[b];
    if (!v) continue;
    deferred += (uint32_t)v;
    touched |= (uint32_t)(v >> 32);
    slot[b] = 0;
  }
  std::memset(w.h_ctr, 0, sizeof(DevCounters) + kBCtrs * sizeof(unsigned));
  if (touched) {
    HIP_OK(hipMemcpy(w.h_ctr, w.ctr, sizeof(DevCounters), hipMemcpyDeviceToHost));
    HIP_OK(hipMemset(w.ctr, 0, sizeof(DevCounters)));
  }
  w.h_bctrs[4] = deferred;
}

// A uniform batch's join arguments (closure.inc CjArgs::pairs; labels.inc LjArgs): the pairs and
// the header in, the packed words out, and the items of the checks it leaves to the bundle stages
// written where those read them (the workspace's item array, which the batch runs on).
template <typename Args>
static void uniform_args(const Workspace& w, Args& j) {
  j.pairs = w.u_pairs;
  j.out_packed = w.u_packed;
  j.items_out = const_cast<gck_item*>(w.b_items);
  j.u_rp = w.u_rp;
  j.u_ss = w.u_ss;
  j.u_ctx = w.u_ctx;
  j.items = nullptr;
}

// The HSA queues do not see the HIP streams' order: a Watch publication's null-stream work (merge,
// label-table marks, program upload; delta.inc device_apply_build) completes before the first join
// dispatched into a queue on its snapshot. Every aql_dispatch of a check batch comes through here.
static void aql_after_build(Engine& e) {
  const uint64_t ps = e.patch_seq;
  if (ps && e.aql_patch_seen.load(std::memory_order_acquire) != ps) {
    spin_event((hipEvent_t)e.build_ev);
    e.aql_patch_seen.store(ps, std::memory_order_release);
  }
}

// Has the last publication's null-stream work completed (no wait)? A batch submitted before it has
// takes the HIP launch instead of the queue dispatch: its stream waits for that work on the device
// (make_ctx), where aql_after_build would hold the host — config 5 submits its check batch right
// after each Watch publication, and the host's spin on the merge cost its step 10-15 us.
static bool aql_build_done(Engine& e) {
  const uint64_t ps = e.patch_seq;
  if (!ps || e.aql_patch_seen.load(std::memory_order_acquire) == ps) return true;
  if (hipEventQuery((hipEvent_t)e.build_ev) != hipSuccess) return false;
  e.aql_patch_seen.store(ps, std::memory_order_release);
  return true;
}

static void bundles_launch(Engine& e, Workspace& w, const gck_item* d_items, uint32_t n, int64_t now_us,
                           uint8_t* d_perm, int32_t* d_err, hipStream_t st, bool host_out) {
  Ctx c = make_ctx(e, w, now_us, st, false);  // (the bundles below wait for the index patch: wait_patch)
  c.ck_items = d_items;
  BundleArgs a = bundle_args(e, w, d_items, n, d_perm, d_err);
  static const char* timing_env = debug_env("GCK_DEBUG_TIMING");
  if (timing_env) HIP_OK(hipMemsetAsync(w.timing, 0, w.timing_cap * 8, st));
  const bool ctr_was_clean = w.ctr_clean && !timing_env;
  if (!w.ctr_clean) HIP_OK(hipMemsetAsync(w.ctr, 0, sizeof(DevCounters) + kBCtrs * sizeof(unsigned), st));  // + b_ctrs
  w.ctr_clean = false;
  // GCK_FLAG_PROFILE: one event opens stage A, one closes it, on every 4th batch of the workspace
  // (each record is a host API call on the per-batch path)
  w.b_timed = (e.cfg.flags & GCK_FLAG_PROFILE) && (w.n_batches++ % 4 == 0);
  // the closure-join stage answers the nested-group checks it can (closure.inc); what it leaves is
  // counted in the published counters and bundled by bundles_finish, so the common batch is two
  // launches: the join and the publication
  const DeviceSnapshot& ds = *e.dev;
  const bool cj_ok = ds.d_cj && !(e.cfg.flags & GCK_FLAG_NO_CLOSURE);
  const bool lj = label_join_on(e);
  const bool cj = cj_ok && !lj;
  // the checks' caveat flags start cleared: by the label join with the caveat plane itself (an AQL
  // dispatch is not ordered after this stream's work), else here
  if (w.cav_on && !(lj && ds.lj_cav)) HIP_OK(hipMemsetAsync(w.cav_flag, 0, n, st));
  w.b_closure = cj || lj;
  w.b_label = lj;
  // chained: the wave bundles over the join's deferred list follow it in stage A, reading the
  // list's length on the device — no host round trip in the wait — when recent batches of the
  // engine left checks (a persistent bundle launch over an empty list costs a few microseconds,
  // the round trip tens; engine.hpp Engine::defer_recent)
  // (not with the resident join: its requests are posted to the running launch, and what they
  // leave is bundled after the wait like an AQL-dispatched join's)
  w.b_chained = w.b_closure && e.defer_recent.load(std::memory_order_relaxed) > 0 && !e.res;
  // the join publishes the batch itself unless something must follow it first: a host batch's
  // copies, the chained bundles, or — for a device batch on the engine's stream, whose caller has
  // no stream to order its reads after the kernel's end — the end-of-kernel L2 write-back
  // (k_publish after the join). (Publishing those from the join too, with the results written
  // through the L2, was measured slower — config 4, 8 in flight: 9.2 vs 10.3 G checks/s; every
  // wave waits for its write-through acknowledgements before its block arrives — and removed.)
  // a device batch on the engine's stream whose join runs alone (no events, no chained bundles, no
  // memset before it on the HIP stream) is dispatched into the engine's HSA queue (aql.inc): its
  // packet's release fence and completion signal end it, so it publishes itself, without k_publish
  // (a profiled batch is timed by its queue's dispatch timestamps; under a tracer that intercepts
  // the queues they are not the packet's own: GCK_AQL_TIMED=0 launches profiled batches through
  // HIP, timed by their events)
  static const bool aql_timed = !(getenv("GCK_AQL_TIMED") && atoi(getenv("GCK_AQL_TIMED")) == 0);
  // (a batch with check contexts: the label join with the caveat plane, whose Ctx travels in the
  // kernarg block and which clears the checks' caveat flags itself — nothing on the HIP stream)
  const bool aql_ok = w.b_own_stream && !host_out && !w.b_chained && ctr_was_clean && e.aql &&
                      w.aql_kernarg && (!w.cav_on || (lj && ds.lj_cav)) && (lj || cj) &&
                      ((aql_timed && e.aql->tick_hz) || !w.b_timed) && aql_build_done(e);
  w.b_aql = false;
  w.b_res = false;
  w.b_sum_blocks = 0;
  // (GCK_DEBUG_HIP_SELFPUB: an engine-stream batch launched through HIP publishes itself from its
  // last block as an AQL-dispatched one does — the dispatch-span attribution of tools/aql_span.sh;
  // its results are not written back before the publication, so only device readers may use them)
  static const bool dbg_selfpub = debug_env("GCK_DEBUG_HIP_SELFPUB") != nullptr;
  const bool self_pub = !host_out && !w.b_chained && (!w.b_own_stream || aql_ok || dbg_selfpub);
  const uint32_t coherent = 0u;  // (results are published by the kernel end's write-back)
  // the join into the HSA queue when aql_ok and the code object has this variant
  auto aql_try = [&](const char* name, const void* args, size_t bytes, uint32_t blocks) {
    if (!aql_ok) return false;
    const AqlKernel* k = aql_kernel(e.aql, name);
    if (!k) return false;
    aql_after_build(e);
    aql_dispatch(*e.aql, w, *k, args, bytes, blocks, w.b_timed);
    w.b_aql = true;
    return true;
  };
  if (lj) {
    // the label join (labels.inc): one round of slot lines per check; what it leaves goes to the
    // wave bundles through the same deferred list as the closure join's
    LjArgs j{};
    j.items = d_items;
    j.n = n;
    j.out_perm = d_perm;
    j.out_err = d_err;
    j.deferred = w.c_deferred;
    j.n_deferred = w.b_ctrs + 4;
    j.table = ds.d_lj;
    j.n_fwd = ds.n_fwd;
    j.table_bytes = (uint32_t)((ds.lj_host.size() + 3) & ~(size_t)3);
    j.o_meta = ds.lj_o_meta;
    j.dirty = ds.lj_dirty;
    j.dov = ds.lj_dov;
    j.csrs = ds.csrs;
    j.afp = ds.lj_afp;
    j.n_csrs = ds.n_csrs;
    j.afp_n = ds.lj_afp_n;
    j.cav_static = ds.cav_static;
    j.anc = ds.lj_anc;
    bool cl = false;
    const bool cav = ds.lj_cav && w.cav_on;  // caveated pairs decided under the check contexts (cav_state)
    if (cav) {
      // the dense outcome table and the instances in LDS when they fit (labels.inc LjCavLds)
      const uint32_t rows = w.cav.n_dist ? (uint32_t)(w.cav.dense.size() / w.cav.n_dist) : 0u;
      cl = !w.cav_lazy && ds.n_cav <= kLjCavInst && w.cav.dense.size() <= kLjCavDense && w.cav.n_ctx <= kLjCavCtx &&
           w.cav.n_dist <= 255 && rows < 0xFFFFu;
      j.cav_n = ds.n_cav;
      j.cav_rows = rows;
    }
    j.timing = a.timing ? a.timing + (size_t)kTimingWords * (n + 1) * 2 : nullptr;
    if (w.b_validate) {
      j.bad_slot = &w.ctr->bad_slot;
      j.slot_limit = w.cav.n_given;
    }
    if (w.u_join) uniform_args(w, j);
    if (self_pub) {  // self-published (see the closure join below)
      j.pub = reinterpret_cast<unsigned*>(w.ctr);
      j.pub_words = kPubWords;
      j.h_out = w.d_hpub;
      j.done = w.b_ctrs + kBDone;
      j.seq = ++w.pub_seq;
      j.coherent = coherent;
      w.b_seq = j.seq;
    }
    static const char* const lj_names[8] = {"void gck::k_label_join<24, 16u, 32u, false>(gck::LjArgs)",
                                            "void gck::k_label_join<24, 32u, 32u, false>(gck::LjArgs)",
                                            "void gck::k_label_join<32, 16u, 32u, false>(gck::LjArgs)",
                                            "void gck::k_label_join<32, 32u, 32u, false>(gck::LjArgs)",
                                            "void gck::k_label_join<24, 16u, 32u, true>(gck::LjArgs)",
                                            "void gck::k_label_join<24, 32u, 32u, true>(gck::LjArgs)",
                                            "void gck::k_label_join<32, 16u, 32u, true>(gck::LjArgs)",
                                            "void gck::k_label_join<32, 32u, 32u, true>(gck::LjArgs)"};
    const int v = (cl ? 4 : 0) + (ds.lj_bits == 24 ? 0 : 2) + (ds.lj_sw == 16 ? 0 : 1);
    const AqlKernel* ak = aql_ok ? aql_kernel(e.aql, lj_names[v]) : nullptr;
    if (cav && ak) {
      j.cx = static_cast<const Ctx*>(aql_extra(w));  // (written with the arguments)
    } else if (cav && e.aql && w.aql_kernarg && w.aql_devargs) {
      aql_put_extra(*e.aql, w, &c, sizeof(Ctx));  // (through the BAR into VRAM: no copy on the stream)
      j.cx = static_cast<const Ctx*>(aql_extra(w));
    } else if (cav) {
      *w.h_ctx = c;
      HIP_OK(hipMemcpyAsync(w.d_ctx, w.h_ctx, sizeof(Ctx), hipMemcpyHostToDevice, st));
      j.cx = w.d_ctx;
    }
    if (ak) {
      const uint32_t blocks = (n + 32u * kWaves - 1) / (32u * kWaves);
      if (j.h_out) aql_summaries(w, j.coherent, j.h_out, j.done, j.n_deferred, blocks);
      aql_after_build(e);
      aql_dispatch(*e.aql, w, *ak, &j, sizeof(j), blocks, w.b_timed,
                   cav ? &c : nullptr, cav ? sizeof(Ctx) : 0);
      w.b_aql = true;
    } else {
      lj_launch(ds, j, n, st, w.b_timed ? w.ev0 : nullptr, w.b_timed && !w.b_chained ? w.ev1 : nullptr, cl);
    }
  } else if (cj) {
    CjArgs j{};
    j.items = d_items;
    j.n = n;
    j.out_perm = d_perm;
    j.out_err = d_err;
    j.deferred = w.c_deferred;
    j.n_deferred = w.b_ctrs + 4;
    j.table = ds.d_cj;
    j.n_fwd = ds.n_fwd;
    j.n_desc = ds.cj_n_desc;
    j.n_types = ds.n_types;
    j.table_bytes = (uint32_t)((ds.cj_host.size() + 3) & ~(size_t)3);
    j.o_meta = ds.cj_o_meta;
    j.o_entries = ds.cj_o_entries;
    j.timing = a.timing ? a.timing + (size_t)kTimingWords * (n + 1) * 2 : nullptr;
    if (w.b_validate) {
      j.bad_slot = &w.ctr->bad_slot;
      j.slot_limit = w.cav.n_given;
    }
    if (w.u_join) uniform_args(w, j);
    // self-published as the label join (a host-side stream query or synchronisation per batch
    // instead costs ~10 us, 11 G -> 3-5 G checks/s)
    if (self_pub) {
      j.pub = reinterpret_cast<unsigned*>(w.ctr);
      j.pub_words = kPubWords;
      j.h_out = w.d_hpub;
      j.done = w.b_ctrs + kBDone;
      j.seq = ++w.pub_seq;
      j.coherent = coherent;
      w.b_seq = j.seq;
    }
    // a timed batch's events are the kernel's own start and stop (hipExtLaunchKernel), not markers
    // around its dispatch, so they agree with a profiler's kernel duration
    // 32 checks per wave where the slot entries are 24-bit and the table is small: each wave waits
    // for the slowest of 64 lines instead of 128 (solo launch 12.1-12.3 vs 12.8-12.9 us, the same
    // throughput, profiles/r02/sweep/cpw*)
    const bool small = j.table_bytes <= kCjLdsBytesSmall;
    const bool fast = ds.slot_bits == 24 && small;
    const uint32_t cpw = fast ? 32u : 64u;
    const dim3 grid((n + cpw * kWaves - 1) / (cpw * kWaves)), block(kBlock);
    // (a timed batch with chained bundles stops its clock after them: stage A is both)
    hipEvent_t e0 = w.b_timed ? w.ev0 : nullptr, e1 = w.b_timed && !w.b_chained ? w.ev1 : nullptr;
    struct {
      Ctx c;
      CjArgs j;
    } cj_args{c, j};  // (the kernarg segment: the two by-value parameters in order)
    static_assert(offsetof(decltype(cj_args), j) == 344, "k_closure_join kernarg layout (Ctx, CjArgs)");
    // (half slots: the first 32 B of each resource slot, closure.inc HALF)
    if (fast && aql_ok && j.h_out && aql_kernel(e.aql, "void gck::k_closure_join<24, 2048u, 32u, true>(gck::Ctx, gck::CjArgs)"))
      aql_summaries(w, cj_args.j.coherent, cj_args.j.h_out, cj_args.j.done, cj_args.j.n_deferred, grid.x);
    // the resident join (resident.inc) takes the request without a dispatch of its own
    const bool res_ok = fast && aql_ok && e.res && !w.b_timed && w.b_sum_blocks == grid.x &&
                        (cj_args.j.coherent & kPubBySignal);
    static const bool dbg_res = debug_env("GCK_DEBUG_RES") != nullptr;  // (why a batch did not go resident)
    if (dbg_res && e.res && !res_ok)
      std::fprintf(stderr, "[gck res] not resident: fast=%d aql_ok=%d own=%d host_out=%d chained=%d clean=%d cav=%d timed=%d sum=%u/%u pub=%u\n",
                   (int)fast, (int)aql_ok, (int)w.b_own_stream, (int)host_out, (int)w.b_chained, (int)ctr_was_clean,
                   (int)w.cav_on, (int)w.b_timed, w.b_sum_blocks, grid.x, cj_args.j.coherent);
    if (res_ok) {
      aql_after_build(e);
      res_post(e, w, cj_args.j, grid.x);
    } else if (fast && aql_try("void gck::k_closure_join<24, 2048u, 32u, true>(gck::Ctx, gck::CjArgs)", &cj_args,
                        sizeof(cj_args), grid.x)) {
    } else if (fast)
      hipExtLaunchKernelGGL((k_closure_join<24, kCjLdsBytesSmall, 32, true>), grid, block, 0, st, e0, e1, 0, c, j);
    else if (ds.slot_bits == 24)
      hipExtLaunchKernelGGL((k_closure_join<24, kCjLdsBytes>), grid, block, 0, st, e0, e1, 0, c, j);
    else if (small)
      hipExtLaunchKernelGGL((k_closure_join<32, kCjLdsBytesSmall>), grid, block, 0, st, e0, e1, 0, c, j);
    else
      hipExtLaunchKernelGGL((k_closure_join<32, kCjLdsBytes>), grid, block, 0, st, e0, e1, 0, c, j);
    HIP_OK(hipGetLastError());
  } else {
    wait_patch(e, w, st);
    if (w.b_timed) HIP_OK(hipEventRecord(w.ev0, st));
    launch_wave_bundles(e, w, c, a, st);
    if (w.b_timed) HIP_OK(hipEventRecord(w.ev1, st));
  }
  if (w.b_chained) {
    BundleArgs b = a;
    b.idx = w.c_deferred;
    b.n_dev = w.b_ctrs + 4;
    wait_patch(e, w, st);
    launch_wave_bundles(e, w, c, b, st);
    if (w.b_timed) HIP_OK(hipEventRecord(w.ev1, st));
  }
  if (host_out) {
    HIP_OK(hipMemcpyAsync(w.b_xperm, d_perm, n, hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(w.b_xerr, d_err, (size_t)n * 4, hipMemcpyDeviceToHost, st));
  }
  if (!w.b_aql && !w.b_res && (!self_pub || !w.b_closure)) publish_launch(w, st);
  static const bool dbg_res_any = debug_env("GCK_DEBUG_RES") != nullptr;
  if (dbg_res_any && e.res && !w.b_res)
    std::fprintf(stderr, "[gck res] batch n=%u not resident: lj=%d cj=%d aql_ok=%d aql=%d chained=%d clean=%d own=%d host_out=%d\n",
                 n, (int)lj, (int)cj, (int)aql_ok, (int)w.b_aql, (int)w.b_chained, (int)ctr_was_clean,
                 (int)w.b_own_stream, (int)host_out);
}

static void debug_dump(Engine& e, Workspace& w, uint32_t n);

constexpr uint32_t kChainLeftovers = 1;  // leftovers of a batch that make the next 16 chain their bundles

// Stages B and C of a bundle batch after stage A was published: the checks stage A deferred
// (giant, or rooted high enough to need exact depth) through the workgroup bundles and/or the
// grid-wide path, synchronously. Returns the device time of the batch.
static float bundles_finish(Engine& e, Workspace& w, const gck_item* d_items, uint32_t n, int64_t now_us,
                            uint8_t* d_perm, int32_t* d_err, hipStream_t st, bool host_out) {
  if (w.b_aql) aql_wait(*e.aql, w);  // (the kernel has ended: its publication is complete)
  if (w.b_res) res_wait(e, w);       // (the resident join has finished the request's last chunk)
  if ((w.b_aql || w.b_res) && w.b_sum_blocks) aql_collect(w);
  else wait_published(w, st, w.b_seq);
  add_counters(e, w, *w.h_ctr);
  w.ctr_clean = true;  // k_publish zeroed the device counters
  if (w.h_ctr->bad_slot) {  // (a zero-copy batch's join found a context slot out of range)
    const uint32_t i = 0xFFFFFFFFu - w.h_ctr->bad_slot;
    slot_error(i, i < n ? d_items[i].context_slot : 0u, w.cav.n_given);
  }
  const bool profile = w.b_timed;
  float ms = 0.f, bm = 0.f, gm = 0.f;
  if (w.b_timed && w.b_aql) ms = aql_elapsed_ms(*e.aql, w);  // (its queue's dispatch timestamps)
  else if (w.b_timed) elapsed_ms(&ms, w.ev0, w.ev1);
  bm = ms;
  const uint32_t n_cj = w.b_closure ? w.h_bctrs[4] : 0u;
  if (n_cj > n) throw Error(GCK_E_DEVICE, "engine invariant violated: closure-join deferred count");
  w.u_ncj = n_cj;
  if (w.b_closure) {
    // the join counts only its task-round checks (DevCounters::closure; usually none, so usually
    // no atomic): the rest of what it answered came from the slots
    const unsigned long long tasks = w.h_ctr->closure;
    if (tasks > n - n_cj) throw Error(GCK_E_DEVICE, "engine invariant violated: closure-join task count");
    std::lock_guard<std::mutex> lk(e.stats_mu);
    e.stats.closure_checks += n - n_cj;
    e.stats.slot_checks += n - n_cj - tasks;
    if (w.b_label) e.stats.label_checks += n - n_cj;
    if (w.b_aql) e.stats.aql_batches++;
    if (w.b_res) e.stats.resident_batches++;
  }
  // recent batches with leftovers make the next ones chain their bundles on the device (config 5
  // since the chain walk leaves ~0.4 per batch — documents whose own wildcard grant a Watch batch
  // changed — in ~70 % of its batches: chained, 419 M checks/s; finished here after the join's
  // own dispatch, 351-375 M, the bundles' launch and round trip inside the next publication)
  if (w.b_closure) {
    if (n_cj >= kChainLeftovers) e.defer_recent.store(16, std::memory_order_relaxed);
    else if (e.defer_recent.load(std::memory_order_relaxed) > 0) e.defer_recent.fetch_sub(1, std::memory_order_relaxed);
  }
  if (n_cj > 0 && !w.b_chained) {
    // the checks the closure join left: the wave bundles over its list (the publish zeroed the
    // count on the device: restore it first)
    Ctx c = make_ctx(e, w, now_us, st);
    c.ck_items = d_items;
    BundleArgs a = bundle_args(e, w, d_items, n, d_perm, d_err);
    a.idx = w.c_deferred;
    a.n_dev = w.b_ctrs + 4;
    w.h_seq[2] = n_cj;
    HIP_OK(hipMemcpyAsync(w.b_ctrs + 4, w.h_seq + 2, sizeof(unsigned), hipMemcpyHostToDevice, st));
    w.ctr_clean = false;
    if (w.b_timed) HIP_OK(hipEventRecord(w.ev0, st));
    launch_wave_bundles(e, w, c, a, st);
    if (w.b_timed) HIP_OK(hipEventRecord(w.ev1, st));
    if (host_out) {
      HIP_OK(hipMemcpyAsync(w.b_xperm, d_perm, n, hipMemcpyDeviceToHost, st));
      HIP_OK(hipMemcpyAsync(w.b_xerr, d_err, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    }
    publish_launch(w, st);
    wait_published(w, st, w.b_seq);
    add_counters(e, w, *w.h_ctr);
    w.ctr_clean = true;
    if (w.b_timed) {
      float am = 0.f;
      elapsed_ms(&am, w.ev0, w.ev1);
      ms += am;
      bm += am;
    }
  }
  const uint32_t n_def = w.h_bctrs[1];
  uint32_t n_def2 = n_def;
  const bool giant = !(e.cfg.flags & GCK_FLAG_NO_GIANT);
  if (n_def > n) throw Error(GCK_E_DEVICE, "engine invariant violated: deferred count");
  if (n_def > 0 && giant) {
    // stage B: giant checks, one 16-wave workgroup each, over stage A's deferred list (the
    // publish zeroed the deferred count on the device: restore it first)
    ensure_giant(w);
    Ctx c = make_ctx(e, w, now_us, st);
    c.ck_items = d_items;
    BundleArgs g = bundle_args(e, w, d_items, n, d_perm, d_err);
    g.idx = w.b_deferred;
    g.n_dev = w.b_ctrs + 1;
    g.deferred = w.g_deferred;
    g.n_deferred = w.b_ctrs + 3;
    g.bundle_ctr = w.b_ctrs + 2;
    g.B = 1;
    g.FC = w.g_fc;
    g.vmask = w.g_vslots - 1;
    g.budget = 0xFFFFFFFFu;
    g.fr_base = w.g_fr;
    g.vis_base = w.g_vis;
    g.vlog_base = w.g_vlog;
    g.dbg = nullptr;
    g.timing = g.timing ? g.timing + (size_t)kTimingWords * (n + 1) : nullptr;
    w.h_seq[1] = n_def;
    HIP_OK(hipMemcpyAsync(w.b_ctrs + 1, w.h_seq + 1, sizeof(unsigned), hipMemcpyHostToDevice, st));
    w.ctr_clean = false;
    if (w.b_timed) HIP_OK(hipEventRecord(w.ev0, st));
    if (program_in_lds(c))
      hipLaunchKernelGGL((k_bundles<kGiantWaves, kLFGiant, true, false>), dim3(w.g_slots),
                         dim3(bundle_block<kGiantWaves>()), 0, st, c, g);
    else
      hipLaunchKernelGGL((k_bundles<kGiantWaves, kLFGiant, false, false>), dim3(w.g_slots),
                         dim3(bundle_block<kGiantWaves>()), 0, st, c, g);
    HIP_OK(hipGetLastError());
    if (w.b_timed) HIP_OK(hipEventRecord(w.ev1, st));
    publish_launch(w, st);
    wait_published(w, st, w.b_seq);
    add_counters(e, w, *w.h_ctr);
    w.ctr_clean = true;
    if (w.b_timed) elapsed_ms(&gm, w.ev0, w.ev1);
    ms += gm;
    n_def2 = w.h_bctrs[3];
    if (n_def2 > n_def) throw Error(GCK_E_DEVICE, "engine invariant violated: deferred count");
  }
  debug_dump(e, w, n);
  {
    std::lock_guard<std::mutex> lk(e.stats_mu);
    if (profile) {
      e.stats.bundle_ms += bm;
      e.stats.giant_ms += gm;
      e.stats.bundle_launches++;
    }
    e.stats.queries += n;
    e.stats.batches++;
    e.stats.deferred += n_def;
    e.stats.deferred_wide += n_def2;
  }
  if (n_def == 0) return ms;
  if (n_def2 > 0) {
    // stage C: the grid-wide level-synchronous path for what outgrew a workgroup bundle or
    // needs exact depth
    const uint32_t* def_idx = giant ? w.g_deferred : w.b_deferred;
    const uint32_t grid = (n_def2 + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_gather, dim3(grid), dim3(kBlock), 0, st, d_items, def_idx, n_def2, w.def_items);
    HIP_OK(hipGetLastError());
    check_range_wide(e, w, w.def_items, n_def2, now_us, w.def_perm, w.def_err, st, &ms, def_idx);
    hipLaunchKernelGGL(k_scatter, dim3(grid), dim3(kBlock), 0, st, def_idx, n_def2, w.def_perm, w.def_err, d_perm,
                       d_err);
    HIP_OK(hipGetLastError());
  }
  if (host_out) {  // the deferred checks' results, in place
    HIP_OK(hipMemcpyAsync(w.b_xperm, d_perm, n, hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(w.b_xerr, d_err, (size_t)n * 4, hipMemcpyDeviceToHost, st));
  }
  HIP_OK(hipStreamSynchronize(st));
  return ms;
}

// GCK_DEBUG_BUNDLE: bundle 0's final query / join tables; GCK_DEBUG_TIMING: both stages'
// per-bundle records appended to <prefix>.bin (kTimingWords u64 each).
static void debug_dump(Engine& e, Workspace& w, uint32_t n) {
  static const bool dbg_on = debug_env("GCK_DEBUG_BUNDLE") != nullptr;
  static const char* timing_env = debug_env("GCK_DEBUG_TIMING");
  if (dbg_on && w.dbg) {
    HIP_OK(hipDeviceSynchronize());
    const size_t dbg_words = 4 + kBQ * 6 + kBJ * 8;
    std::vector<uint32_t> h(dbg_words);
    HIP_OK(hipMemcpy(h.data(), w.dbg, dbg_words * 4, hipMemcpyDeviceToHost));
    fprintf(stderr, "[gck bundle0] queries=%u joins=%u overflow=%u epoch=%u\n", h[0], h[1], h[2], h[3]);
    for (uint32_t k = 0; k < h[0] && k < (uint32_t)kBQ; ++k) {
      const uint32_t* d = h.data() + 4 + k * 6;
      fprintf(stderr, "  q%-3u flags=%#x res=%u pending=%d last_alive=%u parent_join=%d operand=%u check=%u\n", k,
              d[0], (d[0] >> 8) & 0xF, (int)d[1], d[2], (int)d[3], d[4], d[5]);
    }
    for (uint32_t k = 0; k < h[1] && k < (uint32_t)kBJ; ++k) {
      const uint32_t* d = h.data() + 4 + kBQ * 6 + k * 8;
      fprintf(stderr, "  j%-3u parent=%u first=%u n=%u op=%u cond=%u state=%#x remaining=%d\n", k, d[0], d[1], d[2],
              d[3], d[4], d[5], (int)d[6]);
    }
  }
  if (timing_env && w.timing) {
    HIP_OK(hipDeviceSynchronize());  // (a closure join publishes its batch before its last waves end)
    const size_t timing_words = (size_t)kTimingWords * (n + 1) * 2;
    const size_t cj_words = std::max((size_t)kCjTimingWords * (n / 64 + 1), (size_t)kLjTimingWords * (n / 16 + 1));
    std::vector<unsigned long long> h(timing_words + cj_words);
    HIP_OK(hipMemcpy(h.data(), w.timing, (timing_words + cj_words) * 8, hipMemcpyDeviceToHost));
    std::string path = std::string(timing_env) + ".bin";
    if (FILE* f = fopen(path.c_str(), "ab")) {
      unsigned long long hdr[4] = {0xB0DDull, n, w.b_checks, w.h_bctrs[1]};
      fwrite(hdr, 8, 4, f);
      fwrite(h.data(), 8, timing_words, f);
      fclose(f);
    }
    if (w.b_label) {  // the label join's per-wave records: <prefix>_lj.bin
      std::string lpath = std::string(timing_env) + "_lj.bin";
      if (FILE* f = fopen(lpath.c_str(), "ab")) {
        const unsigned long long waves = (n + 31) / 32;
        unsigned long long hdr[2] = {0x1AB0ull, waves};
        fwrite(hdr, 8, 2, f);
        fwrite(h.data() + timing_words, 8, (size_t)kLjTimingWords * waves, f);
        fclose(f);
      }
    } else if (w.b_closure) {  // the closure join's per-wave records: <prefix>_cj.bin
      std::string cpath = std::string(timing_env) + "_cj.bin";
      if (FILE* f = fopen(cpath.c_str(), "ab")) {
        unsigned long long hdr[2] = {0xC10Cull, (n + 63) / 64};
        fwrite(hdr, 8, 2, f);
        fwrite(h.data() + timing_words, 8, (size_t)kCjTimingWords * ((n + 63) / 64), f);
        fclose(f);
      }
    }
  }
  (void)e;
}

static int64_t wall_now_us() {
  using namespace std::chrono;
  return duration_cast<microseconds>(system_clock::now().time_since_epoch()).count();
}

// ---- check-time caveat contexts (engine.hpp CavCall) -----------------------------------------

__global__ void k_cav_fail(const uint8_t* flag, uint32_t n, uint8_t* perm, int32_t* err) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && flag[i]) {
    perm[i] = GCK_PERM_UNSPECIFIED;
    err[i] = GCK_ITEM_ERR_CAVEAT_EVAL;
  }
}

template <class T>
static void grow(Workspace& w, T*& p, size_t& cap, size_t want) {
  if (cap >= want) return;
  if (p) {
    HIP_OK(hipDeviceSynchronize());
    w.allocs.erase(std::remove(w.allocs.begin(), w.allocs.end(), (void*)p), w.allocs.end());
    HIP_OK(hipFree(p));
    p = nullptr;
    w.bytes -= cap * sizeof(T);
  }
  cap = std::max(want, cap * 2);
  HIP_OK(hipMalloc(&p, cap * sizeof(T)));
  w.allocs.push_back(p);
  w.bytes += cap * sizeof(T);
}

// Uploads the lazy map: every pair evaluated so far, open addressing at most half full.
static void upload_cav_map(Workspace& w, hipStream_t st) {
  size_t cap = 1024;
  while (cap < 2 * w.cav_eval.size()) cap *= 2;
  if (w.cav_map_alloc < cap) {
    size_t kc = w.cav_map_alloc, vc = w.cav_map_alloc;
    grow(w, w.cav_keys, kc, cap);
    grow(w, w.cav_vals, vc, cap);
    w.cav_map_alloc = std::min(kc, vc);
  }
  w.cav_map_cap = cap;
  std::vector<unsigned long long> keys(cap, kEmptyKey);
  std::vector<uint8_t> vals(cap, 0);
  for (const auto& kv : w.cav_eval) {
    uint64_t h = mix64(kv.first) & (cap - 1);
    while (keys[h] != kEmptyKey) h = (h + 1) & (cap - 1);
    keys[h] = kv.first;
    vals[h] = kv.second;
  }
  // pageable sources: complete when the calls return
  HIP_OK(hipMemcpyAsync(w.cav_keys, keys.data(), cap * 8, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(w.cav_vals, vals.data(), cap, hipMemcpyHostToDevice, st));
  HIP_OK(hipStreamSynchronize(st));
}

// Stages the call's caveat contexts on the workspace: the dense table, or an empty lazy map
// and a clear request set.
static void stage_caveats(Workspace& w, CavCall&& call, hipStream_t st) {
  w.cav = std::move(call);
  w.cav_on = w.cav.n_ctx > 0;
  w.cav_lazy = w.cav_on && w.cav.dense.empty();
  w.cav_eval.clear();
  w.cav_parsed.clear();
  if (!w.cav_on) return;
  if (!w.cav_lazy) {
    if (w.cav.dense == w.cav_dyn_up && w.cav.of_slot == w.cav_slot_up) return;  // (on the device already)
    w.cav_dyn_up.clear();
    w.cav_slot_up.clear();
    grow(w, w.cav_dyn, w.cav_dyn_cap, w.cav.dense.size());
    grow(w, w.cav_slot, w.cav_slot_cap, w.cav.of_slot.size());
    // pageable sources: complete when the calls return
    HIP_OK(hipMemcpyAsync(w.cav_dyn, w.cav.dense.data(), w.cav.dense.size(), hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(w.cav_slot, w.cav.of_slot.data(), w.cav.of_slot.size() * 4, hipMemcpyHostToDevice, st));
    HIP_OK(hipStreamSynchronize(st));
    w.cav_dyn_up = w.cav.dense;
    w.cav_slot_up = w.cav.of_slot;
    return;
  }
  if (!w.req_set) {
    w.req_set = dalloc<unsigned long long>(w.allocs, kReqSet, &w.bytes);
    w.req_list = dalloc<unsigned long long>(w.allocs, kReqCap, &w.bytes);
    w.req_cnt = dalloc<unsigned>(w.allocs, 1, &w.bytes);
    HIP_OK(hipStreamSynchronize(nullptr));  // the allocations are ordered on the null stream
  }
  HIP_OK(hipMemsetAsync(w.req_set, 0xFF, (size_t)kReqSet * 8, st));
  HIP_OK(hipMemsetAsync(w.req_cnt, 0, 4, st));
  upload_cav_map(w, st);
}

// Evaluates the recorded pairs (row << 32 | slot) on the host, parsing the contexts they need
// first (a malformed one fails the call); an evaluation error is outcome 3.
static void evaluate_pairs(Engine& e, Workspace& w, const std::vector<unsigned long long>& keys) {
  std::vector<uint32_t> need;
  for (unsigned long long k : keys) {
    const uint32_t slot = (uint32_t)k;
    if (!w.cav_parsed.count(slot)) need.push_back(slot);
  }
  std::sort(need.begin(), need.end());
  need.erase(std::unique(need.begin(), need.end()), need.end());
  std::vector<cel::Object> parsed(need.size());
  const std::string& text = *w.cav.text;
  const std::vector<uint32_t>& off = *w.cav.off;
  host_parallel(need.size(), 512, [&](size_t lo, size_t hi) {
    for (size_t k = lo; k < hi; ++k) {
      const uint32_t s = need[k];
      parsed[k] = cel::parse_context(text.substr(off[s - 1], off[s] - off[s - 1]));
    }
  });
  for (size_t k = 0; k < need.size(); ++k) w.cav_parsed.emplace(need[k], std::move(parsed[k]));
  std::vector<uint8_t> out(keys.size());
  host_parallel(keys.size(), 256, [&](size_t lo, size_t hi) {
    for (size_t k = lo; k < hi; ++k) {
      const uint32_t row = (uint32_t)(keys[k] >> 32), slot = (uint32_t)keys[k];
      const uint32_t id = e.caveat_partial[row];
      const cel::Object& ctx = w.cav_parsed.at(slot);
      try {
        out[k] = (uint8_t)cel::evaluate(*e.caveat_expr[id], &e.caveat_ctx[id], &ctx);
      } catch (const Error&) {
        out[k] = 3;
      }
    }
  });
  const size_t n = keys.size();
  for (size_t k = 0; k < n; ++k) w.cav_eval[keys[k]] = out[k];
  std::lock_guard<std::mutex> lk(e.stats_mu);
  e.stats.caveat_evals += n;
}

// ---- batches ---------------------------------------------------------------------------------
//
// A batch is started by submit_batch (everything is queued, nothing waited for) and completed by
// finish_batch (stage A waited for, the later stages run, a host batch's results copied out of
// the pinned staging). The synchronous entry points are the two back to back; gck_check_submit /
// gck_check_wait expose them separately so that the next batch is queued while this one runs.

// Is [p, p + bytes) inside one pinned host buffer of this engine (gck_host_alloc)?
static bool host_pinned(Engine& e, const void* p, size_t bytes) {
  std::lock_guard<std::mutex> lk(e.host_mu);
  if (e.host_bufs.empty()) return false;
  const uintptr_t a = (uintptr_t)p;
  auto it = e.host_bufs.upper_bound(a);
  if (it == e.host_bufs.begin()) return false;
  --it;
  return a >= it->first && a + bytes <= it->first + it->second;
}

void* host_alloc(Engine& e, size_t bytes) {
  HIP_OK(hipSetDevice(e.cfg.device));
  void* p = nullptr;
  HIP_OK(hipHostMalloc(&p, std::max<size_t>(bytes, 1), hipHostMallocDefault));
  std::lock_guard<std::mutex> lk(e.host_mu);
  e.host_bufs[(uintptr_t)p] = bytes;
  return p;
}

void host_free(Engine& e, void* p) {
  {
    std::lock_guard<std::mutex> lk(e.host_mu);
    auto it = e.host_bufs.find((uintptr_t)p);
    if (it == e.host_bufs.end()) throw Error(GCK_E_INVALID_ARGUMENT, "not a gck_host_alloc buffer of this engine");
    e.host_bufs.erase(it);
  }
  HIP_OK(hipHostFree(p));
}

void host_free_all(Engine& e) {
  std::lock_guard<std::mutex> lk(e.host_mu);
  for (auto& kv : e.host_bufs) (void)hipHostFree(reinterpret_cast<void*>(kv.first));
  e.host_bufs.clear();
}

static void submit_batch(Engine& e, Workspace& w, const gck_item* items, uint32_t n, int64_t now_us, uint8_t* perm,
                         int32_t* err, hipStream_t st, bool host, bool own_stream = false, bool uniform_join = false) {
  w.u_join = uniform_join;  // (the join's arguments: bundles_launch)
  w.u_on = false;           // (submit_uniform sets it after this)
  w.b_own_stream = own_stream;
  w.b_n = n;
  w.b_now = now_us;
  w.b_st = host ? w.stream : st;
  w.b_hperm = host ? perm : nullptr;
  w.b_herr = host ? err : nullptr;
  w.b_items = host ? w.d_items : items;
  w.b_dperm = host ? w.d_perm : perm;
  w.b_derr = host ? w.d_err : err;
  w.b_ms = 0.f;
  w.b_cav_req = w.b_cav_err = 0;
  w.fail_code = 0;
  w.fail_msg.clear();
  // host batches on the AQL path (a snapshot with a one-round join): zero-copy — the join reads
  // the items from and writes the results into pinned host memory across PCIe (the caller's
  // gck_host_alloc buffers, or the workspace's staging), so a batch is one packet (no copy-engine
  // transfers, no runtime calls); its later stages, if any, do the same. Without the AQL path
  // (GCK_AQL=0, a profiled batch): the DMA path below.
  w.b_copy_perm = nullptr;
  w.b_copy_err = nullptr;
  w.b_validate = false;
  const bool join = label_join_on(e) || (e.dev->d_cj && !(e.cfg.flags & GCK_FLAG_NO_CLOSURE));
  if (host && e.aql && w.aql_kernarg && !w.cav_on && !(e.cfg.flags & (GCK_FLAG_PROFILE | GCK_FLAG_NO_BUNDLE)) &&
      join) {
    // the join reads every item once, in place: it also checks the context slots (no host pass
    // over the items on the submitting thread)
    w.b_validate = true;
    const bool pin_in = host_pinned(e, items, (size_t)n * sizeof(gck_item));
    const bool pin_out = host_pinned(e, perm, n) && host_pinned(e, err, (size_t)n * 4);
    // pageable buffers go through the workspace's pinned staging — one host copy each way — and
    // the batch is zero-copy over the staging (no copy engine, no runtime call)
    if (!pin_in) std::memcpy(w.h_items, items, (size_t)n * sizeof(gck_item));
    host = false;
    w.b_own_stream = true;
    w.b_hperm = nullptr;
    w.b_herr = nullptr;
    w.b_items = pin_in ? items : w.h_items;
    w.b_dperm = pin_out ? perm : w.h_perm;
    w.b_derr = pin_out ? err : w.h_err;
    if (!pin_out) {
      w.b_copy_perm = perm;
      w.b_copy_err = err;
    }
  }
  if (host) {
    validate_slots(items, n, w.cav.n_given);
    // items: a DMA straight from the caller's buffer when it is pinned (gck_host_alloc), else
    // through the workspace's pinned staging (one host copy, one DMA); results likewise
    if (host_pinned(e, items, (size_t)n * sizeof(gck_item))) {
      HIP_OK(hipMemcpyAsync(w.d_items, items, (size_t)n * sizeof(gck_item), hipMemcpyHostToDevice, w.b_st));
    } else {
      std::memcpy(w.h_items, items, (size_t)n * sizeof(gck_item));
      HIP_OK(hipMemcpyAsync(w.d_items, w.h_items, (size_t)n * sizeof(gck_item), hipMemcpyHostToDevice, w.b_st));
    }
    const bool pin_out = host_pinned(e, perm, n) && host_pinned(e, err, (size_t)n * 4);
    w.b_xperm = pin_out ? perm : w.h_perm;
    w.b_xerr = pin_out ? err : w.h_err;
  }
  w.b_bundles = !(e.cfg.flags & GCK_FLAG_NO_BUNDLE);
  if (w.cav_on && !w.b_bundles) HIP_OK(hipMemsetAsync(w.cav_flag, 0, n, w.b_st));  // (bundles_launch: its own)
  if (w.b_bundles) bundles_launch(e, w, w.b_items, n, now_us, w.b_dperm, w.b_derr, w.b_st, host);
  w.state = 1;
}

// The rest of a pass whose stage A is queued (bundle path), or the whole pass (grid-wide path).
static float finish_pass(Engine& e, Workspace& w) {
  const bool host = w.b_hperm != nullptr;
  if (w.b_bundles) return bundles_finish(e, w, w.b_items, w.b_n, w.b_now, w.b_dperm, w.b_derr, w.b_st, host);
  float ms = 0.f;
  check_range_wide(e, w, w.b_items, w.b_n, w.b_now, w.b_dperm, w.b_derr, w.b_st, &ms);
  if (host) {
    HIP_OK(hipMemcpyAsync(w.b_xperm, w.b_dperm, w.b_n, hipMemcpyDeviceToHost, w.b_st));
    HIP_OK(hipMemcpyAsync(w.b_xerr, w.b_derr, (size_t)w.b_n * 4, hipMemcpyDeviceToHost, w.b_st));
    HIP_OK(hipStreamSynchronize(w.b_st));
  }
  return ms;
}

// Lazy caveat evaluation after a pass: while the pass met pairs not evaluated yet, evaluate the
// ones it recorded and run the batch again (the walk of every check is repeated; a pass that
// sees only evaluated pairs is exact). Then the checks that touched a failing pair get their
// item error.
static void caveat_passes(Engine& e, Workspace& w) {
  const hipStream_t st = w.b_st;
  for (uint32_t pass = 0; w.cav_lazy && w.b_cav_req > 0; ++pass) {
    // each pass evaluates at least one new pair (one a pass met unevaluated is recorded unless
    // the list is full, and a full list holds kReqCap new pairs)
    if (pass > 4096) throw Error(GCK_E_DEVICE, "engine invariant violated: caveat passes do not settle");
    unsigned cnt = 0;
    HIP_OK(hipMemcpyAsync(&cnt, w.req_cnt, 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    cnt = std::min(cnt, kReqCap);
    if (cnt == 0) throw Error(GCK_E_DEVICE, "engine invariant violated: caveat pairs met but none recorded");
    std::vector<unsigned long long> keys(cnt);
    HIP_OK(hipMemcpyAsync(keys.data(), w.req_list, (size_t)cnt * 8, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    for (unsigned long long k : keys) {
      const uint32_t row = (uint32_t)(k >> 32), slot = (uint32_t)k;
      if (row >= e.caveat_partial.size() || slot == 0 || slot > w.cav.n_ctx || w.cav_eval.count(k))
        throw Error(GCK_E_DEVICE, "engine invariant violated: caveat pair request");
    }
    evaluate_pairs(e, w, keys);
    HIP_OK(hipMemsetAsync(w.req_set, 0xFF, (size_t)kReqSet * 8, st));
    HIP_OK(hipMemsetAsync(w.req_cnt, 0, 4, st));
    HIP_OK(hipMemsetAsync(w.cav_flag, 0, w.b_n, st));
    upload_cav_map(w, st);  // (ends with a synchronisation: the pass may be dispatched into an HSA queue)
    w.b_cav_req = w.b_cav_err = 0;
    if (w.b_bundles)
      bundles_launch(e, w, w.b_items, w.b_n, w.b_now, w.b_dperm, w.b_derr, st, w.b_hperm != nullptr);
    w.b_ms += finish_pass(e, w);
    std::lock_guard<std::mutex> lk(e.stats_mu);
    e.stats.caveat_passes++;
  }
  if (w.b_cav_err == 0) return;
  hipLaunchKernelGGL(k_cav_fail, dim3((w.b_n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, w.cav_flag, w.b_n,
                     w.b_dperm, w.b_derr);
  HIP_OK(hipGetLastError());
  if (w.b_hperm) {
    HIP_OK(hipMemcpyAsync(w.b_xperm, w.b_dperm, w.b_n, hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(w.b_xerr, w.b_derr, (size_t)w.b_n * 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
  }
}

// Completes the batch in flight (caller holds w.m). The results are in the caller's device
// buffers, or in the pinned staging for a host batch.
static void finish_batch(Engine& e, Workspace& w) {
  if (w.state != 1) return;
  w.state = 2;
  w.b_ms = finish_pass(e, w);
  if (w.cav_on) caveat_passes(e, w);
}

static void copy_out(Workspace& w) {
  if (w.b_copy_perm) {  // a zero-copy batch over the pinned staging: the results to the caller's buffers
    std::memcpy(w.b_copy_perm, w.h_perm, w.b_n);
    std::memcpy(w.b_copy_err, w.h_err, (size_t)w.b_n * 4);
    return;
  }
  if (!w.b_hperm || w.b_xperm != w.h_perm) return;  // device batch, or results DMA'd in place
  std::memcpy(w.b_hperm, w.h_perm, w.b_n);
  std::memcpy(w.b_herr, w.h_err, (size_t)w.b_n * 4);
}

void drain_batches(Engine& e) {
  struct ResDrain {  // then the resident join (it reads the snapshot a writer is about to change)
    Engine& e;
    ~ResDrain() {
      try {
        res_drain(e);
      } catch (const Error&) {
      }
    }
  } res_drain_after{e};
  std::vector<Workspace*> busy;
  {
    std::lock_guard<std::mutex> lk(e.ws_mu);
    for (Workspace* w : e.ws_pool)
      if (w->busy) busy.push_back(w);
  }
  for (Workspace* w : busy) {
    std::lock_guard<std::mutex> lk(w->m);
    if (w->state != 1) continue;
    try {
      finish_batch(e, *w);
    } catch (const Error& ex) {
      w->fail_code = ex.code;
      w->fail_msg = ex.what();
    }
  }
}

void device_check(Engine& e, Workspace& w, const gck_item* d_items, size_t n, int64_t now_us, uint8_t* d_perm,
                  int32_t* d_err, void* stream, CavCall cav) {
  HIP_OK(hipSetDevice(e.device));
  std::lock_guard<std::mutex> lk(w.m);
  // the caller's stream; NULL is the legacy default stream (never the workspace's own
  // non-blocking stream, which would not be ordered after the caller's writes of the items)
  hipStream_t st = (hipStream_t)stream;
  stage_caveats(w, std::move(cav), st);
  if (now_us == 0) now_us = wall_now_us();
  float ms = 0.f;
  for (size_t pos = 0; pos < n; pos += w.max_batch) {
    const uint32_t len = (uint32_t)std::min(n - pos, w.max_batch);
    submit_batch(e, w, d_items + pos, len, now_us, d_perm + pos, d_err + pos, st, false);
    finish_batch(e, w);
    w.state = 0;
    ms += w.b_ms;
  }
  std::lock_guard<std::mutex> sl(e.stats_mu);
  e.stats.kernel_ms = ms;
}

// Host buffers: chunks of max_batch on two workspaces in turn, so that a chunk's copies and
// host staging overlap the previous chunk's kernels.
void device_check_host(Engine& e, Workspace* w0, Workspace* w1, const gck_item* items, size_t n, int64_t now_us,
                       uint8_t* perm, int32_t* err, const CavCall& cav) {
  HIP_OK(hipSetDevice(e.device));
  if (now_us == 0) now_us = wall_now_us();
  const size_t mb = w0->max_batch;
  const size_t n_chunks = (n + mb - 1) / mb;
  Workspace* ws[2] = {w0, (w1 && n_chunks > 1) ? w1 : w0};
  std::lock_guard<std::mutex> g0(ws[0]->m);
  std::unique_ptr<std::lock_guard<std::mutex>> g1;
  if (ws[1] != ws[0]) g1.reset(new std::lock_guard<std::mutex>(ws[1]->m));
  stage_caveats(*ws[0], CavCall(cav), ws[0]->stream);
  if (ws[1] != ws[0]) stage_caveats(*ws[1], CavCall(cav), ws[1]->stream);
  // several chunks: the context slots are checked here, before any GPU work, so that a bad item
  // fails the call with its request index and no chunk is left writing the caller's buffers (a
  // single chunk's zero-copy join checks its own items in place)
  if (n_chunks > 1) validate_slots(items, (uint32_t)n, ws[0]->cav.n_given);
  float ms = 0.f;
  Workspace* prev = nullptr;
  try {
    for (size_t k = 0; k < n_chunks; ++k) {
      Workspace& w = *ws[k & 1];
      const size_t pos = k * mb;
      const uint32_t len = (uint32_t)std::min(n - pos, mb);
      if (prev == &w) {  // one workspace (a pool of one): the previous chunk completes first
        finish_batch(e, w);
        copy_out(w);
        w.state = 0;
        ms += w.b_ms;
        prev = nullptr;
      }
      submit_batch(e, w, items + pos, len, now_us, perm + pos, err + pos, nullptr, true);
      if (prev) {
        finish_batch(e, *prev);
        copy_out(*prev);
        prev->state = 0;
        ms += prev->b_ms;
      }
      prev = &w;
    }
    if (prev) {
      finish_batch(e, *prev);
      copy_out(*prev);
      prev->state = 0;
      ms += prev->b_ms;
    }
  } catch (...) {
    // a chunk failed: every other chunk still in flight completes (its kernels end and its
    // completion signal is consumed) before the workspaces go back to the pool
    for (Workspace* x : {ws[0], ws[1]}) {
      if (x->state == 1) {
        try {
          finish_batch(e, *x);
        } catch (...) {
        }
      }
      x->state = 0;
    }
    throw;
  }
  std::lock_guard<std::mutex> sl(e.stats_mu);
  e.stats.kernel_ms = ms;
}

void device_submit(Engine& e, Workspace* w, const gck_item* items, size_t n, int64_t now_us, uint8_t* perm,
                   int32_t* err, void* stream, bool host, bool engine_stream, CavCall cav) {
  HIP_OK(hipSetDevice(e.device));
  std::lock_guard<std::mutex> lk(w->m);
  if (n > w->max_batch) throw Error(GCK_E_INVALID_ARGUMENT, "submitted batch above max_batch");
  hipStream_t st = (host || engine_stream) ? w->stream : (hipStream_t)stream;
  stage_caveats(*w, std::move(cav), st);
  if (now_us == 0) now_us = wall_now_us();
  submit_batch(e, *w, items, (uint32_t)n, now_us, perm, err, st, host, !host && engine_stream);
}

// ---- uniform batches (include/gck.h gck_check_bulk_uniform, gck_check_submit_uniform) ----------
// One header and (resource id, subject id) pairs in, 2-bit results out. With a one-round join on
// the engine's queues the join reads the pairs and writes the packed words in place (zero-copy:
// 8 B per check in, 1/4 B out across PCIe) and writes the item of each check it leaves into the
// workspace's item array, where the bundle stages answer it; the wait patches those into the words
// and lists the errors. Otherwise the request is expanded to items and runs as a host batch.
static void submit_uniform(Engine& e, Workspace& w, const gck_uniform& h, const uint32_t* pairs, uint32_t n,
                           int64_t now_us, unsigned long long* packed) {
  const uint32_t rp = (uint32_t)h.resource_type | (uint32_t)h.permission << 16;
  const uint32_t ss = (uint32_t)h.subject_type | (uint32_t)h.subject_relation << 16;
  const bool join = label_join_on(e) || (e.dev->d_cj && !(e.cfg.flags & GCK_FLAG_NO_CLOSURE));
  if (e.aql && w.aql_kernarg && !w.cav_on && !(e.cfg.flags & (GCK_FLAG_PROFILE | GCK_FLAG_NO_BUNDLE)) && join) {
    const size_t words = ((size_t)n + 31u) / 32u;
    const bool pin_in = host_pinned(e, pairs, (size_t)n * 8u), pin_out = host_pinned(e, packed, words * 8u);
    if (!pin_in) std::memcpy(w.h_items, pairs, (size_t)n * 8u);
    w.u_rp = rp;
    w.u_ss = ss;
    w.u_ctx = h.context_slot;
    w.u_pairs = pin_in ? pairs : reinterpret_cast<const uint32_t*>(w.h_items);
    // (the staging's result region holds 4 B per check: room for the words)
    w.u_packed = pin_out ? packed : reinterpret_cast<unsigned long long*>(w.h_err);
    submit_batch(e, w, w.d_items, n, now_us, w.d_perm, w.d_err, w.stream, false, true, true);
  } else {
    w.u_items.resize(n);
    for (uint32_t k = 0; k < n; ++k) {
      gck_item& it = w.u_items[k];
      it.resource_type = h.resource_type;
      it.permission = h.permission;
      it.resource_id = pairs[2 * (size_t)k];
      it.subject_type = h.subject_type;
      it.subject_relation = h.subject_relation;
      it.subject_id = pairs[2 * (size_t)k + 1];
      it.context_slot = h.context_slot;
    }
    w.u_perm.resize(n);
    w.u_err.resize(n);
    w.u_packed = nullptr;
    submit_batch(e, w, w.u_items.data(), n, now_us, w.u_perm.data(), w.u_err.data(), nullptr, true);
  }
  w.u_on = true;
  w.u_out = packed;
  w.u_ncj = 0;
}

// After a uniform batch has finished (finish_batch, copy_out): its words into the caller's buffer
// and its errors, at request offset `pos`, appended to `errs`.
static void uniform_collect(Workspace& w, uint32_t pos, std::vector<gck_item_error>& errs) {
  const uint32_t n = w.b_n;
  const size_t words = ((size_t)n + 31u) / 32u;
  if (w.u_join) {
    unsigned long long* out = w.u_packed;
    if (w.u_ncj) {  // the checks the join left: their results from the bundle stages
      std::vector<uint32_t> idx(w.u_ncj);
      w.u_perm.resize(n);
      w.u_err.resize(n);
      HIP_OK(hipMemcpyAsync(idx.data(), w.c_deferred, idx.size() * 4u, hipMemcpyDeviceToHost, w.stream));
      HIP_OK(hipMemcpyAsync(w.u_perm.data(), w.d_perm, n, hipMemcpyDeviceToHost, w.stream));
      HIP_OK(hipMemcpyAsync(w.u_err.data(), w.d_err, (size_t)n * 4u, hipMemcpyDeviceToHost, w.stream));
      HIP_OK(hipStreamSynchronize(w.stream));
      for (uint32_t i : idx) {
        if (i >= n) throw Error(GCK_E_DEVICE, "engine invariant violated: deferred index");
        if (w.u_err[i]) errs.push_back(gck_item_error{pos + i, w.u_err[i]});
        else out[i >> 5] |= (unsigned long long)(w.u_perm[i] & 3u) << (2u * (i & 31u));
      }
    }
    if (out != w.u_out) std::memcpy(w.u_out, out, words * 8u);
  } else {
    for (size_t k = 0; k < words; ++k) {
      unsigned long long x = 0;
      const uint32_t b = (uint32_t)k * 32u, m = std::min<uint32_t>(32u, n - b);
      for (uint32_t q = 0; q < m; ++q) {
        const uint32_t i = b + q;
        if (w.u_err[i]) errs.push_back(gck_item_error{pos + i, w.u_err[i]});
        else x |= (unsigned long long)(w.u_perm[i] & 3u) << (2u * q);
      }
      w.u_out[k] = x;
    }
  }
}

static void uniform_errors(std::vector<gck_item_error>& errs, gck_item_error* out, size_t cap, size_t* n_errs) {
  std::sort(errs.begin(), errs.end(),
            [](const gck_item_error& x, const gck_item_error& y) { return x.index < y.index; });
  const size_t m = std::min(cap, errs.size());
  if (m && out) std::memcpy(out, errs.data(), m * sizeof(gck_item_error));
  if (n_errs) *n_errs = errs.size();
}

void device_submit_uniform(Engine& e, Workspace* w, const gck_uniform& h, const uint32_t* pairs, size_t n,
                           int64_t now_us, uint64_t* packed, gck_item_error* errs, size_t cap, size_t* n_errs,
                           CavCall cav) {
  HIP_OK(hipSetDevice(e.device));
  std::lock_guard<std::mutex> lk(w->m);
  if (n > w->max_batch) throw Error(GCK_E_INVALID_ARGUMENT, "submitted batch above max_batch");
  stage_caveats(*w, std::move(cav), w->stream);
  if (now_us == 0) now_us = wall_now_us();
  submit_uniform(e, *w, h, pairs, (uint32_t)n, now_us, reinterpret_cast<unsigned long long*>(packed));
  w->u_errs = errs;
  w->u_err_cap = cap;
  w->u_n_errs = n_errs;
}

// Synchronous: chunks of max_batch (a multiple of 32 checks, so that each chunk's words start a
// word) on two workspaces in turn, as device_check_host.
void device_check_uniform(Engine& e, Workspace* w0, Workspace* w1, const gck_uniform& h, const uint32_t* pairs,
                          size_t n, int64_t now_us, uint64_t* packed, gck_item_error* out_errs, size_t cap,
                          size_t* n_errs, const CavCall& cav) {
  HIP_OK(hipSetDevice(e.device));
  if (now_us == 0) now_us = wall_now_us();
  const size_t mb = w0->max_batch >= 32 ? (w0->max_batch & ~(size_t)31) : w0->max_batch;
  if (n > mb && mb % 32 != 0) throw Error(GCK_E_CAPACITY, "a uniform request above max_batch needs max_batch >= 32");
  const size_t n_chunks = (n + mb - 1) / mb;
  Workspace* ws[2] = {w0, (w1 && n_chunks > 1) ? w1 : w0};
  std::lock_guard<std::mutex> g0(ws[0]->m);
  std::unique_ptr<std::lock_guard<std::mutex>> g1;
  if (ws[1] != ws[0]) g1.reset(new std::lock_guard<std::mutex>(ws[1]->m));
  stage_caveats(*ws[0], CavCall(cav), ws[0]->stream);
  if (ws[1] != ws[0]) stage_caveats(*ws[1], CavCall(cav), ws[1]->stream);
  std::vector<gck_item_error> errs;
  size_t pos_of[2] = {0, 0};
  float ms = 0.f;
  Workspace* prev = nullptr;
  auto complete = [&](Workspace& w) {
    finish_batch(e, w);
    copy_out(w);
    uniform_collect(w, (uint32_t)pos_of[&w == ws[0] ? 0 : 1], errs);
    w.state = 0;
    w.u_on = false;
    ms += w.b_ms;
  };
  try {
    for (size_t k = 0; k < n_chunks; ++k) {
      Workspace& w = *ws[k & 1];
      const size_t pos = k * mb;
      const uint32_t len = (uint32_t)std::min(n - pos, mb);
      if (prev == &w) {
        complete(w);
        prev = nullptr;
      }
      pos_of[&w == ws[0] ? 0 : 1] = pos;
      submit_uniform(e, w, h, pairs + 2 * pos, len, now_us, reinterpret_cast<unsigned long long*>(packed + pos / 32));
      if (prev) complete(*prev);
      prev = &w;
    }
    if (prev) complete(*prev);
  } catch (...) {
    for (Workspace* x : {ws[0], ws[1]}) {
      if (x->state == 1) {
        try {
          finish_batch(e, *x);
        } catch (...) {
        }
      }
      x->state = 0;
      x->u_on = false;
    }
    throw;
  }
  uniform_errors(errs, out_errs, cap, n_errs);
  std::lock_guard<std::mutex> sl(e.stats_mu);
  e.stats.kernel_ms = ms;
}

// Completes a submitted batch. Takes no engine lock: a writer that wants to replace the
// snapshot finishes the batch first (drain_batches, under w->m), so the snapshot cannot change
// while this runs the later stages.
void device_wait(Engine& e, Workspace* w) {
  HIP_OK(hipSetDevice(e.device));
  std::lock_guard<std::mutex> lk(w->m);
  finish_batch(e, *w);  // no-op when a writer already finished it (drain_batches)
  w->state = 0;
  const bool uni = w->u_on;
  w->u_on = false;
  if (w->fail_code) throw Error(w->fail_code, w->fail_msg);
  copy_out(*w);
  if (uni) {
    std::vector<gck_item_error> errs;
    uniform_collect(*w, 0, errs);
    uniform_errors(errs, w->u_errs, w->u_err_cap, w->u_n_errs);
  }
  std::lock_guard<std::mutex> sl(e.stats_mu);
  e.stats.kernel_ms = w->b_ms;
}

// Synchronous batches over device buffers on one held workspace (lookups).
static void check_range(Engine& e, Workspace& w, const gck_item* d_items, size_t n, int64_t now_us, uint8_t* d_perm,
                        int32_t* d_err, hipStream_t st, float* ms) {
  for (size_t pos = 0; pos < n; pos += w.max_batch) {
    const uint32_t len = (uint32_t)std::min(n - pos, w.max_batch);
    submit_batch(e, w, d_items + pos, len, now_us, d_perm + pos, d_err + pos, st, false);
    finish_batch(e, w);
    w.state = 0;
    *ms += w.b_ms;
  }
}

// The partitioned batch's workspace: its own, outside the pool (a partitioned batch spans many
// calls, one BFS level each).
static Workspace& part_workspace(Engine& e) {
  std::lock_guard<std::mutex> lk(e.ws_mu);
  if (!e.part_ws) e.part_ws = create_workspace(e);
  ensure_wide(*e.part_ws);
  return *e.part_ws;
}

#include "partition.inc"
#include "lookup.inc"

static PartState& part_state(Workspace& w) {  // (caller holds w.m: part_run)
  if (!w.part) w.part = new PartState();
  return *w.part;
}

#include "delta.inc"

}  // namespace gck

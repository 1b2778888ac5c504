// gck_internal.hpp — shared host/device data layout of the engine.
//
// Layout in HBM (DESIGN.md §"Data layout"):
//   * one CSR per (relation, subject kind) and per edge class:
//       plain  : u32 offsets[n_rows+1], u32 nbr[]         (sorted rows, wildcard id last)
//       ext    : same + u32 caveat[] + i64 expires_at_us[] (caveated or expiring edges)
//   * a node program: DevNode[] (one per schema relation/permission + synthetic join nodes)
//     and DevItem[] (subject kinds of relations, children of unions, operands of joins).
//   * per-batch workspace: checks, queries, joins, two frontiers, row segments, visited hash.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define GCK_HD __host__ __device__
#else
#define GCK_HD
#endif

namespace gck {

// Partitioned graphs (partition.inc): the rank that owns object `obj` (its CSR
// rows, its slots, its frontier entries), and the object's index among that rank's objects.
// Type-independent, so an object id means the same owner in every relation. Ids are interned in
// arrival order, so id mod world is already a hash of the external id that spreads every type
// evenly; and the owner's objects are then ids rank, rank + world, ... — a rank's slot tables
// hold exactly its own objects, indexed by obj / world, with no translation table.
GCK_HD inline uint32_t part_owner(uint32_t obj, uint32_t world) { return obj % world; }
GCK_HD inline uint32_t part_local(uint32_t obj, uint32_t world) { return obj / world; }
// Objects [0, count) of a type that rank `rank` of `world` owns.
GCK_HD inline uint32_t part_local_count(uint32_t count, uint32_t rank, uint32_t world) {
  return count > rank ? (count - 1 - rank) / world + 1 : 0u;
}

constexpr uint16_t kEllipsis = 0xFFFFu;
constexpr uint32_t kWildcard = 0xFFFFFFFFu;
constexpr uint32_t kAbsent = 0xFFFFFFFEu;
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint16_t kNoNode = 0xFFFFu;

// ---- node program -----------------------------------------------------------------------
enum NodeKind : uint8_t {
  NK_RELATION = 0,   // stored tuples: items are subject kinds
  NK_UNION = 1,      // items: IT_COMPUTED / IT_ARROW / IT_SUB
  NK_INTERSECT = 2,  // items: IT_OPERAND (>= 2)
  NK_EXCLUDE = 3,    // items: IT_OPERAND; operand 0 is the base
  NK_ARROW_ALL = 4,  // items: IT_ARROW (target kNoNode => that subject contributes NO)
  NK_NIL = 5,
};

enum NodeFlags : uint8_t {
  NF_REAL = 1,   // a schema relation/permission: the identity filter applies
  NF_BIDIR = 2,  // a forward node whose checks may run bidirectionally (engine.hip build_bidir)
  NF_JUMP = 4,   // a reverse node whose first item is an ancestor-closure jump (bidir.inc)
  NF_DEEP = 8,   // a forward node some of whose objects can reach the depth budget (heights,
                 // engine.hip build_heights): a check rooted at such an object runs exact-depth
};

enum ItemKind : uint8_t {
  IT_KIND = 0,      // relation subject kind (stype, srel); csr_plain/csr_ext; target = srel node
  IT_COMPUTED = 1,  // computed userset on the same object: target node, dispatch (+1 depth)
  IT_ARROW = 2,     // tuple-to-userset over one tupleset kind: csr_*, target node (+1 depth)
  IT_SUB = 3,       // nested join node evaluated inline (no dispatch)
  IT_OPERAND = 4,   // join operand: target node, `dispatch` says whether depth advances
  IT_REV = 5,       // reverse program (bidir.inc): in-edge of a userset / arrow / direct item.
                    // csr_plain = the transposed CSR (subject -> objects), csr_ext = the forward
                    // CSR (probed instead when the target is local to the check's root), target
                    // = rev(node of the forward item)
};

struct DevNode {
  uint16_t type;
  uint8_t kind;
  uint8_t flags;
  uint32_t first;  // first DevItem
  uint32_t count;  // number of DevItems
  // NF_BIDIR roots only, over forward nodes t < 32: bit t of `cmask` = t is in this node's
  // closure; bit t of `lmask` = t is reached from this node through computed usersets only,
  // so a vertex (o, t) of a check's closure has o == the check's resource
  // Reverse nodes: bit t of `cmask` = an in-edge of this node enters forward node t and can be
  // probed on the forward CSR; bit 31 = it has another kind of item.
  uint32_t cmask;
  uint32_t lmask;
  uint16_t canon;  // visited-key node id: the node itself; rev'(t) -> rev(t) (bidir.inc)
  uint16_t lcsr;   // NF_BIDIR roots: the forward CSR whose row R each check caches (0xFFFF: none)
};

struct DevItem {
  uint8_t kind;
  uint8_t dispatch;   // IT_OPERAND: 1 if entering the operand is a dispatch
  uint16_t stype;     // IT_KIND/IT_ARROW: subject type of the kind
  uint16_t srel;      // IT_KIND/IT_ARROW: subject relation (kEllipsis for objects)
  uint16_t target;    // node to enter (kNoNode = none)
  uint32_t csr_plain; // kNone if no plain edges of this kind
  uint32_t csr_ext;   // kNone if no caveated/expiring edges of this kind
};

struct DevCSR {
  const uint32_t* off;
  const uint32_t* nbr;
  const uint32_t* cav;    // ext only
  const int64_t* exp_us;  // ext only
  uint32_t n_rows;
  uint8_t is_ext;
  uint8_t has_wild;  // some row holds the wildcard subject (plain direct CSRs with an index)
  uint16_t pad;
  // membership index of a plain direct-subject CSR: open-addressing set of
  // (object << 32 | subject) keys, 2x oversized, in 64-byte buckets of 8 keys probed
  // bucket-linearly (a lookup reads one bucket in the common case; nullptr = none)
  const unsigned long long* mhash;
  unsigned long long mmask;  // bucket count - 1
};

// ---- per-batch state ----------------------------------------------------------------------
struct DevCheck {  // the subject of a top-level check
  uint32_t sid;
  uint16_t stype;
  uint16_t srel;
};

enum QueryFlags : uint32_t {
  QF_FOUND_Y = 1u,
  QF_FOUND_C = 2u,
  QF_ERR = 4u,
  QF_DONE = 8u,
  QF_CANCELLED = 16u,
  QF_RES_SHIFT = 8,  // result (GCK_PERM_* or 0xF for error) stored in bits 8..11
};

struct DevQuery {
  uint32_t check;        // index of the top-level check (its subject)
  uint32_t parent_join;  // kNone for top-level
  uint32_t flags;        // QueryFlags (atomic)
  int32_t pending_joins; // joins spawned and not resolved (atomic)
  uint32_t last_alive;   // last level an entry for this query was pushed into
  uint32_t operand;      // operand index inside the parent join (bits 0..23) | caveat tag << 24:
                         // how the result combines with the caveat of the edge the operand was
                         // entered through (exact-depth checks; engine.hip and_tag)
};

enum JoinState : uint32_t {
  JS_ANY_Y = 1u,
  JS_ANY_N = 2u,
  JS_ANY_C = 4u,
  JS_ANY_ERR = 8u,
  JS_BASE_Y = 16u,
  JS_BASE_N = 32u,
  JS_BASE_C = 64u,
  JS_BASE_ERR = 128u,
  JS_RESOLVED = 1u << 16,
};

struct DevJoin {
  uint32_t parent_q;
  uint32_t first_child;  // child queries [first_child, first_child + n_ops)
  uint32_t n_ops;
  uint32_t op;           // NK_INTERSECT / NK_EXCLUDE / NK_ARROW_ALL
  uint32_t cond;         // reached through a caveated edge
  int32_t remaining;     // atomic
  uint32_t state;        // JoinState bits (atomic)
  uint32_t pad;
};

struct Entry {  // 12 B frontier record
  uint32_t q;
  uint32_t obj;
  uint16_t node;
  uint8_t depth;
  uint8_t cond;  // bit 0: reached through an unresolved caveat; bit 1: exact-depth check
};

struct Segment {  // one CSR row range to enumerate
  uint64_t edge_start;
  uint32_t q;
  uint32_t begin;   // index into csr nbr[]
  uint32_t len;
  uint32_t csr;
  uint16_t target;
  uint8_t depth;
  uint8_t cond;
  uint32_t pad;
};

struct DevCounters {  // device-side counters, reset per level where noted
  unsigned long long seg_ctr;       // (nseg << 40) | total_edges   (per level)
  unsigned int next_size;           // entries pushed into the next frontier (per level)
  unsigned int n_queries;           // queries allocated (per batch)
  unsigned int n_joins;             // joins allocated (per batch)
  unsigned int overflow;            // bit0 visited, bit1 frontier, bit2 segments, bit3 queries, bit4 joins
  unsigned int last_next;           // next_size of the level just finished (published by k_level_end)
  unsigned long long segs_total;
  unsigned long long row_lookups;
  unsigned long long probes;
  unsigned long long edges;
  unsigned long long ext_edges;
  unsigned long long expanded;
  unsigned long long bidir;         // checks evaluated bidirectionally
  unsigned long long bundle_levels; // BFS levels run by bundles (summed over bundles)
  unsigned long long bundles;       // bundles run
  unsigned long long closure;       // checks the closure join answered in its task rounds (closure.inc;
                                    // the slot-path count is n - deferred - this, on the host)
  unsigned int cav_requests;        // (caveat instance, check context) pairs recorded for evaluation
  unsigned int cav_errors;          // touched pairs whose evaluation failed
  unsigned int bad_slot;            // a host item whose context_slot exceeds the call's contexts (the
                                    // joins validate zero-copy batches): 0xFFFFFFFF - its index, 0 none
};

}  // namespace gck

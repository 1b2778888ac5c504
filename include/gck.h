/*
 * gck.h — C ABI of the MI355X batched permission-check engine (libgck.so).
 *
 * This is the drop-in boundary for gochugaru's check path. A Go caller binds
 * it through cgo; the Python host mirror (gochugaru_amd/engine.py) binds it
 * through ctypes. Signatures use plain pointers and sizes only.
 *
 * Reference interfaces replaced (authzed/gochugaru @ 2025-10-03):
 *   gck_check_bulk / gck_check_bulk_device
 *       replace the CheckBulkPermissions round-trip made by Client.Check
 *       (client/client.go:261-266) and consumed at client/client.go:271-283; transitively
 *       CheckOne/CheckAny/CheckAll/CheckIter (client/client.go:129-180).
 *   gck_load_schema
 *       consumes the schema text returned by Client.ReadSchema (client/client.go:416-422).
 *   gck_begin_snapshot / gck_add_tuples / gck_add_tuples_text / gck_load_csr / gck_commit_snapshot
 *   gck_save_snapshot / gck_load_snapshot_file (on-disk snapshot cache)
 *       consume the relationships streamed by Client.ExportRelationships at the schema's
 *       revision (client/client.go:472-499, rel.FromV1Proto rel/relationship.go:147-172).
 *   gck_intern
 *       replaces the per-item string handling of Client.Check's item loop
 *       (client/client.go:242-259) with batched string -> dense u32 interning.
 *   gck_apply_updates / gck_apply_updates_text (or gck_watch_stage + gck_watch_apply_staged)
 *       consume the rel.Update stream of Client.UpdatesSinceRevision (client/client.go:370-413,
 *       rel.UpdateFromV1Proto rel/relationship.go:296-301) and keep the snapshot current.
 *   gck_check_bulk_ctx / gck_check_bulk_device_ctx
 *       additionally take the check-time caveat contexts (CheckBulkPermissionsRequestItem.Context,
 *       client/client.go:257, from rel.Relationship.MustV1ProtoCaveat rel/relationship.go:174-188).
 *   gck_revision / gck_check_bulk's consistency argument
 *       honour consistency.Strategy (consistency/consistency.go:15-77) as sent in
 *       CheckBulkPermissionsRequest.Consistency (client/client.go:263).
 *
 *   gck_check_submit / gck_check_wait
 *       the same round-trip split in two, so that a caller keeps several CheckBulkPermissions
 *       batches in flight (Client.CheckIter's chunks, client/client.go:164-180, or concurrent
 *       Client.Check calls) and the device overlaps them.
 *   gck_set_head_revision
 *       the revision consistency.Full() (consistency/consistency.go:25-35) must reach: the
 *       ReadAt token of Client.ReadSchema (client/client.go:416-422) or a Watch checkpoint.
 *   gck_check_bulk_at / gck_check_wait_at
 *       the same calls, also returning the revision the batch was evaluated at: the response's
 *       CheckedAt token (CheckBulkPermissionsResponse.CheckedAt, read by consistency users of
 *       client/client.go:261-266).
 *   gck_check_bulk_uniform / gck_check_submit_uniform
 *       the common homogeneous request of Client.Check's item loop (client/client.go:241-259: one
 *       CheckBulkPermissionsRequestItem per relationship, all of one resource type, permission,
 *       subject type and subject relation) as one header and 8-byte (resource id, subject id)
 *       pairs, answered as a packed 2-bit Permissionship plane plus a sparse per-item error list.
 *
 * Ownership: all inputs and outputs are caller-allocated; the engine never retains a caller
 * pointer after a call returns, except that gck_check_submit keeps the output pointers (and, for
 * device batches or host items in gck_host_alloc memory, the item pointer) until the matching
 * gck_check_wait. Return value: GCK_OK (0)
 * or a negative GCK_E_* status; the message is available from gck_last_error() (thread-local; the
 * message of the thread's last failure — a later success leaves it, as errno).
 * Threading: gck_check_bulk*, gck_check_submit / gck_check_wait and the lookups may be called
 * concurrently from any number of threads: each batch in flight runs on its own pooled
 * workspace and HIP stream (gck_config.workspaces of them; a call waits for a free one).
 * Schema, snapshot and Watch calls are exclusive: they first finish every batch in flight,
 * which keeps the results of the snapshot it was submitted against.
 */
#ifndef GCK_H
#define GCK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GCK_ABI_VERSION 13

/* ---- status codes ------------------------------------------------------------------- */
#define GCK_OK 0
#define GCK_E_INVALID_ARGUMENT (-1) /* gRPC InvalidArgument */
#define GCK_E_SCHEMA (-2)           /* schema text failed to parse/validate */
#define GCK_E_NOT_FOUND (-3)        /* unknown type/relation name in a lookup */
#define GCK_E_DEVICE (-4)           /* HIP failure: map to gRPC Unavailable (caller retries) */
#define GCK_E_CAPACITY (-5)         /* a device workspace limit was exceeded */
#define GCK_E_STATE (-6)            /* wrong call order (no schema / no snapshot) */
#define GCK_E_REVISION (-7)         /* consistency requirement not satisfiable locally */
#define GCK_E_NO_DEVICE (-8)        /* no HIP device / HIP runtime unavailable */
#define GCK_E_REVISION_GONE (-9)    /* consistency.Snapshot at a revision the snapshot has moved past:
                                       permanent (SpiceDB: FailedPrecondition), not retriable */

/* ---- Permissionship (authzed v1 CheckPermissionResponse.Permissionship) --------------- */
#define GCK_PERM_UNSPECIFIED 0
#define GCK_PERM_NO 1
#define GCK_PERM_HAS 2
#define GCK_PERM_CONDITIONAL 3

/* ---- per-item errors (CheckBulkPermissionsPair.Error) --------------------------------- */
#define GCK_ITEM_OK 0
#define GCK_ITEM_ERR_MAX_DEPTH 1                /* dispatch depth budget exhausted */
#define GCK_ITEM_ERR_UNKNOWN_PERMISSION 2       /* permission not defined on the type */
#define GCK_ITEM_ERR_UNKNOWN_TYPE 3             /* resource or subject type not defined */
#define GCK_ITEM_ERR_UNKNOWN_SUBJECT_RELATION 4 /* subject relation not defined */
#define GCK_ITEM_ERR_WILDCARD_SUBJECT 5         /* subject id "*" is not checkable */
#define GCK_ITEM_ERR_CAVEAT_EVAL 6              /* a caveat on the check's walk failed to evaluate
                                                   under its context (a type error, a bad value) */

/* ---- special ids ---------------------------------------------------------------------- */
#define GCK_ELLIPSIS 0xFFFFu          /* subject relation "..." (a concrete object) */
#define GCK_ID_WILDCARD 0xFFFFFFFFu   /* subject id "*" */
#define GCK_ID_ABSENT 0xFFFFFFFEu     /* an id that is not in the snapshot */
#define GCK_TYPE_INVALID 0xFFFFu

/* ---- consistency requirement (consistency.Strategy) ------------------------------------ */
#define GCK_CONSISTENCY_MIN_LATENCY 0
#define GCK_CONSISTENCY_FULL 1
#define GCK_CONSISTENCY_AT_LEAST 2
#define GCK_CONSISTENCY_SNAPSHOT 3

/* ---- flags ---------------------------------------------------------------------------- */
#define GCK_INTERN_CREATE 1u     /* gck_intern: create ids for unseen strings */
#define GCK_MEM_DEVICE 1u        /* gck_load_csr: pointers are device memory */
#define GCK_FLAG_PROFILE 1u      /* gck_config.flags: time every kernel with HIP events */
#define GCK_FLAG_NO_BUNDLE 2u    /* gck_config.flags: grid-wide level-synchronous path only */
#define GCK_FLAG_NO_MHASH 4u     /* gck_config.flags: no hashed membership index (binary search) */
#define GCK_FLAG_NO_GIANT 8u     /* gck_config.flags: deferred checks skip the workgroup-bundle stage */
#define GCK_FLAG_NO_BIDIR 16u    /* gck_config.flags: forward-only search (no bidirectional checks) */
#define GCK_FLAG_NO_CLOSURE 32u  /* gck_config.flags: no closure-join stage (nested-group checks take
                                    the bundle search) */
#define GCK_FLAG_NO_SLOTS 128u  /* gck_config.flags: no per-user / per-resource slots for the
                                   closure join (saves ~128 B per user of HBM; slower) */
#define GCK_FLAG_NO_LABELS 256u  /* gck_config.flags: no label-join stage (hub hierarchy labels and
                                    flattened resource slots; labels.inc) */
#define GCK_FLAG_RESIDENT 512u  /* gck_config.flags: nested-group (closure-join) batches dispatched on the
                                    engine's queues go to one resident launch per engine, whose
                                    workgroups take 128-check chunks of the posted requests, instead of
                                    a dispatch each (small requests: a 64K request sharded over GPUs) */
#define GCK_FLAG_LAZY_CAVEATS 64u /* gck_config.flags: always evaluate check-time caveat contexts
                                     lazily (only the pairs a walk meets; by default a call whose
                                     partial instances x distinct contexts is small evaluates them all) */
#define GCK_FLAG_BIG_MHASH 1024u  /* gck_config.flags: build hashed membership indexes above 4 GB too
                                     (by default a larger one is not built: the one-round joins never
                                     read it, and the checks they leave binary-search the row) */

typedef struct gck_engine gck_engine;

typedef struct gck_config {
  int32_t device;              /* HIP device ordinal */
  uint32_t max_depth;          /* dispatch depth budget; 0 = 50 (SpiceDB default) */
  uint32_t max_batch;          /* checks per device launch sequence; 0 = 65536 */
  uint32_t flags;              /* GCK_FLAG_* */
  uint64_t visited_capacity;   /* slots of the per-batch visited hash (power of 2); 0 = auto */
  uint64_t frontier_capacity;  /* entries per frontier buffer; 0 = auto */
  uint64_t segment_capacity;   /* row segments per level; 0 = auto */
  uint64_t query_capacity;     /* queries per batch (checks + sub-queries of joins); 0 = auto */
  uint32_t bundle_checks;      /* checks per wavefront bundle (1..48); 0 = 32 */
  uint32_t bundle_frontier;    /* frontier entries per wavefront; 0 = 4096 */
  uint32_t bundle_visited;     /* visited slots per wavefront (power of 2); 0 = 16384 */
  uint32_t bundle_waves_per_cu;/* resident wavefronts per CU for the bundle kernel; 0 = 8 */
  uint32_t bundle_budget;      /* entries one check may push in a wavefront bundle before it is
                                  handed to a 16-wave workgroup; 0 = 1024 */
  uint32_t giant_frontier;     /* frontier entries per 16-wave workgroup bundle; 0 = 65536 */
  uint32_t giant_visited;      /* visited slots per workgroup bundle (power of 2); 0 = 262144 */
  uint32_t giant_slots;        /* resident workgroup bundles; 0 = one per CU */
  uint32_t bidir_both;         /* bidirectional checks expand both sides while their two
                                  frontiers hold at most this many entries; 0 = 64 */
  uint32_t workspaces;         /* check batches in flight at once (concurrent callers and
                                  submitted batches), one device workspace each; 0 = 4. A
                                  submit waits for a free workspace: one thread must keep at
                                  most this many batches outstanding. Config 4 peaks at ~16
                                  in flight */
} gck_config;

/* One check item, interned: CheckBulkPermissionsRequestItem (client/client.go:244-258). */
typedef struct gck_item {
  uint16_t resource_type;
  uint16_t permission;         /* global relation id (gck_relation_id) */
  uint32_t resource_id;
  uint16_t subject_type;
  uint16_t subject_relation;   /* GCK_ELLIPSIS for a concrete object */
  uint32_t subject_id;
  uint32_t context_slot;       /* 0 = no check-time caveat context; k = contexts[k-1] of the
                                  gck_check_bulk*_ctx call */
} gck_item;                    /* 20 bytes */

/* One relationship, interned: rel.Relationship (rel/relationship.go:28-38). */
typedef struct gck_tuple {
  uint16_t resource_type;
  uint16_t relation;           /* global relation id */
  uint32_t resource_id;
  uint16_t subject_type;
  uint16_t subject_relation;   /* GCK_ELLIPSIS or a relation id of subject_type */
  uint32_t subject_id;         /* GCK_ID_WILDCARD for "type:*" */
  uint32_t caveat;             /* caveat instance id from gck_add_caveat_instance; 0 = none */
  int64_t expires_at_us;       /* unix microseconds; 0 = never */
} gck_tuple;                   /* 32 bytes */

/* One Watch update: rel.Update (rel/relationship.go:291-301), operation = rel.UpdateType. */
#define GCK_UPDATE_CREATE 1u   /* rel.UpdateCreate (applied as an upsert) */
#define GCK_UPDATE_DELETE 2u   /* rel.UpdateDelete */
#define GCK_UPDATE_TOUCH 3u    /* rel.UpdateTouch */
typedef struct gck_update {
  uint32_t op;                 /* GCK_UPDATE_* */
  uint32_t reserved;
  gck_tuple tuple;
} gck_update;                  /* 40 bytes */

typedef struct gck_consistency {
  int32_t requirement;         /* GCK_CONSISTENCY_* */
  uint32_t reserved;
  uint64_t revision;           /* AT_LEAST / SNAPSHOT token, decoded */
} gck_consistency;

typedef struct gck_stats {
  uint64_t batches;
  uint64_t levels;             /* BFS levels executed: grid-wide levels + every bundle's levels */
  uint64_t entries_expanded;   /* (query, object, node) entries expanded */
  uint64_t row_lookups;        /* CSR rows opened (each = one 8-B offset pair) */
  uint64_t membership_probes;  /* 4-B neighbour reads by membership binary searches */
  uint64_t edges_enumerated;   /* 4-B neighbour reads by userset/arrow enumeration */
  uint64_t ext_edges;          /* caveated/expiring edges read (+4 B caveat id +8 B expiry) */
  uint64_t queries;            /* queries allocated (checks + join operands) */
  uint64_t joins;              /* intersection/exclusion/all() joins spawned */
  uint64_t retries;            /* batch splits after a workspace overflow */
  double kernel_ms;            /* GCK_FLAG_PROFILE: device time of the last call's batches that were
                                  timed (HIP events around stage A on every 4th batch of a workspace) */
  double expand_ms;            /* GCK_FLAG_PROFILE: summed k_expand time (all batches) */
  double edges_ms;             /* GCK_FLAG_PROFILE: summed k_edges time */
  double resolve_ms;           /* GCK_FLAG_PROFILE: summed k_resolve time */
  uint64_t expand_launches;    /* GCK_FLAG_PROFILE: k_expand launches timed */
  uint64_t edges_launches;     /* GCK_FLAG_PROFILE: k_edges launches timed */
  double bundle_ms;            /* GCK_FLAG_PROFILE: summed stage-A time (closure join and/or wave
                                  bundles) of the timed batches (every 4th of a workspace) */
  uint64_t bundle_launches;    /* GCK_FLAG_PROFILE: batches whose stage A was timed */
  uint64_t deferred;           /* checks handed from wavefront bundles to workgroup bundles */
  double giant_ms;             /* GCK_FLAG_PROFILE: summed workgroup-bundle kernel time */
  uint64_t deferred_wide;      /* checks handed from workgroup bundles to the grid-wide path */
  uint64_t bidir_checks;       /* checks evaluated bidirectionally (forward + reverse frontier) */
  uint64_t bundles;            /* check bundles run by the bundle kernels (`levels` also sums
                                  their BFS levels) */
  uint64_t closure_checks;     /* checks answered by the closure-join stage (nested groups) */
  uint64_t caveat_evals;       /* (caveat instance, check context) pairs evaluated on the host */
  uint64_t caveat_passes;      /* extra batch passes after lazily evaluated caveat pairs */
  uint64_t slot_checks;        /* checks the closure join decided from their user / resource slots
                                  alone (one read each) */
  uint64_t label_checks;       /* of closure_checks: those the label join (labels.inc k_label_join,
                                  or its partitioned form) answered */
  uint64_t aql_batches;        /* batches whose join the engine dispatched into its own HSA queue
                                  (engine-stream device batches, aql.inc) instead of launching it
                                  through HIP */
  uint64_t resident_batches;   /* batches the resident join took (GCK_FLAG_RESIDENT) */
} gck_stats;

/* ---- lifecycle ------------------------------------------------------------------------ */
int gck_abi_version(void);
const char* gck_last_error(void);
int gck_create(const gck_config* cfg, gck_engine** out);
void gck_destroy(gck_engine* e);

/* ---- schema (Client.ReadSchema text, client/client.go:416-422) ------------------------ */
int gck_load_schema(gck_engine* e, const char* text, size_t len);
int gck_type_id(gck_engine* e, const char* name, size_t len, uint16_t* out);
int gck_relation_id(gck_engine* e, uint16_t type, const char* name, size_t len, uint16_t* out);
int gck_type_count(gck_engine* e, uint32_t* out);
int gck_relation_count(gck_engine* e, uint32_t* out);

/* ---- interning (Client.Check item loop, client/client.go:242-259) --------------------- */
int gck_intern(gck_engine* e, uint16_t type, const char* const* ids, const uint32_t* lens,
               size_t n, uint32_t flags, uint32_t* out_ids);
int gck_object_count(gck_engine* e, uint16_t type, uint32_t* out);
/* Declares ids [0, n) of `type` as existing (anonymous objects for bulk CSR ingest). */
int gck_reserve_objects(gck_engine* e, uint16_t type, uint32_t n);
int gck_object_name(gck_engine* e, uint16_t type, uint32_t id, char* buf, size_t cap,
                    size_t* out_len);

/* ---- caveats (rel.Relationship.CaveatName/CaveatContext) ------------------------------ */
/* A caveat name with its stored context (a JSON object; "" = none). Identical (name, context)
 * pairs return the same id. Errors: GCK_E_INVALID_ARGUMENT for an unknown caveat, malformed
 * JSON, or a stored context on which the expression fails to evaluate. */
int gck_add_caveat_instance(gck_engine* e, const char* name, size_t name_len,
                            const char* context_json, size_t json_len, uint32_t* out_id);

/* The host CEL evaluator on its own: caveat `name` over the stored context merged with the
 * check context (stored values take precedence). *out = 0 false, 1 true, 2 partial (a
 * parameter is missing: CONDITIONAL). GCK_E_NOT_FOUND for an unknown caveat. */
int gck_evaluate_caveat(gck_engine* e, const char* name, size_t name_len, const char* stored_json,
                        size_t stored_len, const char* context_json, size_t context_len, uint8_t* out);

/* ---- snapshot ingest (Client.ExportRelationships, client/client.go:472-499) ----------- */
int gck_begin_snapshot(gck_engine* e, uint64_t revision);
int gck_add_tuples(gck_engine* e, const gck_tuple* tuples, size_t n);
/* Canonical rel.Relationship.String lines (rel/relationship.go:51-90), '\n'-separated. */
int gck_add_tuples_text(gck_engine* e, const char* text, size_t len);
/* Prebuilt CSR for one (relation, subject kind): rows sorted ascending, no duplicates,
 * plain edges only (no caveat/expiration). n_rows = object count of the relation's type. */
int gck_load_csr(gck_engine* e, uint16_t relation, uint16_t subject_type,
                 uint16_t subject_relation, uint32_t n_rows, const uint32_t* offsets,
                 const uint32_t* neighbours, uint64_t n_edges, uint32_t mem_flags);
int gck_commit_snapshot(gck_engine* e);
/* On-disk snapshot cache, in place of re-reading the snapshot through
 * Client.ExportRelationships (client/client.go:472-499) and re-interning it: save writes the
 * committed snapshot (interner, caveat instances, base CSRs, revision) keyed by the schema
 * text; load (same schema text, no staging in progress) replaces the committed snapshot and
 * rebuilds the derived device indexes. GCK_E_SCHEMA when the file was saved under another
 * schema; GCK_E_STATE to save a partitioned engine or with nothing committed. */
int gck_save_snapshot(gck_engine* e, const char* path);
int gck_load_snapshot_file(gck_engine* e, const char* path);
int gck_revision(gck_engine* e, uint64_t* out);
/* The source's head revision, for consistency.Full(): a Full check (or lookup) returns
 * GCK_E_REVISION — gRPC Unavailable, which the client retries — until the applied revision
 * (gck_commit_snapshot / gck_apply_updates) reaches it. 0 (the default) = the local snapshot is
 * the head. The head only moves forward. */
int gck_set_head_revision(gck_engine* e, uint64_t revision);
int gck_tuple_count(gck_engine* e, uint64_t* out);
/* Bytes resident in HBM for the snapshot (CSR + tables). */
int gck_device_bytes(gck_engine* e, uint64_t* out);

/* ---- Watch (Client.UpdatesSinceRevision, client/client.go:370-413) ------------------- */
/* Applies one batch of updates (a Watch response, in stream order) to the committed snapshot
 * and moves it to `revision` (the response's ChangesThrough token, decoded), which must be
 * newer than the current one; an empty batch may also re-state the current revision. The merge
 * runs on the device. Errors: GCK_E_REVISION (stale revision), GCK_E_INVALID_ARGUMENT (unknown
 * operation / relationship the schema rejects; nothing applied), GCK_E_STATE (no snapshot).
 * A device failure during the merge leaves no snapshot (GCK_E_STATE until the next commit). */
int gck_apply_updates(gck_engine* e, uint64_t revision, const gck_update* updates, size_t n);
/* Text form: one "<OP> <relationship>" per line, OP = CREATE | TOUCH | DELETE and the
 * relationship in rel.Relationship.String form (rel/relationship.go:51-90). */
int gck_apply_updates_text(gck_engine* e, uint64_t revision, const char* text, size_t len);
/* Pipelined Watch: a consumer that has the next batch while it applies the previous one stages it
 * — gck_watch_stage returns at once and an engine thread validates and groups the batch meanwhile
 * — then applies it with gck_watch_apply_staged, in stream order, which waits for the grouping and
 * applies as gck_apply_updates does (same errors; a batch the staging rejected, or staged before a
 * schema / snapshot-file / partition change, is grouped again there and its error reported).
 * `updates` must stay valid and unchanged until the ticket is applied or discarded. Up to 4
 * batches may be staged at once (GCK_E_CAPACITY beyond); a ticket is used once. */
int gck_watch_stage(gck_engine* e, const gck_update* updates, size_t n, uint64_t* ticket);
int gck_watch_apply_staged(gck_engine* e, uint64_t revision, uint64_t ticket);
int gck_watch_discard(gck_engine* e, uint64_t ticket);

/* ---- checks (CheckBulkPermissions, client/client.go:261-283) -------------------------- */
/* Host buffers: items[n] in, out_perm[n] (GCK_PERM_*), out_err[n] (GCK_ITEM_*) out.
 * `now_us` = the evaluation time for expiring relationships (unix microseconds; 0 = wall
 * clock). Results are in request order. Caveats are evaluated with the stored context only;
 * one that depends on a missing parameter makes its path CONDITIONAL. */
int gck_check_bulk(gck_engine* e, const gck_consistency* cs, const gck_item* items, size_t n,
                   int64_t now_us, uint8_t* out_perm, int32_t* out_err);
/* Same, with check-time caveat contexts: contexts[k] (JSON object text, context_lens[k] bytes)
 * is the context of every item whose context_slot is k + 1. A caveat is evaluated over its
 * stored context merged with the item's context (stored values take precedence): true = the
 * relationship counts, false = it does not, missing parameter = CONDITIONAL. Only the
 * (caveat instance, context) pairs the checks' walks meet are evaluated once the product of
 * partial instances and distinct contexts is large (the batch then runs again with their
 * outcomes); a pair that fails to evaluate gives the items whose walk met it
 * GCK_ITEM_ERR_CAVEAT_EVAL and nothing else.
 * Errors: GCK_E_INVALID_ARGUMENT (a context_slot > n_contexts, malformed JSON). */
int gck_check_bulk_ctx(gck_engine* e, const gck_consistency* cs, const gck_item* items, size_t n,
                       const char* const* contexts, const size_t* context_lens, size_t n_contexts,
                       int64_t now_us, uint8_t* out_perm, int32_t* out_err);
/* Device-resident buffers on the engine's device. `stream` is the hipStream_t the caller
 * produced the items on and will read the results on; NULL is HIP's default (null) stream, as
 * for any HIP launch, so work the caller queued there (e.g. PyTorch's default stream) is
 * ordered before the check. Returns after the results are written (stream synchronised). */
int gck_check_bulk_device(gck_engine* e, const gck_item* d_items, size_t n, int64_t now_us,
                          uint8_t* d_out_perm, int32_t* d_out_err, void* stream);
/* Device buffers with host-side check contexts (as gck_check_bulk_ctx; a device item's
 * context_slot beyond n_contexts counts as no context). */
int gck_check_bulk_device_ctx(gck_engine* e, const gck_item* d_items, size_t n,
                              const char* const* contexts, const size_t* context_lens, size_t n_contexts,
                              int64_t now_us, uint8_t* d_out_perm, int32_t* d_out_err, void* stream);
/* Asynchronous batches: gck_check_submit starts one batch of n <= max_batch items and returns at
 * once with a handle; gck_check_wait(handle) completes it (results written, handle consumed).
 * Every submitted batch must be waited for exactly once. GCK_SUBMIT_DEVICE: items / out_perm /
 * out_err are device buffers ordered on `stream` (as gck_check_bulk_device_ctx); otherwise they
 * are host buffers (the outputs are written by the wait; pageable items are staged before the
 * call returns, while items in gck_host_alloc memory are read by DMA as the batch runs and must
 * stay unchanged until gck_check_wait returns). Consistency is checked at submit; the batch sees the snapshot current at submit, even if
 * a Watch batch is applied before the wait. GCK_SUBMIT_DEVICE | GCK_SUBMIT_ENGINE_STREAM: device
 * buffers, but the batch runs on the stream of the workspace it holds (created by the engine, one
 * per workspace, so that batches in flight sit on distinct hardware queues) and `stream` is
 * ignored: the items must be complete when the call is made, and the results are complete when
 * gck_check_wait returns. */
typedef struct gck_batch gck_batch;
#define GCK_SUBMIT_DEVICE 1u
#define GCK_SUBMIT_ENGINE_STREAM 2u
int gck_check_submit(gck_engine* e, const gck_consistency* cs, const gck_item* items, size_t n,
                     const char* const* contexts, const size_t* context_lens, size_t n_contexts,
                     int64_t now_us, uint8_t* out_perm, int32_t* out_err, uint32_t flags, void* stream,
                     gck_batch** out);
int gck_check_wait(gck_engine* e, gck_batch* batch);
/* Pinned host memory for request / result buffers: a host batch (gck_check_bulk*,
 * gck_check_submit) whose items or results lie in such a buffer is copied over PCIe by DMA
 * directly, skipping the engine's own staging copy (a submitted batch then reads its items there
 * until gck_check_wait). Freed with gck_host_free (or gck_destroy). */
int gck_host_alloc(gck_engine* e, size_t bytes, void** out);
int gck_host_free(gck_engine* e, void* p);
int gck_last_stats(gck_engine* e, gck_stats* out);
int gck_reset_stats(gck_engine* e);
/* Turns GCK_FLAG_PROFILE on or off for the batches submitted from now on (a timed batch brackets
 * its stage A with the kernel's own start/stop events, every 4th batch of a workspace). */
int gck_set_profile(gck_engine* e, uint32_t on);

/* The revision a check was evaluated at (ABI 13). gck_check_bulk_at is gck_check_bulk_ctx that
 * also writes the revision of the snapshot the batch ran on to *out_revision (may be NULL): the
 * response's CheckedAt. A submitted batch runs on the snapshot current at its submit, and
 * gck_check_wait_at reports that revision — not the one current at the wait, which a Watch batch
 * applied in between may have moved. */
int gck_check_bulk_at(gck_engine* e, const gck_consistency* cs, const gck_item* items, size_t n,
                      const char* const* contexts, const size_t* context_lens, size_t n_contexts,
                      int64_t now_us, uint8_t* out_perm, int32_t* out_err, uint64_t* out_revision);
int gck_check_wait_at(gck_engine* e, gck_batch* batch, uint64_t* out_revision);

/* ---- uniform requests (ABI 13) -------------------------------------------------------
 * A request whose items share (resource type, permission, subject type, subject relation, context
 * slot) — what Client.Check sends for relationships of one shape (client/client.go:241-259) —
 * travels as one header and n (resource id, subject id) pairs: 8 bytes per check over PCIe
 * instead of 20. Results come back packed: check k's Permissionship (GCK_PERM_*) in bits
 * 2(k mod 32) .. 2(k mod 32) + 1 of out_packed[k / 32] (ceil(n / 32) words; GCK_PERM_UNSPECIFIED
 * for a check with an error), and the checks with an error as (index, GCK_ITEM_*) records in
 * ascending index order: *out_n_errs = how many checks have one, the first min(that, err_cap) of
 * them are written to out_errs. Semantics, consistency and request errors are gck_check_bulk_at's;
 * a context_slot beyond n_contexts is GCK_E_INVALID_ARGUMENT. Pairs and results in gck_host_alloc
 * memory are read and written in place by the kernels. */
typedef struct gck_uniform {
  uint16_t resource_type;
  uint16_t permission;         /* global relation id (gck_relation_id) */
  uint16_t subject_type;
  uint16_t subject_relation;   /* GCK_ELLIPSIS for a concrete object */
  uint32_t context_slot;       /* as gck_item.context_slot, for every pair */
  uint32_t reserved;           /* 0 */
} gck_uniform;                 /* 16 bytes */
typedef struct gck_item_error {
  uint32_t index;              /* the check's position in the request */
  int32_t code;                /* GCK_ITEM_* (never GCK_ITEM_OK) */
} gck_item_error;
int gck_check_bulk_uniform(gck_engine* e, const gck_consistency* cs, const gck_uniform* hdr, const uint32_t* pairs,
                           size_t n, const char* const* contexts, const size_t* context_lens, size_t n_contexts,
                           int64_t now_us, uint64_t* out_packed, gck_item_error* out_errs, size_t err_cap,
                           size_t* out_n_errs, uint64_t* out_revision);
/* The same as an asynchronous batch (n <= max_batch; host buffers): completed by gck_check_wait or
 * gck_check_wait_at, which write out_packed, out_errs and *out_n_errs. `pairs`, `hdr` and the
 * outputs must stay valid until the wait returns. */
int gck_check_submit_uniform(gck_engine* e, const gck_consistency* cs, const gck_uniform* hdr, const uint32_t* pairs,
                             size_t n, const char* const* contexts, const size_t* context_lens, size_t n_contexts,
                             int64_t now_us, uint64_t* out_packed, gck_item_error* out_errs, size_t err_cap,
                             size_t* out_n_errs, gck_batch** out);

/* ---- lookups (Client.LookupResources / LookupSubjects, client/client.go:508-599) -------- */
/* Ids of the `resource_type` objects on which the subject has `permission` — HAS or CONDITIONAL,
 * out_perm[k] says which — ascending. Every object of the type is checked on the device (the
 * check path's stages, candidates generated and answers compacted there). *out_n = the number of
 * ids; when it exceeds `cap` nothing is written and GCK_E_CAPACITY is returned: call again with
 * cap >= *out_n (the result of the last lookup is kept per thread, so the retry does not sweep
 * again). Errors: GCK_E_NOT_FOUND (unknown type / permission / subject relation),
 * GCK_E_INVALID_ARGUMENT (a candidate hit the depth budget), GCK_E_REVISION (consistency). */
int gck_lookup_resources(gck_engine* e, const gck_consistency* cs, uint16_t resource_type, uint16_t permission,
                         uint16_t subject_type, uint16_t subject_relation, uint32_t subject_id, int64_t now_us,
                         uint32_t* out_ids, uint8_t* out_perm, size_t cap, size_t* out_n);
/* Ids of the `subject_type` objects (with `subject_relation`, GCK_ELLIPSIS for plain objects)
 * that have `permission` on one resource, ascending; same protocol. As SpiceDB's LookupSubjects:
 * the candidates are the subjects on the relationships the permission's rewrite reaches from the
 * resource (a walk on the device), each checked on the check path; a wildcard grant is reported
 * once, as GCK_ID_WILDCARD (last), not as every subject of the type. */
int gck_lookup_subjects(gck_engine* e, const gck_consistency* cs, uint16_t resource_type, uint32_t resource_id,
                        uint16_t permission, uint16_t subject_type, uint16_t subject_relation, int64_t now_us,
                        uint32_t* out_ids, uint8_t* out_perm, size_t cap, size_t* out_n);

/* ---- partitioned graphs (graphs above one GPU's 288 GB) ----------------
 * Rank r of `world` (one process per GPU) owns the objects whose names hash to it
 * (gck_partition_owner_name, below: decided from the name, before anything is interned; the
 * owner gives the id, local * world + r, so gck_partition_owner(id) = id mod world names the same
 * rank). Every rank reads the whole export / Watch stream and keeps only (every ingest path
 * filters — gck_part_add_tuples_text_with, gck_add_tuples, gck_load_csr, gck_apply_updates —
 * none stores another rank's rows):
 *   - the relationships of the objects it owns;
 *   - the schema's hub hierarchy (the userset and wildcard relationships of "hub" relations —
 *     nested groups, teams — which usersets and arrows point at and which allow no caveat or
 *     expiration), replicated;
 *   - the direct hub memberships of the subjects it owns (their side of the label join: a hub
 *     membership goes to its subject's owner, not its object's).
 * All ranks then check one batch together — every rank calls with the same items and gets every
 * result: the label join (a subject's owner sends its slot to the resource's owner, which decides
 * the check), then an exact-depth level loop over what it left, with intersection, exclusion,
 * all() and caveats, exchanging frontier entries and join state per level. The exchange goes over
 * RCCL inside libgck (gck_part_init + gck_part_check) or over the caller's transport
 * (gck_part_check_with). Check-time caveat contexts are not taken in this mode. A partitioned
 * engine refuses gck_check_bulk*, lookups and snapshot files. */
/* Before the first snapshot: this engine is rank `rank` of `world` (1 = not partitioned). */
int gck_set_partition(gck_engine* e, uint32_t rank, uint32_t world);
uint32_t gck_partition_owner(uint32_t object_id, uint32_t world);

/* A caller's exchange between the ranks of a partition. Device buffers on the engine's device,
 * ordered on `stream` (the engine's work before the call is on it; the engine reads `recv` after
 * the call, on it): the transport may enqueue the transfer there (RCCL) or synchronise the stream
 * and complete it before returning (a host-staged transport).
 *   alltoallv: this rank sends send_bytes[d] bytes to rank d and receives recv_bytes[s] bytes
 *     from rank s; the blocks lie back to back in rank order in `send` and `recv` (the engine
 *     passes 0 for itself). Both sides know the sizes: the engine exchanges them first.
 *   allreduce_max_u8: in place, element-wise MAX over the ranks of n bytes.
 * Each returns 0, or non-zero on failure (the check then fails with GCK_E_DEVICE). */
typedef struct gck_transport {
  void* ctx;
  int (*alltoallv)(void* ctx, const void* d_send, const uint64_t* send_bytes, void* d_recv,
                   const uint64_t* recv_bytes, void* stream);
  int (*allreduce_max_u8)(void* ctx, void* d_buf, uint64_t n, void* stream);
} gck_transport;

/* Object names on a partitioned engine (world > 1; SURVEY.md §8e: owner = hash(type, id) mod G).
 * A name's owner is gck_partition_owner_name(type, name) — FNV-1a over the type (2 bytes, little
 * endian) and the name's bytes, finalised, mod world — decided before anything is interned, and
 * only the owner gives it an id: local * world + owner, in the order the owner meets its names, so
 * that gck_partition_owner(id) is the same rank and every rank holds the same id for a name. A rank
 * keeps only the names of what it owns and of what its rows and checks reference (the replicated
 * hub hierarchy among them); local interning of a new name (gck_intern with GCK_INTERN_CREATE,
 * gck_add_tuples_text, gck_apply_updates_text) is refused with GCK_E_STATE on such an engine.
 * Both calls below are collective: every rank of the partition calls them, in the same order. */
uint32_t gck_partition_owner_name(uint16_t type, const char* name, size_t len, uint32_t world);
/* Every rank its own names (types[i], names[i] of lens[i] bytes) -> out_ids[i]: "*" is
 * GCK_ID_WILDCARD; a name the owner does not know is created with GCK_INTERN_CREATE, else
 * GCK_ID_ABSENT (check items: build them with this, so that every rank has the same items). With
 * GCK_INTERN_CREATE every rank's object counts become world x the largest owner's count. */
int gck_part_intern_with(gck_engine* e, const gck_transport* t, const uint16_t* types, const char* const* names,
                         const uint32_t* lens, size_t n, uint32_t flags, uint32_t* out_ids);
/* The export stream's relationships as text (gck_add_tuples_text's format), the same text on every
 * rank, between gck_begin_snapshot and gck_commit_snapshot: each rank keeps what it owns (decided
 * from the names) and interns the names of those relationships only, through their owners. */
int gck_part_add_tuples_text_with(gck_engine* e, const gck_transport* t, const char* text, size_t len);
/* The names this engine's interner holds for a type (on a partitioned engine: its own objects'
 * and those its rows and checks referenced; otherwise every named object). */
int gck_interned_names(gck_engine* e, uint16_t type, uint32_t* out);

/* The partitioned check over the caller's transport: n device items (the same on every rank) in,
 * every result out on every rank (d_out_perm / d_out_err, device). `now_us` 0 = rank 0's clock. */
int gck_part_check_with(gck_engine* e, const gck_transport* t, const gck_item* d_items, size_t n, int64_t now_us,
                        uint8_t* d_out_perm, int32_t* d_out_err, void* stream);

/* The same over RCCL inside libgck (xGMI between the GPUs of a node: grouped ncclSend / ncclRecv,
 * ncclAllReduce). Rank 0 makes the id (gck_part_unique_id), the caller hands the same bytes to
 * every rank (any transport: a TCP store, MPI, a file), and each rank joins with gck_part_init
 * after gck_set_partition. */
#define GCK_PART_UNIQUE_ID_BYTES 128
int gck_part_unique_id(uint8_t out[GCK_PART_UNIQUE_ID_BYTES]);
int gck_part_init(gck_engine* e, const uint8_t id[GCK_PART_UNIQUE_ID_BYTES]);
int gck_part_check(gck_engine* e, const gck_item* d_items, size_t n, int64_t now_us, uint8_t* d_out_perm,
                   int32_t* d_out_err, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GCK_H */

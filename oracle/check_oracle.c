/*
 * check_oracle.c — TEST INFRASTRUCTURE ONLY. C restatement of SpiceDB's check dispatch used
 * as (a) the scale parity checker for the HIP engine and (b) bench.py's cpu_baseline
 * ("kind": "port"). Nothing in gochugaru_amd/ links or loads this file.
 *
 * Restates the same rules as oracle/spicedb_ref.py, recursively and
 * depth-first like SpiceDB's dispatcher:
 *   dispatch()      — depth budget (dispatch.CheckDepth) + identity filter
 *                     (filterForFoundMemberResource)                     SURVEY §5.1 items 3, 9
 *   check_direct()  — exact subject / wildcard / userset re-dispatch (checkDirect) §5.1 item 3
 *   eval()          — union / intersection / exclusion / computed userset / arrows / nil
 *                                                                         §5.1 items 4-6
 * Tri-state algebra as spicedb_ref.py: union Y > ERR > C > N; intersection N > ERR > C > Y;
 * exclusion N if base N or a subtracted Y, else ERR, else C, else Y. Caveated edges are
 * CONDITIONAL, except under orc_check_quota, which restates one caveat family in C — the
 * threshold `value < limit` (limit stored per relationship, value per check context) — so that
 * large per-relationship x per-request caveat workloads have a scale checker; a caveat that
 * fails to evaluate on a check's walk makes the item GCK_ITEM_ERR_CAVEAT_EVAL (6).
 *
 * Parity pinning: cross-checked against spicedb_ref.py (itself pinned by the reference's
 * known answers, tests/golden) on seeded graphs in tests/test_c_oracle.py.
 *
 * Per-check memo, exact under the depth budget: for a fixed check, dispatch(v, d) is a pure
 * function of the vertex v and the remaining depth d, and it is monotone in d — once it is not
 * ERR at some d it keeps that value at every larger d (by induction over the tri-state algebra:
 * only an ERR operand can change when the budget grows, and a non-ERR result never depends on
 * an ERR operand). So the memo keeps, per vertex, the non-ERR value with the smallest depth it
 * was seen at and the largest depth seen to give ERR, and answers a lookup at d from whichever
 * bound covers d. Cyclic and re-converging data stay polynomial (|vertices| x depth).
 *
 * Input: a relation/permission program (int32 stream, built by oracle/corc.py from the
 * oracle's own schema parser) and per-(relation, subject kind) CSR arrays.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NO 1
#define HAS 2
#define COND 3
#define ERR 15
#define ELLIPSIS 0xFFFFu
#define WILDCARD 0xFFFFFFFFu
#define ABSENT 0xFFFFFFFEu

/* program opcodes */
#define OP_UNION 1
#define OP_INTER 2
#define OP_EXCL 3
#define OP_NIL 4
#define OP_COMP 5
#define OP_ARROW 6

typedef struct {
  const uint32_t* off;
  const uint32_t* nbr;
  const uint32_t* cav; /* NULL for plain */
  const int64_t* exp;  /* NULL for plain */
  uint32_t n_rows;
  uint32_t pad;
} orc_csr;

typedef struct { /* == gck_item */
  uint16_t resource_type, permission;
  uint32_t resource_id;
  uint16_t subject_type, subject_relation;
  uint32_t subject_id, context_slot;
} orc_item;

typedef struct {
  const int32_t* prog;
  const int32_t* rel_at; /* offset of each relation's record */
  int32_t n_types, n_rels;
  const orc_csr* csrs;
  int64_t now_us;
  int max_depth;
  /* threshold caveats (orc_check_quota): edge cav id k > 0 holds while the check's value is
     below limit[k]; the value of context slot s is used[s - 1] (INT64_MIN: the context gives the
     parameter a wrong type, an evaluation error); slot 0 leaves the caveat unresolved. NULL
     limit: every caveated edge is unresolved (CONDITIONAL). */
  const int64_t* cav_limit;
  const int64_t* cav_used;
  uint32_t n_slots;
} orc_program;

typedef struct {
  /* memo: open addressing keyed by (rel, obj) with a generation stamp */
  uint64_t* keys;
  uint32_t* gen;
  uint8_t* val;  /* non-ERR value (0 = none known) */
  uint8_t* okd;  /* ... known from this remaining depth upwards */
  uint8_t* errd; /* ERR known at every remaining depth <= errd (0 = none known) */
  uint32_t cap, mask, cur_gen, used;
  /* subject */
  uint32_t sid;
  uint16_t stype, srel;
  uint32_t slot;  /* the check's context slot */
  int cav_err;    /* the walk met a caveat that failed to evaluate */
  uint64_t rows, probes, edges;
} orc_ctx;

static int union3(int a, int b) {
  if (a == HAS || b == HAS) return HAS;
  if (a == ERR || b == ERR) return ERR;
  if (a == COND || b == COND) return COND;
  return NO;
}

/* a caveated edge conditions what it reaches: spicedb_ref.and3 over the caveat's outcome */
static int and3(int cav, int sub) {
  if (sub == ERR) return ERR;
  if (cav == HAS) return sub;
  if (cav == NO || sub == NO) return NO;
  return COND;
}

static int rel_type(const orc_program* p, int r) { return p->prog[p->rel_at[r]]; }
static int rel_is_perm(const orc_program* p, int r) { return p->prog[p->rel_at[r] + 1]; }

static uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

/* the memo answer for (key, remaining depth dr): a value, ERR, or 0 = unknown */
static int memo_get(orc_ctx* c, uint64_t key, int dr) {
  uint32_t h = (uint32_t)mix64(key) & c->mask;
  for (;;) {
    if (c->gen[h] != c->cur_gen) return 0;
    if (c->keys[h] == key) {
      if (c->val[h] && dr >= c->okd[h]) return c->val[h];
      if (dr <= c->errd[h]) return ERR;
      return 0;
    }
    h = (h + 1) & c->mask;
  }
}

static void memo_put(orc_ctx* c, uint64_t key, int v, int dr) {
  uint32_t h = (uint32_t)mix64(key) & c->mask;
  while (c->gen[h] == c->cur_gen) {
    if (c->keys[h] == key) break;
    h = (h + 1) & c->mask;
  }
  if (c->gen[h] != c->cur_gen) {
    if (c->used * 2 >= c->cap) return; /* full enough: stop adding keys for this check */
    c->gen[h] = c->cur_gen;
    c->keys[h] = key;
    c->val[h] = 0;
    c->okd[h] = 255;
    c->errd[h] = 0;
    c->used++;
  }
  if (dr > 255) dr = 255;
  if (v == ERR) {
    if (dr > c->errd[h]) c->errd[h] = (uint8_t)dr;
  } else if (!c->val[h] || dr < c->okd[h]) {
    c->val[h] = (uint8_t)v;
    c->okd[h] = (uint8_t)dr;
  }
}

static int row_find(orc_ctx* c, const orc_csr* r, uint32_t obj, uint32_t sid, uint32_t* pos) {
  if (obj >= r->n_rows) return 0;
  uint32_t lo = r->off[obj], hi = r->off[obj + 1], end = hi;
  c->rows++;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    c->probes++;
    if (r->nbr[mid] < sid) lo = mid + 1;
    else hi = mid;
  }
  if (lo < end && r->nbr[lo] == sid) {
    *pos = lo;
    return 1;
  }
  return 0;
}

static int visible(const orc_program* p, const orc_csr* r, uint32_t pos) {
  return !r->exp || r->exp[pos] == 0 || r->exp[pos] > p->now_us;
}

/* the outcome of edge pos's caveat for the current check: HAS (no caveat, or it holds), NO
   (it fails) or COND (unresolved) */
static int cav_at(const orc_program* p, orc_ctx* c, const orc_csr* r, uint32_t pos) {
  if (!r->cav || !r->cav[pos]) return HAS;
  if (!p->cav_limit || c->slot == 0 || c->slot > p->n_slots) return COND;
  int64_t u = p->cav_used[c->slot - 1];
  if (u == INT64_MIN) {
    c->cav_err = 1;
    return COND;
  }
  return u < p->cav_limit[r->cav[pos]] ? HAS : NO;
}

static int dispatch(const orc_program* p, orc_ctx* c, int type, uint32_t obj, int rel, int dr);

static int computed(const orc_program* p, orc_ctx* c, int type, uint32_t obj, int rel, int dr) {
  if (rel < 0) return NO; /* TTU target missing on this subject type */
  if (type == c->stype && rel == c->srel && obj == c->sid) return HAS;
  return dispatch(p, c, type, obj, rel, dr - 1);
}

/* relation record: type, is_perm=0, n_kinds, (stype, srel, csr_plain, csr_ext)* */
static int check_direct(const orc_program* p, orc_ctx* c, int rel, uint32_t obj, int dr) {
  const int32_t* rec = p->prog + p->rel_at[rel];
  int nk = rec[2];
  int acc = NO;
  /* pass 1: the subject itself / wildcard */
  for (int k = 0; k < nk; ++k) {
    int stype = rec[3 + 4 * k], srel = rec[4 + 4 * k];
    if (stype != c->stype) continue;
    int direct = srel == c->srel, wild = srel == (int)ELLIPSIS && c->srel == ELLIPSIS;
    if (!direct && !wild) continue;
    for (int pass = 0; pass < 2; ++pass) {
      int ci = rec[5 + 4 * k + pass];
      if (ci < 0) continue;
      const orc_csr* r = &p->csrs[ci];
      uint32_t pos;
      if (direct && row_find(c, r, obj, c->sid, &pos) && visible(p, r, pos)) {
        int v = and3(cav_at(p, c, r, pos), HAS);
        acc = union3(acc, v);
        if (acc == HAS) return HAS;
      }
      if (wild && obj < r->n_rows) {
        uint32_t b = r->off[obj], e = r->off[obj + 1];
        c->probes++;
        if (e > b && r->nbr[e - 1] == WILDCARD && visible(p, r, e - 1)) {
          acc = union3(acc, and3(cav_at(p, c, r, e - 1), HAS));
          if (acc == HAS) return HAS;
        }
      }
    }
  }
  /* pass 2: usersets are re-dispatched */
  for (int k = 0; k < nk; ++k) {
    int stype = rec[3 + 4 * k], srel = rec[4 + 4 * k];
    if (srel == (int)ELLIPSIS) continue;
    for (int pass = 0; pass < 2; ++pass) {
      int ci = rec[5 + 4 * k + pass];
      if (ci < 0) continue;
      const orc_csr* r = &p->csrs[ci];
      if (obj >= r->n_rows) continue;
      c->rows++;
      for (uint32_t e = r->off[obj]; e < r->off[obj + 1]; ++e) {
        c->edges++;
        if (!visible(p, r, e)) continue;
        uint32_t x = r->nbr[e];
        if (x == WILDCARD) continue;
        int sub = dispatch(p, c, stype, x, srel, dr - 1);
        acc = union3(acc, and3(cav_at(p, c, r, e), sub));
        if (acc == HAS) return HAS;
      }
    }
  }
  return acc;
}

/* evaluates the expression at *pc, advancing *pc past it */
static int eval(const orc_program* p, orc_ctx* c, const int32_t** pc, int type, uint32_t obj, int dr);

static void skip(const int32_t** pc) {
  int op = *(*pc)++;
  switch (op) {
    case OP_UNION:
    case OP_INTER:
    case OP_EXCL: {
      int n = *(*pc)++;
      for (int i = 0; i < n; ++i) skip(pc);
      break;
    }
    case OP_NIL:
      break;
    case OP_COMP:
      (*pc)++;
      break;
    case OP_ARROW: {
      (*pc) += 2;
      int nt = *(*pc)++;
      (*pc) += 2 * nt;
      break;
    }
  }
}

static int eval(const orc_program* p, orc_ctx* c, const int32_t** pc, int type, uint32_t obj, int dr) {
  int op = *(*pc)++;
  switch (op) {
    case OP_UNION: {
      int n = *(*pc)++, acc = NO, i = 0;
      for (; i < n; ++i) {
        acc = union3(acc, eval(p, c, pc, type, obj, dr));
        if (acc == HAS) {
          ++i;
          break;
        }
      }
      for (; i < n; ++i) skip(pc);
      return acc;
    }
    case OP_INTER: {
      int n = *(*pc)++, any_err = 0, any_c = 0, no = 0, i = 0;
      for (; i < n; ++i) {
        int v = eval(p, c, pc, type, obj, dr);
        if (v == NO) {
          no = 1;
          ++i;
          break;
        }
        if (v == ERR) any_err = 1;
        if (v == COND) any_c = 1;
      }
      for (; i < n; ++i) skip(pc);
      return no ? NO : any_err ? ERR : any_c ? COND : HAS;
    }
    case OP_EXCL: {
      int n = *(*pc)++, i = 1;
      int base = eval(p, c, pc, type, obj, dr);
      int any_err = base == ERR, any_c = base == COND, no = base == NO;
      for (; i < n && !no; ++i) {
        int v = eval(p, c, pc, type, obj, dr);
        if (v == HAS) no = 1;
        if (v == ERR) any_err = 1;
        if (v == COND) any_c = 1;
      }
      for (; i < n; ++i) skip(pc);
      return no ? NO : any_err ? ERR : any_c ? COND : HAS;
    }
    case OP_NIL:
      return NO;
    case OP_COMP: {
      int rel = *(*pc)++;
      return computed(p, c, type, obj, rel, dr);
    }
    case OP_ARROW: {
      /* tupleset relation, is_all, n_targets, (stype, target_rel)* */
      int ts = *(*pc)++, is_all = *(*pc)++, nt = *(*pc)++;
      const int32_t* tg = *pc;
      (*pc) += 2 * nt;
      const int32_t* rec = p->prog + p->rel_at[ts];
      int nk = rec[2];
      int acc = is_all ? HAS : NO, seen = 0, any_err = 0, any_c = 0;
      for (int k = 0; k < nk; ++k) {
        int stype = rec[3 + 4 * k];
        int target = -1;
        for (int t = 0; t < nt; ++t)
          if (tg[2 * t] == stype) target = tg[2 * t + 1];
        for (int pass = 0; pass < 2; ++pass) {
          int ci = rec[5 + 4 * k + pass];
          if (ci < 0) continue;
          const orc_csr* r = &p->csrs[ci];
          if (obj >= r->n_rows) continue;
          c->rows++;
          for (uint32_t e = r->off[obj]; e < r->off[obj + 1]; ++e) {
            c->edges++;
            if (!visible(p, r, e)) continue;
            int v = and3(cav_at(p, c, r, e), computed(p, c, stype, r->nbr[e], target, dr));
            seen = 1;
            if (is_all) {
              if (v == NO) return NO;
              if (v == ERR) any_err = 1;
              if (v == COND) any_c = 1;
            } else {
              acc = union3(acc, v);
              if (acc == HAS) return HAS;
            }
          }
        }
      }
      if (is_all) return !seen ? NO : any_err ? ERR : any_c ? COND : HAS;
      return acc;
    }
  }
  return ERR;
}

static int dispatch(const orc_program* p, orc_ctx* c, int type, uint32_t obj, int rel, int dr) {
  if (dr <= 0) return ERR;
  if (type == c->stype && rel == c->srel && obj == c->sid) return HAS;
  uint64_t key = ((uint64_t)(uint32_t)rel << 32) | obj;
  int m = memo_get(c, key, dr);
  if (m) return m;
  int v;
  if (rel_is_perm(p, rel)) {
    const int32_t* pc = p->prog + p->rel_at[rel] + 3;
    v = eval(p, c, &pc, type, obj, dr);
  } else {
    v = check_direct(p, c, rel, obj, dr);
  }
  memo_put(c, key, v, dr);
  return v;
}

static int validate(const orc_program* p, const orc_item* it) {
  if (it->resource_type >= p->n_types || it->subject_type >= p->n_types) return 3;
  if (it->permission >= p->n_rels || rel_type(p, it->permission) != it->resource_type) return 2;
  if (it->subject_relation != ELLIPSIS &&
      (it->subject_relation >= p->n_rels || rel_type(p, it->subject_relation) != it->subject_type))
    return 4;
  if (it->subject_id == WILDCARD) return 5;
  return 0;
}

/* Program layout: [n_types, n_rels, rel_off[n_rels]..., records...]. */
int orc_check_quota(const int32_t* prog, const orc_csr* csrs, const orc_item* items, size_t n,
                    int64_t now_us, int max_depth, int threads, uint8_t* out_perm, int32_t* out_err,
                    uint64_t* counters /* [rows, probes, edges] or NULL */, const int64_t* cav_limit,
                    const int64_t* cav_used, uint32_t n_slots) {
  orc_program p;
  p.cav_limit = cav_limit;
  p.cav_used = cav_used;
  p.n_slots = n_slots;
  p.n_types = prog[0];
  p.n_rels = prog[1];
  p.rel_at = prog + 2;
  p.prog = prog;
  p.csrs = csrs;
  p.now_us = now_us;
  p.max_depth = max_depth > 0 ? max_depth : 50;
  uint64_t rows = 0, probes = 0, edges = 0;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel reduction(+ : rows, probes, edges)
#endif
  {
    orc_ctx c;
    memset(&c, 0, sizeof c);
    c.cap = 1u << 20;
    c.mask = c.cap - 1;
    c.keys = (uint64_t*)malloc(sizeof(uint64_t) * c.cap);
    c.gen = (uint32_t*)calloc(c.cap, sizeof(uint32_t));
    c.val = (uint8_t*)malloc(c.cap);
    c.okd = (uint8_t*)malloc(c.cap);
    c.errd = (uint8_t*)malloc(c.cap);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 64)
#endif
    for (long i = 0; i < (long)n; ++i) {
      const orc_item* it = &items[i];
      int e = validate(&p, it);
      out_err[i] = e;
      out_perm[i] = 0;
      if (e) continue;
      c.cur_gen++;
      if (c.cur_gen == 0) {
        memset(c.gen, 0, sizeof(uint32_t) * c.cap);
        c.cur_gen = 1;
      }
      c.used = 0;
      c.sid = it->subject_id;
      c.stype = it->subject_type;
      c.srel = it->subject_relation;
      c.slot = it->context_slot;
      c.cav_err = 0;
      int v = dispatch(&p, &c, it->resource_type, it->resource_id, it->permission, p.max_depth);
      if (c.cav_err) {
        out_err[i] = 6; /* GCK_ITEM_ERR_CAVEAT_EVAL */
      } else if (v == ERR) {
        out_err[i] = 1;
      } else {
        out_perm[i] = (uint8_t)v;
      }
    }
    rows += c.rows;
    probes += c.probes;
    edges += c.edges;
    free(c.keys);
    free(c.gen);
    free(c.val);
    free(c.okd);
    free(c.errd);
  }
  if (counters) {
    counters[0] = rows;
    counters[1] = probes;
    counters[2] = edges;
  }
  return 0;
}

int orc_check(const int32_t* prog, const orc_csr* csrs, const orc_item* items, size_t n,
              int64_t now_us, int max_depth, int threads, uint8_t* out_perm, int32_t* out_err,
              uint64_t* counters) {
  return orc_check_quota(prog, csrs, items, n, now_us, max_depth, threads, out_perm, out_err, counters, NULL,
                         NULL, 0);
}

/*
 * Counting mode for union-only programs (SURVEY.md §8d rule): level-synchronous BFS per
 * check, memoised per check (each (relation, object) expanded at most once), stopping at the
 * end of the first level at which the check is decided. Counts the implementation-
 * independent work: rows opened (8-B offset pairs), membership probes (4-B reads of a binary
 * search) and userset/arrow edges enumerated (4-B reads). Returns -1 if the program has a
 * join (intersection / exclusion / all()).
 */
typedef struct {
  uint32_t obj;
  int32_t rel;
} orc_node;

int orc_count_bfs(const int32_t* prog, const orc_csr* csrs, const orc_item* items, size_t n,
                  int threads, uint64_t* counters /* rows, probes, edges, expanded, levels */) {
  orc_program p;
  p.n_types = prog[0];
  p.n_rels = prog[1];
  p.rel_at = prog + 2;
  p.prog = prog;
  p.csrs = csrs;
  p.now_us = 0;
  p.max_depth = 50;
  uint64_t rows = 0, probes = 0, edges = 0, expanded = 0, levels = 0;
  int bad = 0;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel reduction(+ : rows, probes, edges, expanded, levels) reduction(| : bad)
#endif
  {
    orc_ctx c;
    memset(&c, 0, sizeof c);
    c.cap = 1u << 22;
    c.mask = c.cap - 1;
    c.keys = (uint64_t*)malloc(sizeof(uint64_t) * c.cap);
    c.gen = (uint32_t*)calloc(c.cap, sizeof(uint32_t));
    c.val = (uint8_t*)malloc(c.cap);
    c.okd = (uint8_t*)malloc(c.cap);
    c.errd = (uint8_t*)malloc(c.cap);
    size_t fcap = 1 << 16;
    orc_node* cur = (orc_node*)malloc(sizeof(orc_node) * fcap);
    orc_node* nxt = (orc_node*)malloc(sizeof(orc_node) * fcap);
    size_t ncap = fcap;
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 64)
#endif
    for (long i = 0; i < (long)n; ++i) {
      const orc_item* it = &items[i];
      if (validate(&p, it)) continue;
      c.cur_gen++;
      c.used = 0;
      c.sid = it->subject_id;
      c.stype = it->subject_type;
      c.srel = it->subject_relation;
      size_t nc = 0, nn = 0;
      cur[nc++] = (orc_node){it->resource_id, it->permission};
      int found = 0;
      for (int lvl = 0; nc && !found && lvl < 50; ++lvl) {
        levels++;
        nn = 0;
        for (size_t k = 0; k < nc && !bad; ++k) {
          orc_node nd = cur[k];
          expanded++;
          int type = rel_type(&p, nd.rel);
          if (type == c.stype && nd.rel == c.srel && nd.obj == c.sid) {
            found = 1;
            continue;
          }
          const int32_t* rec = p.prog + p.rel_at[nd.rel];
#define PUSH(o, r)                                                           \
  do {                                                                       \
    uint64_t key_ = ((uint64_t)(uint32_t)(r) << 32) | (o);                   \
    if (!memo_get(&c, key_, 255)) {                                          \
      memo_put(&c, key_, 1, 0);                                              \
      if (nn == ncap) {                                                      \
        ncap *= 2;                                                           \
        nxt = (orc_node*)realloc(nxt, sizeof(orc_node) * ncap);              \
        cur = (orc_node*)realloc(cur, sizeof(orc_node) * ncap);              \
      }                                                                      \
      nxt[nn++] = (orc_node){(o), (r)};                                      \
    }                                                                        \
  } while (0)
          if (!rec[1]) {
            int nk = rec[2], hit = 0;
            for (int q = 0; q < nk && !hit; ++q) { /* pass 1: membership */
              int ci = rec[5 + 4 * q];
              uint32_t pos;
              if (ci >= 0 && rec[3 + 4 * q] == c.stype && rec[4 + 4 * q] == c.srel &&
                  row_find(&c, &p.csrs[ci], nd.obj, c.sid, &pos))
                hit = 1;
            }
            if (hit) {
              found = 1;
              continue;
            }
            for (int q = 0; q < nk; ++q) { /* pass 2: usersets */
              int srel = rec[4 + 4 * q];
              int ci = rec[5 + 4 * q];
              if (ci < 0) continue;
              const orc_csr* r = &p.csrs[ci];
              if (srel != (int)ELLIPSIS && nd.obj < r->n_rows) {
                rows++;
                for (uint32_t e = r->off[nd.obj]; e < r->off[nd.obj + 1]; ++e) {
                  edges++;
                  PUSH(r->nbr[e], srel);
                }
              }
            }
          } else {
            const int32_t* pc = rec + 3;
            int op = *pc++;
            int nchild = 1;
            if (op == OP_UNION) nchild = *pc++;
            else pc--;
            for (int q = 0; q < nchild; ++q) {
              int cop = *pc++;
              if (cop == OP_COMP) {
                int rr = *pc++;
                PUSH(nd.obj, rr);
              } else if (cop == OP_ARROW) {
                int ts = *pc++;
                pc++; /* is_all */
                int nt = *pc++;
                const int32_t* tg = pc;
                pc += 2 * nt;
                const int32_t* trec = p.prog + p.rel_at[ts];
                for (int k = 0; k < trec[2]; ++k) {
                  int ci = trec[5 + 4 * k];
                  int target = -1;
                  for (int t = 0; t < nt; ++t)
                    if (tg[2 * t] == trec[3 + 4 * k]) target = tg[2 * t + 1];
                  if (ci < 0 || target < 0) continue;
                  const orc_csr* r = &p.csrs[ci];
                  if (nd.obj >= r->n_rows) continue;
                  rows++;
                  for (uint32_t e = r->off[nd.obj]; e < r->off[nd.obj + 1]; ++e) {
                    edges++;
                    PUSH(r->nbr[e], target);
                  }
                }
              } else if (cop == OP_NIL) {
              } else {
                bad = 1;
              }
            }
          }
        }
        orc_node* t = cur;
        cur = nxt;
        nxt = t;
        nc = nn;
      }
    }
    rows += c.rows;
    probes += c.probes;
    free(c.keys);
    free(c.gen);
    free(c.val);
    free(c.okd);
    free(c.errd);
    free(cur);
    free(nxt);
  }
  if (counters) {
    counters[0] = rows;
    counters[1] = probes;
    counters[2] = edges;
    counters[3] = expanded;
    counters[4] = levels;
  }
  return bad ? -1 : 0;
}

/* raftref.c — CPU oracle (and CPU baseline) for the batched Raft simulator.
 * TEST INFRASTRUCTURE ONLY: see raftref.h. Semantics: SIM_SPEC.md; every handler cites the
 * reference line it restates. Clusters are independent, so raft_ref_step maps over contiguous
 * cluster chunks with one pthread each (the `pmap` analogue of SURVEY.md §8d) and runs each
 * cluster's ticks back to back.
 */
#include "raftref.h"

typedef struct shard shard_t;
static void sh_destroy(shard_t* s);

#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static __thread char g_err[256];
static int fail(int code, const char* msg) {
  snprintf(g_err, sizeof g_err, "%s", msg);
  return code;
}
const char* raft_ref_last_error(void) { return g_err; }

/* ---------------------------------------------------------------- Philox4x32-10 (SIM_SPEC §5) */
enum { P_INIT = 1, P_EVENT = 2, P_NET = 3, P_CLIENT = 4, P_PART = 6 };

void raft_ref_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3], k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n1 = (uint32_t)p1;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1, n3 = (uint32_t)p0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static void draw(const shard_t* s, uint32_t g, uint32_t nodep, uint32_t t, uint32_t x,
                 uint32_t w[4]);
static uint32_t ppm(uint32_t w) { return (uint32_t)(((uint64_t)w * 1000000u) >> 32); }

/* pw_i = (1-p)^(2^i) in 32-bit fixed point, truncating (SIM_SPEC §4 P0). */
static void client_powers(uint32_t client_ppm, uint64_t pw[32]) {
  pw[0] = ((uint64_t)(1000000u - client_ppm) << 32) / 1000000u;
  for (int i = 1; i < 32; ++i)   /* exact: 2^32 squared (client_ppm = 0) stays 2^32 */
    pw[i] = pw[i - 1] == 1ull << 32 ? pw[i - 1] : (pw[i - 1] * pw[i - 1]) >> 32;
}

/* Geometric gap: greedy search for the largest G with (1-p)^G >= (w+1)/2^32. */
static uint64_t client_gap(uint32_t w, const uint64_t pw[32]) {
  uint64_t u = (uint64_t)w + 1, acc = 1ull << 32, g = 0;
  for (int i = 31; i >= 0; --i) {
    /* exact floor(acc * pw_i / 2^32): both factors are <= 2^32 and equal it together only when
     * client_ppm = 0 (pw_i = 2^32), where the 64-bit product would wrap */
    uint64_t c = acc == 1ull << 32 ? pw[i] : (acc * pw[i]) >> 32;
    if (c >= u) { acc = c; g += 1ull << i; }
  }
  return g;
}

static uint32_t sat_tick(uint64_t x) { return x < 0xFFFFFFFFull ? (uint32_t)x : 0xFFFFFFFFu; }

/* Client schedule (SIM_SPEC §4 P0): bursts of B on-ticks at the start of every period P (P = 0:
 * every tick is on). on_index numbers the on-ticks, on_tick maps a number back to its tick. */
static uint64_t on_index(uint64_t t, uint32_t P, uint32_t B) {
  return P ? (t / P) * B + t % P : t;
}
static uint32_t on_tick(uint64_t j, uint32_t P, uint32_t B) {
  return sat_tick(P ? (j / B) * P + j % B : j);
}

/* ---------------------------------------------------------------- FNV-1a-64 over u32 words */
#define FNV_OFFSET 0xCBF29CE484222325ull
#define FNV_PRIME 0x100000001B3ull
static uint64_t fnv(uint64_t h, uint32_t w) { return (h ^ w) * FNV_PRIME; }
/* the trace hash's multiplier (SIM_SPEC §4): odd, so each step is a bijection of h */
#define TRACE_M 0x9E3779B97F4A7C15ull

/* ---------------------------------------------------------------- simulator state */
struct shard {
  raft_sim_config_t cfg;
  uint32_t N, Q, L, A, C;
  uint32_t key[2];
  uint64_t tick;
  raft_node_t* nodes;   /* [C*N] */
  raft_msg_t* q;        /* [C*N][2][Q], index 0 = head */
  raft_entry_t* arena;  /* [C*N][A] */
  raft_cluster_t* cl;   /* [C] */
  uint32_t* stream;     /* [C*N][S] commit-stream rings (F2), S = commit_stream_cap */
  uint32_t S;
  raft_trace_event_t* tr; /* [C*N][TC] wait-event rings (F3) */
  uint32_t* tcount;       /* [C*N] events recorded per node */
  raft_entry_t* tent;     /* [C*N][TE] :entries carried by recorded append-entries */
  uint32_t* tecount;      /* [C*N] */
  uint32_t TC, TE;
  raft_counters_t ctr;
  int threads;
  int idle_skip;   /* jump over ticks at which no node of a cluster can act (same results) */
  uint64_t client_pw[32];
};

static void draw(const shard_t* s, uint32_t g, uint32_t nodep, uint32_t t, uint32_t x,
                 uint32_t w[4]) {
  uint32_t ctr[4] = {g, nodep, t, x};
  raft_ref_philox(ctr, s->key, w);
}

void raft_ref_default_config(raft_sim_config_t* c) {
  memset(c, 0, sizeof *c);
  c->n_clusters = 1; c->nodes = 5; c->log_cap = 64; c->inbox_cap = 16; c->seed = 42;
  c->hb = 3000; c->el_base = 5000; c->el_span = 5000; c->dmin = 1; c->dmax = 1;
  c->part_epoch = 1000; c->n_devices = 1;
}

static raft_msg_t* qslot(shard_t* s, uint32_t gi, int which) {
  return s->q + ((size_t)gi * 2 + which) * s->Q;
}
static raft_entry_t* arena_of(shard_t* s, uint32_t gi) { return s->arena + (size_t)gi * s->A; }

static int validate_cfg(const raft_sim_config_t* c) {
  if (c->nodes < 2 || c->nodes > RAFT_MAX_NODES) return fail(-EINVAL, "nodes must be 2..9");
  if (c->n_clusters == 0) return fail(-EINVAL, "n_clusters must be > 0");
  if (c->inbox_cap < 1 || c->inbox_cap > RAFT_MAX_INBOX) return fail(-EINVAL, "inbox_cap 1..16");
  if (c->log_cap < 1 || c->log_cap > 65535) return fail(-EINVAL, "log_cap 1..65535");
  uint64_t A = c->arena_cap ? c->arena_cap : 4ull * c->log_cap;
  if (A < 2ull * c->log_cap || A > (1u << 24)) return fail(-EINVAL, "arena_cap must be >= 2*log_cap");
  if (c->hb < 1 || c->el_base < 1) return fail(-EINVAL, "hb and el_base must be >= 1");
  if (c->dmin < 1 || c->dmax < c->dmin || c->dmax > 255) return fail(-EINVAL, "1 <= dmin <= dmax <= 255");
  if (c->part_epoch < 1) return fail(-EINVAL, "part_epoch must be >= 1");
  if (c->drop_ppm > 1000000 || c->dup_ppm > 1000000 || c->part_ppm > 1000000 ||
      c->client_ppm > 1000000) return fail(-EINVAL, "ppm values must be <= 1e6");
  if (c->variant_flags & ~3u) return fail(-EINVAL, "variant_flags: only bits 0-1 are defined");
  if (c->trace_cap > (1u << 20) || c->trace_entry_cap > (1u << 24))
    return fail(-EINVAL, "trace_cap <= 2^20, trace_entry_cap <= 2^24");
  if ((uint64_t)c->cluster_offset + c->n_clusters > (1ull << 32))
    return fail(-EINVAL, "cluster_offset + n_clusters must be <= 2^32");
  if ((uint64_t)c->nodes * c->nodes * c->n_clusters >= (1ull << 31))
    return fail(-EINVAL, "nodes^2 * n_clusters must be < 2^31");
  if (c->client_period && (c->client_burst < 1 || c->client_burst > c->client_period))
    return fail(-EINVAL, "client_burst must be 1..client_period");
  if (c->client_redirects > 16) return fail(-EINVAL, "client_redirects <= 16");
  if (c->n_devices < 0 || c->n_devices > 64) return fail(-EINVAL, "n_devices 0..64");
  return 0;
}

static int sh_create(const raft_sim_config_t* cfg, shard_t** out) {
  if (!cfg || !out) return fail(-EINVAL, "null argument");
  int rc = validate_cfg(cfg);
  if (rc) return rc;
  shard_t* s = (shard_t*)calloc(1, sizeof *s);
  if (!s) return fail(-ENOMEM, "oom");
  s->cfg = *cfg;
  s->N = cfg->nodes; s->Q = cfg->inbox_cap; s->L = cfg->log_cap; s->C = cfg->n_clusters;
  s->A = cfg->arena_cap ? cfg->arena_cap : 4 * cfg->log_cap;
  s->key[0] = (uint32_t)cfg->seed; s->key[1] = (uint32_t)(cfg->seed >> 32);
  s->threads = 1;
  size_t nn = (size_t)s->C * s->N;
  s->nodes = (raft_node_t*)calloc(nn, sizeof(raft_node_t));
  s->q = (raft_msg_t*)calloc(nn * 2 * s->Q, sizeof(raft_msg_t));
  s->arena = (raft_entry_t*)calloc(nn * s->A, sizeof(raft_entry_t));
  s->cl = (raft_cluster_t*)calloc(s->C, sizeof(raft_cluster_t));
  s->S = cfg->commit_stream_cap;
  s->stream = (uint32_t*)calloc(nn * (s->S ? s->S : 1), sizeof(uint32_t));
  s->TC = cfg->trace_cap; s->TE = cfg->trace_entry_cap;
  s->tr = (raft_trace_event_t*)calloc(nn * (s->TC ? s->TC : 1), sizeof(raft_trace_event_t));
  s->tcount = (uint32_t*)calloc(nn, sizeof(uint32_t));
  s->tent = (raft_entry_t*)calloc(nn * (s->TE ? s->TE : 1), sizeof(raft_entry_t));
  s->tecount = (uint32_t*)calloc(nn, sizeof(uint32_t));
  if (!s->nodes || !s->q || !s->arena || !s->cl || !s->stream || !s->tr || !s->tcount || !s->tent ||
      !s->tecount) { sh_destroy(s); return fail(-ENOMEM, "oom"); }
  client_powers(cfg->client_ppm, s->client_pw);
  for (uint32_t c = 0; c < s->C; ++c) {
    uint32_t g = cfg->cluster_offset + c;
    s->cl[c].client_next = 0xFFFFFFFFu;
    if (cfg->client_ppm) {
      uint32_t d[4];
      draw(s, g, P_CLIENT << 8, 0, 1, d);
      s->cl[c].client_next = on_tick(client_gap(d[0], s->client_pw), cfg->client_period,
                                     cfg->client_burst);
    }
    for (uint32_t k = 0; k < s->N; ++k) {
      raft_node_t* n = &s->nodes[(size_t)c * s->N + k];
      n->role = RAFT_FOLLOWER;      /* init-node, core.clj:31-38 */
      n->current_term = 1;
      n->trace_hash = FNV_OFFSET;
      uint32_t w[4];
      draw(s, g, (k + 1) | P_INIT << 8, 0, 0, w);
      n->deadline = cfg->el_base + (uint32_t)(((uint64_t)w[1] * cfg->el_span) >> 32);
    }
  }
  s->ctr.first_violation_tick = UINT64_MAX;
  *out = s;
  return 0;
}

static int sh_set_threads(shard_t* s, int threads) {
  if (!s || threads < 1 || threads > 1024) return fail(-EINVAL, "threads 1..1024");
  s->threads = threads;
  return 0;
}

static void sh_destroy(shard_t* s) {
  if (!s) return;
  free(s->nodes); free(s->q); free(s->arena); free(s->cl); free(s->stream);
  free(s->tr); free(s->tcount); free(s->tent); free(s->tecount); free(s);
}

uint64_t shard_tick(const shard_t* s) { return s ? s->tick : 0; }

/* ---------------------------------------------------------------- per-cluster tick */
typedef struct {
  uint64_t c[RAFT_CTR_COUNT];
  uint64_t first_violation;
  uint64_t payload_max;
} local_ctr_t;

typedef struct { int n; uint32_t arr[2]; raft_msg_t m; } cell_t;

enum { PLAN_NONE = 0, PLAN_PAYLOAD = 1, PLAN_ENTRY = 2 };
typedef struct {
  int kind, reloc;
  uint32_t old_base, old_len, src, poff, pcnt, applied, apply_from;
  raft_entry_t entry;
} plan_t;

typedef struct {
  shard_t* s;
  uint32_t c, g, t, N;
  raft_node_t* nodes;
  local_ctr_t* lc;
  cell_t cell[RAFT_MAX_NODES][RAFT_MAX_NODES]; /* [src-1][dst-1] */
  int part;
  uint32_t sides;
} tick_ctx_t;

static void violation(tick_ctx_t* x, int kind) {
  x->lc->c[kind]++;
  if (x->t < x->lc->first_violation) x->lc->first_violation = x->t;
}

/* val-at (log.clj:20-23) on node k's log; returns a fault code or 0. */
static int val_at(tick_ctx_t* x, uint32_t k, uint32_t idx, int* present, raft_entry_t* e) {
  raft_node_t* n = &x->nodes[k];
  if (idx == 0) { *present = 0; return 0; }
  if (idx > n->log_len) return RAFT_FAULT_IOOBE;
  *e = arena_of(x->s, x->c * x->N + k)[(n->arena_base + idx - 1) % x->s->A];
  *present = 1;
  return 0;
}

/* compare-prev? (log.clj:55-59): whole-entry equality, nil never equal. */
static int compare_prev(tick_ctx_t* x, uint32_t k, uint32_t idx, const raft_msg_t* m, int* out) {
  if (idx == 0) { *out = 1; return 0; }
  int present; raft_entry_t e;
  int f = val_at(x, k, idx, &present, &e);
  if (f) return f;
  int mpresent = (m->hdr >> 8) & 1;
  *out = mpresent && present && e.term == m->eterm && e.val == m->eval;
  return 0;
}

static uint32_t hdr(uint32_t type, uint32_t src, uint32_t flag, uint32_t epresent, uint32_t pcnt) {
  return type | src << 3 | flag << 7 | epresent << 8 | pcnt << 16;
}

typedef struct { uint32_t dst; raft_msg_t m; } emit_t;

/* append-entries-rpc (core.clj:56-67) from the (post-transition) record nn of node k. */
static int ae_broadcast(tick_ctx_t* x, uint32_t k, const raft_node_t* nn, emit_t* em, int* ne) {
  uint32_t id = k + 1;
  int present; raft_entry_t e;
  int f = val_at(x, k, nn->commit_index, &present, &e);   /* last-entry, log.clj:47-49 */
  if (f) return f;
  for (uint32_t p = 1; p <= x->N; ++p) {
    if (p == id) continue;
    if (!nn->ls_present || !((nn->ls_keys >> p) & 1)) return RAFT_FAULT_NPE; /* (- nil 1) */
    if (nn->entries_is_seq) return RAFT_FAULT_CCE;                         /* subvec LazySeq */
  }
  const raft_entry_t* ar = arena_of(x->s, x->c * x->N + k);
  for (uint32_t p = 1; p <= x->N; ++p) {
    if (p == id) continue;
    int32_t next = nn->next_index[p - 1];
    int32_t prev = next - 1 > 0 ? next - 1 : 0;
    uint32_t start = (uint32_t)prev < nn->log_len ? (uint32_t)prev : nn->log_len;
    raft_msg_t m = {0};
    m.term = nn->current_term;
    m.a = nn->commit_index;
    m.b = (uint32_t)prev;
    uint32_t pcnt = 0, ep = 0;
    if (start < nn->log_len) {
      raft_entry_t pe = ar[(nn->arena_base + start) % x->s->A];
      ep = 1; m.eterm = pe.term; m.eval = pe.val;
      pcnt = nn->log_len - start - 1;
    }
    m.poff = pcnt ? nn->arena_base + start + 1 : 0;
    m.hdr = hdr(RAFT_MSG_APPEND_ENTRIES, id, 0, ep, pcnt);
    em[*ne].dst = p; em[*ne].m = m; (*ne)++;
  }
  return 0;
}

/* Plan an append of m entries to node record nn (SIM_SPEC §4 P3: relocation on a dead tail). */
static void plan_append(tick_ctx_t* x, raft_node_t* nn, plan_t* pl, uint32_t m) {
  (void)x;
  pl->old_base = nn->arena_base;
  pl->old_len = nn->log_len;
  pl->reloc = 0;
  if (m > 0) {
    if (nn->arena_base + nn->log_len != nn->arena_frontier) {
      pl->reloc = 1;
      nn->arena_base = nn->arena_frontier;
      nn->arena_frontier += nn->log_len;
    }
    nn->arena_frontier += m;
  }
  nn->log_len += m;
  nn->entries_is_seq = 0; /* (vec (concat ...)), log.clj:64 */
}

static void queue_insert(tick_ctx_t* x, uint32_t k, const raft_msg_t* m) {
  shard_t* s = x->s;
  raft_node_t* n = &x->nodes[k];
  uint32_t type = m->hdr & 7;
  int which = type <= RAFT_MSG_CLIENT_SET ? 0 : 1;
  if (n->fault) { x->lc->c[RAFT_CTR_TO_HALTED]++; return; }
  uint32_t* cnt = which ? &n->res_count : &n->req_count;
  if (*cnt >= s->Q) { x->lc->c[RAFT_CTR_OVERFLOW]++; return; }
  raft_msg_t* q = qslot(s, x->c * x->N + k, which);
  uint32_t pos = *cnt;
  while (pos > 0 && q[pos - 1].arrival > m->arrival) { q[pos] = q[pos - 1]; --pos; }
  q[pos] = *m;
  (*cnt)++;
  x->lc->c[RAFT_CTR_DELIVERED]++;
}

/* Network (SIM_SPEC §4 P2): faults for one emitted message s->r. */
static void transmit(tick_ctx_t* x, uint32_t s_id, uint32_t r_id, const raft_msg_t* m) {
  const raft_sim_config_t* cfg = &x->s->cfg;
  cell_t* rc = &x->cell[s_id - 1][r_id - 1];
  if ((m->hdr & 7) == RAFT_MSG_CLIENT_SET) {  /* a followed redirect: client channel, 1 tick */
    x->lc->c[RAFT_CTR_REDIRECTS]++;
    rc->m = *m; rc->n = 1; rc->arr[0] = x->t + 1;
    return;
  }
  if ((m->hdr & 7) == RAFT_MSG_APPEND_ENTRIES && (m->hdr >> 16) > x->lc->payload_max)
    x->lc->payload_max = m->hdr >> 16;
  x->lc->c[RAFT_CTR_SENT]++;
  if (x->part && (((x->sides >> s_id) ^ (x->sides >> r_id)) & 1)) {
    x->lc->c[RAFT_CTR_PARTITIONED]++;
    return;
  }
  cell_t* cl = &x->cell[s_id - 1][r_id - 1];
  cl->m = *m;
  if (!cfg->drop_ppm && !cfg->dup_ppm && cfg->dmin == cfg->dmax) {
    cl->n = 1; cl->arr[0] = x->t + cfg->dmin;
    return;
  }
  uint32_t w[4];
  draw(x->s, x->g, s_id | P_NET << 8, x->t, r_id, w);
  if (ppm(w[0]) < cfg->drop_ppm) { x->lc->c[RAFT_CTR_DROPPED]++; return; }
  uint32_t span = cfg->dmax - cfg->dmin + 1;
  cl->n = 1;
  cl->arr[0] = x->t + cfg->dmin + (uint32_t)(((uint64_t)w[2] * span) >> 32);
  if (ppm(w[1]) < cfg->dup_ppm) {
    x->lc->c[RAFT_CTR_DUPLICATED]++;
    cl->n = 2;
    cl->arr[1] = x->t + cfg->dmin + (uint32_t)(((uint64_t)w[3] * span) >> 32);
  }
}

/* redirect-client (server.clj:62-63) of a non-leader's client-set-handler (core.clj:152-155): to
 * the :leader-id, or to (rand-nth cluster) when it is nil -- peer index w2*(N-1)>>32 of the peers
 * ascending, w being the node's EVENT draw. The client follows it while the message has hops left
 * (SIM_SPEC §4 D15); otherwise it abandons the command. No state change. */
static void redirect(tick_ctx_t* x, uint32_t k, const raft_msg_t* m, const uint32_t w[4],
                     emit_t* em, int* ne) {
  uint32_t target = x->nodes[k].leader_id;
  if (!target) {
    uint32_t i = (uint32_t)(((uint64_t)w[2] * (x->N - 1)) >> 32);
    target = i + 1 < k + 1 ? i + 1 : i + 2;
  }
  if (m->b >= x->s->cfg.client_redirects) {
    x->lc->c[RAFT_CTR_CLIENT_ABANDONED]++;
    return;
  }
  raft_msg_t r = *m;
  r.arrival = 0;
  r.b = m->b + 1;
  em[*ne].dst = target; em[*ne].m = r; (*ne)++;
}

static uint64_t trace(uint64_t h, uint32_t t, uint32_t ev, uint32_t src, uint32_t mterm,
                      const raft_node_t* n, uint32_t fault) {
  /* SIM_SPEC §4: h <- h * M + x mod 2^64 over two 64-bit words, (t | small << 32) then
     (msg_term | current_term << 32) */
  const uint64_t small = ev | src << 3 | n->role << 7 | fault << 9;
  h = h * TRACE_M + ((uint64_t)t | small << 32);
  return h * TRACE_M + ((uint64_t)mterm | (uint64_t)n->current_term << 32);
}

static uint32_t popcount16(uint32_t v) { return (uint32_t)__builtin_popcount(v & 0xFFFF); }

/* ---------------------------------------------------------------- F4 Spec-Raft (SIM_SPEC §8)
 * NOT reference behaviour: Raft Figure 2 rules on the same state, the correct-protocol control. */

/* "All servers: if RPC term > currentTerm, set currentTerm = term, convert to follower". */
static void spec_step_down(raft_node_t* nn, uint32_t term) {
  nn->current_term = term; nn->voted_for = 0; nn->votes = 0; nn->leader_id = 0;
  nn->role = RAFT_FOLLOWER;
  if (nn->ls_present) {
    nn->ls_present = 0; nn->ls_keys = 0;
    memset(nn->next_index, 0, sizeof nn->next_index);
    memset(nn->match_index, 0, sizeof nn->match_index);
  }
}

/* AppendEntries to every peer: prev = next-1 (clamped to the log), prev-log-term = entry prev,
 * entries [prev, len) (replaces append-entries-rpc, core.clj:56-67). */
static void spec_ae_broadcast(tick_ctx_t* x, uint32_t k, const raft_node_t* nn, emit_t* em,
                              int* ne) {
  uint32_t id = k + 1;
  const raft_entry_t* ar = arena_of(x->s, x->c * x->N + k);
  for (uint32_t p = 1; p <= x->N; ++p) {
    if (p == id) continue;
    int32_t pv = nn->next_index[p - 1] - 1;
    uint32_t prev = pv <= 0 ? 0u : ((uint32_t)pv < nn->log_len ? (uint32_t)pv : nn->log_len);
    raft_msg_t m = {0};
    m.term = nn->current_term; m.a = nn->commit_index; m.b = prev;
    uint32_t ep = 0, pcnt = nn->log_len - prev;
    if (prev) {
      raft_entry_t pe = ar[(nn->arena_base + prev - 1) % x->s->A];
      ep = 1; m.eterm = pe.term; m.eval = pe.val;
    }
    m.poff = pcnt ? nn->arena_base + prev : 0;
    m.hdr = hdr(RAFT_MSG_APPEND_ENTRIES, id, 0, ep, pcnt);
    em[*ne].dst = p; em[*ne].m = m; (*ne)++;
  }
}

static void step_cluster(shard_t* s, uint32_t c, uint32_t t, local_ctr_t* lc) {
  const raft_sim_config_t* cfg = &s->cfg;
  tick_ctx_t X;
  tick_ctx_t* x = &X;
  x->s = s; x->c = c; x->g = cfg->cluster_offset + c; x->t = t; x->N = s->N;
  x->nodes = s->nodes + (size_t)c * s->N; x->lc = lc;
  memset(x->cell, 0, sizeof x->cell);
  const uint32_t N = s->N;
  uint32_t w[4];

  /* P0 client injection (D9): geometric inter-arrival gaps */
  raft_cluster_t* cr = &s->cl[c];
  if (t == cr->client_next) {
    uint32_t d[4];
    draw(s, x->g, P_CLIENT << 8, cr->client_count, 0, d);
    uint32_t target = 1 + (uint32_t)(((uint64_t)d[1] * N) >> 32);
    raft_msg_t m = {0};
    m.arrival = t; m.hdr = hdr(RAFT_MSG_CLIENT_SET, 0, 0, 0, 0); m.a = d[2];
    lc->c[RAFT_CTR_CLIENT_INJECTED]++;
    queue_insert(x, target - 1, &m);
    cr->client_count += 1;
    cr->client_next = on_tick(on_index(t, cfg->client_period, cfg->client_burst) + 1 +
                                  client_gap(d[3], s->client_pw),
                              cfg->client_period, cfg->client_burst);
  }
  x->part = 0; x->sides = 0;
  if (cfg->part_ppm) {
    draw(s, x->g, P_PART << 8, t / cfg->part_epoch, 0, w);
    if (ppm(w[0]) < cfg->part_ppm) { x->part = 1; x->sides = w[1]; }
  }

  plan_t plan[RAFT_MAX_NODES];
  int appended_at[RAFT_MAX_NODES];
  /* F3: append-entries whose :entries the trace records (src, poff, count, ring index) */
  uint32_t tr_src[RAFT_MAX_NODES], tr_poff[RAFT_MAX_NODES], tr_cnt[RAFT_MAX_NODES];
  uint32_t tr_at[RAFT_MAX_NODES];
  memset(tr_cnt, 0, sizeof tr_cnt);
  uint32_t elected = 0, match_changed = 0;
  const uint32_t h_index = cr->hwm_index, h_term = cr->hwm_term, h_val = cr->hwm_val;
  memset(plan, 0, sizeof plan);
  for (uint32_t k = 0; k < N; ++k) appended_at[k] = -1;

  /* pre-tick arena frontiers (Spec-Raft reads payloads in P1 against them, SIM_SPEC §8) */
  const int spec = (cfg->variant_flags & RAFT_VARIANT_SPEC) != 0;
  uint32_t front0[RAFT_MAX_NODES];
  for (uint32_t k = 0; k < N; ++k) front0[k] = x->nodes[k].arena_frontier;

  /* P1 one event per running node (wait, core.clj:176-195) */
  for (uint32_t k = 0; k < N; ++k) {
    raft_node_t* n = &x->nodes[k];
    if (n->fault) continue;
    uint32_t gi = c * N + k, id = k + 1;
    raft_msg_t* rq = qslot(s, gi, 0);
    raft_msg_t* rs = qslot(s, gi, 1);
    int req_ok = n->req_count && rq[0].arrival <= t;
    int res_ok = n->res_count && rs[0].arrival <= t;
    if (!req_ok && !res_ok && t < n->deadline) continue;
    draw(s, x->g, id | P_EVENT << 8, t, 0, w);
    int which = -1;
    if (req_ok && res_ok) which = (w[0] & 1) ? 1 : 0;   /* alts!! choice, core.clj:181 */
    else if (req_ok) which = 0;
    else if (res_ok) which = 1;
    raft_msg_t m = {0};
    if (which >= 0) {      /* take the head */
      raft_msg_t* q = which ? rs : rq;
      uint32_t* cnt = which ? &n->res_count : &n->req_count;
      m = q[0];
      memmove(q, q + 1, (*cnt - 1) * sizeof *q);
      (*cnt)--;
      memset(&q[*cnt], 0, sizeof *q);
    }
    if (s->TC) {               /* `; Node` (prn node) `; Message` (prn message), core.clj:182-186 */
      uint32_t* tc = &s->tcount[gi];
      raft_trace_event_t* ev = &s->tr[(size_t)gi * s->TC + *tc % s->TC];
      memset(ev, 0, sizeof *ev);
      ev->tick = t; ev->seq = *tc; ev->msg = m;
      ev->role = n->role; ev->voted_for = n->voted_for; ev->leader_id = n->leader_id;
      ev->ls_present = n->ls_present; ev->votes = n->votes; ev->ls_keys = n->ls_keys;
      ev->current_term = n->current_term;
      memcpy(ev->next_index, n->next_index, sizeof ev->next_index);
      memcpy(ev->match_index, n->match_index, sizeof ev->match_index);
      ev->entries_seq = s->tecount[gi];
      if ((m.hdr & 7) == RAFT_MSG_APPEND_ENTRIES && which >= 0) {
        tr_src[k] = (m.hdr >> 3) & 15; tr_poff[k] = m.poff; tr_cnt[k] = m.hdr >> 16;
        tr_at[k] = s->tecount[gi];
        s->tecount[gi] += tr_cnt[k];
      }
      (*tc)++;
    }
    raft_node_t nn = *n;
    emit_t em[RAFT_MAX_NODES];
    int ne = 0, fault = 0, elect = 0, mchg = 0, rearm = 0;
    uint32_t ev, msrc = 0, mterm = 0;
    uint64_t appended = 0, applied = 0;
    uint32_t type = m.hdr & 7, src = (m.hdr >> 3) & 15, flag = (m.hdr >> 7) & 1;
    uint32_t pcnt = m.hdr >> 16;
    const raft_entry_t* own = arena_of(s, gi);
    if (spec && which < 0) {
      if (n->role == RAFT_LEADER) {                                  /* heartbeat */
        ev = 7;
        spec_ae_broadcast(x, k, &nn, em, &ne);
      } else {                                                       /* election timeout */
        ev = 6;
        nn.role = RAFT_CANDIDATE; nn.voted_for = (uint8_t)id;
        nn.votes = (uint16_t)(1u << id); nn.current_term = n->current_term + 1;
        raft_msg_t r = {0};
        uint32_t ep = 0;
        r.term = nn.current_term; r.a = n->log_len;
        if (n->log_len) {
          raft_entry_t e = own[(n->arena_base + n->log_len - 1) % s->A];
          ep = 1; r.eterm = e.term; r.eval = e.val;
        }
        r.hdr = hdr(RAFT_MSG_REQUEST_VOTE, id, 0, ep, 0);
        for (uint32_t p = 1; p <= N; ++p)
          if (p != id) { em[ne].dst = p; em[ne].m = r; ne++; }
      }
    } else if (spec) {
      ev = type; msrc = src; mterm = m.term;
      raft_msg_t r = {0};
      int consistent = 0;
      /* OVERFLOW, the only Spec-Raft halt, is decided on the pre-event state */
      if (type == RAFT_MSG_APPEND_ENTRIES && m.term >= n->current_term) {
        consistent = m.b == 0 || (m.b <= n->log_len && ((m.hdr >> 8) & 1) &&
                                  own[(n->arena_base + m.b - 1) % s->A].term == m.eterm);
        if (consistent && (uint64_t)m.b + pcnt > s->L) fault = RAFT_FAULT_OVERFLOW;
      }
      if (type == RAFT_MSG_CLIENT_SET && n->role == RAFT_LEADER && n->log_len + 1 > s->L)
        fault = RAFT_FAULT_OVERFLOW;
      if (!fault && type != RAFT_MSG_CLIENT_SET && m.term > nn.current_term)
        spec_step_down(&nn, m.term);
      switch (fault ? 0 : type) {
        case RAFT_MSG_REQUEST_VOTE: {
          uint32_t lt = n->log_len ? own[(n->arena_base + n->log_len - 1) % s->A].term : 0;
          uint32_t mt = ((m.hdr >> 8) & 1) ? m.eterm : 0;
          int up = (cfg->variant_flags & RAFT_VARIANT_VOTE_NO_LOG_CHECK) || mt > lt ||
                   (mt == lt && m.a >= n->log_len);
          int grant = m.term == nn.current_term &&
                      (nn.voted_for == 0 || nn.voted_for == src) && up;
          if (grant) { nn.voted_for = (uint8_t)src; rearm = 1; }   /* Figure 2 timer reset */
          r.term = nn.current_term;
          r.hdr = hdr(RAFT_MSG_VOTE_RESPONSE, id, (uint32_t)grant, 0, 0);
          em[ne].dst = src; em[ne].m = r; ne++;
          break;
        }
        case RAFT_MSG_APPEND_ENTRIES: {
          r.term = nn.current_term;
          r.hdr = hdr(RAFT_MSG_APPEND_RESPONSE, id, 0, 0, 0);
          if (m.term < nn.current_term) { em[ne].dst = src; em[ne].m = r; ne++; break; }
          nn.role = RAFT_FOLLOWER; nn.votes = 0; nn.leader_id = (uint8_t)src;
          rearm = 1;                                 /* AppendEntries from the current leader */
          if (nn.ls_present) {
            nn.ls_present = 0; nn.ls_keys = 0;
            memset(nn.next_index, 0, sizeof nn.next_index);
            memset(nn.match_index, 0, sizeof nn.match_index);
          }
          if (!consistent) { em[ne].dst = src; em[ne].m = r; ne++; break; }
          /* first conflict in [b, min(len, b+pcnt)); payload read from the sender's arena with
             eviction judged by its pre-tick frontier */
          const raft_entry_t* sa = arena_of(s, c * N + src - 1);
          uint32_t kk = m.b, hi = n->log_len < m.b + pcnt ? n->log_len : m.b + pcnt;
          for (; kk < hi; ++kk) {
            uint32_t i = kk - m.b, pt = 0;
            if ((uint64_t)front0[src - 1] > (uint64_t)m.poff + i + s->A)
              lc->c[RAFT_CTR_PAYLOAD_EVICTED]++;
            else
              pt = sa[(m.poff + i) % s->A].term;
            if (own[(n->arena_base + kk) % s->A].term != pt) break;
          }
          uint32_t mc = m.b + pcnt - kk;
          if (mc) {                      /* truncate at kk, append payload [kk-b, pcnt) */
            plan[k].kind = PLAN_PAYLOAD; plan[k].src = src;
            plan[k].poff = m.poff + (kk - m.b); plan[k].pcnt = mc;
            plan[k].old_base = nn.arena_base; plan[k].old_len = kk; plan[k].reloc = 0;
            if (kk < nn.log_len || nn.arena_base + nn.log_len != nn.arena_frontier) {
              plan[k].reloc = 1;
              nn.arena_base = nn.arena_frontier;
              nn.arena_frontier += kk;
            }
            nn.arena_frontier += mc;
            nn.log_len = m.b + pcnt;
            appended = mc;
            appended_at[k] = (int)kk;
          }
          if (m.a > nn.commit_index) {
            uint32_t nc = m.a < m.b + pcnt ? m.a : m.b + pcnt;
            if (nc > nn.commit_index) {
              applied = nc - nn.commit_index;
              plan[k].applied = (uint32_t)applied; plan[k].apply_from = nn.commit_index;
              nn.commit_index = nc;
            }
          }
          r.hdr = hdr(RAFT_MSG_APPEND_RESPONSE, id, 1, 0, 0);
          r.a = m.a; r.b = m.b + pcnt;
          em[ne].dst = src; em[ne].m = r; ne++;
          break;
        }
        case RAFT_MSG_CLIENT_SET: {                     /* as client-set-handler 151-160 */
          if (n->role != RAFT_LEADER) { redirect(x, k, &m, w, em, &ne); break; }
          plan[k].kind = PLAN_ENTRY;
          plan[k].entry.term = n->current_term; plan[k].entry.val = m.a;
          plan_append(x, &nn, &plan[k], 1);
          appended = 1;
          appended_at[k] = (int)n->log_len;
          break;
        }
        case RAFT_MSG_VOTE_RESPONSE: {
          if (m.term != nn.current_term || !flag || nn.role != RAFT_CANDIDATE) break;
          uint32_t votes = nn.votes | (1u << src);
          if (popcount16(votes) < N / 2 + 1) { nn.votes = (uint16_t)votes; break; }
          nn.role = RAFT_LEADER; nn.votes = 0; nn.leader_id = (uint8_t)id;   /* voted_for kept */
          nn.ls_present = 1; nn.ls_keys = 0;
          for (uint32_t p = 1; p <= N; ++p) {
            nn.next_index[p - 1] = 0; nn.match_index[p - 1] = 0;
            if (p == id) continue;
            nn.ls_keys |= (uint16_t)(1u << p);
            nn.next_index[p - 1] = (int32_t)(nn.log_len + 1);
          }
          spec_ae_broadcast(x, k, &nn, em, &ne);
          elect = 1;
          break;
        }
        case RAFT_MSG_APPEND_RESPONSE: {
          if (m.term != nn.current_term || nn.role != RAFT_LEADER) break;
          if (!flag) {
            int32_t nx = nn.next_index[src - 1] - 1;
            nn.next_index[src - 1] = nx > 1 ? nx : 1;
            break;
          }
          nn.next_index[src - 1] = (int32_t)(m.b + 1);
          nn.match_index[src - 1] = (int32_t)m.b;
          mchg = 1;
          int32_t vals[RAFT_MAX_NODES];
          uint32_t nv = 0;
          vals[nv++] = (int32_t)nn.log_len;
          for (uint32_t p = 1; p <= N; ++p)
            if (p != id) vals[nv++] = nn.match_index[p - 1];
          for (uint32_t i = 1; i < nv; ++i)          /* sort descending */
            for (uint32_t j = i; j > 0 && vals[j - 1] < vals[j]; --j) {
              int32_t tmp = vals[j]; vals[j] = vals[j - 1]; vals[j - 1] = tmp;
            }
          int32_t mm = vals[N / 2];                    /* the maj-th largest */
          if (mm > (int32_t)nn.log_len) mm = (int32_t)nn.log_len;
          if (mm > (int32_t)nn.commit_index &&
              own[(nn.arena_base + (uint32_t)mm - 1) % s->A].term == nn.current_term) {
            applied = (uint32_t)mm - nn.commit_index;
            plan[k].applied = (uint32_t)applied; plan[k].apply_from = nn.commit_index;
            nn.commit_index = (uint32_t)mm;
          }
          break;
        }
        default:
          break;
      }
    } else if (which < 0) {
      if (n->role == RAFT_LEADER) {                          /* heartbeat-handler 162-164 */
        ev = 7;
        fault = ae_broadcast(x, k, &nn, em, &ne);
      } else {                                              /* timeout-handler 166-169 */
        ev = 6;
        nn.role = RAFT_CANDIDATE; nn.voted_for = (uint8_t)id;   /* follower->candidate 69-73 */
        nn.votes = (uint16_t)(1u << id); nn.current_term = n->current_term + 1;
        int present; raft_entry_t e;
        fault = val_at(x, k, n->commit_index, &present, &e);  /* request-vote-rpc 48-54 */
        if (!fault) {
          for (uint32_t p = 1; p <= N; ++p) {
            if (p == id) continue;
            raft_msg_t r = {0};
            r.term = nn.current_term; r.a = n->commit_index;
            if (present) { r.eterm = e.term; r.eval = e.val; }
            r.hdr = hdr(RAFT_MSG_REQUEST_VOTE, id, 0, present, 0);
            em[ne].dst = p; em[ne].m = r; ne++;
          }
        }
      }
    } else {
      ev = type; msrc = src; mterm = m.term;
      raft_msg_t r = {0};
      switch (type) {
        case RAFT_MSG_REQUEST_VOTE: {                       /* request-vote-handler 91-103 */
          int consistent = 1;
          if (!(cfg->variant_flags & RAFT_VARIANT_VOTE_NO_LOG_CHECK))
            fault = compare_prev(x, k, m.a, &m, &consistent);
          if (fault) break;
          int grant = m.term >= n->current_term && n->voted_for == 0 && consistent;
          if (grant) nn.voted_for = (uint8_t)src;
          r.term = n->current_term;
          r.hdr = hdr(RAFT_MSG_VOTE_RESPONSE, id, (uint32_t)grant, 0, 0);
          em[ne].dst = src; em[ne].m = r; ne++;
          break;
        }
        case RAFT_MSG_APPEND_ENTRIES: {                     /* append-entries-handler 105-123 */
          int consistent;
          fault = compare_prev(x, k, m.b, &m, &consistent);
          if (fault) break;
          r.term = n->current_term;
          if (m.term < n->current_term) {
            r.hdr = hdr(RAFT_MSG_APPEND_RESPONSE, id, 0, 0, 0);
          } else if (!consistent) {
            r.hdr = hdr(RAFT_MSG_APPEND_RESPONSE, id, 0, 0, 0);
            nn.log_len = n->log_len > m.b ? n->log_len - m.b : 0; /* remove-from! 78-81 */
            nn.entries_is_seq = 1;
          } else {
            if (n->log_len + pcnt > s->L) { fault = RAFT_FAULT_OVERFLOW; break; }
            plan[k].kind = PLAN_PAYLOAD; plan[k].src = src; plan[k].poff = m.poff;
            plan[k].pcnt = pcnt;
            plan_append(x, &nn, &plan[k], pcnt);                 /* append-entries! 61-64 */
            appended = pcnt;
            if (pcnt) appended_at[k] = (int)n->log_len;
            uint32_t oldc = nn.commit_index;                        /* apply-entries! 69-76 */
            nn.commit_index = nn.log_len;
            applied = nn.commit_index > oldc ? nn.commit_index - oldc : 0;
            plan[k].applied = (uint32_t)applied;
            plan[k].apply_from = oldc;
            r.hdr = hdr(RAFT_MSG_APPEND_RESPONSE, id, 1, 0, 0);
            r.a = m.a; r.b = m.b + pcnt;
            nn.role = RAFT_FOLLWER; nn.voted_for = 0; nn.votes = 0; /* candidate->follower */
            nn.leader_id = (uint8_t)src; nn.current_term = m.term;
          }
          em[ne].dst = src; em[ne].m = r; ne++;
          break;
        }
        case RAFT_MSG_CLIENT_SET: {                          /* client-set-handler 151-160 */
          if (n->role != RAFT_LEADER) { redirect(x, k, &m, w, em, &ne); break; }
          if (n->log_len + 1 > s->L) { fault = RAFT_FAULT_OVERFLOW; break; }
          plan[k].kind = PLAN_ENTRY;
          plan[k].entry.term = n->current_term; plan[k].entry.val = m.a;
          plan_append(x, &nn, &plan[k], 1);
          appended = 1;
          appended_at[k] = (int)n->log_len;
          break;
        }
        case RAFT_MSG_VOTE_RESPONSE: {                       /* vote-response-handler 125-139 */
          int present; raft_entry_t e;
          fault = val_at(x, k, n->commit_index, &present, &e);     /* last-entry first */
          if (fault) break;
          if (m.term > n->current_term) {
            nn.current_term = m.term;
            nn.role = RAFT_FOLLWER; nn.voted_for = 0; nn.votes = 0;
          } else if (!flag || n->role != RAFT_CANDIDATE) {
          } else {
            uint32_t votes = n->votes | (1u << src);
            if (popcount16(votes) < (N + 1) / 2) {             /* majority? 19-21 */
              nn.votes = (uint16_t)votes;
            } else {
              nn.role = RAFT_LEADER; nn.voted_for = 0; nn.votes = 0;   /* candidate->leader */
              nn.leader_id = (uint8_t)id;
              nn.ls_present = 1; nn.ls_keys = 0;                         /* leader-state 40-42 */
              for (uint32_t p = 1; p <= N; ++p) {
                nn.next_index[p - 1] = 0; nn.match_index[p - 1] = 0;
                if (p == id) continue;
                nn.ls_keys |= (uint16_t)(1u << p);
                nn.next_index[p - 1] = (int32_t)(n->commit_index + 1);
              }
              fault = ae_broadcast(x, k, &nn, em, &ne);
              elect = 1;
            }
          }
          break;
        }
        case RAFT_MSG_APPEND_RESPONSE: {                     /* append-response-handler 141-149 */
          if (m.term > n->current_term) {
            nn.current_term = m.term;                        /* leader->follower 86-89 */
            nn.role = RAFT_FOLLOWER; nn.leader_id = 0; nn.ls_present = 0; nn.ls_keys = 0;
            memset(nn.next_index, 0, sizeof nn.next_index);
            memset(nn.match_index, 0, sizeof nn.match_index);
          } else if (!flag) {
            if (!n->ls_present || !((n->ls_keys >> src) & 1)) { fault = RAFT_FAULT_NPE; break; }
            nn.next_index[src - 1] -= 1;
          } else {
            nn.ls_present = 1;
            nn.ls_keys |= (uint16_t)(1u << src);
            nn.next_index[src - 1] = (int32_t)m.b;
            nn.match_index[src - 1] = (int32_t)m.a;
            mchg = 1;
          }
          break;
        }
        default:
          break;
      }
    }
    if (fault) {                                   /* D8: halted, pre-event state, no sends */
      n->fault = (uint8_t)fault;
      n->trace_hash = trace(n->trace_hash, t, ev, msrc, mterm, n, (uint32_t)fault);
      lc->c[RAFT_CTR_HALT_IOOBE + fault - 1]++;
      plan[k].kind = PLAN_NONE;
      appended_at[k] = -1;
      continue;
    }
    /* generate-timeout (core.clj:171-174) for the next wait (D4); Spec-Raft: Raft's timers */
    const uint32_t election = t + cfg->el_base + (uint32_t)(((uint64_t)w[1] * cfg->el_span) >> 32);
    if (!spec)
      nn.deadline = nn.role == RAFT_LEADER ? t + cfg->hb : election;
    else if (nn.role == RAFT_LEADER) {
      if (ev == 7 || elect) nn.deadline = t + cfg->hb;
    } else if (ev == 6 || rearm || n->role == RAFT_LEADER) {
      nn.deadline = election;
    }
    nn.trace_hash = trace(n->trace_hash, t, ev, msrc, mterm, &nn, 0);
    *n = nn;
    lc->c[RAFT_CTR_EV_RV + ev - 1]++;
    lc->c[RAFT_CTR_ENTRIES_APPENDED] += appended;
    lc->c[RAFT_CTR_ENTRIES_APPLIED] += applied;
    if (elect) {
      lc->c[RAFT_CTR_LEADERS]++;
      n->last_led_term = n->current_term;
      elected |= 1u << k;
    }
    if (mchg) match_changed |= 1u << k;
    for (int i = 0; i < ne; ++i) transmit(x, id, em[i].dst, &em[i].m);
  }

  /* P2 delivery: sender id ascending, copy 0 then 1 */
  for (uint32_t r = 0; r < N; ++r)
    for (uint32_t sd = 0; sd < N; ++sd) {
      cell_t* cl = &x->cell[sd][r];
      for (int i = 0; i < cl->n; ++i) {
        raft_msg_t m = cl->m;
        m.arrival = cl->arr[i];
        queue_insert(x, r, &m);
      }
    }

  /* P3 log writes (relocation + payload transfer) */
  for (uint32_t k = 0; k < N; ++k) {
    plan_t* pl = &plan[k];
    if (pl->kind == PLAN_NONE) continue;
    raft_node_t* n = &x->nodes[k];
    raft_entry_t* ar = arena_of(s, c * N + k);
    uint32_t m = pl->kind == PLAN_PAYLOAD ? pl->pcnt : 1;
    if (m == 0) continue;
    if (pl->reloc)
      for (uint32_t i = 0; i < pl->old_len; ++i)
        ar[(n->arena_base + i) % s->A] = ar[(pl->old_base + i) % s->A];
    uint32_t dst = n->arena_base + pl->old_len;
    if (pl->kind == PLAN_ENTRY) {
      ar[dst % s->A] = pl->entry;
    } else {
      const raft_node_t* sn = &x->nodes[pl->src - 1];
      const raft_entry_t* sa = arena_of(s, c * N + pl->src - 1);
      for (uint32_t i = 0; i < m; ++i) {
        raft_entry_t e = {0, 0};
        if ((uint64_t)sn->arena_frontier > (uint64_t)pl->poff + i + s->A)
          lc->c[RAFT_CTR_PAYLOAD_EVICTED]++;
        else
          e = sa[(pl->poff + i) % s->A];
        ar[(dst + i) % s->A] = e;
      }
    }
  }

  /* F3: the :entries of traced append-entries, as P3 resolves them (evicted -> (0,0)) */
  for (uint32_t k = 0; k < N && s->TE; ++k) {
    if (!tr_cnt[k]) continue;
    const raft_node_t* sn = &x->nodes[tr_src[k] - 1];
    const raft_entry_t* sa = arena_of(s, c * N + tr_src[k] - 1);
    raft_entry_t* ring = s->tent + (size_t)(c * N + k) * s->TE;
    for (uint32_t i = 0; i < tr_cnt[k]; ++i) {
      raft_entry_t e = {0, 0};
      if ((uint64_t)sn->arena_frontier <= (uint64_t)tr_poff[k] + i + s->A)
        e = sa[(tr_poff[k] + i) % s->A];
      ring[(tr_at[k] + i) % s->TE] = e;
    }
  }

  /* apply-entries! writes (F2): the :val's of the last `applied` entries (log.clj:69-76) */
  for (uint32_t k = 0; k < N; ++k) {
    uint32_t a = plan[k].applied;
    if (!a) continue;
    raft_node_t* n = &x->nodes[k];
    const raft_entry_t* ar = arena_of(s, c * N + k);
    uint32_t* ring = s->stream + (size_t)(c * N + k) * (s->S ? s->S : 1);
    for (uint32_t i = plan[k].apply_from; i < plan[k].apply_from + a; ++i) {
      if (s->S) ring[n->commit_count % s->S] = ar[(n->arena_base + i) % s->A].val;
      n->commit_count++;
    }
  }

  /* P4 invariant checker */
  {
    for (uint32_t k = 0; k < N; ++k) {
      if (!((elected >> k) & 1)) continue;
      uint32_t T = x->nodes[k].last_led_term;
      for (uint32_t j = 0; j < N; ++j)
        if (j != k && x->nodes[j].last_led_term == T) { violation(x, RAFT_CTR_VIOL_ELECTION); break; }
    }
    for (uint32_t k = 0; k < N; ++k) {
      if (appended_at[k] < 0) continue;
      const raft_node_t* nk = &x->nodes[k];
      const raft_entry_t* ak = arena_of(s, c * N + k);
      int bad = 0;
      for (uint32_t j = 0; j < N && !bad; ++j) {
        if (j == k) continue;
        const raft_node_t* nj = &x->nodes[j];
        const raft_entry_t* aj = arena_of(s, c * N + j);
        uint32_t hi = nk->log_len < nj->log_len ? nk->log_len : nj->log_len;
        for (uint32_t p = (uint32_t)appended_at[k]; p < hi; ++p) {
          raft_entry_t a = ak[(nk->arena_base + p) % s->A], b = aj[(nj->arena_base + p) % s->A];
          if (a.term == b.term && a.val != b.val) { bad = 1; break; }
        }
      }
      if (bad) violation(x, RAFT_CTR_VIOL_LOG);
    }
    for (uint32_t k = 0; k < N; ++k) {
      if (!((elected >> k) & 1) || h_index == 0) continue;
      const raft_node_t* nk = &x->nodes[k];
      const raft_entry_t* ak = arena_of(s, c * N + k);
      int ok = nk->log_len >= h_index;
      if (ok) {
        raft_entry_t e = ak[(nk->arena_base + h_index - 1) % s->A];
        ok = e.term == h_term && e.val == h_val;
      }
      if (!ok) violation(x, RAFT_CTR_VIOL_COMPLETE);
    }
    int32_t best = -1;
    uint32_t nh_index = 0, nh_term = 0, nh_val = 0;
    for (uint32_t k = 0; k < N; ++k) {
      const raft_node_t* nk = &x->nodes[k];
      if (nk->role != RAFT_LEADER || !(((elected | match_changed) >> k) & 1)) continue;
      int32_t vals[RAFT_MAX_NODES];
      uint32_t nv = 0;
      vals[nv++] = (int32_t)nk->log_len;
      for (uint32_t p = 1; p <= N; ++p)
        if (p != k + 1) vals[nv++] = ((nk->ls_keys >> p) & 1) ? nk->match_index[p - 1] : 0;
      for (uint32_t i = 1; i < nv; ++i)       /* sort descending */
        for (uint32_t j = i; j > 0 && vals[j - 1] < vals[j]; --j) {
          int32_t tmp = vals[j]; vals[j] = vals[j - 1]; vals[j - 1] = tmp;
        }
      int32_t mm = vals[(spec ? N / 2 + 1 : (N + 1) / 2) - 1];
      if (mm > (int32_t)nk->log_len) mm = (int32_t)nk->log_len;
      /* Spec-Raft (SIM_SPEC §8): only an entry of the leader's own term is committed by count */
      if (spec && mm > 0 &&
          arena_of(s, c * N + k)[(nk->arena_base + (uint32_t)mm - 1) % s->A].term != nk->current_term)
        continue;
      if (mm > (int32_t)h_index && mm > best) {
        best = mm;
        raft_entry_t e = arena_of(s, c * N + k)[(nk->arena_base + (uint32_t)mm - 1) % s->A];
        nh_index = (uint32_t)mm; nh_term = e.term; nh_val = e.val;
      }
    }
    if (best > 0) { cr->hwm_index = nh_index; cr->hwm_term = nh_term; cr->hwm_val = nh_val; }
  }
}

/* ---------------------------------------------------------------- stepping (pmap over chunks) */
typedef struct {
  shard_t* s;
  uint32_t c0, c1, t0, n;
  local_ctr_t lc;
} job_t;

/* The earliest tick >= t at which cluster c can do anything: a running node's deadline or queue
 * head, or the next client-set (SIM_SPEC §4: nothing else is keyed to a tick). */
static uint32_t next_event(const shard_t* s, uint32_t c) {
  uint32_t m = s->cl[c].client_next;
  for (uint32_t k = 0; k < s->N; ++k) {
    const raft_node_t* n = &s->nodes[(size_t)c * s->N + k];
    if (n->fault) continue;
    if (n->deadline < m) m = n->deadline;
    const raft_msg_t* rq = s->q + ((size_t)(c * s->N + k) * 2) * s->Q;
    const raft_msg_t* rs = rq + s->Q;
    if (n->req_count && rq[0].arrival < m) m = rq[0].arrival;
    if (n->res_count && rs[0].arrival < m) m = rs[0].arrival;
  }
  return m;
}

static void* run_job(void* arg) {
  job_t* j = (job_t*)arg;
  memset(&j->lc, 0, sizeof j->lc);
  j->lc.first_violation = UINT64_MAX;
  const uint64_t end = (uint64_t)j->t0 + j->n;
  for (uint32_t c = j->c0; c < j->c1; ++c) {
    if (!j->s->idle_skip) {
      for (uint32_t i = 0; i < j->n; ++i) step_cluster(j->s, c, j->t0 + i, &j->lc);
      continue;
    }
    for (uint64_t t = j->t0; t < end;) {     /* discrete-event skipping, tick-exact */
      const uint32_t nx = next_event(j->s, c);
      if (nx > t) t = nx < end ? nx : end;
      if (t == end) break;
      step_cluster(j->s, c, (uint32_t)t, &j->lc);
      ++t;
    }
  }
  return NULL;
}

static int sh_step(shard_t* s, uint32_t n_ticks) {
  int T = s->threads;
  if ((uint32_t)T > s->C) T = (int)s->C;
  job_t* jobs = (job_t*)calloc((size_t)T, sizeof *jobs);
  pthread_t* th = (pthread_t*)calloc((size_t)T, sizeof *th);
  if (!jobs || !th) { free(jobs); free(th); return fail(-ENOMEM, "oom"); }
  for (int i = 0; i < T; ++i) {
    jobs[i].s = s; jobs[i].t0 = (uint32_t)s->tick; jobs[i].n = n_ticks;
    jobs[i].c0 = (uint32_t)((uint64_t)s->C * i / T);
    jobs[i].c1 = (uint32_t)((uint64_t)s->C * (i + 1) / T);
  }
  if (T == 1) {
    run_job(&jobs[0]);
  } else {
    for (int i = 0; i < T; ++i) pthread_create(&th[i], NULL, run_job, &jobs[i]);
    for (int i = 0; i < T; ++i) pthread_join(th[i], NULL);
  }
  for (int i = 0; i < T; ++i) {
    for (int k = 0; k < RAFT_CTR_COUNT; ++k) s->ctr.c[k] += jobs[i].lc.c[k];
    if (jobs[i].lc.first_violation < s->ctr.first_violation_tick)
      s->ctr.first_violation_tick = jobs[i].lc.first_violation;
    if (jobs[i].lc.payload_max > s->ctr.payload_max) s->ctr.payload_max = jobs[i].lc.payload_max;
  }
  s->ctr.node_ticks += (uint64_t)s->C * s->N * n_ticks;
  s->tick += n_ticks;
  free(jobs); free(th);
  return 0;
}

/* ---------------------------------------------------------------- state access */
static int check_range(shard_t* s, uint32_t c0, uint32_t nc) {
  if (!s) return fail(-EINVAL, "null sim");
  if ((uint64_t)c0 + nc > s->C) return fail(-EINVAL, "cluster range out of bounds");
  return 0;
}
static int check_node(shard_t* s, uint32_t cluster, uint32_t id) {
  if (!s) return fail(-EINVAL, "null sim");
  if (cluster >= s->C || id < 1 || id > s->N) return fail(-EINVAL, "cluster/node out of bounds");
  return 0;
}

static int sh_read_nodes(shard_t* s, uint32_t c0, uint32_t nc, raft_node_t* out) {
  int rc = check_range(s, c0, nc);
  if (rc) return rc;
  memcpy(out, s->nodes + (size_t)c0 * s->N, (size_t)nc * s->N * sizeof(raft_node_t));
  return 0;
}

static int sh_write_nodes(shard_t* s, uint32_t c0, uint32_t nc, const raft_node_t* in) {
  int rc = check_range(s, c0, nc);
  if (rc) return rc;
  const uint32_t N = s->N, all = ((1u << (N + 1)) - 1) & ~1u;
  for (size_t i = 0; i < (size_t)nc * N; ++i) {
    const raft_node_t* n = &in[i];
    uint32_t id = (uint32_t)(i % N) + 1, peers = all & ~(1u << id);
    if (n->role > 3 || n->voted_for > N || n->leader_id > N || n->fault > 4 ||
        (n->votes & ~all) || (n->ls_keys & ~peers) || n->entries_is_seq > 1 || n->ls_present > 1 ||
        n->log_len > s->L || n->arena_frontier - n->arena_base < n->log_len ||
        n->arena_frontier - n->arena_base > s->L ||
        (n->role == RAFT_LEADER && (!n->ls_present || n->ls_keys != peers)) ||
        (!n->ls_present && n->ls_keys))
      return fail(-EINVAL, "invalid node record");
  }
  for (size_t i = 0; i < (size_t)nc * N; ++i) {
    raft_node_t* d = &s->nodes[(size_t)c0 * N + i];
    uint32_t rq = d->req_count, rs = d->res_count;
    *d = in[i];
    d->req_count = rq; d->res_count = rs;
    d->reserved0 = 0;
    for (uint32_t p = N; p < RAFT_MAX_NODES; ++p) { d->next_index[p] = 0; d->match_index[p] = 0; }
  }
  return 0;
}

static int sh_read_queue(shard_t* s, uint32_t cluster, uint32_t id, uint32_t which,
                        raft_msg_t* out, uint32_t cap) {
  int rc = check_node(s, cluster, id);
  if (rc) return rc;
  if (which > 1) return fail(-EINVAL, "which must be 0 (req) or 1 (res)");
  raft_node_t* n = &s->nodes[(size_t)cluster * s->N + id - 1];
  uint32_t cnt = which ? n->res_count : n->req_count;
  uint32_t m = cnt < cap ? cnt : cap;
  if (out && m) memcpy(out, qslot(s, cluster * s->N + id - 1, (int)which), m * sizeof(raft_msg_t));
  return (int)cnt;
}

static int sh_write_queue(shard_t* s, uint32_t cluster, uint32_t id, uint32_t which,
                         const raft_msg_t* in, uint32_t count) {
  int rc = check_node(s, cluster, id);
  if (rc) return rc;
  if (which > 1 || count > s->Q) return fail(-EINVAL, "bad queue or count");
  for (uint32_t i = 0; i < count; ++i) {
    uint32_t type = in[i].hdr & 7, src = (in[i].hdr >> 3) & 15;
    int want = type <= RAFT_MSG_CLIENT_SET ? 0 : 1;
    if (type < 1 || type > 5 || want != (int)which || src > s->N || src == id ||
        (type == RAFT_MSG_CLIENT_SET) != (src == 0) ||
        (i > 0 && in[i].arrival < in[i - 1].arrival))
      return fail(-EINVAL, "invalid message or order");
  }
  raft_msg_t* q = qslot(s, cluster * s->N + id - 1, (int)which);
  memset(q, 0, s->Q * sizeof *q);
  if (count) memcpy(q, in, count * sizeof *q);
  raft_node_t* n = &s->nodes[(size_t)cluster * s->N + id - 1];
  if (which) n->res_count = count; else n->req_count = count;
  return 0;
}

static int sh_read_arena(shard_t* s, uint32_t cluster, uint32_t id, raft_entry_t* out,
                        uint32_t cap) {
  int rc = check_node(s, cluster, id);
  if (rc) return rc;
  uint32_t m = cap < s->A ? cap : s->A;
  if (out && m) memcpy(out, arena_of(s, cluster * s->N + id - 1), m * sizeof(raft_entry_t));
  return (int)s->A;
}

static int sh_write_arena(shard_t* s, uint32_t cluster, uint32_t id, const raft_entry_t* in,
                         uint32_t count) {
  int rc = check_node(s, cluster, id);
  if (rc) return rc;
  if (count > s->A) return fail(-EINVAL, "count > arena_cap");
  raft_entry_t* a = arena_of(s, cluster * s->N + id - 1);
  memset(a, 0, s->A * sizeof *a);
  if (count) memcpy(a, in, count * sizeof *a);
  return 0;
}

static int sh_read_commit_stream(shard_t* s, uint32_t cluster, uint32_t id, uint32_t* out,
                                uint32_t cap) {
  int rc = check_node(s, cluster, id);
  if (rc) return rc;
  const raft_node_t* n = &s->nodes[(size_t)cluster * s->N + id - 1];
  uint32_t kept = n->commit_count < s->S ? n->commit_count : s->S;
  if (kept > cap) kept = cap;
  const uint32_t* ring = s->stream + (size_t)(cluster * s->N + id - 1) * (s->S ? s->S : 1);
  for (uint32_t i = 0; i < kept; ++i) out[i] = ring[(n->commit_count - kept + i) % s->S];
  return (int)kept;
}

static int sh_write_commit_stream(shard_t* s, uint32_t cluster, uint32_t id, const uint32_t* in,
                                 uint32_t count) {
  int rc = check_node(s, cluster, id);
  if (rc) return rc;
  const raft_node_t* n = &s->nodes[(size_t)cluster * s->N + id - 1];
  if (count > s->S || count > n->commit_count) return fail(-EINVAL, "count exceeds ring or commit_count");
  uint32_t* ring = s->stream + (size_t)(cluster * s->N + id - 1) * (s->S ? s->S : 1);
  for (uint32_t i = 0; i < count; ++i) ring[(n->commit_count - count + i) % s->S] = in[i];
  return 0;
}

static int sh_read_trace(shard_t* s, uint32_t cluster, uint32_t id, uint32_t first,
                        raft_trace_event_t* out, uint32_t cap) {
  int rc = check_node(s, cluster, id);
  if (rc) return rc;
  uint32_t gi = cluster * s->N + id - 1, cnt = s->tcount[gi];
  uint32_t lo = cnt > s->TC ? cnt - s->TC : 0;
  if (first > lo) lo = first;
  uint32_t n = 0;
  for (uint32_t i = lo; i < cnt && n < cap; ++i) out[n++] = s->tr[(size_t)gi * s->TC + i % s->TC];
  return (int)n;
}

static int sh_read_trace_entries(shard_t* s, uint32_t cluster, uint32_t id, uint32_t first,
                                raft_entry_t* out, uint32_t cap) {
  int rc = check_node(s, cluster, id);
  if (rc) return rc;
  if (!s->TE) return fail(-ERANGE, "trace_entry_cap is 0");
  uint32_t gi = cluster * s->N + id - 1, cnt = s->tecount[gi];
  uint32_t lo = cnt > s->TE ? cnt - s->TE : 0;
  if (first < lo) return fail(-ERANGE, "trace entries overwritten (ring holds the newest)");
  lo = first;
  uint32_t n = 0;
  for (uint32_t i = lo; i < cnt && n < cap; ++i) out[n++] = s->tent[(size_t)gi * s->TE + i % s->TE];
  return (int)n;
}

static int sh_read_clusters(shard_t* s, uint32_t c0, uint32_t nc, raft_cluster_t* out) {
  int rc = check_range(s, c0, nc);
  if (rc) return rc;
  memcpy(out, s->cl + c0, nc * sizeof *out);
  return 0;
}

static int sh_write_clusters(shard_t* s, uint32_t c0, uint32_t nc, const raft_cluster_t* in) {
  int rc = check_range(s, c0, nc);
  if (rc) return rc;
  memcpy(s->cl + c0, in, nc * sizeof *in);
  for (uint32_t i = 0; i < nc; ++i) memset(s->cl[c0 + i].reserved, 0, sizeof in->reserved);
  return 0;
}

static int sh_read_counters(shard_t* s, raft_counters_t* out) {
  if (!s || !out) return fail(-EINVAL, "null argument");
  *out = s->ctr;
  return 0;
}

static int sh_digest(shard_t* s, uint32_t c0, uint32_t nc, uint64_t* out) {
  int rc = check_range(s, c0, nc);
  if (rc) return rc;
  const uint32_t N = s->N;
  for (uint32_t ci = 0; ci < nc; ++ci) {
    uint32_t c = c0 + ci;
    uint64_t h = FNV_OFFSET;
    for (uint32_t k = 0; k < N; ++k) {
      const raft_node_t* n = &s->nodes[(size_t)c * N + k];
      uint32_t hdrw[12] = {n->role, n->voted_for, n->leader_id, n->fault, n->entries_is_seq,
                           n->ls_present, n->votes, n->ls_keys, n->current_term,
                           n->commit_index, n->log_len, n->deadline};
      for (int i = 0; i < 12; ++i) h = fnv(h, hdrw[i]);
      for (uint32_t p = 0; p < N; ++p) h = fnv(h, (uint32_t)n->next_index[p]);
      for (uint32_t p = 0; p < N; ++p) h = fnv(h, (uint32_t)n->match_index[p]);
      h = fnv(h, n->last_led_term);
      h = fnv(h, (uint32_t)n->trace_hash);
      h = fnv(h, (uint32_t)(n->trace_hash >> 32));
      h = fnv(h, n->arena_base);
      h = fnv(h, n->arena_frontier);
      h = fnv(h, n->commit_count);
      if (s->S) {
        const uint32_t* ring = s->stream + (size_t)(c * N + k) * s->S;
        uint32_t kept = n->commit_count < s->S ? n->commit_count : s->S;
        for (uint32_t i = n->commit_count - kept; i != n->commit_count; ++i) h = fnv(h, ring[i % s->S]);
      }
      if (s->TC) {                /* F3 trace rings, retained part, oldest first */
        uint32_t gi = c * N + k, cnt = s->tcount[gi], kept = cnt < s->TC ? cnt : s->TC;
        h = fnv(h, cnt);
        for (uint32_t i = cnt - kept; i != cnt; ++i) {
          const uint32_t* wds = (const uint32_t*)&s->tr[(size_t)gi * s->TC + i % s->TC];
          for (int j = 0; j < 32; ++j) h = fnv(h, wds[j]);
        }
      }
      if (s->TE) {
        uint32_t gi = c * N + k, cnt = s->tecount[gi], kept = cnt < s->TE ? cnt : s->TE;
        h = fnv(h, cnt);
        for (uint32_t i = cnt - kept; i != cnt; ++i) {
          raft_entry_t e = s->tent[(size_t)gi * s->TE + i % s->TE];
          h = fnv(h, e.term);
          h = fnv(h, e.val);
        }
      }
      for (int which = 0; which < 2; ++which) {
        uint32_t cnt = which ? n->res_count : n->req_count;
        h = fnv(h, cnt);
        const raft_msg_t* q = qslot(s, c * N + k, which);
        for (uint32_t i = 0; i < cnt; ++i) {
          const uint32_t* wds = (const uint32_t*)&q[i];
          for (int j = 0; j < 8; ++j) h = fnv(h, wds[j]);
        }
      }
      const raft_entry_t* a = arena_of(s, c * N + k);
      for (uint32_t i = 0; i < n->log_len; ++i) {
        raft_entry_t e = a[(n->arena_base + i) % s->A];
        h = fnv(h, e.term);
        h = fnv(h, e.val);
      }
    }
    h = fnv(h, s->cl[c].hwm_index);
    h = fnv(h, s->cl[c].hwm_term);
    h = fnv(h, s->cl[c].hwm_val);
    h = fnv(h, s->cl[c].client_next);
    h = fnv(h, s->cl[c].client_count);
    out[ci] = h;
  }
  return 0;
}

int raft_ref_abi_version(void) { return RAFT_SIM_ABI_VERSION; }

/* ---------------------------------------------------------------- the handle: G shards
 * Mirrors the product's n_devices (include/raftsim.h): clusters split into contiguous shards
 * [C*d/G, C*(d+1)/G), each simulated independently with its global cluster ids; calls addressed
 * to clusters are routed to the shard that owns them, counters are reduced (SUM, MIN, MAX). */
struct raft_ref {
  raft_sim_config_t cfg;
  int G;
  shard_t* sh[64];
  uint32_t lo[65];   /* shard d owns local clusters [lo[d], lo[d+1]) */
  uint64_t tick;
};

int raft_ref_create(const raft_sim_config_t* cfg, raft_ref_t** out) {
  if (!cfg || !out) return fail(-EINVAL, "null argument");
  int rc = validate_cfg(cfg);
  if (rc) return rc;
  raft_ref_t* r = (raft_ref_t*)calloc(1, sizeof *r);
  if (!r) return fail(-ENOMEM, "oom");
  r->cfg = *cfg;
  r->G = cfg->n_devices > 1 ? cfg->n_devices : 1;
  if ((uint32_t)r->G > cfg->n_clusters) r->G = (int)cfg->n_clusters;
  for (int d = 0; d <= r->G; ++d) r->lo[d] = (uint32_t)((uint64_t)cfg->n_clusters * d / r->G);
  for (int d = 0; d < r->G; ++d) {
    raft_sim_config_t c = *cfg;
    c.n_clusters = r->lo[d + 1] - r->lo[d];
    c.cluster_offset = cfg->cluster_offset + r->lo[d];
    c.n_devices = 1;
    if ((rc = sh_create(&c, &r->sh[d]))) { raft_ref_destroy(r); return rc; }
  }
  *out = r;
  return 0;
}

void raft_ref_destroy(raft_ref_t* r) {
  if (!r) return;
  for (int d = 0; d < r->G; ++d) sh_destroy(r->sh[d]);
  free(r);
}

int raft_ref_set_idle_skip(raft_ref_t* r, int on) {
  if (!r) return fail(-EINVAL, "null sim");
  for (int d = 0; d < r->G; ++d) r->sh[d]->idle_skip = on != 0;
  return 0;
}

int raft_ref_set_threads(raft_ref_t* r, int threads) {
  if (!r) return fail(-EINVAL, "null sim");
  for (int d = 0; d < r->G; ++d) {
    int rc = sh_set_threads(r->sh[d], threads);
    if (rc) return rc;
  }
  return 0;
}

/* SIM_SPEC §4 D1: no deadline or arrival may reach 2^32-1 (the "never" marker) */
static int horizon_ok(const raft_sim_config_t* c, uint64_t tick, uint32_t n) {
  uint64_t longest = c->hb;
  if ((uint64_t)c->el_base + c->el_span > longest) longest = (uint64_t)c->el_base + c->el_span;
  if (c->dmax > longest) longest = c->dmax;
  return tick + n + longest < 0xFFFFFFFFull;
}

int raft_ref_step(raft_ref_t* r, uint32_t n_ticks) {
  if (!r) return fail(-EINVAL, "null sim");
  if (!horizon_ok(&r->cfg, r->tick, n_ticks))
    return fail(-ERANGE, "tick + n_ticks + the longest timer would reach 2^32-1");
  for (int d = 0; d < r->G; ++d) {
    int rc = sh_step(r->sh[d], n_ticks);
    if (rc) return rc;
  }
  r->tick += n_ticks;
  return 0;
}
int raft_ref_step_async(raft_ref_t* r, uint32_t n_ticks) { return raft_ref_step(r, n_ticks); }
int raft_ref_sync(raft_ref_t* r) { return r ? 0 : fail(-EINVAL, "null sim"); }
uint64_t raft_ref_tick(const raft_ref_t* r) { return r ? r->tick : 0; }

int raft_ref_set_tick(raft_ref_t* r, uint64_t tick) {
  if (!r) return fail(-EINVAL, "null sim");
  if (!horizon_ok(&r->cfg, tick, 0)) return fail(-ERANGE, "tick beyond the 32-bit horizon");
  r->tick = tick;
  for (int d = 0; d < r->G; ++d) r->sh[d]->tick = tick;
  return 0;
}

/* the shard owning local cluster c, and c's index inside it */
static shard_t* owner(raft_ref_t* r, uint32_t c, uint32_t* lc) {
  int d = 0;
  while (d + 1 < r->G && c >= r->lo[d + 1]) ++d;
  *lc = c - r->lo[d];
  return r->sh[d];
}

static int check_span(raft_ref_t* r, uint32_t c0, uint32_t nc) {
  if (!r) return fail(-EINVAL, "null sim");
  if ((uint64_t)c0 + nc > r->cfg.n_clusters) return fail(-EINVAL, "cluster range out of bounds");
  return 0;
}

/* Apply `fn` to the pieces of [c0, c0+nc) per shard; `stride` elements per cluster in `buf`. */
#define FOR_PIECES(r, c0, nc, BODY)                                                     \
  for (uint32_t done = 0; done < (nc);) {                                               \
    uint32_t lc_;                                                                       \
    shard_t* sh_ = owner((r), (c0) + done, &lc_);                                        \
    uint32_t n_ = sh_->C - lc_;                                                          \
    if (n_ > (nc) - done) n_ = (nc) - done;                                              \
    BODY;                                                                               \
    done += n_;                                                                         \
  }

int raft_ref_read_nodes(raft_ref_t* r, uint32_t c0, uint32_t nc, raft_node_t* out) {
  int rc = check_span(r, c0, nc);
  if (rc) return rc;
  FOR_PIECES(r, c0, nc, if ((rc = sh_read_nodes(sh_, lc_, n_, out + (size_t)done * r->cfg.nodes))) return rc)
  return 0;
}
int raft_ref_write_nodes(raft_ref_t* r, uint32_t c0, uint32_t nc, const raft_node_t* in) {
  int rc = check_span(r, c0, nc);
  if (rc) return rc;
  FOR_PIECES(r, c0, nc, if ((rc = sh_write_nodes(sh_, lc_, n_, in + (size_t)done * r->cfg.nodes))) return rc)
  return 0;
}
int raft_ref_read_clusters(raft_ref_t* r, uint32_t c0, uint32_t nc, raft_cluster_t* out) {
  int rc = check_span(r, c0, nc);
  if (rc) return rc;
  FOR_PIECES(r, c0, nc, if ((rc = sh_read_clusters(sh_, lc_, n_, out + done))) return rc)
  return 0;
}
int raft_ref_write_clusters(raft_ref_t* r, uint32_t c0, uint32_t nc, const raft_cluster_t* in) {
  int rc = check_span(r, c0, nc);
  if (rc) return rc;
  FOR_PIECES(r, c0, nc, if ((rc = sh_write_clusters(sh_, lc_, n_, in + done))) return rc)
  return 0;
}
int raft_ref_digest(raft_ref_t* r, uint32_t c0, uint32_t nc, uint64_t* out) {
  int rc = check_span(r, c0, nc);
  if (rc) return rc;
  FOR_PIECES(r, c0, nc, if ((rc = sh_digest(sh_, lc_, n_, out + done))) return rc)
  return 0;
}

static shard_t* node_owner(raft_ref_t* r, uint32_t cluster, uint32_t* lc) {
  if (!r || cluster >= r->cfg.n_clusters) return NULL;
  return owner(r, cluster, lc);
}
#define ROUTE_NODE(call)                                                         \
  uint32_t lc;                                                                   \
  shard_t* sh = node_owner(r, cluster, &lc);                                     \
  if (!sh) return fail(-EINVAL, "cluster/node out of bounds");                   \
  return call;

int raft_ref_read_queue(raft_ref_t* r, uint32_t cluster, uint32_t id, uint32_t which,
                        raft_msg_t* out, uint32_t cap) {
  ROUTE_NODE(sh_read_queue(sh, lc, id, which, out, cap))
}
int raft_ref_write_queue(raft_ref_t* r, uint32_t cluster, uint32_t id, uint32_t which,
                         const raft_msg_t* in, uint32_t count) {
  ROUTE_NODE(sh_write_queue(sh, lc, id, which, in, count))
}
int raft_ref_read_arena(raft_ref_t* r, uint32_t cluster, uint32_t id, raft_entry_t* out,
                        uint32_t cap) {
  ROUTE_NODE(sh_read_arena(sh, lc, id, out, cap))
}
int raft_ref_write_arena(raft_ref_t* r, uint32_t cluster, uint32_t id, const raft_entry_t* in,
                         uint32_t count) {
  ROUTE_NODE(sh_write_arena(sh, lc, id, in, count))
}
int raft_ref_read_commit_stream(raft_ref_t* r, uint32_t cluster, uint32_t id, uint32_t* out,
                                uint32_t cap) {
  ROUTE_NODE(sh_read_commit_stream(sh, lc, id, out, cap))
}
int raft_ref_write_commit_stream(raft_ref_t* r, uint32_t cluster, uint32_t id, const uint32_t* in,
                                 uint32_t count) {
  ROUTE_NODE(sh_write_commit_stream(sh, lc, id, in, count))
}
int raft_ref_read_trace(raft_ref_t* r, uint32_t cluster, uint32_t id, uint32_t first,
                        raft_trace_event_t* out, uint32_t cap) {
  ROUTE_NODE(sh_read_trace(sh, lc, id, first, out, cap))
}
int raft_ref_read_trace_entries(raft_ref_t* r, uint32_t cluster, uint32_t id, uint32_t first,
                                raft_entry_t* out, uint32_t cap) {
  ROUTE_NODE(sh_read_trace_entries(sh, lc, id, first, out, cap))
}

int raft_ref_read_counters(raft_ref_t* r, raft_counters_t* out) {
  if (!r || !out) return fail(-EINVAL, "null argument");
  memset(out, 0, sizeof *out);
  out->first_violation_tick = UINT64_MAX;
  for (int d = 0; d < r->G; ++d) {
    raft_counters_t c = {0};
    sh_read_counters(r->sh[d], &c);
    out->node_ticks += c.node_ticks;
    for (int i = 0; i < RAFT_CTR_COUNT; ++i) out->c[i] += c.c[i];
    if (c.first_violation_tick < out->first_violation_tick)
      out->first_violation_tick = c.first_violation_tick;
    if (c.payload_max > out->payload_max) out->payload_max = c.payload_max;
  }
  return 0;
}

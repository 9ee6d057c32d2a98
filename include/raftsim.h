/* raftsim.h — C ABI of libraftsim.so, the MI355X batched Raft simulator.
 *
 * The reference (angelini/raft-simulation) has no FFI; its seams are the handler loop and the
 * three side-effect functions it calls. Each entry point below says which reference interface it
 * replaces. Semantics: SIM_SPEC.md. Conventions: 0 on success, a negative errno on failure
 * (-EINVAL bad argument, -ENOMEM allocation, -EIO HIP error); nothing throws across the ABI;
 * output buffers are caller-allocated; the library owns device memory; a handle is used by one
 * host thread at a time. `raft_sim_last_error()` explains the last failure (thread-local).
 */
#ifndef RAFTSIM_H
#define RAFTSIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RAFT_SIM_ABI_VERSION 2
#define RAFT_MAX_NODES 9
#define RAFT_MAX_INBOX 16

/* :state values of the node map (core.clj:33,70,76,81,87); 3 is the `:follwer` typo of
 * candidate->follower (core.clj:76), a distinct fourth value. */
enum raft_role { RAFT_FOLLOWER = 0, RAFT_CANDIDATE = 1, RAFT_LEADER = 2, RAFT_FOLLWER = 3 };

/* :type values (server.clj:8-12 for requests, core.clj:95,109 for replies). */
enum raft_msg_type {
  RAFT_MSG_REQUEST_VOTE = 1,
  RAFT_MSG_APPEND_ENTRIES = 2,
  RAFT_MSG_CLIENT_SET = 3,
  RAFT_MSG_VOTE_RESPONSE = 4,
  RAFT_MSG_APPEND_RESPONSE = 5
};

/* Exceptions that end a node's `loop` (core.clj:202-203), SIM_SPEC D8. */
enum raft_fault {
  RAFT_RUNNING = 0,
  RAFT_FAULT_IOOBE = 1,    /* nth past the end: val-at log.clj:23 */
  RAFT_FAULT_NPE = 2,      /* (dec nil): core.clj:146 */
  RAFT_FAULT_CCE = 3,      /* subvec of a LazySeq: log.clj:53 */
  RAFT_FAULT_OVERFLOW = 4  /* log capacity exceeded (simulator limit) */
};

/* Bug-injection / correct-protocol flags (SIM_SPEC §4, §8). */
enum raft_variant {
  RAFT_VARIANT_VOTE_NO_LOG_CHECK = 1, /* drop core.clj:96,99 (with SPEC: drop the up-to-date check) */
  RAFT_VARIANT_SPEC = 2               /* F4 Spec-Raft control: Raft Figure 2 rules (SIM_SPEC §8) */
};

/* How clusters are packed onto waves before each launch. Clusters are independent and Philox is
 * keyed by the global cluster id, so every packing gives bit-identical results; it only decides
 * which clusters share a wave, i.e. how many of a wave's ticks are active. */
enum raft_schedule {
  RAFT_SCHED_ALIGNED = 0, /* regroup clusters by their next event tick before every launch */
  RAFT_SCHED_FIXED = 1    /* cluster c always on wave c / floor(64/N) */
};

/* Replaces `-main`'s argv (core.clj:197-200), the hard-coded timeouts (core.clj:173-174) and the
 * chan buffer sizes (server.clj:37, client.clj:18). Defaults: raft_sim_default_config().
 * Limits (-EINVAL otherwise): cluster_offset + n_clusters <= 2^32 (global ids key Philox), and
 * nodes^2 * n_clusters < 2^31 (per-peer rows are indexed in 32 bits). */
typedef struct raft_sim_config {
  uint32_t n_clusters;     /* clusters simulated by this handle */
  uint32_t cluster_offset; /* global id of the first one (keys Philox: shard-invariant) */
  uint32_t nodes;          /* N, 2..9 */
  uint32_t log_cap;        /* L, max entries per log */
  uint32_t arena_cap;      /* A >= 2L log-arena slots per node; 0 -> 4L */
  uint32_t inbox_cap;      /* Q per queue, 1..16 */
  uint64_t seed;
  uint32_t hb, el_base, el_span;       /* 3000 / 5000 / 5000 ticks */
  uint32_t drop_ppm, dup_ppm, dmin, dmax;
  uint32_t part_ppm, part_epoch;
  uint32_t client_ppm;
  uint32_t variant_flags;
  int32_t device;            /* HIP device ordinal */
  uint32_t ticks_per_launch; /* ticks fused into one kernel launch; 0 -> default */
  uint32_t commit_stream_cap; /* per-node ring of committed :val's (log.clj:69-76); 0 = off */
  uint32_t trace_cap;         /* per-node ring of `wait` events (core.clj:182-186); 0 = off */
  uint32_t trace_entry_cap;   /* per-node ring of the :entries those events carried */
  uint32_t schedule;          /* cluster->wave packing, enum raft_schedule (results identical) */
  /* Client traffic (SIM_SPEC §4 P0, D9/D14/D15): client-sets arrive at client_ppm per tick during
   * bursts of client_burst ticks at the start of every client_period ticks (period 0: always on),
   * and a client follows up to client_redirects redirect-client hops (server.clj:62-63) towards the
   * :leader-id before it abandons the command (0: a redirect ends the command). */
  uint32_t client_period;
  uint32_t client_burst;      /* 1..client_period when client_period > 0 */
  uint32_t client_redirects;  /* 0..16 */
  /* Multi-GPU inside one handle: the clusters are split into n_devices contiguous shards
   * [n*d/G, n*(d+1)/G) (the split raftsim.dist.shard uses), shard d on HIP device
   * (device + d) mod the visible device count, one stream each; steps run on all shards at
   * once and raft_sim_read_counters reduces them (SUM; MIN first violation; MAX payload).
   * 0 means 1. Results are identical for every G (Philox is keyed by the global cluster id). */
  int32_t n_devices;
} raft_sim_config_t;

/* Canonical node record: the node map of init-node (core.clj:31-38) plus the log atom
 * (log.clj:33-34) and simulator bookkeeping. next/match are indexed by id-1; 0 where absent. */
typedef struct raft_node {
  uint8_t role, voted_for, leader_id, fault;
  uint8_t entries_is_seq, ls_present;
  uint16_t votes;   /* bit i: id i in the :votes set */
  uint16_t ls_keys; /* bit i: peer i has :next-index and :match-index keys */
  uint16_t reserved0;
  uint32_t current_term, commit_index, log_len, deadline;
  int32_t next_index[RAFT_MAX_NODES];
  int32_t match_index[RAFT_MAX_NODES];
  uint32_t last_led_term;
  uint32_t arena_base, arena_frontier;
  uint32_t req_count, res_count; /* read-only: set through raft_sim_write_queue */
  uint32_t commit_count;         /* lines apply-entries! has written to node_<id>.log so far */
  uint64_t trace_hash;
} raft_node_t;

/* One queued message (SIM_SPEC §3): hdr = type | src<<3 | flag<<7 | epresent<<8 | pcnt<<16. */
typedef struct raft_msg {
  uint32_t arrival, hdr, term, a, b, eterm, eval, poff;
} raft_msg_t;

typedef struct raft_entry {
  uint32_t term, val;
} raft_entry_t;

/* Per-cluster record: the leader-completeness checker's high-water mark (SIM_SPEC §4 P4) and the
 * client-set injection cursor (next injection tick, draws consumed; SIM_SPEC §4 P0). */
typedef struct raft_cluster {
  uint32_t hwm_index, hwm_term, hwm_val;
  uint32_t client_next, client_count;
  uint32_t reserved[3];
} raft_cluster_t;

/* F3: one iteration of `wait` as it prints (core.clj:182-186): the node map before the handler
 * (`; Node` / `(prn node)`) and the message alts!! returned (`; Message` / `(prn message)`). A
 * timeout (`nil`) has an all-zero msg. An append-entries' :entries are the msg.hdr>>16 entries of
 * the node's trace-entry ring starting at entries_seq (SIM_SPEC §7). */
typedef struct raft_trace_event {
  uint32_t tick;
  uint32_t seq;            /* this node's event number, from 0 */
  raft_msg_t msg;          /* as queued: arrival, hdr, term, a, b, eterm, eval, poff */
  uint8_t role, voted_for, leader_id, ls_present;
  uint16_t votes, ls_keys;
  uint32_t current_term;
  int32_t next_index[RAFT_MAX_NODES];
  int32_t match_index[RAFT_MAX_NODES];
  uint32_t entries_seq;
} raft_trace_event_t;

enum raft_counter {
  RAFT_CTR_EV_RV = 0, RAFT_CTR_EV_AE, RAFT_CTR_EV_CS, RAFT_CTR_EV_VR, RAFT_CTR_EV_AR,
  RAFT_CTR_EV_TIMEOUT, RAFT_CTR_EV_HEARTBEAT, RAFT_CTR_LEADERS, RAFT_CTR_SENT,
  RAFT_CTR_DELIVERED, RAFT_CTR_DROPPED, RAFT_CTR_PARTITIONED, RAFT_CTR_DUPLICATED,
  RAFT_CTR_OVERFLOW, RAFT_CTR_TO_HALTED, RAFT_CTR_CLIENT_INJECTED, RAFT_CTR_HALT_IOOBE,
  RAFT_CTR_HALT_NPE, RAFT_CTR_HALT_CCE, RAFT_CTR_HALT_OVERFLOW, RAFT_CTR_ENTRIES_APPENDED,
  RAFT_CTR_ENTRIES_APPLIED, RAFT_CTR_PAYLOAD_EVICTED, RAFT_CTR_VIOL_ELECTION,
  RAFT_CTR_VIOL_LOG, RAFT_CTR_VIOL_COMPLETE,
  RAFT_CTR_REDIRECTS,        /* client-sets re-sent along a redirect-client (server.clj:62-63) */
  RAFT_CTR_CLIENT_ABANDONED, /* client-sets a non-leader received with no redirect hop left */
  RAFT_CTR_COUNT
};

typedef struct raft_counters {
  uint64_t node_ticks;
  uint64_t first_violation_tick; /* UINT64_MAX when none */
  uint64_t c[RAFT_CTR_COUNT];    /* sums */
  uint64_t payload_max;          /* most :entries any append-entries carried (a maximum) */
} raft_counters_t;

typedef struct raft_sim raft_sim_t;

int raft_sim_abi_version(void);
void raft_sim_default_config(raft_sim_config_t* cfg);

/* Replaces raft-system + component/start (core.clj:23-29,201): allocates every cluster's nodes in
 * HBM in the init-node state (core.clj:31-38) with empty logs (log.clj:33-34). */
int raft_sim_create(const raft_sim_config_t* cfg, raft_sim_t** out);

/* Replaces the `(loop [node ...] (recur (wait system node)))` of -main (core.clj:202-203) for every
 * node of every cluster: advances all clusters by n_ticks (synchronous). A HIP failure part-way
 * through a step leaves the state between ticks the handle cannot name, so the handle is then
 * poisoned: every later step returns -EIO. */
int raft_sim_step(raft_sim_t* sim, uint32_t n_ticks);

/* raft_sim_step without the wait: enqueues the launches for n_ticks on every shard's stream and
 * returns. Reads, digests and the next step are stream-ordered after it; raft_sim_sync waits for
 * everything enqueued and makes raft_sim_last_step_timing cover those launches. Many steps
 * queued between syncs pay no host round trip per step. */
int raft_sim_step_async(raft_sim_t* sim, uint32_t n_ticks);
int raft_sim_sync(raft_sim_t* sim);

/* Ticks simulated so far (the next tick to run). */
uint64_t raft_sim_tick(const raft_sim_t* sim);

/* Resume: set the next tick to run, for state restored through the write_* calls below (deadlines
 * and arrivals are absolute ticks). Steps are refused (-ERANGE) once tick + n_ticks plus the
 * longest timer or delay (max(hb, el_base + el_span, dmax)) could reach 2^32 - 1, the "never"
 * marker, so no deadline or arrival can wrap. */
int raft_sim_set_tick(raft_sim_t* sim, uint64_t tick);

/* Replaces `(prn node)` of wait (core.clj:182-183): canonical records, N per cluster. */
int raft_sim_read_nodes(raft_sim_t* sim, uint32_t c0, uint32_t nc, raft_node_t* out);
int raft_sim_write_nodes(raft_sim_t* sim, uint32_t c0, uint32_t nc, const raft_node_t* in);

/* The req-chan (which=0, server.clj:37) or resp-chan (which=1, client.clj:18) contents of node
 * `node_id` (1..N), head first. read returns the count (>= 0) or a negative errno. */
int raft_sim_read_queue(raft_sim_t* sim, uint32_t cluster, uint32_t node_id, uint32_t which,
                        raft_msg_t* out, uint32_t cap);
int raft_sim_write_queue(raft_sim_t* sim, uint32_t cluster, uint32_t node_id, uint32_t which,
                         const raft_msg_t* in, uint32_t count);

/* The raw log arena (arena_cap entries) behind the Log atom's :entries (log.clj:33-34). */
int raft_sim_read_arena(raft_sim_t* sim, uint32_t cluster, uint32_t node_id, raft_entry_t* out,
                        uint32_t cap);
int raft_sim_write_arena(raft_sim_t* sim, uint32_t cluster, uint32_t node_id,
                         const raft_entry_t* in, uint32_t count);

/* F2: the newest min(count, commit_stream_cap, cap) values apply-entries! wrote to node_<id>.log
 * (log.clj:16-18,69-76), oldest first; returns how many were copied. write_commit_stream stores
 * `count` values as the newest ones ending at the node record's commit_count. */
int raft_sim_read_commit_stream(raft_sim_t* sim, uint32_t cluster, uint32_t node_id,
                                uint32_t* out, uint32_t cap);
int raft_sim_write_commit_stream(raft_sim_t* sim, uint32_t cluster, uint32_t node_id,
                                 const uint32_t* in, uint32_t count);

/* F3: the retained events of node `node_id` with seq >= first_seq, oldest first (the newest
 * trace_cap are kept); returns how many were copied. read_trace_entries copies the entries with
 * ring index first, first+1, ... (at most cap, up to the newest) and returns how many; -ERANGE if
 * entry `first` has already been overwritten (only the newest trace_entry_cap are kept). */
int raft_sim_read_trace(raft_sim_t* sim, uint32_t cluster, uint32_t node_id, uint32_t first_seq,
                        raft_trace_event_t* out, uint32_t cap);
int raft_sim_read_trace_entries(raft_sim_t* sim, uint32_t cluster, uint32_t node_id,
                                uint32_t first, raft_entry_t* out, uint32_t cap);

int raft_sim_read_clusters(raft_sim_t* sim, uint32_t c0, uint32_t nc, raft_cluster_t* out);
int raft_sim_write_clusters(raft_sim_t* sim, uint32_t c0, uint32_t nc, const raft_cluster_t* in);

/* Counters of this handle's clusters (no reference counterpart; see SIM_SPEC §4). */
int raft_sim_read_counters(raft_sim_t* sim, raft_counters_t* out);

/* Per-cluster FNV-1a-64 digest of the canonical state (SIM_SPEC §6). */
int raft_sim_digest(raft_sim_t* sim, uint32_t c0, uint32_t nc, uint64_t* out);

/* Average device time of the tick-kernel launches of the last raft_sim_step (or of the
 * raft_sim_step_async calls since the previous sync, once raft_sim_sync returned) alone, and the
 * launch count; for bench.py's roofline. An event pair in a launch's dispatch packet times it:
 * every general-kernel launch, and of the steady-path launches (~0.025 ms at config 2) only one
 * that comes first after a sync, since such a pair costs ~6 us per launch on MI355X; with
 * RAFTSIM_LAUNCH_EVENTS=1 in the environment at create every launch is timed. */
int raft_sim_last_step_timing(raft_sim_t* sim, double* avg_kernel_ms, uint32_t* launches);

/* Device time of everything the last raft_sim_step (or every raft_sim_step_async since the
 * previous sync, once raft_sim_sync returned) enqueued, from a HIP event before its first launch
 * to one after its last, on each shard's stream; the maximum over shards. Host time spent between
 * steps is not in it; gaps between the queued launches are. For bench.py's throughput. */
int raft_sim_last_span(raft_sim_t* sim, double* span_ms);

void raft_sim_destroy(raft_sim_t* sim);
const char* raft_sim_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* RAFTSIM_H */

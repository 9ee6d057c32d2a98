/* raftref.h — CPU oracle for the batched Raft simulator. TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of SIM_SPEC.md (itself restating src/raft/core.clj:19-195 and
 * src/raft/log.clj:5-87 of the reference). Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product (libraftsim.so) never does. It reuses the public ABI
 * types of include/raftsim.h so that records compare field for field. Same calls as the product
 * ABI with the raft_ref_ prefix, plus raft_ref_set_threads (the pmap analogue for the CPU
 * baseline: clusters are split into contiguous chunks, one std thread each).
 *
 * Parity status: PARITY UNPINNED by the reference, which ships no tests or golden vectors and
 * cannot run here (Clojure 1.6 on a JVM that this image lacks: SURVEY.md §8c). Pinned instead by
 * hand-derived known-answer scenarios (tests/scenarios.py, each citing its source lines), the
 * Random123 Philox vectors, and agreement with the independent Python restatement oracle/pyref.py
 * on random configurations and random states (tests/test_oracle.py, tests/test_fuzz.py).
 */
#ifndef RAFTREF_H
#define RAFTREF_H

#include "../include/raftsim.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct raft_ref raft_ref_t;

int raft_ref_abi_version(void);
void raft_ref_default_config(raft_sim_config_t* cfg);
int raft_ref_create(const raft_sim_config_t* cfg, raft_ref_t** out);
int raft_ref_set_threads(raft_ref_t* sim, int threads);
/* CPU baseline mode: visit only the ticks at which some node of a cluster can act (the same
 * discrete-event skipping the tick kernel does per wave); results are identical. */
int raft_ref_set_idle_skip(raft_ref_t* sim, int on);
int raft_ref_step(raft_ref_t* sim, uint32_t n_ticks);
int raft_ref_set_tick(raft_ref_t* sim, uint64_t tick);
int raft_ref_step_async(raft_ref_t* sim, uint32_t n_ticks);   /* = raft_ref_step (CPU) */
int raft_ref_sync(raft_ref_t* sim);                             /* no-op */
uint64_t raft_ref_tick(const raft_ref_t* sim);
int raft_ref_read_nodes(raft_ref_t* sim, uint32_t c0, uint32_t nc, raft_node_t* out);
int raft_ref_write_nodes(raft_ref_t* sim, uint32_t c0, uint32_t nc, const raft_node_t* in);
int raft_ref_read_queue(raft_ref_t* sim, uint32_t cluster, uint32_t node_id, uint32_t which,
                        raft_msg_t* out, uint32_t cap);
int raft_ref_write_queue(raft_ref_t* sim, uint32_t cluster, uint32_t node_id, uint32_t which,
                         const raft_msg_t* in, uint32_t count);
int raft_ref_read_arena(raft_ref_t* sim, uint32_t cluster, uint32_t node_id, raft_entry_t* out,
                        uint32_t cap);
int raft_ref_write_arena(raft_ref_t* sim, uint32_t cluster, uint32_t node_id,
                         const raft_entry_t* in, uint32_t count);
int raft_ref_read_commit_stream(raft_ref_t* sim, uint32_t cluster, uint32_t node_id,
                                uint32_t* out, uint32_t cap);
int raft_ref_write_commit_stream(raft_ref_t* sim, uint32_t cluster, uint32_t node_id,
                                 const uint32_t* in, uint32_t count);
int raft_ref_read_trace(raft_ref_t* sim, uint32_t cluster, uint32_t node_id, uint32_t first_seq,
                        raft_trace_event_t* out, uint32_t cap);
int raft_ref_read_trace_entries(raft_ref_t* sim, uint32_t cluster, uint32_t node_id,
                                uint32_t first, raft_entry_t* out, uint32_t cap);
int raft_ref_read_clusters(raft_ref_t* sim, uint32_t c0, uint32_t nc, raft_cluster_t* out);
int raft_ref_write_clusters(raft_ref_t* sim, uint32_t c0, uint32_t nc, const raft_cluster_t* in);
int raft_ref_read_counters(raft_ref_t* sim, raft_counters_t* out);
int raft_ref_digest(raft_ref_t* sim, uint32_t c0, uint32_t nc, uint64_t* out);
void raft_ref_destroy(raft_ref_t* sim);
const char* raft_ref_last_error(void);

/* Philox4x32-10 exposed for the KAT test. */
void raft_ref_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

#ifdef __cplusplus
}
#endif
#endif

// device.hpp — device-side building blocks of the tick kernel (gfx950 / CDNA4).
//
// Layout in HBM (node index gi = cluster * N + k, k = id - 1):
//   hot state        hot[c][HB]: one 128-B-aligned block per cluster holding every per-node word
//                    the tick kernel loads at launch start and stores at its end, field-major
//                    inside the block (word f * N + k = field f of node k; fields HotField below,
//                    next_index / match_index as N fields each), then the cluster's 8 words
//                    (raft_cluster_t: hwm index, term, val, client_next, client_count, 0, 0, 0).
//                    A wave's clusters come from the packing permutation, i.e. from anywhere in
//                    the shard: a block per cluster makes the wave's state load touch only its own
//                    clusters' lines (the structure-of-arrays layout read ~13 lines per load)
//   queues           8-word messages, one ring per node and queue, sorted by arrival: REQ rings
//                    slot-major qbuf[0][slot][gi], RES rings node-major qbuf[1][gi][slot] (qslots)
//   log arenas       arena[gi][A] of (term, val)
//   cold node words  ccount (commit_count), commit-stream / trace rings               [NN]...
// A wave owns floor(64 / N) whole clusters, one lane per node; a cluster never spans waves, so all
// intra-cluster traffic is lane-to-lane inside one wave (LDS cells + ds_bpermute).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/raftsim.h"

namespace rs {

constexpr uint32_t INF = 0xFFFFFFFFu;
enum { P_INIT = 1, P_EVENT = 2, P_NET = 3, P_CLIENT = 4, P_PART = 6 };
enum { PLAN_NONE = 0, PLAN_PAYLOAD = 1, PLAN_ENTRY = 2 };
constexpr int LCTR_FIRSTVIOL = RAFT_CTR_COUNT;       // per-wave LDS slot: min violation tick
constexpr int LCTR_PAYLOADMAX = RAFT_CTR_COUNT + 1;  // per-wave LDS slot: max AE payload
constexpr int LCTR_WORDS = 32;
constexpr int PW_WORDS = 32;    // the 32 client-gap powers' low words at the start of the wave's LDS
static_assert(LCTR_PAYLOADMAX < LCTR_WORDS, "counter block");
// Waves flush their counters into one of CTR_COPIES copies of the counter block (wave index mod
// CTR_COPIES): thousands of waves ending together otherwise serialise on the same few words of
// device-scope atomics (C2: 5,724 waves x up to 30 counters). The host reduces the copies.
constexpr int CTR_COPIES = 64;
// one counter block: the RAFT_CTR_COUNT sums, then the first violation tick (MIN over waves) and
// the largest append-entries payload (MAX over waves)
constexpr int CTR_STRIDE = RAFT_CTR_COUNT + 2;

// Exact unsigned division by a launch-invariant d >= 1 (Granlund & Montgomery, round-up variant):
// one v_mul_hi_u32 and a few shifts instead of the ~20-instruction division sequence, for every
// 32-bit x. The client schedule divides by its period and burst and the partition draw by its
// epoch on every injection and emission.
struct DivU32 {
  uint32_t d, m, s1, s2;
};
inline DivU32 make_div(uint32_t d) {
  uint32_t l = 0;
  while (l < 32 && (1ull << l) < d) ++l;
  return {d, (uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d + 1), l < 1 ? l : 1u,
          l > 1 ? l - 1 : 0u};
}
__device__ __forceinline__ uint32_t udiv(const DivU32& v, uint32_t x) {
  const uint32_t t1 = __umulhi(v.m, x);
  return (t1 + ((x - t1) >> v.s1)) >> v.s2;
}

struct DevSim {
  uint32_t C, N, Q, L, A, NN, goff, key0, key1;
  uint32_t hb, el_base, el_span, drop_ppm, dup_ppm, dmin, dmax, part_ppm, part_epoch,
      client_ppm, variant, client_period, client_burst, client_redirects;
  DivU32 div_period, div_burst, div_epoch;   // client_period (when > 0), client_burst, part_epoch
  uint32_t* hot;          // [C][HB] cluster blocks (HotField, hot_cl_off, hot_block_words)
  uint32_t HB;            // hot_block_words(N)
  uint32_t* qbuf;         // REQ [Q][NN][8], then RES [NN][Q][8]
  uint32_t* arena;        // [NN][A][2]
  uint32_t* ccount;       // [NN] commit_count (F2)
  uint32_t* stream;       // [NN][SC] commit-stream rings (F2)
  uint32_t SC;            // commit_stream_cap
  uint32_t* tr;           // [NN][TC][32] wait-event records (F3, raft_trace_event_t)
  uint32_t* tcount;       // [NN]
  uint2* tent;            // [NN][TE] :entries of recorded append-entries
  uint32_t* tecount;      // [NN]
  uint32_t TC, TE;
  const unsigned long long* client_pw;  // [32] powers of (1-p) (SIM_SPEC P0); staged into LDS
  int client_top;                       // highest i with client_pw[i] > 0, -1 if none,
                                        // 32 when client_ppm == 0 (every power 2^32)
  unsigned long long* ctr;  // [CTR_COPIES][CTR_STRIDE]: [RAFT_CTR_COUNT] sums, then the first
                            // violation (min) and the largest payload (max); summed by the host
  const uint32_t* perm;     // [slots] wave slot -> cluster or INF (RAFT_SCHED_ALIGNED), null = identity
  const uint32_t* nslots;   // RAFT_SCHED_ALIGNED: slots in use this launch (device word)
  uint32_t* skey;           // [C] RAFT_SCHED_ALIGNED: cluster's next event - next launch's t0
  uint32_t* shist;          // [SCHED_BUCKETS] histogram of skey (null: schedule fixed)
  uint32_t* wavelog;        // diagnostic builds (RS_WAVELOG) only: [waves][8] per-wave timeline
  uint32_t lite;            // no client traffic (and no finite client cursor), no faults, fixed
                            // delay: the LITE tick kernel applies
  // Steady kernel (steady_kernel.hip): clusters it stops ("bails") at a tick it does not model
  // are run from that tick by the same workgroup through the general tick body; their count is
  // summed here for the host's path choice (speed only).
  uint32_t* nbail;          // device word: clusters bailed this launch
  uint32_t* nbail_zero;     // the previous steady launch's word (two alternate): reported to
                            // bail_report and zeroed by this launch
  uint32_t* bail_report;    // host-mapped word (the host picks the next launches' path from it)
  // Storm launches (storm_kernel.hip): the clusters the lane-per-cluster kernel leaves to the
  // general STORM body, and their number (device word)
  uint32_t* storm_list;
  uint32_t* storm_count;
};

// The kernel's DevSim argument, read where a field is used. The kernels that run the tick body
// (tick_kernel, steady_lane_kernel) take their DevSim unmodified as the first argument, at offset
// 0 of the kernarg segment. A field read through this opaque constant-address pointer is a scalar
// load at its use; read from the plain parameter it is loaded once and held in an SGPR across the
// trip loop, whose uniform values exceed the SGPR file (the excess is spilled to VGPR lanes and
// costs a v_readlane at every use and two VGPRs). For the fields the trip loop uses rarely.
using KDevSim = const __attribute__((address_space(4))) DevSim;
__device__ __forceinline__ KDevSim* kargs() {
  KDevSim* p = (KDevSim*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}
__device__ __forceinline__ DivU32 kdiv(const __attribute__((address_space(4))) DivU32& v) {
  return DivU32{v.d, v.m, v.s1, v.s2};
}

// A cluster block: the cluster's 8 words (hot_cl_off = 0), then the node fields, field-major
// (word HOT_CW + f * N + k is field f of node k): the HotField fields, next_index of peer id p as
// field HF_NEXT + p - 1, match_index as HF_NEXT + N + p - 1, then the arena cursors and the
// last-led term (hf_abase / hf_afront / hf_led). Blocks are whole 128-B lines. The order puts what
// a steady-state launch writes -- every node's deadline and trace hash -- in one line (words 8-22
// at N = 5), and everything the steady kernel reads in the first four lines (words 0-122).
constexpr uint32_t HOT_CW = 8;
enum HotField : uint32_t {
  HF_DEADLINE, HF_TRACE_LO, HF_TRACE_HI, HF_QMETA, HF_REQ_ARR, HF_RES_ARR, HF_REQ_TAIL,
  HF_RES_TAIL, HF_FLAGS, HF_MASKS, HF_TERM, HF_COMMIT, HF_LEN, HF_NEXT
};
__host__ __device__ constexpr uint32_t hf_abase(uint32_t N) { return HF_NEXT + 2 * N; }
__host__ __device__ constexpr uint32_t hf_afront(uint32_t N) { return HF_NEXT + 2 * N + 1; }
__host__ __device__ constexpr uint32_t hf_led(uint32_t N) { return HF_NEXT + 2 * N + 2; }
__host__ __device__ constexpr uint32_t hot_cl_off(uint32_t) { return 0; }
__host__ __device__ constexpr uint32_t hot_block_words(uint32_t N) {
  return (HOT_CW + (hf_led(N) + 1) * N + 31) & ~31u;
}
// Word 0 of node k's fields in cluster c's block (field f at [f * N]) / the cluster's 8 words.
__device__ __forceinline__ uint32_t* hot_node(const DevSim& S, uint32_t c, uint32_t k) {
  return S.hot + (size_t)c * S.HB + HOT_CW + k;
}
__device__ __forceinline__ uint32_t* hot_cl(const DevSim& S, uint32_t c) {
  return S.hot + (size_t)c * S.HB + hot_cl_off(S.N);
}

constexpr uint32_t SCHED_BUCKETS = 16384;   // keys clamp to SCHED_BUCKETS - 1
constexpr uint32_t SCHED_PAST = 16;         // bucket of "now": keys keep 16 ticks of past

// The histogram bucket of a cluster whose next event is `ev`, for a launch starting at t0. Events
// up to SCHED_PAST ticks in the past (messages that arrived but wait behind others, e.g. a
// leader's remaining append-responses in mid round) keep their tick: they tell a cluster that is
// 3 ticks into a heartbeat round from one that starts a round at t0, whose later rounds would
// otherwise stay 3 ticks apart in the same wave.
__device__ __forceinline__ uint32_t sched_bucket(uint32_t ev, uint32_t t0) {
  const uint64_t k = (uint64_t)ev + SCHED_PAST;
  if (k <= t0) return 0;
  const uint64_t d = k - t0;
  return d < SCHED_BUCKETS - 1 ? (uint32_t)d : SCHED_BUCKETS - 1;
}

// Slots the padded wave packing may use (RAFT_SCHED_ALIGNED): twice the clusters plus one partial
// wave per plan chunk (SCHED_PLAN_CHUNKS), so the unpadded fallback always fits; the tick kernel's
// grid covers this many and waves past the slots in use exit at once.
constexpr uint32_t SCHED_PLAN_CHUNKS = 1024;
__host__ __device__ inline uint32_t sched_slots_bound(uint32_t C, uint32_t N) {
  const uint32_t CPW = 64 / N;
  return ((2 * C + CPW - 1) / CPW + SCHED_PLAN_CHUNKS) * CPW;
}

// Philox4x32-10 (Random123; round and key schedule of rocrand_philox4x32_10.h).
__host__ __device__ __forceinline__ uint4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                 uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one 32x32->64 product (v_mad_u64_u32) gives both halves (against a mul_lo + mul_hi pair:
    // C4-N9 -5.5 %, C3 -1.6 %)
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c0 = hi1 ^ c1 ^ k0;
    c1 = lo1;
    c2 = hi0 ^ c3 ^ k1;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return make_uint4(c0, c1, c2, c3);
}

__device__ __forceinline__ uint32_t ppm(uint32_t w) { return __umulhi(w, 1000000u); }

// pw_i = (1-p)^(2^i) in 32-bit fixed point, truncating (SIM_SPEC §4 P0); computed on the host.
inline void client_powers(uint32_t client_ppm, uint64_t pw[32]) {
  pw[0] = ((uint64_t)(1000000u - client_ppm) << 32) / 1000000u;
  for (int i = 1; i < 32; ++i)   // exact: 2^32 squared (client_ppm = 0) stays 2^32
    pw[i] = pw[i - 1] == 1ull << 32 ? pw[i - 1] : (pw[i - 1] * pw[i - 1]) >> 32;
}

// Geometric gap G(w) of SIM_SPEC §4 P0: the greedy power search over pw[top..0] (higher powers
// are 0 and never fire). The accumulator starts at 2^32 and every power is below 2^32 when
// client_ppm > 0, so after its first step it fits 32 bits and (acc * pw) >> 32 is one
// v_mul_hi_u32 instead of a 64x64-bit product; c >= w + 1 is c > w. pw: the low words of the
// powers (the wave's LDS copy, or the kernel argument's u64 table). The low GAP_UNROLL powers
// are loaded together before the chain (the accumulator does not decide which power a step
// reads), so a step costs its multiply and select rather than a load's latency: 600 -> ~ cycles
// per draw at four waves per SIMD (scripts/p0_probe.hip; a loop with a load per step waited on
// each); powers above them (client_ppm < ~2 %) take a step per loop trip first.
constexpr int GAP_UNROLL = 12;
template <typename P>
__device__ inline uint64_t client_gap(uint32_t w, P pw, int top) {
  // client_ppm == 0 (top == 32; reachable only through a host-written client cursor): every
  // power is 2^32, so the search takes every step
  if (top > 31) return 0xFFFFFFFFull;
  uint32_t acc = 0, g = 0;
  bool full = true;                 // acc == 2^32
  int i = top;
  for (; i >= GAP_UNROLL; --i) {
    const uint32_t p = (uint32_t)pw[i];
    const uint32_t c = full ? p : __umulhi(acc, p);
    if (c > w) {
      acc = c;
      full = false;
      g += 1u << i;
    }
  }
  uint32_t p[GAP_UNROLL];
#pragma unroll
  for (int j = 0; j < GAP_UNROLL; ++j) p[j] = (uint32_t)pw[j];
#pragma unroll
  for (int j = GAP_UNROLL - 1; j >= 0; --j) {
    const uint32_t c = full ? p[j] : __umulhi(acc, p[j]);
    const bool fire = j <= i && c > w;
    acc = fire ? c : acc;
    full = full && !fire;
    g += fire ? 1u << j : 0u;
  }
  return g;
}

// The powers' low words (DevSim::client_pw) read through the constant address space: the table is
// written by the host only, so the compiler may load it with uniform scalar loads into SGPRs (a
// vector load of each power held twelve VGPRs during the gap search).
struct PowersS {
  const __attribute__((address_space(4))) uint32_t* p;
  __device__ explicit PowersS(const unsigned long long* pw)
      : p((const __attribute__((address_space(4))) uint32_t*)pw) {}
  __device__ uint32_t operator[](int i) const { return p[2 * i]; }
};

// The client schedule (SIM_SPEC §4 P0, D14): bursts of B on-ticks at the start of every period P
// (P = 0: every tick is on). Injections are spaced by geometric gaps counted in on-ticks: the tick
// of on-tick number j, saturating at 2^32 - 1 = never (j >= 2^32 is never, as tick(j) >= j).
__device__ inline uint32_t on_tick(uint64_t j, uint32_t P, const DivU32& B) {
  if (j >= 0xFFFFFFFFull) return 0xFFFFFFFFu;
  const uint32_t j32 = (uint32_t)j;
  const uint32_t q = P ? udiv(B, j32) : 0u;
  const uint64_t t = P ? (uint64_t)q * P + (j32 - q * B.d) : j32;
  return t < 0xFFFFFFFFull ? (uint32_t)t : 0xFFFFFFFFu;
}
// The on-tick number of on-tick t (the inverse of on_tick).
__device__ __forceinline__ uint64_t on_index(uint32_t t, const DevSim& S) {
  const uint32_t P = S.client_period;
  const uint32_t q = P ? udiv(S.div_period, t) : 0u;
  return P ? (uint64_t)q * S.div_burst.d + (t - q * P) : t;
}
// The next injection after the one at tick t (an on-tick), drawing gap word w.
__device__ inline uint32_t client_next_tick(uint32_t t, uint32_t w, const DevSim& S,
                                            const uint32_t* pw) {
  return on_tick(on_index(t, S) + 1 + client_gap(w, pw, S.client_top), S.client_period,
                 S.div_burst);
}
__device__ __forceinline__ uint64_t fnv(uint64_t h, uint32_t w) {
  return (h ^ w) * 0x100000001B3ull;
}

// The trace hash's step (SIM_SPEC §4): h <- (h * M + x0) * M + x1 mod 2^64 over two 64-bit words,
// x0 = t | (ev | src << 3 | role << 7 | fault << 9) << 32, x1 = msg_term | current_term << 32,
// computed as h * M^2 + (x0 * M + x1): the event's own term is off the hash's dependency chain,
// which is one 64-bit multiply-add per event. A polynomial hash, so a run of events whose words
// only shift by a constant tick offset folds into one multiply-add per run (steady_kernel.hip).
constexpr uint64_t TRACE_M = 0x9E3779B97F4A7C15ull;
constexpr uint64_t TRACE_M2 = TRACE_M * TRACE_M;
__device__ __forceinline__ uint64_t trace_term(uint32_t t, uint32_t ev, uint32_t src,
                                               uint32_t mterm, uint32_t role, uint32_t term,
                                               uint32_t fault) {
  const uint64_t x0 = (uint64_t)t | (uint64_t)(ev | src << 3 | role << 7 | fault << 9) << 32;
  const uint64_t x1 = (uint64_t)mterm | (uint64_t)term << 32;
  return x0 * TRACE_M + x1;
}
__device__ __forceinline__ uint64_t trace_event(uint64_t h, uint32_t t, uint32_t ev, uint32_t src,
                                                uint32_t mterm, uint32_t role, uint32_t term,
                                                uint32_t fault) {
  return h * TRACE_M2 + trace_term(t, ev, src, mterm, role, term, fault);
}

// A deferred timer in the stored state. A non-leader's re-armed deadline is t + el_base + the
// EVENT draw of (its cluster, its id, t) scaled to el_span (SIM_SPEC D4); the kernels only compare
// it with ticks at or past t + el_base, so they keep t + el_base and draw when a tick reaches it
// (tick_wave's dpend, the steady kernel's fpend). FL_DRAW in the flags word carries that state
// across launches: the stored deadline is the lower bound t + el_base and the draw is still owed.
// Whatever reads the state resolves it (exact_deadline): the digest kernel, raft_sim_read_nodes;
// the value is the one the draw would have given at any time.
constexpr uint32_t FL_DRAW = 1u << 15;
// The steady certificate: cluster word CL_CERT = CERT_MAGIC | L, written by the steady kernel for a
// cluster it leaves at its fixed point (steady_kernel.hip) with node L as leader, promises that the
// block's lines past the second hold that fixed point's words (empty logs, commit 0, the leader's
// next / match rows 0) -- the next steady launch then reads the first two lines only. Every other
// writer of a block clears it: the general tick body's write-back, raft_sim_write_nodes,
// raft_sim_write_queue and raft_sim_write_clusters (whose reserved words it is; reads return them
// zeroed), and the init kernel.
constexpr uint32_t CL_CERT = 7;
constexpr uint32_t CERT_MAGIC = 0x5EAD0000u;
__host__ __device__ __forceinline__ uint32_t exact_deadline(uint32_t g, uint32_t id, uint32_t lb,
                                                            uint32_t el_base, uint32_t el_span,
                                                            uint32_t k0, uint32_t k1) {
  const uint4 w = philox(g, id | P_EVENT << 8, lb - el_base, 0, k0, k1);
  return lb + (uint32_t)(((uint64_t)w.y * el_span) >> 32);
}

// The EVENT draw of node id at tick t (SIM_SPEC §3): alts!! bit, timeout, rand-nth peer.
__device__ __forceinline__ uint4 event_draw(uint32_t g, uint32_t id, uint32_t t, const DevSim& S) {
  return philox(g, id | P_EVENT << 8, t, 0, S.key0, S.key1);
}

// Flags word: role 0-1 | voted_for 2-5 | leader_id 6-9 | fault 10-12 | is_seq 13 | ls_present 14
__host__ __device__ __forceinline__ uint32_t pack_flags(uint32_t role, uint32_t vf, uint32_t lid,
                                                        uint32_t fault, uint32_t seq,
                                                        uint32_t lsp) {
  return role | vf << 2 | lid << 6 | fault << 10 | seq << 13 | lsp << 14;
}
// qmeta: req_head 0-3 | req_cnt 4-8 | res_head 9-12 | res_cnt 13-17
__host__ __device__ __forceinline__ uint32_t pack_qmeta(uint32_t rqh, uint32_t rqc, uint32_t rsh,
                                                        uint32_t rsc) {
  return rqh | rqc << 4 | rsh << 9 | rsc << 13;
}

// One queue's registers: ring head, count, head arrival (INF when empty), tail arrival.
struct QueueR {
  uint32_t h, c, arr, tail;
};

// Node registers held by one lane for a whole launch. Queues are named fields (never indexed by a
// runtime value) so that they stay in VGPRs.
struct NodeR {
  // keys: the leader-state's peer keys (bits 1..N) and, in bit 0, whether it is present (ls_present;
  // a state with keys but no leader-state is rejected by raft_sim_write_nodes)
  uint32_t role, vf, lid, fault, seq, votes, keys;
  uint32_t term, commit, len, deadline;
  QueueR rq, rs;
  uint32_t base, front, led;
  uint64_t trace;
};

// Wave-wide unsigned minimum (all 64 lanes must be active): DPP row shifts build per-row prefix
// minima, row_bcast15/31 carry them across rows, lane 63 ends with the wave's minimum.
__device__ __forceinline__ uint32_t wave_min(uint32_t x) {
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)INF, (int)x, 0x111, 0xf, 0xf, false));
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)INF, (int)x, 0x112, 0xf, 0xf, false));
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)INF, (int)x, 0x114, 0xf, 0xf, false));
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)INF, (int)x, 0x118, 0xf, 0xf, false));
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)INF, (int)x, 0x142, 0xa, 0xf, false));
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)INF, (int)x, 0x143, 0xc, 0xf, false));
  return __builtin_amdgcn_readlane(x, 63);
}

// Wave-wide sum (all 64 lanes active), uniform: DPP row shifts and broadcasts as in wave_min.
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
  return __builtin_amdgcn_readlane(x, 63);
}

__device__ __forceinline__ uint32_t wrapq(uint32_t x, uint32_t Q) { return x >= Q ? x - Q : x; }

// Slot 0 of node gi's queue `which`; slot i is qslots(...) + i * qstride(S, which). REQ rings are
// slot-major ([slot][gi]: the followers of a cluster take their append-entries in the same tick
// from adjacent words), RES rings node-major ([gi][slot]: a leader takes its responses one per
// tick from consecutive slots of one line).
__device__ __forceinline__ uint32_t* qslots(const DevSim& S, uint32_t gi, int which) {
  return S.qbuf + (which ? (size_t)S.Q * S.NN + (size_t)gi * S.Q : (size_t)gi) * 8;
}
__device__ __forceinline__ size_t qstride(const DevSim& S, int which) {
  return which ? 8 : (size_t)S.NN * 8;
}

// slots of padding after the last node's arena: the chunked arena loops (tick_wave.hpp) may read
// up to 7 slots past a run's end
constexpr uint32_t ARENA_PAD_SLOTS = 16;
__device__ __forceinline__ uint2* arena_of(const DevSim& S, uint32_t gi) {
  return reinterpret_cast<uint2*>(S.arena) + (size_t)gi * S.A;
}

#ifndef RS_KO_CTR
#define RS_KO_CTR 0     // knock-out switch of timing-only diagnostic builds: never set in the product
#endif
__device__ __forceinline__ void lctr_add(uint32_t* lctr, int i, uint32_t v) {
  if (!RS_KO_CTR && v) atomicAdd(&lctr[i], v);
}

// Stable insert of message (m0 = arrival,hdr,term,a ; m1 = b,eterm,eval,poff) into the node's own
// queue `which` (SIM_SPEC §4 P2: after every queued message whose arrival <= the new one).
// (rdel / rhalt: the caller's register counts of delivered messages and of messages reaching a
// halted node, or null for the LDS counters)
__device__ __forceinline__ void qinsert(const DevSim& S, uint32_t gi, uint32_t fault, int which,
                                        QueueR& q, uint4 m0, uint4 m1, uint32_t* lctr,
                                        uint32_t* rdel = nullptr, uint32_t* rhalt = nullptr) {
  if (fault) {
    if (rhalt) *rhalt += 1;
    else lctr_add(lctr, RAFT_CTR_TO_HALTED, 1);
    return;
  }
  const uint32_t Q = S.Q;
  if (q.c >= Q) {
    lctr_add(lctr, RAFT_CTR_OVERFLOW, 1);
    return;
  }
  uint32_t* qb = qslots(S, gi, which);
  const size_t qs = qstride(S, which);
  const uint32_t arr = m0.x, head = q.h;
  uint32_t pos = q.c;
  if (pos > 0 && arr < q.tail) {
    while (pos > 0) {
      const uint32_t prev = wrapq(head + pos - 1, Q);
      if (qb[prev * qs] <= arr) break;
      const uint32_t dst = wrapq(head + pos, Q);
      uint4* sp = reinterpret_cast<uint4*>(qb + prev * qs);
      uint4* dp = reinterpret_cast<uint4*>(qb + dst * qs);
      dp[0] = sp[0];
      dp[1] = sp[1];
      --pos;
    }
  } else {
    q.tail = arr;
  }
  uint4* dp = reinterpret_cast<uint4*>(qb + wrapq(head + pos, Q) * qs);
  dp[0] = m0;
  dp[1] = m1;
  q.c += 1;
  if (pos == 0) q.arr = arr;
  if (rdel) *rdel += 1;
  else lctr_add(lctr, RAFT_CTR_DELIVERED, 1);
}

}  // namespace rs

// tick_wave.hpp — the general tick body for gfx950 (MI355X): one wave's clusters over a launch.
//
// One lane per node, one wave per floor(64/N) clusters, `nt` ticks fused per launch with all hot
// node state in VGPRs. Per tick a lane does the reference's `wait` (src/raft/core.clj:176-195) once:
// pick at most one event (D3), run the handler (core.clj:91-169, log.clj:5-87), emit messages into
// LDS cells, then — only when some lane of the wave did something — the wave runs the network
// (P2), log transfer (P3) and checker (P4) phases of SIM_SPEC.md §4. Idle ticks cost a handful of
// VALU instructions and one ballot. Used by the general tick kernel (tick_kernel.hip) and by the
// steady kernel's in-workgroup catch-up (steady_kernel.hip).
#pragma once
#include "device.hpp"

namespace rs {

#ifndef RS_PROV
#define RS_PROV 1
#endif
#ifndef RS_PROV_SEARCH
#define RS_PROV_SEARCH 1
#endif
#ifndef RS_PROV_MIN_N
#define RS_PROV_MIN_N 6
#endif
#ifndef RS_RC_MIN_N
#define RS_RC_MIN_N 6
#endif
#ifndef RS_REGS_MIN_N
#define RS_REGS_MIN_N 6
#endif
#ifndef RS_KA_HOIST
#define RS_KA_HOIST 1
#endif
#ifndef RS_SHFL_GUARD
#define RS_SHFL_GUARD 1
#endif
#ifndef RS_BURST
#define RS_BURST 1
#endif
#ifndef RS_BURST_KO_CMP  // timing-only knock-out of the burst engine's log-matching loads (wrong results)
#define RS_BURST_KO_CMP 0
#endif
#ifndef RS_BURST_MIN      // the shortest engine run worth an entry (ticks)
#define RS_BURST_MIN 16
#endif
#ifndef RS_BURST_SKIP     // trips a wave skips the engine's entry check after one that found no entry
#define RS_BURST_SKIP 8
#endif
#ifndef RS_BURST_PRE      // evaluate the engine's entry only on trips with an injection or a queued leader
#define RS_BURST_PRE 0
#endif
#ifndef RS_BURST_DIAG   // timing-only diagnostic builds: engine ticks, entries, yields and trips in
#define RS_BURST_DIAG 0 // four counters C4 never uses (wrong counters): never set in the product
#endif

// knock-out switches of timing-only diagnostic builds (wrong results): never set in the product
#ifndef RS_KO_P4
#define RS_KO_P4 0
#endif
#ifndef RS_KO_LOGM
#define RS_KO_LOGM 0
#endif

__device__ __forceinline__ void violation(uint32_t* lctr, int kind, uint32_t t) {
  atomicAdd(&lctr[kind], 1u);
  atomicMin(&lctr[LCTR_FIRSTVIOL], t);
}

// LDS message cells. A node emits either one broadcast or one reply per tick, and the words
// (term, a) of a broadcast are the same for every peer, so they live once per sender in a 2-word
// sender record; each (sender, receiver) pair cell holds the other six: hdr, b, eterm, eval, poff
// and the delivery pack transmit() adds. 26 words per five-node sender instead of 32 keeps a
// block of four waves under 1/6 of the CU's LDS.
constexpr int CELLW = 6;
constexpr int SRECW = 2;

// One emitted message a = (hdr, term, a, b), b = (eterm, eval, poff, -) into its pair cell (the
// sender record is written once per emission by the caller).
__device__ __forceinline__ void cell_put(uint32_t* cl, uint4 a, uint4 b) {
  reinterpret_cast<uint2*>(cl)[0] = make_uint2(a.x, a.w);
  reinterpret_cast<uint2*>(cl)[1] = make_uint2(b.x, b.y);
  cl[4] = b.z;
}

// P2 fault draws for one network message from node `src` to node `id` emitted at tick t (keyed by
// cluster, sender, tick and receiver). Returns the delivery pack: copy 0's delay in bits 0-7, copy
// 1's in bits 8-15, the copy count (0: lost) in bits 16-17. (Made by the receivers' lanes instead
// -- a broadcast's draws in parallel -- C3 was 3 % slower: a leader's N - 1 responses then cost
// its lane N - 1 draws in a row.)
template <bool LITE>
__device__ __forceinline__ uint32_t deliver_pack(const DevSim& S, uint32_t g, uint32_t t,
                                                 uint32_t src, uint32_t id, uint32_t pstate,
                                                 uint32_t* lctr) {
  if (LITE) return S.dmin | 1u << 16;
  KDevSim* const K = kargs();
  const uint32_t drop = K->drop_ppm, dup = K->dup_ppm, dmin = K->dmin, dmax = K->dmax;
  if (!drop && !dup && !K->part_ppm && dmin == dmax) return dmin | 1u << 16;
  // pstate: the cluster's partition draw of this epoch (bit 0: partitioned, bit i: node i's side)
  if ((pstate & 1) && (((pstate >> id) ^ (pstate >> src)) & 1)) {
    lctr_add(lctr, RAFT_CTR_PARTITIONED, 1);
    return 0;
  }
  if (!drop && !dup && dmin == dmax) return dmin | 1u << 16;
  const uint4 w = philox(g, src | P_NET << 8, t, id, S.key0, S.key1);
  if (ppm(w.x) < drop) {
    lctr_add(lctr, RAFT_CTR_DROPPED, 1);
    return 0;
  }
  const uint32_t span = dmax - dmin + 1;
  uint32_t pack = (dmin + __umulhi(w.z, span)) | 1u << 16;
  if (ppm(w.y) < dup) {
    lctr_add(lctr, RAFT_CTR_DUPLICATED, 1);
    pack = (pack & 0xFF) | (dmin + __umulhi(w.w, span)) << 8 | 2u << 16;
  }
  return pack;
}

// A node's leader-state words next_index / match_index (peer p = id - 1). In HBM they are fields
// of the cluster block (stride N); kernels with a small N keep the wave's rows in LDS for the whole
// launch (NM_LDS below) so heartbeats and append-responses pay no global round trip for them.
struct PeerW {
  int32_t* nx;
  int32_t* mt;
  uint32_t stride;
  __device__ __forceinline__ int32_t& next(uint32_t p) const { return nx[p * stride]; }
  __device__ __forceinline__ int32_t& match(uint32_t p) const { return mt[p * stride]; }
};

// F3: record one `wait` iteration (core.clj:182-186) — the node map before the handler and the
// message alts!! returned — as a raft_trace_event_t (32 words) in the node's ring.
template <int N>
__device__ __forceinline__ void trace_record(const DevSim& S, uint32_t gi, uint32_t t,
                                             const NodeR& n, const PeerW& lsw, uint4 m0, uint4 m1,
                                             uint32_t tes) {
  const uint32_t seq = S.tcount[gi];
  S.tcount[gi] = seq + 1;
  uint32_t w[32];
  w[0] = t; w[1] = seq;
  w[2] = m0.x; w[3] = m0.y; w[4] = m0.z; w[5] = m0.w;
  w[6] = m1.x; w[7] = m1.y; w[8] = m1.z; w[9] = m1.w;
  w[10] = n.role | n.vf << 8 | n.lid << 16 | (n.keys & 1u) << 24;
  w[11] = n.votes | (n.keys & ~1u) << 16;
  w[12] = n.term;
#pragma unroll
  for (int p = 0; p < RAFT_MAX_NODES; ++p) {
    w[13 + p] = p < N ? (uint32_t)lsw.next(p) : 0u;
    w[22 + p] = p < N ? (uint32_t)lsw.match(p) : 0u;
  }
  w[31] = tes;
  uint4* rec = reinterpret_cast<uint4*>(S.tr + ((size_t)gi * S.TC + seq % S.TC) * 32);
#pragma unroll
  for (int i = 0; i < 8; ++i) rec[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}

// Arena runs. A node's arena is A slots; a run of consecutive log positions starts at some slot
// and wraps at A. The loops below take a run W (or B) slots at a time with one address per
// run and immediate-offset loads -- a chunk ends at the run's end or at either arena's wrap point,
// whichever is first -- so a position costs a few VALU instead of the ~16 of a per-slot wrap and
// 64-bit address. A chunk's loads may read up to W - 1 slots past its end: inside the next node's
// arena, or the ARENA_PAD_SLOTS of padding after the last one (raftsim.hip); those lanes of the
// chunk are masked.

// One chunk of a Log Matching run: compares up to W consecutive positions of two logs whose next
// slots are xi in arena xa and yi in arena ya (cnt positions left in the run). Returns the
// positions consumed (the chunk ends at the run's end or at either arena's wrap point) and sets
// hit when one of them has the same term and a different value. The caller advances xi / yi
// (wrapping at A) and loops; the checker (P4) interleaves these steps over a wave's lanes.
template <int W = 8>
__device__ __forceinline__ uint32_t log_conflict_chunk(const uint2* xa, uint32_t xi,
                                                       const uint2* ya, uint32_t yi, uint32_t cnt,
                                                       uint32_t A, bool& hit) {
  const uint32_t c = min(min(cnt, (uint32_t)W), min(A - xi, A - yi));
  const uint2* xp = xa + xi;
  const uint2* yp = ya + yi;
  uint2 x[W], y[W];
#pragma unroll
  for (int j = 0; j < W; ++j) {
    x[j] = xp[j];
    y[j] = yp[j];
  }
  hit = false;
#pragma unroll
  for (int j = 0; j < W; ++j) hit |= (uint32_t)j < c && x[j].x == y[j].x && x[j].y != y[j].y;
  return c;
}

// Copy `cnt` arena entries from slot si of `src` to slot di of `dst`, in ascending order with every
// load of a B-slot chunk ahead of its stores. That reproduces the oracle's element-by-element copy
// also for a relocation inside one arena (dst = the frontier, src = the old base): the distance
// d = frontier - base satisfies cnt <= d < A (a log never exceeds L <= A / 2 positions past its
// base), so a slot the copy overwrites is one it read at an earlier position (or in the same
// chunk, before the chunk's stores).
template <uint32_t B = 8>
__device__ __forceinline__ void arena_copy(uint2* dst, uint32_t di, const uint2* src, uint32_t si,
                                           uint32_t cnt, uint32_t A) {
  while (cnt) {
    if (cnt >= B && si + B <= A && di + B <= A) {
      uint2 v[B];
      const uint2* sp = src + si;
      uint2* dp = dst + di;
#pragma unroll
      for (int j = 0; j < (int)B; ++j) v[j] = sp[j];
#pragma unroll
      for (int j = 0; j < (int)B; ++j) dp[j] = v[j];
      si += B;
      di += B;
      cnt -= B;
    } else {
      dst[di] = src[si];
      ++si;
      ++di;
      --cnt;
    }
    si = si == A ? 0 : si;
    di = di == A ? 0 : di;
  }
}

// F4 Spec-Raft control (SIM_SPEC §8): one event of a running node under Raft's Figure 2 rules.
// NOT reference behaviour. Same contract as the faithful handler below it in tick_kernel: decide
// `fault` (OVERFLOW only) before touching the node, then mutate `n` in place and describe the
// emission (emit/ra/rb), the leader-state writes (nm) and the P3 log plan.
template <int N, uint32_t MAJ>
__device__ __forceinline__ void spec_handle(
    const DevSim& S, NodeR& n, const PeerW& lsw, const uint2* sar, const uint32_t* fr,
    uint32_t* lctr, int which,
    uint32_t id, int k, int bl, uint32_t sgi, uint32_t peers, uint4 m0, uint4 m1,
    uint32_t& fault, uint32_t& ev, int& emit, int& nm, uint4& ra, uint4& rb, uint32_t& appended,
    uint32_t& applied, uint32_t& pkind, uint32_t& psrc, uint32_t& ppoff, uint32_t& ppcnt,
    uint32_t& pold_base, uint32_t& preloc, uint32_t& papplied, bool& elected, bool& mchg,
    bool& rearm, uint32_t pk, uint32_t pm) {
  const uint32_t A = S.A;
  if (which < 0) {
    if (n.role == RAFT_LEADER) {                                  // heartbeat
      ev = 7;
      emit = 2;
    } else {                                                      // election timeout
      ev = 6;
      uint32_t ep = 0, et = 0, evl = 0;
      if (n.len) {
        const uint2 e = sar[(n.base + n.len - 1) % A];
        ep = 1; et = e.x; evl = e.y;
      }
      n.role = RAFT_CANDIDATE; n.vf = id; n.votes = 1u << id; n.term += 1;
      ra = make_uint4(RAFT_MSG_REQUEST_VOTE | id << 3 | ep << 8, n.term, n.len, 0);
      rb = make_uint4(et, evl, 0, 0);
      emit = 1;
    }
    return;
  }
  const uint32_t hdr = m0.y, mterm = m0.z, ma = m0.w, mb = m1.x, met = m1.y, mpoff = m1.w;
  const uint32_t type = hdr & 7, src = (hdr >> 3) & 15, flag = (hdr >> 7) & 1,
                 mep = (hdr >> 8) & 1, pcnt = hdr >> 16;
  ev = type;
  // OVERFLOW, the only Spec-Raft halt, is decided on the pre-event state
  bool consistent = false;
  if (type == RAFT_MSG_APPEND_ENTRIES && mterm >= n.term) {
    consistent = mb == 0;
    if (!consistent && mb <= n.len && mep) consistent = sar[(n.base + mb - 1) % A].x == met;
    if (consistent && mb + pcnt > kargs()->L) fault = RAFT_FAULT_OVERFLOW;
  }
  if (type == RAFT_MSG_CLIENT_SET && n.role == RAFT_LEADER && n.len + 1 > kargs()->L)
    fault = RAFT_FAULT_OVERFLOW;
  if (fault) return;
  if (type != RAFT_MSG_CLIENT_SET && mterm > n.term) {          // term rule: step down
    n.term = mterm; n.vf = 0; n.votes = 0; n.lid = 0; n.role = RAFT_FOLLOWER;
    if (n.keys & 1u) { n.keys = 0; nm = 2; }
  }
  switch (type) {
    case RAFT_MSG_REQUEST_VOTE: {
      const uint32_t lt = n.len ? sar[(n.base + n.len - 1) % A].x : 0u;
      const uint32_t mt = mep ? met : 0u;
      const bool up = (kargs()->variant & RAFT_VARIANT_VOTE_NO_LOG_CHECK) || mt > lt ||
                      (mt == lt && ma >= n.len);
      const uint32_t grant = mterm == n.term && (n.vf == 0 || n.vf == src) && up;
      ra = make_uint4(RAFT_MSG_VOTE_RESPONSE | id << 3 | grant << 7, n.term, 0, 0);
      if (grant) {
        n.vf = src;
        rearm = true;                       // Figure 2: granting a vote resets the timer
      }
      emit = 3;
      break;
    }
    case RAFT_MSG_APPEND_ENTRIES: {
      ra = make_uint4(RAFT_MSG_APPEND_RESPONSE | id << 3, n.term, 0, 0);
      emit = 3;
      if (mterm < n.term) break;
      n.role = RAFT_FOLLOWER; n.votes = 0; n.lid = src;
      rearm = true;                         // AppendEntries from the current leader
      if (n.keys & 1u) { n.keys = 0; nm = 2; }
      if (!consistent) break;
      // first conflict in [b, min(len, b + pcnt)); the payload is read from the sender's arena,
      // an entry its pre-tick frontier has overwritten reading (0, 0)
      // (payload position i reads (0, 0) iff the sender's pre-tick frontier passed mpoff + i + A:
      // a prefix i < E of the payload; evictions are counted over the positions compared)
      const uint64_t sf0 = fr[bl + (int)src - 1];
      const uint2* sa = arena_of(S, sgi - k + src - 1);
      const uint32_t hi = n.len < mb + pcnt ? n.len : mb + pcnt;
      const int64_t ev64 = (int64_t)sf0 - (int64_t)mpoff - (int64_t)A;
      const uint32_t E = ev64 <= 0 ? 0u : (ev64 >= (int64_t)pcnt ? pcnt : (uint32_t)ev64);
      uint32_t kk = mb;
      // Payload provenance (tick_wave's PROV): when this node's positions [mb, hi) are unevicted
      // copies of the same sender slots this payload names (key mpoff - mb) and none of the
      // payload is evicted, every term agrees and the search ends at hi.
      if (RS_PROV_SEARCH && E == 0 && pm && (pm & 15) == src && pk == mpoff - mb && ((pm >> 4) & 0x3FFFu) <= mb &&
          hi <= (pm >> 18))
        kk = hi > mb ? hi : mb;
      if (kk < hi) {
        uint32_t yi = (n.base + kk) % A, xi = mpoff % A, rem = hi - kk;
        constexpr int W = 8;
        while (rem) {
          const uint32_t c = min(min(rem, (uint32_t)W), min(A - xi, A - yi));
          const uint2* xp = sa + xi;
          const uint2* yp = sar + yi;
          uint32_t xt[W], yt[W];
#pragma unroll
          for (int j = 0; j < W; ++j) {
            xt[j] = xp[j].x;
            yt[j] = yp[j].x;
          }
          const uint32_t i0 = kk - mb;
          uint32_t mism = 0;
#pragma unroll
          for (int j = 0; j < W; ++j)
            mism |= (uint32_t)((uint32_t)j < c && yt[j] != (i0 + j < E ? 0u : xt[j])) << j;
          if (mism) {
            kk += __builtin_ctz(mism);
            break;
          }
          kk += c;
          rem -= c;
          xi += c;
          yi += c;
          xi = xi == A ? 0 : xi;
          yi = yi == A ? 0 : yi;
        }
      }
      // positions compared: [mb, kk] on a mismatch at kk (< hi), else [mb, hi)
      const uint32_t ncmp = kk < hi ? kk - mb + 1 : hi > mb ? hi - mb : 0u;
      lctr_add(lctr, RAFT_CTR_PAYLOAD_EVICTED, ncmp < E ? ncmp : E);
      const uint32_t mc = mb + pcnt - kk;
      if (mc) {                               // truncate at kk, append payload [kk - b, pcnt)
        pkind = PLAN_PAYLOAD; psrc = src; ppoff = mpoff + (kk - mb); ppcnt = mc;
        pold_base = n.base;
        if (kk < n.len || n.base + n.len != n.front) {
          preloc = 1;
          n.base = n.front;
          n.front += kk;
        }
        n.front += mc;
        n.len = mb + pcnt;
        appended = mc;
      }
      if (ma > n.commit) {
        const uint32_t nc = ma < mb + pcnt ? ma : mb + pcnt;
        if (nc > n.commit) {
          applied = nc - n.commit; papplied = applied;
          n.commit = nc;
        }
      }
      ra = make_uint4(RAFT_MSG_APPEND_RESPONSE | id << 3 | 1u << 7, n.term, ma, mb + pcnt);
      break;
    }
    case RAFT_MSG_CLIENT_SET: {                                   // as client-set-handler 151-160
      if (n.role != RAFT_LEADER) {
        emit = 4;                                                 // redirect-client
        break;
      }
      pkind = PLAN_ENTRY; ppoff = n.term; ppcnt = ma;
      pold_base = n.base;
      if (n.base + n.len != n.front) {
        preloc = 1;
        n.base = n.front;
        n.front += n.len;
      }
      n.front += 1;
      n.len += 1;
      n.seq = 0;
      appended = 1;
      break;
    }
    case RAFT_MSG_VOTE_RESPONSE: {
      if (mterm != n.term || !flag || n.role != RAFT_CANDIDATE) break;
      const uint32_t votes = n.votes | 1u << src;
      if (__popc(votes) < MAJ) {
        n.votes = votes;
        break;
      }
      n.role = RAFT_LEADER; n.votes = 0; n.lid = id;              // voted_for kept
      n.keys = peers | 1u;
      nm = 1;
      emit = 2;
      elected = true;
      break;
    }
    case RAFT_MSG_APPEND_RESPONSE: {
      if (mterm != n.term || n.role != RAFT_LEADER) break;
      if (!flag) {
        nm = 3;
        break;
      }
      nm = 4;
      mchg = true;
      // majority commit: the MAJ-th largest of {log_len} ∪ match_index (own slot holds log_len),
      // by an unrolled compare-exchange network
      int32_t vals[N];
#pragma unroll
      for (int p = 1; p <= N; ++p)
        vals[p - 1] = p == (int)id ? (int32_t)n.len
                                   : (p == (int)src ? (int32_t)mb : lsw.match(p - 1));
#pragma unroll
      for (int i = 1; i < N; ++i)
#pragma unroll
        for (int q = i; q > 0; --q)
          if (vals[q - 1] < vals[q]) {
            const int32_t tmp = vals[q]; vals[q] = vals[q - 1]; vals[q - 1] = tmp;
          }
      int32_t mm = vals[MAJ - 1];
      if (mm > (int32_t)n.len) mm = (int32_t)n.len;
      if (mm > (int32_t)n.commit && sar[(n.base + (uint32_t)mm - 1) % A].x == n.term) {
        applied = (uint32_t)mm - n.commit; papplied = applied;
        n.commit = (uint32_t)mm;
      }
      break;
    }
    default:
      break;
  }
}

// The wave's lanes that hold node index a (lane l is node l mod N of cluster l / N; lanes past the
// wave's whole clusters are idle).
template <int N>
__device__ __forceinline__ uint64_t node_lanes(int a) {
  uint64_t m = 0;
#pragma unroll
  for (int c = 0; c < 64 / N; ++c) m |= 1ull << (c * N);
  return m << a;
}

// LDS words per wave: pair cells [cluster][sender][receiver other than the sender] of CELLW
// words, then sender records [cluster][sender] of SRECW words, counters, and (Spec-Raft) the
// wave's pre-tick arena frontiers.
template <int N>
constexpr int pair_words() { return (64 / N) * N * (N - 1) * CELLW; }
template <int N>
constexpr int cell_words() { return pair_words<N>() + (64 / N) * N * SRECW; }
// NM_LDS: the wave's next_index / match_index rows live in LDS during a launch ([2][N][64]
// words), for the N whose block then still fits four per CU.
template <int N>
constexpr bool nm_lds() { return N <= 5; }
// TRIP words: per cluster slot, the event ticks the cluster ran in this launch (the activity
// packing key); DPEND_WORDS: per lane, 1 while its node's deadline is a deferred re-arm's lower
// bound; PART words: per cluster slot, the partition epoch last drawn and its draw
// (deliver_pack's pstate); CQ words: the client-set batch (below), per lane its injection's value
// and the tick of the injection after it, its target node as a byte, and per cluster slot the
// injection count the batch starts at.
template <int N>
constexpr int trip_words() { return 64 / N; }
constexpr int DPEND_WORDS = 64;
template <int N>
constexpr int part_words() { return 2 * (64 / N); }
template <int N>
constexpr int cq_words() { return 64 + 64 + 16 + 64 / N; }
// (the STORM body has no leader, whose rows NM_LDS would hold: its waves take 2.5 KB less at N = 5,
// five per SIMD instead of four)
template <int N, bool STORM = false>
constexpr bool nm_lds_in() { return nm_lds<N>() && !STORM; }
template <int N, bool SPEC, bool STORM = false>
constexpr int wave_lds_words() {
  return cell_words<N>() + LCTR_WORDS + (SPEC ? 64 : 0) + (nm_lds_in<N, STORM>() ? 2 * N * 64 : 0) +
         trip_words<N>() + DPEND_WORDS + part_words<N>() + cq_words<N>();
}
template <int N, bool SPEC, bool STORM = false>
constexpr size_t block_lds_bytes() {
  return wave_lds_words<N, SPEC, STORM>() * sizeof(uint32_t);
}
// N <= 5 kernels run four waves per SIMD: sixteen one-wave blocks must fit the CU's 160 KB
static_assert(block_lds_bytes<5, true>() * 16 <= 160 * 1024, "N = 5 LDS budget");
static_assert(block_lds_bytes<4, true>() * 16 <= 160 * 1024, "N = 4 LDS budget");

// SPEC selects the Spec-Raft control of SIM_SPEC §8 (variant flag 2) at compile time, so the
// faithful kernel carries none of its code.

// RAFT_SCHED_ALIGNED packing key of a node: its next event (deadline or queue head).
__device__ __forceinline__ uint32_t sched_key_of(uint32_t deadline, const QueueR& rq,
                                                 const QueueR& rs) {
  return min(deadline, min(rq.arr, rs.arr));
}
// LITE: the launch has no client traffic, no faults and a fixed delay (DevSim::lite, set by the
// host; C2): P0, client-set handling and redirects cannot occur, every emission takes the
// fault-free delivery pack, and P3/P4 copy and compare one entry per memory round trip (they only
// see host-written logs there). The compiler then drops that code: 121 -> ~100 VGPRs at N = 5.
//
// STORM: the launch lies before any timer can fire in a handle fresh from init-node (ticks
// [0, el_base): init-node's deadlines and every re-arm are el_base or more ahead), so no node is
// or becomes a candidate or a leader and no network message exists: the only events are
// client-sets at followers, which redirect (SIM_SPEC D15; redirects are outside the fault model).
// The host picks it (raftsim.hip, storm_until); the compiler drops the other handlers, the
// emission and fault draws, P3, P4 and the drain.
//
// tick_wave runs one wave's clusters: `smem` is the wave's LDS (block_lds_bytes), `lane` its lane,
// and the wave takes wave slots wave0, wave0 + wstride, ... below nslots; slot s holds clusters
// perm[s * CPW ...] (null perm: the identity). CATCH: each cluster resumes at resume[slot] (the
// tick the steady kernel stopped it before) instead of t0. The wave's counters go to copy
// ctr_copy (mod CTR_COPIES) of the counter block.
template <int N, bool TRACE, bool SPEC, bool LITE, bool CATCH = false, bool STORM = false>
__device__ __forceinline__ void tick_wave(const DevSim& S, uint32_t t0, uint32_t nt, uint32_t* smem,
                                          int lane, uint32_t wave0, uint32_t wstride,
                                          const uint32_t* perm, uint32_t nslots,
                                          const uint32_t* resume, uint32_t ctr_copy) {
  static_assert(!LITE || (!TRACE && !SPEC), "LITE is the plain faithful kernel");
  static_assert(!CATCH || LITE, "catch-up launches follow the steady kernel (LITE only)");
  static_assert(!STORM || (!LITE && !TRACE && !CATCH), "STORM: client traffic, no trace rings");
  constexpr int CPW = 64 / N;
  constexpr uint32_t ALL = ((1u << (N + 1)) - 1) & ~1u;
  constexpr uint32_t MAJ = SPEC ? N / 2 + 1 : (N + 1) / 2;   // majority? (core.clj:19-21) / strict
  // payload provenance for the checker (below): the kernels with long replicated runs
  constexpr bool PROV = RS_PROV && !LITE && !STORM && (SPEC || N >= RS_PROV_MIN_N);
  // RC: the counters a client burst bumps on every trip (client-set events, redirects, deliveries,
  // appended entries, injections, messages to halted nodes) are kept per lane in registers and
  // added to the wave's LDS counters once at the end: N >= 7 (three waves per SIMD anyway; C4
  // -5 %) and Spec-Raft (C3-spec -3 %); the faithful N <= 5 kernel measured the same either way,
  // and the faithful N = 6 kernel keeps its four waves per SIMD without them
  constexpr bool RC = !LITE && ((N >= RS_RC_MIN_N && N >= 7) || (SPEC && !STORM));
  uint32_t rc_cs = 0, rc_red = 0, rc_del = 0, rc_app = 0, rc_inj = 0, rc_halt = 0;
  uint32_t* const rdel = RC ? &rc_del : nullptr;
  uint32_t* const rhalt = RC ? &rc_halt : nullptr;
  // REGS: the per-cluster trip count (the packing key), the client batch's start and the per-lane
  // deferred-draw bit in registers instead of LDS where registers are to spare (N >= 7, and the
  // Spec-Raft N = 6 kernel): LDS round trips off every trip's chain (C4-N9 -9 %)
  constexpr bool REGS = !LITE && N >= RS_REGS_MIN_N && (N >= 7 || (SPEC && !STORM));
  uint32_t trips_r = 0, dpend_r = 0, cb_r = 0;   // cb_r: the client batch's start (cq_base)
  // (REGS kernels also read the kernel-argument fields a trip's common handlers use once, here,
  // instead of a scalar load and its wait at every use)
  uint32_t ka_el_base = 0, ka_el_span = 0, ka_hb = 0, ka_L = 0, ka_redir = 0;
  bool ka_fixd = false;
  if constexpr (REGS && RS_KA_HOIST) {
    KDevSim* const K0 = kargs();
    ka_el_base = K0->el_base; ka_el_span = K0->el_span; ka_hb = K0->hb; ka_L = K0->L;
    ka_redir = K0->client_redirects; ka_fixd = K0->dmin == K0->dmax;
  }
  constexpr bool KAH = REGS && RS_KA_HOIST;
  // BURST: the faithful N >= 7 kernels run a cluster's client burst under a stable leader in a
  // lane loop of its own (the burst engine in the tick loop below)
  constexpr bool BURST = RS_BURST && KAH && !SPEC && !STORM && !TRACE && !LITE && !CATCH && N >= 7;
  // the wave's cells, counters, leader rows and per-lane / per-cluster words
  uint32_t* cells = smem;
  uint32_t* lctr = cells + cell_words<N>();
  uint32_t* fr = lctr + LCTR_WORDS;           // SPEC: pre-tick arena frontier per lane
  int32_t* nmL = reinterpret_cast<int32_t*>(fr + (SPEC ? 64 : 0));   // NM_LDS rows
  if (lane < LCTR_WORDS) lctr[lane] = lane == LCTR_FIRSTVIOL ? INF : 0u;
  // in LDS: one more loop-carried VGPR cost C3's kernel a wave per SIMD
  uint32_t* tripsL = reinterpret_cast<uint32_t*>(nmL) + (nm_lds_in<N, STORM>() ? 2 * N * 64 : 0);
  uint32_t* const dpend = tripsL + trip_words<N>();      // (likewise)
  dpend[lane] = 0;
  uint32_t* const pcache = dpend + DPEND_WORDS;    // [CPW] epochs, then [CPW] draws
  uint32_t* const cq_val = pcache + part_words<N>();
  uint32_t* const cq_nxt = cq_val + 64;
  uint8_t* const cq_tgt = reinterpret_cast<uint8_t*>(cq_nxt + 64);
  uint32_t* const cq_base = cq_nxt + 64 + 16;
  __builtin_amdgcn_wave_barrier();

  // RAFT_SCHED_ALIGNED launches a grid sized for the padded packing; waves past its slots exit.
  uint32_t wave = wave0;
  if (wave * CPW >= nslots) return;
  do {
    if (lane < CPW) {
      tripsL[lane] = 0;
      pcache[lane] = INF;                             // no partition epoch drawn yet
    }
    const int cs = lane / N, k0 = lane - cs * N;
    const uint32_t slot = wave * CPW + cs;      // wave slot; the cluster is perm[slot]
    const uint32_t c0 = lane < CPW * N && slot < nslots ? (perm ? perm[slot] : slot) : INF;
    const bool active = c0 != INF;
    const uint32_t c = active ? c0 : 0u;
    const uint32_t gi = c * N + k0;
    const uint32_t g = S.goff + c;
    const int bl0 = (cs < CPW ? cs : 0) * N;     // the cluster's first lane
    const uint32_t A = S.A;
    constexpr uint32_t HB = hot_block_words(N), CLW = hot_cl_off(N);
    // this node's words in its cluster's block (field f at hp[f * N]) and the cluster's words
    uint32_t* const hp = S.hot + (size_t)c * HB + HOT_CW + k0;
    uint32_t* const hc = S.hot + (size_t)c * HB + CLW;

    NodeR n = {};
    uint32_t hidx = 0, hterm = 0, hval = 0;   // checker high-water mark (cluster-replicated)
    // Payload provenance (PROV; launch-local, not state). Arena slots are written only at a
    // node's frontier, so an entry copied from sender S's arena at absolute position key + p
    // (key = source offset - appended_at) without eviction equals every other unevicted copy of
    // that slot. pk = key and pm = S | from << 4 | to << 18 of the lane's last payload append
    // (pm = 0: none, or an eviction): its log positions [from, to) hold S's slots key + p. Later
    // entry appends land at to or past it, remove-from! clamps to, a payload append replaces both.
    // The checker then skips a pair whose positions are such copies on both sides (P4).
    uint32_t pk = 0, pm = 0;
    uint32_t cnext = INF, ccount = 0;         // client-set injection cursor (cluster-replicated)
    if (active) {
      const uint32_t fl = hp[HF_FLAGS * N], mk = hp[HF_MASKS * N], qm = hp[HF_QMETA * N];
      n.role = fl & 3; n.vf = (fl >> 2) & 15; n.lid = (fl >> 6) & 15; n.fault = (fl >> 10) & 7;
      n.seq = (fl >> 13) & 1;
      n.votes = mk & 0xFFFF; n.keys = mk >> 16 | ((fl >> 14) & 1);
      n.term = hp[HF_TERM * N]; n.commit = hp[HF_COMMIT * N]; n.len = hp[HF_LEN * N];
      n.deadline = hp[HF_DEADLINE * N];
      if (!SPEC) {                                        // a deferred draw carried over
        if constexpr (REGS) dpend_r = (fl & FL_DRAW) ? 1u : 0u;
        else dpend[lane] = (fl & FL_DRAW) ? 1u : 0u;
      }
      n.rq.h = qm & 15; n.rq.c = (qm >> 4) & 31; n.rs.h = (qm >> 9) & 15; n.rs.c = (qm >> 13) & 31;
      n.rq.arr = hp[HF_REQ_ARR * N]; n.rs.arr = hp[HF_RES_ARR * N];
      n.rq.tail = hp[HF_REQ_TAIL * N]; n.rs.tail = hp[HF_RES_TAIL * N];
      n.base = hp[hf_abase(N) * N]; n.front = hp[hf_afront(N) * N]; n.led = hp[hf_led(N) * N];
      n.trace = (uint64_t)hp[HF_TRACE_HI * N] << 32 | hp[HF_TRACE_LO * N];
      hidx = hc[0]; hterm = hc[1]; hval = hc[2]; cnext = hc[3]; ccount = hc[4];
      if constexpr (nm_lds_in<N, STORM>()) {   // each lane only touches its own LDS column
  #pragma unroll
        for (int p = 0; p < N; ++p) {
          nmL[p * 64 + lane] = hp[(HF_NEXT + p) * N];
          nmL[(N + p) * 64 + lane] = hp[(HF_NEXT + N + p) * N];
        }
      }
    }

    // Per-cluster reductions over the cluster's N lanes (every lane of the wave must be active).
    const uint32_t cmask = (1u << N) - 1;
    auto cluster_min = [&](uint32_t x) {
      uint32_t m = x;
  #pragma unroll
      for (int s = 0; s < N; ++s) m = min(m, (uint32_t)__shfl(x, bl0 + s));
      return m;
    };
    auto cluster_any = [&](bool x) { return ((uint32_t)(__ballot(x) >> bl0) & cmask) != 0; };
    const uint32_t tend = t0 + nt;
    // Dead waves. A cluster whose every node is halted changes nothing but its client cursor and
    // two counters from here on: a halt is permanent (D8) and a halted node drops what reaches it
    // (core.clj:202-203), so its only events are client-sets into halted nodes (SIM_SPEC P0 + P2,
    // to_halted). A wave holding only such clusters (the activity packing gives them waves of their
    // own) runs their injections up to the launch's end here, one Philox draw each, with no trip;
    // its trip loop then finds no event before tend. A wave that mixes live clusters in takes the
    // trips (draining a dead cluster's injections there would stall its live wave mates).
    // Injections into a dead cluster are independent draws (keyed by the injection count), so the
    // wave runs them 64 at a time, one cluster after another: lane l draws the gap after the
    // cluster's (count + l)-th injection, an inclusive scan of (1 + gap) over the lanes gives the
    // next 64 injections' on-tick numbers, and the first one at or past tend ends the cluster's
    // run (SIM_SPEC P0; the Spec-Raft control's client-sets reach halted nodes the same way).
    if constexpr (!LITE && !STORM) {
      const bool dead = ((uint32_t)(__ballot(active && n.fault) >> bl0) & cmask) == cmask;
      if (kargs()->client_ppm && !__ballot(active && !dead) && __ballot(active && cnext < tend)) {
        const uint64_t heads = __ballot(active && k0 == 0);
  #pragma unroll 1
        for (int cs2 = 0; cs2 < CPW; ++cs2) {
          const int b2 = cs2 * N;
          if (!((heads >> b2) & 1)) continue;                               // wave-uniform
          const uint32_t g2 = (uint32_t)__builtin_amdgcn_readlane((int)g, b2);
          uint32_t cc = (uint32_t)__builtin_amdgcn_readlane((int)ccount, b2);
          uint32_t cn = (uint32_t)__builtin_amdgcn_readlane((int)cnext, b2);
          uint32_t cnt = 0;
          while (cn < tend) {                                               // wave-uniform
            const uint4 d = philox(g2, P_CLIENT << 8, cc + (uint32_t)lane, 0, S.key0, S.key1);
            uint64_t x = 1 + client_gap(d.w, PowersS(S.client_pw), S.client_top);
  #pragma unroll
            for (int o = 1; o < 64; o <<= 1) {                              // inclusive scan
              const uint64_t y = (uint64_t)(uint32_t)__shfl_up((int)(uint32_t)x, o) |
                                 (uint64_t)(uint32_t)__shfl_up((int)(uint32_t)(x >> 32), o) << 32;
              if (lane >= o) x += y;
            }
            // the injection after lane's own: its tick (lane's own fired: it is at or before
            // the lane below's successor)
            const uint32_t nxt = on_tick(on_index(cn, S) + x, S.client_period, S.div_burst);
            const uint64_t stop = __ballot(nxt >= tend);
            const int l = stop ? __builtin_ctzll(stop) : 63;                // last one fired
            cnt += (uint32_t)l + 1;
            cc += (uint32_t)l + 1;
            cn = (uint32_t)__builtin_amdgcn_readlane((int)nxt, l);
            if (stop) break;
          }
          if (lane >= b2 && lane < b2 + N) {
            ccount = cc;
            cnext = cn;
          }
          if (lane == b2) {
            lctr_add(lctr, RAFT_CTR_CLIENT_INJECTED, cnt);
            lctr_add(lctr, RAFT_CTR_TO_HALTED, cnt);
          }
        }
      }
    }

    // Earliest tick at which any node of the lane's cluster can have an event (deadline, queue head
    // or the next client-set), the same for all the cluster's lanes.
    auto next_event = [&]() {
      const uint32_t m = n.fault ? INF : min(n.deadline, min(n.rq.arr, n.rs.arr));
      return cluster_min(active ? (LITE ? m : min(m, cnext)) : INF);
    };
  #ifdef RS_WAVELOG   // diagnostic build: per-wave start/end (100 MHz clock), active ticks, placement
    const uint64_t wl_start = wall_clock64();
    uint32_t wl_active = 0, wl_first = INF, wl_drain = 0, wl_inj = 0, wl_dead = 0;
    {
      const uint64_t fm = __ballot(active && n.fault);
      const uint32_t all = (1u << N) - 1;
      wl_dead = __popcll(__ballot(active && k0 == 0 && ((uint32_t)(fm >> bl0) & all) == all));
    }
    uint32_t wl_kmin = INF, wl_kmax = 0;
    {
      const uint32_t key = (active && k0 == 0 && S.skey) ? S.skey[c] : INF;
      wl_kmin = wave_min(key);
      wl_kmax = ~wave_min(key == INF ? ~0u : ~key);
    }
    // per-phase shader cycles summed over the wave's trips, stamped where the wave enters a block
    // (a skipped stamp merges its interval into the next): 11 P0's draws, 0 P0's queue insert, 1
    // P1's queue pop, 2 the handler, 10 timer/hash/counters, 3 redirects, emission and fault
    // draws, 4 P2, 5 P3, 6 P4, 7 the append-response drain, 8 the trip's loop head (next event,
    // exit ballot); 9 the launch-start state load
    uint32_t wl_ph[17] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    // wave-level passes of each Philox call site (the first active lane counts the pass; summed
    // over the lanes at the end): 0 client, 1 deferred timer, 2 alts!!, 3 Spec re-arm, 4 redirect, 5 partition,
    // 6 fault draws of replies, 7 fault draws of broadcasts (per peer)
    uint32_t wl_px0 = 0, wl_px1 = 0, wl_px2 = 0, wl_px3 = 0, wl_px4 = 0, wl_px5 = 0, wl_px6 = 0,
             wl_px7 = 0;
  #define RS_PX(v) (v) += (uint32_t)(lane == (int)__builtin_ctzll(__ballot(1)))
    uint64_t wl_ts = 0;
    const uint64_t wl_mt0 = __builtin_amdgcn_s_memtime();
  #define RS_PHASE(i)                                          \
    do {                                                       \
      const uint64_t now_ = __builtin_amdgcn_s_memtime();      \
      wl_ph[i] += (uint32_t)(now_ - wl_ts);                    \
      wl_ts = now_;                                            \
    } while (0)
  #else
  #define RS_PHASE(i) do {} while (0)
  #define RS_PX(v) do {} while (0)
  #endif


    // Every cluster keeps its own clock. Ticks before a cluster's next event change nothing for it
    // (every handler, injection and delivery is keyed to a deadline, a queue head or the injection
    // cursor), and clusters never interact, so each trip of the loop runs every cluster's next
    // event tick -- not the wave's: a wave makes as many trips as its busiest cluster has event
    // ticks, instead of the union of its clusters' event ticks (discrete-event skipping per
    // cluster, tick-exact; Philox draws are keyed by the cluster's own tick).
    // the cluster's first tick not yet simulated (catch-up: the tick it was bailed before)
    uint32_t tnext = CATCH && active ? resume[slot] : t0;
  #ifdef RS_WAVELOG
    wl_ts = __builtin_amdgcn_s_memtime();
    wl_ph[9] = (uint32_t)(wl_ts - wl_mt0);
  #endif
    // Client-set batches. A cluster's injections are keyed by its injection count (SIM_SPEC P0),
    // so its next N are drawn together, one per lane of the cluster: lane k draws injection
    // count + k (target node, value, gap), an inclusive scan of (1 + gap) over the cluster's lanes
    // gives the on-tick number of the injection after each, and the batch sits in LDS until the
    // cluster has used it up. A refill is one wave-wide Philox pass that refills every cluster of
    // the wave from its current count (the draws do not depend on when they are made): a wave
    // makes about one pass per N injections of its busiest cluster instead of one per injecting
    // trip, and the gap search and tick arithmetic go with it. P0 calls it when a cluster that
    // injects at this trip has used its batch up; it refills the clusters whose next injection
    // is inside the launch. (C3 first launch 68.4 -> 60.2 ms, C4-N9 17.1 -> 15.1 ms.)
    auto refill_batch = [&](uint32_t t) {
      if constexpr (!LITE) {
        const uint32_t cw = (uint32_t)bl0 / N;
        const bool want = active && cnext < tend;
        if (__ballot(want && t == cnext && ccount - (REGS ? cb_r : cq_base[cw]) >= (uint32_t)N)) {
          RS_PX(wl_px0);
          const uint4 d = philox(g, P_CLIENT << 8, ccount + (uint32_t)k0, 0, S.key0, S.key1);
          // (the fields by scalar loads here: kargs)
          KDevSim* const K = kargs();
          // (1 + gap) summed in 32 bits, saturating: a sum of 2^32 - 1 or more is past any tick
          // (on_tick's never) either way
          const uint64_t g1 = 1 + client_gap(d.w, PowersS(K->client_pw), K->client_top);
          uint32_t x = g1 >> 32 ? 0xFFFFFFFFu : (uint32_t)g1;
  #pragma unroll
          for (int o = 1; o < N; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, o);
            if (k0 >= o) x = x + y < x ? 0xFFFFFFFFu : x + y;
          }
          if (want) {
            cq_val[lane] = d.z;
            const uint32_t P = K->client_period;
            const DivU32 dp = kdiv(K->div_period), db = kdiv(K->div_burst);
            const uint32_t q = P ? udiv(dp, cnext) : 0u;
            const uint64_t oi = P ? (uint64_t)q * db.d + (cnext - q * P) : cnext;   // on_index
            cq_nxt[lane] = on_tick(oi + x, P, db);
            cq_tgt[lane] = (uint8_t)(1 + __umulhi(d.y, N));
            if constexpr (REGS) cb_r = ccount;          // (every lane of the cluster)
            else if (k0 == 0) cq_base[cw] = ccount;
          }
        }
      }
    };
    if constexpr (!LITE) {
      if constexpr (REGS) cb_r = ccount - N;              // empty
      else if (active && k0 == 0) cq_base[cs] = ccount - N;
    }
    // A non-leader's re-armed timer (D4: t + el_base + the EVENT draw's word 1) is only compared
    // with ticks at or past t + el_base, so its draw is deferred (dpend) unless the event drew
    // anyway (the alts!! bit, a rand-nth redirect): the deadline holds that lower bound, which
    // also serves as the cluster's next event; when a tick at or past it comes with no message
    // ready (a message wins, D3, and in the faithful model its event re-arms the timer anyway) the
    // draw is made in P1 and the timeout decided on the exact deadline, else at the write-back.
    // the burst engine's launch-wide gate: client traffic, and ticks that fit its 28-bit arrivals
    constexpr uint32_t BAM = (1u << 28) - 1;
    const bool bclient = BURST && kargs()->client_ppm != 0 && tend <= BAM;
    // (wave-uniform) trips left before the entry check runs again: a check that finds no cluster
    // to enter costs about a tenth of a trip, and states change slowly against trips
    uint32_t bskip = 0;
    for (;;) {
      uint32_t t = max(tnext, next_event());
      t = t < tend ? t : tend;
      // ------------------------------------------------------------------ burst engine (BURST)
      // A client burst under a stable leader is a chain of events that each touch one node: a
      // client-set injected at a follower is redirected to the :leader-id (server.clj:62-63)
      // and reaches the leader at t + 1 (D15); the leader takes one client-set per tick and
      // appends it (core.clj:157-160), re-arming its timer every time, so no heartbeat fires and
      // no network message exists. A cluster whose state at its next event tick is such a state
      // -- one live leader L with empty RES and REQ queues, its log at its arena frontier and no
      // owed draw; every other live node a non-leader with :leader-id L, empty queues and a
      // deadline ahead; halted nodes anywhere -- runs its ticks here, its N lanes in step, one
      // loop trip per event tick, instead of a trip of the tick loop with its five phases. Every
      // lane tracks the leader's ring (at most two client-sets: one arrives per tick, one leaves),
      // its log length and deadline, so the target of each injection decides each lane's work
      // without a shuffle. The loop stops before the first tick with anything else -- a
      // follower's deadline (its deferred draw, a timeout), the leader's heartbeat, the leader's
      // OVERFLOW, a full one-slot inbox, the launch's end -- and the tick loop resumes the cluster
      // there (all ticks before it are done: `tnext`). Per tick and node it does what the phases
      // do: P0's injection (batch, counters, to-halted), P1's handlers (trace hash, re-arm, the
      // deferred draw of a follower, redirect or abandon), P2's delivery to the leader, P3's entry
      // append and P4's log matching of the new entry against every other node's log.
      if constexpr (BURST) {
        if (bskip) {
          --bskip;
        } else if (bclient && (!RS_BURST_PRE ||
                        __ballot(active && t < tend &&
                                 (t == cnext || (n.role == RAFT_LEADER && n.rq.c == 1))))) {
          const bool live0 = active && !n.fault;
          const uint32_t lmask = (uint32_t)(__ballot(live0) >> bl0) & cmask;
          const uint32_t ldm = (uint32_t)(__ballot(live0 && n.role == RAFT_LEADER) >> bl0) & cmask;
          const int Lk = ldm ? (int)__builtin_ctz(ldm) : 0;
          const bool isL = k0 == Lk;
          const bool lok = !live0 ||
                           (isL ? (n.rq.c <= 1 && n.rs.c == 0 && n.base + n.len == n.front && !dpend_r)
                                : (n.lid == (uint32_t)Lk + 1 && n.rq.c == 0 && n.rs.c == 0 &&
                                   n.deadline > t));
          bool bok = active && t < tend && __popc(ldm) == 1 && !cluster_any(!lok);
          const bool Lq = cluster_any(isL && n.rq.c != 0);    // (one queued message at most)
          bok = bok && (t == cnext || Lq);
          // Clusters that stay with the tick loop bound the run: an engine cluster runs no tick
          // past the latest next-event tick among them (after its first), so a burst's engine ticks
          // spread over the trips the other clusters take anyway instead of following them; the
          // run then yields (the tick loop takes its next tick, and the next trip re-enters). A
          // cluster that could run fewer than BURST_MIN ticks that way stays with this trip (an
          // entry costs about a trip).
          const bool oth = active && !bok && t < tend;
          const uint32_t tlim = __ballot(oth) ? ~wave_min(oth ? ~t : ~0u) : INF;
          constexpr uint32_t BURST_MIN = RS_BURST_MIN;
          bok = bok && (tlim == INF || tlim >= t + BURST_MIN);
          if (!__ballot(bok)) bskip = RS_BURST_SKIP;
          if (__ballot(bok)) {
            // the leader's queued message enters with the cluster if it is a client-set due by t
            uint4 lm0 = make_uint4(0, 0, 0, 0), lm1 = make_uint4(0, 0, 0, 0);
            if (bok && Lq) {
              const uint32_t* qb = qslots(S, c * N + (uint32_t)Lk, 0) +
                                   (uint32_t)__shfl((int)n.rq.h, bl0 + Lk) * qstride(S, 0);
              lm0 = *reinterpret_cast<const uint4*>(qb);
              lm1 = *reinterpret_cast<const uint4*>(qb + 4);
              bok = lm0.y == RAFT_MSG_CLIENT_SET && lm0.z == 0 && lm0.x <= t && lm1.x < 16 &&
                    !lm1.y && !lm1.z && !lm1.w;
            }
            if (bok) {                                   // whole clusters: cluster-uniform below
              const uint32_t Lid = (uint32_t)Lk + 1;
              const uint32_t Llen0 = (uint32_t)__shfl((int)n.len, bl0 + Lk);
              const uint32_t Lterm = (uint32_t)__shfl((int)n.term, bl0 + Lk);
              uint32_t Llen = Llen0, Ldl = (uint32_t)__shfl((int)n.deadline, bl0 + Lk);
              // the live followers' earliest deadline, kept as a lower bound (an event re-arms its
              // follower to tc + el_base) and recomputed when a tick reaches it; the longest other
              // log (the checker compares only positions it reaches)
              const bool fol = live0 && !isL;
              uint32_t fmin = cluster_min(fol ? n.deadline : INF);
              const uint32_t omax = ~cluster_min(isL ? ~0u : ~n.len);
              // the leader's REQ ring: at most one client-set (arrival | hops << 28, value) between
              // ticks -- a tick adds at most one and the leader takes one whenever it holds any
              uint32_t rc = Lq ? 1u : 0u, qa0 = lm0.x | lm1.x << 28, qv0 = lm0.w, binj = 0, eticks = 0;
              uint2* const own = arena_of(S, gi);
              // the lane's arena slot of log position Llen, and its entry there (the checker's next
              // comparison, loaded a tick ahead of its use)
              uint32_t as = (n.base + Llen0) % A;
              uint2 pre = make_uint2(0, 0);
              if (!RS_BURST_KO_CMP && !isL && n.len > Llen0) pre = own[as];
              uint32_t tc = t;
              for (;;) {
                if (tc >= tend || (tc > tlim && tc != t)) break;
                if (tc >= fmin) {                        // a follower's deadline may be due
                  fmin = cluster_min(fol ? n.deadline : INF);
                  if (tc >= fmin) break;
                }
                const bool injn = tc == cnext;
                uint32_t tgt = 0, val = 0, nxt = 0;
                if (injn) {
                  refill_batch(tc);
                  const uint32_t s = (uint32_t)bl0 + (ccount - cb_r);
                  tgt = cq_tgt[s];
                  val = cq_val[s];
                  nxt = cq_nxt[s];
                }
                const bool toL = injn && tgt == Lid;
                const bool evL = rc || toL;
                if ((!evL && Ldl <= tc) || (evL && Llen >= ka_L) || rc >= S.Q) break;
                ++eticks;
                if (RS_BURST_DIAG && k0 == 0) lctr_add(lctr, RAFT_CTR_DROPPED, 1);
                // a live follower's event: redirect-client (server.clj:62-63), or abandon
                const bool tof = injn && !toL && ((lmask >> (tgt - 1)) & 1);
                const bool red = tof && ka_redir != 0;
                const uint32_t pv = rc ? qv0 : val;      // the client-set the leader takes
                // the ring after the tick: the injection behind a queued one, or a redirect
                // arriving at tc + 1 (P2), else empty
                const bool keep = rc && toL;
                qa0 = keep ? tc : (tc + 1) | 1u << 28;
                qv0 = val;
                rc = keep || red ? 1u : 0u;
                if (injn) {
                  ccount += 1;
                  cnext = nxt;
                  binj += k0 == 0 ? 1u : 0u;
                }
                // one handler per lane: the leader's append (client-set-handler 157-160) or the
                // target follower's redirect; every event re-arms the timer (a follower's draw is
                // deferred: no EVENT draw at a known :leader-id)
                const bool me = isL ? evL : tof && k0 + 1 == (int)tgt;
                if (me) {
                  n.trace = trace_event(n.trace, tc, RAFT_MSG_CLIENT_SET, 0, 0, n.role, n.term, 0);
                  ++rc_cs;
                  rc_app += isL ? 1u : 0u;
                  if (!isL) {
                    n.deadline = tc + ka_el_base;
                    dpend_r = 1;
                  }
                }
                if (tof) fmin = min(fmin, tc + ka_el_base);   // (every lane of the cluster)
                // deliveries (the injection taken or queued, the redirect into the leader's ring),
                // redirects, abandoned client-sets, injections into halted nodes
                rc_del += isL ? (toL ? 1u : 0u) + (red ? 1u : 0u) : (me ? 1u : 0u);
                if (!isL && me) {
                  if (red) ++rc_red;
                  else lctr_add(lctr, RAFT_CTR_CLIENT_ABANDONED, 1);
                }
                rc_halt += injn && !toL && !tof && k0 + 1 == (int)tgt ? 1u : 0u;
                if (evL) {
                  // P3 / P4: the entry (Lterm, pv) at position p, and log matching against every
                  // other node's log that reaches p
                  const uint32_t p = Llen;
                  Llen = p + 1;
                  Ldl = tc + ka_hb;
                  if (isL) own[as] = make_uint2(Lterm, pv);
                  const bool conf = !isL && n.len > p && pre.x == Lterm && pre.y != pv;
                  as = as + 1 == A ? 0u : as + 1;
                  if (!RS_BURST_KO_CMP && !isL && n.len > p + 1) pre = own[as];
                  if (p < omax && cluster_any(conf) && isL) violation(lctr, RAFT_CTR_VIOL_LOG, tc);
                }
                tc = max(tc + 1, min(min(cnext, rc ? tc + 1 : INF), min(min(Ldl, fmin), tend)));
              }
              if (isL) {                                 // the leader's words, its ring as the tick loop keeps it
                if (Llen != Llen0) {
                  n.front += Llen - Llen0; n.len = Llen; n.seq = 0; n.deadline = Ldl;
                }
                if (rc) {
                  uint32_t* const qb = qslots(S, gi, 0);
                  *reinterpret_cast<uint4*>(qb) = make_uint4(qa0 & BAM, RAFT_MSG_CLIENT_SET, 0, qv0);
                  *reinterpret_cast<uint4*>(qb + 4) = make_uint4(qa0 >> 28, 0, 0, 0);
                }
                n.rq.h = 0; n.rq.c = rc; n.rq.arr = rc ? qa0 & BAM : INF; n.rq.tail = rc ? qa0 & BAM : 0u;
              }
              if (k0 == 0) lctr_add(lctr, RAFT_CTR_CLIENT_INJECTED, binj);
              // the packing key counts an engine tick as an eighth of a trip: clusters the tick loop
              // keeps busy through a burst are then packed together, ahead of the engine's
              trips_r += eticks >> 3;
              if (RS_BURST_DIAG && k0 == 0) {
                lctr_add(lctr, RAFT_CTR_DUPLICATED, 1);
                lctr_add(lctr, RAFT_CTR_PARTITIONED, tc > tlim && tc < tend ? 1u : 0u);
              }
              tnext = tc;
            }
            t = max(tnext, next_event());
            t = t < tend ? t : tend;
          }
        }
      }
      const bool on = active && t < tend;     // the cluster has a tick to run in this trip
      if (!__ballot(on)) break;
      if (BURST && RS_BURST_DIAG && on && k0 == 0) lctr_add(lctr, RAFT_CTR_PAYLOAD_EVICTED, 1);
      if constexpr (REGS) trips_r += on;        // (cluster-uniform; used with client traffic)
      else if (!LITE && k0 == 0 && kargs()->client_ppm) tripsL[(uint32_t)bl0 / N] += on;
  #ifdef RS_WAVELOG
      RS_PHASE(8);
  #endif
      const bool live = on && !n.fault;
      // Opaque per-tick copies of the lane's indices: they keep the compiler from hoisting every
      // address and shuffle index the active-tick phases use out of the tick loop, where each would
      // hold a VGPR across all ticks (~50 VGPRs in all); recomputing them costs a few VALU per
      // active tick.
      uint32_t sgi = gi, sg = g;
      int k = k0, bl = bl0;
      asm volatile("" : "+v"(sgi), "+v"(sg), "+v"(k), "+v"(bl));
      const uint32_t id = k + 1, peers = ALL & ~(1u << id);
      uint32_t* const mycells = cells + bl * (N - 1) * CELLW;
      uint32_t* const mysrec = cells + pair_words<N>() + bl * SRECW;
      uint2* const sar = arena_of(S, sgi);
      int32_t* const hnm = reinterpret_cast<int32_t*>(S.hot + (size_t)(sg - S.goff) * HB + HOT_CW + k);
      const PeerW lsw = nm_lds_in<N, STORM>() ? PeerW{nmL + lane, nmL + N * 64 + lane, 64u}
                                   : PeerW{hnm + HF_NEXT * N, hnm + (HF_NEXT + N) * N, (uint32_t)N};
      if constexpr (SPEC) {          // payloads are judged against the senders' pre-tick frontiers
        fr[lane] = n.front;
        __builtin_amdgcn_wave_barrier();
      }

      // ---------------------------------------------------------- P0 client injection (D9, D14)
      bool inj = false;
      uint32_t injv = 0;
      const bool cinj = !LITE && on && t == cnext;
  #ifdef RS_WAVELOG
      wl_inj += __ballot(cinj) ? 1 : 0;
  #endif
      // P0 takes the injection from the cluster's client-set batch (refill_batch above)
      if constexpr (!LITE) {
        if (__ballot(cinj)) {
          refill_batch(t);
          const uint32_t cw = (uint32_t)bl / N;          // the cluster's wave slot
          const uint64_t heads = __ballot(cinj && k == 0);
          if constexpr (RC) rc_inj += (uint32_t)__popcll(heads);        // (wave-uniform)
          else if (lane == 0) lctr_add(lctr, RAFT_CTR_CLIENT_INJECTED, (uint32_t)__popcll(heads));
          if (cinj) {
            const uint32_t s = (uint32_t)bl + (ccount - (REGS ? cb_r : cq_base[cw]));
            if (cq_tgt[s] == id) {
              inj = true;
              injv = cq_val[s];
            }
            ccount += 1;
            cnext = cq_nxt[s];
          }
        }
      }
      RS_PHASE(11);

      // A client-set that lands in an empty REQ queue would be its head at arrival t, so it is
      // kept in registers (dcs) instead of a global store + same-tick load; it is written to the
      // queue only if this tick's alts!! choice takes the RES queue instead.
      bool dcs = false;
      if (!LITE && __ballot(inj)) {
        if (inj) {
          if (live && n.rq.c == 0) dcs = true;
          else qinsert(S, sgi, n.fault, 0, n.rq, make_uint4(t, RAFT_MSG_CLIENT_SET, 0, injv),
                       make_uint4(0, 0, 0, 0), lctr, rdel, rhalt);
        }
      }

      RS_PHASE(0);
      // ---------------------------------------------------------------- P1 one event per node
      const bool req_ok = live && (dcs || n.rq.arr <= t);
      const bool res_ok = live && n.rs.arr <= t;
      uint32_t sentmask = 0;
      // P3 plan: PAYLOAD copies ppcnt entries from psrc's arena slot ppoff, ENTRY appends the
      // entry (ppoff, ppcnt) = (term, val); the old log starts at pold_base and (preloc) is first
      // moved to the node's new base. The old length (n.len - entries added) and the first applied
      // position (n.commit - papplied) are derived in P3 rather than held across P2.
      uint32_t pkind = PLAN_NONE, psrc = 1, ppoff = 0, ppcnt = 0, pold_base = 0, preloc = 0,
               papplied = 0;
      bool elected = false, mchg = false;
      uint32_t pmax = 0;                                        // largest AE payload emitted
      uint32_t tr_cnt = 0, tr_src = 1, tr_poff = 0, tr_at = 0;   // F3 :entries capture (TRACE)
      // The EVENT draws of this tick, in one Philox pass for the wave (the draws are keyed by
      // cluster, node and tick, so only the pass count depends on where they are made):
      //  - the alts!! choice (core.clj:181) when both queues are ready;
      //  - a non-leader without a leader id that takes a REQ message: a client-set there is
      //    redirected by rand-nth (core.clj:153-155; the redirect storm of a leaderless burst);
      //  - a deferred timer due at this tick with no message ready: its own tick's draw
      //    (deadline - el_base) decides whether the node times out now.
      // The next timeout of a non-leader (core.clj:174) takes the tick's draw when there is one,
      // else its draw is deferred (leaders' events need none).
      uint4 w = make_uint4(0, 0, 0, 0);
      const bool tdraw = !SPEC && !STORM && live && (REGS ? dpend_r : dpend[lane]) && !req_ok && !res_ok &&
                         n.deadline <= t;
      bool have_w = (req_ok && res_ok) ||
                    (!LITE && req_ok && n.role != RAFT_LEADER && n.lid == 0);
      if (have_w || tdraw) {
        RS_PX(wl_px2);
        w = event_draw(sg, id, tdraw ? n.deadline - (KAH ? ka_el_base : kargs()->el_base) : t, S);
      }
      if (tdraw) {
        n.deadline += __umulhi(w.y, KAH ? ka_el_span : kargs()->el_span);
        if constexpr (REGS) dpend_r = 0;
        else dpend[lane] = 0;
      }
      if (live && (req_ok || res_ok || t >= n.deadline)) {
        int which = -1;
        if (req_ok && res_ok) {
          which = (w.x & 1) ? 1 : 0;
        } else if (req_ok) {
          which = 0;
        } else if (res_ok) {
          which = 1;
        }
        uint4 m0 = make_uint4(0, 0, 0, 0), m1 = make_uint4(0, 0, 0, 0);
        if (dcs) {
          if (which == 0) {
            m0 = make_uint4(t, RAFT_MSG_CLIENT_SET, 0, injv);
            if constexpr (RC) ++rc_del;
            else lctr_add(lctr, RAFT_CTR_DELIVERED, 1);
          } else {
            qinsert(S, sgi, 0, 0, n.rq, make_uint4(t, RAFT_MSG_CLIENT_SET, 0, injv),
                    make_uint4(0, 0, 0, 0), lctr, rdel, rhalt);
          }
        }
        if (which >= 0 && !(dcs && which == 0)) {
          // Take the queue head (qpop): both loads are issued first, and a non-leader's EVENT draw
          // (needed for its next timeout whatever the message does, unless it becomes leader) is
          // computed in their shadow. The next head's arrival is loaded unconditionally (a slot of
          // the ring is always in bounds) and used only when the queue stays non-empty.
          const QueueR q = which ? n.rs : n.rq;
          const uint32_t* qb = qslots(S, sgi, which);
          const size_t qs = qstride(S, which);
          const uint4* sp = reinterpret_cast<const uint4*>(qb + q.h * qs);
          m0 = sp[0];
          m1 = sp[1];
          const uint32_t nh = wrapq(q.h + 1, S.Q);
          // Only a queue that stays non-empty has a next head. Its arrival is known without a load
          // when one message remains or all queued ones share the head's arrival (the queue is
          // sorted, so head == tail means all equal): then nothing this tick waits on memory.
          uint32_t narr = INF;
          if (q.c > 1) narr = (q.c == 2 || q.arr == q.tail) ? q.tail : qb[nh * qs];
          QueueR r = q;
          r.h = nh;
          r.c -= 1;
          r.arr = r.c ? narr : INF;
          r.tail = r.c ? r.tail : 0u;
          // A queue that drains restarts its ring at slot 0 (the ring position is not state: reads
          // linearise from the head). Steady-state traffic then lands in slots 0..P-1, where a
          // cluster's nodes are adjacent, instead of walking all Q slots of the [slot][node] layout.
          if (!r.c) r.h = 0;
          if (which) n.rs = r;
          else n.rq = r;
        }
        const uint32_t hdr = m0.y, mterm = m0.z, ma = m0.w, mb = m1.x, met = m1.y, mev = m1.z,
                       mpoff = m1.w;
  #ifdef RS_WAVELOG
        asm volatile("" ::"v"(hdr), "v"(mb));   // the pop's wait lands before the stamp
        RS_PHASE(1);
  #endif
        const uint32_t type = hdr & 7, src = (hdr >> 3) & 15, flag = (hdr >> 7) & 1,
                       mep = (hdr >> 8) & 1, pcnt = hdr >> 16;
        if constexpr (TRACE) {
          const uint32_t tes = S.tecount[sgi];
          trace_record<N>(S, sgi, t, n, lsw, m0, m1, tes);
          if (which >= 0 && type == RAFT_MSG_APPEND_ENTRIES && pcnt) {
            tr_cnt = pcnt; tr_src = src; tr_poff = mpoff; tr_at = tes;
            S.tecount[sgi] = tes + pcnt;
          }
        }

        // Every throw site of the reference precedes every mutation of its handler (SIM_SPEC D8),
        // so each case decides `fault` first and only then updates the node in place.
        uint32_t fault = 0, ev = 0;
        // 1 request-vote bcast, 2 append-entries bcast, 3 one reply, 4 redirect-client
        int emit = 0;
        int nm = 0;                   // next/match: 1 init, 2 clear, 3 dec next[src], 4 set src
        uint4 ra = make_uint4(0, 0, 0, 0), rb = make_uint4(0, 0, 0, 0);  // reply cell words
        uint32_t appended = 0, applied = 0;
        const bool was_leader = n.role == RAFT_LEADER;
        bool rearm = false;           // SPEC: the event resets the election timer (SIM_SPEC §8)

        if constexpr (STORM) {
          ev = type;                  // a client-set at a follower: redirect-client (below)
          emit = 4;
        } else if constexpr (SPEC) {
          spec_handle<N, MAJ>(S, n, lsw, sar, fr, lctr, which, id, k, bl, sgi, peers, m0, m1, fault, ev,
                              emit, nm, ra, rb, appended, applied, pkind, psrc, ppoff, ppcnt,
                              pold_base, preloc, papplied, elected, mchg, rearm, pk, pm);
        } else if (which < 0) {
          if (n.role == RAFT_LEADER) {                        // heartbeat-handler 162-164
            ev = 7;
            // append-entries-rpc (core.clj:56-67): last-entry, then per peer in doseq order
            // (- nil 1) and subvec of a LazySeq
            const uint32_t first = id == 1 ? 2u : 1u;
            if (n.commit > n.len) fault = RAFT_FAULT_IOOBE;
            else if (!(n.keys & 1u) || !((n.keys >> first) & 1)) fault = RAFT_FAULT_NPE;
            else if (n.seq) fault = RAFT_FAULT_CCE;
            else if ((n.keys & peers) != peers) fault = RAFT_FAULT_NPE;
            else emit = 2;
          } else {                                            // timeout-handler 166-169
            ev = 6;
            if (n.commit > n.len) {                           // last-entry (log.clj:47-49)
              fault = RAFT_FAULT_IOOBE;
            } else {
              uint32_t ep = 0, et = 0, evl = 0;
              if (n.commit) {
                const uint2 e = sar[(n.base + n.commit - 1) % A];
                ep = 1; et = e.x; evl = e.y;
              }
              n.role = RAFT_CANDIDATE; n.vf = id; n.votes = 1u << id; n.term += 1;  // 69-73
              ra = make_uint4(RAFT_MSG_REQUEST_VOTE | id << 3 | ep << 8, n.term, n.commit, 0);
              rb = make_uint4(et, evl, 0, 0);
              emit = 1;
            }
          }
        } else {
          ev = type;
          switch (type) {
            case RAFT_MSG_REQUEST_VOTE: {                     // request-vote-handler 91-103
              uint32_t consistent = 1;
              if (!(kargs()->variant & RAFT_VARIANT_VOTE_NO_LOG_CHECK) && ma != 0) {
                if (ma > n.len) {
                  fault = RAFT_FAULT_IOOBE;
                  break;
                }
                const uint2 e = sar[(n.base + ma - 1) % A];
                consistent = mep && e.x == met && e.y == mev;
              }
              const uint32_t grant = mterm >= n.term && n.vf == 0 && consistent;
              ra = make_uint4(RAFT_MSG_VOTE_RESPONSE | id << 3 | grant << 7, n.term, 0, 0);
              if (grant) n.vf = src;
              emit = 3;
              break;
            }
            case RAFT_MSG_APPEND_ENTRIES: {                   // append-entries-handler 105-123
              uint32_t consistent = 1;
              if (mb != 0) {
                if (mb > n.len) {
                  fault = RAFT_FAULT_IOOBE;
                  break;
                }
                const uint2 e = sar[(n.base + mb - 1) % A];
                consistent = mep && e.x == met && e.y == mev;
              }
              if (mterm < n.term) {
                ra = make_uint4(RAFT_MSG_APPEND_RESPONSE | id << 3, n.term, 0, 0);
              } else if (!consistent) {
                ra = make_uint4(RAFT_MSG_APPEND_RESPONSE | id << 3, n.term, 0, 0);
                n.len = n.len > mb ? n.len - mb : 0;          // remove-from! 78-81
                if constexpr (PROV) {
                  if ((pm >> 18) > n.len) pm = (pm & 0x3FFFFu) | n.len << 18;
                }
                n.seq = 1;
              } else {
                if (n.len + pcnt > (KAH ? ka_L : kargs()->L)) {
                  fault = RAFT_FAULT_OVERFLOW;
                  break;
                }
                ra = make_uint4(RAFT_MSG_APPEND_RESPONSE | id << 3 | 1u << 7, n.term, ma, mb + pcnt);
                pkind = PLAN_PAYLOAD; psrc = src; ppoff = mpoff; ppcnt = pcnt;
                pold_base = n.base;
                if (pcnt) {                                    // append-entries! 61-64
                  if (n.base + n.len != n.front) {
                    preloc = 1;
                    n.base = n.front;
                    n.front += n.len;
                  }
                  n.front += pcnt;
                          }
                const uint32_t oldc = n.commit;
                n.len += pcnt;
                n.seq = 0;
                appended = pcnt;
                n.commit = n.len;                              // apply-entries! 69-76
                applied = n.commit > oldc ? n.commit - oldc : 0;
                papplied = applied;
                n.role = RAFT_FOLLWER; n.vf = 0; n.votes = 0;  // candidate->follower 75-78
                n.lid = src; n.term = mterm;
              }
              emit = 3;
              break;
            }
            case RAFT_MSG_CLIENT_SET: {                        // client-set-handler 151-160
              if (LITE) break;                                 // (no client traffic)
              if (n.role != RAFT_LEADER) {                     // redirect-client: no state change
                emit = 4;
                break;
              }
              if (n.len + 1 > (KAH ? ka_L : kargs()->L)) {
                fault = RAFT_FAULT_OVERFLOW;
                break;
              }
              pkind = PLAN_ENTRY; ppoff = n.term; ppcnt = ma;
              pold_base = n.base;
              if (n.base + n.len != n.front) {
                preloc = 1;
                n.base = n.front;
                n.front += n.len;
              }
              n.front += 1;
                    n.len += 1;
              n.seq = 0;
              appended = 1;
              break;
            }
            case RAFT_MSG_VOTE_RESPONSE: {                     // vote-response-handler 125-139
              if (n.commit > n.len) {                          // last-entry first
                fault = RAFT_FAULT_IOOBE;
                break;
              }
              if (mterm > n.term) {
                n.term = mterm;
                n.role = RAFT_FOLLWER; n.vf = 0; n.votes = 0;
              } else if (flag && n.role == RAFT_CANDIDATE) {
                const uint32_t votes = n.votes | 1u << src;
                if (__popc(votes) < (N + 1) / 2) {             // majority? 19-21
                  n.votes = votes;
                } else if (n.seq) {
                  fault = RAFT_FAULT_CCE;      // append-entries-rpc's entries-from (log.clj:53)
                } else {                                       // candidate->leader 80-84
                  n.role = RAFT_LEADER; n.vf = 0; n.votes = 0; n.lid = id;
                  n.keys = peers | 1u;                         // leader-state 40-42
                  nm = 1;
                  emit = 2;
                  elected = true;
                }
              }
              break;
            }
            case RAFT_MSG_APPEND_RESPONSE: {                   // append-response-handler 141-149
              if (mterm > n.term) {                            // leader->follower 86-89
                n.term = mterm;
                n.role = RAFT_FOLLOWER; n.lid = 0; n.keys = 0;
                nm = 2;
              } else if (!flag) {
                if (!(n.keys & 1u) || !((n.keys >> src) & 1)) {
                  fault = RAFT_FAULT_NPE;                      // (dec nil)
                  break;
                }
                nm = 3;
              } else {
                n.keys |= 1u | 1u << src;
                nm = 4;
                mchg = true;
              }
              break;
            }
            default:
              break;
          }
        }
        RS_PHASE(2);
        const uint32_t tsrc = which >= 0 ? src : 0, tterm = which >= 0 ? mterm : 0;
        if (fault) {                                   // D8: halted with the pre-event state
          n.fault = fault;
          n.trace = trace_event(n.trace, t, ev, tsrc, tterm, n.role, n.term, fault);
          lctr_add(lctr, RAFT_CTR_HALT_IOOBE + fault - 1, 1);
          pkind = PLAN_NONE;
          papplied = 0;
          elected = false;
          mchg = false;
        } else {
          // generate-timeout (core.clj:171-174) for the next wait: every event re-arms the timer
          // (D4); Spec-Raft keeps Raft's timers (SIM_SPEC §8)
          if (n.role == RAFT_LEADER) {
            if (!SPEC || ev == 7 || elected) {
              n.deadline = t + (KAH ? ka_hb : kargs()->hb);
              if constexpr (REGS) dpend_r = 0;
              else dpend[lane] = 0;
            }
          } else if (!SPEC || ev == 6 || rearm || was_leader) {
            // Spec-Raft re-arms on few events (SIM_SPEC §8): drawn at once there
            if (SPEC && !have_w) w = event_draw(sg, id, t, S);
            const bool defer = !SPEC && !have_w;
            KDevSim* const K = kargs();
            n.deadline = t + (KAH ? ka_el_base : K->el_base) +
                         (defer ? 0u : __umulhi(w.y, KAH ? ka_el_span : K->el_span));
            if (!SPEC) {                                       // the draw is deferred
              if constexpr (REGS) dpend_r = defer;
              else dpend[lane] = defer;
            }
            have_w = have_w || SPEC;
          }
          n.trace = trace_event(n.trace, t, ev, tsrc, tterm, n.role, n.term, 0);
          // leader-state words (cold, in HBM)
          if (nm == 1 || nm == 2) {
            const int32_t first_next = (int32_t)((SPEC ? n.len : n.commit) + 1);
  #pragma unroll
            for (int p = 1; p <= N; ++p) {
              lsw.next(p - 1) = (nm == 1 && p != (int)id) ? first_next : 0;
              lsw.match(p - 1) = 0;
            }
          } else if (nm == 3) {
            if constexpr (SPEC) {
              const int32_t nx = lsw.next(src - 1) - 1;
              lsw.next(src - 1) = nx > 1 ? nx : 1;
            } else {
              lsw.next(src - 1) -= 1;
            }
          } else if (nm == 4) {
            lsw.next(src - 1) = (int32_t)(SPEC ? mb + 1 : mb);
            lsw.match(src - 1) = (int32_t)(SPEC ? mb : ma);
          }
          if (RC && ev == RAFT_MSG_CLIENT_SET) ++rc_cs;
          else lctr_add(lctr, RAFT_CTR_EV_RV + ev - 1, 1);
          if constexpr (RC) rc_app += appended;
          else lctr_add(lctr, RAFT_CTR_ENTRIES_APPENDED, appended);
          lctr_add(lctr, RAFT_CTR_ENTRIES_APPLIED, applied);
          if (elected) {
            lctr_add(lctr, RAFT_CTR_LEADERS, 1);
            n.led = n.term;
          }
          RS_PHASE(10);
          // ------------------------------------------------ redirect-client (server.clj:62-63)
          // to the :leader-id, else (rand-nth cluster) by w2 of the EVENT draw (core.clj:153-155);
          // the client follows it while the message has hops left (SIM_SPEC D15): a client-set
          // {a, b + 1} arriving at t + 1 outside the fault model. A redirect to the node itself
          // (a stepped-down leader keeps its :leader-id) goes through the sender record alone.
          if (!LITE && emit == 4) {
            emit = 0;
            if (mb >= (KAH ? ka_redir : kargs()->client_redirects)) {
              lctr_add(lctr, RAFT_CTR_CLIENT_ABANDONED, 1);
            } else {
              uint32_t dst = n.lid;
              if (!dst) {
                if (!have_w) { RS_PX(wl_px4); w = event_draw(sg, id, t, S); }   // (the timer stays deferred)
                const uint32_t i = __umulhi(w.z, N - 1);
                dst = i + 1 < id ? i + 1 : i + 2;
              }
              if constexpr (RC) ++rc_red;
              else lctr_add(lctr, RAFT_CTR_REDIRECTS, 1);
              *reinterpret_cast<uint2*>(mysrec + k * SRECW) =
                  make_uint2(dst == id ? mb + 1 : 0u, ma);
              if (dst != id) {
                uint32_t* cl =
                    mycells + (k * (N - 1) + (dst - 1 < (uint32_t)k ? dst - 1 : dst - 2)) * CELLW;
                cell_put(cl, make_uint4(RAFT_MSG_CLIENT_SET, 0, 0, mb + 1), make_uint4(0, 0, 0, 0));
                cl[CELLW - 1] = 1u | 1u << 16;     // one copy at t + 1 (SIM_SPEC D15)
              }
              sentmask |= 1u << dst;
            }
          }
          RS_PHASE(12);
          // ------------------------------------------------ emission (rpc / respond)
          // The message words go to the pair cells, then each message's fault draws (its delivery
          // pack, in the cell's last word) and the receiver's bit into sentmask.
          if (!STORM && emit) {
            RS_PHASE(13);
            // the cluster's partition draw for this tick's epoch, made once per epoch (SIM_SPEC P2)
            uint32_t pstate = 0;
            if (!LITE && kargs()->part_ppm) {
              const int cw = bl / N;
              KDevSim* const K = kargs();
              const DivU32 de = kdiv(K->div_epoch);
              const uint32_t e = udiv(de, t);
              pstate = pcache[CPW + cw];
              if (pcache[cw] != e) {
                RS_PX(wl_px5);
                const uint4 pw = philox(sg, P_PART << 8, e, 0, S.key0, S.key1);
                pstate = (pw.y & ~1u) | (ppm(pw.x) < K->part_ppm ? 1u : 0u);
                pcache[cw] = e;          // (the cluster's lanes that draw write the same words)
                pcache[CPW + cw] = pstate;
              }
            }
            RS_PHASE(14);
            *reinterpret_cast<uint2*>(mysrec + k * SRECW) =
                emit == 2 ? make_uint2(n.term, n.commit) : make_uint2(ra.y, ra.z);
            if (emit == 3) {
              uint32_t* cl =
                  mycells + (k * (N - 1) + (src - 1 < (uint32_t)k ? src - 1 : src - 2)) * CELLW;
              cell_put(cl, ra, rb);
              lctr_add(lctr, RAFT_CTR_SENT, 1);
              RS_PX(wl_px6);
              const uint32_t pack = deliver_pack<LITE>(S, sg, t, id, src, pstate, lctr);
              cl[CELLW - 1] = pack;
              if (pack >> 16) sentmask |= 1u << src;
            } else {
              // Message words for every peer at once: the next-index reads and then the prev-entry
              // loads of all peers are independent and issued together (one memory round trip for
              // the broadcast); a slot is always read, inside the arena, and used only when needed.
              if (emit == 2) {
                // prev of peer p (SPEC: SIM_SPEC §8's clamp(next - 1); faithful: core.clj:59-66's
                // max(next - 1, 0), whose entry is at min(prev, len)), read twice from the rows
                auto prev_of = [&](int p) -> uint32_t {
                  const int32_t pv = lsw.next(p) - 1;
                  if constexpr (SPEC) return pv <= 0 ? 0u : ((uint32_t)pv < n.len ? (uint32_t)pv : n.len);
                  return pv > 0 ? (uint32_t)pv : 0u;
                };
                // (an empty log sends no prev entry: no loads, e.g. every election from init-node)
                const uint32_t bm = n.base % A;
                uint2 e[N];
  #pragma unroll
                for (int p = 0; p < N; ++p) e[p] = make_uint2(0, 0);
                if (n.len) {
  #pragma unroll
                  for (int p = 0; p < N; ++p) {
                    const uint32_t prev = prev_of(p);
                    const uint32_t at = SPEC ? (prev ? prev - 1 : 0u) : (prev < n.len ? prev : 0u);
                    uint32_t slot = bm + at;
                    slot = slot >= A ? slot - A : slot;
                    e[p] = sar[slot];
                  }
                }
  #pragma unroll
                for (int p = 1; p <= N; ++p) {
                  if (p == (int)id) continue;
                  const uint2 ep2 = e[p - 1];
                  const uint32_t prev = prev_of(p - 1);
                  if constexpr (SPEC) {
                    const uint32_t ep = prev ? 1u : 0u;
                    const uint32_t pc = n.len - prev;
                    pmax = pc > pmax ? pc : pmax;
                    ra = make_uint4(RAFT_MSG_APPEND_ENTRIES | id << 3 | ep << 8 | pc << 16, n.term,
                                    n.commit, prev);
                    rb = make_uint4(ep ? ep2.x : 0u, ep ? ep2.y : 0u, pc ? n.base + prev : 0, 0);
                  } else {
                    const uint32_t start = prev < n.len ? prev : n.len;
                    const bool has = start < n.len;
                    const uint32_t pc = has ? n.len - start - 1 : 0u;
                    pmax = pc > pmax ? pc : pmax;
                    ra = make_uint4(RAFT_MSG_APPEND_ENTRIES | id << 3 | (has ? 1u : 0u) << 8 | pc << 16,
                                    n.term, n.commit, prev);
                    rb = make_uint4(has ? ep2.x : 0u, has ? ep2.y : 0u, pc ? n.base + start + 1 : 0u, 0);
                  }
                  cell_put(mycells + (k * (N - 1) + (p - 1 < k ? p - 1 : p - 2)) * CELLW, ra, rb);
                }
              } else {                                // request-vote: the same words for every peer
  #pragma unroll
                for (int j = 0; j < N - 1; ++j) cell_put(mycells + (k * (N - 1) + j) * CELLW, ra, rb);
              }
              RS_PHASE(15);
              if (pmax) atomicMax(&lctr[LCTR_PAYLOADMAX], pmax);
              lctr_add(lctr, RAFT_CTR_SENT, N - 1);
  #pragma unroll 1
              for (int p = 1; p <= N; ++p) {
                if (p == (int)id) continue;
                RS_PX(wl_px7);
                const uint32_t pack = deliver_pack<LITE>(S, sg, t, id, (uint32_t)p, pstate, lctr);
                mycells[(k * (N - 1) + (p - 1 < k ? p - 1 : p - 2)) * CELLW + CELLW - 1] = pack;
                if (pack >> 16) sentmask |= 1u << p;
              }
            }
            RS_PHASE(16);
          }
        }
      }

      RS_PHASE(3);
      // ---------------------------------------------------------------- P2 network delivery
      if (__ballot(sentmask != 0)) {
        // Senders that addressed this lane this tick (one ds_bpermute per cluster slot), then one
        // copy per loop trip in (sender id, copy) order: a single qinsert call site for the wave.
        uint32_t inmask = 0;
  #pragma unroll
        for (int s = 0; s < N; ++s) {
          const uint32_t sm = __shfl(sentmask, bl + s);
          inmask |= ((sm >> id) & 1u) << s;
        }
        if (!on) inmask = 0;
        uint32_t copy = 0;
        while (inmask) {
          const int s = __builtin_ctz(inmask);
          const uint2 sr = *reinterpret_cast<const uint2*>(mysrec + s * SRECW);
          uint2 c0 = make_uint2(RAFT_MSG_CLIENT_SET, sr.x), c1 = make_uint2(0, 0),
                c2 = make_uint2(0, 1u | 1u << 16);           // a redirect to this node itself
          if (s != k) {
            const uint2* cl = reinterpret_cast<const uint2*>(
                mycells + (s * (N - 1) + (k < s ? k : k - 1)) * CELLW);
            c0 = cl[0]; c1 = cl[1]; c2 = cl[2];
          }
          const uint32_t d = (LITE || copy == 0) ? (c2.y & 0xFF) : ((c2.y >> 8) & 0xFF);
          const int which = (c0.x & 7) <= RAFT_MSG_CLIENT_SET ? 0 : 1;
          QueueR q = which ? n.rs : n.rq;
          const uint4 q0 = make_uint4(t + d, c0.x, s != k ? sr.x : 0u, sr.y),
                      q1 = make_uint4(c0.y, c1.x, c1.y, c2.x);
          qinsert(S, sgi, n.fault, which, q, q0, q1, lctr, rdel, rhalt);
          if (which) n.rs = q;
          else n.rq = q;
          if (LITE || ++copy >= (c2.y >> 16)) {   // LITE: one copy per message
            copy = 0;
            inmask &= inmask - 1;
          }
        }
      }

      RS_PHASE(4);
      // ---------------------------------------------------------------- P3 log writes
      // m entries were added at position n.len - m (appended_at, -1 when none)
      const uint32_t m = pkind == PLAN_PAYLOAD ? ppcnt : (pkind == PLAN_ENTRY ? 1u : 0u);
      const int appended_at = m ? (int)(n.len - m) : -1;
      if (!STORM && __ballot(m || papplied || (TRACE && tr_cnt))) {
        // (the sender's frontier matters to payload appends only: no shuffle on entry-only trips)
        const uint32_t sfront = !RS_SHFL_GUARD || __ballot(m && pkind == PLAN_PAYLOAD)
                                    ? (uint32_t)__shfl(n.front, bl + (int)psrc - 1) : 0u;
        if (m) {
          const uint32_t pold_len = n.len - m;
          // physical slots advance with a wrap instead of a per-entry modulo
          if (preloc)
            arena_copy<LITE ? 1 : 8>(sar, n.base % A, sar, pold_base % A, pold_len, A);
          uint32_t di = (n.base + pold_len) % A;
          if (pkind == PLAN_ENTRY) {
            sar[di] = make_uint2(ppoff, ppcnt);
          } else {
            // entries i with sender frontier > poff + i + A were overwritten (SIM_SPEC P3)
            const int64_t ev = (int64_t)sfront - (int64_t)A - (int64_t)ppoff;
            const uint32_t evicted = ev <= 0 ? 0u : (ev >= (int64_t)m ? m : (uint32_t)ev);
            const uint2* sa = arena_of(S, sgi - k + psrc - 1);
            uint32_t si = (ppoff + evicted) % A;
            for (uint32_t i = 0; i < evicted; ++i) {
              sar[di] = make_uint2(0, 0);
              di = di + 1 == A ? 0 : di + 1;
            }
            arena_copy<LITE ? 1 : 8>(sar, di, sa, si, m - evicted, A);
            lctr_add(lctr, RAFT_CTR_PAYLOAD_EVICTED, evicted);
            if constexpr (PROV) {
              pk = ppoff - pold_len;
              pm = evicted == 0 && n.len < (1u << 14) ? psrc | pold_len << 4 | n.len << 18 : 0u;
            }
          }
        }
        if (papplied) {          // apply-entries! writes the last `applied` :val's (log.clj:69-76)
          KDevSim* const K = kargs();
          uint32_t* const cca = K->ccount;
          const uint32_t SC = K->SC;
          uint32_t cc = cca[sgi];
          if (SC) {
            uint32_t si = (n.base + n.commit - papplied) % A, so = cc % SC;
            uint32_t* const ring = K->stream + (size_t)sgi * SC;
            for (uint32_t i = 0; i < papplied; ++i) {
              ring[so] = sar[si].y;
              si = si + 1 == A ? 0 : si + 1;
              so = so + 1 == SC ? 0 : so + 1;
            }
          }
          cca[sgi] = cc + papplied;
        }
        if constexpr (TRACE) {   // the traced message's :entries, resolved like the payload above
          const uint32_t tfront = __shfl(n.front, bl + (int)tr_src - 1);
          if (tr_cnt && S.TE) {
            const int64_t ev = (int64_t)tfront - (int64_t)A - (int64_t)tr_poff;
            const uint32_t evicted = ev <= 0 ? 0u : (ev >= (int64_t)tr_cnt ? tr_cnt : (uint32_t)ev);
            const uint2* sa = arena_of(S, sgi - k + tr_src - 1);
            uint2* ring = S.tent + (size_t)sgi * S.TE;
            for (uint32_t i = 0; i < tr_cnt; ++i)
              ring[(tr_at + i) % S.TE] =
                  i < evicted ? make_uint2(0, 0) : sa[(tr_poff + i) % A];
          }
        }
      }

      RS_PHASE(5);
      // ---------------------------------------------------------------- P4 invariant checker
      // the majority-match scan can raise hwm only when the leader's log reaches past it
      const bool mcheck = (elected || mchg) && n.len > hidx;
      if (!RS_KO_P4 && !STORM && __ballot(elected || appended_at >= 0 || mcheck)) {
        if (__ballot(elected)) {                       // election safety
          bool bad = false;
  #pragma unroll
          for (int s = 0; s < N; ++s) {
            const uint32_t ls = __shfl(n.led, bl + s);
            bad |= elected && s != k && ls == n.led;
          }
          if (bad) violation(lctr, RAFT_CTR_VIOL_ELECTION, t);
        }
        if (!RS_KO_LOGM && __ballot(appended_at >= 0)) {              // log matching
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");   // peers' P3 arena writes
          // Each lane b compares its own log with the new entries of every other node a of its
          // cluster that appended this tick, pair after pair, W positions per trip of one
          // wave-wide loop (a wave runs as many trips as its busiest lane needs, not the sum over
          // node indices of the busiest lane per index); a counts one violation if any peer found
          // a position with the same term and another value. The appenders' (appended_at, base,
          // len) go through LDS (the cells: P2 is done with them) so a lane can read any
          // appender's words from inside the divergent loop.
          // Copies of one payload: a payload append's entry at position p comes from its sender's
          // arena slot key + p (key = source offset - appended_at; evicted ones read (0, 0) the
          // same way, SIM_SPEC P3), so two nodes that appended payloads of the same sender with the
          // same key in this tick hold the same entries where both appended (no write this tick
          // reaches a slot that is not evicted). A lane therefore compares one member of each group
          // of appenders with the same (sender, key, appended_at, len) and gives the group its
          // result, and skips positions where it appended a copy of the same payload itself: the
          // followers of a broadcast that all appended the leader's entries in one tick cost one
          // comparison per lane instead of one per follower (C4). Only with a fixed delay, where a
          // broadcast's copies land in one tick (with random delays they rarely do), as separate
          // code (sharing the loop with the plain form cost C3's kernel 2 % in registers).
          uint32_t* const apw = cells;
          apw[lane] = (uint32_t)appended_at;
          apw[64 + lane] = n.base;
          apw[128 + lane] = n.len;
          if constexpr (PROV) {   // this tick's payload append and its provenance (0: none)
            apw[320 + lane] = appended_at >= 0 && pkind == PLAN_PAYLOAD ? pm : 0u;
            apw[384 + lane] = pk;
          }
          const uint32_t apc = (uint32_t)(__ballot(active && appended_at >= 0) >> bl) & cmask;
          constexpr int W = LITE ? 1 : 8;
          uint32_t found = 0;
          auto log_match = [&](auto grouping) {
            constexpr bool G = decltype(grouping)::value;
            const bool pay = G && pkind == PLAN_PAYLOAD && appended_at >= 0;
            if constexpr (G) {
              apw[192 + lane] = ppoff - (uint32_t)appended_at;  // key (payload appends)
              apw[256 + lane] = pay ? psrc : 0u;               // sender, 0: no payload
            }
            __builtin_amdgcn_wave_barrier();
            uint32_t todo = active ? apc & ~(1u << k) : 0u;
            uint32_t cur = 0, rem = 0, xi = 0, yi = 0;
            const uint2* xa = sar;
            while (__ballot(todo || rem)) {
              if (!rem && todo) {
                const int a = __builtin_ctz(todo);
                const uint32_t aat = apw[bl + a], ab = apw[64 + bl + a], al = apw[128 + bl + a];
                uint32_t grp = 1u << a;
                uint32_t hi = al < n.len ? al : n.len;
                if constexpr (G) {
                  const uint32_t akey = apw[192 + bl + a], asrc = apw[256 + bl + a];
                  if (asrc) {
  #pragma unroll
                    for (int s2 = 0; s2 < N; ++s2)
                      grp |= (uint32_t)(((todo >> s2) & 1) && apw[bl + s2] == aat &&
                                        apw[128 + bl + s2] == al && apw[192 + bl + s2] == akey &&
                                        apw[256 + bl + s2] == asrc) << s2;
                  }
                  if (asrc && pay && psrc == asrc && ppoff - (uint32_t)appended_at == akey)
                    hi = min(hi, (uint32_t)appended_at);     // where this lane holds the same copy
                }
                if constexpr (PROV) {
                  // a's new entries are copies of S's slots akey + p: equal to this lane's
                  // entries when this lane is S at base akey (its log position p is slot
                  // base + p), or when its positions [aat, hi) are copies of the same slots
                  const uint32_t am = apw[320 + bl + a];
                  if (am) {
                    const uint32_t akey = apw[384 + bl + a];
                    const bool same = ((am & 15) == id && akey == n.base) ||
                                      ((pm & 15) == (am & 15) && pk == akey &&
                                       ((pm >> 4) & 0x3FFFu) <= aat && hi <= (pm >> 18));
                    if (same) hi = aat;
                  }
                }
                todo &= ~grp;
                rem = hi > aat ? hi - aat : 0u;
                xi = (ab + aat) % A;
                yi = (n.base + aat) % A;
                xa = arena_of(S, sgi - k + a);
                cur = grp;
              }
              if (rem) {
                bool hit;
                const uint32_t c = log_conflict_chunk<W>(xa, xi, sar, yi, rem, A, hit);
                if (hit) {
                  found |= cur;
                  rem = 0;
                } else {
                  rem -= c;
                  xi += c;
                  yi += c;
                  xi = xi == A ? 0 : xi;
                  yi = yi == A ? 0 : yi;
                }
              }
            }
          };
          // (N <= 5 kernels run four waves per SIMD at 128 VGPRs: the grouped form costs them
          // scratch, and their payloads are short)
          KDevSim* const KG = kargs();
          if constexpr (N >= 6) {
            if (KAH ? ka_fixd : KG->dmin == KG->dmax) log_match(std::true_type{});
            else log_match(std::false_type{});
          } else {
            log_match(std::false_type{});
          }
          uint32_t fa = 0;
          if (!RS_SHFL_GUARD || __ballot(found != 0)) {       // (a conflict is rare)
  #pragma unroll
            for (int s = 0; s < N; ++s) fa |= (uint32_t)__shfl((int)found, bl + s);
          }
          const bool bad = active && ((fa >> k) & 1);
          if (bad) violation(lctr, RAFT_CTR_VIOL_LOG, t);
        }
        if (elected && hidx > 0) {                     // leader completeness (pre-tick hwm)
          bool ok = n.len >= hidx;
          if (ok) {
            const uint2 e = sar[(n.base + hidx - 1) % A];
            ok = e.x == hterm && e.y == hval;
          }
          if (!ok) violation(lctr, RAFT_CTR_VIOL_COMPLETE, t);
        }
        int32_t cm = -1;
        uint32_t ct = 0, cv = 0;
        if (on && n.role == RAFT_LEADER && mcheck) {
          // {log_len} ∪ match_index of the peers, the own slot holding log_len: the network
          // sorts the multiset, so the slot order does not matter, and a fixed slot per peer keeps
          // the array in registers (a running index over the peers put it on the stack)
          int32_t vals[N];
  #pragma unroll
          for (int p = 1; p <= N; ++p)
            vals[p - 1] = p == (int)id ? (int32_t)n.len
                                       : (((n.keys >> p) & 1) ? lsw.match(p - 1) : 0);
  #pragma unroll
          for (int i = 1; i < N; ++i)
  #pragma unroll
            for (int q = i; q > 0; --q)
              if (vals[q - 1] < vals[q]) {
                const int32_t tmp = vals[q]; vals[q] = vals[q - 1]; vals[q - 1] = tmp;
              }
          int32_t mm = vals[MAJ - 1];
          if (mm > (int32_t)n.len) mm = (int32_t)n.len;
          if (mm > (int32_t)hidx) {
            const uint2 e = sar[(n.base + (uint32_t)mm - 1) % A];
            if (!SPEC || e.x == n.term) {   // SIM_SPEC §8: committed only in the leader's term
              cm = mm;
              ct = e.x; cv = e.y;
            }
          }
        }
        if (__ballot(cm >= 0)) {                       // cluster argmax, lowest id on ties
          int32_t best = -1;
          uint32_t bt = 0, bv = 0;
  #pragma unroll
          for (int s = 0; s < N; ++s) {
            const int32_t sm = __shfl(cm, bl + s);
            const uint32_t st = __shfl(ct, bl + s), sv = __shfl(cv, bl + s);
            if (sm > best) { best = sm; bt = st; bv = sv; }
          }
          if (on && best > 0) { hidx = (uint32_t)best; hterm = bt; hval = bv; }
        }
      }
      RS_PHASE(6);
  #ifdef RS_WAVELOG
      ++wl_active;
      wl_first = wl_first == INF ? t - t0 : wl_first;
  #endif

      // ------------------------------------------------------- append-response drain (faithful)
      // A leader answers each append-response with no message, no log write and -- while its log
      // does not reach past the checker's high-water mark -- no check: the event touches its own
      // words only (core.clj:141-149, timer 171-174). Ticks at which a cluster's only events are
      // such responses are therefore run here without P0 and P2-P4, one response per leader per
      // tick as above, until the cluster's next other event E (the REQ head and client-set of every
      // node, and the deadline and RES head of every node that is not a live leader). A tick at
      // which a leader's event is anything else (a heartbeat, or a head message that is not such
      // a response) ends the cluster's drain before that tick; the loop above then runs it. Steady
      // state: a heartbeat round's four responses at the leader take one trip through here, not four ticks.
      // Only where it pays: clusters of up to five nodes without client traffic (C2; with client
      // traffic a cluster has an event nearly every tick of a burst: measured C3 +3 % with one
      // wave-wide clock, unchanged with per-cluster clocks, C4-N9 +1 %), and it would cost the
      // larger-N kernels occupancy (N = 9: 125 -> 129 VGPRs).
      if constexpr (!SPEC && !TRACE && !STORM && N <= 5) if (LITE || !kargs()->client_ppm) {
        // leaders whose responses can drain: a log past the hwm makes a success response a
        // checker event (C3/C4 replication), so those leaders stay with the loop
        const bool elig = on && !n.fault && n.role == RAFT_LEADER && n.len <= hidx;
        if (__ballot(elig && n.rs.c)) {
          const uint32_t oth = (!on || n.fault) ? INF
                               : elig ? min(n.rq.arr, cnext)
                                      : min(min(n.deadline, n.rq.arr), min(n.rs.arr, cnext));
          // the cluster's next other event E; a cluster drains while its leaders' responses are
          // its only events before E
          const uint32_t E = min(cluster_min(oth), tend);
          const bool any_res = cluster_any(elig && n.rs.c);
          const bool any_ready = cluster_any(elig && n.rs.arr < E);
          bool dr = on && any_res && any_ready && E > t + 1;
          if (__ballot(dr)) {
            const uint32_t* qb = qslots(S, sgi, 1);
            const size_t qs = qstride(S, 1);
            // A cluster with one eligible leader (the usual case) drains in that lane alone: its
            // ticks are the leader's own, so the loop needs no cluster reductions per tick. The
            // stop rules are the cluster loop's below: tau reaches E, a heartbeat falls due, or the
            // head message is not such a response.
            const uint32_t em = (uint32_t)(__ballot(elig) >> bl0) & cmask;
            const bool solo = dr && __popc(em) == 1;
            if (__ballot(solo)) {
              if (solo && elig) {
                for (;;) {
                  const uint32_t tau = max(min(n.rs.arr, n.deadline), t + 1);
                  if (tau >= E || n.rs.arr > tau) break;       // E, or the heartbeat's tick
                  const uint4* sp = reinterpret_cast<const uint4*>(qb + n.rs.h * qs);
                  const uint4 m0 = sp[0], m1 = sp[1];
                  const uint32_t nh = wrapq(n.rs.h + 1, S.Q);
                  uint32_t narr = INF;
                  if (n.rs.c > 1)
                    narr = (n.rs.c == 2 || n.rs.arr == n.rs.tail) ? n.rs.tail : qb[nh * qs];
                  const uint32_t hdr = m0.y, mterm = m0.z, src = (hdr >> 3) & 15,
                                 flag = (hdr >> 7) & 1;
                  if (!((hdr & 7) == RAFT_MSG_APPEND_RESPONSE && mterm <= n.term &&
                        (flag ? n.len <= hidx : (n.keys & 1u) && ((n.keys >> src) & 1))))
                    break;
                  QueueR r = n.rs;
                  r.h = nh;
                  r.c -= 1;
                  r.arr = r.c ? narr : INF;
                  r.tail = r.c ? r.tail : 0u;
                  if (!r.c) r.h = 0;
                  n.rs = r;
                  if (flag) {                                // append-response-handler 145-149
                    n.keys |= 1u | 1u << src;
                    lsw.next(src - 1) = (int32_t)m1.x;
                    lsw.match(src - 1) = (int32_t)m0.w;
                  } else {                                   // 143-144: (dec next-index)
                    lsw.next(src - 1) -= 1;
                  }
                  n.deadline = tau + kargs()->hb;
                  n.trace = trace_event(n.trace, tau, RAFT_MSG_APPEND_RESPONSE, src, mterm, n.role,
                                        n.term, 0);
                  lctr_add(lctr, RAFT_CTR_EV_AR, 1);
                  t = tau;
                }
              }
              const uint32_t lt = __shfl(t, bl0 + (em ? (int)__builtin_ctz(em) : 0));
              if (solo) t = lt;                              // the cluster takes the leader's clock
              dr = dr && !solo;
            }
            for (;;) {
              const uint32_t nxt = elig ? min(n.rs.arr, n.deadline) : INF;   // leader's next event
              const uint32_t tau = max(cluster_min(nxt), t + 1);
              dr = dr && tau < E;
              const bool ev = dr && elig && n.rs.arr <= tau;  // a ready message beats the timer
              const bool hbeat = dr && elig && !ev && n.deadline <= tau;
              uint4 m0 = make_uint4(0, 0, 0, 0), m1 = make_uint4(0, 0, 0, 0);
              uint32_t narr = INF;
              const uint32_t nh = wrapq(n.rs.h + 1, S.Q);
              if (ev) {
                const uint4* sp = reinterpret_cast<const uint4*>(qb + n.rs.h * qs);
                m0 = sp[0];
                m1 = sp[1];
                if (n.rs.c > 1)
                  narr = (n.rs.c == 2 || n.rs.arr == n.rs.tail) ? n.rs.tail : qb[nh * qs];
              }
              const uint32_t hdr = m0.y, mterm = m0.z, src = (hdr >> 3) & 15, flag = (hdr >> 7) & 1;
              const bool simple = (hdr & 7) == RAFT_MSG_APPEND_RESPONSE && mterm <= n.term &&
                                  (flag ? n.len <= hidx : (n.keys & 1u) && ((n.keys >> src) & 1));
              // a tick at which any node of the cluster needs the loop above is the loop's to run
              dr = dr && !cluster_any(hbeat || (ev && !simple));
              if (!__ballot(dr)) break;
              if (dr && ev) {
                QueueR r = n.rs;
                r.h = nh;
                r.c -= 1;
                r.arr = r.c ? narr : INF;
                r.tail = r.c ? r.tail : 0u;
                if (!r.c) r.h = 0;
                n.rs = r;
                if (flag) {                                  // append-response-handler 145-149
                  n.keys |= 1u | 1u << src;
                  lsw.next(src - 1) = (int32_t)m1.x;
                  lsw.match(src - 1) = (int32_t)m0.w;
                } else {                                     // 143-144: (dec next-index)
                  lsw.next(src - 1) -= 1;
                }
                n.deadline = tau + kargs()->hb;
                n.trace = trace_event(n.trace, tau, RAFT_MSG_APPEND_RESPONSE, src, mterm, n.role,
                                      n.term, 0);
                lctr_add(lctr, RAFT_CTR_EV_AR, 1);
              }
              if (dr) t = tau;
  #ifdef RS_WAVELOG
              ++wl_drain;
  #endif
            }
          }
        }
      }
      RS_PHASE(7);
      tnext = t + 1;
    }
  #ifdef RS_WAVELOG
    uint32_t wl_px[8] = {wl_px0, wl_px1, wl_px2, wl_px3, wl_px4, wl_px5, wl_px6, wl_px7};
  #pragma unroll
    for (int q = 0; q < 8; ++q)
  #pragma unroll
      for (int o = 32; o > 0; o >>= 1) wl_px[q] += (uint32_t)__shfl_xor((int)wl_px[q], o);
    if (lane == 0 && S.wavelog) {
      const uint64_t wl_end = wall_clock64();
      uint32_t hw, xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      uint4* rec = reinterpret_cast<uint4*>(S.wavelog + (size_t)wave * 48);
      rec[0] = make_uint4((uint32_t)wl_start, (uint32_t)(wl_start >> 32), (uint32_t)wl_end,
                          (uint32_t)(wl_end >> 32));
      rec[1] = make_uint4(wl_active, hw, xcc, (wl_kmax - wl_kmin) << 16 | (wl_first & 0xFFFF));
      rec[2] = make_uint4(wl_ph[0], wl_ph[1], wl_ph[2], wl_ph[3]);
      rec[3] = make_uint4(wl_ph[4], wl_ph[5], wl_ph[6], wl_ph[7]);
      rec[4] = make_uint4(wl_ph[8], wl_ph[9], wl_ph[10], wl_ph[11]);
      rec[5] = make_uint4(wl_drain, wl_inj, wl_dead, wl_ph[12]);
      rec[6] = make_uint4(wl_px[0], wl_px[1], wl_px[2], wl_px[3]);
      rec[7] = make_uint4(wl_px[4], wl_px[5], wl_px[6], wl_px[7]);
      rec[8] = make_uint4(wl_ph[13], wl_ph[14], wl_ph[15], wl_ph[16]);
    }
  #endif

    // ---------------------------------------------------------------- write back
    // a deferred draw stays owed in the stored state (FL_DRAW, device.hpp)
    const uint32_t owed = !SPEC && active && (REGS ? dpend_r : dpend[lane]) ? FL_DRAW : 0u;
    if (!SPEC) dpend[lane] = 0;
    KDevSim* const KW = kargs();
    if (KW->shist) {
      // RAFT_SCHED_ALIGNED: the cluster's packing key relative to the next launch, counted into the
      // bucket histogram the host turns into the next launch's wave packing (sched_range_kernel)
      const uint32_t me = active && !n.fault ? sched_key_of(n.deadline, n.rq, n.rs) : INF;
      uint32_t cm = active ? cnext : INF;
  #pragma unroll
      for (int s = 0; s < N; ++s) cm = min(cm, (uint32_t)__shfl(me, bl0 + s));
      const bool head = active && k0 == 0;
      // With client traffic every cluster is busy on most ticks of a burst and a wave lasts as
      // long as its busiest cluster (per-cluster clocks): clusters are then packed by how many
      // event ticks they ran in this launch, busiest first (they start first and are done before
      // the tail), instead of by their next event.
      // The last bucket is kept for dead clusters (every node halted), which the next launch then
      // packs into waves of their own and runs without trips (below the state load).
      const bool dead = ((uint32_t)(__ballot(active && n.fault) >> bl0) & cmask) == cmask;
      const uint32_t key = !head ? INF
                           : KW->client_ppm
                               ? (dead ? SCHED_BUCKETS - 1
                                       : SCHED_BUCKETS - 2 -
                                             min(REGS ? trips_r : tripsL[cs], SCHED_BUCKETS - 2))
                               : sched_bucket(cm, tend);
      if (head) KW->skey[c] = key;
      // a packed wave's clusters usually share their next key: one histogram atomic for the wave
      const uint32_t kmin = wave_min(key), kmax = ~wave_min(head ? ~key : ~0u);
      const uint32_t heads = (uint32_t)__popcll(__ballot(head));   // (ballot outside any branch)
      if (kmin == kmax) {
        if (lane == 0 && kmin != INF) atomicAdd(&KW->shist[kmin], heads);
      } else if (head) {
        atomicAdd(&KW->shist[key], 1u);
      }
    }
    if (active) {
      // the block's addresses again from the cluster index (held across the tick loop they would
      // take four VGPRs there)
      uint32_t cw = c;
      asm volatile("" : "+v"(cw));
      uint32_t* const hp = S.hot + (size_t)cw * HB + HOT_CW + k0;
      uint32_t* const hc = S.hot + (size_t)cw * HB + CLW;
      hp[HF_FLAGS * N] = pack_flags(n.role, n.vf, n.lid, n.fault, n.seq, n.keys & 1u) | owed;
      hp[HF_MASKS * N] = n.votes | (n.keys & ~1u) << 16;
      hp[HF_TERM * N] = n.term; hp[HF_COMMIT * N] = n.commit; hp[HF_LEN * N] = n.len;
      hp[HF_DEADLINE * N] = n.deadline;
      hp[HF_QMETA * N] = pack_qmeta(n.rq.h, n.rq.c, n.rs.h, n.rs.c);
      hp[HF_REQ_ARR * N] = n.rq.arr; hp[HF_RES_ARR * N] = n.rs.arr;
      hp[HF_REQ_TAIL * N] = n.rq.tail; hp[HF_RES_TAIL * N] = n.rs.tail;
      hp[hf_abase(N) * N] = n.base; hp[hf_afront(N) * N] = n.front; hp[hf_led(N) * N] = n.led;
      hp[HF_TRACE_LO * N] = (uint32_t)n.trace; hp[HF_TRACE_HI * N] = (uint32_t)(n.trace >> 32);
      if constexpr (nm_lds_in<N, STORM>()) {
  #pragma unroll
        for (int p = 0; p < N; ++p) {
          hp[(HF_NEXT + p) * N] = nmL[p * 64 + lane];
          hp[(HF_NEXT + N + p) * N] = nmL[(N + p) * 64 + lane];
        }
      }
      if (k0 == 0) {
        hc[0] = hidx; hc[1] = hterm; hc[2] = hval; hc[3] = cnext; hc[4] = ccount;
        hc[CL_CERT] = 0;                    // the steady certificate no longer holds (device.hpp)
      }
    }
  } while (CATCH && (wave += wstride) * CPW < nslots);   // the general grid covers every slot
  if constexpr (RC) {
    lctr_add(lctr, RAFT_CTR_EV_CS, rc_cs);
    lctr_add(lctr, RAFT_CTR_REDIRECTS, rc_red);
    lctr_add(lctr, RAFT_CTR_DELIVERED, rc_del);
    lctr_add(lctr, RAFT_CTR_ENTRIES_APPENDED, rc_app);
    lctr_add(lctr, RAFT_CTR_TO_HALTED, rc_halt);
    if (lane == 0) lctr_add(lctr, RAFT_CTR_CLIENT_INJECTED, rc_inj);
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  unsigned long long* const ctr = kargs()->ctr + (size_t)(ctr_copy % CTR_COPIES) * CTR_STRIDE;
  if (lane < RAFT_CTR_COUNT) {
    const uint32_t v = lctr[lane];
    if (v) atomicAdd(&ctr[lane], (unsigned long long)v);
  } else if (lane == LCTR_FIRSTVIOL) {
    const uint32_t v = lctr[lane];
    if (v != INF) atomicMin(&ctr[RAFT_CTR_COUNT], (unsigned long long)v);
  } else if (lane == LCTR_PAYLOADMAX) {
    const uint32_t v = lctr[lane];
    if (v) atomicMax(&ctr[RAFT_CTR_COUNT + 1], (unsigned long long)v);
  }
}

}  // namespace rs

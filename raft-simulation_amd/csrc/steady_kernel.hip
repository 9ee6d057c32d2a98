// steady_kernel.hip — the steady-state tick kernel of LITE launches for gfx950 (MI355X).
//
// In a LITE launch (no client traffic, no faults, fixed delay: BASELINE config 2) a cluster that
// has elected its leader repeats one heartbeat round forever: the leader's heartbeat broadcasts an
// empty append-entries (heartbeat-handler, core.clj:162-164; append-entries-rpc 56-67), every
// follower answers it (append-entries-handler 105-123) and the leader takes the answers, one per
// tick (append-response-handler 141-149). This kernel runs exactly those events, bit for bit as
// the general tick kernel does (SIM_SPEC.md §4), and nothing else: a cluster about to run any other
// event (an election, a log entry, a halt, a message it cannot hold) is stopped ("bailed") before
// that tick with its state written back, and the catch-up launch of the general kernel runs it from
// that tick to the launch's end (DevSim::bail_c / bail_t / nbail). Results are therefore identical
// to the general kernel's for any state; only the speed depends on how steady the clusters are.
//
// What the narrow event set buys: no log arena, no HBM queue traffic and a small register set.
// * Queues live in LDS for the whole launch. Every ordered (sender, receiver) pair of a cluster
//   owns one 4-word cell (arrival, term, a, b | hdr << 24); a node's REQ and RES queues are lists of
//   sender ids (4 bits each) in one VGPR. A message whose pair cell is still occupied, or one the
//   cell cannot express (entries, a payload reference, b >= 2^24), bails its cluster. The HBM rings
//   are read at launch start and written at the end (heads at slot 0; ring positions are not state).
// * The leader-state rows (next-index / match-index) of the cluster's one ls_present node live in
//   LDS; the other nodes' rows are never touched (a second ls_present node bails the cluster).
// * Log length, arena cursors, last-led term and commit counts cannot change here, so they are
//   neither loaded nor stored.
// Registers: ~60 VGPRs against the general kernel's 117, so a wave slot per SIMD more than the
// whole config-2 grid needs: one generation of waves instead of two.
#include <hip/hip_ext.h>

#include "device.hpp"

namespace rs {

constexpr int SCW = 4;   // words per pair cell: arrival, term, a, b | hdr << 24 (free: word 3 == 0)

// clusters per wave (whole clusters, one lane per node)
template <int N>
constexpr int steady_cpw() { return 64 / N; }
// words of pad after each cluster's cells (spreads the clusters' cells over the LDS banks)
#ifndef RS_CPAD
#define RS_CPAD 0
#endif
template <int N>
constexpr int steady_cluster_words() { return N * (N - 1) * SCW + RS_CPAD; }
template <int N>
constexpr int steady_cell_words() { return steady_cpw<N>() * steady_cluster_words<N>(); }
template <int N>
constexpr size_t steady_lds_bytes() {
  return (size_t)(steady_cell_words<N>() + steady_cpw<N>() * 2 * N + LCTR_WORDS) * sizeof(uint32_t);
}

// fl bits kept beside the packed flags word (pack_flags) while the kernel runs
constexpr uint32_t SF_ACKBAD = 1u << 15;   // log_len > checker hwm: a success response is a check
// every queued message of the REQ (RES) list has the head's arrival, so a pop knows the next head's
// arrival without reading its cell (messages delivered in one tick share their arrival)
constexpr uint32_t SF_REQSAME = 1u << 16, SF_RESSAME = 1u << 17;

template <int N>
__global__ void __launch_bounds__(64) steady_kernel(DevSim S, uint32_t t0, uint32_t nt) {
  static_assert(N >= 2 && N <= 5, "4-bit sender lists of at most four entries");
  constexpr int CPW = steady_cpw<N>();
  constexpr uint32_t ALL = ((1u << (N + 1)) - 1) & ~1u;
  constexpr uint32_t HB = hot_block_words(N), CLW = hot_cl_off(N);
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t* const cells = smem;                      // [CPW][N][N-1][SCW] (+ pad per cluster)
  int32_t* const rows = reinterpret_cast<int32_t*>(smem + steady_cell_words<N>());  // [CPW][2N]
  uint32_t* const lctr = smem + steady_cell_words<N>() + CPW * 2 * N;
  const int lane = threadIdx.x;
  if (lane < LCTR_WORDS) lctr[lane] = lane == LCTR_FIRSTVIOL ? INF : 0u;
  if (blockIdx.x == 0 && lane == 0) *S.nbail_zero = 0;   // the bail counter of the next launch

  const uint32_t wave = blockIdx.x;
  const uint32_t nslots = S.perm ? *S.nslots : S.C;
  if (wave * CPW >= nslots) return;
  const int cs = lane / N, k = lane - cs * N;
  const int bl = (cs < CPW ? cs : 0) * N;
  const uint32_t slot = wave * CPW + cs;
  const uint32_t c0 = cs < CPW && slot < nslots ? (S.perm ? S.perm[slot] : slot) : INF;
  const bool active = c0 != INF;
  const uint32_t c = active ? c0 : 0u;
  const uint32_t g = S.goff + c, gi = c * N + k, id = k + 1;
  const uint32_t peers = ALL & ~(1u << id);
  const uint32_t cmask = (1u << N) - 1;
  uint32_t* const hp = S.hot + (size_t)c * HB + k;
  uint32_t* const hc = S.hot + (size_t)c * HB + CLW;
  int32_t* const myrows = rows + (cs < CPW ? cs : 0) * 2 * N;    // next[N], then match[N]
  // this lane's pair cells: outgoing (to receiver index j) and incoming (from sender index s)
  uint32_t* const ccells = cells + (cs < CPW ? cs : 0) * steady_cluster_words<N>();
  auto cell_out = [&](int j) { return ccells + (k * (N - 1) + (j < k ? j : j - 1)) * SCW; };
  auto cell_in = [&](int s) { return ccells + (s * (N - 1) + (k < s ? k : k - 1)) * SCW; };
  if (cs < CPW) {                  // every pair cell starts free
#pragma unroll
    for (int j = 0; j < N - 1; ++j) ccells[(k * (N - 1) + j) * SCW + 3] = 0;
  }
  __builtin_amdgcn_wave_barrier();

  auto cluster_any = [&](bool x) { return ((uint32_t)(__ballot(x) >> bl) & cmask) != 0; };
  auto cluster_min = [&](uint32_t x) {
    uint32_t m = x;
#pragma unroll
    for (int s = 0; s < N; ++s) m = min(m, (uint32_t)__shfl(x, bl + s));
    return m;
  };

#ifdef RS_WAVELOG   // diagnostic build: per-wave timeline + per-phase cycles (scripts/wavelog_probe.py)
  const uint64_t wl_start = wall_clock64();
  uint32_t wl_trips = 0, wl_ph[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t wl_ts = __builtin_amdgcn_s_memtime();
#define RS_PHASE(i)                                          \
  do {                                                       \
    const uint64_t now_ = __builtin_amdgcn_s_memtime();      \
    wl_ph[i] += (uint32_t)(now_ - wl_ts);                    \
    wl_ts = now_;                                            \
  } while (0)
#else
#define RS_PHASE(i) do {} while (0)
#endif
  // ------------------------------------------------------------------ state load (launch start)
  uint32_t fl = 0, mk = 0, term = 0, commit = 0, len = 0, deadline = INF, rqa = INF, rsa = INF;
  uint32_t lists = 0;             // REQ senders (id) in nibbles 0-3, RES senders in nibbles 4-7
  uint64_t trace = 0;
  bool bad = false;               // the cluster's start state is outside this kernel's model
  if (active) {
    fl = hp[HF_FLAGS * N]; mk = hp[HF_MASKS * N];
    term = hp[HF_TERM * N]; commit = hp[HF_COMMIT * N]; len = hp[HF_LEN * N];
    deadline = hp[HF_DEADLINE * N];
    const uint32_t qm = hp[HF_QMETA * N];
    rqa = hp[HF_REQ_ARR * N]; rsa = hp[HF_RES_ARR * N];
    trace = (uint64_t)hp[HF_TRACE_HI * N] << 32 | hp[HF_TRACE_LO * N];
    if (len > hc[0]) fl |= SF_ACKBAD;
    // queued messages into the pair cells, in ring order
    const uint32_t rqh = qm & 15, rqc = (qm >> 4) & 31, rsh = (qm >> 9) & 15, rsc = (qm >> 13) & 31;
    if (rqc + rsc > N - 1) bad = true;
    uint32_t used = 0;
    for (uint32_t i = 0; i < rqc + rsc && !bad; ++i) {
      const bool res = i >= rqc;
      const uint32_t pos = wrapq((res ? rsh + i - rqc : rqh + i), S.Q);
      const uint4* mp = reinterpret_cast<const uint4*>(qslots(S, gi, res) + pos * qstride(S, res));
      const uint4 m0 = mp[0], m1 = mp[1];
      const uint32_t hdr = m0.y, src = (hdr >> 3) & 15;
      if ((hdr >> 8) || m1.y || m1.z || m1.w || m1.x >= (1u << 24) || src < 1 || src > N ||
          src == id || ((used >> src) & 1) || m0.x > t0 + S.dmin) {
        bad = true;
      } else {
        used |= 1u << src;
        *reinterpret_cast<uint4*>(cell_in(src - 1)) = make_uint4(m0.x, m0.z, m0.w, m1.x | hdr << 24);
        const uint32_t n = res ? i - rqc : i;
        lists |= src << (4 * n + (res ? 16 : 0));
      }
    }
  }
  // the leader-state rows of the cluster's ls_present node (at most one)
  const bool lsp = active && ((fl >> 14) & 1);
  const uint32_t lspm = (uint32_t)(__ballot(lsp) >> bl) & cmask;
  bad = bad || __popc(lspm) > 1;
  if (lsp) {
#pragma unroll
    for (int p = 0; p < 2 * N; ++p) myrows[p] = (int32_t)hp[(HF_NEXT + p) * N];
  }
  // a cluster outside the model from the start bails at t0 with its state untouched
  const bool bad0 = cluster_any(bad);
  if (active && bad0 && k == 0) {
    const uint32_t i = atomicAdd(S.nbail, 1u);
    S.bail_c[i] = c;
    S.bail_t[i] = t0;
  }
  const bool wb = active && !bad0;          // state to write back at the end
  bool run = wb;                            // the cluster still runs here (not bailed)
  __builtin_amdgcn_wave_barrier();

  RS_PHASE(9);
  const uint32_t tend = t0 + nt, d = S.dmin;
  uint32_t tnext = t0;
  for (;;) {
    const bool liv0 = run && !((fl >> 10) & 7);
    uint32_t t = max(tnext, cluster_min(liv0 ? min(deadline, min(rqa, rsa)) : INF));
    t = t < tend ? t : tend;
    const bool on = run && t < tend;
    if (!__ballot(on)) break;
#ifdef RS_WAVELOG
    ++wl_trips;
#endif
    RS_PHASE(8);
    const bool live = on && !((fl >> 10) & 7);
    const uint32_t role = fl & 3;
    const bool rqok = live && rqa <= t, rsok = live && rsa <= t;
    const bool ev = rqok || rsok || (live && t >= deadline);
    // ------------------------------------------------ decide (no state changes yet)
    // The EVENT draw: for the alts!! choice when both queues are ready, and for the next election
    // timeout of a node that is not leader after the event (a follower's append-entries, a
    // leader's append-entries of a newer term; core.clj:171-174).
    uint4 w = make_uint4(0, 0, 0, 0);
    if (ev && (rqok || role != RAFT_LEADER)) w = event_draw(g, id, t, S);
    const int which = rqok && rsok ? (int)(w.x & 1) : rqok ? 0 : rsok ? 1 : -1;
    const int s = which >= 0 ? (int)((lists >> (which ? 16 : 0)) & 15) - 1 : 0;
    uint4 m = make_uint4(0, 0, 0, 0);
    if (which >= 0) m = *reinterpret_cast<const uint4*>(cell_in(s));
    const uint32_t mterm = m.y, ma = m.z, mb = m.w & 0xFFFFFFu, hdr = m.w >> 24;
    const uint32_t type = hdr & 7, flag = (hdr >> 7) & 1, src = (uint32_t)s + 1;
    const uint32_t keys = mk >> 16;
    bool ok = true;
    if (ev) {
      if (which < 0) {
        // heartbeat: leader with full leader-state, no LazySeq log, commit within the log (the
        // IOOBE/NPE/CCE checks of append-entries-rpc pass), an empty broadcast (every peer's
        // prev-index at or past the log's end) and every outgoing cell free. The row and cell
        // reads are independent (all in flight at once).
        ok = role == RAFT_LEADER && ((fl >> 14) & 1) && (keys & peers) == peers &&
             !((fl >> 13) & 1) && commit <= len;
#pragma unroll
        for (int j = 0; j < N; ++j) {
          if (j == k) continue;
          const int32_t nx = myrows[j];
          const uint32_t prev = nx - 1 > 0 ? (uint32_t)(nx - 1) : 0u;
          ok = ok && prev >= len && prev < (1u << 24) && cell_out(j)[3] == 0;
        }
      } else if (which == 0) {
        // append-entries with prev-index 0 and no entries (consistent without a log read); a
        // newer term sets commit = log_len, which applies nothing when commit >= log_len
        ok = type == RAFT_MSG_APPEND_ENTRIES && mb == 0 && (mterm < term || len <= commit) &&
             cell_out(s)[3] == 0;
      } else {
        // append-response of no newer term to the row owner; a success response is checker
        // work once the log passes the hwm (P4)
        ok = type == RAFT_MSG_APPEND_RESPONSE && ((fl >> 14) & 1) && mterm <= term &&
             (flag ? !(fl & SF_ACKBAD) : ((keys >> src) & 1) != 0);
      }
    }
    if (cluster_any(ev && !ok)) {           // bail before this tick: the general kernel runs it
      if (on && k == 0) {
        const uint32_t i = atomicAdd(S.nbail, 1u);
        S.bail_c[i] = c;
        S.bail_t[i] = t;
      }
      run = false;
      continue;
    }
    RS_PHASE(3);
    // ------------------------------------------------ run the event
    uint32_t sent = 0;             // receivers (bits 1..N); bit 31: replies (RES queues)
    if (ev) {
      uint32_t evc, tsrc = 0, tterm = 0;
      if (which >= 0) {            // pop the head: free the cell, next head's arrival
        cell_in(s)[3] = 0;
        const int sh = which ? 16 : 0;
        const uint32_t rest = ((lists >> sh) & 0xFFFFu) >> 4;
        lists = (lists & ~(0xFFFFu << sh)) | rest << sh;
        const uint32_t same = fl & (which ? SF_RESSAME : SF_REQSAME);
        const uint32_t na = !rest ? INF : same ? (which ? rsa : rqa) : cell_in((int)(rest & 15) - 1)[0];
        if (which) rsa = na;
        else rqa = na;
        tsrc = src;
        tterm = mterm;
      }
      if (which < 0) {             // heartbeat-handler: append-entries to every peer
        evc = 7;
#pragma unroll
        for (int j = 0; j < N; ++j) {
          if (j == k) continue;
          const int32_t nx = myrows[j];
          const uint32_t pv = nx - 1 > 0 ? (uint32_t)(nx - 1) : 0u;
          *reinterpret_cast<uint4*>(cell_out(j)) =
              make_uint4(t + d, term, commit, pv | (RAFT_MSG_APPEND_ENTRIES | id << 3) << 24);
        }
        sent = peers;
        lctr_add(lctr, RAFT_CTR_SENT, N - 1);
      } else if (which == 0) {     // append-entries-handler
        evc = RAFT_MSG_APPEND_ENTRIES;
        uint32_t rh = RAFT_MSG_APPEND_RESPONSE | id << 3, ra = 0;
        const uint32_t rterm = term;
        if (mterm >= term) {
          rh |= 1u << 7;
          ra = ma;
          commit = len;                                   // apply-entries! (nothing applied)
          term = mterm;
          // role :follwer, voted-for and votes cleared, leader-id = src, LazySeq flag cleared
          fl = (fl & ~(3u | 15u << 2 | 15u << 6 | 1u << 13)) | RAFT_FOLLWER | src << 6;
          mk &= 0xFFFF0000u;
        }
        *reinterpret_cast<uint4*>(cell_out(s)) = make_uint4(t + d, rterm, ra, rh << 24);
        sent = 1u << src | 1u << 31;
        lctr_add(lctr, RAFT_CTR_SENT, 1);
      } else {                     // append-response-handler
        evc = RAFT_MSG_APPEND_RESPONSE;
        if (flag) {
          mk |= 1u << (16 + src);
          myrows[s] = (int32_t)mb;
          myrows[N + s] = (int32_t)ma;
        } else {
          myrows[s] -= 1;
        }
      }
      const uint32_t r2 = fl & 3;
      deadline = r2 == RAFT_LEADER ? t + S.hb : t + S.el_base + __umulhi(w.y, S.el_span);
      trace = trace_event(trace, t, evc, tsrc, tterm, r2, term, 0);
      lctr_add(lctr, RAFT_CTR_EV_RV + evc - 1, 1);
    }
    RS_PHASE(4);
    // ------------------------------------------------ P2: deliveries, in sender id order
    if (__ballot(sent != 0)) {
      uint32_t inm = 0, rep = 0;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const uint32_t sm = __shfl(sent, bl + j);
        inm |= ((sm >> id) & 1u) << j;
        rep |= (sm >> 31) << j;
      }
      if (!on) inm = 0;              // padding lanes alias cluster 0's lanes
      while (inm) {
        const int j = __builtin_ctz(inm);
        inm &= inm - 1;
        const int sh = ((rep >> j) & 1) ? 16 : 0;
        const uint32_t q = (lists >> sh) & 0xFFFFu;
        const uint32_t cnt = q ? (35u - __clz(q)) >> 2 : 0u;     // nibbles in use
        if ((fl >> 10) & 7) {
          lctr_add(lctr, RAFT_CTR_TO_HALTED, 1);
          cell_in(j)[3] = 0;
        } else if (cnt >= S.Q) {
          lctr_add(lctr, RAFT_CTR_OVERFLOW, 1);
          cell_in(j)[3] = 0;
        } else {
          lists |= (uint32_t)(j + 1) << (sh + 4 * cnt);
          const uint32_t sb = sh ? SF_RESSAME : SF_REQSAME;
          if (!cnt) {
            fl |= sb;
            if (sh) rsa = t + d;
            else rqa = t + d;
          } else if ((sh ? rsa : rqa) != t + d) {
            fl &= ~sb;
          }
          lctr_add(lctr, RAFT_CTR_DELIVERED, 1);
        }
      }
    }
    RS_PHASE(5);
    // ------------------------------------------------ the leader's append-response drain
    // Ticks at which the cluster's only event is an append-response at its row owner (the leader)
    // run here, one response per tick as above, without the cluster's trip: up to the cluster's
    // next other event E (every other node's next event and the leader's REQ head), the leader's
    // heartbeat tick, or a response outside the model (the trip then decides it).
    const bool drl = on && lsp && (fl & (3u | 7u << 10)) == RAFT_LEADER && (lists >> 16) != 0;
    if (__ballot(drl)) {
      const uint32_t oth = !on || ((fl >> 10) & 7) ? INF : drl ? rqa : min(deadline, min(rqa, rsa));
      const uint32_t E = min(cluster_min(oth), tend);
      uint32_t tl = t;
      if (drl) {
        for (;;) {
          const uint32_t tau = max(min(rsa, deadline), tl + 1);
          if (tau >= E || rsa > tau) break;
          const int hs = (int)((lists >> 16) & 15) - 1;
          const uint4 x = *reinterpret_cast<const uint4*>(cell_in(hs));
          const uint32_t xh = x.w >> 24, xf = (xh >> 7) & 1, xs = (uint32_t)hs + 1;
          if ((xh & 7) != RAFT_MSG_APPEND_RESPONSE || x.y > term ||
              (xf ? (fl & SF_ACKBAD) != 0 : ((mk >> (16 + xs)) & 1) == 0))
            break;
          cell_in(hs)[3] = 0;
          const uint32_t rest = (lists >> 20) & 0xFFFu;
          lists = (lists & 0xFFFFu) | rest << 16;
          rsa = !rest ? INF : (fl & SF_RESSAME) ? rsa : cell_in((int)(rest & 15) - 1)[0];
          if (xf) {
            mk |= 1u << (16 + xs);
            myrows[hs] = (int32_t)(x.w & 0xFFFFFFu);
            myrows[N + hs] = (int32_t)x.z;
          } else {
            myrows[hs] -= 1;
          }
          deadline = tau + S.hb;
          trace = trace_event(trace, tau, RAFT_MSG_APPEND_RESPONSE, xs, x.y, RAFT_LEADER, term, 0);
          lctr_add(lctr, RAFT_CTR_EV_AR, 1);
          tl = tau;
        }
      }
      if (lspm) t = max(t, __shfl(tl, bl + __builtin_ctz(lspm)));   // the cluster takes its clock
    }
    RS_PHASE(6);
    tnext = t + 1;
  }
#ifdef RS_WAVELOG
  if (lane == 0 && S.wavelog) {
    const uint64_t wl_end = wall_clock64();
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    uint4* rec = reinterpret_cast<uint4*>(S.wavelog + (size_t)wave * 32);
    rec[0] = make_uint4((uint32_t)wl_start, (uint32_t)(wl_start >> 32), (uint32_t)wl_end,
                        (uint32_t)(wl_end >> 32));
    rec[1] = make_uint4(wl_trips, hw, xcc, 0);
    rec[2] = make_uint4(wl_ph[0], wl_ph[1], wl_ph[2], wl_ph[3]);
    rec[3] = make_uint4(wl_ph[4], wl_ph[5], wl_ph[6], wl_ph[7]);
    rec[4] = make_uint4(wl_ph[8], wl_ph[9], wl_ph[10], wl_ph[11]);
    rec[5] = make_uint4(0, 0, 0, 0);
  }
#endif

  // ------------------------------------------------------------------ write back
  if (S.shist) {
    // packing key for the next launch (as the general kernel's, keys of running clusters only:
    // a bailed cluster's key comes from the catch-up launch)
    const uint32_t me = wb && !((fl >> 10) & 7) ? min(deadline, min(rqa, rsa)) : INF;
    const uint32_t cm = cluster_min(me);
    const bool head = wb && run && k == 0;
    const uint32_t key = head ? sched_bucket(cm, tend) : INF;
    if (head) S.skey[c] = key;
    const uint32_t kmin = wave_min(key), kmax = ~wave_min(head ? ~key : ~0u);
    const uint32_t heads = (uint32_t)__popcll(__ballot(head));
    if (kmin == kmax) {
      if (lane == 0 && kmin != INF) atomicAdd(&S.shist[kmin], heads);
    } else if (head) {
      atomicAdd(&S.shist[key], 1u);
    }
  }
  if (wb) {
    hp[HF_FLAGS * N] = fl & 0x7FFFu;
    hp[HF_MASKS * N] = mk;
    hp[HF_TERM * N] = term; hp[HF_COMMIT * N] = commit; hp[HF_DEADLINE * N] = deadline;
    hp[HF_TRACE_LO * N] = (uint32_t)trace; hp[HF_TRACE_HI * N] = (uint32_t)(trace >> 32);
    // queues back to the rings, heads at slot 0; tail = the last message's arrival (0 if empty)
    uint32_t cnt[2] = {0, 0}, tail[2] = {0, 0};
#pragma unroll
    for (int which = 0; which < 2; ++which) {
      uint32_t q = (lists >> (which ? 16 : 0)) & 0xFFFFu;
      uint32_t* qb = qslots(S, gi, which);
      const size_t qs = qstride(S, which);
      for (uint32_t i = 0; q; ++i, q >>= 4) {
        const uint32_t sj = (q & 15) - 1;
        const uint4 x = *reinterpret_cast<const uint4*>(cell_in((int)sj));
        uint4* dp = reinterpret_cast<uint4*>(qb + i * qs);
        dp[0] = make_uint4(x.x, x.w >> 24, x.y, x.z);
        dp[1] = make_uint4(x.w & 0xFFFFFFu, 0, 0, 0);
        cnt[which] = i + 1;
        tail[which] = x.x;
      }
    }
    hp[HF_QMETA * N] = pack_qmeta(0, cnt[0], 0, cnt[1]);
    hp[HF_REQ_ARR * N] = rqa; hp[HF_RES_ARR * N] = rsa;
    hp[HF_REQ_TAIL * N] = tail[0]; hp[HF_RES_TAIL * N] = tail[1];
    if (lsp) {
#pragma unroll
      for (int p = 0; p < 2 * N; ++p) hp[(HF_NEXT + p) * N] = (uint32_t)myrows[p];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  unsigned long long* const ctr = S.ctr + (size_t)(wave % CTR_COPIES) * CTR_STRIDE;
  if (lane < RAFT_CTR_COUNT) {
    const uint32_t v = lctr[lane];
    if (v) atomicAdd(&ctr[lane], (unsigned long long)v);
  }
}

// ---------------------------------------------------------------------------------------------
// Lane-per-cluster form of the steady kernel. One lane runs one whole cluster: the leader and its
// N-1 followers are named registers (follower slot j is the j-th non-leader node in id order), the
// messages in flight are registers too (a follower holds at most one append-entries from the
// leader; the leader's append-responses all share one arrival and pop in sender id order), and no
// event needs another lane: no shuffles, ballots or LDS inside the tick loop, and a wave runs 64
// clusters instead of 12. The events and their order are the steady kernel's (heartbeat-handler,
// append-entries-handler and append-response-handler of core.clj:105-164, SIM_SPEC.md §4), and any
// cluster outside this narrower model (no single leader with full leader-state, a halted node, a
// message of another shape, a follower timing out, a response of a newer term, ...) is bailed
// before that tick exactly as above, so results are the general kernel's for any state.
// Grid: 256-thread workgroups, one cluster per thread, slots in the packing's order (clusters with
// the same next event share a wave, so lanes take the same branch on every trip).
constexpr int LANE_WG = 256;
// clusters per wave: 64, or 32 (half the lanes idle, twice the waves: two per SIMD hide each
// other's dependency latency)
#ifndef RS_LANE_CPW
#define RS_LANE_CPW 64
#endif
constexpr int LANE_CPW = RS_LANE_CPW;
constexpr int LANE_CPB = LANE_WG / 64 * LANE_CPW;   // clusters per workgroup
#ifndef RS_STEADY_LANE
#define RS_STEADY_LANE 1
#endif
#ifndef RS_LANE_DRAIN
#define RS_LANE_DRAIN 1
#endif
#ifndef RS_LANE_ROUND
#define RS_LANE_ROUND 1
#endif

// v = vals[k] for a runtime k < N, as masks (a select chain over an array is turned back into an
// indexed load from memory by the compiler; this keeps the array in registers)
template <int N>
__device__ __forceinline__ uint32_t pick(const uint32_t (&vals)[N], uint32_t k) {
  uint32_t v = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) v |= vals[i] & (0u - (uint32_t)(k == (uint32_t)i));
  return v;
}
// a ? x : y without a select the compiler could fold into an indexed load
__device__ __forceinline__ uint32_t msel(bool a, uint32_t x, uint32_t y) {
  const uint32_t m = 0u - (uint32_t)a;
  return (x & m) | (y & ~m);
}

template <int N>
__global__ void __launch_bounds__(LANE_WG) steady_lane_kernel(DevSim S, uint32_t t0, uint32_t nt) {
  static_assert(N >= 2 && N <= 5, "follower masks and the response queue fit four followers");
  constexpr int F = N - 1;
  constexpr uint32_t HB = hot_block_words(N), CLW = hot_cl_off(N);
  constexpr int NW4 = (int)(CLW + 4) / 4;          // uint4s up to and including the checker hwm
  __shared__ uint32_t sctr[4];
  const uint32_t nslots = S.perm ? *S.nslots : S.C;
  if (blockIdx.x == 0 && threadIdx.x == 0) *S.nbail_zero = 0;   // the next launch's bail counter
  if (blockIdx.x * LANE_CPB >= nslots) return;                  // workgroup-uniform
  if (threadIdx.x < 4) sctr[threadIdx.x] = 0;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t slot = blockIdx.x * LANE_CPB + threadIdx.x / 64 * LANE_CPW + lane;
  const uint32_t c0 = lane < (uint32_t)LANE_CPW && slot < nslots ? (S.perm ? S.perm[slot] : slot)
                                                                 : INF;
  const bool active = c0 != INF;
  const uint32_t c = active ? c0 : 0u;
  const uint32_t g = S.goff + c;
  uint32_t* const blk = S.hot + (size_t)c * HB;
#ifdef RS_WAVELOG   // diagnostic build: per-wave timeline (scripts/lane_timeline.py)
  const uint64_t wl_start = wall_clock64();
  uint32_t wl_trips = 0, wl_first = 0, wl_ph[6] = {0, 0, 0, 0, 0, 0};
  uint64_t wl_loop = 0, wl_ts = 0;
#define RS_LPH(i)                                         \
  do {                                                    \
    const uint64_t now_ = __builtin_amdgcn_s_memtime();   \
    wl_ph[i] += (uint32_t)(now_ - wl_ts);                 \
    wl_ts = now_;                                         \
  } while (0)
#else
#define RS_LPH(i) do {} while (0)
#endif

  // ------------------------------------------- load: fields FLAGS..RES_TAIL, TRACE, checker hwm
  uint32_t w[NW4 * 4];
#pragma unroll
  for (int i = 0; i < NW4 * 4; ++i) w[i] = 0;
  if (active) {
#pragma unroll
    for (int i = 0; i < NW4; ++i) {
      const int lo = 4 * i, hi = 4 * i + 3;
      const bool need = lo < (int)(HF_ABASE * N) ||
                        (hi >= (int)(HF_TRACE_LO * N) && lo < (int)(HF_NEXT * N)) ||
                        (lo <= (int)CLW && hi >= (int)CLW);
      if (need) {
        const uint4 x = reinterpret_cast<const uint4*>(blk)[i];
        w[lo] = x.x; w[lo + 1] = x.y; w[lo + 2] = x.z; w[lo + 3] = x.w;
      }
    }
  }
  auto field = [&](int f, uint32_t (&out)[N]) {
#pragma unroll
    for (int k = 0; k < N; ++k) out[k] = w[f * N + k];
  };
  uint32_t nfl[N], nqm[N];
  field(HF_FLAGS, nfl);
  field(HF_QMETA, nqm);
  // exactly one leader; every node running; only the leader has leader-state
  uint32_t L = 0, nlead = 0, badn = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const uint32_t f = nfl[k];
    const bool lead = (f & 3) == RAFT_LEADER;
    L = lead ? (uint32_t)k : L;
    nlead += lead;
    badn |= ((f >> 10) & 7) | (lead != (((f >> 14) & 1) != 0));
  }
  bool bad = !active || nlead != 1 || badn != 0 || S.Q < (uint32_t)F;
  const uint32_t Lid = L + 1;
  // follower slot j is node j (j < L) or j + 1 (j >= L)
  auto fsel = [&](const uint32_t (&v)[N], int j) { return msel((uint32_t)j >= L, v[j + 1], v[j]); };
  auto fk = [&](int j) { return (uint32_t)j + ((uint32_t)j >= L ? 1u : 0u); };

  uint32_t tmp[N];
  // leader registers
  const uint32_t Lfl = pick<N>(nfl, L);
  field(HF_MASKS, tmp); uint32_t Lmk = pick<N>(tmp, L);
  uint32_t fmk[F];
#pragma unroll
  for (int j = 0; j < F; ++j) fmk[j] = fsel(tmp, j);
  field(HF_TERM, tmp); const uint32_t Lterm = pick<N>(tmp, L);
  uint32_t fterm[F];
#pragma unroll
  for (int j = 0; j < F; ++j) fterm[j] = fsel(tmp, j);
  field(HF_COMMIT, tmp); const uint32_t Lcommit = pick<N>(tmp, L);
  uint32_t fcommit[F];
#pragma unroll
  for (int j = 0; j < F; ++j) fcommit[j] = fsel(tmp, j);
  field(HF_LEN, tmp); const uint32_t Llen = pick<N>(tmp, L);
  uint32_t flen[F];
#pragma unroll
  for (int j = 0; j < F; ++j) flen[j] = fsel(tmp, j);
  field(HF_DEADLINE, tmp); uint32_t Ldl = pick<N>(tmp, L);
  uint32_t fdl[F];
#pragma unroll
  for (int j = 0; j < F; ++j) fdl[j] = fsel(tmp, j);
  uint32_t tlo[N], thi[N];
  field(HF_TRACE_LO, tlo);
  field(HF_TRACE_HI, thi);
  uint64_t Ltr = (uint64_t)pick<N>(thi, L) << 32 | pick<N>(tlo, L);
  uint64_t ftr[F];
  uint32_t ffl[F];
#pragma unroll
  for (int j = 0; j < F; ++j) {
    ftr[j] = (uint64_t)fsel(thi, j) << 32 | fsel(tlo, j);
    ffl[j] = fsel(nfl, j);
  }
  // the leader's rows for its followers: next_index / match_index of peer id fk(j) + 1
  int32_t nx[F], mt[F];
#pragma unroll
  for (int j = 0; j < F; ++j) {
    nx[j] = active ? (int32_t)blk[(HF_NEXT + fk(j)) * N + L] : 0;
    mt[j] = active ? (int32_t)blk[(HF_NEXT + N + fk(j)) * N + L] : 0;
  }
  int32_t nx0[F], mt0[F];                     // as loaded: unchanged words are not stored back
#pragma unroll
  for (int j = 0; j < F; ++j) {
    nx0[j] = nx[j];
    mt0[j] = mt[j];
  }
  const bool ackbad = Llen > w[CLW];          // a success response would be checker work (P4)
  const uint32_t Lkeys = Lmk >> 16;
  // heartbeats need full leader-state, no LazySeq log and commit within the log
  // (append-entries-rpc's IOOBE/NPE/CCE checks, core.clj:56-67): constant over the launch
  bad = bad || (Lkeys & (((1u << (N + 1)) - 1) & ~1u & ~(1u << Lid))) !=
                   (((1u << (N + 1)) - 1) & ~1u & ~(1u << Lid)) ||
        ((Lfl >> 13) & 1) || Lcommit > Llen;

  // ---------------------------------------------------------------- queued messages
  uint32_t qmask = 0, rmask = 0, resA = INF;
  uint32_t qA[F], qT[F], qa[F], qb[F], rT[F], rA[F], rB[F], rH[F];
#pragma unroll
  for (int j = 0; j < F; ++j) {
    qA[j] = INF; qT[j] = qa[j] = qb[j] = 0;
    rT[j] = rA[j] = rB[j] = rH[j] = 0;
  }
  if (!bad) {
    const uint32_t Lqm = pick<N>(nqm, L);
    bad = (Lqm >> 4) & 31;                                   // the leader's REQ queue is empty
    const uint32_t rsh = (Lqm >> 9) & 15, rsc = (Lqm >> 13) & 31;
#pragma unroll
    for (int j = 0; j < F; ++j) {
      const uint32_t qm = fsel(nqm, j);
      const uint32_t rqh = qm & 15, rqc = (qm >> 4) & 31;
      bad = bad || rqc > 1 || ((qm >> 13) & 31) != 0;       // <= 1 request, no responses
      if (!bad && rqc) {                                    // the leader's append-entries
        const uint4* mp = reinterpret_cast<const uint4*>(qslots(S, c * N + fk(j), 0) +
                                                         rqh * qstride(S, 0));
        const uint4 m0 = mp[0], m1 = mp[1];
        bad = m0.y != (RAFT_MSG_APPEND_ENTRIES | Lid << 3) || m1.y || m1.z || m1.w;
        qmask |= 1u << j;
        qA[j] = m0.x; qT[j] = m0.z; qa[j] = m0.w; qb[j] = m1.x;
      }
    }
    bad = bad || rsc > (uint32_t)F;
    uint32_t last = 0;
    for (uint32_t i = 0; i < rsc && !bad; ++i) {            // append-responses, sender order
      const uint4* mp = reinterpret_cast<const uint4*>(qslots(S, c * N + L, 1) +
                                                       wrapq(rsh + i, S.Q) * qstride(S, 1));
      const uint4 m0 = mp[0], m1 = mp[1];
      const uint32_t hdr = m0.y, src = (hdr >> 3) & 15;
      bad = (hdr & 7) != RAFT_MSG_APPEND_RESPONSE || (hdr >> 8) || m1.y || m1.z || m1.w ||
            src <= last || src > (uint32_t)N || src == Lid || (i && m0.x != resA);
      last = src;
      resA = m0.x;
      const uint32_t j = src - 1 - (src > Lid ? 1u : 0u);
      rmask |= 1u << j;
#pragma unroll
      for (int jj = 0; jj < F; ++jj) {
        if ((uint32_t)jj == j) {
          rT[jj] = m0.z; rA[jj] = m0.w; rB[jj] = m1.x; rH[jj] = (hdr >> 7) & 1;
        }
      }
    }
    if (!rmask) resA = INF;
  }
  if (active && bad) {                      // outside the model from the start: bail at t0
    const uint32_t i = atomicAdd(S.nbail, 1u);
    S.bail_c[i] = c;
    S.bail_t[i] = t0;
  }
  const bool wb = active && !bad;
  bool run = wb;

  // ---------------------------------------------------------------- the cluster's ticks
  const uint32_t tend = t0 + nt, d = S.dmin;
  uint32_t tn = t0, nhb = 0, nae = 0, nar = 0;
  auto next_event = [&]() {
    uint32_t m = min(Ldl, resA);
#pragma unroll
    for (int j = 0; j < F; ++j) m = min(m, min(fdl[j], qA[j]));
    return m;
  };
#ifdef RS_WAVELOG
  wl_loop = wall_clock64();
  wl_ts = __builtin_amdgcn_s_memtime();
#endif
  for (;;) {
    const uint32_t t = max(tn, next_event());
    const bool on = run && t < tend;
    if (!__builtin_amdgcn_ballot_w64(on)) break;
#ifdef RS_WAVELOG
    if (!wl_trips) wl_first = (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(on));
    ++wl_trips;
#endif
    RS_LPH(0);
    if (!on) continue;
    // ------------------------------------------------ decide on the pre-tick state
    const bool lres = rmask != 0 && resA <= t;               // a message beats the deadline
    const bool lhb = !lres && Ldl <= t;
    uint32_t fae = 0, fto = 0;
#pragma unroll
    for (int j = 0; j < F; ++j) {
      const bool a = qA[j] <= t;
      fae |= (uint32_t)a << j;
      fto |= (uint32_t)(!a && fdl[j] <= t) << j;
    }
    bool bail = fto != 0;                                    // a follower's election timeout
    if (lhb) {
      bail = bail || qmask != 0;                             // a follower still holds one
#pragma unroll
      for (int j = 0; j < F; ++j) {
        const uint32_t pv = nx[j] - 1 > 0 ? (uint32_t)(nx[j] - 1) : 0u;
        bail = bail || pv < Llen || pv >= (1u << 24);        // entries to ship
      }
    }
    const int hs = __builtin_ctz(rmask | (1u << F));
    uint32_t xT = 0, xA = 0, xB = 0, xH = 0;
#pragma unroll
    for (int j = 0; j < F; ++j) {
      if (j == hs) {
        xT = rT[j]; xA = rA[j]; xB = rB[j]; xH = rH[j];
      }
    }
    const uint32_t xid = (uint32_t)hs + 1 + ((uint32_t)hs >= L ? 1u : 0u);
    if (lres)
      bail = bail || xT > Lterm || (xH ? ackbad : ((Lmk >> (16 + xid)) & 1) == 0);
    if (fae) {
      bail = bail || rmask != 0;                             // responses of two ticks
#pragma unroll
      for (int j = 0; j < F; ++j)
        if ((fae >> j) & 1)
          bail = bail || qb[j] != 0 || !(qT[j] < fterm[j] || flen[j] <= fcommit[j]);
    }
    RS_LPH(1);
    if (bail) {                              // the general kernel runs this tick
      const uint32_t i = atomicAdd(S.nbail, 1u);
      S.bail_c[i] = c;
      S.bail_t[i] = t;
      run = false;
      continue;
    }
    // ------------------------------------------------ run
    uint32_t tl = t;                         // the last tick run (a round or a drain runs more)
    bool round = false;
    if (lhb) {                               // heartbeat-handler: empty append-entries to all
#pragma unroll
      for (int j = 0; j < F; ++j) {
        qA[j] = t + d; qT[j] = Lterm; qa[j] = Lcommit;
        qb[j] = nx[j] - 1 > 0 ? (uint32_t)(nx[j] - 1) : 0u;
      }
      qmask = (1u << F) - 1;
      Ldl = t + S.hb;
      Ltr = trace_event(Ltr, t, 7, 0, 0, RAFT_LEADER, Lterm, 0);
      ++nhb;
#if RS_LANE_ROUND
      // The whole heartbeat round in this trip when nothing else can happen before its last
      // response: every follower takes the append-entries at t + d (no follower deadline before
      // it; the handler's checks pass), the followers' re-armed deadlines (>= t + d + el_base) and
      // the leader's (t + hb) fall after the responses at t + 2d .. t + 2d + F - 1, and the round
      // ends before the launch does (and no older response is still queued). The responses then
      // run as a drain (which stops at one outside the model; the next trip decides it).
      round = rmask == 0 && S.hb >= 2 * d + F && S.el_base >= d + F && tend - t > 2 * d + F;
#pragma unroll
      for (int j = 0; j < F; ++j)
        round = round && fdl[j] >= t + d && qb[j] == 0 && (Lterm < fterm[j] || flen[j] <= fcommit[j]);
#endif
    }
    RS_LPH(2);
    if (fae || round) {                      // append-entries-handler at each follower
      // every follower's handler is computed and kept where it ran: the four Philox draws and
      // trace hashes are independent chains the compiler interleaves (in a round every follower
      // answers the same heartbeat on the same tick)
      const uint32_t ta = round ? t + d : t;
      const uint32_t fa = round ? (1u << F) - 1 : fae;
#pragma unroll
      for (int j = 0; j < F; ++j) {
        const bool run_j = (fa >> j) & 1;
        const uint32_t fid = fk(j) + 1;
        const uint4 wd = event_draw(g, fid, ta, S);
        const uint32_t mterm = qT[j], rterm = fterm[j];
        const bool ok = mterm >= fterm[j];
        const uint32_t nfl2 = ok ? (ffl[j] & ~(3u | 15u << 2 | 15u << 6 | 1u << 13)) | RAFT_FOLLWER |
                                       Lid << 6
                                 : ffl[j];
        const uint32_t nterm = ok ? mterm : fterm[j];
        const uint64_t ntr = trace_event(ftr[j], ta, RAFT_MSG_APPEND_ENTRIES, Lid, mterm, nfl2 & 3,
                                         nterm, 0);
        if (run_j) {
          if (ok) {
            fcommit[j] = flen[j];                            // apply-entries! (nothing applied)
            fmk[j] &= 0xFFFF0000u;
          }
          fterm[j] = nterm;
          ffl[j] = nfl2;
          // the response: to the leader's RES queue, in sender id order
          rT[j] = rterm; rA[j] = ok ? qa[j] : 0u; rB[j] = 0; rH[j] = ok;
          qA[j] = INF;
          fdl[j] = ta + S.el_base + __umulhi(wd.y, S.el_span);
          ftr[j] = ntr;
        }
      }
      qmask &= ~fa;
      rmask = fa;
      resA = ta + d;
      nae += __popc(fa);
      tl = ta;
    }
    RS_LPH(3);
    if (lres || round) {                     // append-response-handler, heads in sender order
      // from tick tau0 one response per tick while nothing else in the cluster is due (the
      // followers' next events and the launch end; the leader's own deadline moves past each):
      // the decided response at t, or a round's responses from t + 2d. A response outside the
      // model ends the run of responses and the next trip decides it.
      const uint32_t tau0 = round ? t + 2 * d : t;
      uint32_t E = tend;
#pragma unroll
      for (int j = 0; j < F; ++j) E = min(E, min(fdl[j], qA[j]));
      if (lres) E = max(E, t + 1);           // decided: the first response runs
      if (!RS_LANE_DRAIN) E = min(E, tau0 + 1);
      for (uint32_t tau = tau0; rmask && tau < E; ++tau) {
        const int h2 = __builtin_ctz(rmask);
        uint32_t yT = 0, yA = 0, yB = 0, yH = 0;
#pragma unroll
        for (int j = 0; j < F; ++j) {
          if (j == h2) {
            yT = rT[j]; yA = rA[j]; yB = rB[j]; yH = rH[j];
          }
        }
        const uint32_t yid = (uint32_t)h2 + 1 + ((uint32_t)h2 >= L ? 1u : 0u);
        if (yT > Lterm || (yH ? ackbad : ((Lmk >> (16 + yid)) & 1) == 0)) break;
        rmask &= rmask - 1;
        if (!rmask) resA = INF;
        Lmk |= yH << (16 + yid);
#pragma unroll
        for (int j = 0; j < F; ++j) {
          if (j == h2) {
            nx[j] = yH ? (int32_t)yB : nx[j] - 1;
            mt[j] = yH ? (int32_t)yA : mt[j];
          }
        }
        Ldl = tau + S.hb;
        Ltr = trace_event(Ltr, tau, RAFT_MSG_APPEND_RESPONSE, yid, yT, RAFT_LEADER, Lterm, 0);
        ++nar;
        tl = tau;
      }
    }
    RS_LPH(4);
    tn = tl + 1;
  }

#ifdef RS_WAVELOG
  const uint64_t wl_lend = wall_clock64();
  const uint32_t wl_events = nhb + nae + nar;
#endif
  // ---------------------------------------------------------------- write back
  if (S.shist) {
    // packing key for the next launch (bailed clusters get theirs from the catch-up launch); the
    // wave's clusters share a few keys: one histogram atomic per distinct key
    const bool kl = wb && run;
    const uint32_t key = kl ? sched_bucket(next_event(), tend) : INF;
    if (kl) S.skey[c] = key;
    uint64_t pend = __builtin_amdgcn_ballot_w64(kl);
    while (pend) {
      const uint32_t k = (uint32_t)__shfl((int)key, (int)__builtin_ctzll(pend));
      const uint64_t same = __builtin_amdgcn_ballot_w64(kl && key == k);
      if (lane == (uint32_t)__builtin_ctzll(pend)) atomicAdd(&S.shist[k], (uint32_t)__popcll(same));
      pend &= ~same;
    }
  }
  if (wb) {
    // every word of fields FLAGS..RES_TAIL and TRACE_LO/HI, from registers (LEN unchanged)
    constexpr int NV = 16;
    uint32_t v[NV][N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
      // node k is the leader (k == L) or follower slot k - 1 (k > L) / k (k < L)
      const bool isL = (uint32_t)k == L;
      const int jl = k > 0 ? k - 1 : 0, jh = k < F ? k : F - 1;
      const bool lo = (uint32_t)k > L;
      auto fv = [&](const uint32_t* x) { return msel(lo, x[jl], x[jh]); };
      const uint32_t fq = (qmask >> (lo ? jl : jh)) & 1;
      const uint32_t fqa = fv(qA);
      const uint64_t trf = (uint64_t)msel(lo, (uint32_t)(ftr[jl] >> 32), (uint32_t)(ftr[jh] >> 32)) << 32 |
                          msel(lo, (uint32_t)ftr[jl], (uint32_t)ftr[jh]);
      const uint64_t tr = isL ? Ltr : trf;
      v[HF_FLAGS][k] = isL ? Lfl : fv(ffl);
      v[HF_MASKS][k] = isL ? Lmk : fv(fmk);
      v[HF_TERM][k] = isL ? Lterm : fv(fterm);
      v[HF_COMMIT][k] = isL ? Lcommit : fv(fcommit);
      v[HF_LEN][k] = isL ? Llen : fv(flen);
      v[HF_DEADLINE][k] = isL ? Ldl : fv(fdl);
      v[HF_QMETA][k] = isL ? pack_qmeta(0, 0, 0, __popc(rmask)) : pack_qmeta(0, fq, 0, 0);
      v[HF_REQ_ARR][k] = isL ? INF : (fq ? fqa : INF);
      v[HF_RES_ARR][k] = isL ? resA : INF;
      v[HF_REQ_TAIL][k] = isL ? 0u : (fq ? fqa : 0u);
      v[HF_RES_TAIL][k] = isL ? (rmask ? resA : 0u) : 0u;
      v[HF_TRACE_LO][k] = (uint32_t)tr;
      v[HF_TRACE_HI][k] = (uint32_t)(tr >> 32);
    }
    auto live = [](int q) {
      return q < (int)(HF_ABASE * N) || (q >= (int)(HF_TRACE_LO * N) && q < (int)(HF_NEXT * N));
    };
    auto val = [&](int q) { return v[q / N][q % N]; };
    // Only words that changed are stored (in a heartbeat round the deadlines and trace hashes do;
    // flags, terms, masks, commits, queue words and rows come back unchanged): a lane's stores
    // each go to a different cluster's block, one L2 request per lane, and the write-back of the
    // whole grid at the launch end is bound by that request rate.
#pragma unroll
    for (int i = 0; i < (int)(HF_NEXT * N + 3) / 4; ++i) {
      const int lo = 4 * i;
      if (live(lo) && live(lo + 1) && live(lo + 2) && live(lo + 3)) {
        if (val(lo) != w[lo] || val(lo + 1) != w[lo + 1] || val(lo + 2) != w[lo + 2] ||
            val(lo + 3) != w[lo + 3])
          reinterpret_cast<uint4*>(blk)[i] =
              make_uint4(val(lo), val(lo + 1), val(lo + 2), val(lo + 3));
      } else {
#pragma unroll
        for (int q = lo; q < lo + 4; ++q)
          if (live(q) && val(q) != w[q]) blk[q] = val(q);
      }
    }
    // the leader's rows (node L): next / match of peer fk(j) + 1
#pragma unroll
    for (int j = 0; j < F; ++j) {
      if (nx[j] != nx0[j]) blk[(HF_NEXT + fk(j)) * N + L] = (uint32_t)nx[j];
      if (mt[j] != mt0[j]) blk[(HF_NEXT + N + fk(j)) * N + L] = (uint32_t)mt[j];
    }
    // queues back to the rings, heads at slot 0
#pragma unroll
    for (int j = 0; j < F; ++j) {
      if ((qmask >> j) & 1) {
        uint4* dp = reinterpret_cast<uint4*>(qslots(S, c * N + fk(j), 0));
        dp[0] = make_uint4(qA[j], RAFT_MSG_APPEND_ENTRIES | Lid << 3, qT[j], qa[j]);
        dp[1] = make_uint4(qb[j], 0, 0, 0);
      }
    }
    uint4* rp = reinterpret_cast<uint4*>(qslots(S, c * N + L, 1));
    uint32_t n = 0;
#pragma unroll
    for (int j = 0; j < F; ++j) {
      if ((rmask >> j) & 1) {
        const uint32_t sid = fk(j) + 1;
        uint4* dp = rp + 2 * n;
        dp[0] = make_uint4(resA, RAFT_MSG_APPEND_RESPONSE | sid << 3 | rH[j] << 7, rT[j], rA[j]);
        dp[1] = make_uint4(rB[j], 0, 0, 0);
        ++n;
      }
    }
  }
#ifdef RS_WAVELOG
  {
    const uint64_t wl_end = wall_clock64();
    const uint32_t emax = ~wave_min(~wl_events), emin = wave_min(wl_events);
    if ((threadIdx.x & 63) == 0 && S.wavelog) {
      uint32_t hw, xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      uint4* rec = reinterpret_cast<uint4*>(S.wavelog + (size_t)(blockIdx.x * 4 + threadIdx.x / 64) * 32);
      rec[0] = make_uint4((uint32_t)wl_start, (uint32_t)(wl_start >> 32), (uint32_t)wl_end,
                          (uint32_t)(wl_end >> 32));
      rec[1] = make_uint4(wl_trips, hw, xcc, wl_first);
      rec[2] = make_uint4((uint32_t)(wl_loop - wl_start), (uint32_t)(wl_lend - wl_start), emin, emax);
      rec[3] = make_uint4(wl_ph[0], wl_ph[1], wl_ph[2], wl_ph[3]);
      rec[4] = make_uint4(wl_ph[4], 0, 0, 0);
    }
  }
#endif
  // counters: heartbeats, append-entries, append-responses; every message is delivered
  if (nhb) atomicAdd(&sctr[0], nhb);
  if (nae) atomicAdd(&sctr[1], nae);
  if (nar) atomicAdd(&sctr[2], nar);
  __syncthreads();
  unsigned long long* const ctr = S.ctr + (size_t)(blockIdx.x % CTR_COPIES) * CTR_STRIDE;
  if (threadIdx.x < 5) {
    const uint32_t h = sctr[0], a = sctr[1], r = sctr[2];
    const uint32_t msgs = (uint32_t)F * h + a;
    const uint32_t x = threadIdx.x;
    const int idx = x == 0 ? RAFT_CTR_EV_HEARTBEAT : x == 1 ? RAFT_CTR_EV_AE
                  : x == 2 ? RAFT_CTR_EV_AR : x == 3 ? RAFT_CTR_SENT : RAFT_CTR_DELIVERED;
    const uint32_t v = x == 0 ? h : x == 1 ? a : x == 2 ? r : msgs;
    if (v) atomicAdd(&ctr[idx], (unsigned long long)v);
  }
}


hipError_t configure_steady() { return hipSuccess; }   // (no attributes needed)

// The steady kernel for N <= 5 (LITE launches; the caller checks). Grid: the packing's slots.
hipError_t launch_steady(const DevSim& S, uint32_t t0, uint32_t nt, hipStream_t st,
                         hipEvent_t ev0) {
  const uint32_t slots = S.perm ? sched_slots_bound(S.C, S.N) : S.C;
  if (RS_STEADY_LANE) {
    // a dense packing has exactly one slot per cluster: no grid past the clusters
    const uint32_t lslots = S.perm && !S.perm_dense ? slots : S.C;
    const dim3 grid((lslots + LANE_CPB - 1) / LANE_CPB);
    switch (S.N) {
#define RS_LANE(NN)                                                                             \
  case NN:                                                                                      \
    hipExtLaunchKernelGGL((steady_lane_kernel<NN>), grid, dim3(LANE_WG), 0, st, \
                          ev0, nullptr, 0, S, t0, nt);                                          \
    break;
      RS_LANE(2) RS_LANE(3) RS_LANE(4) RS_LANE(5)
#undef RS_LANE
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  switch (S.N) {
#define RS_STEADY(NN)                                                                            \
  case NN:                                                                                       \
    hipExtLaunchKernelGGL((steady_kernel<NN>),                                                   \
                          dim3((slots + steady_cpw<NN>() - 1) / steady_cpw<NN>()), dim3(64),     \
                          steady_lds_bytes<NN>(), st, ev0, nullptr, 0, S, t0, nt);              \
    break;
    RS_STEADY(2) RS_STEADY(3) RS_STEADY(4) RS_STEADY(5)
#undef RS_STEADY
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace rs

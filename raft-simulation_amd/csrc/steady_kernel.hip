// steady_kernel.hip — the steady-state kernel of LITE launches for gfx950 (MI355X).
//
// In a LITE launch (no client traffic, no faults, fixed delay: BASELINE config 2) a cluster that
// has elected its leader repeats one heartbeat round forever: the leader's heartbeat broadcasts an
// empty append-entries (heartbeat-handler, core.clj:162-164; append-entries-rpc 56-67), every
// follower answers it (append-entries-handler 105-123) and the leader takes the answers, one per
// tick (append-response-handler 141-149). This kernel runs exactly those events, bit for bit as
// the general tick body does (SIM_SPEC.md §4), and nothing else: a cluster about to run any other
// event (an election, a log entry, a halt, a message it cannot hold) is stopped ("bailed") before
// that tick with its state written back, and the same workgroup then runs it from that tick to
// the launch's end through the general tick body (tick_wave, CATCH form). Results are therefore
// identical to the general kernel's for any state; only the speed depends on how steady the
// clusters are. One dispatch per launch: there is no separate catch-up launch.
//
// Lane per cluster. One lane runs one whole cluster: the leader and its N-1 followers are named
// registers (follower slot j is the j-th non-leader node in id order, so deliveries in sender
// order are slot order), the messages in flight are registers too (a follower holds at most one
// append-entries from the leader; the leader's append-responses all share one arrival and pop in
// sender id order), and no event needs another lane: no shuffles, ballots or LDS inside the tick
// loop. A wave runs 64 clusters; C2's 65,536 clusters are 1,024 waves, one per SIMD.
//
// What a heartbeat round costs is its multiplies: Philox draws (the followers' election timers)
// and the trace hash. A follower's re-armed deadline (t + el_base + draw) is only compared with
// ticks before the next append-entries reaches it, and in steady state (el_base > hb) none is, so
// the draw is deferred: the deadline holds its lower bound t + el_base and a pending bit, and the
// draw is made when a tick at or past that bound is about to be decided, or at write-back — one
// draw per follower per launch instead of one per round, with identical results.
#include <hip/hip_ext.h>

#include "tick_wave.hpp"

namespace rs {

constexpr int LANE_WG = 256;                 // four waves, 64 clusters each

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

// The state image. A wave stages its 64 clusters' blocks (the first IMG_SLOTS 16-B chunks of each:
// four 128-B lines at N >= 4) in LDS: loads and stores then move whole lines, eight lines per wave
// instruction, where a lane reading its own cluster's block straight into registers touches 64
// lines per instruction (one per lane, the texture path's rate) -- the load phase's cost.
// Two halves: lines 0-1 of every cluster, then lines 2-3 (loaded only when some cluster of the
// wave has no steady certificate, device.hpp). In a half, chunk i of the wave's cluster l sits in
// slot i ^ (l & 15) of l's 256-B row: the LDS-DMA loads (global_load_lds: lane-linear destination)
// take the swizzle on their source addresses, and a lane reading chunk i of its own cluster, or
// writing it back, meets no bank conflict (the 16 lanes of a ds_read_b128 group have distinct
// l & 15).
constexpr int IMG_SLOTS = 32;                               // chunks per cluster, both halves
constexpr uint32_t IMG_HALF = 64 * 16 * 16;                 // 16 KiB: 64 clusters x 16 chunks
constexpr uint32_t IMG_WAVE = 2 * IMG_HALF;                 // 32 KiB per wave
__device__ __forceinline__ uint32_t img_off(uint32_t l, uint32_t i) {
  return (i >> 4) * IMG_HALF + l * 256u + 16u * ((i & 15u) ^ (l & 15u));
}
template <typename T>
__device__ __forceinline__ T* lds_at(char* img, uint32_t off) {
  return reinterpret_cast<T*>(img + off);
}

// Dynamic LDS of a steady workgroup: the four waves' state images. A wave that bailed clusters
// runs them through the general tick body with its own image as that body's LDS block (the image
// is dead once the write-back has read it): the waves of a workgroup never wait for each other.
template <int N>
constexpr size_t steady_lds_bytes() {
  static_assert(block_lds_bytes<N, false>() <= IMG_WAVE, "the catch-up block fits a wave's image");
  return 4 * (size_t)IMG_WAVE;
}

// M2^n and 1 + M2 + ... + M2^(n-1) mod 2^64 (the trace hash's multiplier per event, device.hpp)
template <int n>
__host__ __device__ constexpr uint64_t trace_pow() {
  uint64_t x = 1;
  for (int i = 0; i < n; ++i) x *= TRACE_M2;
  return x;
}
template <int n>
__host__ __device__ constexpr uint64_t trace_geo() {
  uint64_t s = 0, x = 1;
  for (int i = 0; i < n; ++i) {
    s += x;
    x *= TRACE_M2;
  }
  return s;
}

// A cluster at its fixed point, lane-resident: every follower took the leader's append-entries
// (flags, votes, term and commit are what another one sets again), every response succeeded (next /
// match / keys as another one sets them), the log is empty (a heartbeat ships nothing). With the
// followers' re-armed timers (>= t_ae + el_base) unable to fire before the next round's
// append-entries (el_base >= the round period P = 2d + F - 1 + hb) and the leader's responses all
// before its next heartbeat (hb >= 2d + F), every round is the last one shifted by P: only the
// ticks in the trace hashes change. Follower slot j is node j (j < L) or j + 1 (j >= L).
template <int N>
struct FixedPoint {
  static constexpr int F = N - 1;
  uint32_t L, Lid, Lterm, Lcommit;
  uint64_t Ltr, ftr[F];
  uint32_t Ldl, fdl[F], fpend;                       // fpend: followers whose draw is owed
  uint32_t qmask, qA[F], qT[F], qa[F], qb[F];        // append-entries in flight, per follower
  uint32_t rmask, resA, rT[F], rA[F], rB[F], rH[F];  // responses queued at the leader
  uint32_t nhb, nae, nar;

  __device__ __forceinline__ uint32_t fk(int j) const { return (uint32_t)j + ((uint32_t)j >= L ? 1u : 0u); }

  // The append-entries of the round with heartbeat th reach every follower at ta = th + d.
  __device__ __forceinline__ void append_entries(uint32_t ta, uint32_t d, uint32_t el_base) {
#pragma unroll
    for (int j = 0; j < F; ++j) {
      ftr[j] = trace_event(ftr[j], ta, RAFT_MSG_APPEND_ENTRIES, Lid, Lterm, RAFT_FOLLWER, Lterm, 0);
      fdl[j] = ta + el_base;                          // + the owed draw
      rT[j] = Lterm; rA[j] = Lcommit; rB[j] = 0; rH[j] = 1;
      qA[j] = INF;
    }
    fpend = (1u << F) - 1;
    qmask = 0;
    rmask = (1u << F) - 1;
    resA = ta + d;
    nae += F;
  }
  // The responses of the round with heartbeat th still queued, one per tick in slot order, up to
  // tend - 1.
  __device__ __forceinline__ void responses(uint32_t th, uint32_t tend, uint32_t d, uint32_t hb) {
#pragma unroll
    for (int j = 0; j < F; ++j) {
      const uint32_t tau = th + 2 * d + j;
      if (((rmask >> j) & 1) && tau < tend) {
        Ltr = trace_event(Ltr, tau, RAFT_MSG_APPEND_RESPONSE, fk(j) + 1, Lterm, RAFT_LEADER,
                          Lterm, 0);
        rmask &= ~(1u << j);
        Ldl = tau + hb;
        ++nar;
      }
    }
    if (!rmask) resA = INF;
  }
  // From the fixed point with the next heartbeat at th, every round to the launch's end: the rounds
  // that end before it as trace hashes alone, then the one it cuts (heartbeat, append-entries and
  // responses up to tend - 1; what is left stays queued as the general body leaves it). Every next
  // event of the cluster is then at or after tend.
  __device__ __forceinline__ void rounds(uint32_t th, uint32_t tend, uint32_t d, uint32_t hb,
                                         uint32_t el_base) {
    const uint32_t P = 2 * d + F - 1 + hb, last = 2 * d + F - 1;
    const uint32_t K = tend > th + last ? (tend - th - last - 1) / P + 1 : 0;
    const uint32_t tk = th + K * P;
    if (K) {
      // The trace hash is polynomial (device.hpp): a round's F + 1 leader events take the
      // leader's hash h to h * M2^(F+1) + a, with a the Horner sum of the events' terms, and a
      // round P ticks later adds P * M * (1 + M2 + ... + M2^F) to a; a follower's one event per
      // round takes h to h * M2 + c, and c grows by P * M. One multiply-add per hash per round.
      uint64_t a = trace_term(th, 7, 0, 0, RAFT_LEADER, Lterm, 0);
#pragma unroll
      for (int j = 0; j < F; ++j)
        a = a * TRACE_M2 + trace_term(th + 2 * d + j, RAFT_MSG_APPEND_RESPONSE, fk(j) + 1, Lterm,
                                      RAFT_LEADER, Lterm, 0);
      const uint64_t da = (uint64_t)P * (TRACE_M * trace_geo<F + 1>());
      const uint64_t df = (uint64_t)P * TRACE_M;
      uint64_t cf = trace_term(th + d, RAFT_MSG_APPEND_ENTRIES, Lid, Lterm, RAFT_FOLLWER, Lterm, 0);
      for (uint32_t r = 0; r < K; ++r) {
        Ltr = Ltr * trace_pow<F + 1>() + a;
        a += da;
#pragma unroll
        for (int j = 0; j < F; ++j) ftr[j] = ftr[j] * TRACE_M2 + cf;
        cf += df;
      }
#pragma unroll
      for (int j = 0; j < F; ++j) fdl[j] = tk - P + d + el_base;   // + the owed draw
      fpend = (1u << F) - 1;
      Ldl = tk;                                   // = the last response + hb
      nhb += K;
      nae += F * K;
      nar += F * K;
    }
    if (tk < tend) {                              // the round the launch's end cuts
      Ltr = trace_event(Ltr, tk, 7, 0, 0, RAFT_LEADER, Lterm, 0);
      ++nhb;
      Ldl = tk + hb;
#pragma unroll
      for (int j = 0; j < F; ++j) {
        qA[j] = tk + d; qT[j] = Lterm; qa[j] = Lcommit; qb[j] = 0;
      }
      qmask = (1u << F) - 1;
      if (tk + d < tend) {                        // the append-entries, then responses in time
        append_entries(tk + d, d, el_base);
        responses(tk, tend, d, hb);
      }
    }
  }
};

template <int N>
__global__ void __launch_bounds__(LANE_WG) steady_lane_kernel(DevSim S, uint32_t t0, uint32_t nt) {
  static_assert(N >= 2 && N <= 5, "follower masks and the response queue fit four followers");
  constexpr int F = N - 1;
  constexpr uint32_t HB = hot_block_words(N), CLW = hot_cl_off(N);
  // the words read: the cluster's (checker hwm) and every node field up to the leader-state rows
  // (device.hpp: words 0-122 at N = 5, four lines) -- the leader's rows are picked from them once
  // its id is known, with no second round trip. The image holds whole lines of the block.
  constexpr int NWORDS = (int)(HOT_CW + hf_abase(N) * N);
  constexpr int NW4 = (NWORDS + 3) / 4;
  constexpr int IMGC = (int)(HB / 4) < IMG_SLOTS ? (int)(HB / 4) : IMG_SLOTS;   // chunks staged
  static_assert(NW4 <= IMGC && IMGC % 8 == 0, "the image holds the words read, in whole lines");
  static_assert(CLW == 0, "the cluster words lead the block");
  __shared__ uint32_t bl_c[LANE_WG], bl_t[LANE_WG];   // per wave: bailed cluster, tick it stopped before
  extern __shared__ __attribute__((aligned(16))) uint32_t dsm[];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    // the previous steady launch's bail count (complete: that launch has ended) to the host, which
    // picks the next launches' path from it (speed only); that word is this launch's successor's
    // (host memory is written only when there is something to report: the host zeroes its copy
    // when it acts on it, and a store there holds the launch's end for a bus round trip)
    const uint32_t prev = *S.nbail_zero;
    if (S.bail_report && prev) *S.bail_report = prev;
    if (prev) *S.nbail_zero = 0;
  }
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t cbase = blockIdx.x * LANE_WG + wave * 64;      // the wave's clusters, in id order
  const uint32_t c0 = cbase + lane < S.C ? cbase + lane : INF;
  const bool active = c0 != INF;
  const uint32_t c = active ? c0 : 0u;
  const uint32_t g = S.goff + c;
  char* const img = reinterpret_cast<char*>(dsm) + wave * IMG_WAVE;
  uint32_t* const blc = bl_c + wave * 64;
  uint32_t* const blt = bl_t + wave * 64;
  uint32_t nbw = 0;                                   // clusters this wave bailed (uniform)
  // a compaction point: every lane of the wave active
  auto record_bail = [&](bool b, uint32_t tick) {
    const uint64_t m = __builtin_amdgcn_ballot_w64(b);
    if (b) {
      const uint32_t i = nbw + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      blc[i] = c;
      blt[i] = tick;
    }
    nbw += (uint32_t)__popcll(m);
  };
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

  // ------------------------------------------- load: the wave's blocks into its image (LDS-DMA)
  // half h (lines 2h, 2h + 1): wave instruction j takes clusters 4j .. 4j + 3, 16 slots each
  auto load_half = [&](int h) {
    const uint32_t p = lane & 15;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t cc = 4 * j + (lane >> 4);
      const uint32_t i = 16 * h + (p ^ (cc & 15u));
      const uint32_t cg = min(cbase + cc, S.C - 1);  // past the shard's end: any block, unused
      if (i < (uint32_t)IMGC)
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(S.hot + (size_t)cg * HB + 4 * i),
            (__attribute__((address_space(3))) void*)(img + h * IMG_HALF + j * 1024), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the wave's own LDS-DMA writes landed
  };
  uint32_t w[NW4 * 4];
#pragma unroll
  for (int i = 0; i < NW4 * 4; ++i) w[i] = 0;
  load_half(0);
#pragma unroll
  for (int i = 0; i < (NW4 < 16 ? NW4 : 16); ++i) {
    const uint4 x = *lds_at<const uint4>(img, img_off(lane, i));
    w[4 * i] = x.x; w[4 * i + 1] = x.y; w[4 * i + 2] = x.z; w[4 * i + 3] = x.w;
  }
  // The steady certificate (device.hpp): a cluster the last steady launch left at its fixed point
  // with leader L needs only the first two lines. The rest is loaded when some cluster of the wave
  // lacks one; otherwise those words read as the fixed point's (zero).
  uint32_t Lc = 0, nlc = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const bool lead = (w[HOT_CW + HF_FLAGS * N + k] & 3) == RAFT_LEADER;
    Lc = lead ? (uint32_t)k : Lc;
    nlc += lead;
  }
  static_assert(HOT_CW + (HF_FLAGS + 1) * N <= 64, "the flags are in the first two lines");
  const bool cert = active && nlc == 1 && w[CL_CERT] == (CERT_MAGIC | Lc);
  const bool full = IMGC > 16 && __builtin_amdgcn_ballot_w64(active && !cert) != 0;   // uniform
  if (full) {
    load_half(1);
#pragma unroll
    for (int i = 16; i < NW4; ++i) {
      const uint4 x = *lds_at<const uint4>(img, img_off(lane, i));
      w[4 * i] = x.x; w[4 * i + 1] = x.y; w[4 * i + 2] = x.z; w[4 * i + 3] = x.w;
    }
  }
  const bool vouched = cert && !full;         // its lines past the second are the fixed point's
  const uint32_t tend = t0 + nt, d = S.dmin;
  const uint32_t P = 2 * d + F - 1 + S.hb, allF = (1u << F) - 1;
  uint32_t dl = 0, nhb = 0, nae = 0, nar = 0;  // lines of the block changed; events run
  bool el = false;                             // the cluster's election ran here (general path)
  uint32_t el_to = 0;                          // its timeouts (two candidates: a tie)
#ifdef RS_WAVELOG
  uint64_t wl_x1 = 0, wl_x2 = 0, wl_x3 = 0, wl_lend = 0;
#endif

  // ------------------------------------------- the certified path
  // A wave whose every cluster is vouched for by its certificate (device.hpp), on the fixed
  // point's period-P schedule (its round in progress at t0: none, the append-entries in flight, or
  // the responses the last launch's end cut) and with its followers' draws owed (FL_DRAW) runs the
  // whole launch from the first two lines of its blocks: the rest of that round, then
  // FixedPoint::rounds. Queued messages are not read: a certified cluster's are the fixed point's
  // (whatever else writes a ring clears the certificate), and so are its leader's commit (0) and
  // the rest of its state. Any other wave takes the general path below.
  FixedPoint<N> fx;
  uint32_t lmid = 0, lth0 = 0;
  bool lean = vouched && S.el_base >= P && S.hb >= 2 * d + F && S.Q >= (uint32_t)F;
  {
    const uint32_t L = Lc;
    auto lw = [&](int f, int k) { return w[HOT_CW + f * N + k]; };
    auto lpick = [&](int f) {                       // field f of the leader
      uint32_t v = 0;
#pragma unroll
      for (int k = 0; k < N; ++k) v |= lw(f, k) & (0u - (uint32_t)(L == (uint32_t)k));
      return v;
    };
    auto lfol = [&](int f, int j) {                 // field f of follower slot j
      const uint32_t m = 0u - (uint32_t)((uint32_t)j >= L);
      return (lw(f, j + 1) & m) | (lw(f, j) & ~m);
    };
    fx.L = L; fx.Lid = L + 1; fx.Lterm = lpick(HF_TERM); fx.Lcommit = 0;
    fx.Ldl = lpick(HF_DEADLINE);
    fx.Ltr = (uint64_t)lpick(HF_TRACE_HI) << 32 | lpick(HF_TRACE_LO);
    fx.qmask = fx.rmask = 0; fx.resA = INF; fx.fpend = allF; fx.nhb = fx.nae = fx.nar = 0;
    const uint32_t Lqm = lpick(HF_QMETA);
    const uint32_t rsc = (Lqm >> 13) & 31;
    uint32_t need = 0;
#pragma unroll
    for (int j = 0; j < F; ++j) {
      fx.fdl[j] = lfol(HF_DEADLINE, j);
      fx.ftr[j] = (uint64_t)lfol(HF_TRACE_HI, j) << 32 | lfol(HF_TRACE_LO, j);
      const uint32_t qm = lfol(HF_QMETA, j);
      lean = lean && (lfol(HF_FLAGS, j) & FL_DRAW) && ((qm >> 4) & 31) <= 1 && !((qm >> 13) & 31);
      need |= (((qm >> 4) & 31) ? 1u : 0u) << j;
      fx.qA[j] = INF; fx.qT[j] = fx.qa[j] = fx.qb[j] = 0;
      fx.rT[j] = fx.rA[j] = fx.rB[j] = fx.rH[j] = 0;
    }
    lean = lean && !((Lqm >> 4) & 31) && rsc <= (uint32_t)F && !(need && rsc) &&
           (need == 0 || need == allF);
    lth0 = fx.Ldl;
    if (need) {                                     // the append-entries in flight
      lmid = 1;
      const uint32_t ta = lfol(HF_REQ_ARR, 0);
      lth0 = ta - d;
      lean = lean && ta >= t0 && ta >= d && fx.Ldl == lth0 + S.hb;
#pragma unroll
      for (int j = 0; j < F; ++j) {
        lean = lean && lfol(HF_REQ_ARR, j) == ta;
        fx.qA[j] = ta; fx.qT[j] = fx.Lterm;
      }
      fx.qmask = allF;
    } else if (rsc) {                               // the responses the last launch's end cut
      lmid = 2;
      const uint32_t ra = lpick(HF_RES_ARR), j0 = (uint32_t)F - rsc;
      lth0 = ra - 2 * d;
      const int64_t cut = (int64_t)t0 - ((int64_t)lth0 + 2 * d);
      lean = lean && ra >= 2 * d && (int64_t)j0 == (cut < 0 ? 0 : cut > F ? (int64_t)F : cut) &&
             fx.Ldl == (j0 ? lth0 + 2 * d + j0 - 1 : lth0) + S.hb;
      fx.rmask = allF & ~((1u << j0) - 1);
      fx.resA = ra;
#pragma unroll
      for (int j = 0; j < F; ++j) {
        fx.rT[j] = fx.Lterm; fx.rH[j] = 1;
      }
    } else {
      lean = lean && fx.Ldl >= t0;
    }
    const uint32_t nxt = min((lmid == 2 ? lth0 + P : lth0) + d, tend);   // the next AE (or end)
#pragma unroll
    for (int j = 0; j < F; ++j) lean = lean && fx.fdl[j] >= nxt;
  }
  const bool lean_wave = !__builtin_amdgcn_ballot_w64(active && !lean);     // uniform
  bool wb = false;
  if (lean_wave) {
    if (active) {
      bool whole = true;                      // the round in progress finished in this launch
      if (lmid == 1) {
        if (fx.qA[0] < tend) fx.append_entries(fx.qA[0], d, S.el_base);
        else whole = false;
      }
      if (lmid && whole) {
        fx.responses(lth0, tend, d, S.hb);
        whole = !fx.rmask;
      }
      if (whole) fx.rounds(lmid ? lth0 + P : lth0, tend, d, S.hb, S.el_base);
      nhb = fx.nhb; nae = fx.nae; nar = fx.nar;
      // fields DEADLINE .. RES_TAIL of every node back into the image (the rest is unchanged)
      const uint32_t L = fx.L;
      uint32_t v[HF_FLAGS][N];
#pragma unroll
      for (int k = 0; k < N; ++k) {
        const bool isL = (uint32_t)k == L;
        const int jl = k > 0 ? k - 1 : 0, jh = k < F ? k : F - 1;
        const bool lo = (uint32_t)k > L;
        auto fv = [&](const uint32_t* x) { return msel(lo, x[jl], x[jh]); };
        const uint32_t fq = (fx.qmask >> (lo ? jl : jh)) & 1, fqa = fv(fx.qA);
        const uint64_t trf = (uint64_t)msel(lo, (uint32_t)(fx.ftr[jl] >> 32),
                                            (uint32_t)(fx.ftr[jh] >> 32)) << 32 |
                             msel(lo, (uint32_t)fx.ftr[jl], (uint32_t)fx.ftr[jh]);
        const uint64_t tr = isL ? fx.Ltr : trf;
        v[HF_DEADLINE][k] = isL ? fx.Ldl : fv(fx.fdl);
        v[HF_TRACE_LO][k] = (uint32_t)tr;
        v[HF_TRACE_HI][k] = (uint32_t)(tr >> 32);
        v[HF_QMETA][k] = isL ? pack_qmeta(0, 0, 0, __popc(fx.rmask)) : pack_qmeta(0, fq, 0, 0);
        v[HF_REQ_ARR][k] = isL ? INF : (fq ? fqa : INF);
        v[HF_RES_ARR][k] = isL ? fx.resA : INF;
        v[HF_REQ_TAIL][k] = isL ? 0u : (fq ? fqa : 0u);
        v[HF_RES_TAIL][k] = isL ? (fx.rmask ? fx.resA : 0u) : 0u;
      }
      auto in = [](int q) { return q >= (int)HOT_CW && q < (int)(HOT_CW + HF_FLAGS * N); };
      auto val = [&](int q) { return v[(q - HOT_CW) / N][(q - HOT_CW) % N]; };
#pragma unroll
      for (int i = (int)HOT_CW / 4; i < (int)(HOT_CW + HF_FLAGS * N + 3) / 4; ++i) {
        const int q = 4 * i;
        const uint4 x = make_uint4(in(q) ? val(q) : w[q], in(q + 1) ? val(q + 1) : w[q + 1],
                                   in(q + 2) ? val(q + 2) : w[q + 2],
                                   in(q + 3) ? val(q + 3) : w[q + 3]);
        *lds_at<uint4>(img, img_off(lane, i)) = x;
        dl |= (uint32_t)(x.x != w[q] || x.y != w[q + 1] || x.z != w[q + 2] || x.w != w[q + 3])
              << (i / 8);
      }
    }
    // messages in flight at the launch's end back to the rings, heads at slot 0 (rare)
    if (__builtin_amdgcn_ballot_w64(active && (fx.qmask || fx.rmask))) {   // wave-uniform
#pragma unroll
      for (int j = 0; j < F; ++j) {
        if (active && ((fx.qmask >> j) & 1)) {
          uint4* dp = reinterpret_cast<uint4*>(qslots(S, c * N + fx.fk(j), 0));
          dp[0] = make_uint4(fx.qA[j], RAFT_MSG_APPEND_ENTRIES | fx.Lid << 3, fx.qT[j], fx.qa[j]);
          dp[1] = make_uint4(fx.qb[j], 0, 0, 0);
        }
      }
      uint4* rp = reinterpret_cast<uint4*>(qslots(S, c * N + fx.L, 1));
      uint32_t n = 0;
#pragma unroll
      for (int j = 0; j < F; ++j) {
        if (active && ((fx.rmask >> j) & 1)) {
          uint4* dp = rp + 2 * n;
          dp[0] = make_uint4(fx.resA, RAFT_MSG_APPEND_RESPONSE | (fx.fk(j) + 1) << 3 | fx.rH[j] << 7,
                             fx.rT[j], fx.rA[j]);
          dp[1] = make_uint4(fx.rB[j], 0, 0, 0);
          ++n;
        }
      }
    }
#ifdef RS_WAVELOG
    wl_loop = wl_x1 = wl_x2 = wl_x3 = wl_lend = wall_clock64();
#endif
  } else {
#ifdef RS_WAVELOG
    wl_loop = wall_clock64();
#endif
    auto field = [&](int f, uint32_t (&out)[N]) {
#pragma unroll
      for (int k = 0; k < N; ++k) out[k] = w[HOT_CW + f * N + k];
    };
    // ------------------------------------------- the election from init-node, in closed form
    // A cluster still in init-node's state (core.clj:31-38: every node a follower of the same term
    // with no vote, leader, log, leader-state or message; no checker mark) elects the node whose
    // timer fires first, and with no faults, no client and a fixed delay d that election is one
    // script when no other timer fires before the request-vote reaches it (D_k >= t1 + d):
    //   t1            candidate c times out (timeout-handler 166-169): term T + 1, request-vote
    //                 to every peer;
    //   t1 + d        every follower grants it (request-vote-handler 91-103: vote, no term change);
    //   t1 + 2d + i   c takes the i-th vote response in sender order (vote-response-handler
    //                 125-139) and is leader at the one that makes a majority (i_L), broadcasting
    //                 an empty append-entries (candidate->leader 80-84, append-entries-rpc 56-67);
    //   tL + d        every follower takes it (append-entries-handler 105-123: term T + 1, :follwer,
    //                 leader id) and answers; c takes the rest of the votes, then the F responses
    //                 one per tick from max(t1 + 2d + F, tL + 2d) (append-response-handler 141-149).
    // Every timer re-arm is one the general body defers (followers' draws stay owed), the leader's
    // rows end as init-node's (next = mb = 0, match = 0) and nothing is left queued: the script
    // writes the cluster's state after its last event into the registers below, and the cluster is
    // then at the fixed point, which the rest of this path runs to the launch's end (trace hashes,
    // deadlines and counters as the general body gives them). Two timers firing in the same tick
    // (delay 1) have a script of their own below. Anything else -- near ties, three timers, an
    // election cut by the launch's end, a state that only looks like init-node -- is bailed.
    {
      auto ifield = [&](int f, int k) { return w[HOT_CW + f * N + k]; };
      bool pat = active && w[0] == 0 && S.Q >= 2u * F && S.el_base >= P && S.hb >= 2 * d + F;
      const uint32_t T = ifield(HF_TERM, 0);
#pragma unroll
      for (int k = 0; k < N; ++k) {
        pat = pat && ifield(HF_FLAGS, k) == 0 && ifield(HF_MASKS, k) == 0 &&
              ifield(HF_TERM, k) == T && ifield(HF_COMMIT, k) == 0 && ifield(HF_LEN, k) == 0 &&
              ifield(HF_QMETA, k) == 0 && ifield(HF_REQ_ARR, k) == INF &&
              ifield(HF_RES_ARR, k) == INF;
#pragma unroll
        for (int p = 0; p < 2 * N; ++p) pat = pat && ifield(HF_NEXT + p, k) == 0;
      }
      pat = pat && T != INF;
      // the candidate: the earliest deadline (the lower index of two equal ones, a tie)
      uint32_t cidx = 0, t1 = INF, ntie = 0, bidx = 0;
#pragma unroll
      for (int k = 0; k < N; ++k) {
        const uint32_t dk = ifield(HF_DEADLINE, k);
        cidx = dk < t1 ? (uint32_t)k : cidx;
        t1 = min(t1, dk);
      }
      bool single = true;
#pragma unroll
      for (int k = 0; k < N; ++k) {
        const uint32_t dk = ifield(HF_DEADLINE, k);
        ntie += dk == t1;
        bidx = dk == t1 && (uint32_t)k != cidx ? (uint32_t)k : bidx;
        single = single && ((uint32_t)k == cidx || (uint64_t)dk >= (uint64_t)t1 + d);
      }
      // two timers firing together (the delay 1: every other one is then at least d later)
      const bool tie = ntie == 2 && d == 1 && N >= 3;
      constexpr uint32_t iL = (N + 1) / 2 >= 2 ? (N + 1) / 2 - 2 : 0;   // the electing response
      const uint64_t tL = (uint64_t)t1 + 2 * d + iL;
      const uint64_t tau0 = max((uint64_t)t1 + 2 * d + F, tL + 2 * d);  // the first response
      const uint64_t tlast = tau0 + F - 1;
      pat = pat && (single || tie) && t1 >= t0 && (tie || tlast < tend) &&
            (uint64_t)t1 + 4 * N + 8 < 0xFFFFFFFFull;
      // the election-safety check (P4) compares the new leader's led term with the others'
      // (words past the image: read only when some cluster of the wave qualifies)
      if (__builtin_amdgcn_ballot_w64(pat)) {                 // wave-uniform
        const uint32_t* lp = S.hot + (size_t)c * HB + HOT_CW + hf_led(N) * N;
        uint32_t led[N];
#pragma unroll
        for (int k = 0; k < N; ++k) led[k] = lp[k];
#pragma unroll
        for (int k = 0; k < N; ++k) pat = pat && ((uint32_t)k == cidx || led[k] != T + 1);
      }
      const uint32_t T1 = T + 1, cid = cidx + 1, peers = ((1u << (N + 1)) - 1) & ~1u & ~(1u << cid);
      if (pat && single) {
        el = true;
        el_to = 1;
        // the candidate's events (node cidx), then each follower's
        uint64_t hc = 0;
#pragma unroll
        for (int k = 0; k < N; ++k)
          if ((uint32_t)k == cidx)
            hc = (uint64_t)ifield(HF_TRACE_HI, k) << 32 | ifield(HF_TRACE_LO, k);
        hc = trace_event(hc, t1, 6, 0, 0, RAFT_CANDIDATE, T1, 0);
#pragma unroll
        for (int i = 0; i < F; ++i) {
          const uint32_t sid = (uint32_t)i + ((uint32_t)i >= cidx ? 2u : 1u);   // slot i's id
          hc = trace_event(hc, t1 + 2 * d + i, RAFT_MSG_VOTE_RESPONSE, sid, T,
                           (uint32_t)i >= iL ? RAFT_LEADER : RAFT_CANDIDATE, T1, 0);
        }
#pragma unroll
        for (int j = 0; j < F; ++j) {
          const uint32_t sid = (uint32_t)j + ((uint32_t)j >= cidx ? 2u : 1u);
          hc = trace_event(hc, (uint32_t)tau0 + j, RAFT_MSG_APPEND_RESPONSE, sid, T, RAFT_LEADER,
                           T1, 0);
        }
#pragma unroll
        for (int k = 0; k < N; ++k) {
          const bool isc = (uint32_t)k == cidx;
          uint64_t h = (uint64_t)ifield(HF_TRACE_HI, k) << 32 | ifield(HF_TRACE_LO, k);
          h = trace_event(h, t1 + d, RAFT_MSG_REQUEST_VOTE, cid, T1, RAFT_FOLLOWER, T, 0);
          h = trace_event(h, (uint32_t)tL + d, RAFT_MSG_APPEND_ENTRIES, cid, T1, RAFT_FOLLWER, T1, 0);
          h = isc ? hc : h;
          w[HOT_CW + HF_FLAGS * N + k] = isc ? pack_flags(RAFT_LEADER, 0, cid, 0, 0, 1)
                                             : pack_flags(RAFT_FOLLWER, 0, cid, 0, 0, 0) | FL_DRAW;
          w[HOT_CW + HF_MASKS * N + k] = isc ? peers << 16 : 0u;
          w[HOT_CW + HF_TERM * N + k] = T1;
          w[HOT_CW + HF_DEADLINE * N + k] = isc ? (uint32_t)tlast + S.hb
                                                : (uint32_t)tL + d + S.el_base;   // + the owed draw
          w[HOT_CW + HF_REQ_TAIL * N + k] = 0;
          w[HOT_CW + HF_RES_TAIL * N + k] = 0;
          w[HOT_CW + HF_TRACE_LO * N + k] = (uint32_t)h;
          w[HOT_CW + HF_TRACE_HI * N + k] = (uint32_t)(h >> 32);
        }
        nae = F;                                    // the followers' append-entries and their
        nar = F;                                    // responses (the rest is counted as el_to)
      } else if (pat && tie) {
        // Two timers at t1 (d = 1): candidates a < b (ids A, B) both time out and send
        // request-votes; at t1 + 1 every other node grants A's (the lower id's, queued first) and
        // a and b deny each other (each voted for itself); at t1 + 2 those nodes deny B's. a takes
        // its vote responses one per tick from t1 + 2 in sender order and is leader at the
        // majority's one (tL); b takes a's denial at t1 + 2, then the others' from t1 + 3, and
        // a's append-entries when it arrives at tL + 1 -- when both of b's queues are ready the
        // alts!! bit of its EVENT draw picks (core.clj:181), and that draw re-arms its timer
        // exactly. a then takes the responses: the others' at tL + 2 and b's the tick after b
        // took the append-entries, by (arrival, sender id).
        const uint32_t a = cidx, b = bidx, B = b + 1;
        const uint32_t A = cid;
        constexpr uint32_t M = (N + 1) / 2;                  // majority? (core.clj:19-21)
        uint64_t ha = 0, hbb = 0;
#pragma unroll
        for (int k = 0; k < N; ++k) {
          const uint64_t h0 = (uint64_t)ifield(HF_TRACE_HI, k) << 32 | ifield(HF_TRACE_LO, k);
          if ((uint32_t)k == a) ha = h0;
          if ((uint32_t)k == b) hbb = h0;
        }
        ha = trace_event(ha, t1, 6, 0, 0, RAFT_CANDIDATE, T1, 0);
        ha = trace_event(ha, t1 + 1, RAFT_MSG_REQUEST_VOTE, B, T1, RAFT_CANDIDATE, T1, 0);
        uint32_t votes = 1, tLt = INF, role = RAFT_CANDIDATE;
#pragma unroll
        for (int k = 0; k < N; ++k) {                        // a's vote responses, id order
          if ((uint32_t)k == a) continue;
          const uint32_t i = (uint32_t)k - ((uint32_t)k > a ? 1u : 0u), tau = t1 + 2 + i;
          const bool grant = (uint32_t)k != b;
          if (grant && role == RAFT_CANDIDATE && ++votes >= M) {
            role = RAFT_LEADER;
            tLt = tau;
          }
          ha = trace_event(ha, tau, RAFT_MSG_VOTE_RESPONSE, (uint32_t)k + 1, grant ? T : T1, role,
                           T1, 0);
        }
        // b: the denials, then a's append-entries
        hbb = trace_event(hbb, t1, 6, 0, 0, RAFT_CANDIDATE, T1, 0);
        hbb = trace_event(hbb, t1 + 1, RAFT_MSG_REQUEST_VOTE, A, T1, RAFT_CANDIDATE, T1, 0);
        hbb = trace_event(hbb, t1 + 2, RAFT_MSG_VOTE_RESPONSE, A, T1, RAFT_CANDIDATE, T1, 0);
        uint32_t tb = t1 + 3, j = 0, tbae = INF, brole = RAFT_CANDIDATE, bdl = 0;
        bool bexact = false;
        for (int it = 0; it < N + 1; ++it) {
          const bool res = j < (uint32_t)N - 2, req = tbae == INF;
          if (!res && !req) break;
          if (!res && tb < tLt + 1) tb = tLt + 1;             // idle until the append-entries
          const bool rq = req && tb >= tLt + 1;
          bool take_req = rq;
          bexact = false;
          if (res && rq) {                                    // alts!! (core.clj:181)
            const uint4 ew = event_draw(g, B, tb, S);
            take_req = !(ew.x & 1);
            bexact = true;
            bdl = tb + S.el_base + __umulhi(ew.y, S.el_span);
          }
          if (take_req) {                                     // append-entries-handler 105-123
            hbb = trace_event(hbb, tb, RAFT_MSG_APPEND_ENTRIES, A, T1, RAFT_FOLLWER, T1, 0);
            brole = RAFT_FOLLWER;
            tbae = tb;
          } else {                                            // the j-th other node's denial
            uint32_t fid = 0, cnt = 0;
#pragma unroll
            for (int k = 0; k < N; ++k) {
              const bool other = (uint32_t)k != a && (uint32_t)k != b;
              fid = other && cnt == j ? (uint32_t)k + 1 : fid;
              cnt += other;
            }
            hbb = trace_event(hbb, tb, RAFT_MSG_VOTE_RESPONSE, fid, T, brole, T1, 0);
            ++j;
          }
          if (!bexact) bdl = tb + S.el_base;                  // + the owed draw
          ++tb;
        }
        const uint32_t tbl = tb - 1;                          // b's last event
        // a's responses: the others' at tLt + 2, b's at tbae + 1, by (arrival, sender id)
        uint32_t ta = t1 + N + 1;                             // after its N - 1 vote responses
        const uint32_t fa = tLt + 2, ba = tbae + 1;
#pragma unroll
        for (int k = 0; k < N; ++k) {
          if ((uint32_t)k == a) continue;
          const bool isb = (uint32_t)k == b;
          if (isb && ba != fa) continue;
          ta = max(ta, fa);
          ha = trace_event(ha, ta, RAFT_MSG_APPEND_RESPONSE, (uint32_t)k + 1, isb ? T1 : T,
                           RAFT_LEADER, T1, 0);
          ++ta;
        }
        if (ba != fa) {
          ta = max(ta, ba);
          ha = trace_event(ha, ta, RAFT_MSG_APPEND_RESPONSE, B, T1, RAFT_LEADER, T1, 0);
          ++ta;
        }
        const uint32_t tal = ta - 1;                          // a's last event
        if (tbae != INF && tLt != INF && max(tal, tbl) < tend) {
          el = true;
          el_to = 2;
#pragma unroll
          for (int k = 0; k < N; ++k) {
            const bool isa = (uint32_t)k == a, isb = (uint32_t)k == b;
            uint64_t h = (uint64_t)ifield(HF_TRACE_HI, k) << 32 | ifield(HF_TRACE_LO, k);
            h = trace_event(h, t1 + 1, RAFT_MSG_REQUEST_VOTE, A, T1, RAFT_FOLLOWER, T, 0);
            h = trace_event(h, t1 + 2, RAFT_MSG_REQUEST_VOTE, B, T1, RAFT_FOLLOWER, T, 0);
            h = trace_event(h, tLt + 1, RAFT_MSG_APPEND_ENTRIES, A, T1, RAFT_FOLLWER, T1, 0);
            h = isa ? ha : isb ? hbb : h;
            w[HOT_CW + HF_FLAGS * N + k] =
                isa ? pack_flags(RAFT_LEADER, 0, A, 0, 0, 1)
                    : pack_flags(RAFT_FOLLWER, 0, A, 0, 0, 0) | (isb && bexact ? 0u : FL_DRAW);
            w[HOT_CW + HF_MASKS * N + k] = isa ? peers << 16 : 0u;
            w[HOT_CW + HF_TERM * N + k] = T1;
            w[HOT_CW + HF_DEADLINE * N + k] = isa ? tal + S.hb : isb ? bdl : tLt + 1 + S.el_base;
            w[HOT_CW + HF_REQ_TAIL * N + k] = 0;
            w[HOT_CW + HF_RES_TAIL * N + k] = 0;
            w[HOT_CW + HF_TRACE_LO * N + k] = (uint32_t)h;
            w[HOT_CW + HF_TRACE_HI * N + k] = (uint32_t)(h >> 32);
          }
          nae = F;
          nar = F;
        }
      }
    }
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
      badn |= ((f >> 10) & 7) | (lead != (((f >> 14) & 1) != 0)) | (lead && (f & FL_DRAW));
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
    {
      uint32_t rn[N], rm[N];                    // the leader's next / match of each peer id p + 1
#pragma unroll
      for (int p = 0; p < N; ++p) {
        field(HF_NEXT + p, tmp);
        rn[p] = pick<N>(tmp, L);
        field(HF_NEXT + N + p, tmp);
        rm[p] = pick<N>(tmp, L);
      }
#pragma unroll
      for (int j = 0; j < F; ++j) {
        nx[j] = (int32_t)fsel(rn, j);
        mt[j] = (int32_t)fsel(rm, j);
      }
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

#ifdef RS_WAVELOG
    asm volatile("" ::"v"(Ltr), "v"(fdl[0]), "v"(nx[0]));
    wl_x1 = wall_clock64();                     // fields extracted
#endif
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
      uint32_t need = 0, rqh[F];
#pragma unroll
      for (int j = 0; j < F; ++j) {
        const uint32_t qm = fsel(nqm, j);
        const uint32_t rqc = (qm >> 4) & 31;
        rqh[j] = qm & 15;
        bad = bad || rqc > 1 || ((qm >> 13) & 31) != 0;       // <= 1 request, no responses
        need |= (uint32_t)(rqc != 0) << j;
      }
      bad = bad || rsc > (uint32_t)F;
      // The messages: loaded by every lane of a wave in which any lane has one (a message in flight
      // at the launch's start is rare), all loads issued before any is looked at -- one memory round
      // trip, where loads under per-lane branches each waited for the last. Slot indices are
      // clamped into the ring for lanes whose queue words are not looked at.
      uint4 qm0[F], qm1[F], rm0[F], rm1[F];
      if (__builtin_amdgcn_ballot_w64(!bad && (need || rsc))) {     // wave-uniform
#pragma unroll
        for (int j = 0; j < F; ++j) {                          // the leader's append-entries
          const uint4* mp = reinterpret_cast<const uint4*>(
              qslots(S, c * N + fk(j), 0) + min(rqh[j], S.Q - 1) * qstride(S, 0));
          qm0[j] = mp[0];
          qm1[j] = mp[1];
        }
#pragma unroll
        for (int i = 0; i < F; ++i) {                          // append-responses, sender order
          const uint4* mp = reinterpret_cast<const uint4*>(
              qslots(S, c * N + L, 1) + min(wrapq(rsh + i, S.Q), S.Q - 1) * qstride(S, 1));
          rm0[i] = mp[0];
          rm1[i] = mp[1];
        }
      }
      if (!bad) {
#pragma unroll
        for (int j = 0; j < F; ++j) {
          if ((need >> j) & 1) {
            const uint4 m0 = qm0[j], m1 = qm1[j];
            bad = bad || m0.y != (RAFT_MSG_APPEND_ENTRIES | Lid << 3) || m1.y || m1.z || m1.w;
            qmask |= 1u << j;
            qA[j] = m0.x; qT[j] = m0.z; qa[j] = m0.w; qb[j] = m1.x;
          }
        }
        uint32_t last = 0;
#pragma unroll
        for (int i = 0; i < F; ++i) {
          if ((uint32_t)i < rsc && !bad) {
            const uint4 m0 = rm0[i], m1 = rm1[i];
            const uint32_t hdr = m0.y, src = (hdr >> 3) & 15;
            bad = (hdr & 7) != RAFT_MSG_APPEND_RESPONSE || (hdr >> 8) || m1.y || m1.z || m1.w ||
                  src <= last || src > (uint32_t)N || src == Lid || (i && m0.x != resA);
            last = src;
            resA = m0.x;
            const uint32_t j = src - 1 - (src > Lid ? 1u : 0u);
            if (!bad) {
              rmask |= 1u << j;
#pragma unroll
              for (int jj = 0; jj < F; ++jj) {
                if ((uint32_t)jj == j) {
                  rT[jj] = m0.z; rA[jj] = m0.w; rB[jj] = m1.x; rH[jj] = (hdr >> 7) & 1;
                }
              }
            }
          }
        }
      }
      if (!rmask) resA = INF;
    }
    record_bail(active && bad, t0);           // outside the model from the start: bail at t0
    wb = active && !bad;
    bool run = wb;

    // ---------------------------------------------------------------- the cluster's ticks
    uint32_t tn = t0;
    // followers whose deadline holds its lower bound t_ae + el_base (the draw is deferred)
    // (a draw owed from an earlier launch: FL_DRAW in the follower's flags, device.hpp)
    uint32_t fpend = 0;
#pragma unroll
    for (int j = 0; j < F; ++j) fpend |= ((ffl[j] & FL_DRAW) ? 1u : 0u) << j;
    auto draw_deadlines = [&](uint32_t due) {
#pragma unroll
      for (int j = 0; j < F; ++j) {
        if ((due >> j) & 1) {
          const uint4 wd = event_draw(g, fk(j) + 1, fdl[j] - S.el_base, S);   // D4, core.clj:174
          fdl[j] += __umulhi(wd.y, S.el_span);
        }
      }
      fpend &= ~due;
    };
    auto next_event = [&]() {
      uint32_t m = min(Ldl, resA);
#pragma unroll
      for (int j = 0; j < F; ++j) m = min(m, min(fdl[j], qA[j]));
      return m;
    };
    // The cluster at its fixed point: every follower took the leader's append-entries (flags,
    // votes, term and commit are what another one sets again), every response succeeded (next /
    // match / keys as another one sets them), the log is empty (a heartbeat ships nothing) and no
    // message is in flight. If the followers' re-armed timers (>= t_ae + el_base) cannot fire
    // before the next round's append-entries (el_base >= the round period P) and the leader's
    // responses all fit before its next heartbeat (hb >= 2d + F), every later round is this one
    // shifted by a multiple of P: only the ticks in the trace hashes change.
    auto at_fixed_point_state = [&]() {
      bool ok = Llen == 0 && !ackbad;
#pragma unroll
      for (int j = 0; j < F; ++j)
        ok = ok && fterm[j] == Lterm &&
             (ffl[j] & (3u | 15u << 2 | 15u << 6 | 1u << 13)) == (RAFT_FOLLWER | Lid << 6) &&
             fcommit[j] == flen[j] && (fmk[j] & 0xFFFFu) == 0 && nx[j] == 0 &&
             mt[j] == (int32_t)Lcommit;
      return ok;
    };
    auto at_fixed_point = [&]() {
      return S.el_base >= P && S.hb >= 2 * d + F && !qmask && !rmask && at_fixed_point_state();
    };
    // From the fixed point with the next heartbeat at th, every round to the launch's end as trace
    // hashes: the rounds that end before it, then the one it cuts (heartbeat, append-entries and
    // responses up to tend - 1; what is left is queued as the general body leaves it): every next
    // event of the cluster is then at or after tend.
    auto fixed_point_rounds = [&](uint32_t th) {   // FixedPoint::rounds on this path's registers
      FixedPoint<N> x;
      x.L = L; x.Lid = Lid; x.Lterm = Lterm; x.Lcommit = Lcommit;
      x.Ltr = Ltr; x.Ldl = Ldl; x.fpend = fpend; x.qmask = qmask; x.rmask = rmask; x.resA = resA;
      x.nhb = nhb; x.nae = nae; x.nar = nar;
#pragma unroll
      for (int j = 0; j < F; ++j) {
        x.ftr[j] = ftr[j]; x.fdl[j] = fdl[j];
        x.qA[j] = qA[j]; x.qT[j] = qT[j]; x.qa[j] = qa[j]; x.qb[j] = qb[j];
        x.rT[j] = rT[j]; x.rA[j] = rA[j]; x.rB[j] = rB[j]; x.rH[j] = rH[j];
      }
      x.rounds(th, tend, d, S.hb, S.el_base);
      Ltr = x.Ltr; Ldl = x.Ldl; fpend = x.fpend; qmask = x.qmask; rmask = x.rmask; resA = x.resA;
      nhb = x.nhb; nae = x.nae; nar = x.nar;
#pragma unroll
      for (int j = 0; j < F; ++j) {
        ftr[j] = x.ftr[j]; fdl[j] = x.fdl[j];
        qA[j] = x.qA[j]; qT[j] = x.qT[j]; qa[j] = x.qa[j]; qb[j] = x.qb[j];
        rT[j] = x.rT[j]; rA[j] = x.rA[j]; rB[j] = x.rB[j]; rH[j] = x.rH[j];
      }
    };

    // ------------------------------------------- the fixed-point path (C2's steady state)
    // A cluster at its fixed point (above) whose round in progress at t0 is on the period-P
    // schedule -- none (the next heartbeat at Ldl >= t0), its append-entries in flight, or its
    // responses pending exactly as the last launch's end cut them -- and whose followers' timers
    // cannot fire before their next append-entries runs every event of the launch here: the rest
    // of that round event by event, then fixed_point_rounds. Everything else is the general loop's.
    bool fp = wb && S.el_base >= P && S.hb >= 2 * d + F && (vouched || at_fixed_point_state());
    uint32_t th0 = Ldl, mid = 0;               // the round's heartbeat; 1 AEs in flight, 2 responses
    if (qmask) {
      mid = 1;
      th0 = qA[0] - d;
      fp = fp && qmask == allF && !rmask && qA[0] >= t0 && qA[0] >= d && Ldl == th0 + S.hb;
#pragma unroll
      for (int j = 0; j < F; ++j)
        fp = fp && qA[j] == qA[0] && qT[j] == Lterm && qa[j] == Lcommit && qb[j] == 0;
    } else if (rmask) {
      mid = 2;
      th0 = resA - 2 * d;
      const uint32_t j0 = (uint32_t)F - __popc(rmask);          // responses already taken
      const int64_t cut = (int64_t)t0 - ((int64_t)th0 + 2 * d);  // what the last launch's end cut
      fp = fp && resA >= 2 * d && rmask == (allF & ~((1u << j0) - 1)) &&
           (int64_t)j0 == (cut < 0 ? 0 : cut > F ? (int64_t)F : cut) &&
           Ldl == (j0 ? th0 + 2 * d + j0 - 1 : th0) + S.hb;
#pragma unroll
      for (int j = 0; j < F; ++j)
        fp = fp && (!((rmask >> j) & 1) ||
                    (rT[j] == Lterm && rA[j] == Lcommit && rB[j] == 0 && rH[j] == 1));
    } else {
      fp = fp && Ldl >= t0;
    }
    {
      const uint32_t nxt = min((mid == 2 ? th0 + P : th0) + d, tend);   // the next AE (or the end)
#pragma unroll
      for (int j = 0; j < F; ++j) fp = fp && fdl[j] >= nxt;
    }
    // A vouched cluster off the fixed-point path (set_tick moved the clock, ...) has no full state
    // here: the general body runs it from t0.
    const bool vbail = vouched && wb && !fp;
    record_bail(vbail, t0);
    if (vbail) wb = run = false;
#ifdef RS_WAVELOG
    asm volatile("" ::"v"(fp), "v"(th0));
    wl_x2 = wall_clock64();                     // queued messages read, fixed-point path decided
#endif
    if (fp) {
      run = false;
      bool whole = true;                        // the round in progress finished in this launch
      if (mid == 1) {
        const uint32_t ta = qA[0];
        if (ta < tend) {                        // the append-entries
#pragma unroll
          for (int j = 0; j < F; ++j) {
            ftr[j] = trace_event(ftr[j], ta, RAFT_MSG_APPEND_ENTRIES, Lid, Lterm, RAFT_FOLLWER,
                                 Lterm, 0);
            fdl[j] = ta + S.el_base;
            qA[j] = INF;
            rT[j] = Lterm; rA[j] = Lcommit; rB[j] = 0; rH[j] = 1;
          }
          fpend = allF;
          qmask = 0;
          rmask = allF;
          resA = ta + d;
          nae += F;
        } else {
          whole = false;
        }
      }
      if (mid && whole) {                       // the responses, one per tick in slot order
#pragma unroll
        for (int j = 0; j < F; ++j) {
          const uint32_t tau = th0 + 2 * d + j;
          if (((rmask >> j) & 1) && tau < tend) {
            Ltr = trace_event(Ltr, tau, RAFT_MSG_APPEND_RESPONSE, fk(j) + 1, Lterm, RAFT_LEADER,
                              Lterm, 0);
            rmask &= ~(1u << j);
            Ldl = tau + S.hb;
            ++nar;
          }
        }
        if (rmask) whole = false;
        else resA = INF;
      }
      if (whole) fixed_point_rounds(mid ? th0 + P : th0);
    }
#ifdef RS_WAVELOG
    asm volatile("" ::"v"(Ltr), "v"(ftr[0]), "v"(Ldl));
    wl_x3 = wall_clock64();                     // the fixed-point path's rounds done
#endif
#ifdef RS_WAVELOG
    wl_ts = __builtin_amdgcn_s_memtime();
#endif
    bool pbail = false;                        // bailed in the last trip, not yet recorded
    uint32_t pbt = 0;
    for (;;) {
      record_bail(pbail, pbt);                 // the loop's head: every lane active
      pbail = false;
      uint32_t t = max(tn, next_event());
      // a deferred deadline at or before the tick to decide is drawn first (it can only move later)
      for (;;) {
        uint32_t due = 0;
#pragma unroll
        for (int j = 0; j < F; ++j) due |= (uint32_t)(fdl[j] <= t) << j;
        due &= fpend;
        if (!run || t >= tend || !due) break;
        draw_deadlines(due);
        t = max(tn, next_event());
      }
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
      uint32_t xT = 0, xH = 0;
#pragma unroll
      for (int j = 0; j < F; ++j) {
        if (j == hs) {
          xT = rT[j]; xH = rH[j];
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
      if (bail) {                              // the general tick body runs this tick
        pbail = true;
        pbt = t;
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
        // The whole heartbeat round in this trip when nothing else can happen before its last
        // response: every follower takes the append-entries at t + d (no follower deadline before
        // it; the handler's checks pass), the followers' re-armed deadlines (>= t + d + el_base) and
        // the leader's (t + hb) fall after the responses at t + 2d .. t + 2d + F - 1, and the
        // append-entries come before the launch ends (and no older response is still queued). The
        // responses then run in slot order up to the launch end (the rest stay queued) and stop at
        // one outside the model (the next trip decides it). A deferred deadline counts with its
        // lower bound here (a round not taken is run tick by tick).
        round = rmask == 0 && S.hb >= 2 * d + F && S.el_base >= d + F && tend - t > d;
#pragma unroll
        for (int j = 0; j < F; ++j)
          round = round && fdl[j] >= t + d && qb[j] == 0 && (Lterm < fterm[j] || flen[j] <= fcommit[j]);
      }
      RS_LPH(2);
      // A trip runs exactly one of: a whole round (below), a heartbeat alone (its round did not fit:
      // the append-entries are taken one tick later as `fae`), append-entries that arrived (fae),
      // or queued responses (lres): a heartbeat with a follower still holding an append-entries,
      // and append-entries with responses still queued, were bailed above.
      auto append_entries = [&](uint32_t ta, uint32_t fa) {   // append-entries-handler, followers fa
#pragma unroll
        for (int j = 0; j < F; ++j) {
          if ((fa >> j) & 1) {
            const uint32_t mterm = qT[j], rterm = fterm[j];
            const bool ok = mterm >= fterm[j];
            const uint32_t nfl2 = ok ? (ffl[j] & ~(3u | 15u << 2 | 15u << 6 | 1u << 13)) |
                                           RAFT_FOLLWER | Lid << 6
                                     : ffl[j];
            const uint32_t nterm = ok ? mterm : fterm[j];
            ftr[j] = trace_event(ftr[j], ta, RAFT_MSG_APPEND_ENTRIES, Lid, mterm, nfl2 & 3, nterm, 0);
            if (ok) {
              fcommit[j] = flen[j];                            // apply-entries! (nothing applied)
              fmk[j] &= 0xFFFF0000u;
            }
            fterm[j] = nterm;
            ffl[j] = nfl2;
            // the response: to the leader's RES queue, in sender id order
            rT[j] = rterm; rA[j] = ok ? qa[j] : 0u; rB[j] = 0; rH[j] = ok;
            qA[j] = INF;
            fdl[j] = ta + S.el_base;                           // + the deferred draw
          }
        }
        fpend |= fa;
        qmask &= ~fa;
        rmask = fa;
        resA = ta + d;
        nae += __popc(fa);
        tl = ta;
      };
      // append-response-handler for follower slot j's response at tick tau (core.clj:141-149);
      // false (and nothing done) when it is outside the model: a newer term, a success response
      // that would be checker work, or a failure without the peer's key (NPE)
      auto response = [&](int j, uint32_t tau, uint32_t yT, uint32_t yA, uint32_t yB, uint32_t yH,
                          int32_t& nxj, int32_t& mtj) {
        const uint32_t yid = fk(j) + 1;
        if (yT > Lterm || (yH ? ackbad : ((Lmk >> (16 + yid)) & 1) == 0)) return false;
        rmask &= ~(1u << j);
        Lmk |= yH << (16 + yid);
        nxj = yH ? (int32_t)yB : nxj - 1;
        mtj = yH ? (int32_t)yA : mtj;
        Ldl = tau + S.hb;
        Ltr = trace_event(Ltr, tau, RAFT_MSG_APPEND_RESPONSE, yid, yT, RAFT_LEADER, Lterm, 0);
        ++nar;
        tl = tau;
        return true;
      };
      if (round) {
        // every follower at t + d, then the responses at t + 2d .. t + 2d + F - 1 in slot order (the
        // round's conditions put them all before the launch end and every follower's next event):
        // straight-line code, every index static
        append_entries(t + d, (1u << F) - 1);
        bool go = true;
#pragma unroll
        for (int j = 0; j < F; ++j)     // (a round cut by the launch end leaves the rest queued)
          go = go && t + 2 * d + j < tend &&
               response(j, t + 2 * d + j, rT[j], rA[j], rB[j], rH[j], nx[j], mt[j]);
        if (!rmask) resA = INF;
        if (at_fixed_point()) {
          fixed_point_rounds(t + P);
          tl = tend - 1;                       // nothing of the cluster is left before tend
        }
      } else if (fae || lres) {
        // fae: the append-entries at t, then their responses from t + d in the same trip unless
        // the leader's heartbeat falls due before them. The responses run one per tick, heads in
        // sender order, while nothing else in the cluster is due (the followers' next events and
        // the launch end; the leader's own deadline moves past each); lres: the first one at t
        // was decided above. A response outside the model ends the run and the next trip
        // decides it. A round finished here (one the last launch cut) continues at the fixed point.
        uint32_t tau0 = t;
        if (fae) {
          append_entries(t, fae);
          tau0 = Ldl >= t + d ? t + d : tend;
        }
        uint32_t E = tend;
#pragma unroll
        for (int j = 0; j < F; ++j) E = min(E, min(fdl[j], qA[j]));
        if (lres) E = max(E, t + 1);
        for (uint32_t tau = tau0; rmask && tau < E; ++tau) {
          const int h2 = __builtin_ctz(rmask);
          bool ok = true;
#pragma unroll
          for (int j = 0; j < F; ++j)
            if (j == h2) ok = response(j, tau, rT[j], rA[j], rB[j], rH[j], nx[j], mt[j]);
          if (!ok) break;
          if (!rmask) resA = INF;
        }
        if (at_fixed_point() && Ldl > tl) {
          fixed_point_rounds(Ldl);
          tl = tend - 1;
        }
      }
      RS_LPH(4);
      tn = tl + 1;
    }
    // the draws still owed stay owed in the stored state (FL_DRAW): a cluster at its fixed point
    // makes none at all

#ifdef RS_WAVELOG
    wl_lend = wall_clock64();
#endif
    // ---------------------------------------------------------------- write back
    if (S.shist) {
      // packing key for the next launch (bailed clusters get theirs from the catch-up below); the
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
    // (a cluster that ran its election here changed flags, masks and terms too)
    const bool wfp = !__builtin_amdgcn_ballot_w64(wb && (!fp || el));
    if (wb) {
      // every word of fields DEADLINE..LEN, from registers (LEN unchanged)
      constexpr int NV = HF_NEXT;
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
        v[HF_FLAGS][k] = isL ? Lfl : (fv(ffl) & ~FL_DRAW) | (((fpend >> (lo ? jl : jh)) & 1) ? FL_DRAW : 0u);
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
      auto live = [](int q) { return q >= (int)HOT_CW && q < (int)(HOT_CW + HF_NEXT * N); };
      auto val = [&](int q) { return v[(q - HOT_CW) / N][(q - HOT_CW) % N]; };
      // The changed chunks into the image (in a heartbeat round the deadlines and trace hashes
      // change, all in the block's first line; flags, terms, masks, commits, queue words and rows
      // come back unchanged); the lines they dirty go back to memory whole, below.
      // A wave whose written-back clusters all took the fixed-point path changed nothing past the
      // queue words and the flags' FL_DRAW (masks, terms, commits, lengths and rows are the fixed
      // point's).
      const int ch_end = wfp ? (int)(HOT_CW + (HF_FLAGS + 1) * N + 3) / 4
                             : (int)(HOT_CW + HF_NEXT * N + 3) / 4;
      // (every chunk is written back to the image, changed or not: no branch per chunk)
#pragma unroll
      for (int i = (int)HOT_CW / 4; i < (int)(HOT_CW + HF_NEXT * N + 3) / 4; ++i) {
        if (i < ch_end) {                                    // wave-uniform
          const int q = 4 * i;
          const uint4 x = make_uint4(live(q) ? val(q) : w[q], live(q + 1) ? val(q + 1) : w[q + 1],
                                     live(q + 2) ? val(q + 2) : w[q + 2],
                                     live(q + 3) ? val(q + 3) : w[q + 3]);
          *lds_at<uint4>(img, img_off(lane, i)) = x;
          dl |= (uint32_t)(x.x != w[q] || x.y != w[q + 1] || x.z != w[q + 2] || x.w != w[q + 3])
                << (i / 8);
        }
      }
      if (el) {
        // the words the election changed are compared with the registers it wrote: its lines are
        // dirty; and the new leader's led term (P4), in the image or past it
        dl |= (1u << ((HOT_CW + HF_NEXT * N + 31) / 32)) - 1;
        const uint32_t q = HOT_CW + hf_led(N) * N + L;
        if (q < (uint32_t)IMGC * 4) {
          *lds_at<uint32_t>(img, img_off(lane, q / 4) + 4 * (q % 4)) = Lterm;
          dl |= 1u << (q / 32);
        } else {
          S.hot[(size_t)c * HB + q] = Lterm;
        }
      }
      // the steady certificate for the next launch: the cluster stays at its fixed point
      const uint32_t cn = fp || (full && at_fixed_point_state()) ? (CERT_MAGIC | L) : 0u;
      *lds_at<uint4>(img, img_off(lane, CL_CERT / 4)) = make_uint4(w[4], w[5], w[6], cn);
      dl |= (uint32_t)(cn != w[CL_CERT]);
      // the leader's rows (node L): next / match of peer fk(j) + 1
      if (!wfp) {
#pragma unroll
        for (int j = 0; j < F; ++j) {
          const uint32_t qn = HOT_CW + (HF_NEXT + fk(j)) * N + L;
          const uint32_t qt = HOT_CW + (HF_NEXT + N + fk(j)) * N + L;
          if (nx[j] != nx0[j]) {
            *lds_at<uint32_t>(img, img_off(lane, qn / 4) + 4 * (qn % 4)) = (uint32_t)nx[j];
            dl |= 1u << (qn / 32);
          }
          if (mt[j] != mt0[j]) {
            *lds_at<uint32_t>(img, img_off(lane, qt / 4) + 4 * (qt % 4)) = (uint32_t)mt[j];
            dl |= 1u << (qt / 32);
          }
        }
      }
    }
    // queues back to the rings, heads at slot 0 (a message in flight at the launch's end: rare)
    if (__builtin_amdgcn_ballot_w64(wb && (qmask || rmask))) {            // wave-uniform
#pragma unroll
      for (int j = 0; j < F; ++j) {
        if (wb && ((qmask >> j) & 1)) {
          uint4* dp = reinterpret_cast<uint4*>(qslots(S, c * N + fk(j), 0));
          dp[0] = make_uint4(qA[j], RAFT_MSG_APPEND_ENTRIES | Lid << 3, qT[j], qa[j]);
          dp[1] = make_uint4(qb[j], 0, 0, 0);
        }
      }
      uint4* rp = reinterpret_cast<uint4*>(qslots(S, c * N + L, 1));
      uint32_t n = 0;
#pragma unroll
      for (int j = 0; j < F; ++j) {
        if (wb && ((rmask >> j) & 1)) {
          const uint32_t sid = fk(j) + 1;
          uint4* dp = rp + 2 * n;
          dp[0] = make_uint4(resA, RAFT_MSG_APPEND_RESPONSE | sid << 3 | rH[j] << 7, rT[j], rA[j]);
          dp[1] = make_uint4(rB[j], 0, 0, 0);
          ++n;
        }
      }
    }
  }   // the general path
  // Dirty lines back to memory whole: a wave instruction writes eight clusters' line (8 lanes x
  // 16 B each), read from the image (line ln of cluster cc is its chunks 8 ln .. 8 ln + 7): the
  // eight reads of a line first, then the stores. The stores write through to memory (sc1: the
  // lines leave the XCD's L2 as the waves end, not at the launch's end; the next launch reads them
  // from the Infinity Cache either way). They are not in the compiler's wait counts: the catch-up
  // below waits for them itself.
  {
    uint32_t* const wbase = S.hot + (size_t)cbase * HB;      // the wave's first block
    const uint32_t sub = lane >> 3, q8 = lane & 7;
#pragma unroll
    for (int ln = 0; ln < IMGC / 8; ++ln) {
      const uint64_t bal = __builtin_amdgcn_ballot_w64((dl >> ln) & 1);
      if (!bal) continue;                                  // wave-uniform
      uint4 xs[8];
#pragma unroll
      for (int gq = 0; gq < 8; ++gq)
        xs[gq] = *lds_at<const uint4>(img, img_off(8 * gq + sub, 8 * ln + q8));
#pragma unroll
      for (int gq = 0; gq < 8; ++gq) {
        const uint32_t cc = 8 * gq + sub;
        if ((bal >> cc) & 1) {
          typedef uint32_t v4u __attribute__((ext_vector_type(4)));
          const v4u xv = {xs[gq].x, xs[gq].y, xs[gq].z, xs[gq].w};
          uint32_t* const dst = wbase + cc * HB + 4 * (8 * ln + q8);
          asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(dst), "v"(xv) : "memory");
        }
      }
    }
  }
#ifdef RS_WAVELOG
  {
    const uint64_t wl_end = wall_clock64();
    const uint32_t wl_events = nhb + nae + nar;
    const uint32_t emax = ~wave_min(~wl_events), emin = wave_min(wl_events);
    if (lane == 0 && S.wavelog) {
      uint32_t hw, xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      uint4* rec = reinterpret_cast<uint4*>(S.wavelog + (size_t)(blockIdx.x * 4 + wave) * 32);
      rec[0] = make_uint4((uint32_t)wl_start, (uint32_t)(wl_start >> 32), (uint32_t)wl_end,
                          (uint32_t)(wl_end >> 32));
      rec[1] = make_uint4(wl_trips, hw, xcc, wl_first);
      rec[2] = make_uint4((uint32_t)(wl_loop - wl_start), (uint32_t)(wl_lend - wl_start), emin, emax);
      rec[3] = make_uint4(wl_ph[0], wl_ph[1], wl_ph[2], wl_ph[3]);
      rec[4] = make_uint4(wl_ph[4], 0, 0, 0);
      rec[5] = make_uint4((uint32_t)(wl_x1 - wl_start), (uint32_t)(wl_x2 - wl_start),
                          (uint32_t)(wl_x3 - wl_start), 0);
    }
  }
#endif
  // counters: heartbeats, append-entries, append-responses; every message is delivered. One
  // wave-wide sum each, added by five lanes to the wave's copy of the counter block.
  // Elections run here add a timeout, F request-votes and F vote responses, a leader, and the
  // request-vote, vote-response and append-entries messages (3F; the responses are in a).
  {
    const uint32_t h = wave_sum(nhb), a = wave_sum(nae), r = wave_sum(nar);
    unsigned long long* const ctr =
        S.ctr + (size_t)((blockIdx.x * 4 + wave) % CTR_COPIES) * CTR_STRIDE;
    if (lane < 5) {
      const uint32_t msgs = (uint32_t)F * h + a;
      const int idx = lane == 0 ? RAFT_CTR_EV_HEARTBEAT : lane == 1 ? RAFT_CTR_EV_AE
                    : lane == 2 ? RAFT_CTR_EV_AR : lane == 3 ? RAFT_CTR_SENT : RAFT_CTR_DELIVERED;
      const uint32_t v = lane == 0 ? h : lane == 1 ? a : lane == 2 ? r : msgs;
      if (v) atomicAdd(&ctr[idx], (unsigned long long)v);
    }
    if (__builtin_amdgcn_ballot_w64(el)) {                   // wave-uniform
      // per election: el_to timeouts, F request-votes and F vote responses per timeout, one
      // leader, and the request-vote, vote-response and append-entries messages
      const uint32_t ne = wave_sum(el ? 1u : 0u), nt = wave_sum(el_to);
      if (lane < 6) {
        const int idx = lane == 0 ? RAFT_CTR_EV_TIMEOUT : lane == 1 ? RAFT_CTR_EV_RV
                      : lane == 2 ? RAFT_CTR_EV_VR : lane == 3 ? RAFT_CTR_LEADERS
                      : lane == 4 ? RAFT_CTR_SENT : RAFT_CTR_DELIVERED;
        const uint32_t v = lane == 0 ? nt : lane == 3 ? ne : lane <= 2 ? (uint32_t)F * nt
                                                                   : (uint32_t)F * (2 * nt + ne);
        atomicAdd(&ctr[idx], (unsigned long long)v);
      }
    }
  }
  // ---------------------------------------------------------------- catch-up
  // The wave's bailed clusters, each from the tick it stopped before to the launch's end, through
  // the general tick body, with the wave's image as its LDS block (the write-back above read the
  // image: a wave's LDS operations complete in order). The blocks it reads are this wave's own
  // stores: they are waited for first.
  if (nbw) {                                                  // wave-uniform
    if (lane == 0) atomicAdd(S.nbail, nbw);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    tick_wave<N, false, false, true, true>(S, t0, nt, reinterpret_cast<uint32_t*>(img), (int)lane,
                                           0, 1, blc, nbw, blt, blockIdx.x * 4 + wave);
  }
#ifdef RS_WAVELOG   // the wave's end: its stores issued, counted, its catch-up run
  if (lane == 0 && S.wavelog) {
    const uint64_t wl_done = wall_clock64();
    uint32_t* rec = S.wavelog + (size_t)(blockIdx.x * 4 + wave) * 32;
    rec[17] = (uint32_t)wl_done;
    rec[18] = (uint32_t)(wl_done >> 32);
  }
#endif
}

hipError_t configure_steady() {
  hipError_t e = hipSuccess;
#define RS_CFG(NN)                                                                         \
  if (e == hipSuccess)                                                                     \
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(steady_lane_kernel<NN>),         \
                            hipFuncAttributeMaxDynamicSharedMemorySize,                    \
                            (int)steady_lds_bytes<NN>());
  RS_CFG(2) RS_CFG(3) RS_CFG(4) RS_CFG(5)
#undef RS_CFG
  return e;
}

// The steady kernel for N <= 5 (LITE launches; the caller checks): one thread per cluster, in id
// order. Its timestamps go into ev0/ev1 through its dispatch packet.
hipError_t launch_steady(const DevSim& S, uint32_t t0, uint32_t nt, hipStream_t st,
                         hipEvent_t ev0, hipEvent_t ev1) {
  if (S.perm) return hipErrorInvalidValue;                     // clusters in id order only
  const dim3 grid((S.C + LANE_WG - 1) / LANE_WG);
  switch (S.N) {
#define RS_LANE(NN)                                                                             \
  case NN:                                                                                      \
    hipExtLaunchKernelGGL((steady_lane_kernel<NN>), grid, dim3(LANE_WG), steady_lds_bytes<NN>(), \
                          st, ev0, ev1, 0, S, t0, nt);                                          \
    break;
    RS_LANE(2) RS_LANE(3) RS_LANE(4) RS_LANE(5)
#undef RS_LANE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace rs

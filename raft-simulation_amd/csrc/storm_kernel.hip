// storm_kernel.hip — the storm ticks of a fresh handle, one lane per cluster, for gfx950 (MI355X).
//
// Before any timer can fire in a handle fresh from init-node (ticks [0, el_base), tick_wave.hpp's
// STORM) every node is a follower without a leader id and the only events are client-sets: P0
// injects one into a node's REQ ring, the node takes it (client-set-handler, core.clj:151-160) and
// redirects it (server.clj:62-63) to a rand-nth peer drawn from its EVENT word 2, arriving the next
// tick, until it has used its hops (SIM_SPEC D14, D15). Each such event touches one node and one
// queue, so a lane can run a whole cluster: this kernel takes, per lane, the cluster's events one
// at a time in the order the general body runs them -- by tick, and within a tick the injection
// (P0) first, then the nodes in id order (P1), each appending its redirect to the receiver's ring
// at once (P2 inserts in sender order, and a redirect arriving at t + 1 is behind anything a node
// could take at t) -- with the cluster's rings in registers, at most QC messages each. A node takes
// one message per tick (D2): node k's next event is at max(its head's arrival, the tick after its
// last event). A lane whose cluster does not fit (a ring would pass QC messages, a state that is
// not a storm state) leaves it untouched and lists it; the host then runs the listed clusters
// through the general STORM body (tick_kernel) over the same ticks. Results are the general
// kernel's either way.
//
// Against the lane-per-node STORM body, whose trips run every phase for a wave of twelve clusters
// of which a few nodes act, one event here costs one Philox draw and a few dozen selects for 64
// clusters at once.
#include <hip/hip_ext.h>

#include "tick_wave.hpp"

namespace rs {

constexpr int STORM_QC = 4;   // messages a node's ring holds here (the general body: inbox_cap)

template <int N>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(N <= 5 ? 4 : 1, 8)))
storm_lane_kernel(DevSim S, uint32_t t0, uint32_t nt,
                                                        uint32_t* bail_list, uint32_t* bail_count) {
  constexpr int QC = STORM_QC;
  constexpr uint32_t HB = hot_block_words(N);
  const uint32_t lane = threadIdx.x;
  const uint32_t c0 = blockIdx.x * 64 + lane;
  const bool active = c0 < S.C;
  const uint32_t c = active ? c0 : 0u;
  const uint32_t g = S.goff + c;
  const uint32_t tend = t0 + nt;
  KDevSim* const K = kargs();
  const uint32_t el_base = K->el_base, el_span = K->el_span, R = K->client_redirects;
  (void)el_base;
  const bool spec = (K->variant & RAFT_VARIANT_SPEC) != 0;
  const uint32_t QL = min((uint32_t)QC, S.Q);       // a full ring: the general body's to run
  uint32_t* const hc = S.hot + (size_t)c * HB;
  uint32_t* const hp = hc + HOT_CW;

  // ------------------------------------------------------------------ load
  // Registers per node: its trace hash, ring count, the tick after its last event, and QC messages
  // as (arrival | hops << 28, value) -- the host runs this kernel only while ticks stay below 2^28
  // and hops below 16. Every node of a storm cluster has the same term and role (init-node's),
  // and a node's deadline after the launch follows from its last event (redrawn at the end), so
  // neither is held per event: 12 words per node.
  constexpr uint32_t AM = (1u << 28) - 1;
  uint32_t cnext = hc[3], ccount = hc[4];
  uint32_t qn[N], nb[N];
  uint64_t tr[N];
  uint32_t qa[N][QC], qv[N][QC];
  const uint32_t term = hp[HF_TERM * N], role = hp[HF_FLAGS * N] & 3;
  bool ok = active && hc[CL_CERT] == 0;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const uint32_t fl = hp[HF_FLAGS * N + k], qm = hp[HF_QMETA * N + k];
    tr[k] = (uint64_t)hp[HF_TRACE_HI * N + k] << 32 | hp[HF_TRACE_LO * N + k];
    qn[k] = (qm >> 4) & 31;
    nb[k] = t0;
    // a follower without a leader id, not halted, no owed draw, no responses, no timer inside the
    // launch; the cluster's common term and role
    ok = ok && (fl & ~(15u << 2)) == role && role != RAFT_LEADER && role != RAFT_CANDIDATE &&
         hp[HF_TERM * N + k] == term && ((qm >> 13) & 31) == 0 && qn[k] <= QL &&
         hp[HF_DEADLINE * N + k] >= tend;
#pragma unroll
    for (int s = 0; s < QC; ++s) qa[k][s] = qv[k][s] = 0;
  }
  // the queued client-sets (a storm launch after another), all loads issued together
  uint32_t anyq = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) anyq |= qn[k];
  if (__builtin_amdgcn_ballot_w64(ok && anyq)) {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const uint32_t qm = hp[HF_QMETA * N + k], h = qm & 15;
      const uint32_t* qb = qslots(S, c * N + k, 0);
      const size_t qs = qstride(S, 0);
#pragma unroll
      for (int s = 0; s < QC; ++s) {
        if (ok && (uint32_t)s < qn[k]) {
          const uint32_t slot = wrapq(h + s, S.Q);
          const uint4 m0 = *reinterpret_cast<const uint4*>(qb + slot * qs);
          const uint4 m1 = *reinterpret_cast<const uint4*>(qb + slot * qs + 4);
          ok = ok && m0.y == RAFT_MSG_CLIENT_SET && m0.z == 0 && !m1.y && !m1.z && !m1.w &&
               m0.x <= AM && m1.x < 16;
          qa[k][s] = m0.x | m1.x << 28;
          qv[k][s] = m0.w;
        }
      }
    }
  }

  // ------------------------------------------------------------------ events
  uint32_t n_inj = 0, n_del = 0, n_cs = 0, n_red = 0, n_ab = 0;
  uint32_t trips = 0, tlast = INF;                // the cluster's event ticks (its packing key)
  bool run = ok;
  // append message (arrival | hops << 28, value) to node j's ring (j a runtime index: selects)
  auto append = [&](uint32_t j, uint32_t ah, uint32_t val) {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const bool me = (uint32_t)k == j;
#pragma unroll
      for (int s = 0; s < QC; ++s) {
        const bool at = me && qn[k] == (uint32_t)s;
        qa[k][s] = at ? ah : qa[k][s];
        qv[k][s] = at ? val : qv[k][s];
      }
      qn[k] += me ? 1u : 0u;
    }
  };
  for (;;) {
    // the lane's next event: the injection, then the nodes in id order, at the earliest tick
    uint32_t te = cnext, who = N;             // N: the injection
#pragma unroll
    for (int k = N - 1; k >= 0; --k) {
      const uint32_t a = qn[k] ? max(qa[k][0] & AM, nb[k]) : INF;
      const bool better = a < te || (a == te && who != N);
      te = better ? a : te;
      who = better ? (uint32_t)k : who;
    }
    const bool go = run && te < tend;
    if (!__builtin_amdgcn_ballot_w64(go)) break;
    if (!go) continue;
    const bool inj = who == (uint32_t)N;
    trips += te != tlast;
    tlast = te;
    // one Philox pass: the client draw of injection ccount, or node who's EVENT draw at te
    const uint4 w = philox(g, inj ? (uint32_t)P_CLIENT << 8 : (who + 1) | P_EVENT << 8,
                           inj ? ccount : te, 0, S.key0, S.key1);
    uint32_t dst = 0, ah = 0, val = 0;          // the message this event queues (dst 1-based)
    if (inj) {                                  // P0 (SIM_SPEC D14): into the target's ring
      dst = __umulhi(w.y, N) + 1;
      ah = te;
      val = w.z;
      ++n_inj;
      ccount += 1;
      cnext = on_tick(on_index(te, S) + 1 + client_gap(w.w, PowersS(K->client_pw), K->client_top),
                      K->client_period, kdiv(K->div_burst));
    } else {                                    // P1: node who takes its head
      uint32_t hops = 0;
#pragma unroll
      for (int k = 0; k < N; ++k) {
        if ((uint32_t)k == who) {
          hops = qa[k][0] >> 28;
          val = qv[k][0];
#pragma unroll
          for (int s = 0; s + 1 < QC; ++s) {
            qa[k][s] = qa[k][s + 1];
            qv[k][s] = qv[k][s + 1];
          }
          qn[k] -= 1;
          nb[k] = te + 1;
          tr[k] = trace_event(tr[k], te, RAFT_MSG_CLIENT_SET, 0, 0, role, term, 0);
        }
      }
      ++n_cs;
      if (hops >= R) {
        ++n_ab;                                 // the client gives up (D15)
      } else {                                  // redirect-client: a rand-nth peer, next tick
        const uint32_t i = __umulhi(w.z, N - 1), id = who + 1;
        dst = i + 1 < id ? i + 1 : i + 2;
        ah = (te + 1) | (hops + 1) << 28;
        ++n_red;
      }
    }
    if (dst) {
      uint32_t q = 0;
#pragma unroll
      for (int k = 0; k < N; ++k) q = (uint32_t)k == dst - 1 ? qn[k] : q;
      if (q >= QL) {                            // the ring would pass what lanes hold here
        run = false;
        ok = false;
        continue;
      }
      append(dst - 1, ah, val);
      ++n_del;
    }
  }

  // ------------------------------------------------------------------ write back or list
  if (!ok) n_inj = n_del = n_cs = n_red = n_ab = 0;    // a listed cluster is counted by its rerun
  if (active && !ok) {
    const uint32_t i = atomicAdd(bail_count, 1u);
    bail_list[i] = c;
  }
  if (ok) {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      // generate-timeout (core.clj:171-174) at the node's last event, whose EVENT draw the
      // general body made there (Spec-Raft keeps the timer)
      if (!spec && nb[k] != t0) {
        const uint4 wd = event_draw(g, k + 1, nb[k] - 1, S);
        hp[HF_DEADLINE * N + k] = nb[k] - 1 + el_base + __umulhi(wd.y, el_span);
      }
      hp[HF_TRACE_LO * N + k] = (uint32_t)tr[k];
      hp[HF_TRACE_HI * N + k] = (uint32_t)(tr[k] >> 32);
      hp[HF_QMETA * N + k] = pack_qmeta(0, qn[k], 0, 0);
      uint32_t tail = 0;
#pragma unroll
      for (int s = 0; s < QC; ++s) tail = (uint32_t)s + 1 == qn[k] ? qa[k][s] & AM : tail;
      hp[HF_REQ_ARR * N + k] = qn[k] ? qa[k][0] & AM : INF;
      hp[HF_REQ_TAIL * N + k] = qn[k] ? tail : 0u;
      uint32_t* const qb = qslots(S, c * N + k, 0);
      const size_t qs = qstride(S, 0);
#pragma unroll
      for (int s = 0; s < QC; ++s) {
        if ((uint32_t)s < qn[k]) {
          *reinterpret_cast<uint4*>(qb + s * qs) =
              make_uint4(qa[k][s] & AM, RAFT_MSG_CLIENT_SET, 0, qv[k][s]);
          *reinterpret_cast<uint4*>(qb + s * qs + 4) = make_uint4(qa[k][s] >> 28, 0, 0, 0);
        }
      }
    }
    hc[3] = cnext;
    hc[4] = ccount;
    // the packing key for the next launch, as the general body writes it with client traffic: the
    // busiest clusters first (tick_wave.hpp's write-back; listed clusters get theirs from the rerun)
    if (S.shist) {
      const uint32_t key = SCHED_BUCKETS - 2 - min(trips, SCHED_BUCKETS - 2);
      S.skey[c] = key;
      atomicAdd(&S.shist[key], 1u);
    }
  }
  // counters: one wave sum each, added by five lanes
  const uint32_t a0 = wave_sum(n_inj), a1 = wave_sum(n_del), a2 = wave_sum(n_cs),
                 a3 = wave_sum(n_red), a4 = wave_sum(n_ab);
  unsigned long long* const ctr = S.ctr + (size_t)(blockIdx.x % CTR_COPIES) * CTR_STRIDE;
  if (lane < 5) {
    const int idx = lane == 0 ? RAFT_CTR_CLIENT_INJECTED : lane == 1 ? RAFT_CTR_DELIVERED
                  : lane == 2 ? RAFT_CTR_EV_CS : lane == 3 ? RAFT_CTR_REDIRECTS
                  : RAFT_CTR_CLIENT_ABANDONED;
    const uint32_t v = lane == 0 ? a0 : lane == 1 ? a1 : lane == 2 ? a2 : lane == 3 ? a3 : a4;
    if (v) atomicAdd(&ctr[idx], (unsigned long long)v);
  }
}

hipError_t launch_storm_body(const DevSim& S, uint32_t t0, uint32_t nt, hipStream_t st,
                             hipEvent_t ev0, hipEvent_t ev1);

// The storm ticks [t0, t0 + nt) of every cluster: this kernel, then the general STORM body over
// the clusters it listed (S.perm = the list, S.nslots = its length). ev0 / ev1: the first kernel's
// start and the second's end.
hipError_t launch_storm(const DevSim& S, uint32_t t0, uint32_t nt, hipStream_t st, hipEvent_t ev0,
                        hipEvent_t ev1) {
  uint32_t* const bail_list = S.storm_list;
  uint32_t* const bail_count = S.storm_count;
  hipError_t e = hipMemsetAsync(bail_count, 0, sizeof(uint32_t), st);
  if (e != hipSuccess) return e;
  const dim3 grid((S.C + 63) / 64);
  switch (S.N) {
#define RS_STORM(NN)                                                                            \
  case NN:                                                                                      \
    hipExtLaunchKernelGGL((storm_lane_kernel<NN>), grid, dim3(64), 0, st, ev0, nullptr, 0, S, t0, \
                          nt, bail_list, bail_count);                                           \
    break;
    RS_STORM(2) RS_STORM(3) RS_STORM(4) RS_STORM(5) RS_STORM(6) RS_STORM(7) RS_STORM(8)
    RS_STORM(9)
#undef RS_STORM
    default: return hipErrorInvalidValue;
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  DevSim F = S;
  F.perm = bail_list;
  F.nslots = bail_count;
  return launch_storm_body(F, t0, nt, st, nullptr, ev1);
}

}  // namespace rs

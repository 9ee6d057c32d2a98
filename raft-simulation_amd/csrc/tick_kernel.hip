// tick_kernel.hip — the general tick kernel for gfx950 (MI355X) and its helpers: the wave packing
// (schedule kernels), init-node, the per-cluster digest and the launchers. The tick body itself is
// tick_wave (tick_wave.hpp).
#include <hip/hip_ext.h>

#include "tick_wave.hpp"

namespace rs {

// The general tick kernel: one wave per workgroup (wave lifetimes differ by up to 2x under load,
// and a multi-wave workgroup holds its CU slot and LDS until its slowest wave ends; measured:
// 4-wave workgroups 1-2 % slower on C2/C3/C4). The grid covers the packing's slot bound. The
// compiler is asked for 4 waves per SIMD (<= 128 VGPRs) where it meets that without spilling:
// N <= 5, and the faithful kernels up to N = 6 (N = 7, 8 would spill).
template <int N, bool TRACE, bool SPEC, bool LITE, bool STORM = false>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(STORM && N <= 5 ? 5 : !TRACE && (N <= 5 || (!SPEC && N <= 6)) ? 4 : 1, 8)))
tick_kernel(DevSim S, uint32_t t0, uint32_t nt) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  tick_wave<N, TRACE, SPEC, LITE, false, STORM>(S, t0, nt, smem, (int)threadIdx.x, blockIdx.x,
                                                gridDim.x, S.perm, S.perm ? *S.nslots : S.C,
                                                nullptr, blockIdx.x);
}

// RAFT_SCHED_ALIGNED wave packing: a counting sort of the clusters by their next event tick
// (min over running nodes of deadline and queue heads, and the next client-set) relative to the
// launch's first tick. Clusters with the same next event then share waves, and a steady-state
// cluster's later events (heartbeat every hb ticks) stay aligned with its wave mates', so a
// wave's active ticks are nearly those of one cluster instead of the union of twelve. The order
// inside a bucket is whatever the LDS atomics give: any packing yields identical results.
//
// sched_key_kernel: keys + histogram from the state (first launch, or after host writes);
// the tick kernel writes both at its end for the next launch.
__global__ void sched_key_kernel(DevSim S, uint32_t t0) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= S.C) return;
  uint32_t m = hot_cl(S, c)[3];
  for (uint32_t k = 0; k < S.N; ++k) {
    const uint32_t* h = hot_node(S, c, k);
    if ((h[HF_FLAGS * S.N] >> 10) & 7) continue;
    const uint32_t qm = h[HF_QMETA * S.N];
    const QueueR rq = {0, (qm >> 4) & 31, h[HF_REQ_ARR * S.N], 0},
                 rs = {0, (qm >> 13) & 31, h[HF_RES_ARR * S.N], 0};
    m = min(m, sched_key_of(h[HF_DEADLINE * S.N], rq, rs));
  }
  const uint32_t key = sched_bucket(m, t0);
  S.skey[c] = key;
  atomicAdd(&S.shist[key], 1u);
}

// Packing keys in order. Launches with client traffic pack by activity (the tick kernel's key:
// event ticks run in the previous launch) and keep waves key-pure (a zero-tick window, padded
// slots): a wave lasts as long as its busiest cluster. Launches without client traffic (C2) pack
// by next event tick with no padding: with per-cluster clocks, clusters whose heartbeat rounds are
// a few ticks apart still run the same phase on the same trips (each on its own tick), so a wave
// needs similar keys, not equal ones. Measured (C2 tick kernel per launch): with one wave-wide
// clock a one-tick window cost 0.115 ms against 0.093 key-pure (most waves straddled two keys and
// ran the broadcast and the replies side by side); with per-cluster clocks key-pure 0.094 ms,
// one-tick window 0.087, unpadded 0.087 (fewest waves). C3 with activity keys: unpadded -1.6 %,
// C4-N9 +3.8 %: key-pure kept there. Wider windows under one wave-wide clock mixed up to ten
// phases per wave (the slowest C2 wave 60 active ticks).
//
// The plan is made per chunk of SCHED_CHUNK buckets, one thread each, restarting at every chunk;
// chunk totals are whole waves. If the padded plan would exceed the grid bound
// (sched_slots_bound), every chunk falls back to the plain counting sort.
constexpr uint32_t SCHED_CHUNK = 16;
constexpr uint32_t SCHED_CHUNKS = SCHED_BUCKETS / SCHED_CHUNK;     // 1024, one per thread
static_assert(SCHED_CHUNKS == SCHED_PLAN_CHUNKS, "grid bound covers one partial wave per chunk");
// Workgroups of the schedule kernel, each owning SCHED_KB buckets. Measured per rebuild (C2 65,536
// / C3 1M clusters): 16 blocks 27.4 us / -, 64: 14.5 / 443 us, 256: 11.3 / 402 us, 512: 16.6 /
// 322 us, 1024: 28.5 / 337 us (every block reads all keys; fewer buckets per block place faster).
constexpr uint32_t SCHED_RANGE_BLOCKS = 256;
constexpr uint32_t SCHED_KB = SCHED_BUCKETS / SCHED_RANGE_BLOCKS;  // 64 buckets per block
constexpr uint32_t SCHED_WINDOW = 0;
static_assert(SCHED_CHUNKS == 1024 && SCHED_KB % SCHED_CHUNK == 0, "one chunk per thread");

template <uint32_t CPW>
__device__ uint32_t plan_chunk(const uint32_t (&cnt)[SCHED_CHUNK], uint32_t (&st)[SCHED_CHUNK],
                               bool window) {
  uint32_t slot = 0, f = 0;                           // f = slot % CPW
  int kw = -(int)SCHED_CHUNK;                         // bucket where the open wave began
#pragma unroll
  for (uint32_t i = 0; i < SCHED_CHUNK; ++i) {
    const uint32_t n = cnt[i];
    if (window && n && f && (int)i > kw + (int)SCHED_WINDOW) {
      slot += CPW - f;                                // close the open wave, pad its tail
      f = 0;
    }
    st[i] = slot;
    if (n && (f == 0 || f + n > CPW)) kw = (int)i;    // the wave open after this bucket began here
    slot += n;
    f = (f + n) % CPW;
  }
  return slot + (f ? CPW - f : 0);
}

// One launch: every block plans all chunks from the histogram (L2-resident, 64 KiB), scans the
// chunk totals, and places the clusters of its own SCHED_KB-bucket range at their bucket's slot plus
// their rank (LDS atomics, no global ones). It first marks its slots empty (padding reads INF).
// Each block reads all keys (L2-resident, 4 B per cluster). The histogram is double-buffered: this
// kernel reads S.shist and zeroes `zero`, which the next tick launch fills (the host swaps the
// two). Block 0 publishes the slot count the tick kernel's grid covers.
template <uint32_t CPW>
__global__ void __launch_bounds__(1024) sched_range_kernel(DevSim S, uint32_t* zero,
                                                           uint32_t* perm, uint32_t* nslots) {
  constexpr uint32_t KB = SCHED_KB;
  __shared__ uint32_t cbase[SCHED_CHUNKS + 1];
  __shared__ uint32_t loff[KB];
  __shared__ uint32_t wsum[16];
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint32_t k0 = blockIdx.x * KB;
  if (t < KB) zero[k0 + t] = 0;
  uint32_t cnt[SCHED_CHUNK], st[SCHED_CHUNK];
  const uint4* h4 = reinterpret_cast<const uint4*>(S.shist + t * SCHED_CHUNK);
#pragma unroll
  for (uint32_t i = 0; i < SCHED_CHUNK / 4; ++i) {
    const uint4 v = h4[i];
    cnt[4 * i] = v.x; cnt[4 * i + 1] = v.y; cnt[4 * i + 2] = v.z; cnt[4 * i + 3] = v.w;
  }
  // client traffic (activity keys): key-pure waves; otherwise keys in order without padding
  uint32_t tot = plan_chunk<CPW>(cnt, st, S.client_ppm != 0);
  // exclusive scan of the chunk totals: wave scan, then the 16 wave totals
  uint32_t inc = tot;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t x = __shfl_up(inc, d);
    if (lane >= d) inc += x;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t all = 0, below = 0;
#pragma unroll
  for (uint32_t j = 0; j < 16; ++j) {
    below += j < w ? wsum[j] : 0u;
    all += wsum[j];
  }
  if (all > sched_slots_bound(S.C, 64 / CPW)) {          // block-uniform: plain sort fits
    __syncthreads();
    tot = plan_chunk<CPW>(cnt, st, false);                                // plain counting sort
    inc = tot;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t x = __shfl_up(inc, d);
      if (lane >= d) inc += x;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    all = below = 0;
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
      below += j < w ? wsum[j] : 0u;
      all += wsum[j];
    }
  }
  const uint32_t base = below + inc - tot;
  cbase[t] = base;
  if (t == SCHED_CHUNKS - 1) cbase[SCHED_CHUNKS] = all;
  if (blockIdx.x == 0 && t == 0) *nslots = all;
  constexpr uint32_t CPB = KB / SCHED_CHUNK;            // chunks per block
  if (t / CPB == blockIdx.x) {                           // this block's chunks: bucket offsets
#pragma unroll
    for (uint32_t i = 0; i < SCHED_CHUNK; ++i) loff[(t % CPB) * SCHED_CHUNK + i] = base + st[i];
  }
  __syncthreads();
  const uint32_t s0 = cbase[blockIdx.x * CPB], s1 = cbase[(blockIdx.x + 1) * CPB];
  for (uint32_t i = s0 + t; i < s1; i += 1024) perm[i] = INF;
  __syncthreads();                      // the empty marks land before the placements
  // keys as 16-byte vectors, sixteen loads in flight per thread (64 keys), then the scalar tail
  const uint32_t C4 = S.C / 4;
  const uint4* k4 = reinterpret_cast<const uint4*>(S.skey);
  for (uint32_t vb = t; vb < C4; vb += 16 * 1024) {
    uint4 v[16];
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
      const uint32_t q = vb + j * 1024;
      v[j] = q < C4 ? k4[q] : make_uint4(INF, INF, INF, INF);
    }
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
      const uint32_t c = 4 * (vb + j * 1024);
      const uint32_t r0 = v[j].x - k0, r1 = v[j].y - k0, r2 = v[j].z - k0, r3 = v[j].w - k0;
      if (r0 < KB) perm[atomicAdd(&loff[r0], 1u)] = c;
      if (r1 < KB) perm[atomicAdd(&loff[r1], 1u)] = c + 1;
      if (r2 < KB) perm[atomicAdd(&loff[r2], 1u)] = c + 2;
      if (r3 < KB) perm[atomicAdd(&loff[r3], 1u)] = c + 3;
    }
  }
  for (uint32_t c = 4 * C4 + t; c < S.C; c += 1024) {
    const uint32_t r = S.skey[c] - k0;
    if (r < KB) perm[atomicAdd(&loff[r], 1u)] = c;
  }
}

hipError_t launch_sched_key(const DevSim& S, uint32_t t0, hipStream_t st) {
  hipLaunchKernelGGL(sched_key_kernel, dim3((S.C + 255) / 256), dim3(256), 0, st, S, t0);
  return hipGetLastError();
}

hipError_t launch_sched_perm(const DevSim& S, uint32_t* zero, uint32_t* perm, uint32_t* nslots,
                             hipStream_t st) {
  switch (64 / S.N) {
#define RS_PLAN(CPW)                                                                             \
  case CPW:                                                                                      \
    hipLaunchKernelGGL(sched_range_kernel<CPW>, dim3(SCHED_RANGE_BLOCKS), dim3(1024), 0, st, S,  \
                       zero, perm, nslots);                                                      \
    break;
    RS_PLAN(32) RS_PLAN(21) RS_PLAN(16) RS_PLAN(12) RS_PLAN(10) RS_PLAN(9) RS_PLAN(8) RS_PLAN(7)
#undef RS_PLAN
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// Initial state: init-node (core.clj:31-38) and an empty log (log.clj:33-34) for every node.
__global__ void init_kernel(DevSim S) {
  const uint32_t gi = blockIdx.x * blockDim.x + threadIdx.x;
  if (gi >= S.NN) return;
  const uint32_t c = gi / S.N, id = gi - c * S.N + 1;
  const uint4 w = philox(S.goff + c, id | P_INIT << 8, 0, 0, S.key0, S.key1);
  uint32_t* h = hot_node(S, c, id - 1);
  const uint32_t N = S.N;
  for (uint32_t f = 0; f <= hf_led(N); ++f) h[f * N] = 0;          // incl. next / match
  h[HF_TERM * N] = 1;
  h[HF_DEADLINE * N] = S.el_base + __umulhi(w.y, S.el_span);
  h[HF_REQ_ARR * N] = INF; h[HF_RES_ARR * N] = INF;
  h[HF_TRACE_LO * N] = 0x84222325u; h[HF_TRACE_HI * N] = 0xCBF29CE4u;
  S.ccount[gi] = 0;
  if (id == 1) {                                   // cluster record: no hwm, first client-set
    uint32_t first = INF;
    if (S.client_ppm) {
      const uint4 d = philox(S.goff + c, P_CLIENT << 8, 0, 1, S.key0, S.key1);
      first = on_tick(client_gap(d.x, S.client_pw, S.client_top), S.client_period, S.div_burst);
    }
    uint32_t* cw = hot_cl(S, c);
    for (int i = 0; i < 8; ++i) cw[i] = 0;
    cw[3] = first;
  }
}

// Per-cluster canonical digest (SIM_SPEC §6), one thread per cluster.
__global__ void digest_kernel(DevSim S, uint32_t c0, uint32_t nc, unsigned long long* out) {
  const uint32_t ci = blockIdx.x * blockDim.x + threadIdx.x;
  if (ci >= nc) return;
  const uint32_t c = c0 + ci, N = S.N;
  uint64_t h = 0xCBF29CE484222325ull;
  for (uint32_t k = 0; k < N; ++k) {
    const uint32_t gi = c * N + k;
    const uint32_t* hw = hot_node(S, c, k);
    const uint32_t fl = hw[HF_FLAGS * N], mk = hw[HF_MASKS * N], qm = hw[HF_QMETA * N];
    const uint32_t dl = (fl & FL_DRAW) ? exact_deadline(S.goff + c, k + 1, hw[HF_DEADLINE * N],
                                                        S.el_base, S.el_span, S.key0, S.key1)
                                       : hw[HF_DEADLINE * N];
    const uint32_t w[12] = {fl & 3, (fl >> 2) & 15, (fl >> 6) & 15, (fl >> 10) & 7,
                            (fl >> 13) & 1, (fl >> 14) & 1, mk & 0xFFFF, mk >> 16,
                            hw[HF_TERM * N], hw[HF_COMMIT * N], hw[HF_LEN * N], dl};
    for (int i = 0; i < 12; ++i) h = fnv(h, w[i]);
    for (uint32_t p = 0; p < 2 * N; ++p) h = fnv(h, hw[(HF_NEXT + p) * N]);   // next, then match
    h = fnv(h, hw[hf_led(N) * N]);
    h = fnv(h, hw[HF_TRACE_LO * N]);
    h = fnv(h, hw[HF_TRACE_HI * N]);
    h = fnv(h, hw[hf_abase(N) * N]);
    h = fnv(h, hw[hf_afront(N) * N]);
    const uint32_t cc = S.ccount[gi];
    h = fnv(h, cc);
    if (S.SC) {
      const uint32_t kept = cc < S.SC ? cc : S.SC;
      for (uint32_t i = cc - kept; i != cc; ++i) h = fnv(h, S.stream[(size_t)gi * S.SC + i % S.SC]);
    }
    if (S.TC) {                                     // F3 trace rings, retained part
      const uint32_t cnt = S.tcount[gi], kept = cnt < S.TC ? cnt : S.TC;
      h = fnv(h, cnt);
      for (uint32_t i = cnt - kept; i != cnt; ++i) {
        const uint32_t* r = S.tr + ((size_t)gi * S.TC + i % S.TC) * 32;
        for (int j = 0; j < 32; ++j) h = fnv(h, r[j]);
      }
    }
    if (S.TE) {
      const uint32_t cnt = S.tecount[gi], kept = cnt < S.TE ? cnt : S.TE;
      h = fnv(h, cnt);
      for (uint32_t i = cnt - kept; i != cnt; ++i) {
        const uint2 e = S.tent[(size_t)gi * S.TE + i % S.TE];
        h = fnv(h, e.x);
        h = fnv(h, e.y);
      }
    }
    const uint32_t qh[2] = {qm & 15, (qm >> 9) & 15}, qc[2] = {(qm >> 4) & 31, (qm >> 13) & 31};
    for (int which = 0; which < 2; ++which) {
      h = fnv(h, qc[which]);
      const uint32_t* qb = qslots(S, gi, which);
      for (uint32_t i = 0; i < qc[which]; ++i) {
        const uint32_t* m = qb + ((qh[which] + i) % S.Q) * qstride(S, which);
        for (int j = 0; j < 8; ++j) h = fnv(h, m[j]);
      }
    }
    const uint2* ar = arena_of(S, gi);
    const uint32_t base = hw[hf_abase(N) * N], len = hw[HF_LEN * N];
    for (uint32_t i = 0; i < len; ++i) {
      const uint2 e = ar[(base + i) % S.A];
      h = fnv(h, e.x);
      h = fnv(h, e.y);
    }
  }
  for (int i = 0; i < 5; ++i) h = fnv(h, hot_cl(S, c)[i]);
  out[ci] = h;
}

// The tick kernel's own start/stop timestamps go into ev0/ev1 (null: none) through its dispatch
// packet (hipExtLaunchKernelGGL: no marker packets between launches, each of which cost ~5.7 us of
// idle GPU); the host times one launch per sync that way (raftsim.hip, launch_events).
hipError_t launch_steady(const DevSim& S, uint32_t t0, uint32_t nt, hipStream_t st,
                         hipEvent_t ev0, hipEvent_t ev1);

hipError_t launch_storm(const DevSim& S, uint32_t t0, uint32_t nt, hipStream_t st, hipEvent_t ev0,
                        hipEvent_t ev1);

// The general STORM body over the clusters S.perm lists (S.nslots of them: the storm kernel's
// leftovers): one wave slot per listed cluster at most, waves past the list exit at once.
template <int N, bool SPEC>
hipError_t launch_storm_body_ns(const DevSim& S, uint32_t t0, uint32_t nt, hipStream_t st,
                                hipEvent_t ev0, hipEvent_t ev1) {
  constexpr int CPW = 64 / N;
  hipExtLaunchKernelGGL((tick_kernel<N, false, SPEC, false, true>), dim3((S.C + CPW - 1) / CPW),
                        dim3(64), block_lds_bytes<N, SPEC, true>(), st, ev0, ev1, 0, S, t0, nt);
  return hipGetLastError();
}
hipError_t launch_storm_body(const DevSim& S, uint32_t t0, uint32_t nt, hipStream_t st,
                             hipEvent_t ev0, hipEvent_t ev1) {
  const bool spec = S.variant & RAFT_VARIANT_SPEC;
  switch (S.N) {
#define RS_SB(NN)                                                                            \
  case NN:                                                                                   \
    return spec ? launch_storm_body_ns<NN, true>(S, t0, nt, st, ev0, ev1)                    \
                : launch_storm_body_ns<NN, false>(S, t0, nt, st, ev0, ev1);
    RS_SB(2) RS_SB(3) RS_SB(4) RS_SB(5) RS_SB(6) RS_SB(7) RS_SB(8) RS_SB(9)
#undef RS_SB
    default: return hipErrorInvalidValue;
  }
}

template <int N, bool SPEC>
hipError_t launch_tick_ns(const DevSim& S, uint32_t t0, uint32_t nt, hipStream_t st, hipEvent_t ev0,
                    hipEvent_t ev1, bool steady, bool storm) {
  constexpr int CPW = 64 / N;
  constexpr size_t lds = block_lds_bytes<N, SPEC>();
  const uint32_t waves = S.perm ? sched_slots_bound(S.C, N) / CPW : (S.C + CPW - 1) / CPW;
  if constexpr (N <= 5 && !SPEC) {
    // the steady kernel, whose workgroups run the clusters they bail through tick_wave
    if (steady) return launch_steady(S, t0, nt, st, ev0, ev1);
  }
  if (storm && !S.TC && !S.lite && S.storm_list)
    return launch_storm(S, t0, nt, st, ev0, ev1);
  if (storm && !S.TC && !S.lite)
    hipExtLaunchKernelGGL((tick_kernel<N, false, SPEC, false, true>), dim3(waves), dim3(64),
                          block_lds_bytes<N, SPEC, true>(), st, ev0, ev1, 0, S, t0, nt);
  else if (S.TC)
    hipExtLaunchKernelGGL((tick_kernel<N, true, SPEC, false>), dim3(waves), dim3(64), lds, st, ev0,
                          ev1, 0, S, t0, nt);
  else if (!SPEC && S.lite)
    hipExtLaunchKernelGGL((tick_kernel<N, false, false, true>), dim3(waves), dim3(64), lds, st, ev0,
                          ev1, 0, S, t0, nt);
  else
    hipExtLaunchKernelGGL((tick_kernel<N, false, SPEC, false>), dim3(waves), dim3(64), lds, st,
                          ev0, ev1, 0, S, t0, nt);
  return hipGetLastError();
}

template <int N>
hipError_t launch_tick_n(const DevSim& S, uint32_t t0, uint32_t nt, hipStream_t st,
                         hipEvent_t ev0, hipEvent_t ev1, bool steady, bool storm) {
  if (S.variant & RAFT_VARIANT_SPEC)
    return launch_tick_ns<N, true>(S, t0, nt, st, ev0, ev1, false, storm);
  return launch_tick_ns<N, false>(S, t0, nt, st, ev0, ev1, steady, storm);
}

// steady: a LITE launch at N <= 5 without TRACE runs the steady kernel; storm: a launch before any
// timer can fire in a handle fresh from init-node runs the STORM body (tick_wave.hpp). The caller
// decides; results are the same either way.
hipError_t launch_tick(const DevSim& S, uint32_t t0, uint32_t nt, hipStream_t st, hipEvent_t ev0,
                       hipEvent_t ev1, bool steady, bool storm) {
  switch (S.N) {
    case 2: return launch_tick_n<2>(S, t0, nt, st, ev0, ev1, steady, storm);
    case 3: return launch_tick_n<3>(S, t0, nt, st, ev0, ev1, steady, storm);
    case 4: return launch_tick_n<4>(S, t0, nt, st, ev0, ev1, steady, storm);
    case 5: return launch_tick_n<5>(S, t0, nt, st, ev0, ev1, steady, storm);
    case 6: return launch_tick_n<6>(S, t0, nt, st, ev0, ev1, false, storm);
    case 7: return launch_tick_n<7>(S, t0, nt, st, ev0, ev1, false, storm);
    case 8: return launch_tick_n<8>(S, t0, nt, st, ev0, ev1, false, storm);
    case 9: return launch_tick_n<9>(S, t0, nt, st, ev0, ev1, false, storm);
    default: return hipErrorInvalidValue;
  }
}

template <int N, bool TRACE, bool SPEC, bool LITE = false, bool STORM = false>
hipError_t configure_one() {
  return hipFuncSetAttribute(reinterpret_cast<const void*>(tick_kernel<N, TRACE, SPEC, LITE, STORM>),
                             hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)block_lds_bytes<N, SPEC, STORM>());
}

template <int N>
hipError_t configure_n() {
  hipError_t e = hipSuccess;
  if ((e = configure_one<N, false, false>()) || (e = configure_one<N, true, false>()) ||
      (e = configure_one<N, false, true>()) || (e = configure_one<N, true, true>()) ||
      (e = configure_one<N, false, false, true>()) ||
      (e = configure_one<N, false, false, false, true>()) ||
      (e = configure_one<N, false, true, false, true>()))
    return e;
  return hipSuccess;
}

hipError_t configure_steady();

hipError_t configure_kernels() {
  hipError_t e = hipSuccess;
  if ((e = configure_n<2>()) || (e = configure_n<3>()) || (e = configure_n<4>()) ||
      (e = configure_n<5>()) || (e = configure_n<6>()) || (e = configure_n<7>()) ||
      (e = configure_n<8>()) || (e = configure_n<9>()) || (e = configure_steady()))
    return e;
  return hipSuccess;
}


hipError_t launch_init(const DevSim& S, hipStream_t st) {
  hipLaunchKernelGGL(init_kernel, dim3((S.NN + 255) / 256), dim3(256), 0, st, S);
  return hipGetLastError();
}

hipError_t launch_digest(const DevSim& S, uint32_t c0, uint32_t nc, unsigned long long* out,
                         hipStream_t st) {
  hipLaunchKernelGGL(digest_kernel, dim3((nc + 127) / 128), dim3(128), 0, st, S, c0, nc, out);
  return hipGetLastError();
}

}  // namespace rs

// raftsim.hip — C ABI of libraftsim.so (include/raftsim.h) over the gfx950 tick kernel.
#include <errno.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "device.hpp"

namespace rs {
hipError_t launch_tick(const DevSim& S, uint32_t t0, uint32_t nt, hipStream_t st, hipEvent_t ev0,
                       hipEvent_t ev1, bool steady, bool storm);
hipError_t launch_sched_key(const DevSim& S, uint32_t t0, hipStream_t st);
hipError_t launch_sched_perm(const DevSim& S, uint32_t* zero, uint32_t* perm, uint32_t* nslots,
                             hipStream_t st);
hipError_t launch_init(const DevSim& S, hipStream_t st);
hipError_t launch_digest(const DevSim& S, uint32_t c0, uint32_t nc, unsigned long long* out,
                         hipStream_t st);
hipError_t configure_kernels();
}  // namespace rs

using rs::DevSim;

static thread_local char g_err[512];

static int fail(int code, const char* fmt, const char* detail = "") {
  snprintf(g_err, sizeof g_err, fmt, detail);
  return code;
}

#define HIP_OK(expr)                                                               \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) return fail(-EIO, "HIP error: %s (" #expr ")",           \
                                      hipGetErrorString(e_));                      \
  } while (0)


struct Shard {
  raft_sim_config_t cfg;
  uint32_t N, Q, L, A, C, NN, tpl;
  uint64_t tick;        // the shard's next tick
  uint64_t ticks_run;   // ticks simulated by this handle (node_ticks counts these)
  hipStream_t stream;
  hipEvent_t ev_start, ev_stop;
  // Start/stop events in a launch's dispatch packet time the kernel alone, but measured 8.2 against
  // 2.5 us per back-to-back launch of an empty kernel on MI355X (scripts/launch_probe.hip): a
  // steady-path launch (~0.025 ms at C2) carries them only when it is the first after a sync
  // (the kernel time reported is that launch's); general-kernel launches (milliseconds, and their
  // cost changes over a run as logs grow and nodes halt) are all timed. RAFTSIM_LAUNCH_EVENTS=1
  // times every launch (diagnostic).
  bool launch_events;
  std::vector<uint8_t> ktimed;   // per launch since the last sync: carries an event pair
  std::vector<hipEvent_t> kev;   // per tick-kernel launch of a step: start, stop
  DevSim d;
  std::vector<void*> allocs;
  double last_ms, last_step_ms;
  uint32_t last_timed;           // launches of the last sync window that carried an event pair
  bool pending;                  // launches enqueued since the last sync
  uint32_t pending_launches;
  uint32_t last_launches;
  unsigned long long* client_pw;
  // RAFT_SCHED_ALIGNED: the spare histogram (the schedule kernel zeroes it while reading d.shist;
  // the two swap every rebuild) and the wave-slot -> cluster map of the next launch. keys_written:
  // the last tick launch wrote every cluster's key and the matching histogram into d.skey /
  // d.shist; otherwise a rebuild zeroes d.shist and computes both from the state (sched_key).
  // Stale keys (after host writes or set_tick) change the packing (speed), never the results; a
  // histogram always counts each cluster once, so a packing always places each cluster once.
  uint32_t *soff, *sperm, *snslots;   // + the slot count of the packing
  bool keys_written;
  uint64_t resort_ctr = 0;             // tick launches since create
  uint32_t resort_every;               // rebuild period (fixed at create)
  // steady kernel (steady_kernel.hip): LITE launches at N <= 5 without TRACE; the two bail
  // counters alternate between steady launches (each reports and zeroes the other)
  bool steady_ok;
  bool last_steady;                    // the last tick launch took the steady path
  uint32_t* nbail2;
  uint32_t steady_parity;
  // Path choice per launch (speed only: both paths give the same state). RAFTSIM_STEADY=auto
  // (default): the steady kernel unless the last catch-up launch the host has seen (bail_host,
  // written by the GPU; a few launches stale at most) took more than 1/16 of the clusters, then
  // the general kernel for the next STEADY_COOLDOWN launches. The first launch of a handle is
  // steady too: the steady kernel runs init-node's election in closed form (steady_kernel.hip).
  // "always" / "never" force a path.
  int steady_mode;                     // 0 auto, 1 always, 2 never
  uint32_t* bail_host;                 // host-mapped word (hipHostMalloc)
  uint32_t steady_cooldown;
  // Ticks before this one are storm ticks (tick_wave.hpp, STORM): the handle is fresh from
  // init-node with client traffic, so no timer fires before el_base and the only events are
  // client-sets at followers. Any host write of state or of the clock ends it (0).
  uint32_t storm_until;
  bool storm_ran = false;              // a storm-kernel launch has run (raftsim_diag_storm_bails)
};
constexpr uint32_t STEADY_COOLDOWN = 2;
// The wave packing is rebuilt every RESORT_EVERY-th tick launch and reused in between: with
// key-pure waves a steady-state cluster keeps its wave mates' phase, so a packing stays good for
// more than one 10k-tick launch, and skipping the schedule kernel (C2: 14.6 us) every other
// launch measured C2 step wall 0.127 -> 0.119 ms with the tick kernel unchanged (every 4th: no
// further gain). Results never depend on the packing.
constexpr uint32_t RESORT_EVERY = 2;
// LITE handles: a steady-state packing is a rotation of itself one launch later (every cluster's
// next event moves by the same launch length), so it is rebuilt every 8th launch
constexpr uint32_t RESORT_EVERY_LITE = 8;

// Exported functions take their C linkage from the declarations in include/raftsim.h.

const char* raft_sim_last_error(void) { return g_err; }
int raft_sim_abi_version(void) { return RAFT_SIM_ABI_VERSION; }

void raft_sim_default_config(raft_sim_config_t* c) {
  memset(c, 0, sizeof *c);
  c->n_clusters = 1; c->nodes = 5; c->log_cap = 64; c->inbox_cap = 16; c->seed = 42;
  c->hb = 3000; c->el_base = 5000; c->el_span = 5000; c->dmin = 1; c->dmax = 1;
  c->part_epoch = 1000; c->n_devices = 1;
}

static int validate_cfg(const raft_sim_config_t* c) {
  if (c->nodes < 2 || c->nodes > RAFT_MAX_NODES) return fail(-EINVAL, "nodes must be 2..9");
  if (c->n_clusters == 0) return fail(-EINVAL, "n_clusters must be > 0");
  if ((uint64_t)c->n_clusters * c->nodes > 0x7FFFFFFFull) return fail(-EINVAL, "too many nodes");
  if (c->inbox_cap < 1 || c->inbox_cap > RAFT_MAX_INBOX) return fail(-EINVAL, "inbox_cap 1..16");
  if (c->log_cap < 1 || c->log_cap > 65535) return fail(-EINVAL, "log_cap 1..65535");
  uint64_t A = c->arena_cap ? c->arena_cap : 4ull * c->log_cap;
  if (A < 2ull * c->log_cap || A > (1u << 24))
    return fail(-EINVAL, "arena_cap must be >= 2*log_cap");
  if (c->hb < 1 || c->el_base < 1) return fail(-EINVAL, "hb and el_base must be >= 1");
  if (c->dmin < 1 || c->dmax < c->dmin || c->dmax > 255)
    return fail(-EINVAL, "1 <= dmin <= dmax <= 255");
  if (c->part_epoch < 1) return fail(-EINVAL, "part_epoch must be >= 1");
  if (c->drop_ppm > 1000000 || c->dup_ppm > 1000000 || c->part_ppm > 1000000 ||
      c->client_ppm > 1000000)
    return fail(-EINVAL, "ppm values must be <= 1e6");
  if (c->variant_flags & ~3u) return fail(-EINVAL, "variant_flags: only bits 0-1 are defined");
  if (c->schedule > RAFT_SCHED_FIXED) return fail(-EINVAL, "schedule: 0 (aligned) or 1 (fixed)");
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

// Zero every copy of the counter block, with "no violation" (UINT64_MAX) in the first-violation
// slots (rs::CTR_COPIES copies of rs::CTR_STRIDE words, reduced by sh_read_counters).
static hipError_t init_counters(Shard* s) {
  std::vector<unsigned long long> c((size_t)rs::CTR_COPIES * rs::CTR_STRIDE, 0ull);
  for (int k = 0; k < rs::CTR_COPIES; ++k) c[(size_t)k * rs::CTR_STRIDE + RAFT_CTR_COUNT] = ~0ull;
  return hipMemcpy(s->d.ctr, c.data(), c.size() * 8, hipMemcpyHostToDevice);   // blocking: c dies
}

template <typename T>
static int dalloc(Shard* s, T** p, size_t count) {
  void* v = nullptr;
  hipError_t e = hipMalloc(&v, std::max<size_t>(count, 1) * sizeof(T));
  if (e != hipSuccess) return fail(-ENOMEM, "hipMalloc failed: %s", hipGetErrorString(e));
  s->allocs.push_back(v);
  *p = static_cast<T*>(v);
  return 0;
}

static void sh_destroy(Shard* s) {
  if (!s) return;
  (void)hipSetDevice(s->cfg.device);
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  for (void* p : s->allocs) (void)hipFree(p);
  if (s->bail_host) (void)hipHostFree(s->bail_host);
  if (s->ev_start) (void)hipEventDestroy(s->ev_start);
  if (s->ev_stop) (void)hipEventDestroy(s->ev_stop);
  for (hipEvent_t e : s->kev) (void)hipEventDestroy(e);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  delete s;
}

// One shard: cfg holds its own cluster count, global offset and device (validated by the caller).
static int sh_create(const raft_sim_config_t* cfg, Shard** out) {
  int rc = 0;
  HIP_OK(hipSetDevice(cfg->device));
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, cfg->device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(-EIO, "device is %s; libraftsim.so is built for gfx950", prop.gcnArchName);
  HIP_OK(rs::configure_kernels());

  Shard* s = new Shard();
  s->cfg = *cfg;
  s->N = cfg->nodes; s->Q = cfg->inbox_cap; s->L = cfg->log_cap; s->C = cfg->n_clusters;
  s->A = cfg->arena_cap ? cfg->arena_cap : 4 * cfg->log_cap;
  s->NN = s->C * s->N;
  s->tpl = cfg->ticks_per_launch ? std::min<uint32_t>(cfg->ticks_per_launch, 65536u) : 10000u;
  DevSim& d = s->d;
  d.C = s->C; d.N = s->N; d.Q = s->Q; d.L = s->L; d.A = s->A; d.NN = s->NN;
  d.goff = cfg->cluster_offset;
  d.key0 = (uint32_t)cfg->seed; d.key1 = (uint32_t)(cfg->seed >> 32);
  d.hb = cfg->hb; d.el_base = cfg->el_base; d.el_span = cfg->el_span;
  d.drop_ppm = cfg->drop_ppm; d.dup_ppm = cfg->dup_ppm; d.dmin = cfg->dmin; d.dmax = cfg->dmax;
  d.part_ppm = cfg->part_ppm; d.part_epoch = cfg->part_epoch; d.client_ppm = cfg->client_ppm;
  d.variant = cfg->variant_flags;
  d.client_period = cfg->client_period; d.client_burst = cfg->client_burst;
  d.client_redirects = cfg->client_redirects;
  d.div_period = rs::make_div(cfg->client_period ? cfg->client_period : 1);
  d.div_burst = rs::make_div(cfg->client_burst ? cfg->client_burst : 1);
  d.div_epoch = rs::make_div(cfg->part_epoch);
  d.SC = cfg->commit_stream_cap;
  d.TC = cfg->trace_cap;
  d.TE = cfg->trace_entry_cap;
  uint64_t pw[32];
  rs::client_powers(cfg->client_ppm, pw);
  d.client_pw = nullptr;
  d.lite = cfg->client_ppm == 0 && cfg->drop_ppm == 0 && cfg->dup_ppm == 0 && cfg->part_ppm == 0 &&
           cfg->dmin == cfg->dmax;
  d.client_top = -1;
  for (int i = 0; i < 32; ++i)
    if (pw[i]) d.client_top = i;
  if (pw[0] >> 32) d.client_top = 32;   // client_ppm == 0: every power is 2^32 (rs::client_gap)
  const size_t NN = s->NN;
  d.HB = rs::hot_block_words(s->N);
  if ((rc = dalloc(s, &d.hot, (size_t)s->C * d.HB)) ||
      (rc = dalloc(s, &d.qbuf, NN * 2 * s->Q * 8)) ||
      (rc = dalloc(s, &d.arena, (NN * (size_t)s->A + rs::ARENA_PAD_SLOTS) * 2)) ||
      (rc = dalloc(s, &d.ctr, (size_t)rs::CTR_COPIES * rs::CTR_STRIDE)) || (rc = dalloc(s, &s->client_pw, 32)) ||
      (rc = dalloc(s, &d.ccount, NN)) ||
      (rc = dalloc(s, &d.stream, NN * std::max<uint32_t>(cfg->commit_stream_cap, 1))) ||
      (rc = dalloc(s, &d.tr, NN * std::max<uint32_t>(d.TC, 1) * 32)) ||
      (rc = dalloc(s, &d.tcount, NN)) ||
      (rc = dalloc(s, &d.tent, NN * std::max<uint32_t>(d.TE, 1))) ||
      (rc = dalloc(s, &d.tecount, NN))) {
    sh_destroy(s);
    return rc;
  }
  d.client_pw = s->client_pw;
  d.wavelog = nullptr;
#ifdef RS_WAVELOG
  if ((rc = dalloc(s, &d.wavelog, (size_t)rs::sched_slots_bound(s->C, s->N) * 12))) {
    sh_destroy(s);
    return rc;
  }
#endif
  s->steady_ok = d.lite && s->N <= 5 && !d.TC && !(cfg->variant_flags & RAFT_VARIANT_SPEC);
  // init-node's deadlines are el_base or more ahead and every re-arm is too (SIM_SPEC D4; the
  // Spec-Raft control re-arms on fewer events): until el_base, client-sets are the only events
  s->storm_until = cfg->client_ppm && !d.TC ? cfg->el_base : 0u;
  s->resort_every = d.lite ? RESORT_EVERY_LITE : RESORT_EVERY;
  {
    const char* le = getenv("RAFTSIM_LAUNCH_EVENTS");
    s->launch_events = le && !strcmp(le, "1");
  }
  if (s->steady_ok && (rc = dalloc(s, &s->nbail2, 2))) {
    sh_destroy(s);
    return rc;
  }
  // the storm kernel's leftover list (storm_kernel.hip), while storm ticks lie ahead. One lane per
  // cluster needs clusters enough to fill the chip (two 64-cluster waves per SIMD at least: at
  // C4's 16,384 clusters its 256 waves ran 36 ms against the lane-per-node body's 14): below that
  // the storm ticks run the general STORM body.
  // (Its registers hold arrivals below 2^28 and hop counts below 16.)
  uint32_t storm_min = 131072;
  if (const char* sm = getenv("RAFTSIM_STORM_MIN_CLUSTERS")) storm_min = (uint32_t)strtoul(sm, nullptr, 10);
  if (s->storm_until && s->C >= storm_min && cfg->el_base < (1u << 28) && cfg->client_redirects < 16 &&
      ((rc = dalloc(s, &s->d.storm_list, s->C)) ||
                         (rc = dalloc(s, &s->d.storm_count, 1)))) {
    sh_destroy(s);
    return rc;
  }
  if (s->steady_ok) {
    const char* m = getenv("RAFTSIM_STEADY");
    s->steady_mode = m && !strcmp(m, "always") ? 1 : m && !strcmp(m, "never") ? 2 : 0;

    s->steady_cooldown = 0;
    void* hp = nullptr;
    if (hipHostMalloc(&hp, sizeof(uint32_t), hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void**>(&d.bail_report), hp, 0) != hipSuccess) {
      if (hp) (void)hipHostFree(hp);
      sh_destroy(s);
      return fail(-ENOMEM, "hipHostMalloc (bail report) failed");
    }
    s->bail_host = static_cast<uint32_t*>(hp);
    *s->bail_host = 0;
  }
  if (cfg->schedule == RAFT_SCHED_ALIGNED) {
    if ((rc = dalloc(s, &d.skey, s->C)) || (rc = dalloc(s, &d.shist, rs::SCHED_BUCKETS)) ||
        (rc = dalloc(s, &s->soff, rs::SCHED_BUCKETS)) ||
        (rc = dalloc(s, &s->sperm, rs::sched_slots_bound(s->C, s->N))) ||
        (rc = dalloc(s, &s->snslots, 1))) {
      sh_destroy(s);
      return rc;
    }
  }
  hipError_t e;
  if ((e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking)) != hipSuccess ||
      (e = hipEventCreate(&s->ev_start)) != hipSuccess ||
      (e = hipEventCreate(&s->ev_stop)) != hipSuccess ||
      (e = hipMemsetAsync(d.hot, 0, (size_t)s->C * d.HB * 4, s->stream)) != hipSuccess ||
      (e = hipMemsetAsync(d.qbuf, 0, NN * 2 * s->Q * 32, s->stream)) != hipSuccess ||
      (e = hipMemsetAsync(d.arena, 0, (NN * (size_t)s->A + rs::ARENA_PAD_SLOTS) * 8, s->stream)) != hipSuccess ||
      (e = hipMemsetAsync(d.stream, 0, NN * std::max<uint32_t>(cfg->commit_stream_cap, 1) * 4,
                          s->stream)) != hipSuccess ||
      (e = hipMemsetAsync(d.tr, 0, NN * std::max<uint32_t>(d.TC, 1) * 128, s->stream)) != hipSuccess ||
      (e = hipMemsetAsync(d.tcount, 0, NN * 4, s->stream)) != hipSuccess ||
      (e = hipMemsetAsync(d.tent, 0, NN * std::max<uint32_t>(d.TE, 1) * 8, s->stream)) != hipSuccess ||
      (e = hipMemsetAsync(d.tecount, 0, NN * 4, s->stream)) != hipSuccess ||
      (d.shist && (e = hipMemsetAsync(d.shist, 0, rs::SCHED_BUCKETS * 4, s->stream)) != hipSuccess) ||
      (s->nbail2 && (e = hipMemsetAsync(s->nbail2, 0, 8, s->stream)) != hipSuccess) ||
      (e = init_counters(s)) != hipSuccess ||
      (e = hipMemcpyAsync(s->client_pw, pw, sizeof pw, hipMemcpyHostToDevice, s->stream)) !=
          hipSuccess ||
      (e = rs::launch_init(d, s->stream)) != hipSuccess ||
      (e = hipStreamSynchronize(s->stream)) != hipSuccess) {
    sh_destroy(s);
    return fail(-EIO, "HIP error during create: %s", hipGetErrorString(e));
  }
  *out = s;
  return 0;
}

// Enqueue n_ticks on the shard's stream. s->tick advances launch by launch, so after a failure it
// still names the tick the state has reached (the handle is then poisoned anyway).
static int sh_step_async(Shard* s, uint32_t n_ticks) {
  HIP_OK(hipSetDevice(s->cfg.device));
  uint32_t launches = s->pending_launches;
  if (!s->pending) {
    HIP_OK(hipEventRecord(s->ev_start, s->stream));
    launches = 0;
    s->pending = true;
  }
  for (uint32_t done = 0; done < n_ticks;) {
    uint32_t nt = std::min(s->tpl, n_ticks - done);
    const uint32_t t0 = (uint32_t)s->tick;
    // storm ticks run alone in a launch of their own (the STORM body)
    const bool storm = t0 < s->storm_until;
    if (storm) nt = std::min(nt, s->storm_until - t0);
    // Path (speed only: both paths give the same state). Host writes may have cleared lite.
    bool steady = s->steady_ok && s->d.lite;
    if (steady && s->steady_mode == 2) steady = false;
    if (steady && s->steady_mode == 0) {
      if (s->steady_cooldown) {
        --s->steady_cooldown;
        steady = false;
      } else if (__atomic_load_n(s->bail_host, __ATOMIC_RELAXED) > s->C / 16) {
        __atomic_store_n(s->bail_host, 0u, __ATOMIC_RELAXED);
        s->steady_cooldown = STEADY_COOLDOWN - 1;
        steady = false;
      }
    }
    bool no_keys = false;                // this launch writes no packing keys
    bool no_perm = false;
    if (steady) {
      // the steady kernel runs the clusters in id order: no packing, no keys. (Packed by next
      // event, 64 to a wave, the same launch took 0.0329 against 0.0318 ms: a lane runs its own
      // cluster's clock, and the packing's perm load sat in front of every state load.)
      no_perm = no_keys = true;
      s->keys_written = false;
    } else if (s->cfg.schedule == RAFT_SCHED_ALIGNED && s->resort_ctr == 0 && !s->d.client_ppm) {
      // The handle's first launch without client traffic (every cluster from init-node or as the
      // host wrote it): clusters in id order. Per-cluster clocks make a wave's trips its busiest
      // cluster's event ticks whatever its mates are, and the packing's key and sort kernels
      // measured +35-40 us on the 100-us first launch of 65,536 clusters (scripts/init_probe.py).
      // Keys are not written: the next launch's rebuild computes them from the state.
      no_perm = no_keys = true;
      s->keys_written = false;
      ++s->resort_ctr;
    } else if (s->cfg.schedule == RAFT_SCHED_ALIGNED) {
      // pack clusters with the same next event onto the same waves for this launch: keys and
      // histogram come from the previous tick launch, or are computed from the state. The
      // packing is rebuilt every resort_every-th launch and reused in between (any packing gives
      // the same results); only the launch before a rebuild writes keys.
      if (s->resort_ctr % s->resort_every == 0) {
        if (!s->keys_written) {
          HIP_OK(hipMemsetAsync(s->d.shist, 0, rs::SCHED_BUCKETS * 4, s->stream));
          HIP_OK(rs::launch_sched_key(s->d, t0, s->stream));
        }
        HIP_OK(rs::launch_sched_perm(s->d, s->soff, s->sperm, s->snslots, s->stream));
        // the schedule kernel read d.shist and zeroed soff: the next key-writing launch fills it
        std::swap(s->d.shist, s->soff);
        s->d.perm = s->sperm;
        s->d.nslots = s->snslots;
      }
      ++s->resort_ctr;
      s->keys_written = s->resort_ctr % s->resort_every == 0;   // the next launch rebuilds
      no_keys = !s->keys_written;
    }
    const bool timed = s->launch_events || launches == 0 || !steady;
    if (s->ktimed.size() < launches + 1) s->ktimed.resize(launches + 1);
    s->ktimed[launches] = timed;
    while (timed && s->kev.size() < 2 * (size_t)(launches + 1)) {
      hipEvent_t e;   // timing only: no system-scope fence (cache writeback) per launch
      HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
      s->kev.push_back(e);
    }
#ifdef RS_WAVELOG
    HIP_OK(hipMemsetAsync(s->d.wavelog, 0,
                          (size_t)rs::sched_slots_bound(s->C, s->N) * 192 / (64 / s->N), s->stream));
#endif
    s->last_steady = steady;
    if (storm && !steady && s->d.storm_list && !s->d.TC && !s->d.lite) s->storm_ran = true;
    if (steady) {
      s->d.nbail = s->nbail2 + s->steady_parity;
      s->d.nbail_zero = s->nbail2 + (s->steady_parity ^ 1);
      s->steady_parity ^= 1;
    }
    DevSim D = s->d;
    if (no_perm) D.perm = nullptr;
    if (no_keys) D.shist = nullptr;
    HIP_OK(rs::launch_tick(D, t0, nt, s->stream,
                           timed ? s->kev[2 * launches] : nullptr,
                           timed ? s->kev[2 * launches + 1] : nullptr, steady, storm && !steady));
    done += nt;
    s->tick += nt;
    s->ticks_run += nt;
    ++launches;
    s->pending_launches = launches;
  }
  return 0;
}

static int sh_sync(Shard* s) {
  if (!s) return fail(-EINVAL, "null sim");
  HIP_OK(hipSetDevice(s->cfg.device));
  if (!s->pending) {
    HIP_OK(hipStreamSynchronize(s->stream));
    return 0;
  }
  const uint32_t launches = s->pending_launches;
  s->pending = false;
  s->pending_launches = 0;
  HIP_OK(hipEventRecord(s->ev_stop, s->stream));
  HIP_OK(hipEventSynchronize(s->ev_stop));
  float ms = 0, kms = 0;
  HIP_OK(hipEventElapsedTime(&ms, s->ev_start, s->ev_stop));
  uint32_t timed = 0;
  for (uint32_t i = 0; i < launches; ++i) {
    if (!s->ktimed[i]) continue;
    float one = 0;
    HIP_OK(hipEventElapsedTime(&one, s->kev[2 * i], s->kev[2 * i + 1]));
    kms += one;
    ++timed;
  }
  s->last_ms = timed ? kms / timed : 0.0;         // per timed tick-kernel launch
  s->last_timed = timed;
  s->last_step_ms = ms;                           // + the schedule's key and sort kernels
  s->last_launches = launches;
  return 0;
}


static int check_range(Shard* s, uint32_t c0, uint32_t nc) {
  if (!s) return fail(-EINVAL, "null sim");
  if ((uint64_t)c0 + nc > s->C) return fail(-EINVAL, "cluster range out of bounds");
  return 0;
}

// Slot 0 of node gi's queue `which` and the ring's slot pitch in bytes (rs::qslots: REQ rings
// slot-major, RES rings node-major).
static uint32_t* qring(Shard* s, uint32_t gi, uint32_t which) {
  return s->d.qbuf + (which ? (size_t)s->Q * s->NN + (size_t)gi * s->Q : (size_t)gi) * 8;
}
static size_t qpitch(Shard* s, uint32_t which) {
  return (which ? 1 : (size_t)s->NN) * sizeof(raft_msg_t);
}

// Field `f` of node `id` in cluster `cluster`'s hot block (rs::HotField).
static uint32_t* hot_word(Shard* s, uint32_t cluster, uint32_t id, uint32_t f) {
  return s->d.hot + (size_t)cluster * s->d.HB + rs::HOT_CW + (size_t)f * s->N + (id - 1);
}
static uint32_t* cl_words(Shard* s, uint32_t cluster) {
  return s->d.hot + (size_t)cluster * s->d.HB + rs::hot_cl_off(s->N);
}

static int check_node(Shard* s, uint32_t cluster, uint32_t id) {
  if (!s) return fail(-EINVAL, "null sim");
  if (cluster >= s->C || id < 1 || id > s->N) return fail(-EINVAL, "cluster/node out of bounds");
  return 0;
}

template <typename T>
static hipError_t d2h(Shard* s, T* host, const T* dev, size_t count) {
  return hipMemcpyAsync(host, dev, count * sizeof(T), hipMemcpyDeviceToHost, s->stream);
}
template <typename T>
static hipError_t h2d(Shard* s, T* dev, const T* host, size_t count) {
  return hipMemcpyAsync(dev, host, count * sizeof(T), hipMemcpyHostToDevice, s->stream);
}

static int sh_read_nodes(Shard* s, uint32_t c0, uint32_t nc, raft_node_t* out) {
  int rc = check_range(s, c0, nc);
  if (rc) return rc;
  if (!out) return fail(-EINVAL, "null output");
  HIP_OK(hipSetDevice(s->cfg.device));
  const size_t n0 = (size_t)c0 * s->N, cnt = (size_t)nc * s->N, N = s->N, HB = s->d.HB;
  std::vector<uint32_t> blk(nc * HB), cc(cnt);
  HIP_OK(d2h(s, blk.data(), s->d.hot + (size_t)c0 * HB, nc * HB));
  HIP_OK(d2h(s, cc.data(), s->d.ccount + n0, cnt));
  HIP_OK(hipStreamSynchronize(s->stream));
  for (size_t i = 0; i < cnt; ++i) {
    const uint32_t* h = &blk[(i / N) * HB + rs::HOT_CW + i % N];     // field f at h[f * N]
    auto f = [&](uint32_t fld) { return h[fld * N]; };
    raft_node_t& r = out[i];
    memset(&r, 0, sizeof r);
    const uint32_t fl = f(rs::HF_FLAGS), mk = f(rs::HF_MASKS), qm = f(rs::HF_QMETA);
    r.role = fl & 3; r.voted_for = (fl >> 2) & 15; r.leader_id = (fl >> 6) & 15;
    r.fault = (fl >> 10) & 7; r.entries_is_seq = (fl >> 13) & 1; r.ls_present = (fl >> 14) & 1;
    r.votes = mk & 0xFFFF; r.ls_keys = mk >> 16;
    r.current_term = f(rs::HF_TERM); r.commit_index = f(rs::HF_COMMIT);
    r.log_len = f(rs::HF_LEN); r.deadline = f(rs::HF_DEADLINE);
    if (fl & rs::FL_DRAW)        // a deferred timer draw still owed in the stored state
      r.deadline = rs::exact_deadline((uint32_t)(s->cfg.cluster_offset + c0 + i / N),
                                      (uint32_t)(i % N) + 1, r.deadline, s->cfg.el_base,
                                      s->cfg.el_span, s->d.key0, s->d.key1);
    for (size_t p = 0; p < N; ++p) {
      r.next_index[p] = (int32_t)f(rs::HF_NEXT + p);
      r.match_index[p] = (int32_t)f(rs::HF_NEXT + N + p);
    }
    r.last_led_term = f(rs::hf_led(N));
    r.arena_base = f(rs::hf_abase(N)); r.arena_frontier = f(rs::hf_afront(N));
    r.req_count = (qm >> 4) & 31; r.res_count = (qm >> 13) & 31;
    r.trace_hash = (uint64_t)f(rs::HF_TRACE_HI) << 32 | f(rs::HF_TRACE_LO);
    r.commit_count = cc[i];
  }
  return 0;
}

static int sh_write_nodes(Shard* s, uint32_t c0, uint32_t nc, const raft_node_t* in) {
  int rc = check_range(s, c0, nc);
  if (rc) return rc;
  s->storm_until = 0;
  if (!in) return fail(-EINVAL, "null input");
  HIP_OK(hipSetDevice(s->cfg.device));
  const uint32_t N = s->N, all = ((1u << (N + 1)) - 1) & ~1u;
  const size_t n0 = (size_t)c0 * N, cnt = (size_t)nc * N;
  for (size_t i = 0; i < cnt; ++i) {
    const raft_node_t* n = &in[i];
    uint32_t id = (uint32_t)(i % N) + 1, peers = all & ~(1u << id);
    if (n->role > 3 || n->voted_for > N || n->leader_id > N || n->fault > 4 ||
        (n->votes & ~all) || (n->ls_keys & ~peers) || n->entries_is_seq > 1 ||
        n->ls_present > 1 || n->log_len > s->L ||
        n->arena_frontier - n->arena_base < n->log_len ||
        n->arena_frontier - n->arena_base > s->L ||
        (n->role == RAFT_LEADER && (!n->ls_present || n->ls_keys != peers)) ||
        (!n->ls_present && n->ls_keys))
      return fail(-EINVAL, "invalid node record");
  }
  // the queue words of the blocks (qmeta, head/tail arrivals) and the cluster words are kept
  const size_t HB = s->d.HB;
  std::vector<uint32_t> blk(nc * HB), ccv(cnt);
  HIP_OK(d2h(s, blk.data(), s->d.hot + (size_t)c0 * HB, nc * HB));
  HIP_OK(hipStreamSynchronize(s->stream));
  for (size_t i = 0; i < cnt; ++i) {
    const raft_node_t& r = in[i];
    uint32_t* h = &blk[(i / N) * HB + rs::HOT_CW + i % N];
    auto f = [&](uint32_t fld) -> uint32_t& { return h[fld * N]; };
    f(rs::HF_FLAGS) = rs::pack_flags(r.role, r.voted_for, r.leader_id, r.fault, r.entries_is_seq,
                                     r.ls_present);
    f(rs::HF_MASKS) = r.votes | (uint32_t)r.ls_keys << 16;
    f(rs::HF_TERM) = r.current_term; f(rs::HF_COMMIT) = r.commit_index;
    f(rs::HF_LEN) = r.log_len; f(rs::HF_DEADLINE) = r.deadline;
    f(rs::hf_abase(N)) = r.arena_base; f(rs::hf_afront(N)) = r.arena_frontier;
    f(rs::hf_led(N)) = r.last_led_term;
    f(rs::HF_TRACE_LO) = (uint32_t)r.trace_hash; f(rs::HF_TRACE_HI) = (uint32_t)(r.trace_hash >> 32);
    ccv[i] = r.commit_count;
    for (size_t p = 0; p < N; ++p) {
      f(rs::HF_NEXT + p) = (uint32_t)r.next_index[p];
      f(rs::HF_NEXT + N + p) = (uint32_t)r.match_index[p];
    }
  }
  for (size_t c = 0; c < nc; ++c) blk[c * HB + rs::CL_CERT] = 0;   // the steady certificate
  HIP_OK(h2d(s, s->d.hot + (size_t)c0 * HB, blk.data(), nc * HB));
  HIP_OK(h2d(s, s->d.ccount + n0, ccv.data(), cnt));
  HIP_OK(hipStreamSynchronize(s->stream));
  return 0;
}

static int sh_read_queue(Shard* s, uint32_t cluster, uint32_t id, uint32_t which,
                        raft_msg_t* out, uint32_t cap) {
  int rc = check_node(s, cluster, id);
  if (rc) return rc;
  if (which > 1) return fail(-EINVAL, "which must be 0 (req) or 1 (res)");
  HIP_OK(hipSetDevice(s->cfg.device));
  const uint32_t gi = cluster * s->N + id - 1;
  uint32_t qm = 0;
  std::vector<raft_msg_t> slots(s->Q);
  HIP_OK(d2h(s, &qm, hot_word(s, cluster, id, rs::HF_QMETA), 1));
  HIP_OK(hipMemcpy2DAsync(slots.data(), sizeof(raft_msg_t), qring(s, gi, which),
                          qpitch(s, which), sizeof(raft_msg_t), s->Q,
                          hipMemcpyDeviceToHost, s->stream));
  HIP_OK(hipStreamSynchronize(s->stream));
  const uint32_t head = which ? (qm >> 9) & 15 : qm & 15;
  const uint32_t cnt = which ? (qm >> 13) & 31 : (qm >> 4) & 31;
  for (uint32_t i = 0; i < cnt && i < cap && out; ++i) out[i] = slots[(head + i) % s->Q];
  return (int)cnt;
}

static int sh_write_queue(Shard* s, uint32_t cluster, uint32_t id, uint32_t which,
                         const raft_msg_t* in, uint32_t count) {
  int rc = check_node(s, cluster, id);
  if (!rc) s->storm_until = 0;
  if (rc) return rc;
  if (which > 1 || count > s->Q || (count && !in)) return fail(-EINVAL, "bad queue or count");
  for (uint32_t i = 0; i < count; ++i) {
    uint32_t type = in[i].hdr & 7, src = (in[i].hdr >> 3) & 15;
    int want = type <= RAFT_MSG_CLIENT_SET ? 0 : 1;
    if (type < 1 || type > 5 || want != (int)which || src > s->N || src == id ||
        (type == RAFT_MSG_CLIENT_SET) != (src == 0) ||
        (i > 0 && in[i].arrival < in[i - 1].arrival))
      return fail(-EINVAL, "invalid message or order");
  }
  for (uint32_t i = 0; i < count; ++i)   // a queued client-set needs the general kernel (LITE)
    if ((in[i].hdr & 7) == RAFT_MSG_CLIENT_SET) s->d.lite = 0;
  HIP_OK(hipSetDevice(s->cfg.device));
  const uint32_t gi = cluster * s->N + id - 1;
  std::vector<raft_msg_t> slots(s->Q);
  memset(slots.data(), 0, s->Q * sizeof(raft_msg_t));
  for (uint32_t i = 0; i < count; ++i) slots[i] = in[i];
  uint32_t qm = 0;
  HIP_OK(d2h(s, &qm, hot_word(s, cluster, id, rs::HF_QMETA), 1));
  HIP_OK(hipStreamSynchronize(s->stream));
  if (which) qm = (qm & ~(0xFu << 9 | 0x1Fu << 13)) | count << 13;
  else qm = (qm & ~0x1FFu) | count << 4;
  const uint32_t harr = count ? in[0].arrival : rs::INF, tail = count ? in[count - 1].arrival : 0;
  HIP_OK(hipMemcpy2DAsync(qring(s, gi, which), qpitch(s, which), slots.data(),
                          sizeof(raft_msg_t), sizeof(raft_msg_t), s->Q, hipMemcpyHostToDevice,
                          s->stream));
  HIP_OK(h2d(s, hot_word(s, cluster, id, rs::HF_QMETA), &qm, 1));
  HIP_OK(h2d(s, hot_word(s, cluster, id, which ? rs::HF_RES_ARR : rs::HF_REQ_ARR), &harr, 1));
  HIP_OK(h2d(s, hot_word(s, cluster, id, which ? rs::HF_RES_TAIL : rs::HF_REQ_TAIL), &tail, 1));
  const uint32_t zero = 0;                                        // the steady certificate
  HIP_OK(h2d(s, cl_words(s, cluster) + rs::CL_CERT, &zero, 1));
  HIP_OK(hipStreamSynchronize(s->stream));
  return 0;
}

static int sh_read_arena(Shard* s, uint32_t cluster, uint32_t id, raft_entry_t* out,
                        uint32_t cap) {
  int rc = check_node(s, cluster, id);
  if (rc) return rc;
  if (out && cap) {
    HIP_OK(hipSetDevice(s->cfg.device));
    const size_t gi = (size_t)cluster * s->N + id - 1;
    HIP_OK(hipMemcpyAsync(out, s->d.arena + gi * s->A * 2,
                          std::min(cap, s->A) * sizeof(raft_entry_t), hipMemcpyDeviceToHost,
                          s->stream));
    HIP_OK(hipStreamSynchronize(s->stream));
  }
  return (int)s->A;
}

static int sh_write_arena(Shard* s, uint32_t cluster, uint32_t id, const raft_entry_t* in,
                         uint32_t count) {
  int rc = check_node(s, cluster, id);
  if (!rc) s->storm_until = 0;
  if (rc) return rc;
  if (count > s->A || (count && !in)) return fail(-EINVAL, "count > arena_cap");
  HIP_OK(hipSetDevice(s->cfg.device));
  std::vector<raft_entry_t> buf(s->A);
  memset(buf.data(), 0, s->A * sizeof(raft_entry_t));
  if (count) memcpy(buf.data(), in, count * sizeof(raft_entry_t));
  const size_t gi = (size_t)cluster * s->N + id - 1;
  HIP_OK(hipMemcpyAsync(s->d.arena + gi * s->A * 2, buf.data(), s->A * sizeof(raft_entry_t),
                        hipMemcpyHostToDevice, s->stream));
  HIP_OK(hipStreamSynchronize(s->stream));
  return 0;
}

static int sh_read_commit_stream(Shard* s, uint32_t cluster, uint32_t id, uint32_t* out,
                                uint32_t cap) {
  int rc = check_node(s, cluster, id);
  if (rc) return rc;
  HIP_OK(hipSetDevice(s->cfg.device));
  const uint32_t SC = s->cfg.commit_stream_cap;
  const size_t gi = (size_t)cluster * s->N + id - 1;
  uint32_t cc = 0;
  std::vector<uint32_t> ring(std::max<uint32_t>(SC, 1));
  HIP_OK(d2h(s, &cc, s->d.ccount + gi, 1));
  if (SC) HIP_OK(d2h(s, ring.data(), s->d.stream + gi * SC, SC));
  HIP_OK(hipStreamSynchronize(s->stream));
  uint32_t kept = std::min(std::min(cc, SC), cap);
  for (uint32_t i = 0; i < kept && out; ++i) out[i] = ring[(cc - kept + i) % SC];
  return (int)kept;
}

static int sh_write_commit_stream(Shard* s, uint32_t cluster, uint32_t id, const uint32_t* in,
                                 uint32_t count) {
  int rc = check_node(s, cluster, id);
  if (!rc) s->storm_until = 0;
  if (rc) return rc;
  HIP_OK(hipSetDevice(s->cfg.device));
  const uint32_t SC = s->cfg.commit_stream_cap;
  const size_t gi = (size_t)cluster * s->N + id - 1;
  uint32_t cc = 0;
  HIP_OK(d2h(s, &cc, s->d.ccount + gi, 1));
  HIP_OK(hipStreamSynchronize(s->stream));
  if (count > SC || count > cc || (count && !in))
    return fail(-EINVAL, "count exceeds ring or commit_count");
  if (!count) return 0;
  std::vector<uint32_t> ring(SC);
  HIP_OK(d2h(s, ring.data(), s->d.stream + gi * SC, SC));
  HIP_OK(hipStreamSynchronize(s->stream));
  for (uint32_t i = 0; i < count; ++i) ring[(cc - count + i) % SC] = in[i];
  HIP_OK(h2d(s, s->d.stream + gi * SC, ring.data(), SC));
  HIP_OK(hipStreamSynchronize(s->stream));
  return 0;
}

// F3 rings: copy the retained items with index >= first (oldest first), at most cap of them;
// `strict` rejects a `first` that has been overwritten instead of starting at the oldest kept.
template <typename T>
static int read_ring(Shard* s, const uint32_t* dcount, const T* dring, uint32_t R, uint32_t gi,
                     uint32_t first, T* out, uint32_t cap, bool strict) {
  uint32_t cnt = 0;
  HIP_OK(d2h(s, &cnt, dcount + gi, 1));
  HIP_OK(hipStreamSynchronize(s->stream));
  uint32_t lo = cnt > R ? cnt - R : 0;
  if (strict && first < lo) return fail(-ERANGE, "trace entries overwritten (ring holds the newest)");
  if (first > lo) lo = first;
  const uint32_t n = lo < cnt ? std::min(cnt - lo, cap) : 0;
  if (n && !out) return fail(-EINVAL, "null output");
  // at most two contiguous pieces of the ring
  for (uint32_t done = 0; done < n;) {
    const uint32_t slot = (lo + done) % R, run = std::min(n - done, R - slot);
    HIP_OK(d2h(s, out + done, dring + (size_t)gi * R + slot, run));
    done += run;
  }
  HIP_OK(hipStreamSynchronize(s->stream));
  return (int)n;
}

static int sh_read_trace(Shard* s, uint32_t cluster, uint32_t id, uint32_t first,
                        raft_trace_event_t* out, uint32_t cap) {
  static_assert(sizeof(raft_trace_event_t) == 128, "trace record is 32 words");
  int rc = check_node(s, cluster, id);
  if (rc) return rc;
  HIP_OK(hipSetDevice(s->cfg.device));
  if (!s->d.TC) return 0;
  return read_ring(s, s->d.tcount, reinterpret_cast<const raft_trace_event_t*>(s->d.tr),
                   s->d.TC, cluster * s->N + id - 1, first, out, cap, false);
}

static int sh_read_trace_entries(Shard* s, uint32_t cluster, uint32_t id, uint32_t first,
                                raft_entry_t* out, uint32_t cap) {
  int rc = check_node(s, cluster, id);
  if (rc) return rc;
  HIP_OK(hipSetDevice(s->cfg.device));
  if (!s->d.TE) return fail(-ERANGE, "trace_entry_cap is 0");
  return read_ring(s, s->d.tecount, reinterpret_cast<const raft_entry_t*>(s->d.tent), s->d.TE,
                   cluster * s->N + id - 1, first, out, cap, true);
}

static int sh_read_clusters(Shard* s, uint32_t c0, uint32_t nc, raft_cluster_t* out) {
  int rc = check_range(s, c0, nc);
  if (rc) return rc;
  HIP_OK(hipSetDevice(s->cfg.device));
  static_assert(sizeof(raft_cluster_t) == 32, "cluster record is 8 words");
  if (nc)    // the cluster words sit at a fixed offset of each block
    HIP_OK(hipMemcpy2DAsync(out, sizeof(raft_cluster_t), cl_words(s, c0), (size_t)s->d.HB * 4,
                            sizeof(raft_cluster_t), nc, hipMemcpyDeviceToHost, s->stream));
  HIP_OK(hipStreamSynchronize(s->stream));
  // the reserved words are the kernels' (the steady certificate, rs::CL_CERT): not state
  for (uint32_t i = 0; i < nc; ++i) out[i].reserved[0] = out[i].reserved[1] = out[i].reserved[2] = 0;
  return 0;
}

static int sh_write_clusters(Shard* s, uint32_t c0, uint32_t nc, const raft_cluster_t* in) {
  int rc = check_range(s, c0, nc);
  if (rc) return rc;
  s->storm_until = 0;
  HIP_OK(hipSetDevice(s->cfg.device));
  std::vector<raft_cluster_t> buf(in, in + nc);
  for (auto& h : buf) {
    h.reserved[0] = h.reserved[1] = h.reserved[2] = 0;
    if (h.client_next != 0xFFFFFFFFu) s->d.lite = 0;   // a client-set is due: P0 is needed
  }
  if (nc)
    HIP_OK(hipMemcpy2DAsync(cl_words(s, c0), (size_t)s->d.HB * 4, buf.data(),
                            sizeof(raft_cluster_t), sizeof(raft_cluster_t), nc,
                            hipMemcpyHostToDevice, s->stream));
  HIP_OK(hipStreamSynchronize(s->stream));
  return 0;
}

static int sh_read_counters(Shard* s, raft_counters_t* out) {
  if (!s || !out) return fail(-EINVAL, "null argument");
  HIP_OK(hipSetDevice(s->cfg.device));
  std::vector<unsigned long long> buf((size_t)rs::CTR_COPIES * rs::CTR_STRIDE);
  HIP_OK(hipMemcpyAsync(buf.data(), s->d.ctr, buf.size() * 8, hipMemcpyDeviceToHost, s->stream));
  HIP_OK(hipStreamSynchronize(s->stream));
  memset(out->c, 0, sizeof out->c);
  out->first_violation_tick = ~0ull;
  out->payload_max = 0;
  for (int k = 0; k < rs::CTR_COPIES; ++k) {        // the copies the waves flushed into
    const unsigned long long* b = &buf[(size_t)k * rs::CTR_STRIDE];
    for (int i = 0; i < RAFT_CTR_COUNT; ++i) out->c[i] += b[i];
    out->first_violation_tick = std::min<uint64_t>(out->first_violation_tick, b[RAFT_CTR_COUNT]);
    out->payload_max = std::max<uint64_t>(out->payload_max, b[RAFT_CTR_COUNT + 1]);
  }
  out->node_ticks = (uint64_t)s->NN * s->ticks_run;
  return 0;
}

static int sh_digest(Shard* s, uint32_t c0, uint32_t nc, uint64_t* out) {
  int rc = check_range(s, c0, nc);
  if (rc) return rc;
  if (!out) return fail(-EINVAL, "null output");
  HIP_OK(hipSetDevice(s->cfg.device));
  unsigned long long* dout = nullptr;
  HIP_OK(hipMalloc(reinterpret_cast<void**>(&dout), std::max<size_t>(nc, 1) * 8));
  hipError_t e = rs::launch_digest(s->d, c0, nc, dout, s->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(out, dout, (size_t)nc * 8, hipMemcpyDeviceToHost, s->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
  (void)hipFree(dout);
  if (e != hipSuccess) return fail(-EIO, "HIP error in digest: %s", hipGetErrorString(e));
  return 0;
}


// ---------------------------------------------------------------------------------------------
// The handle: n_devices shards, each a contiguous cluster range [C*d/G, C*(d+1)/G) on device
// (device + d) mod the visible devices, with its own stream. The global cluster id keys Philox
// (SIM_SPEC D13), so every G gives bit-identical clusters; calls addressed to clusters are routed
// to their shard and counters are reduced on the host (SUM; MIN first violation; MAX payload).
// Across processes (torchrun, one rank per GPU) bench.py reduces the same vector over RCCL.
struct raft_sim {
  raft_sim_config_t cfg;
  std::vector<Shard*> sh;
  std::vector<uint32_t> lo;   // shard d owns clusters [lo[d], lo[d+1])
  uint64_t tick;
  bool poisoned;              // a step failed part-way: the state no longer matches `tick`
};

void raft_sim_destroy(raft_sim_t* r) {
  if (!r) return;
  for (Shard* s : r->sh) sh_destroy(s);
  delete r;
}

int raft_sim_create(const raft_sim_config_t* cfg, raft_sim_t** out) {
  if (!cfg || !out) return fail(-EINVAL, "null argument");
  int rc = validate_cfg(cfg);
  if (rc) return rc;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(-EIO, "no HIP device visible: libraftsim.so requires an MI355X (gfx950)");
  if (cfg->device < 0 || cfg->device >= ndev) return fail(-EINVAL, "device ordinal out of range");
  const uint32_t G = std::min<uint32_t>(cfg->n_devices > 1 ? cfg->n_devices : 1, cfg->n_clusters);
  for (uint32_t d = 0; d < G; ++d) {
    const int dev = (cfg->device + (int)d) % ndev;
    hipDeviceProp_t prop;
    HIP_OK(hipGetDeviceProperties(&prop, dev));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
      return fail(-EIO, "device is %s; libraftsim.so is built for gfx950", prop.gcnArchName);
    HIP_OK(hipSetDevice(dev));
    HIP_OK(rs::configure_kernels());
  }
  raft_sim* r = new raft_sim();
  r->cfg = *cfg;
  for (uint32_t d = 0; d <= G; ++d) r->lo.push_back((uint32_t)((uint64_t)cfg->n_clusters * d / G));
  for (uint32_t d = 0; d < G; ++d) {
    raft_sim_config_t c = *cfg;
    c.n_clusters = r->lo[d + 1] - r->lo[d];
    c.cluster_offset = cfg->cluster_offset + r->lo[d];
    c.device = (cfg->device + (int)d) % ndev;
    c.n_devices = 1;
    Shard* s = nullptr;
    if ((rc = sh_create(&c, &s))) {
      raft_sim_destroy(r);
      return rc;
    }
    r->sh.push_back(s);
  }
  *out = r;
  return 0;
}

// SIM_SPEC D1: no deadline or arrival may reach 2^32 - 1, the "never" marker.
static bool horizon_ok(const raft_sim_config_t& c, uint64_t tick, uint32_t n) {
  const uint64_t longest = std::max<uint64_t>({c.hb, (uint64_t)c.el_base + c.el_span, c.dmax});
  return tick + n + longest < 0xFFFFFFFFull;
}

int raft_sim_step_async(raft_sim_t* r, uint32_t n_ticks) {
  if (!r) return fail(-EINVAL, "null sim");
  if (r->poisoned) return fail(-EIO, "a previous step failed part-way; the handle is unusable");
  if (!horizon_ok(r->cfg, r->tick, n_ticks))
    return fail(-ERANGE, "tick + n_ticks + the longest timer would reach 2^32-1");
  for (Shard* s : r->sh) {
    const int rc = sh_step_async(s, n_ticks);
    if (rc) {
      r->poisoned = true;
      return rc;
    }
  }
  r->tick += n_ticks;
  return 0;
}

int raft_sim_sync(raft_sim_t* r) {
  if (!r) return fail(-EINVAL, "null sim");
  for (Shard* s : r->sh) {
    const int rc = sh_sync(s);
    if (rc) {
      r->poisoned = true;
      return rc;
    }
  }
  return 0;
}

int raft_sim_step(raft_sim_t* r, uint32_t n_ticks) {
  const int rc = raft_sim_step_async(r, n_ticks);
  return rc ? rc : raft_sim_sync(r);
}

uint64_t raft_sim_tick(const raft_sim_t* r) { return r ? r->tick : 0; }

int raft_sim_set_tick(raft_sim_t* r, uint64_t tick) {
  if (!r) return fail(-EINVAL, "null sim");
  if (!horizon_ok(r->cfg, tick, 0)) return fail(-ERANGE, "tick beyond the 32-bit horizon");
  for (Shard* s : r->sh) {
    const int rc = sh_sync(s);
    if (rc) return rc;
    s->tick = tick;
    s->storm_until = 0;
    // the packing keys are relative to the next launch's first tick: the next rebuild computes
    // them from the state
    s->keys_written = false;
  }
  r->tick = tick;
  return 0;
}

int raft_sim_last_step_timing(raft_sim_t* r, double* avg_kernel_ms, uint32_t* launches) {
  if (!r || !avg_kernel_ms || !launches) return fail(-EINVAL, "null argument");
  double sum = 0;
  uint32_t n = 0;
  for (Shard* s : r->sh) {
    sum += s->last_ms * s->last_launches;
    n += s->last_launches;
  }
  *avg_kernel_ms = n ? sum / n : 0.0;
  *launches = r->sh.empty() ? 0 : r->sh[0]->last_launches;
  return 0;
}

int raft_sim_last_span(raft_sim_t* r, double* span_ms) {
  if (!r || !span_ms) return fail(-EINVAL, "null argument");
  double m = 0;
  for (Shard* s : r->sh) m = std::max(m, s->last_step_ms);
  *span_ms = m;
  return 0;
}

// The shard owning cluster c, and c's index inside it.
static Shard* owner(raft_sim* r, uint32_t c, uint32_t* lc) {
  const size_t d = std::upper_bound(r->lo.begin() + 1, r->lo.end() - 1, c) - (r->lo.begin() + 1);
  *lc = c - r->lo[d];
  return r->sh[d];
}

// Run `fn(shard, local c0, count, offset into the caller's range)` over the per-shard pieces.
template <typename F>
static int pieces(raft_sim* r, uint32_t c0, uint32_t nc, F fn) {
  if (!r) return fail(-EINVAL, "null sim");
  if ((uint64_t)c0 + nc > r->cfg.n_clusters) return fail(-EINVAL, "cluster range out of bounds");
  for (uint32_t done = 0; done < nc;) {
    uint32_t lc;
    Shard* s = owner(r, c0 + done, &lc);
    const uint32_t n = std::min(s->C - lc, nc - done);
    const int rc = fn(s, lc, n, (size_t)done);
    if (rc) return rc;
    done += n;
  }
  return 0;
}

int raft_sim_read_nodes(raft_sim_t* r, uint32_t c0, uint32_t nc, raft_node_t* out) {
  if (!out) return fail(-EINVAL, "null output");
  return pieces(r, c0, nc, [&](Shard* s, uint32_t lc, uint32_t n, size_t off) {
    return sh_read_nodes(s, lc, n, out + off * r->cfg.nodes);
  });
}
int raft_sim_write_nodes(raft_sim_t* r, uint32_t c0, uint32_t nc, const raft_node_t* in) {
  if (!in) return fail(-EINVAL, "null input");
  return pieces(r, c0, nc, [&](Shard* s, uint32_t lc, uint32_t n, size_t off) {
    return sh_write_nodes(s, lc, n, in + off * r->cfg.nodes);
  });
}
int raft_sim_read_clusters(raft_sim_t* r, uint32_t c0, uint32_t nc, raft_cluster_t* out) {
  if (!out) return fail(-EINVAL, "null output");
  return pieces(r, c0, nc, [&](Shard* s, uint32_t lc, uint32_t n, size_t off) {
    return sh_read_clusters(s, lc, n, out + off);
  });
}
int raft_sim_write_clusters(raft_sim_t* r, uint32_t c0, uint32_t nc, const raft_cluster_t* in) {
  if (!in) return fail(-EINVAL, "null input");
  return pieces(r, c0, nc, [&](Shard* s, uint32_t lc, uint32_t n, size_t off) {
    return sh_write_clusters(s, lc, n, in + off);
  });
}
int raft_sim_digest(raft_sim_t* r, uint32_t c0, uint32_t nc, uint64_t* out) {
  if (!out) return fail(-EINVAL, "null output");
  return pieces(r, c0, nc, [&](Shard* s, uint32_t lc, uint32_t n, size_t off) {
    return sh_digest(s, lc, n, out + off);
  });
}

#define ROUTE_NODE(call)                                                                  \
  if (!r || cluster >= r->cfg.n_clusters) return fail(-EINVAL, "cluster/node out of bounds"); \
  uint32_t lc;                                                                            \
  Shard* s = owner(r, cluster, &lc);                                                      \
  return call;

int raft_sim_read_queue(raft_sim_t* r, uint32_t cluster, uint32_t id, uint32_t which,
                        raft_msg_t* out, uint32_t cap) {
  ROUTE_NODE(sh_read_queue(s, lc, id, which, out, cap))
}
int raft_sim_write_queue(raft_sim_t* r, uint32_t cluster, uint32_t id, uint32_t which,
                         const raft_msg_t* in, uint32_t count) {
  ROUTE_NODE(sh_write_queue(s, lc, id, which, in, count))
}
int raft_sim_read_arena(raft_sim_t* r, uint32_t cluster, uint32_t id, raft_entry_t* out,
                        uint32_t cap) {
  ROUTE_NODE(sh_read_arena(s, lc, id, out, cap))
}
int raft_sim_write_arena(raft_sim_t* r, uint32_t cluster, uint32_t id, const raft_entry_t* in,
                         uint32_t count) {
  ROUTE_NODE(sh_write_arena(s, lc, id, in, count))
}
int raft_sim_read_commit_stream(raft_sim_t* r, uint32_t cluster, uint32_t id, uint32_t* out,
                                uint32_t cap) {
  ROUTE_NODE(sh_read_commit_stream(s, lc, id, out, cap))
}
int raft_sim_write_commit_stream(raft_sim_t* r, uint32_t cluster, uint32_t id, const uint32_t* in,
                                 uint32_t count) {
  ROUTE_NODE(sh_write_commit_stream(s, lc, id, in, count))
}
int raft_sim_read_trace(raft_sim_t* r, uint32_t cluster, uint32_t id, uint32_t first,
                        raft_trace_event_t* out, uint32_t cap) {
  ROUTE_NODE(sh_read_trace(s, lc, id, first, out, cap))
}
int raft_sim_read_trace_entries(raft_sim_t* r, uint32_t cluster, uint32_t id, uint32_t first,
                                raft_entry_t* out, uint32_t cap) {
  ROUTE_NODE(sh_read_trace_entries(s, lc, id, first, out, cap))
}

int raft_sim_read_counters(raft_sim_t* r, raft_counters_t* out) {
  if (!r || !out) return fail(-EINVAL, "null argument");
  memset(out, 0, sizeof *out);
  out->first_violation_tick = UINT64_MAX;
  for (Shard* s : r->sh) {
    raft_counters_t c;
    const int rc = sh_read_counters(s, &c);
    if (rc) return rc;
    out->node_ticks += c.node_ticks;
    for (int i = 0; i < RAFT_CTR_COUNT; ++i) out->c[i] += c.c[i];
    out->first_violation_tick = std::min(out->first_violation_tick, c.first_violation_tick);
    out->payload_max = std::max(out->payload_max, c.payload_max);
  }
  return 0;
}

// Build identity (not part of include/raftsim.h): the hash of the kernel sources this library was
// compiled from (raftsim/_build.py; __graft_entry__.build_lib passes it), also findable in the
// file's bytes as "RAFTSIM_SRC_HASH=<hash>" without loading it.
#ifndef RAFTSIM_SRC_HASH
#define RAFTSIM_SRC_HASH "unknown"
#endif
static const char g_src_tag[] = "RAFTSIM_SRC_HASH=" RAFTSIM_SRC_HASH;
extern "C" const char* raftsim_src_hash(void) { return g_src_tag + 17; }

// Diagnostic (not part of include/raftsim.h): how many launches of the last sync window the
// average of raft_sim_last_step_timing is taken over (every general launch; the first steady
// launch after a sync), summed over shards.
extern "C" int raftsim_last_timed_launches(raft_sim_t* r) {
  if (!r) return fail(-EINVAL, "null sim");
  int n = 0;
  for (Shard* s : r->sh) n += (int)s->last_timed;
  return n;
}

// Diagnostic (not part of include/raftsim.h): clusters the steady kernel handed to the catch-up
// launch in the handle's last tick launch, summed over shards; -1 if that launch did not take the
// steady path (tests use it to check which path ran; results never depend on it).
extern "C" int raftsim_diag_last_bails(raft_sim_t* r) {
  if (!r) return fail(-EINVAL, "null sim");
  int total = 0;
  for (Shard* s : r->sh) {
    if (!s->steady_ok || !s->last_steady) return -1;
    uint32_t v = 0;
    HIP_OK(hipSetDevice(s->cfg.device));
    HIP_OK(hipStreamSynchronize(s->stream));
    HIP_OK(hipMemcpy(&v, s->nbail2 + (s->steady_parity ^ 1), 4, hipMemcpyDeviceToHost));
    total += (int)v;
  }
  return total;
}

// Diagnostic (not part of include/raftsim.h): clusters the storm kernel listed for the
// lane-per-node STORM body in the last storm-kernel launch (storm_kernel.hip), summed over shards;
// -1 if no shard has run one. Tests bound it: a regression that reruns most clusters shows here.
extern "C" int raftsim_diag_storm_bails(raft_sim_t* r) {
  if (!r) return fail(-EINVAL, "null sim");
  int total = 0;
  bool any = false;
  for (Shard* s : r->sh) {
    if (!s->storm_ran) continue;
    any = true;
    uint32_t v = 0;
    HIP_OK(hipSetDevice(s->cfg.device));
    HIP_OK(hipStreamSynchronize(s->stream));
    HIP_OK(hipMemcpy(&v, s->d.storm_count, 4, hipMemcpyDeviceToHost));
    total += (int)v;
  }
  return any ? total : -1;
}

#ifdef RS_WAVELOG
// Diagnostic builds only (not part of include/raftsim.h): the per-wave timeline of shard 0's last
// tick-kernel launch, 8 words per wave: start lo/hi, end lo/hi (100 MHz), active ticks, HW_ID,
// XCC_ID, launch t0. Returns the number of waves.
extern "C" int raftsim_diag_wavelog(raft_sim_t* r, uint32_t* out, uint32_t cap_waves) {
  Shard* s = r->sh[0];
  const uint32_t waves = rs::sched_slots_bound(s->C, s->N) / (64 / s->N);
  const uint32_t n = std::min(waves, cap_waves);
  HIP_OK(hipSetDevice(s->cfg.device));
  HIP_OK(hipMemcpy(out, s->d.wavelog, (size_t)n * 192, hipMemcpyDeviceToHost));
  return (int)n;
}
#endif

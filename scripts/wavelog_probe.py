"""Per-wave timeline of one general-kernel launch from a -DRS_WAVELOG build (diagnostic only):
lifetime distribution, start-time generations, per-CU/SIMD packing, per-phase shader cycles.
Usage: wavelog_probe.py LIB [clusters] [c2|c3|c3_spec|c4_n9|c4_spec] [launches]"""
import ctypes
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd")]
from raftsim._backend import Backend  # noqa: E402

lib = sys.argv[1]
C = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
WL = sys.argv[3] if len(sys.argv) > 3 else "c2"
C3 = dict(nodes=5, seed=1, log_cap=256, client_ppm=80000, client_period=16384, client_burst=2048,
          client_redirects=4, drop_ppm=100000, dup_ppm=10000, dmin=1, dmax=50, part_ppm=100000)
C4 = dict(nodes=9, seed=5, log_cap=4096, client_ppm=500000, client_period=8192, client_burst=2048,
          client_redirects=4)
CFG = {"c2": dict(nodes=5, seed=42), "c3": C3, "c3_spec": dict(C3, variant_flags=2, log_cap=1024), "c4_n9": C4,
       "c4_spec": dict(C4, variant_flags=2)}[WL]
LAUNCHES = int(sys.argv[4]) if len(sys.argv) > 4 else 4
sim = Backend(lib, "raft_sim_", n_clusters=C, **CFG)
for _ in range(LAUNCHES):                       # from init-node, as the bench's C3 window
    sim.step(10000)
waves = 2 * C // (64 // CFG["nodes"]) + 1000    # >= the padded packing's grid
buf = (ctypes.c_uint32 * (waves * 48))()
n = sim._lib.raftsim_diag_wavelog(sim._h, buf, waves)
a = np.frombuffer(buf, dtype=np.uint32).reshape(-1, 48)[:n].astype(np.int64)
a = a[(a[:, 0] | a[:, 1]) != 0]                 # waves that ran (padding waves exit first)
n = len(a)
start = (a[:, 0] | (a[:, 1] << 32)); end = (a[:, 2] | (a[:, 3] << 32))
t0 = start.min()
st, en = (start - t0) / 100.0, (end - t0) / 100.0        # microseconds
life = en - st
act = a[:, 4]
hw, xcc = a[:, 5], a[:, 6]
simd = (hw >> 4) & 3; cu = (hw >> 8) & 15; sh = (hw >> 12) & 1; se = (hw >> 13) & 7
print(f"kernel_ms {sim.last_step_timing()[0]:.3f} waves {n}  span {en.max():.1f} us")
q = lambda x: " ".join(f"{v:7.1f}" for v in np.percentile(x, [0, 10, 50, 90, 99, 100]))
print("life  us p0/10/50/90/99/100:", q(life))
print("start us p0/10/50/90/99/100:", q(st))
print("end   us p0/10/50/90/99/100:", q(en))
print("active ticks p0/10/50/90/99/100:", q(act))
print("us per active tick p0/10/50/90/99/100:", q(life / np.maximum(act, 1)))
for lo, hi in ((0, 5), (5, 40), (40, 100), (100, 1e9)):
    m = (st >= lo) & (st < hi)
    if m.any():
        print(f"started [{lo},{hi}) us: {m.sum():5d} waves, life median {np.median(life[m]):6.1f} us, "
              f"active median {np.median(act[m]):5.1f}, end max {en[m].max():6.1f}")
kspread, first = a[:, 7] >> 16, a[:, 7] & 0xFFFF
print("key spread in wave p0/10/50/90/99/100:", q(kspread))
print("first active tick p0/10/50/90/99/100:", q(first))
for lo_a in (18, 25, 35, 50):
    m = act >= lo_a
    print(f"waves with >= {lo_a} active: {m.sum():5d}  key spread median {np.median(kspread[m]) if m.any() else 0}"
          f"  first tick median {np.median(first[m]) if m.any() else 0}")
slow = life > np.percentile(life, 90)
print("slowest 10%: active median", np.median(act[slow]), "start median", np.median(st[slow]),
      "index median", np.median(np.nonzero(slow)[0]))
key = xcc * 10000 + se * 1000 + sh * 100 + cu * 4 + simd
u, cnt = np.unique(key, return_counts=True)
print("distinct SIMDs", len(u), "waves per SIMD p0/50/100", cnt.min(), np.median(cnt), cnt.max())
busy = {}
for k in u:
    m = key == k
    busy[k] = life[m].sum()
b = np.array(list(busy.values()))
print("per-SIMD summed wave-us p0/50/100:", b.min(), np.median(b), b.max())
per_xcc = [np.median(life[xcc == x]) for x in range(8)]
print("per-XCC median life:", " ".join(f"{v:.1f}" for v in per_xcc))
# wave-uniform phase stamps (shader cycles per wave, summed over its trips): rec[2..4] = ph0..11
# rec[2..4] = ph0..11: 11 P0 draws, 0 P0 insert, 1 pop, 2 handler, 10 timer/hash, 3 emission,
# 4 P2, 5 P3, 6 P4, 7 drain, 8 loop head
ph = a[:, [19, 8, 9, 10, 18, 23, 11, 12, 13, 14, 15, 16]].astype(np.float64)
names = ("P0-draw", "P0-ins", "P1-pop", "P1-hdl", "P1-tmr", "P1-redir", "P1-emit", "P2", "P3", "P4",
         "drain", "loop-head")
tot = ph.sum(axis=1)
trips = np.maximum(act, 1)[:, None]
print("phase cycles per trip (mean over waves): " + "  ".join(
    f"{nm} {v:7.0f}" for nm, v in zip(names, (ph / trips).mean(axis=0))))
print("phase cycles per wave (mean): " + "  ".join(
    f"{nm} {v:8.0f}" for nm, v in zip(names, ph.mean(axis=0))) + f"  load {a[:, 17].mean():8.0f}")
px = a[:, 24:32].astype(np.float64)
print("Philox passes per wave (mean): " + "  ".join(
    f"{nm} {v:7.1f}" for nm, v in zip(("client", "deferred", "alts", "spec-rearm", "redirect",
                                         "partition", "reply-net", "bcast-net"), px.mean(axis=0))))
print("drained ticks per wave p0/10/50/90/99/100:", q(a[:, 20]))
print("client-injection ticks per wave p0/10/50/90/99/100:", q(a[:, 21]))
print("dead clusters per wave at launch start p0/10/50/90/99/100:", q(a[:, 22]))
print("emission sub-phases per trip (partition, reply, bcast words, deliver): " + "  ".join(
    f"{v:7.0f}" for v in (a[:, 32:36].astype(np.float64) / np.maximum(act, 1)[:, None]).mean(axis=0)))
print(f"stamped cycles / lifetime cycles (2.4 GHz nominal): {np.median(tot / (life * 2400)):.2f}")

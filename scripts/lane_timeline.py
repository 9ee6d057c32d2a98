"""Per-wave timeline of the lane-per-cluster steady kernel from a -DRS_WAVELOG build (diagnostic
only): wave start/end, load / loop / write-back split, loop trips and events per lane.
Usage: lane_timeline.py LIB [clusters] [launches]"""
import ctypes
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd")]
from raftsim._backend import Backend  # noqa: E402

C = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
LAUNCHES = int(sys.argv[3]) if len(sys.argv) > 3 else 6
sim = Backend(sys.argv[1], "raft_sim_", n_clusters=C, nodes=5, seed=42)
for _ in range(LAUNCHES):
    sim.step(10000)
waves = 2 * C // 12 + 1000
buf = (ctypes.c_uint32 * (waves * 32))()
n = sim._lib.raftsim_diag_wavelog(sim._h, buf, waves)
a = np.frombuffer(buf, dtype=np.uint32).reshape(-1, 32)[:n].astype(np.int64)
a = a[(a[:, 0] | a[:, 1]) != 0]
start = a[:, 0] | (a[:, 1] << 32)
end = a[:, 2] | (a[:, 3] << 32)
t0 = start.min()
st, en = (start - t0) / 100.0, (end - t0) / 100.0
q = lambda x: " ".join(f"{v:8.1f}" for v in np.percentile(x, [0, 10, 50, 90, 99, 100]))
print(f"kernel_ms {sim.last_step_timing()[0]:.4f} waves {len(a)} span {en.max():.1f} us")
print("start us    p0/10/50/90/99/100:", q(st))
print("life us     p0/10/50/90/99/100:", q(en - st))
print("load us     p0/10/50/90/99/100:", q(a[:, 8] / 100.0))
print("loop us     p0/10/50/90/99/100:", q((a[:, 9] - a[:, 8]) / 100.0))
print("wb us       p0/10/50/90/99/100:", q((end - start - a[:, 9]) / 100.0))
print("trips       p0/10/50/90/99/100:", q(a[:, 4]))
if (a[:, 20] | a[:, 21] | a[:, 22]).any():   # fixed-point path stamps (round-5 builds)
    x1, x2, x3 = a[:, 20], a[:, 21], a[:, 22]
    print("  load..extracted  us:", q((x1 - a[:, 8]) / 100.0))
    print("  ..fp decided     us:", q((x2 - x1) / 100.0))
    print("  ..fp rounds done us:", q((x3 - x2) / 100.0))
    print("  ..general loop   us:", q((a[:, 9] - x3) / 100.0))
print("lanes on    p0/10/50/90/99/100:", q(a[:, 7]))
print("events/lane min p0/10/50/90/99/100:", q(a[:, 10]))
print("events/lane max p0/10/50/90/99/100:", q(a[:, 11]))
print("us per trip p0/10/50/90/99/100:", q((a[:, 9] - a[:, 8]) / 100.0 / np.maximum(a[:, 4], 1)))
done = a[:, 17] | (a[:, 18] << 32)
done = done[done != 0]
if len(done):
    print(f"workgroup done (stores drained, counters added) us after the first start: "
          f"p50 {np.percentile((done - t0) / 100.0, 50):.1f} max {(done.max() - t0) / 100.0:.1f}")
hw, xcc = a[:, 5], a[:, 6]
simd = (hw >> 4) & 3; cu = (hw >> 8) & 15; sh = (hw >> 12) & 1; se = (hw >> 13) & 7
key = xcc * 10000 + se * 1000 + sh * 100 + cu * 4 + simd
u, cnt = np.unique(key, return_counts=True)
print("distinct SIMDs", len(u), "waves per SIMD p0/50/100", cnt.min(), np.median(cnt), cnt.max())
ph = a[:, 12:17].astype(np.float64)
trips = np.maximum(a[:, 4], 1)[:, None]
names = ("head", "decide", "heartbeat", "-", "run (append-entries + responses)")
print("shader cycles per trip (mean over waves): " + "  ".join(
    f"{nm} {v:7.0f}" for nm, v in zip(names, (ph / trips).mean(axis=0))))
print("shader cycles per wave (mean): " + "  ".join(f"{nm} {v:8.0f}" for nm, v in zip(names, ph.mean(axis=0))))

"""Wave lifetimes from an RS_WAVETIME diagnostic build (-DRS_WAVETIME), launches after the first:
mean lifetime and active ticks of all waves and of slow ones (>= 150 us), how many slow waves were
dispatched in the second residency round (wave >= 4096), waves with > 40 active ticks, and the
slowest wave (lifetime, active ticks, wave index). s_memrealtime runs at 100 MHz.
Usage: python scripts/wavetime_probe.py LIB [clusters ...]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "raft-simulation_amd")]
from raftsim._backend import Backend  # noqa: E402

lib = sys.argv[1]
for c in [int(x) for x in sys.argv[2:]] or [65536, 16384]:
    sim = Backend(lib, "raft_sim_", n_clusters=c, nodes=5, seed=42)
    sim.step(10000)
    for rep in range(3):
        b = sim.counters()
        sim.step(10000)
        a = sim.counters()
        d = {k: a[k] - b[k] for k in a if isinstance(a[k], int) and isinstance(b[k], int)}
        waves = (c + 11) // 12
        slow = max(1, d["duplicated"])
        mx = a["to_halted"]
        print(f"clusters {c} waves {waves}: kernel {sim.last_step_timing()[0] * 1e3:.1f} us | all: life "
              f"{d['dropped'] * 0.01 / waves:.1f} us, active {d['partitioned'] / waves:.1f}, >40 active "
              f"{d['viol_election']} | slow: {d['duplicated']} waves, life {d['client_injected'] * 0.01 / slow:.1f} us, "
              f"active {d['overflow'] / slow:.1f}, 2nd round {d['entries_applied']} | slowest so far: "
              f"{(mx >> 40) * 0.01:.1f} us, active {(mx >> 24) & 0xFFFF}, wave {mx & 0xFFFFFF}", flush=True)
    sim.close()

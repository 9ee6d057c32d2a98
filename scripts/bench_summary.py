"""One line per workload of a bench.py JSON line: value, ms/step, frac, traffic, live, ev_ae, CPU."""
import json
import sys

rec = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
rows = [("c2(head)", rec)] + list(rec.get("workloads", {}).items())
for name, r in rows:
    rf = r["roofline"]
    cpu = r.get("cpu_baseline", {})
    print(f"{name:10s} value {r['value']:.3e} ms/step {r.get('ms_per_step', float('nan')):.4f} "
          f"launch {rf['avg_launch_ms']:.4f} frac {rf['frac']:.4f} ev-frac {rf['frac_event_model']:.3f} "
          f"traffic {rf['traffic'] or 0:.3e} live {r.get('live_node_frac_end', float('nan')):.3f} "
          f"ev_ae {r.get('ev_ae', '-')} pmax {r.get('payload_max', '-')} "
          f"cpu {cpu.get('value', 0):.3e} fv {r.get('first_violation_tick', '-')}")

"""One line per workload of bench.py's compact JSON line: value, ms/step, frac, frac_measured,
traffic, LDS conflicts, waves per SIMD, live fraction, ev_ae, CPU rate."""
import json
import sys

rec = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
head = dict(rec["roofline"], value=rec["value"], ms_per_step=rec["ms_per_step"],
            cpu=rec.get("cpu_baseline", {}).get("value"))
rows = [("c2(head)", head)] + list(rec.get("workloads", {}).items())


def f(x, spec):
    return format(x, spec) if isinstance(x, (int, float)) else "-"


for name, r in rows:
    print(f"{name:10s} value {f(r['value'], '.3e')} ms/step {f(r.get('ms_per_step'), '.4f')} "
          f"frac {f(r.get('frac'), '.4f')} meas {f(r.get('frac_measured'), '.4f')} "
          f"traffic {f(r.get('traffic'), '.3e')} ldsc {f(r.get('lds_bank_conflict_per_lds_inst'), '.3f')} "
          f"w/simd {f(r.get('waves_per_simd'), '.2f')} live {f(r.get('live_node_frac_end'), '.3f')} "
          f"ev_ae {r.get('ev_ae', '-')} cpu {f(r.get('cpu'), '.3e')} "
          f"fv {r.get('first_violation_tick', '-')}")
print(len(json.dumps(rec)), "chars")

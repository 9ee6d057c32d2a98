# Cost attribution (diagnostic only): builds with one piece of per-event work removed -- their
# results are wrong by construction and they never ship -- timed against the product build in one
# process (scripts/ab_probe.py). Usage: bash scripts/cost_probe.sh (build here), then on the GPU:
#   python scripts/ab_probe.py build/libraftsim_new.so build/libraftsim_cost_*.so --c2 --c3
set -e
bash "$(dirname "$0")/build_variants.sh" cost_noctr "-DRS_COST_NOCTR" cost_notrace "-DRS_COST_NOTRACE" \
  cost_nophilox "-DRS_COST_NOPHILOX" cost_noevctr "-DRS_COST_NOEVCTR" cost_none "-DRS_COST_NOCTR -DRS_COST_NOTRACE -DRS_COST_NOPHILOX"

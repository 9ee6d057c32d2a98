# Build kernel variants for scripts/ab_probe.py: build/libraftsim_<name>.so with extra -D flags.
# Usage: bash scripts/build_variants.sh name1 "-DFLAG=1 ..." name2 "..." ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/raft-simulation_amd/csrc
while [ $# -ge 2 ]; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall $2 \
    -o $R/raft-simulation_amd/build/libraftsim_$1.so $C/tick_kernel.hip $C/steady_kernel.hip $C/storm_kernel.hip $C/raftsim.hip &
  shift 2
done
wait

# VGPRs / occupancy of ONE tick-kernel instantiation (fast: the launchers that instantiate every N
# are compiled out). Usage: bash scripts/quick_vgpr.sh N TRACE SPEC LITE [extra hipcc flags]
R=$(cd "$(dirname "$0")/.." && pwd)
F=$(mktemp /tmp/qv_XXXX.hip)
printf '#define RS_KERNEL_ONLY\n#include "%s/raft-simulation_amd/csrc/tick_kernel.hip"\ntemplate __global__ void rs::tick_kernel<%s, %s, %s, %s>(rs::DevSim, uint32_t, uint32_t);\n' \
  "$R" "$1" "$2" "$3" "$4" > $F
shift 4
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -S --cuda-device-only "$@" -o $F.s $F 2>&1 | grep -v warning
python3 - $F.s <<'PY'
import re, sys
s = open(sys.argv[1]).read()
i = s.index('_ZN2rs11tick_kernel'); t = s[s.index('.Lfunc_end', i):][:4000]
pat = lambda k: re.search("; " + k + r": (\d+)", t)[1]
print(" ".join(k + "=" + pat(k) for k in ("NumVgprs", "TotalNumSgprs", "ScratchSize", "Occupancy")))
PY
rm -f $F $F.s

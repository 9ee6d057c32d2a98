# Registers, scratch and occupancy of every tick-kernel instantiation as the compiler reports them
# (ISA comments of hipcc -S), written to profiles/TAG_kernel_resources.txt. rocprofv3's
# VGPR_Count column uses a different encoding; these are the compiler's own counts.
# Usage: bash scripts/kernel_resources.sh TAG
set -e
TAG=${1:-r12}
R=$(cd "$(dirname "$0")/.." && pwd)
S=$(mktemp /tmp/tick_kernel_XXXX.s)
S2=$(mktemp /tmp/steady_kernel_XXXX.s)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -S --cuda-device-only -o $S \
  $R/raft-simulation_amd/csrc/tick_kernel.hip 2>/dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -S --cuda-device-only -o $S2 \
  $R/raft-simulation_amd/csrc/steady_kernel.hip 2>/dev/null
python3 - "$S" "$S2" > $R/profiles/${TAG}_kernel_resources.txt <<'PY'
import re, sys
s = open(sys.argv[1]).read() + open(sys.argv[2]).read()
print(f"{'kernel':48s} {'VGPRs':>5s} {'SGPRs':>5s} {'scratch':>7s} {'waves/SIMD':>10s}")
for m in re.finditer(r'^(_ZN2rs\w+):\s', s, re.M):
    name = m.group(1)
    body = s[m.end():s.index('.Lfunc_end', m.end())]
    tail = s[s.index('.Lfunc_end', m.end()):][:4000]
    get = lambda k: (re.search(r'; ' + k + r': (\d+)', tail) or [None, '?'])[1]
    pretty = name.replace('_ZN2rs', 'rs::')
    mt = re.match(r'rs::11tick_kernelILi(\d)ELb(\d)ELb(\d)ELb(\d)ELb(\d)', pretty)
    if mt:
        pretty = (f"tick_kernel<N={mt.group(1)}, TRACE={mt.group(2)}, SPEC={mt.group(3)}, "
                  f"LITE={mt.group(4)}{', STORM' if mt.group(5) == '1' else ''}>")
    ml = re.match(r'rs::18steady_lane_kernelILi(\d)E', pretty)
    if ml:
        pretty = f"steady_lane_kernel<N={ml.group(1)}>"
    print(f"{pretty[:48]:48s} {get('NumVgprs'):>5s} {get('TotalNumSgprs'):>5s} {get('ScratchSize'):>7s} {get('Occupancy'):>10s}")
PY
rm -f $S $S2
cat $R/profiles/${TAG}_kernel_resources.txt

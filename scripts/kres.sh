# Print VGPR / scratch / occupancy of every tick kernel (gfx950) and dump tick_kernel<5>'s ISA to /tmp/k5.s.
cd /tmp && hipcc --offload-arch=gfx950 -O3 -std=c++17 -c $GRAFT_SRC/raft-simulation_amd/csrc/tick_kernel.hip -save-temps -Rpass-analysis=kernel-resource-usage -o /tmp/tk.o 2>&1 \
 | python3 -c "
import sys,re
name=None; row={}
for l in sys.stdin:
    m=re.search(r'Function Name: (\S+)',l)
    if m:
        name=m.group(1); continue
    m=re.search(r'(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)',l)
    if m and name and 'tick' in name:
        row.setdefault(name,[]).append(m.group(2))
for k,v in row.items(): print(re.search(r'ILi(\d)',k).group(1), 'vgpr/scratch/occ', v)
"
awk '/^_ZN2rs11tick_kernelILi5EEEvNS_6DevSimEjj:/,/s_endpgm/' /tmp/tick_kernel-hip-amdgcn-amd-amdhsa-gfx950.s > /tmp/k5.s

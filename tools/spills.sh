#!/bin/bash
# VGPR / spill counts of k_trace<false> (rtg_kernels.hip) and k_shade<false> (rtg_shade.hip, with its
# build flags) for a set of -D flags: spills.sh "-DFOO=1" ...
D="$(dirname "$0")/../raytracingrenderer_amd/csrc/device"
for flags in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 --cuda-device-only -S $flags \
    -o /tmp/spills_k.s "$D/rtg_kernels.hip" 2>/dev/null
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 --cuda-device-only -S $flags \
    -mllvm -amdgpu-sched-strategy=max-ilp -o /tmp/spills_s.s "$D/rtg_shade.hip" 2>/dev/null
  python3 - "$flags" <<'PY'
import re, sys
out = []
for f in ('/tmp/spills_k.s', '/tmp/spills_s.s'):
    s = open(f).read()
    md = s[s.index('amdhsa.kernels'):]
    for blk in md.split('  - .agpr_count')[1:]:
        name = re.search(r'\.name:\s+(\S+)', blk).group(1)
        if name.startswith(('_Z7k_traceILb0E', '_Z7k_shadeILb0E')):
            g = lambda k: re.search(r'\.' + k + r':\s+(\d+)', blk).group(1)
            out.append('%s v%s/spill%s s-spill%s' % (name[7:20], g('vgpr_count'), g('vgpr_spill_count'), g('sgpr_spill_count')))
print(repr(sys.argv[1]), ' | '.join(out))
PY
done

#!/bin/bash
# build A/B variants of librtg into raytracingrenderer_amd/lib/ab: mkab.sh name "-DFOO=1" [name "-D..."]...
set -e
cd "$(dirname "$0")/.."
mkdir -p raytracingrenderer_amd/lib/ab
D=raytracingrenderer_amd/csrc/device
while [ $# -ge 2 ]; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -fPIC -shared $2 \
    -o raytracingrenderer_amd/lib/ab/$1.so $D/rtg_kernels.hip $D/rtg_shade.hip $D/rtg_light.hip $D/rtg_multi.hip \
    -ldl -Wl,-rpath,/opt/rocm/lib &
  shift 2
done
wait

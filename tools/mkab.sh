#!/bin/bash
# build A/B variants of librtg into raytracingrenderer_amd/lib/ab (the product's units and per-unit
# flags, build.py build_variant): mkab.sh name "-DFOO=1" [name "-D..."]...  ("" = the product as is)
set -e
cd "$(dirname "$0")/.."
rm -rf raytracingrenderer_amd/lib/ab; mkdir -p raytracingrenderer_amd/lib/ab
while [ $# -ge 2 ]; do
  python3 -c "import sys; from raytracingrenderer_amd import build; build.build_variant(sys.argv[1], sys.argv[2].split())" "$1" "$2" &
  shift 2
done
wait
ls raytracingrenderer_amd/lib/ab

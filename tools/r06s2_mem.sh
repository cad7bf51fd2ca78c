#!/bin/bash
# Round 6 (late): the chunk memory budget (lib/ab: a_prod = half the free HBM, b_mem60 = 60 %): C5 at
# 32 spp (two 16-spp chunks vs one 32-spp chunk) and C3 / C4 (unchanged chunking).
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
CFGS="${CFGS:-C5 C3 C4}" timeout -k 10 900 bash tools/ab_cfg.sh > gpurun_out/ab_mem.txt 2>&1 || { cat gpurun_out/ab_mem.txt; exit 1; }
cat gpurun_out/ab_mem.txt

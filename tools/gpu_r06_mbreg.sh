#!/bin/bash
# round 6: the register-resident pop engine (tools/mb/heap_pop k_heap_reg) against the shipped one (v34 = v40)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${OUTDIR:-r06mbr}
mkdir -p $OUT
D=pfilter-noetic_amd/var/dumps
HEAP_DUMP=$D/c4heaps.bin timeout -k 10 120 ./tools/mb/heap_pop 2 34 > $OUT/mb_c4.txt 2>&1 || { tail -5 $OUT/mb_c4.txt; exit 1; }
grep -v "^full" $OUT/mb_c4.txt

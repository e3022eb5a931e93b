#!/bin/bash
# round 6: the shipped pop engine (tools/mb/heap_pop v34 = v40) on real depth-limit segments dumped by the
# oracle (PFREF_HEAP_DUMP): headline S64 frames 3000-3120 and configs[4]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${OUTDIR:-r06mbd}
mkdir -p $OUT
D=pfilter-noetic_amd/var/dumps
HEAP_DUMP=$D/s64heaps.bin HEAP_DUMP_SKIP=${SKIP:-455} HEAP_DUMP_MAX=24 timeout -k 10 120 ./tools/mb/heap_pop 2 ${V:-34} > $OUT/mb_s64.txt 2>&1 || { tail -5 $OUT/mb_s64.txt; exit 1; }
HEAP_DUMP=$D/c4heaps.bin timeout -k 10 120 ./tools/mb/heap_pop 2 ${V:-34} > $OUT/mb_c4.txt 2>&1 || { tail -5 $OUT/mb_c4.txt; exit 1; }
grep -E "dump|asc|map  " $OUT/mb_s64.txt | grep -v "^full"
grep -E "dump" $OUT/mb_c4.txt | grep -v "^full"

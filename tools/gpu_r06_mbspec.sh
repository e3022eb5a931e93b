#!/bin/bash
# round 6: the speculative-start pop engine (tools/mb/heap_pop v35-37 = pops_spec<1,2,4>) against the
# shipped one (v34 = v40), synthetic cases and real dumped depth-limit segments (headline S64, configs[4])
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${OUTDIR:-r06mbs}
mkdir -p $OUT
D=pfilter-noetic_amd/var/dumps
HEAP_DUMP=$D/c4heaps.bin timeout -k 10 120 ./tools/mb/heap_pop 2 34 ${VHI:-38} > $OUT/mb_c4.txt 2>&1 || { tail -5 $OUT/mb_c4.txt; exit 1; }
HEAP_DUMP=$D/s64heaps.bin HEAP_DUMP_MAX=12 timeout -k 10 120 ./tools/mb/heap_pop 2 34 ${VHI:-38} > $OUT/mb_s64.txt 2>&1 || { tail -5 $OUT/mb_s64.txt; exit 1; }
grep -v "^full" $OUT/mb_c4.txt | grep -v "^reg"
grep -E "dump" $OUT/mb_s64.txt

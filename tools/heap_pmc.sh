#!/bin/bash
# PMC of k_tie_heap's pop pipeline alone: tools/heap_prof.py on one depth-0 segment of N keys (every key
# heap-sorted, three calls), k_tie_heap only, one counter group per pass. The dispatch's counters are
# then those of the one workgroup that sorts (the others exit at once): instructions per pop, and
# where the pop wave's cycles go (VALU issue, issue stalls, s_waitcnt waits).
#   tools/heap_pmc.sh N
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
N=${1:-15000}
OUT=gpurun_out/heappmc_$N
mkdir -p $OUT
GROUPS_=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_BRANCH"
)
i=0
for grp in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_tie_heap" -d $OUT/p$i -o run \
      --output-format csv -- python3 tools/heap_prof.py $N > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/frame_pmc.py $OUT --source "rocprofv3 --pmc (tools/heap_pmc.sh $N): k_tie_heap on one depth-0 segment of $N keys (tools/heap_prof.py)"
find $OUT -name "*.csv" -delete

#!/bin/bash
# PMC passes over the odometry frame path (eager launches, so every kernel is its own dispatch): one
# counter group per pass, each pass under its own limit; then the per-kernel table for the stage-B
# kernels (tools/frame_pmc.py -> gpurun_out/framepmc/frame_pmc.json).
#   tools/frame_pmc.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/framepmc
mkdir -p $OUT
GROUPS_=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for grp in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -s KILL ${PASS_LIMIT:-120} rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- \
      python3 bench.py --steps ${STEPS:-100} --warmup 10 --no-graph --only-headline --order ${ORDER:-stable} \
      > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/frame_pmc.py $OUT --source "rocprofv3 --pmc passes (tools/frame_pmc.sh) over bench.py --steps ${STEPS:-100} --warmup 10 --no-graph --order ${ORDER:-stable} (configs[1], S64)"
# gpurun copies back at most 64 MiB: keep the summary, drop the per-dispatch counter rows
find $OUT -name "*.csv" -delete

#!/bin/bash
# PMC of the tie-order sort's kernels (k_tie_*, k_rg_dep) over a window of the headline sequence:
# the estimator state before the window is saved by an unprofiled process (tools/snap_probe.py), and
# each counter pass profiles only the window (eager launches, the tie kernels only), so that neither the
# frames before it nor its own packets wrap the AQL ring (rocprofv3's interception reads past the ring's
# end on a wrapped batch: profiles/r05_graph_ring/). One counter group per pass, each under its own limit.
#   tools/tie_pmc.sh K N     (window frames K .. K+N-1)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
K=${1:-3500}; N=${2:-120}
OUT=gpurun_out/tiepmc_$K
mkdir -p $OUT
timeout -k 10 200 python3 tools/snap_probe.py save $K $OUT/snap.bin > $OUT/save.log 2>&1 || { echo "save failed"; tail -5 $OUT/save.log; exit 1; }
GROUPS_=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for grp in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_tie|k_rg_dep" -d $OUT/p$i -o run \
      --output-format csv -- python3 tools/snap_probe.py run $K $N $OUT/snap.bin eager \
      > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/frame_pmc.py $OUT --source "rocprofv3 --pmc passes (tools/tie_pmc.sh $K $N): frames $K..$((K+N-1)) of the headline sequence (configs[1], S64, reference tie order) from a saved state, eager launches, tie kernels only"
find $OUT -name "*.csv" -delete
rm -f $OUT/snap.bin

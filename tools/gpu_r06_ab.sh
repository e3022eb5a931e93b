#!/bin/bash
# round 6: pop-engine variants, partition-tier level profile (LDS rank cache on / off), tie / odometry tests,
# headline A/B: default (aux heap launch + rank cache), PF_TIE_AUX=0, rank cache off (var/nocache)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${OUTDIR:-r06ab}
mkdir -p $OUT
timeout -k 10 120 ./tools/mb/heap_pop 3 > $OUT/heap_pop.txt 2>&1 || { tail -5 $OUT/heap_pop.txt; exit 1; }
grep -v "^full" $OUT/heap_pop.txt | grep -v small | grep -E "ties +n  15000|map|dist" 
for v in tieprof6n tieprof6; do for a in "26000 -3500" "26000 -300"; do
  PFILTER_HIP_LIB=pfilter-noetic_amd/var/$v/libpfilter_hip.so timeout -k 10 120 python3 tools/tie_prof.py $a > "$OUT/${v}_${a// /_}.txt" 2>&1 || { tail -5 "$OUT/${v}_${a// /_}.txt"; exit 1; }
done; done
timeout -k 10 900 python -u -m pytest tests/test_gpu_tie.py tests/test_gpu_odom.py tests/test_gpu_rgm.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "not long_sequence and not full_sequence" > $OUT/pytest.txt 2>&1
rc=$?; tail -3 $OUT/pytest.txt; [ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --only-headline > $OUT/headline_$name.json 2> $OUT/headline_$name.err || { tail -5 $OUT/headline_$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/headline_$name.json').read().strip().splitlines()[-1]); print('$name value', d['value'], d.get('stage_us'))"
}
run base PF_TIE_AUX=1
run noaux PF_TIE_AUX=0
run nocache PF_TIE_AUX=1 PFILTER_HIP_LIB=pfilter-noetic_amd/var/nocache/libpfilter_hip.so
run pop1 PF_TIE_AUX=1 PFILTER_HIP_LIB=pfilter-noetic_amd/var/pop1/libpfilter_hip.so
run base2 PF_TIE_AUX=1

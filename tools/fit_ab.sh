cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in "" NOEIG NOQR NOPUSH; do
  if [ -n "$v" ]; then export PFILTER_HIP_LIB=pfilter-noetic_amd/var/$v/libpfilter_hip.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pv_$v -o run --output-format csv -- python3 bench.py --steps 300 --no-cpu --no-graph --no-roofline --bpf-frames 0 > /dev/null 2>&1 || exit 1
  echo "== ${v:-main} $(grep -h 'k_assoc' $(find gpurun_out/pv_$v -name '*kernel_stats.csv') | cut -d, -f4)"
done

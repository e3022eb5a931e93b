set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/tie
timeout -k 10 300 python -u tools/tie_probe.py 1000 > gpurun_out/tie/probe.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tie/prof -o run --output-format csv -- python3 tools/tie_probe.py 300 S64 tie > gpurun_out/tie/prof.txt 2>&1 &&
python3 tools/kstats.py $(find gpurun_out/tie/prof -name "*kernel_stats.csv" | head -1) 30 > gpurun_out/tie/kstats.txt; find gpurun_out/tie/prof -name "*_kernel_trace.csv" -delete; cat gpurun_out/tie/probe.txt gpurun_out/tie/kstats.txt

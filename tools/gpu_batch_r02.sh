set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -s -p no:cacheprovider --timeout 250 --timeout-method thread tests/test_gpu_odom.py -k "full_sequence" > gpurun_out/t_full.log 2>&1 || exit 1
PFILTER_HIP_LIB=pfilter-noetic_amd/var/bounds/libpfilter_hip.so timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_cls.py tests/test_gpu_bpf.py tests/test_gpu_fe.py > gpurun_out/t_bounds.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --sequences kitti11 > gpurun_out/b_kitti11.json 2> gpurun_out/b_kitti11.err || exit 1
timeout -k 10 200 python bench.py --knn-shard > gpurun_out/b_knn.json 2> gpurun_out/b_knn.err || exit 1
timeout -k 10 600 python bench.py > gpurun_out/b_full.json 2> gpurun_out/b_full.err || exit 1

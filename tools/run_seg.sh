# Segmentation tests + bench (with the raw-document line) + kernel trace.
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-seg}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_segment_gpu.py > $O/seg_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --steps 3 --no-cpu-baseline --no-alt-rng > $O/bench_c2.log 2>&1 || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o b -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-alt-rng > $O/trace.log 2>&1 || exit 4
echo ALLDONE

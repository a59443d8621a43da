cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-seg2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_segment_gpu.py > $O/seg_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/seg_bench.py 2 > $O/seg_bench.log 2>&1 || exit 2
echo ALLDONE

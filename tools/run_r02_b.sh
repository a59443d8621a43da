cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_utf8_gpu.py tests/test_output_gpu.py tests/test_segment_gpu.py > $O/gpu_tests.log 2>&1
bash tools/run_e2e.sh $1 || exit 1
echo ALLDONE

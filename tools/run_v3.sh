cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/v4
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_output_gpu.py > gpurun_out/v4/tests.log 2>&1 || exit 1
bash tools/run_variants.sh v4 base || exit 2
echo ALLDONE

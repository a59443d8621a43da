cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/x1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_output_gpu.py > gpurun_out/x1/tests.log 2>&1 || exit 1
bash tools/prof_mix.sh x1 || exit 2
echo ALLDONE

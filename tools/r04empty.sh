set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r04empty
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_pairs_gpu.py -k empty > gpurun_out/r04empty/tests.log 2>&1
echo "rc=$?"

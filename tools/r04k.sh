set -o pipefail
mkdir -p gpurun_out/r04k
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_native_gpu.py tests/test_pairs_gpu.py tests/test_output_gpu.py > gpurun_out/r04k/tests.log 2>&1
echo "tests rc=$?"
AB_TESTS=none bash tools/ab.sh r04k/ab base plain nomask notokst

set -o pipefail
mkdir -p gpurun_out/r04p
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_tokenize_gpu.py > gpurun_out/r04p/tests.log 2>&1
echo "tests rc=$?"
LDDL_SHUFFLE_GLOBAL=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_pairs_gpu.py > gpurun_out/r04p/tests_global.log 2>&1
echo "global tests rc=$?"
bash tools/run_trace_copies.sh r04p/trace || exit 1

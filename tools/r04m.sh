set -o pipefail
mkdir -p gpurun_out/r04m
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_output_gpu.py > gpurun_out/r04m/tests.log 2>&1
echo "tests rc=$?"
bash tools/run_trace_copies.sh r04m/trace || exit 1
bash tools/r04l.sh

set -o pipefail
mkdir -p gpurun_out/r04zb
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04zb/tests.log 2>&1 || exit 1
echo tests ok
bash tools/run_trace_copies.sh r04zb/trace || exit 1

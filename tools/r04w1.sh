set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r04w1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_output_gpu.py tests/test_balance.py > gpurun_out/r04w1/tests.log 2>&1 || exit 1
echo tests ok
bash tools/run_trace_copies.sh r04w1/trace --workload c3 || exit 1

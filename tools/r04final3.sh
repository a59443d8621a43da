set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r04f3
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04f3/gpu_tests_pre.log 2>&1 || exit 1
echo tests ok
bash tools/prof_counters.sh r04pmc3 || exit 2
echo pmc ok
bash tools/run_full.sh r04f3 || exit 3
echo full ok
bash tools/run_trace_copies.sh r04f3/trace_native --rng native || exit 4
echo ALLDONE

# half-wave planner: pair parity tests, then C2 bench with the new planner and with LDDL_PLAN_V1=1
# usage: bash tools/run_planh.sh <tag> [tests]
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu ${2:-tests/test_pairs_gpu.py tests/test_output_gpu.py tests/test_native_gpu.py} > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench_half_$r.log 2>&1 || exit 2
  echo "half r$r $(grep -o '"stages_ms": {[^}]*}' $O/bench_half_$r.log)" >> $O/summary.txt
  LDDL_PLAN_V1=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench_v1_$r.log 2>&1 || exit 3
  echo "v1 r$r $(grep -o '"stages_ms": {[^}]*}' $O/bench_v1_$r.log)" >> $O/summary.txt
done
echo ALLDONE

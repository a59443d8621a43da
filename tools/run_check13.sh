# round-2 final checkpoint: GPU tests, smoke, default C2 bench, C4 / C5 lines, then the counter
# passes + kernel trace of tools/prof_counters.sh. usage: bash tools/run_check13.sh <tag> <prof tag>
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > $O/bench_c2.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline > $O/bench_c4.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > $O/bench_c5.log 2>&1 || exit 5
bash tools/prof_counters.sh $2 || exit 6
echo ALLDONE

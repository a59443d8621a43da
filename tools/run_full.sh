# Round checkpoint: full GPU tests, smoke, default bench (driver command), C5, C4 at N=1.
# usage: bash tools/run_full.sh <tag>
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 900 python -u -m pytest --maxfail=10 -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py > $O/bench_c2.log 2>&1 || exit 2
timeout -k 10 600 python -u bench.py --workload c5 --steps 200 --warmup 20 > $O/bench_c5.log 2>&1 || exit 3
timeout -k 10 600 python -u bench.py --workload c4 --no-cpu-baseline --no-segmented-line > $O/bench_c4.log 2>&1 || exit 4
echo ALLDONE

# checkpoint: full GPU tests, smoke, default bench (driver command) -> <tag>; usage: bash tools/run_ckpt.sh <tag>
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 900 python -u -m pytest --maxfail=10 -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py > $O/bench_c2.log 2>&1 || exit 2
echo ALLDONE

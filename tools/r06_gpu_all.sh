# round 6: the GPU test suite in one process, then the default bench line
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-r06g}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest --maxfail=5 -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" $O/gpu_tests.log | head -20; tail -5 $O/gpu_tests.log; exit 2; }
tail -2 $O/gpu_tests.log
[ -n "$2" ] && { timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 $O/bench.log; exit 3; }; tail -c 3000 $O/bench.log; }
echo ALLDONE

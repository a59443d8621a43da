# round 6: pair tests, then C3 (seq 512, 64 bins, balance into 8 shards) with a kernel trace
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-r06k}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_pairs_gpu.py > $O/pairs_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/pairs_tests.log; exit 2; }
tail -1 $O/pairs_tests.log
timeout -k 10 600 python -u bench.py --workload c3 --no-cpu-baseline --no-alt-rng --no-segmented-line > $O/bench_c3.log 2>&1 || { echo BENCH_FAILED; tail -20 $O/bench_c3.log; exit 3; }
python - $O/bench_c3.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('C3', d['value'] / 1e9, d['ms_per_step'], d['stages_ms'])
PY
( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /root/repo/$O/tr -o k -- python3 /root/repo/bench.py --workload c3 --no-cpu-baseline --no-alt-rng --no-segmented-line --steps 1 --warmup 0 > /root/repo/$O/tr.log 2>&1 ) || { echo TRACE_FAILED; tail -5 $O/tr.log; exit 4; }
python tools/prof_summary.py $O/tr $O/c3_kernels && head -8 $O/c3_kernels.txt | cut -c1-120
echo ALLDONE

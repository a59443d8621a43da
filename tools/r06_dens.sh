# round 6: densify with 4 chunks' loads in flight + masked-only gather staging writes: GPU tests, C2 kernel stats (replay + native)
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-r06x}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_native_gpu.py tests/test_output_gpu.py > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_native -o run -- python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --rng native --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench_native.log 2>&1 || { echo NATIVE_FAILED; exit 4; }
python tools/prof_summary.py $O/prof_native $O/kernels_native && head -12 $O/kernels_native.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 --warmup 1 --no-segmented-line --no-extra-lines > $O/bench_c2.log 2>&1 || { echo BENCH_FAILED; exit 5; }
python - $O/bench_c2.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('C2 %.2f G/s' % (d['value'] / 1e9), 'ms %.1f' % d['ms_per_step'], d['stages_ms'], 'native', d['alt_rng'])
PY
echo ALLDONE

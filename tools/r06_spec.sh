# round 6 A/B: speculative prefetch of the random-next document's length window (base) vs none (nospec)
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-r06s2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_output_gpu.py > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
i=0
for v in base nospec base nospec; do
  i=$((i+1))
  lib=lddl_amd/_lib/liblddl_amd.so; [ $v != base ] && lib=lddl_amd/_lib_$v/liblddl_amd.so
  LDDL_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench_${v}_$i.log 2>&1 || { echo BENCH_FAILED $v; tail -3 $O/bench_${v}_$i.log; exit 3; }
  python - $O/bench_${v}_$i.log $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('C2', sys.argv[2], '%.2f G/s' % (d['value'] / 1e9), '%.1f ms' % d['ms_per_step'], 'plan', d['stages_ms'].get('per_step_plan'))
PY
done
for v in base nospec; do
  lib=lddl_amd/_lib/liblddl_amd.so; [ $v != base ] && lib=lddl_amd/_lib_$v/liblddl_amd.so
  LDDL_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --workload c3 --no-cpu-baseline --steps 3 --warmup 1 --no-alt-rng --no-segmented-line --no-extra-lines > $O/c3_$v.log 2>&1 || { echo C3_FAILED $v; exit 4; }
  python - $O/c3_$v.log $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('C3', sys.argv[2], '%.2f G/s' % (d['value'] / 1e9), 'plan', d['stages_ms'].get('per_step_plan'))
PY
done
echo ALLDONE

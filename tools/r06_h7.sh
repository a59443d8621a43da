# round 6 A/B: planner launch bound (64, 7) (h7: 94 SGPRs, 82 spilled, 8 waves/SIMD by LDS) vs (64, 6) (product: 106 SGPRs, 7 waves/SIMD)
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-r06h7}
mkdir -p $O
LDDL_AMD_LIB=lddl_amd/_lib_h7/liblddl_amd.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pairs_gpu.py -k golden > $O/tests_h7.log 2>&1 || { echo TESTS_FAILED; tail -20 $O/tests_h7.log; exit 1; }
tail -1 $O/tests_h7.log
i=0
for v in base h7 base h7; do
  i=$((i+1))
  lib=lddl_amd/_lib/liblddl_amd.so; [ $v != base ] && lib=lddl_amd/_lib_$v/liblddl_amd.so
  LDDL_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench_${v}_$i.log 2>&1 || { echo BENCH_FAILED $v; tail -3 $O/bench_${v}_$i.log; exit 3; }
  python - $O/bench_${v}_$i.log $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('C2', sys.argv[2], '%.2f G/s' % (d['value'] / 1e9), '%.1f ms' % d['ms_per_step'], 'plan', d['stages_ms'].get('per_step_plan'))
PY
done
echo ALLDONE

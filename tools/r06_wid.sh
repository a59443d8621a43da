# round 6 A/B: wave-uniform wave index (wave_id) in densify / mask_native / gathers / Punkt / render / collate
# kernels (product) vs before (pold): GPU test suite, then C2 bench lines (replay + native + segmented) x2
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-r06w2}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest --maxfail=5 -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" $O/gpu_tests.log | head -20; tail -5 $O/gpu_tests.log; exit 2; }
tail -1 $O/gpu_tests.log
i=0
for v in base pold base pold; do
  i=$((i+1))
  lib=lddl_amd/_lib/liblddl_amd.so; [ $v != base ] && lib=lddl_amd/_lib_$v/liblddl_amd.so
  LDDL_AMD_LIB=$lib timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --no-extra-lines > $O/bench_${v}_$i.log 2>&1 || { echo BENCH_FAILED $v; tail -3 $O/bench_${v}_$i.log; exit 3; }
  python - $O/bench_${v}_$i.log $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('C2', sys.argv[2], '%.2f G/s' % (d['value'] / 1e9), '%.1f ms' % d['ms_per_step'], 'tok %.1f' % d['stages_ms']['tokenize'], 'native %.2f' % (d['alt_rng']['value'] / 1e9), 'seg %.2f' % (d['with_segmentation']['value'] / 1e9))
PY
done
echo ALLDONE

# round 6 A/B: tokenizer variants (product vs lddl_amd/_lib_<variant>), GPU tokenizer tests + 2 GB timing + C2
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-r06tk}
V=${2:-tokold}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tokenize_gpu.py > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/r06_memovar.sh ${1:-r06tk} prod $V prod $V || exit 2
for v in base $V; do
  lib=lddl_amd/_lib/liblddl_amd.so; [ $v != base ] && lib=lddl_amd/_lib_$v/liblddl_amd.so
  LDDL_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench_$v.log 2>&1 || { echo BENCH_FAILED $v; tail -3 $O/bench_$v.log; exit 3; }
  python - $O/bench_$v.log $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('C2', sys.argv[2], '%.2f G/s' % (d['value'] / 1e9), '%.1f ms' % d['ms_per_step'], 'tok', d['stages_ms'].get('tokenize'))
PY
done
echo ALLDONE

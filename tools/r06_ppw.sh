# round 6 A/B: partitions per planner wave (LDDL_PLAN_PPW) x planner occupancy (LDDL_PLAN_OCC build), C2 planner time
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-r06u}
mkdir -p $O
LDDL_PLAN_PPW=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_output_gpu.py > $O/tests_ppw2.log 2>&1 || { echo TESTS_FAILED; tail -20 $O/tests_ppw2.log; exit 1; }
for v in "prod 1" "prod 2" "prod 3" "occ8 1" "occ8 2"; do
  set -- $v
  lib=lddl_amd/_lib/liblddl_amd.so; [ $1 = occ8 ] && lib=lddl_amd/_lib_occ8/liblddl_amd.so
  LDDL_AMD_LIB=$lib LDDL_PLAN_PPW=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench_$1_ppw$2.log 2>&1 || { echo BENCH_FAILED $v; tail -5 $O/bench_$1_ppw$2.log; exit 2; }
  python - $O/bench_$1_ppw$2.log "$v" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], 'value %.2f G/s' % (d['value'] / 1e9), 'ms %.1f' % d['ms_per_step'], 'plan', d['stages_ms'].get('per_step_plan'))
PY
done
LDDL_AMD_LIB=lddl_amd/_lib_diag/liblddl_amd.so LDDL_PLAN_PPW=2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 1 --warmup 0 --no-alt-rng --no-segmented-line --no-extra-lines > $O/stamps_ppw2.log 2>&1 || exit 3
grep -E "^\[(timeline|stamps)" $O/stamps_ppw2.log
for gb in 536870912 1073741824; do
  timeout -k 10 300 python -u tools/cli_e2e.py --bytes 1e9 --num-blocks 1024 --gpu-batch-bytes $gb > $O/e2e_1GB_b$gb.log 2>&1 || { echo E2E_FAILED; tail -5 $O/e2e_1GB_b$gb.log; exit 4; }
  echo "1GB batch $gb: $(grep -o '"cli_wall_s": [0-9.]*' $O/e2e_1GB_b$gb.log) $(grep 'stage seconds' $O/e2e_1GB_b$gb.log | tail -1)"
done
echo ALLDONE

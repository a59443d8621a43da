# round 6: the other configurations on the current build — C3, C4, C5, end-to-end CLI
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-r06q}
mkdir -p $O
[ -n "$SKIP_C3" ] || timeout -k 10 600 python -u bench.py --workload c3 --no-cpu-baseline > $O/bench_c3.log 2>&1 || { echo C3_FAILED; tail -5 $O/bench_c3.log; exit 2; }
timeout -k 10 900 python -u bench.py --workload c4 --no-cpu-baseline --no-alt-rng > $O/bench_c4.log 2>&1 || { echo C4_FAILED; tail -5 $O/bench_c4.log; exit 3; }
timeout -k 10 600 python -u bench.py --workload c5 > $O/bench_c5.log 2>&1 || { echo C5_FAILED; tail -5 $O/bench_c5.log; exit 4; }
timeout -k 10 300 python -u tools/cli_e2e.py --bytes 100e6 --num-blocks 128 > $O/e2e_100MB.log 2>&1 || { echo E2E_FAILED; tail -5 $O/e2e_100MB.log; exit 5; }
timeout -k 10 600 python -u tools/cli_e2e.py --bytes 1e9 --num-blocks 1024 > $O/e2e_1GB.log 2>&1 || { echo E2E_FAILED; tail -5 $O/e2e_1GB.log; exit 6; }
timeout -k 10 600 python -u tools/cli_e2e.py --bytes 1e9 --num-blocks 1024 --seq 512 --bin-size 8 --num-shards 8 > $O/e2e_1GB_c3.log 2>&1 || { echo E2E_FAILED; tail -5 $O/e2e_1GB_c3.log; exit 7; }
python - $O <<'PY'
import json, sys, os
O = sys.argv[1]
for n in ('bench_c3', 'bench_c4', 'bench_c5'):
    if not os.path.exists(os.path.join(O, n + '.log')): continue
    d = json.loads([l for l in open(os.path.join(O, n + '.log')) if l.startswith('{')][-1])
    print(n, d['value'], d['unit'], d['ms_per_step'], d.get('stages_ms'), (d.get('alt_rng') or {}).get('value'))
for n in ('e2e_100MB', 'e2e_1GB', 'e2e_1GB_c3'):
    print(n, open(os.path.join(O, n + '.log')).read()[-600:])
PY
echo ALLDONE

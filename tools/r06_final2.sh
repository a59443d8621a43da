# round 6 final build, part 2: smoke, the default bench line (C2 + CPU baseline), C3
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-r06z2}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench_c2.log 2>&1 || { echo BENCH_FAILED; tail -20 $O/bench_c2.log; exit 2; }
timeout -k 10 500 python -u bench.py --workload c3 --no-cpu-baseline > $O/bench_c3.log 2>&1 || { echo C3_FAILED; tail -20 $O/bench_c3.log; exit 3; }
[ -n "$WITH_C4" ] && { timeout -k 10 600 python -u bench.py --workload c4 --no-cpu-baseline --no-alt-rng > $O/bench_c4.log 2>&1 || { echo C4_FAILED; tail -20 $O/bench_c4.log; exit 4; }; }
python - $O <<'PY'
import json, sys, os
for n in [x for x in ('bench_c2', 'bench_c3', 'bench_c4') if os.path.exists(os.path.join(sys.argv[1], x + '.log'))]:
    d = json.loads([l for l in open(os.path.join(sys.argv[1], n + '.log')) if l.startswith('{')][-1])
    print(n, '%.2f G/s' % (d['value'] / 1e9), '%.1f ms' % d['ms_per_step'], d['stages_ms'], 'native', (d.get('alt_rng') or {}).get('value'), 'roofline', d['roofline'].get('frac'), d['roofline'].get('traffic'), 'path', d.get('roofline_path'), 'cpu', (d.get('cpu_baseline') or {}).get('value'), [x.get('same_build') for x in d.get('issue_roofline', [])])
PY
echo ALLDONE_FINAL2

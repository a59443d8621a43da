# kernel traces of one C2 and one C4 bench step (which kernels run, incl. any ATen ones) + the
# output / balance GPU tests; usage: bash tools/run_trace2.sh <tag>
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_output_gpu.py tests/test_balance.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c2 -o b -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines > $O/c2.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c4 -o b -- python3 bench.py --workload c4 --batch-bytes 4000000000 --sub-batch-bytes 2000000000 --steps 1 --warmup 1 --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines > $O/c4.log 2>&1 || exit 3
echo ALLDONE
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_tokenize_gpu.py > $O/tests_tok.log 2>&1 || exit 4
for r in 1 2; do timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench_$r.log 2>&1 || exit 5; echo "r$r $(grep -o '"stages_ms": {[^}]*}' $O/bench_$r.log)" >> $O/summary.txt; done
echo ALLDONE2

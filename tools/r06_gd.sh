# round 6 A/B: gather16 masks written straight to their rank slots (LDDL_GATHER_DIRECT build) vs staged rows
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-r06v}
mkdir -p $O
LDDL_AMD_LIB=lddl_amd/_lib_gd/liblddl_amd.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_output_gpu.py > $O/tests_gd.log 2>&1 || { echo TESTS_FAILED; tail -20 $O/tests_gd.log; exit 1; }
tail -1 $O/tests_gd.log
i=0
for v in prod gd prod gd; do
  i=$((i+1))
  lib=lddl_amd/_lib/liblddl_amd.so; [ $v = gd ] && lib=lddl_amd/_lib_gd/liblddl_amd.so
  LDDL_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${v}_$i -o run -- python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench_${v}_$i.log 2>&1 || { echo BENCH_FAILED $v; tail -5 $O/bench_${v}_$i.log; exit 2; }
  python tools/prof_summary.py $O/prof_${v}_$i $O/kernels_${v}_$i && echo "== $v $i" && grep -E "gather16|plan_replay|tokenize_batch" $O/kernels_${v}_$i.txt
done
echo ALLDONE

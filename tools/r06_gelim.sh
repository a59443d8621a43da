# round 6: gather16 LDS-conflict attribution (elimination builds ge1 / ge2 / ge8: no decision-table
# scatter / no staging writes / no staging read-back; ge4: staging writes of masked elements only,
# exec-masked - a real candidate) + the native line's kernels
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-r06w}
mkdir -p $O
LDDL_AMD_LIB=lddl_amd/_lib_ge4/liblddl_amd.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_output_gpu.py > $O/tests_ge4.log 2>&1 || { echo TESTS_FAILED; tail -20 $O/tests_ge4.log; exit 1; }
tail -1 $O/tests_ge4.log
for v in base ge1 ge2 ge4 ge8; do
  bash tools/pmc_pass.sh ${1:-r06w} $v gather16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU > /dev/null || { echo PMC_FAILED $v; exit 2; }
  echo "== $v"; cat $O/pmc_$v.txt
done
for v in base ge4 base ge4; do
  lib=lddl_amd/_lib/liblddl_amd.so; [ $v = ge4 ] && lib=lddl_amd/_lib_ge4/liblddl_amd.so
  rm -rf $O/prof_$v
  LDDL_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench_$v.log 2>&1 || { echo BENCH_FAILED $v; exit 3; }
  python tools/prof_summary.py $O/prof_$v $O/kernels_$v && echo "== time $v" && grep -E "gather16" $O/kernels_$v.txt
done
rm -rf $O/prof_native
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_native -o run -- python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --rng native --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench_native.log 2>&1 || { echo NATIVE_FAILED; exit 4; }
python tools/prof_summary.py $O/prof_native $O/kernels_native && head -20 $O/kernels_native.txt
echo ALLDONE

# round 6 diagnostics: gather16 with 16-byte aligned token stores (gst) / loads (gld) (wrong output, time only),
# densify with 8 chunks in flight (dn8, native line)
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-r06y}
mkdir -p $O
for v in base gst gld base; do
  lib=lddl_amd/_lib/liblddl_amd.so; [ $v != base ] && lib=lddl_amd/_lib_$v/liblddl_amd.so
  rm -rf $O/prof_$v
  LDDL_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench_$v.log 2>&1 || { echo BENCH_FAILED $v; exit 3; }
  python tools/prof_summary.py $O/prof_$v $O/kernels_$v && echo "== $v $(grep -E 'gather16' $O/kernels_$v.txt)"
done
for v in base dn8 base dn8; do
  lib=lddl_amd/_lib/liblddl_amd.so; [ $v != base ] && lib=lddl_amd/_lib_$v/liblddl_amd.so
  rm -rf $O/profn_$v
  LDDL_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/profn_$v -o run -- python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --rng native --no-alt-rng --no-segmented-line --no-extra-lines > $O/benchn_$v.log 2>&1 || { echo BENCH_FAILED $v; exit 4; }
  python tools/prof_summary.py $O/profn_$v $O/kernelsn_$v && echo "== native $v $(grep -E 'densify' $O/kernelsn_$v.txt)"
done
echo ALLDONE

# A/B of library variants on the C2 bench + a kernel trace of each:
#   bash tools/run_variants.sh <outdir> <variant>...   (base = lddl_amd/_lib)
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
for v in "$@"; do
  if [ "$v" = base ]; then L=lddl_amd/_lib/liblddl_amd.so; else L=lddl_amd/_lib_$v/liblddl_amd.so; fi
  LDDL_AMD_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-alt-rng --steps 3 > $O/c2_$v.log 2>&1 || exit 1
  LDDL_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr_$v -o b -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-alt-rng > $O/tr_$v.log 2>&1 || exit 2
done
echo ALLDONE

# Kernel traces of library variants on the default C2 bench (1 timed step):
#   bash tools/run_variants_short.sh <outdir> <variant>...   (base = lddl_amd/_lib)
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
for v in "$@"; do
  if [ "$v" = base ]; then L=lddl_amd/_lib/liblddl_amd.so; else L=lddl_amd/_lib_$v/liblddl_amd.so; fi
  LDDL_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr_$v -o b -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-alt-rng --no-segmented-line > $O/tr_$v.log 2>&1 || exit 1
done
echo ALLDONE

set -o pipefail
mkdir -p gpurun_out/r04t
export TMPDIR=/tmp
for v in base gns gnr gnb; do
  if [ "$v" = base ]; then L=lddl_amd/_lib/liblddl_amd.so; else L=lddl_amd/_lib_$v/liblddl_amd.so; fi
  LDDL_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04t/$v -o k -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-alt-rng --no-extra-lines --no-segmented-line > gpurun_out/r04t/$v.log 2>&1 || exit 1
  echo "$v done"
done

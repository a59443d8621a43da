set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r04gv
for v in gnm gns2; do
  LDDL_AMD_LIB=lddl_amd/_lib_$v/liblddl_amd.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04gv/$v -o k -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-alt-rng --no-extra-lines --no-segmented-line > gpurun_out/r04gv/$v.log 2>&1 || exit 1
  echo "$v done"
done

set -o pipefail
mkdir -p gpurun_out/r04u
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_output_gpu.py tests/test_native_gpu.py > gpurun_out/r04u/tests.log 2>&1 || exit 1
echo tests ok
for v in base gw8; do
  if [ "$v" = base ]; then L=lddl_amd/_lib/liblddl_amd.so; else L=lddl_amd/_lib_$v/liblddl_amd.so; fi
  LDDL_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04u/$v -o k -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-alt-rng --no-extra-lines --no-segmented-line > gpurun_out/r04u/$v.log 2>&1 || exit 1
  echo "$v done"
done

set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r04sched
for v in maxilp maxmemoryclause iterativeilp; do
  L=lddl_amd/_lib_$v/liblddl_amd.so
  LDDL_AMD_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_tokenize_gpu.py > gpurun_out/r04sched/tests_$v.log 2>&1 || exit 1
  LDDL_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04sched/$v -o k -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-alt-rng --no-extra-lines --no-segmented-line > gpurun_out/r04sched/$v.log 2>&1 || exit 2
  echo "$v done"
done

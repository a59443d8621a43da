# pair parity tests (default library) + a kernel trace of a short C2 bench per library variant
# usage: bash tools/run_pairs_var.sh <tag> [variants...]
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_output_gpu.py tests/test_native_gpu.py > $O/tests.log 2>&1 || exit 1
for v in base "$@"; do
  if [ "$v" = base ]; then L=lddl_amd/_lib/liblddl_amd.so; else L=lddl_amd/_lib_$v/liblddl_amd.so; fi
  LDDL_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$v -o bench -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench_$v.log 2>&1 || exit 2
done
echo ALLDONE

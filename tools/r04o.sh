set -o pipefail
mkdir -p gpurun_out/r04o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_output_gpu.py tests/test_tokenize_gpu.py > gpurun_out/r04o/tests.log 2>&1
echo "tests rc=$?"
bash tools/run_trace_copies.sh r04o/trace || exit 1
for v in base tp2; do
  if [ "$v" = base ]; then L=lddl_amd/_lib/liblddl_amd.so; else L=lddl_amd/_lib_$v/liblddl_amd.so; fi
  LDDL_AMD_LIB=$L timeout -k 10 300 python -u tools/tok_bench.py 2147483648 > gpurun_out/r04o/tok_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/r04o/tok_$v.log)"
done

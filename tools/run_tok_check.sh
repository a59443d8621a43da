# tokenizer parity tests + timing (2 GiB); usage: bash tools/run_tok_check.sh <tag> [variants...]
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_tokenize_gpu.py tests/test_pairs_gpu.py tests/test_segment_gpu.py > $O/tests.log 2>&1 || exit 1
for v in base "$@"; do
  if [ "$v" = base ]; then L=lddl_amd/_lib/liblddl_amd.so; else L=lddl_amd/_lib_$v/liblddl_amd.so; fi
  LDDL_AMD_LIB=$L timeout -k 10 200 python -u tools/tok_bench.py 2147483648 > $O/tok_$v.log 2>&1 || exit 2
done
echo ALLDONE

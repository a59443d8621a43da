cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests -k "txt_output or collate" > $O/gpu_tests.log 2>&1
for v in base nowp; do
  if [ "$v" = base ]; then L=lddl_amd/_lib/liblddl_amd.so; else L=lddl_amd/_lib_$v/liblddl_amd.so; fi
  LDDL_AMD_LIB=$L timeout -k 10 200 python -u tools/tok_bench.py 2147483648 > $O/tok_$v.log 2>&1 || exit 2
done
bash tools/run_c5.sh $1 || exit 3
timeout -k 10 900 python -u bench.py > $O/bench_c2.log 2>&1 || exit 4
echo ALLDONE

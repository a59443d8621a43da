# tokenizer library variants timed by tools/tok_bench.py (2 GiB); usage: bash tools/run_tokv.sh <tag> v1 v2 ...
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
for v in "$@"; do
  if [ "$v" = base ]; then L=lddl_amd/_lib/liblddl_amd.so; else L=lddl_amd/_lib_$v/liblddl_amd.so; fi
  LDDL_AMD_LIB=$L timeout -k 10 200 python -u tools/tok_bench.py 2147483648 > $O/tok_$v.log 2>&1 || exit 2
done
echo ALLDONE

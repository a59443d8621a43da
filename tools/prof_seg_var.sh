cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
for v in "$@"; do
  LDDL_AMD_LIB=lddl_amd/_lib_$v/liblddl_amd.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$v -o b -- python3 tools/seg_bench.py 2 > $O/trace_$v.log 2>&1 || exit 1
done
echo ALLDONE

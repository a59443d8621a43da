cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-segv}
mkdir -p $O
shift
timeout -k 10 200 python -u tools/seg_bench.py 2 > $O/seg_base.log 2>&1 || exit 1
for v in "$@"; do
  LDDL_AMD_LIB=lddl_amd/_lib_$v/liblddl_amd.so timeout -k 10 200 python -u tools/seg_bench.py 2 > $O/seg_$v.log 2>&1 || exit 2
done
echo ALLDONE

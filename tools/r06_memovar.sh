# round 6: word memo tuning variants (sample divisor, table size) on 2 GB
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-r06m}
mkdir -p $O
shift
for v in "$@"; do
  lib=lddl_amd/_lib_$v/liblddl_amd.so
  [ $v = prod ] && lib=lddl_amd/_lib/liblddl_amd.so
  LDDL_AMD_LIB=$lib timeout -k 10 300 python -u tools/tok_ab.py 2e9 fused fused > $O/ab_$v.log 2>&1 || { echo AB_FAILED $v; tail -5 $O/ab_$v.log; exit 3; }
  echo "== $v"; grep '^\[' $O/ab_$v.log
done
echo ALLDONE

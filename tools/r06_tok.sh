# round 6: tokenizer split form — parity tests, then fused vs split on 2 GB (+ tuning variants)
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-r06a}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_tokenize_gpu.py > $O/tok_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tok_tests.log; exit 2; }
grep -c PASSED $O/tok_tests.log
timeout -k 10 300 python -u tools/tok_ab.py 2e9 fused split fused split > $O/tok_ab.log 2>&1 || { echo AB_FAILED; tail -20 $O/tok_ab.log; exit 3; }
cat $O/tok_ab.log
for v in h512w6 h512w8 s5h8 s6h8; do
  LDDL_AMD_LIB=lddl_amd/_lib_$v/liblddl_amd.so timeout -k 10 200 python -u tools/tok_ab.py 2e9 split split > $O/tok_ab_$v.log 2>&1 || { echo AB_FAILED $v; tail -20 $O/tok_ab_$v.log; exit 4; }
  echo "== $v"; grep '\[' $O/tok_ab_$v.log
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/$O/prof -o tok -- python3 /root/repo/tools/tok_ab.py 2e9 fused split > /root/repo/$O/prof.log 2>&1 || { echo PROF_FAILED; tail -20 /root/repo/$O/prof.log; exit 5; }
cd /root/repo
python tools/prof_summary.py $O/prof $O/prof_kernels && head -20 $O/prof_kernels.txt
echo ALLDONE

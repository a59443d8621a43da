# round 6: tokenizer word memo — parity tests, then memo vs plain on 2 GB (+ kernel trace)
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-r06l}
mkdir -p $O
timeout -k 10 600 python -u -m pytest --maxfail=3 -q --timeout 200 --timeout-method thread tests/test_tokenize_gpu.py > $O/tok_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|assert|sentence" $O/tok_tests.log | head -20; tail -5 $O/tok_tests.log; exit 2; }
tail -1 $O/tok_tests.log
timeout -k 10 300 python -u tools/tok_ab.py 2e9 fused plain fused plain > $O/tok_ab.log 2>&1 || { echo AB_FAILED; tail -20 $O/tok_ab.log; exit 3; }
grep '^\[' $O/tok_ab.log
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/$O/tr -o k -- python3 /root/repo/tools/tok_ab.py 2e9 fused > /root/repo/$O/tr.log 2>&1 ) || { echo TRACE_FAILED; tail -5 $O/tr.log; exit 4; }
python tools/prof_summary.py $O/tr $O/memo_kernels && head -6 $O/memo_kernels.txt | cut -c1-120
echo ALLDONE

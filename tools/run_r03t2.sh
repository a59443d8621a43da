# tokenizer retune under the streaming design (units per pass, sentences per chunk) + C5 HIP trace
cd /root/repo
export TMPDIR=/tmp
AB_TESTS="tests/test_tokenize_gpu.py" AB_TEST_VARIANTS="sf128 ch64 ch256" bash tools/ab.sh r03t2 base sf128 ch64 ch256 || exit 1
bash tools/run_c5_hiptrace.sh r03h || exit 2
echo ALLDONE

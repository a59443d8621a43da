# Tokenizer change check: GPU tokenizer tests, 1 GiB throughput, SQ mix.
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-tokc}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_tokenize_gpu.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/tok_bench.py 1073741824 > $O/tok.log 2>&1 || exit 2
bash tools/prof_tok_variants.sh ${1:-tokc} base || exit 3
echo ALLDONE

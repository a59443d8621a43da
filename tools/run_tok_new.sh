# tokenizer check: GPU tokenizer tests, then tok_bench at 2 GiB; usage: bash tools/run_tok_new.sh <tag>
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_tokenize_gpu.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/tok_bench.py 2147483648 > $O/tok.log 2>&1 || exit 2
echo ALLDONE

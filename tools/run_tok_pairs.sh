# tokenizer + pair parity tests, tokenizer timing (2 GiB) and a short C2 bench with its kernel trace
# usage: bash tools/run_tok_pairs.sh <tag>
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_tokenize_gpu.py tests/test_pairs_gpu.py tests/test_segment_gpu.py tests/test_output_gpu.py tests/test_native_gpu.py tests/test_collate_gpu.py tests/test_balance.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/tok_bench.py 2147483648 > $O/tok.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o bench -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench.log 2>&1 || exit 3
echo ALLDONE

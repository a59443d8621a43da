# end-to-end CLI timing (tools/cli_e2e.py) at 100 MB (C1) and 1 GB; usage: bash tools/run_e2e.sh <tag>
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u tools/cli_e2e.py --bytes 100e6 --num-blocks 128 > $O/e2e_100MB.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/cli_e2e.py --bytes 1e9 --num-blocks 1024 > $O/e2e_1GB.log 2>&1 || exit 2
timeout -k 10 600 python -u tools/cli_e2e.py --bytes 1e9 --num-blocks 1024 --seq 512 --bin-size 8 --num-shards 8 > $O/e2e_1GB_c3.log 2>&1 || exit 3
echo ALLDONE

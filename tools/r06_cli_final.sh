# round 6 final build: the CLI end to end (tools/cli_e2e.py): 100 MB, 1 GB seq 128, 1 GB seq 512 sharded, 4 GB seq 128
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-r06h}
mkdir -p $O
timeout -k 10 300 python -u tools/cli_e2e.py --bytes 100e6 --num-blocks 128 > $O/e2e_100MB.log 2>&1 || { echo E2E_FAILED; tail -5 $O/e2e_100MB.log; exit 1; }
timeout -k 10 600 python -u tools/cli_e2e.py --bytes 1e9 --num-blocks 1024 > $O/e2e_1GB.log 2>&1 || { echo E2E_FAILED; tail -5 $O/e2e_1GB.log; exit 2; }
timeout -k 10 600 python -u tools/cli_e2e.py --bytes 1e9 --num-blocks 1024 --seq 512 --bin-size 8 --num-shards 8 > $O/e2e_1GB_c3.log 2>&1 || { echo E2E_FAILED; tail -5 $O/e2e_1GB_c3.log; exit 3; }
timeout -k 10 900 python -u tools/cli_e2e.py --bytes 4e9 --num-blocks 4096 > $O/e2e_4GB.log 2>&1 || { echo E2E_FAILED; tail -5 $O/e2e_4GB.log; exit 4; }
for n in e2e_100MB e2e_1GB e2e_1GB_c3 e2e_4GB; do echo "== $n"; grep -E "stage seconds" $O/$n.log | tail -1; grep -o '"cli_wall_s": [0-9.]*, "source_MB_per_s": [0-9.]*' $O/$n.log; done
echo ALLDONE

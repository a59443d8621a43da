bash tools/ab.sh r03p7 t5 base || exit 1
timeout -k 10 300 python -u bench.py --workload c5 --steps 200 --warmup 20 > gpurun_out/r03p7/c5r.log 2>&1 || exit 2
for gb in 268435456 536870912 1073741824; do timeout -k 10 300 python -u tools/cli_e2e.py --bytes 1e9 --num-blocks 1024 --gpu-batch-bytes $gb > gpurun_out/r03p7/e2e_$gb.log 2>&1 || exit 3; done
echo ALLDONE

set -o pipefail
mkdir -p gpurun_out/r04q
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pairs_gpu.py > gpurun_out/r04q/tests.log 2>&1 || exit 1
echo tests ok
bash tools/run_trace_copies.sh r04q/trace || exit 1
B="python3 bench.py --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines --steps 1 --warmup 0"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/r04q/pmc -o p -- $B > gpurun_out/r04q/pmc.log 2>&1 || exit 2
python3 tools/pmc_summary.py $(find gpurun_out/r04q/pmc -name "*.db" | head -1) > gpurun_out/r04q/pmc.txt
echo ALLDONE

set -o pipefail
mkdir -p gpurun_out/r04c
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r04c/tests.log 2>&1
echo "tests rc=$?"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04c/smoke.log 2>&1
echo "smoke rc=$?"
timeout -k 10 600 python -u bench.py > gpurun_out/r04c/bench_c2.log 2>&1 || exit 1
echo bench done
LDDL_BENCH_SHARE_DEVICE=1 timeout -k 10 600 python -u bench.py --workload c4 --gpus 2 --batch-bytes 2000000000 --steps 3 > gpurun_out/r04c/bench_c4_n2_share.log 2>&1
echo "c4 n2 rc=$?"

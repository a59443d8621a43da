set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r04f4
timeout -k 10 900 python -u bench.py > gpurun_out/r04f4/bench_c2.log 2>&1 || exit 1
echo ALLDONE

set -o pipefail
cd /root/repo
export TMPDIR=/tmp
bash tools/run_bench_n2.sh r04n2 || exit 1
echo ALLDONE

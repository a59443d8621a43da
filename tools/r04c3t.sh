set -o pipefail
cd /root/repo
export TMPDIR=/tmp
bash tools/run_trace_copies.sh r04c3t/trace --workload c3 || exit 1

# e2e CLI on 1 GB with the host pipeline timeline (LDDL_TRACE_PIPELINE) and process CPU time;
# usage: bash tools/run_e2e_trace.sh <tag> [cli_e2e args]
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
LDDL_TRACE_PIPELINE=1 timeout -k 10 600 python -u tools/cli_e2e.py --bytes 1e9 --num-blocks 1024 "$@" > $O/e2e_1GB.log 2> $O/e2e_1GB.err || exit 2
echo ALLDONE

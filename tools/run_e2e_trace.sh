# e2e CLI on 1 GB with the host pipeline timeline (LDDL_TRACE_PIPELINE); usage: bash tools/run_e2e_trace.sh <tag>
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
LDDL_TRACE_PIPELINE=1 timeout -k 10 600 python -u tools/cli_e2e.py --bytes 1e9 --num-blocks 1024 > $O/e2e_1GB.log 2> $O/e2e_1GB.err || exit 2
echo ALLDONE
LDDL_D2H_PAGEABLE=1 LDDL_TRACE_PIPELINE=1 timeout -k 10 600 python -u tools/cli_e2e.py --bytes 1e9 --num-blocks 1024 > $O/e2e_1GB_pageable.log 2> $O/e2e_1GB_pageable.err || exit 3
echo ALLDONE2

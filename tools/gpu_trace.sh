set -u
export TMPDIR=/tmp
timeout -k 10 180 python tools/settle_trace.py 1250000 1 > gpurun_out/trace_big.log 2>&1 || exit $?
timeout -k 10 180 python tools/settle_trace.py 156250 1 > gpurun_out/trace_small.log 2>&1 || exit $?

# round 6: the per-GPU share of an N = 8 run (one 1.25M-row shard, bench.py --rank-share 0/8): bench line at
# 4 and 1 in flight, and a kernel trace of the one-in-flight chain
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_run.sh 'bench:--rank-share+0/8+--steps+400+--no-cpu-baseline' || exit $?
cp gpurun_out/bench.json gpurun_out/bench_share.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/share_trace -o run -- \
    python3 bench.py --rank-share 0/8 --steps 200 --warmup 20 --inflight 1 --no-cpu-baseline > gpurun_out/share_trace.log 2>&1 || exit 1
echo share-done

# round 6, final tree: the headline at 200 steps (the driver times 20) and at the driver's own command
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh 'bench:--steps+200+--warmup+10' || exit $?
cp gpurun_out/bench.json gpurun_out/bench_200.json
bash tools/gpu_run.sh 'bench:--gpus+1+--steps+20+--warmup+5' || exit $?
cp gpurun_out/bench.json gpurun_out/bench_20.json

# round 6: adaptive pilot rows (≥ 64k sampled rows per shard) — the at-size configs first (the C4-shaped 6.5M
# b1024 test had every query's queues overflow), then the whole suite, the batched configs and C2's ablation traces
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh 'test:test_gpu_configs_at_size or test_gpu_wide' test \
  'cmd:600:cfg15_batched.jsonl:python -u tools/bench_configs.py --only C2,C3,C4 --c2-batches 256 --c3-batches 256 --c4-batches 1024 --steps 6' || exit $?
export TMPDIR=/tmp
for ab in 0 4 1; do
  ABLATE=$ab timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c2_abl$ab -o run -- \
      python3 tools/wide_ablate.py C2 256 > gpurun_out/c2_abl$ab.log 2>&1 || { echo "c2 ablate $ab trace failed"; exit 1; }
done
echo traces-done

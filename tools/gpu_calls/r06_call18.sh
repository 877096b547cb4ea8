# round 6: the rows kernel's queues with a shared pool per owner (no drops when one producer's sub-queue fills),
# quarters back to ≤ 16,384 rows, per-view quarter descriptor table — wide / NaN / at-size tests and the full-size C4 tests (fallback-free asserts),
# the batched configs, C4's clocks and counters
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh 'test:test_gpu_wide or test_gpu_nan or test_gpu_configs_at_size or test_c4_full' \
  'cmd:600:cfg18_batched.jsonl:python -u tools/bench_configs.py --only C2,C4 --c2-batches 256 --c4-batches 1024 --steps 6' \
  'cmd:300:clk18_c4.log:ABLATE=0 python -u tools/wide_ablate.py C4 256' \
  'cmd:300:clk18_c2.log:ABLATE=0 python -u tools/wide_ablate.py C2 256' || exit $?

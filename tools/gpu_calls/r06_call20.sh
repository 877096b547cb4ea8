# round 6: dynamic group claims in sq8_wide_rows — the wide / NaN / at-size tests, C2 / C4 with claims on and off,
# the rows kernel's clocks
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh 'test:test_gpu_wide or test_gpu_nan or test_gpu_configs_at_size' \
  'cmd:600:cfg20_claim1.jsonl:python -u tools/bench_configs.py --only C2,C4 --c2-batches 256 --c4-batches 1024 --steps 6' \
  'cmd:600:cfg20_claim0.jsonl:python -u tools/bench_configs.py --only C2,C4 --c2-batches 256 --c4-batches 1024 --steps 6 --tune sq8_wide_rows_claim=0' \
  'cmd:600:cfg20_claim1b.jsonl:python -u tools/bench_configs.py --only C2,C4 --c2-batches 256 --c4-batches 1024 --steps 6' \
  'cmd:300:clk20_c4.log:ABLATE=0,1 python -u tools/wide_ablate.py C4 256' \
  'cmd:300:clk20_c2.log:ABLATE=0 python -u tools/wide_ablate.py C2 256' || exit $?

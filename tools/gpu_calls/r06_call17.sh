# round 6: the pilot on the rows kernel (≤ 128 dims), rows-kernel quarters up to 32,768 rows — the wide / NaN /
# at-size tests, the batched configs, the rows kernel's clocks (setup split), C4 / C2 launch traces
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh 'test:test_gpu_wide or test_gpu_nan or test_gpu_configs_at_size or test_gpu_prefilter' \
  'cmd:600:cfg17_batched.jsonl:python -u tools/bench_configs.py --only C2,C4 --c2-batches 256 --c4-batches 1024 --steps 6' \
  'cmd:300:clk17_c2.log:ABLATE=0,1 python -u tools/wide_ablate.py C2 256' \
  'cmd:300:clk17_c4.log:ABLATE=0 python -u tools/wide_ablate.py C4 256' \
  'cmd:400:prof17_c2.log:bash tools/prof_wide.sh r06b_c2 "--only C2 --c2-batches 256 --steps 5"' \
  'cmd:700:prof17_c4.log:bash tools/prof_wide.sh r06b_c4 "--only C4 --c4-batches 1024 --steps 3"' || exit $?

# round 6: sq8_wide_rows EUCLIDEAN per-row fast test; the single-query scan at 8 row groups per wave —
# wide/NaN/deep-scan tests, C2 ablations, C2 phase / rows variants, small views b1 deep on/off, C4
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh 'test:test_gpu_wide or test_gpu_nan or valudeep' \
  'cmd:400:ablate_c2_rows.log:ABLATE=0,4,1 python -u tools/wide_ablate.py C2 256' \
  'cmd:300:cfg_c2_def.jsonl:python -u tools/bench_configs.py --only C2 --c2-batches 256 --steps 10' \
  'cmd:300:cfg_c2_ph1.jsonl:python -u tools/bench_configs.py --only C2 --c2-batches 256 --steps 10 --tune sq8_wide_phase=1' \
  'cmd:300:cfg_c2_ring.jsonl:python -u tools/bench_configs.py --only C2 --c2-batches 256 --steps 10 --tune sq8_wide_rows=0' \
  'cmd:300:cfg_small_d0.jsonl:python -u tools/bench_configs.py --only C1,C2 --c2-batches 1 --steps 50' \
  'cmd:300:cfg_small_d1.jsonl:python -u tools/bench_configs.py --only C1,C2 --c2-batches 1 --steps 50 --tune sq8_scan_deep=1' \
  'cmd:600:cfg_c4.jsonl:python -u tools/bench_configs.py --only C4 --c4-batches 1024 --steps 6'

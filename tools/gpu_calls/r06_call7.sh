# round 6: sq8_wide_rows with one vote per group — wide tests, C4/C2 ablations, C2/C4 configs
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh 'test:test_gpu_wide or test_gpu_nan' \
  'cmd:400:ablate_c4_rows.log:ABLATE=0,1 python -u tools/wide_ablate.py C4 256' \
  'cmd:400:ablate_c2_rows.log:ABLATE=0,1 python -u tools/wide_ablate.py C2 256' \
  'cmd:600:cfg_rows1.jsonl:python -u tools/bench_configs.py --only C2,C4 --c4-batches 1024 --c2-batches 256 --steps 8'
bash tools/gpu_run.sh 'cmd:300:prof_c2.log:timeout -k 10 250 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06b_c2/trace -o run -- python3 tools/bench_configs.py --only C2 --c2-batches 256 --steps 5'

# round 6: sq8_mfma insertions bounded one pair per lane (instances not capped at 128 VGPRs: C3 b32) — prefilter /
# NaN / at-size tests, C3 / C4 b32 configs, their ablations and C3's SQ passes
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh 'test:test_gpu_prefilter or test_gpu_nan or test_gpu_configs_at_size or test_gpu_batched' \
  'cmd:400:cfg24_b32.jsonl:python -u tools/bench_configs.py --only C3,C4 --c3-batches 32 --c4-batches 32 --steps 6' \
  'cmd:400:abl24_c3.log:ABLATE=0,1,3 python -u tools/mfma_ablate.py C3 32' \
  'cmd:400:abl24_c4.log:ABLATE=0,1,3 python -u tools/mfma_ablate.py C4 32' \
  'cmd:600:pmc24_c3.log:bash tools/pmc_mfma_sq.sh C3' \
  'cmd:120:pmc24_sum.log:KINDS=pilot,main python3 tools/pmc_sq_summary.py gpurun_out/pmc_mfma_C3.json gpurun_out/pmc_mfma_C3_1 gpurun_out/pmc_mfma_C3_2 C3b32_laneins' || exit $?

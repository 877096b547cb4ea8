# round 6, final tree: the whole GPU suite, smoke, the N = 2/4/8 rehearsal (gloo ranks on the one GPU, results
# identical to N = 1), then C2 b256 variants (single main pass, 256 pilot rows)
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh test smoke rehearse \
  'cmd:300:cfg21_c2.jsonl:python -u tools/bench_configs.py --only C2 --c2-batches 256 --steps 10 && python -u tools/bench_configs.py --only C2 --c2-batches 256 --steps 10 --tune sq8_wide_phase=1 && python -u tools/bench_configs.py --only C2 --c2-batches 256 --steps 10 --tune sq8_wide_pilot_rows=256' || exit $?

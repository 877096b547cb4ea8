# round 6: the pilot bounds one row per lane (its best approximate score) — the whole GPU suite, then the batched
# configs (C2 b256, C3 b256, C4 b1024)
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh test \
  'cmd:600:cfg13_batched.jsonl:python -u tools/bench_configs.py --only C2,C3,C4 --c2-batches 256 --c3-batches 256 --c4-batches 1024 --steps 6' || exit $?
# C2's passes under the ablations, launch by launch (testing build): 0 full, 4 no slow path, 1 streaming only
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
for ab in 0 4 1; do
  ABLATE=$ab timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c2_abl$ab -o run -- \
      python3 tools/wide_ablate.py C2 256 > gpurun_out/c2_abl$ab.log 2>&1 || { echo "c2 ablate $ab trace failed"; exit 1; }
done
echo traces-done

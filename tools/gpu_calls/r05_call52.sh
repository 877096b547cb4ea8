# the wide quarter size on the final tree (C4 b1024, C3 b256): 8,192 / 16,384 (auto cap) / 32,768 rows
set -u
cd $GRAFT_REPO_ROOT
steps=()
for t in "sq8_wide_quarter_rows=0" "sq8_wide_quarter_rows=8192" "sq8_wide_quarter_rows=32768" "sq8_wide_quarter_rows=0"; do
  n=${t//=/_}
  steps+=("cmd:300:tune52_$n.jsonl:python -u tools/bench_configs.py --only C4,C3 --c4-batches 1024 --c3-batches 256 --steps 20 --tune $t")
done
bash tools/gpu_run.sh "${steps[@]}"

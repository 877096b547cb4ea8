# re-tune of the wide kernel's two-pass split and pilot on the final tree (C4 b1024 / b256; C3 b256):
# sq8_wide_phase 4 / 8 (default) / 12 / 16, pilot rows 128 (default) / 256; interleaved, two runs of the default
set -u
cd $GRAFT_REPO_ROOT
steps=()
for t in "sq8_wide_phase=8" "sq8_wide_phase=4" "sq8_wide_phase=12" "sq8_wide_phase=16" "sq8_wide_pilot_rows=256" "sq8_wide_phase=8"; do
  n=${t//=/_}
  steps+=("cmd:300:tune50_$n.jsonl:python -u tools/bench_configs.py --only C4,C3 --c4-batches 256,1024 --c3-batches 256 --steps 20 --tune $t")
done
bash tools/gpu_run.sh "${steps[@]}"

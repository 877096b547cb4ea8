# sq8_wide: the one-statement DMA issue at 6 units per wave (KS = 12: 4 + 2): wide + prefilter + sizes parity,
# (parity: passed in the first run of this script, 698 tests) then C3 b256 / C4 A/B against the previous build (abl/libosknn_base.so), interleaved, two runs each
set -u
cd $GRAFT_REPO_ROOT
steps=()
for rep in 1 2; do
  for L in abl/libosknn_base.so opensearch_amd/libosknn.so; do
    n=$(basename $(dirname $L))_$rep
    steps+=("cmd:300:ab41_$n.jsonl:OSKNN_LIB=\$PWD/$L python -u tools/bench_configs.py --only C3,C4 --c4-batches 1024 --c3-batches 256 --steps 20")
  done
done
bash tools/gpu_run.sh "${steps[@]}"

# sq8_wide: the floors pointer from LDS in the step loop; parity (wide, prefilter, sizes),
# then C4 / C3 / C2 A/B against the previous build (abl/libosknn_base.so), interleaved, two runs each
set -u
cd $GRAFT_REPO_ROOT
steps=("test:wide or prefilter or configs_at_size")
for rep in 1 2; do
  for L in abl/libosknn_base.so opensearch_amd/libosknn.so; do
    n=$(basename $(dirname $L))_$rep
    steps+=("cmd:300:ab56_$n.jsonl:OSKNN_LIB=\$PWD/$L python -u tools/bench_configs.py --only C4,C3,C2 --c4-batches 256,1024 --c3-batches 256 --c2-batches 256 --steps 20")
  done
done
bash tools/gpu_run.sh "${steps[@]}"

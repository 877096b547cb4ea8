# sq8_wide: 256-row steps with a 2-slot ring at KS = 2 (half the barriers per row), runtime event loop: wide + prefilter parity,
# then C4 b1024 / C2 b256 A/B against the previous build (abl/libosknn_base.so), interleaved, two runs each
set -u
cd $GRAFT_REPO_ROOT
steps=("test:wide or prefilter")
for rep in 1 2; do
  for L in abl/libosknn_base.so opensearch_amd/libosknn.so; do
    n=$(basename $(dirname $L))_$rep
    steps+=("cmd:300:ab37_$n.jsonl:OSKNN_LIB=\$PWD/$L python -u tools/bench_configs.py --only C4,C2 --c4-batches 256,1024 --c2-batches 128,256 --steps 20")
  done
done
bash tools/gpu_run.sh "${steps[@]}"

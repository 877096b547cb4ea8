# SGPR-held quarter descriptors in sq8_wide: wide parity tests, then C4 b1024 / C3 b256 A/B against the
# previous build (abl/libosknn_base.so), interleaved, two runs each
set -u
cd $GRAFT_REPO_ROOT
steps=("test:wide")
for rep in 1 2; do
  for L in abl/libosknn_base.so opensearch_amd/libosknn.so; do
    n=$(basename $(dirname $L))_$rep
    steps+=("cmd:300:ab29_$n.jsonl:OSKNN_LIB=\$PWD/$L python -u tools/bench_configs.py --only C4,C3 --c4-batches 1024 --c3-batches 256 --steps 20")
  done
done
bash tools/gpu_run.sh "${steps[@]}"

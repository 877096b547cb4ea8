# the wide pilot's 256-row default at >= 512 dims: wide / prefilter / sizes parity, C3 b256 and C4 against HEAD
set -u
cd $GRAFT_REPO_ROOT
steps=("test:wide or prefilter or configs_at_size")
for rep in 1 2; do
  for L in abl/libosknn_base.so opensearch_amd/libosknn.so; do
    n=$(basename $(dirname $L))_$rep
    steps+=("cmd:300:ab51_$n.jsonl:OSKNN_LIB=\$PWD/$L python -u tools/bench_configs.py --only C3,C4 --c4-batches 1024 --c3-batches 256 --steps 20")
  done
done
bash tools/gpu_run.sh "${steps[@]}"

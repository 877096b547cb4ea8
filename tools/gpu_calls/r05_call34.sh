# experiment: the wide kernel's ring depth at KS = 2 (NS 4 -> 3), C4 A/B (is the ring in series with the step?)
set -u
cd $GRAFT_REPO_ROOT
steps=()
for rep in 1 2; do
  for L in abl/libosknn_base.so opensearch_amd/libosknn.so; do
    n=$(basename $(dirname $L))_$rep
    steps+=("cmd:300:ab34_$n.jsonl:OSKNN_LIB=\$PWD/$L python -u tools/bench_configs.py --only C4 --c4-batches 256,1024 --steps 20")
  done
done
bash tools/gpu_run.sh "${steps[@]}"

# which of call 42's two changes cost time: packed fast-test fma (abl/libosknn_pk.so) or the two-way vm_wait
# (abl/libosknn_vw.so) against HEAD (abl/libosknn_base.so); C4 b1024 / b256, interleaved, two runs each
set -u
cd $GRAFT_REPO_ROOT
steps=()
for rep in 1 2; do
  for L in abl/libosknn_base.so abl/libosknn_pk.so abl/libosknn_vw.so; do
    n=$(basename $L .so)_$rep
    steps+=("cmd:300:ab43_$n.jsonl:OSKNN_LIB=\$PWD/$L python -u tools/bench_configs.py --only C4 --c4-batches 256,1024 --steps 20")
  done
done
bash tools/gpu_run.sh "${steps[@]}"

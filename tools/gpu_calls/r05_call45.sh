# experiment: sq8_wide with 4 waves of 64 queries (one per SIMD; the in-tree libraries are built with
# OSK_WIDE_WAVES=4 here): the wide parity tests on it, then C4 A/B: HEAD (abl/libosknn_base.so), this tree at
# 8 waves (abl/libosknn_w8.so) and at 4 waves (abl/libosknn_w4.so), interleaved, two runs each
set -u
cd $GRAFT_REPO_ROOT
steps=("test:wide")
for rep in 1 2; do
  for L in abl/libosknn_base.so abl/libosknn_w8.so abl/libosknn_w4.so; do
    n=$(basename $L .so)_$rep
    steps+=("cmd:300:ab45_$n.jsonl:OSKNN_LIB=\$PWD/$L python -u tools/bench_configs.py --only C4 --c4-batches 256,1024 --steps 20")
  done
done
bash tools/gpu_run.sh "${steps[@]}"

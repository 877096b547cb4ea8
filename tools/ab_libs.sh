#!/usr/bin/env bash
# A/B two builds of libosknn in one GPU call (OSKNN_LIB): batched prefilter configs.
#   bash tools/ab_libs.sh LIB_A LIB_B   (default: ab/libosknn_head.so vs opensearch_amd/libosknn.so)
set -e
A=${1:-ab/libosknn_head.so}; B=${2:-opensearch_amd/libosknn.so}
mkdir -p gpurun_out
for L in $A $B; do
  n=$(basename $L .so)
  OSKNN_LIB=$PWD/$L timeout -k 10 200 python -u tools/bench_configs.py --only C4 --c4-batches 32 > gpurun_out/ab_c4_$n.jsonl 2>gpurun_out/ab_c4_$n.err
  for b in ${AB_BATCHES:-8 32}; do
    OSKNN_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --batch $b --inflight 1 --no-cpu-baseline --steps 40 > gpurun_out/ab_c3b${b}_$n.log 2>&1
  done
done

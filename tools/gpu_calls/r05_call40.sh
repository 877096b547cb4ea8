# LDS-DMA immediate-offset semantics first (a one-workgroup probe, in-bounds either way); only if the offset
# moves the LDS destination (what glds16_run now assumes) the wide parity tests and the A/B follow
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 ./tools/glds_offset_probe > gpurun_out/glds_offset_probe.txt 2>&1 || { cat gpurun_out/glds_offset_probe.txt; exit 1; }
cat gpurun_out/glds_offset_probe.txt
grep -q "offset applies to the LDS address too" gpurun_out/glds_offset_probe.txt || { echo "probe: not the assumed semantics, stopping"; exit 3; }
steps=("test:wide or prefilter or configs_at_size")
for rep in 1 2; do
  for L in abl/libosknn_base.so opensearch_amd/libosknn.so; do
    n=$(basename $(dirname $L))_$rep
    steps+=("cmd:300:ab40_$n.jsonl:OSKNN_LIB=\$PWD/$L python -u tools/bench_configs.py --only C4,C2,C3 --c4-batches 256,1024 --c2-batches 128,256 --c3-batches 256 --steps 20")
  done
done
bash tools/gpu_run.sh "${steps[@]}"

# rocprof evidence of the wide kernel on the final tree: C4 b1024 kernel trace + stats, FETCH / WRITE passes
set -u
cd $GRAFT_REPO_ROOT
bash tools/prof_wide.sh r05q_c4 "--only C4 --c4-batches 1024 --steps 3" && python3 tools/wide_launch_sets.py gpurun_out/r05q_c4 gpurun_out/r05q_c4/wide_launch_sets.json "C4 b1024 sq8_wide (round 5 final tree)" "per 256 queries: 100M rows x (128 B tiled int8 + 18 B staged terms) = 14.6 GB for a full pass"

# the final wide kernel's instruction mix (C4 b256; two SQ passes)
set -u
cd $GRAFT_REPO_ROOT
bash tools/pmc_wide_sq.sh C4 256 && python3 tools/pmc_sq_summary.py gpurun_out/pmc_sq_C4_256.json gpurun_out/pmc_sq_C4_256_1 gpurun_out/pmc_sq_C4_256_2 "C4 b256 sq8_wide (round 5 final tree)" > gpurun_out/pmc_sq_C4_256.txt && echo ok

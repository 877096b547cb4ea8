# round 6: sq8_mfma at b32 — ablations (0 full, 1 no epilogue: quick test + insertions, 3 loads only)
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh 'cmd:400:abl23_c4.log:ABLATE=0,1,3 python -u tools/mfma_ablate.py C4 32' \
  'cmd:400:abl23_c3.log:ABLATE=0,1,3 python -u tools/mfma_ablate.py C3 32' || exit $?

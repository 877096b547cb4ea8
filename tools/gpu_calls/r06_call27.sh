# round 6: where the ring kernel spends C3 b256 (768 dims) — ablations: 0 full, 32 quick tests without the
# insertions, 64 the ring alone, 8 no step barrier (results wrong)
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh 'cmd:600:abl27_c3.log:ABLATE=0,32,64,8 python -u tools/wide_ablate.py C3 256' || exit $?

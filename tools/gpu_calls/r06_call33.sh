# round 6: the rows kernel's queue pool and group claims under the rows-vs-ring parity test (qcap 0/1/8/64/128,
# claims on/off), then the whole wide / NaN files
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh 'test:test_gpu_wide or test_gpu_nan' || exit $?

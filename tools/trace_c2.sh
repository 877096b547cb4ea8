#!/usr/bin/env bash
# Kernel trace of C2 b256 on the wide prefilter (forced), one- and two-pass floors: gpurun_out/c2w{0,8}/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for ph in 0 8; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c2w$ph -o run -- \
      python3 tools/bench_configs.py --only C2 --c2-batches 256 --steps 5 --tune sq8_wide_force=1 \
      --tune sq8_wide_phase=$ph > gpurun_out/c2w$ph.log 2>&1 || exit $?
done
echo done

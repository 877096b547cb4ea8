cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
for ab in 3 0; do
  ABLATE=$ab timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT --kernel-include-regex sq8_wide -d gpurun_out/pmcw$ab -o pmc --output-format csv -- python3 tools/wide_ablate.py C4 256 > gpurun_out/pmcw$ab.log 2>&1 || exit $?
done

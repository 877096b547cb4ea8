set -u
# rehearsal of the N > 1 bench flow on the box's one GPU: ranks share the card, gloo replaces RCCL
# (numbers meaningless; checks the sharding, the exchange, the merge and the JSON line), and the
# merged results of 8 batches at N = 2, 4, 8 equal the 1-GPU results bit for bit
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --dump $OUT/res_1.npz > $OUT/rehearse_1.log 2>&1 || { echo rc=$?; tail -30 $OUT/rehearse_1.log; exit 1; }
for n in 2 4 8; do
  echo "== N=$n" | tee -a $OUT/steps.log
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2951$n \
      bench.py --gpus $n --exchange torch --dist-backend gloo --steps 20 --warmup 2 --no-cpu-baseline --dump $OUT/res_$n.npz > $OUT/rehearse_$n.log 2>&1 || { echo rc=$?; tail -30 $OUT/rehearse_$n.log; exit 1; }
  tail -1 $OUT/rehearse_$n.log | cut -c1-200
done
python - <<'PY'
import numpy as np
a = np.load("gpurun_out/res_1.npz")
for n in (2, 4, 8):
    b = np.load(f"gpurun_out/res_{n}.npz")
    same = all(np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8)) for k in a.files)
    print(f"N={n}: merged results of 8 batches identical to N=1: {same}")
    assert same
PY

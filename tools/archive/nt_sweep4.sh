# Config 4 (auto-reset) and the training loop with nontemporal state loads forced on / off.
set -u
mkdir -p gpurun_out/nt4
for rep in 1 2; do
  for v in 0 1; do
    SHIPENV_NT_LOADS=$v timeout -k 10 200 python3 tools/size_sweep.py --log2n 20 --log2n4 20,21,22,23,24 --out gpurun_out/nt4/c4_nt${v}_$rep.json > gpurun_out/nt4/c4_nt${v}_$rep.log 2>&1 || exit $?
    SHIPENV_NT_LOADS=$v timeout -k 10 200 python3 tools/time_train.py --iters 40 > gpurun_out/nt4/train_nt${v}_$rep.log 2>&1 || exit $?
  done
done

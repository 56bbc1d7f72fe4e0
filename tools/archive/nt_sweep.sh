# Nontemporal state loads forced on and off (SHIPENV_NT_LOADS) against N, at the shipped grid cap.
set -u
mkdir -p gpurun_out/nt
for rep in 1 2; do
  for v in 0 1; do
    SHIPENV_NT_LOADS=$v timeout -k 10 200 python3 tools/size_sweep.py --log2n ${LOG2N:-20,22,23,24,25} --log2n4 ${LOG2N4:-20,24} --out gpurun_out/nt/nt${v}_$rep.json > gpurun_out/nt/nt${v}_$rep.log 2>&1 || exit $?
  done
done

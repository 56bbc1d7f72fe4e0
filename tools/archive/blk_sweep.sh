# Step-kernel workgroup cap (SHIPENV_STEP_BLOCKS) against N: one size sweep per cap.
#   BLOCKS="2048 16384" bash tools/blk_sweep.sh
set -u
mkdir -p gpurun_out/blk
for b in ${BLOCKS:-2048 4096 8192 16384 1024}; do
  SHIPENV_STEP_BLOCKS=$b timeout -k 10 200 python3 tools/size_sweep.py --log2n ${LOG2N:-22,23,24,25} --log2n4 ${LOG2N4:-24} --out gpurun_out/blk/b$b.json > gpurun_out/blk/b$b.log 2>&1 || exit $?
done

# A/B of the training loop's parts over every build under shippingenv_amd/_lib/abl
# (tools/time_train.py, one process per library, alternating, two rounds).
set -u
for rep in 1 2; do for lib in shippingenv_amd/_lib/abl/*.so; do
  timeout -k 10 120 python3 tools/time_train.py --lib $lib --iters 30 2>/dev/null | tail -1 || exit $?
done; done

# step-time regimes of one library build (stepbench): warm-up length x timed length
set -u
L=${1:-shippingenv_amd/_lib/libshipenv_hip.so}
C=${2:-3}
for r in "5 20" "5 20" "50 20" "50 20" "500 20" "500 20" "5 1000" "50 1000" "1000 1000"; do
  set -- $r
  timeout -k 10 60 tools/stepbench --config $C --warm $1 --steps $2 $L || exit $?
done

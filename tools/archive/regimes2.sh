# Where the driver's short run (5 warm-up + 20 timed steps) loses time against the
# steady state: warm-up length, timed length, and timed rows generated right before
# timing (stepbench --gen-late), one library build.
set -u
L=${1:-shippingenv_amd/_lib/libshipenv_hip.so}
C=${2:-3}
for rep in 1 2; do
for r in "5 20" "5 20 --gen-late" "50 20" "50 20 --gen-late" "500 20" "5 200" "5 200 --gen-late" "50 1000" "50 1000 --gen-late"; do
  set -- $r
  timeout -k 10 60 tools/stepbench --config $C --warm $1 --steps $2 ${3:-} $L || exit $?
done
done

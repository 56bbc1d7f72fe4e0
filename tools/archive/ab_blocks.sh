set -u
for rep in 1 2; do
for b in 2048 512 256; do
  for lib in shippingenv_amd/_lib/abl/*.so; do
    for r in "3 50 1000" "3 5 20"; do
      set -- $r
      echo -n "blocks=$b "
      SHIPENV_STEP_BLOCKS=$b timeout -k 10 60 tools/stepbench --config $1 --warm $2 --steps $3 $lib || exit $?
    done
  done
done
done

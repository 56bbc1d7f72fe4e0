# A/B step timing of every build under shippingenv_amd/_lib/abl (tools/stepbench, one
# process per library and regime, alternating libraries, two rounds). REGIMES holds
# "config:warm-up:steps" words; the default covers the driver's short run (5 warm-up +
# 20 timed steps), the steady state and config 4.
set -u
for rep in 1 2; do
  for lib in shippingenv_amd/_lib/abl/*.so; do
    for r in ${REGIMES:-3:5:20 3:50:1000 4:50:1000}; do
      IFS=: read -r c w s <<< "$r"
      timeout -k 10 60 tools/stepbench --config $c --warm $w --steps $s $lib || exit $?
    done
  done
done

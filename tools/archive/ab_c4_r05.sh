#!/bin/bash
# round 5: config 4 (64 ports, auto-reset) (and with WITH_C3=1 config 3) in steady state at
# N = 2^24 and 2^20, every library under shippingenv_amd/_lib/abl (tools/stepbench, 1000-step
# pre-roll), ROUNDS rounds alternating builds; EXTRA_ENV="VAR=v" adds runs with that setting.
# One JSON line per run on stdout (the setting in "env").
set -u
run() {  # lib envspec args...
  local lib=$1 e=$2
  shift 2
  env $e timeout -k 10 90 tools/stepbench "$@" $lib | sed "s/^{/{\"env\": \"$e\", /" || return 1
}
for rep in $(seq 1 ${ROUNDS:-3}); do
  for lib in shippingenv_amd/_lib/abl/*.so; do
    for e in NONE=0 ${EXTRA_ENV:-}; do
      run $lib $e --config 4 --n 16777216 --preroll 1000 --warm 5 --steps 100 || exit 1
      run $lib $e --config 4 --preroll 1000 --warm 5 --steps 200 || exit 1
      if [ -n "${WITH_C3:-}" ]; then run $lib $e --config 3 --preroll 1000 --warm 5 --steps 200 || exit 1; fi
    done
  done
done
exit 0

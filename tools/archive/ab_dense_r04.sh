#!/bin/bash
# round 4: config 4 (steady state, tools/stepbench) with the done list's dense layout (dense,
# padding to the line beyond 2^23 envs; SHIPENV_DONE_PAD=0/1 forces it off/on) against the
# per-segment layout (head) and the timing-only build without record stores (norecs);
# N = 2^24 and 2^20, five rounds alternating
set -u
L=shippingenv_amd/_lib/abl
for rep in 1 2 3 4 5; do
  for v in head dense dense0 dense1 norecs; do
    lib=$L/${v%[01]}.so
    case $v in dense0) export SHIPENV_DONE_PAD=0;; dense1) export SHIPENV_DONE_PAD=1;; *) unset SHIPENV_DONE_PAD;; esac
    timeout -k 10 90 tools/stepbench --config 4 --n 16777216 --preroll 1000 --warm 5 --steps 100 $lib | sed "s/\"lib\": \"[^\"]*\"/\"lib\": \"$v\"/" || exit $?
    timeout -k 10 60 tools/stepbench --config 4 --preroll 1000 --warm 5 --steps 200 $lib | sed "s/\"lib\": \"[^\"]*\"/\"lib\": \"$v\"/" || exit $?
  done
done

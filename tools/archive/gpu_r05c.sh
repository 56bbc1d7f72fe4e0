set -u
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "mask or observe" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for P in 5 64; do for tiled in 0 1 0 1; do SHIPENV_MASK_TILED=$tiled timeout -k 10 120 python tools/time_obs.py --ports $P --reps 50 | sed "s/^{/{\"tiled\": $tiled, /" >> $O/time_obs.jsonl || exit 1; done; done
ROUNDS=2 EXTRA_ENV=SHIPENV_NT_LOADS=1 tools/ab_c4_r05.sh > $O/ab_c4.jsonl 2> $O/ab.err || exit 1
echo done

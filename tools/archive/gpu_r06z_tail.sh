# round 6: the tail of gpu_final.sh r06z after stepbench (rebuilt for gfx950) crashed there
set -u
OUT=gpurun_out/r06z; mkdir -p $OUT
timeout -k 10 200 tools/stepbench --config 4 --steps 200 --preroll 1000 --floor 5 shippingenv_amd/_lib/libshipenv_hip.so > $OUT/c4_floor.txt 2>&1 || exit $?
timeout -k 10 200 tools/stepbench --config 3 --steps 200 --preroll 1000 --floor 5 shippingenv_amd/_lib/libshipenv_hip.so > $OUT/c3_floor.txt 2>&1 || exit $?
timeout -k 10 120 python3 tools/time_server.py > $OUT/time_server.jsonl 2>&1 || exit $?
cat $OUT/c4_floor.txt $OUT/c3_floor.txt $OUT/time_server.jsonl

set -u
for lib in tq0 tp1 tq0 tp1; do
timeout -k 10 120 python3 tools/time_policy.py --precision f32 --launches 5 --preroll 300 --trace --lib shippingenv_amd/_lib/abl/$lib.so || exit 1
done
timeout -k 10 120 python3 tools/time_policy.py --precision f32 --launches 5 --preroll 300 --trace --n 262144 --lib shippingenv_amd/_lib/abl/tq0.so || exit 1

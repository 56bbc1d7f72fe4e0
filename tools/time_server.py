"""Per-call time of the N = 1 GPU stepper (shipping/_device.py DeviceStepper), both forms:
the resident stepper wave (se_server_call, csrc/server.h) and one se_step_replay launch +
synchronise per step; and the raw se_server_call round trip without the Python packing.

    python tools/time_server.py [--steps 2000]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=2000)
    a = p.parse_args()
    import numpy as np

    from shippingenv_amd import _native as N
    from shippingenv_amd.maps import builtin_water
    from shippingenv_amd.shipping._device import DeviceStepper

    water = np.ascontiguousarray(builtin_water(), np.uint8)
    px, py = [41, 60, 78], [40, 22, 29]
    nan = float("nan")
    for server in (True, False):
        st = DeviceStepper(water, px, py, [100] * 3, [10] * 3, server=server)
        st.reset_to(0, 1)
        r = st.step(41, 40, 200.0, 0, 0, 1, 1, 0, 1, (0.5, 0.5, nan, nan, -1))
        t0 = time.perf_counter()
        for k in range(a.steps):
            # MOVE east and back: each step moves the ship (fuel draw used)
            r = st.step(r.x, r.y, r.fuel if r.fuel > 10 else 200.0, r.cargo, r.origin, r.dest, 1, 0,
                        1 if k % 2 == 0 else -1, (0.5, 0.5, nan, nan, -1))
        dt = (time.perf_counter() - t0) / a.steps
        rec = {"form": "stepper wave" if server else "launch + synchronise", "us_per_step": round(dt * 1e6, 2)}
        if server:
            t0 = time.perf_counter()
            for _ in range(a.steps):
                N.check(N.lib().se_server_call(st._srv, N.SERVER_STEP))
            rec["us_per_raw_call"] = round((time.perf_counter() - t0) / a.steps * 1e6, 2)
            rec["launches"] = st.launches()
        st.close()
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()

"""Where the N = 1 drop-in step spends its time (diagnostic): the bare launch +
synchronise of the device stepper, an empty-stream synchronise, and the full
Environment.step."""
import random
import sys
import time

import torch

sys.path.insert(0, ".")
from shippingenv_amd.shipping import ShipMove, environment  # noqa: E402


def per_call(f, n=2000):
    f()
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    return (time.perf_counter() - t0) / n * 1e6


random.seed(0)
env = environment.Environment("mapa_mundi_binario.jpg")
for p in ([41, 40], [60, 22], [78, 29], [49, 72], [62, 72]):
    env.add_port(p)
env.reset()
st = env._stepper
x, y = env._ship_xy()
s = torch.cuda.current_stream()
print("sync only us", per_call(lambda: s.synchronize()))
print("stepper.step us", per_call(lambda: st.step(x, y, 200.0, 0, 0, 1, 1, 0, 1, [0.5, 0.5, float("nan"), float("nan"), -1])))
print("world key us", per_call(lambda: env._world()))
import ctypes as C  # noqa: E402
from shippingenv_amd import _native as N  # noqa: E402
b = st._base


def launch():
    N.lib().se_step_replay(st._h, C.c_void_p(b + 160), C.c_void_p(b + 176), C.c_void_p(b + 192),
                           C.c_void_p(b + 208), C.c_void_p(s.cuda_stream))


def launch_sync():
    launch()
    s.synchronize()


def launch_spin():
    launch()
    while not s.query():
        pass


def launch_event():
    launch()
    e = torch.cuda.Event()
    e.record(s)
    e.synchronize()


print("launch+sync us", per_call(launch_sync))
print("launch+query-spin us", per_call(launch_spin))
print("launch+event sync us", per_call(launch_event))
t0 = time.perf_counter()
for _ in range(2000):
    launch()
t1 = time.perf_counter()
s.synchronize()
t2 = time.perf_counter()
print("launch only us", (t1 - t0) / 2000 * 1e6, "gpu per step us", (t2 - t0) / 2000 * 1e6)
moves = [ShipMove.NORTH, ShipMove.EAST, ShipMove.SOUTH, ShipMove.WEST]
pick = random.Random(1)


def one():
    try:
        _, _, done, _ = env.step([environment.ActionType.MOVE_SHIP, moves[pick.randrange(4)]])
    except ValueError:
        return
    if done:
        env.reset()


print("env.step us", per_call(one))

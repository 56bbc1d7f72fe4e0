"""Cost of the MCTS agent's per-simulation environment copy (agents/mcts.py:192-209:
Environment(map) + attribute assignment, then steps) through the drop-in package."""
import random
import sys
import time

sys.path.insert(0, ".")
from shippingenv_amd.shipping import environment  # noqa: E402

random.seed(0)
base = environment.Environment("mapa_mundi_binario.jpg")
for p in ([41, 40], [60, 22], [78, 29], [49, 72], [62, 72]):
    base.add_port(p)
base.reset()


def copy_env():
    e = environment.Environment("mapa_mundi_binario.jpg")
    e.port_positions = [list(p) for p in base.port_positions]
    e.port_cargo = list(base.port_cargo)
    e.port_fuel = list(base.port_fuel)
    e.ship_position = list(base.ship_position)
    e.cargo, e.fuel = base.cargo, base.fuel
    e.origin_port_index, e.destination_port_index = base.origin_port_index, base.destination_port_index
    e.np_game = base.np_game.copy()
    return e


for k in range(3):
    t0 = time.perf_counter()
    envs = [copy_env() for _ in range(50)]
    t1 = time.perf_counter()
    for e in envs:
        e.step([environment.ActionType.MOVE_SHIP, (0, 1)]) if e.np_game[41, 41] else None
    t2 = time.perf_counter()
    del envs
    t3 = time.perf_counter()
    print(f"50 copies {1e3 * (t1 - t0):.2f} ms, first steps {1e3 * (t2 - t1):.2f} ms, drop {1e3 * (t3 - t2):.2f} ms")

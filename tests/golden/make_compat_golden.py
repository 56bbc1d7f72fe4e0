"""Golden traces of the reference's Environment under a seeded global `random`.

TEST INFRASTRUCTURE, build container only (imports /root/reference with the cv2
stub of cv2stub/). Writes tests/golden/compat_seed{S}.json: one script of API
calls per seed (add_port, reset, step, sample_action, agent-side random()
draws) with everything the reference returned or raised, Python types
included. tests/test_compat_*.py replay the script against
shippingenv_amd.shipping.Environment and require identical results and an
identical `random` stream.

    python tests/golden/make_compat_golden.py
"""
import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, os.path.join(HERE, "cv2stub"))
sys.path.insert(0, REF)

from shipping import Environment  # noqa: E402

MAP = os.path.join(REF, "mapa_mundi_binario.jpg")
DEFAULT_PORTS = [[41, 40], [60, 22], [78, 29], [49, 72], [62, 72]]  # utils/constants.py:57-63


def tname(v):
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, (int, np.integer)) and not isinstance(v, np.integer):
        return "int"
    if isinstance(v, np.floating):
        return "np.float64"
    if isinstance(v, float):
        return "float"
    if isinstance(v, np.integer):
        return "np.int"
    if v is None:
        return "None"
    return type(v).__name__


def snap(env):
    st = env._build_state()["ship"]
    pos = st["position"]
    return {
        "position": [int(pos[0]), int(pos[1])] if len(pos) else [],
        "fuel": float(st["fuel"]), "fuel_type": tname(st["fuel"]),
        "cargo_field": float(st["cargo"]),
        "cargo": int(env.cargo),
        "origin": st["origin_port_index"], "dest": st["destination_port_index"],
        "aliases_port": any(pos is p for p in env.port_positions),
    }


def bfs(nonground, target):
    from collections import deque

    H, W = nonground.shape
    dist = np.full((H, W), -1, np.int32)
    dist[target[0], target[1]] = 0
    q = deque([tuple(target)])
    while q:
        x, y = q.popleft()
        for dx, dy in ((0, -1), (-1, 0), (0, 1), (1, 0)):
            nx, ny = x + dx, y + dy
            if 0 <= nx < H and 0 <= ny < W and nonground[nx, ny] and dist[nx, ny] < 0:
                dist[nx, ny] = dist[x, y] + 1
                q.append((nx, ny))
    return dist


FIELDS = {}


def make_action(rng, env):
    P = len(env.port_positions)
    r = rng.random()
    at = env._get_current_port_idx()
    if at is not None and r < 0.3:
        return [4 if rng.random() < 0.6 else 3, rng.randint(-1, 22)]
    if r < 0.6 and env.destination_port_index is not None:
        key = (id(env), env.destination_port_index)
        if key not in FIELDS:
            FIELDS[key] = bfs(env.np_game != 0, env.port_positions[env.destination_port_index])
        d = FIELDS[key]
        x, y = env.ship_position
        for dx, dy in ((0, -1), (-1, 0), (0, 1), (1, 0)):
            nx, ny = x + dx, y + dy
            if 0 <= nx < d.shape[0] and 0 <= ny < d.shape[1] and 0 <= d[nx, ny] < d[x, y]:
                return [1, (dx, dy)]
    if r < 0.75:
        return [1, rng.choice([(0, -1), (-1, 0), (0, 1), (1, 0)])]
    if r < 0.8:
        return [1, (rng.randint(-3, 3), rng.randint(-3, 3))]
    if r < 0.84:
        return [2, rng.randint(-1, P)]
    if r < 0.9:
        return [4, rng.randint(-1, 22)]
    if r < 0.95:
        return [3, rng.randint(-1, 22)]
    if r < 0.97:
        return [rng.choice([0, 5]), 1]
    return [1, (1, 0, 0)]  # malformed move tuple


def run(seed, n_events, ports):
    random.seed(seed)
    rng = random.Random(10_000 + seed)  # the script's own choices (not the env's RNG)
    env = Environment(MAP)
    events = []
    # a step before reset: destination None
    for p in ports:
        env.add_port(list(p))
    events.append({"op": "add_ports", "ports": ports, "port_fuel": list(env.port_fuel),
                   "port_cargo": list(env.port_cargo)})
    try:
        env.step([1, (0, 1)])
        events.append({"op": "step", "action": [1, [0, 1]], "exc": None})
    except Exception as e:  # noqa: BLE001
        events.append({"op": "step", "action": [1, [0, 1]], "exc": [type(e).__name__, str(e)], "after": snap(env)})
    env.reset()
    events.append({"op": "reset", "after": snap(env), "probe": random.random()})
    while len(events) < n_events:
        r = rng.random()
        if r < 0.05:
            try:
                a = env.sample_action()
                events.append({"op": "sample_action", "result": [a[0], list(a[1]) if isinstance(a[1], tuple) else a[1]], "exc": None})
            except Exception as e:  # noqa: BLE001
                events.append({"op": "sample_action", "exc": [type(e).__name__, str(e)]})
            continue
        if r < 0.07:
            env.reset()
            events.append({"op": "reset", "after": snap(env), "probe": random.random()})
            continue
        if r < 0.09:  # an agent assigns the fuel attribute (agents/mcts.py:205-206 style)
            v = rng.choice([0.5, 1, 2, 3.25, 250])
            env.fuel = v
            events.append({"op": "set_fuel", "value": v, "value_type": tname(v)})
            continue
        act = make_action(rng, env)
        ev = {"op": "step", "action": [act[0], list(act[1]) if isinstance(act[1], tuple) else act[1]]}
        try:
            _, reward, done, info = env.step([act[0], act[1]])
            ev.update({"exc": None, "reward": float(reward), "reward_type": tname(reward),
                       "done": bool(done), "done_type": tname(done)})
        except Exception as e:  # noqa: BLE001
            ev.update({"exc": [type(e).__name__, str(e)]})
        ev["after"] = snap(env)
        if rng.random() < 0.3:
            ev["probe"] = random.random()  # agent-side draw: checks the RNG stream position
        events.append(ev)
        if ev.get("done"):
            env.reset()
            events.append({"op": "reset", "after": snap(env), "probe": random.random()})
    return {"seed": seed, "events": events}


def main():
    rng = random.Random(5)
    water = None
    for seed in range(6):
        if seed < 4:
            ports = DEFAULT_PORTS
        else:
            env = Environment(MAP)
            cells = [(int(a), int(b)) for a, b in zip(*np.nonzero(env.np_game == 1))]
            ports = [list(c) for c in rng.sample(cells, 12)]
        out = run(seed, 700, ports)
        with open(os.path.join(HERE, f"compat_seed{seed}.json"), "w") as f:
            json.dump(out, f, separators=(",", ":"))
        steps = [e for e in out["events"] if e["op"] == "step"]
        arrivals = sum(1 for a, b in zip(out["events"], out["events"][1:])
                       if b["op"] == "step" and not b.get("exc") and "after" in a and "after" in b
                       and a["after"]["dest"] != b["after"]["dest"] and b["action"][0] == 1)
        losses = sum(1 for a, b in zip(out["events"], out["events"][1:])
                     if b["op"] == "step" and not b.get("exc") and "after" in a and "after" in b
                     and b["after"]["cargo"] < a["after"]["cargo"] and b["action"][0] == 1)
        print(seed, len(out["events"]), "steps", len(steps), "errors",
              sum(1 for e in steps if e.get("exc")), "done", sum(1 for e in steps if e.get("done")),
              "arrivals", arrivals, "losses", losses)


if __name__ == "__main__":
    main()

"""Generate the golden fixtures that pin the oracle and the HIP path to the reference.

TEST INFRASTRUCTURE. Runs only in the build container (it imports the reference
from /root/reference, which does not exist on the GPU box); its outputs are the
small committed files next to it. Usage:

    python tests/golden/make_golden.py            # rewrites tests/golden/*.npz|*.bin|*.json

What it does
------------
* Imports the reference ``shipping`` package with ``cv2stub/cv2.py`` on the path
  (opencv is not installed here; see that file's header).
* Replaces the ``random`` module the reference environment calls
  (shipping/environment.py:3, draws at :63,:64,:104,:157,:177,:195,:320) with a
  ``Recorder`` around ``random.Random(seed)`` that returns exactly what CPython's
  own methods return and logs the API-level variates: the 53-bit ``random()``
  behind ``uniform`` (CPython: ``a + (b-a)*random()``), the gate / loss-type
  ``random()`` draws, ``betavariate`` results and ``randint`` results.
* Drives one reference Environment per seed with a mixed policy and, for every
  ``step``/``reset``, stores (pre-state, action, variates, post-state, reward,
  done, error class). A step is thereby a pure function of (state, action,
  variates): the contract both the C oracle (replay mode) and the HIP kernel
  (replay mode) must reproduce bit for bit.

Files written
-------------
* ``map_water_100x100.bits``: np.packbits of the 100x100 0/1 map after
  _initialize_map (shipping/environment.py:45-55), before any port is stamped.
* ``golden_meta.json``: sha256 of the above, ports tables, error-code table.
* ``tape_seed{S}.npz``: per-record arrays (see FIELDS below).
* ``valid_mask_seed0.npz``: DQN ``is_valid_action`` bits (agents/dqn.py:125-175)
  for the post-state of the first records of seed 0.
"""
from __future__ import annotations

import hashlib
import json
import math
import os
import random as _stdlib_random
import sys
from collections import deque

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, os.path.join(HERE, "cv2stub"))
sys.path.insert(0, REF)

import shipping.environment as ref_env  # noqa: E402
from shipping import Environment  # noqa: E402
from utils.preprocessing import preprocess_state  # noqa: E402

MAP = os.path.join(REF, "mapa_mundi_binario.jpg")
DEFAULT_PORTS = [[41, 40], [60, 22], [78, 29], [49, 72], [62, 72]]  # utils/constants.py:57-63

# Error classes, keyed on (exception type, message) raised by the reference.
ERRORS = {
    ("ValueError", "Move is out of range"): 1,  # environment.py:284
    ("Exception", "Destination port must be different from current one"): 2,  # :267
    ("IndexError", "Port index is out of range"): 3,  # :269
    ("Exception", "Not currently at port"): 4,  # :343, :352
    ("ValueError", "Invalid fuel amount"): 5,  # :346, :355
    ("Exception", "Cannot move without destination port"): 6,  # :276
    ("ValueError", "Action category unknown"): 7,  # :374
    ("Exception", "No ports available"): 8,  # :360, :156
}


class Recorder:
    """Drop-in for the ``random`` module as used by shipping/environment.py."""

    def __init__(self, seed):
        self.r = _stdlib_random.Random(seed)
        self.log = []

    def random(self):
        u = self.r.random()
        self.log.append(("random", u))
        return u

    def uniform(self, a, b):  # CPython Lib/random.py: a + (b - a) * self.random()
        u = self.r.random()
        self.log.append(("uniform", u))
        return a + (b - a) * u

    def randint(self, a, b):
        v = self.r.randint(a, b)
        self.log.append(("randint", v))
        return v

    def betavariate(self, a, b):
        v = self.r.betavariate(a, b)
        self.log.append(("beta", v))
        return v

    def choice(self, seq):
        v = self.r.choice(seq)
        self.log.append(("choice", v))
        return v

    def take(self):
        out, self.log = self.log, []
        return out


FIELDS_I32 = [
    "kind", "act_type", "act_a", "act_b", "agent_idx",
    "pre_x", "pre_y", "pre_cargo", "pre_origin", "pre_dest",
    "post_x", "post_y", "post_cargo", "post_origin", "post_dest",
    "arrive_dest", "reset_origin", "reset_dest", "err", "done",
    "post_fuel_is_int",
]
FIELDS_F64 = ["pre_fuel", "post_fuel", "u_fuel", "u_gate", "u_type", "beta", "reward"]


def snapshot(env):
    x, y = env.ship_position if env.ship_position else (-1, -1)
    o = -1 if env.origin_port_index is None else env.origin_port_index
    d = -1 if env.destination_port_index is None else env.destination_port_index
    return int(x), int(y), float(env.fuel), int(env.cargo), int(o), int(d)


def agent_index(act_type, a, b, P):
    """Inverse of utils/preprocessing.py:111-137 where the action is representable."""
    if act_type == 1:
        moves = [(0, -1), (-1, 0), (0, 1), (1, 0)]  # N, E, S, W (:126)
        return moves.index((a, b)) if (a, b) in moves else -1
    if act_type == 2:
        return 4 + a if 0 <= a < P else -1
    if act_type == 4:
        return 4 + P + a if 0 <= a < 50 else -1
    if act_type == 3:
        return 4 + P + 50 + a if 0 <= a < 200 else -1
    return -1


def bfs_field(nonground, target, H, W):
    dist = np.full((H, W), -1, np.int32)
    tx, ty = target
    dist[tx, ty] = 0
    q = deque([(tx, ty)])
    while q:
        x, y = q.popleft()
        for dx, dy in ((0, -1), (-1, 0), (0, 1), (1, 0)):
            nx, ny = x + dx, y + dy
            if 0 <= nx < H and 0 <= ny < W and nonground[nx, ny] and dist[nx, ny] < 0:
                dist[nx, ny] = dist[x, y] + 1
                q.append((nx, ny))
    return dist


def choose_action(rng, env, fields, P):
    x, y = env.ship_position
    at_port = env._get_current_port_idx()
    r = rng.random()
    if at_port is not None and r < 0.35:
        if rng.random() < 0.6:
            return [4, rng.randint(1, env.port_cargo[at_port])]
        return [3, rng.randint(1, env.port_fuel[at_port])]
    r = rng.random()
    if r < 0.66:
        d = fields[env.destination_port_index]
        if d[x, y] > 0 and rng.random() < 0.8:
            best = None
            for dx, dy in ((0, -1), (-1, 0), (0, 1), (1, 0)):
                nx, ny = x + dx, y + dy
                if 0 <= nx < d.shape[0] and 0 <= ny < d.shape[1] and 0 <= d[nx, ny] < d[x, y]:
                    best = (dx, dy)
            if best is not None:
                return [1, best]
        return [1, rng.choice([(0, -1), (-1, 0), (0, 1), (1, 0)])]
    if r < 0.74:
        return [1, (rng.randint(-3, 3), rng.randint(-3, 3))]
    if r < 0.79:
        return [2, rng.randint(-1, P)]
    if r < 0.87:
        return [4, rng.randint(-1, 22)]
    if r < 0.95:
        return [3, rng.randint(-1, 22)]
    if r < 0.97:
        return [rng.choice([0, 5, 7]), rng.randint(0, 3)]
    return [1, rng.choice([(0, -1), (-1, 0), (0, 1), (1, 0)])]


def parse_move_draws(log):
    """Split one MOVE's logged draws into the fixed tape slots (Appendix A order)."""
    u_fuel = u_gate = u_type = beta = math.nan
    arrive = -1
    i = 0
    if i < len(log) and log[i][0] == "uniform":
        u_fuel = log[i][1]
        i += 1
    if i < len(log) and log[i][0] == "random":
        u_gate = log[i][1]
        i += 1
    if i < len(log) and log[i][0] == "random":
        u_type = log[i][1]
        i += 1
    if i < len(log) and log[i][0] == "beta":
        beta = log[i][1]
        i += 1
    while i < len(log) and log[i][0] == "randint":
        arrive = log[i][1]
        i += 1
    assert i == len(log), log
    return u_fuel, u_gate, u_type, beta, arrive


def run_seed(seed, n_records, ports_kind, with_valid=False):
    rec = Recorder(1000 + seed)
    ref_env.random = rec
    env = Environment(MAP)
    base_map = env.np_game.copy()
    H, W = base_map.shape
    if ports_kind == "default":
        ports = [list(p) for p in DEFAULT_PORTS]
    else:
        prng = _stdlib_random.Random(77 + seed)
        water = [(int(a), int(b)) for a, b in zip(*np.nonzero(base_map == 1))]
        ports = [list(p) for p in prng.sample(water, 64)]
    for p in ports:
        env.add_port(p)
    rec.take()
    P = len(ports)
    nonground = env.np_game != 0
    fields = [bfs_field(nonground, p, H, W) for p in ports]
    prng = _stdlib_random.Random(seed)

    cols = {k: [] for k in FIELDS_I32 + FIELDS_F64}
    obs6 = []
    valid = []
    port_block = None

    def push(kind, act, pre, post, reward, done, err, tape, fuel_is_int):
        t, a, b = act
        cols["kind"].append(kind)
        cols["act_type"].append(t)
        cols["act_a"].append(a)
        cols["act_b"].append(b)
        cols["agent_idx"].append(agent_index(t, a, b, P) if kind == 0 else -1)
        for name, v in zip(("x", "y", "fuel", "cargo", "origin", "dest"), pre):
            cols["pre_" + name].append(v)
        for name, v in zip(("x", "y", "fuel", "cargo", "origin", "dest"), post):
            cols["post_" + name].append(v)
        u_fuel, u_gate, u_type, beta, arrive, r_o, r_d = tape
        cols["u_fuel"].append(u_fuel)
        cols["u_gate"].append(u_gate)
        cols["u_type"].append(u_type)
        cols["beta"].append(beta)
        cols["arrive_dest"].append(arrive)
        cols["reset_origin"].append(r_o)
        cols["reset_dest"].append(r_d)
        cols["reward"].append(float(reward))
        cols["done"].append(int(bool(done)))
        cols["err"].append(err)
        cols["post_fuel_is_int"].append(int(fuel_is_int))

    def do_reset():
        nonlocal port_block
        pre = snapshot(env)
        state = env.reset()
        log = rec.take()
        draws = [v for k, v in log if k == "randint"]
        assert all(k == "randint" for k, _ in log)
        post = snapshot(env)
        push(1, (0, 0, 0), pre, post, 0.0, 0, 0,
             (math.nan,) * 4 + (-1, draws[0], draws[-1]), isinstance(env.fuel, int))
        row = preprocess_state(state)[0]
        obs6.append(np.asarray(row[:6], np.float64))
        if port_block is None:
            port_block = np.asarray(row[6:], np.float64)
        if with_valid and len(valid) < 600:
            valid.append(valid_bits(env, P))

    do_reset()
    ep_len = 0
    while len(cols["kind"]) < n_records:
        act = choose_action(prng, env, fields, P)
        t, v = act
        a, b = (v if t == 1 else (v, 0))
        pre = snapshot(env)
        err, reward, done = 0, 0.0, False
        state = None
        try:
            state, reward, done, _ = env.step([t, tuple(v) if t == 1 else v])
        except Exception as e:  # noqa: BLE001 - exceptions are the reference's control flow
            err = ERRORS[(type(e).__name__, str(e))]
        log = rec.take()
        post = snapshot(env)
        if t == 1 and err == 0:
            tape = parse_move_draws(log) + (-1, -1)
        else:
            assert not log, (act, log)
            tape = (math.nan,) * 4 + (-1, -1, -1)
        push(0, (t, a, b), pre, post, reward, done, err, tape, isinstance(env.fuel, int))
        if state is None:
            state = env._build_state()
        obs6.append(np.asarray(preprocess_state(state)[0][:6], np.float64))
        if with_valid and len(valid) < 600:
            valid.append(valid_bits(env, P))
        ep_len += 1
        if done or ep_len >= 600 or prng.random() < 0.002:
            do_reset()
            ep_len = 0

    n = len(cols["kind"])
    out = {k: np.asarray(cols[k], np.int32) for k in FIELDS_I32}
    out.update({k: np.asarray(cols[k], np.float64) for k in FIELDS_F64})
    out["obs6"] = np.stack(obs6).astype(np.float64)
    out["port_block"] = port_block
    out["port_x"] = np.asarray([p[0] for p in ports], np.int32)
    out["port_y"] = np.asarray([p[1] for p in ports], np.int32)
    out["port_fuel"] = np.asarray(env.port_fuel, np.int32)
    out["port_cargo"] = np.asarray(env.port_cargo, np.int32)
    if with_valid:
        out["valid_bits"] = np.stack(valid)
    assert all(len(v) == n for v in cols.values())
    return out, base_map


def _dqn_agent_class():
    # agents/__init__.py imports sarsa.py -> matplotlib (absent here); register a bare
    # package object so only agents/base.py and agents/dqn.py are executed.
    import types

    if "agents" not in sys.modules:
        pkg = types.ModuleType("agents")
        pkg.__path__ = [os.path.join(REF, "agents")]
        sys.modules["agents"] = pkg
    from agents.dqn import DQNAgent

    return DQNAgent


def valid_bits(env, P):
    """agents/dqn.py:125-175 is_valid_action for every agent index, packed."""
    DQNAgent = _dqn_agent_class()

    class _Self:
        pass

    s = _Self()
    s.env = env
    A = 4 + P + 50 + 200  # utils/preprocessing.py:93-108
    bits = np.array([DQNAgent.is_valid_action(s, a) for a in range(A)], np.uint8)
    return np.packbits(bits)


def run_random_states(seed, n_records, ports_kind):
    """Independent records from randomised pre-states (set the way agents/mcts.py:200-208
    sets them), so that every branch of _move_ship and every error class is hit often:
    edges (OOB), fuel-out, cargo >= 50 (gate always fires), ships next to their
    destination (arrival), destination None (error 6), and an env without ports (8)."""
    rec = Recorder(5000 + seed)
    ref_env.random = rec
    env = Environment(MAP)
    if ports_kind == "default":
        ports = [list(p) for p in DEFAULT_PORTS]
    else:
        prng = _stdlib_random.Random(77 + seed)
        water = [(int(a), int(b)) for a, b in zip(*np.nonzero(env.np_game == 1))]
        ports = [list(p) for p in prng.sample(water, 64)]
    for p in ports:
        env.add_port(p)
    rec.take()
    P = len(ports)
    H, W = env.np_game.shape
    clean = env.np_game.copy()
    nonground = [(int(a), int(b)) for a, b in zip(*np.nonzero(clean != 0))]
    prng = _stdlib_random.Random(9000 + seed)
    empty = Environment(MAP)  # no ports: every step raises "No ports available"

    cols = {k: [] for k in FIELDS_I32 + FIELDS_F64}
    unit = [(0, -1), (-1, 0), (0, 1), (1, 0)]
    for i in range(n_records):
        env.np_game[...] = clean
        o = prng.randrange(P)
        d = prng.choice([k for k in range(P) if k != o])
        r = prng.random()
        if r < 0.35:  # next to (or on) the destination port
            px, py = ports[d]
            cands = [(px + dx, py + dy) for dx, dy in unit + [(0, 0)]
                     if 0 <= px + dx < H and 0 <= py + dy < W]
            x, y = prng.choice(cands)
        elif r < 0.55:  # on an edge row / column
            x, y = prng.choice([(0, prng.randrange(W)), (H - 1, prng.randrange(W)),
                                (prng.randrange(H), 0), (prng.randrange(H), W - 1)])
        elif r < 0.65:  # on a port
            x, y = ports[prng.randrange(P)]
        else:
            x, y = prng.choice(nonground)
        fr = prng.random()
        if fr < 0.25:
            fuel = prng.randint(0, 250)  # still a Python int (no water move yet)
        elif fr < 0.5:
            fuel = prng.uniform(0.0, 1.3)  # fuel-out territory
        else:
            fuel = prng.uniform(-20.0, 400.0)
        cargo = prng.choice([0, prng.randint(0, 49), prng.randint(50, 90)])
        if prng.random() < 0.03:
            d = None
        env.ship_position = [x, y]
        env.fuel, env.cargo = fuel, cargo
        env.origin_port_index, env.destination_port_index = o, d
        ar = prng.random()
        if ar < 0.55:
            act = [1, prng.choice(unit)]
        elif ar < 0.7:
            act = [1, (prng.randint(-4, 4), prng.randint(-4, 4))]
        elif ar < 0.78:
            act = [2, prng.randint(-2, P + 1)]
        elif ar < 0.86:
            act = [4, prng.randint(-2, 25)]
        elif ar < 0.94:
            act = [3, prng.randint(-2, 25)]
        else:
            act = [prng.choice([-1, 0, 5, 9]), prng.randint(0, 3)]
        target = env
        if prng.random() < 0.01:
            target = empty
            target.ship_position = [x, y]
            target.fuel, target.cargo = fuel, cargo
            target.origin_port_index, target.destination_port_index = o, d
        t, v = act
        a, b = (v if t == 1 else (v, 0))
        pre = snapshot(target)
        err, reward, done = 0, 0.0, False
        try:
            _, reward, done, _ = target.step([t, v])
        except Exception as e:  # noqa: BLE001
            err = ERRORS[(type(e).__name__, str(e))]
        log = rec.take()
        post = snapshot(target)
        if t == 1 and err == 0:
            tape = parse_move_draws(log) + (-1, -1)
        else:
            assert not log, (act, log)
            tape = (math.nan,) * 4 + (-1, -1, -1)
        cols["kind"].append(2 if target is empty else 0)
        cols["act_type"].append(t)
        cols["act_a"].append(a)
        cols["act_b"].append(b)
        cols["agent_idx"].append(agent_index(t, a, b, P))
        for name, val in zip(("x", "y", "fuel", "cargo", "origin", "dest"), pre):
            cols["pre_" + name].append(val)
        for name, val in zip(("x", "y", "fuel", "cargo", "origin", "dest"), post):
            cols["post_" + name].append(val)
        u_fuel, u_gate, u_type, beta, arrive, r_o, r_d = tape
        for name, val in (("u_fuel", u_fuel), ("u_gate", u_gate), ("u_type", u_type),
                          ("beta", beta), ("arrive_dest", arrive), ("reset_origin", r_o),
                          ("reset_dest", r_d)):
            cols[name].append(val)
        cols["reward"].append(float(reward))
        cols["done"].append(int(bool(done)))
        cols["err"].append(err)
        cols["post_fuel_is_int"].append(int(isinstance(target.fuel, int)))
    out = {k: np.asarray(cols[k], np.int32) for k in FIELDS_I32}
    out.update({k: np.asarray(cols[k], np.float64) for k in FIELDS_F64})
    out["port_x"] = np.asarray([p[0] for p in ports], np.int32)
    out["port_y"] = np.asarray([p[1] for p in ports], np.int32)
    out["port_fuel"] = np.asarray(env.port_fuel, np.int32)
    out["port_cargo"] = np.asarray(env.port_cargo, np.int32)
    return out


def summarize(out):
    return {
        "records": int(len(out["kind"])),
        "resets": int((out["kind"] == 1).sum()),
        "arrivals": int((out["arrive_dest"] >= 0).sum()),
        "beta_events": int(np.isfinite(out["beta"]).sum()),
        "loss_type_draws": int(np.isfinite(out["u_type"]).sum()),
        "fuel_out": int(out["done"].sum()),
        "errors": {str(c): int((out["err"] == c).sum()) for c in range(1, 9)},
    }


def main():
    counts = {}
    meta = {"ports": {}, "errors": {f"{k[0]}: {k[1]}": v for k, v in ERRORS.items()}}
    base_map = None
    for seed in range(8):
        kind = "default" if seed < 6 else "random64"
        out, base_map = run_seed(seed, 2500, kind, with_valid=(seed == 0))
        np.savez_compressed(os.path.join(HERE, f"tape_seed{seed}.npz"), **out)
        meta["ports"][f"seed{seed}"] = {
            "x": out["port_x"].tolist(), "y": out["port_y"].tolist(),
            "fuel": out["port_fuel"].tolist(), "cargo": out["port_cargo"].tolist(),
        }
        counts[f"tape{seed}"] = summarize(out)
    for seed, kind in ((0, "default"), (1, "random64")):
        out = run_random_states(seed, 6000, kind)
        np.savez_compressed(os.path.join(HERE, f"states_seed{seed}.npz"), **out)
        counts[f"states{seed}"] = summarize(out)
    bits = np.packbits(base_map.astype(np.uint8).reshape(-1))
    with open(os.path.join(HERE, "map_water_100x100.bits"), "wb") as f:
        f.write(bits.tobytes())
    meta["map"] = {
        "shape": [100, 100],
        "sha256_u8_rowmajor": hashlib.sha256(base_map.astype(np.uint8).tobytes()).hexdigest(),
        "sha256_packbits": hashlib.sha256(bits.tobytes()).hexdigest(),
        "water_cells": int(base_map.sum()),
    }
    meta["counts"] = counts
    with open(os.path.join(HERE, "golden_meta.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(json.dumps(counts, indent=1))


if __name__ == "__main__":
    main()

"""shipping.environment — the reference's Environment API on the gfx950 step kernel.

Drop-in for /root/reference/shipping/environment.py:28-376: same constructor,
public methods, private helpers the agents call (_build_state,
_get_current_port_idx, _sample_random_*), attributes (port_positions,
port_fuel, port_cargo, ship_position, fuel, cargo, origin_port_index,
destination_port_index, np_game, size_game) and exceptions (type and message).

How a step runs. Attributes stay on the host because agents read and assign
them directly (agents/mcts.py:200-208). ``step`` ships the state and the action
to the HIP kernel (se_step_replay on a one-env handle, ``_device.py``), which
computes the whole transition. The variates come from the global ``random``
module in the reference's order, exactly as the reference draws them:
``random()`` behind ``uniform`` for the fuel cost, ``random()`` for the loss
gate, then, only where the kernel reports the reference would draw them, the
loss type, ``betavariate(2, 2)`` and the ``randint`` destination redraw. When
the kernel needs a variate not drawn yet it answers SE_ERR_NEED_DRAW without
effect; the host draws exactly that one and steps again. Seeded with
``random.seed`` this reproduces the reference's trajectories bit for bit,
including the RNG state the agents see between steps.

Python types follow the reference: fuel stays an int until the first move onto
water, then becomes an np.float64 (:39, :298); rewards are ints for SELECT and
for moves blocked by ground, floats otherwise; done is a bool.
"""
from __future__ import annotations

import math
import operator
import random

import numpy as np

from .. import _native as N
from ..maps import load_water
from .type import ActionType, Color, Entity, ShipMove  # noqa: F401 (re-exported like the reference)
from .util import calculate_euclidean_distance, normalize  # noqa: F401


class Initial:
    CARGO = 0
    FUEL = 200
    MAX_CARGO_CAPACITY = 50


class Reward:
    CARGO_DELIVER = 2
    REACH_DESTINATION = 10
    CLOSER_TO_DESTINATION = 2
    TAKE_FUEL = 0.05
    TAKE_CARGO = 0.05


class Penalty:
    RUN_OUT_OF_FUEL = -10
    MOVE_ON_GROUND = -5
    MOVE_ON_WATER = -1
    CARGO_LOSS = -3
    FARTHER_FROM_DESTINATION = -2
    USE_FUEL = -0.0001


# SE_ERR_* -> the exception the reference raises (environment.py line)
_ERRORS = {
    N.ERR_OOB: (ValueError, "Move is out of range"),  # :284
    N.ERR_SAME_PORT: (Exception, "Destination port must be different from current one"),  # :267
    N.ERR_PORT_RANGE: (IndexError, "Port index is out of range"),  # :269
    N.ERR_NOT_AT_PORT: (Exception, "Not currently at port"),  # :343, :352
    N.ERR_AMOUNT: (ValueError, "Invalid fuel amount"),  # :346, :355
    N.ERR_NO_DEST: (Exception, "Cannot move without destination port"),  # :276
    N.ERR_BAD_CATEGORY: (ValueError, "Action category unknown"),  # :374
    N.ERR_NO_PORTS: (Exception, "No ports available"),  # :360
}

# Builds the stepper of a new environment: the host stepper (_host.HostStepper: the step
# kernels' per-env code compiled for the host, one C call per step) unless
# SHIPENV_STEPPER=gpu selects the kernel (_device.DeviceStepper: one launch and one
# stream synchronise per step). Tests may install another with _set_stepper_factory.
_STEPPER_FACTORY = None


def _set_stepper_factory(factory):
    global _STEPPER_FACTORY
    _STEPPER_FACTORY = factory


def stepper_kind():
    """'host' (default) or 'gpu', from SHIPENV_STEPPER."""
    import os

    kind = os.environ.get("SHIPENV_STEPPER", "host").strip().lower()
    if kind not in ("host", "gpu"):
        raise ValueError(f"SHIPENV_STEPPER must be 'host' or 'gpu', not {kind!r}")
    return kind


def _new_stepper(water, px, py, pf, pc):
    if _STEPPER_FACTORY is not None:
        return _STEPPER_FACTORY(water, px, py, pf, pc)
    if stepper_kind() == "gpu":
        from ._device import DeviceStepper

        return DeviceStepper(water, px, py, pf, pc)
    from ._host import HostStepper

    return HostStepper(water, px, py, pf, pc)


def _port_key(positions):
    """Port positions as int tuples: add_port keeps `pos` as given (:57-65), and a list,
    tuple or numpy array must key the same way (ndarray == ndarray has no truth value)."""
    return tuple(tuple(int(v) for v in p) for p in positions)


def _category(c):
    """`match action_category` compares by equality (:364-374)."""
    if type(c) is int and 1 <= c <= 4:  # the plain ints of ActionType
        return c
    for t in (ActionType.MOVE_SHIP, ActionType.SELECT_PORT, ActionType.TAKE_FUEL,
              ActionType.TAKE_CARGO):
        try:
            if c == t:
                return t
        except Exception:  # noqa: BLE001 - exotic objects simply do not match
            pass
    return 0


class Environment:
    def __init__(self, map_path, game_size=(100, 100)):
        self.size_game = game_size
        if game_size[0] != game_size[1]:
            # the reference resizes to (W, H) but bounds-checks x against size[0] (:53, :99-100)
            raise ValueError("non-square game_size is not supported (SURVEY.md §4, defect 7)")
        self.port_positions = []
        self.port_fuel = []
        self.port_cargo = []
        self.ship_position = []
        self.cargo = Initial.CARGO
        self.fuel = Initial.FUEL
        self.origin_port_index = None
        self.destination_port_index = None
        self._stepper = None
        self._world_key = None
        self._g_ref = self._ground = None
        self._pp = self._pp_raw = self._pf = self._pc = None
        self._initialize_map(map_path)

    # ------------------------------------------------------------------ setup
    def _initialize_map(self, map_path):
        """:45-55 (JPEG -> gray -> crop -> INTER_AREA resize -> threshold), see maps.py."""
        self.np_game = load_water(map_path, self.size_game).astype(int)

    def add_port(self, pos):
        x, y = pos[0], pos[1]
        if not self._is_within_map(x, y):
            raise ValueError("Coordinates not within map")
        self.port_positions.append(pos)
        self.port_fuel.append(random.randint(5, 20))
        self.port_cargo.append(random.randint(5, 20))
        self.np_game[x, y] = Entity.PORT

    def remove_port(self, idx):
        # The reference compares an int with a list here and always raises TypeError
        # (defect 6); the same comparison keeps that behaviour.
        if 0 <= idx < self.port_positions and 0 <= idx < self.port_cargo:
            x, y = self.port_positions[idx]
            self.np_game[x, y] = Entity.GROUND
            self.port_fuel.pop(idx)
            self.port_cargo.pop(idx)
            return self.port_positions.pop(idx)
        raise IndexError("Invalid index")

    def _is_within_map(self, x, y):
        within_width = 0 <= x < self.size_game[0]
        within_height = 0 <= y < self.size_game[1]
        return within_width and within_height

    def _calculate_fuel_cost(self, start, end):
        return calculate_euclidean_distance(start, end) * (1 + random.uniform(-0.1, 0.1))

    def render_real_time(self, render_size=(355, 533)):
        """The cv2 window of :106-143 is out of scope (GUI only); nothing is drawn."""
        return None

    # ------------------------------------------------------------------ queries
    def _get_current_port_idx(self):
        for idx, port_position in enumerate(self.port_positions):
            if port_position == self.ship_position:
                return idx
        return None

    def _sample_random_port(self):
        if len(self.port_positions) == 0:
            raise Exception("No ports available")
        return random.randint(0, len(self.port_positions) - 1)

    def _sample_random_cargo(self, port_idx):
        return random.randint(1, self.port_cargo[port_idx])

    def _sample_random_fuel(self, port_idx):
        # indexes self.fuel like the reference (:163): TypeError (defect 5)
        return random.randint(1, self.fuel[port_idx])

    def _sample_random_move(self):
        return random.choice([ShipMove.NORTH, ShipMove.EAST, ShipMove.SOUTH, ShipMove.WEST])

    def _build_state(self):
        ship = {
            "position": self.ship_position,
            "fuel": self.fuel,
            "cargo": self.fuel,  # the reference reports fuel as cargo (:206)
            "origin_port_index": self.origin_port_index,
            "destination_port_index": self.destination_port_index,
        }
        ports = [
            {"index": idx, "position": pos, "fuel": self.port_fuel[idx],
             "cargo": self.port_cargo[idx]}
            for idx, pos in enumerate(self.port_positions)
        ]
        return {"ship": ship, "ports": ports}

    def sample_action(self):
        current_port_idx = self._get_current_port_idx()
        if self.destination_port_index is None and current_port_idx is not None:
            port_index = self._sample_random_port()
            while port_index == current_port_idx:
                port_index = self._sample_random_port()
            return [ActionType.SELECT_PORT, port_index]
        elif self.cargo == 0 and current_port_idx is not None:
            return [ActionType.TAKE_CARGO, self._sample_random_cargo(current_port_idx)]
        elif self.fuel == 0 and current_port_idx is not None:
            return [ActionType.TAKE_FUEL, self._sample_random_fuel(current_port_idx)]
        else:
            return [ActionType.MOVE_SHIP, self._sample_random_move()]

    # ------------------------------------------------------------------ device
    def _world(self, cell=None):
        """The stepper follows assignments to np_game / port lists (agents/mcts.py:200-208)
        and in-place edits of np_game: the reference reads the ground test live on every
        move (environment.py:293). The full check keys the device world on the ground
        mask's bytes and the port lists; it runs when np_game is another object, a port
        list changed, or the one cell this step's kernel reads (a move's target, `cell`)
        disagrees with the mask the device holds. A step reads no other cell, so the
        fast path (no pass over the grid: the full key cost ~15 us of a ~30 us step) is
        exact for every read the kernel makes."""
        g = self.np_game
        if (self._stepper is not None and g is self._g_ref and type(g) is np.ndarray
                and self._ports_unchanged()
                and self.port_fuel == self._pf and self.port_cargo == self._pc
                and (cell is None or (g.item(cell) == Entity.GROUND) == self._ground.item(cell))):
            return self._stepper
        ground = np.asarray(g) == Entity.GROUND
        ports = _port_key(self.port_positions)
        key = (ground.shape, ground.tobytes(), ports, tuple(self.port_fuel), tuple(self.port_cargo))
        if self._stepper is None or key != self._world_key:
            water = (~ground).astype(np.uint8)
            px = [int(p[0]) for p in self.port_positions]
            py = [int(p[1]) for p in self.port_positions]
            if self._stepper is None:
                self._stepper = _new_stepper(water, px, py, self.port_fuel, self.port_cargo)
            else:
                self._stepper.set_world(water, px, py, self.port_fuel, self.port_cargo)
            self._world_key = key
        self._g_ref, self._ground = g, ground
        self._pp = ports
        # list positions compare as lists (one C-level comparison); any other indexable
        # is compared through its int key (_ports_unchanged)
        self._pp_raw = [list(p) if type(p) is list else tuple(q) for p, q in zip(self.port_positions, ports)]
        self._pf, self._pc = list(self.port_fuel), list(self.port_cargo)
        return self._stepper

    def _ports_unchanged(self):
        """port_positions still equal the positions the device world was built from: the
        list comparison first (the common case: add_port with lists), then, when that is
        False or has no truth value (numpy positions), the int keys."""
        try:
            if self.port_positions == self._pp_raw:
                return True
        except ValueError:  # ndarray == ndarray inside the list comparison
            pass
        return _port_key(self.port_positions) == self._pp

    def _ship_xy(self):
        if len(self.ship_position) == 0:
            return 0, 0
        return int(self.ship_position[0]), int(self.ship_position[1])

    # ------------------------------------------------------------------ reset / step
    def reset(self):
        self.np_game[((self.np_game == Entity.BOAT) + (self.np_game == Entity.TRAVEL))] = Entity.WATER
        self.cargo = Initial.CARGO
        self.fuel = Initial.FUEL
        self.origin_port_index = self._sample_random_port()
        self.destination_port_index = self._sample_random_port()
        while self.origin_port_index == self.destination_port_index:
            self.destination_port_index = self._sample_random_port()
        res = self._world().reset_to(self.origin_port_index, self.destination_port_index)
        current_port = self.port_positions[self.origin_port_index]
        assert (res.x, res.y) == (int(current_port[0]), int(current_port[1]))
        self.np_game[current_port[0], current_port[1]] = Entity.BOAT
        self.ship_position = current_port  # aliases the port's list like :241
        return self._build_state()

    def _run(self, act_type, a, b):
        """Step on the device, drawing the reference's variates as the kernel asks for them."""
        rs = random
        x, y = self._ship_xy()
        cell = None  # the one grid cell this step reads: a move's target (:293)
        if act_type == ActionType.MOVE_SHIP:
            g = self.np_game
            shp = g.shape if type(g) is np.ndarray else np.shape(g)
            H, W = shp[0], shp[1]
            if 0 <= x + a < H and 0 <= y + b < W:
                cell = (x + a, y + b)
        stepper = self._world(cell)
        tape = [math.nan, math.nan, math.nan, math.nan, -1]
        ahead = False
        if act_type == ActionType.MOVE_SHIP and self.destination_port_index is not None:
            if cell is not None:
                # a MOVE that raises neither at :276 nor at :284 draws uniform() then
                # random() (:104, :320): draw them ahead, saving the kernel's request
                ahead = True
                tape[0] = rs.random()
                tape[1] = rs.random()
        while True:
            res = stepper.step(x, y, float(self.fuel), int(self.cargo), self.origin_port_index,
                               self.destination_port_index, act_type, a, b, tape)
            if res.err != N.ERR_NEED_DRAW:
                break
            if math.isnan(tape[0]):
                tape[0] = rs.random()
                tape[1] = rs.random()
            elif res.used & N.USED_LOSS_TYPE and math.isnan(tape[2]):
                tape[2] = rs.random()
            elif res.used & N.USED_BETA and math.isnan(tape[3]):
                tape[3] = rs.betavariate(2, 2)
            elif res.used & N.USED_ARRIVE and tape[4] < 0:
                new_origin = self.destination_port_index  # :332
                d = self._sample_random_port()
                while d == new_origin:
                    d = self._sample_random_port()
                tape[4] = d
            else:
                raise RuntimeError("step kernel asked for a variate the protocol cannot supply")
        if ahead and not (res.used & N.USED_FUEL_GATE):
            raise RuntimeError("the step kernel raised a move the host expected to draw for")
        return res

    def step(self, action):
        if len(self.port_positions) == 0:
            raise Exception("No ports available")
        action_category, action_value = action
        act_type = _category(action_category)
        if act_type == ActionType.MOVE_SHIP:
            if len(action_value) != 2:
                raise ValueError("Move needs to be of format (x,y) or [x, y]")
            a, b = operator.index(action_value[0]), operator.index(action_value[1])
        elif act_type == 0:
            a = b = 0
        else:
            a, b = operator.index(action_value), 0
        res = self._run(act_type, a, b)
        if res.err != N.ERR_OK:
            exc, msg = _ERRORS[res.err]
            raise exc(msg)

        moved = bool(res.used & N.USED_MOVED)
        if act_type == ActionType.MOVE_SHIP:
            if moved:  # :297-304
                ox, oy = self._ship_xy()
                self.ship_position = [res.x, res.y]
                self.np_game[ox, oy] = Entity.TRAVEL
                self.np_game[res.x, res.y] = Entity.BOAT
            reward = int(res.reward) if not moved else float(res.reward)
        else:
            reward = int(res.reward) if act_type == ActionType.SELECT_PORT else float(res.reward)
        # `fuel -= np.float64` on a water move makes it an np.float64 (:298); otherwise
        # (blocked move, `fuel += int` at a port) it keeps its Python type
        self.fuel = np.float64(res.fuel) if moved else type(self.fuel)(res.fuel)
        self.cargo = res.cargo
        self.origin_port_index = None if res.origin < 0 else res.origin
        self.destination_port_index = None if res.dest < 0 else res.dest
        return self._build_state(), reward, res.done, {}

"""Enumerations of the reference's shipping/type.py (same values; agents and
utils compare against them)."""


class ActionType:
    """The `action[0]` categories of Environment.step (shipping/type.py:1-5)."""

    MOVE_SHIP = 1
    SELECT_PORT = 2
    TAKE_FUEL = 3
    TAKE_CARGO = 4


class ShipMove:
    """(dx, dy) moves; x is the map row (shipping/type.py:8-16)."""

    NORTH = (0, -1)
    SOUTH = (0, 1)
    EAST = (-1, 0)
    WEST = (1, 0)


class Entity:
    """np_game cell codes (shipping/type.py:19-30); the step only tests GROUND."""

    GROUND = 0
    WATER = 1
    PORT = 2
    DESTINY_PORT = 3
    BOAT = 5
    STORM = 6
    TRAVEL = 7


class Color:
    """BGR colours of the reference's cv2 renderer (shipping/type.py:33-46)."""

    WATER = [255, 0, 0]
    GROUND = [37, 73, 141]
    TRAVEL = [0, 0, 255]
    PORT = [154, 152, 150]
    DESTINY_PORT = [0, 255, 0]
    STORM = [128, 128, 128]
    BOAT = [65, 138, 222]
    WHITE = [255, 255, 255]
    BLACK = [0, 0, 0]

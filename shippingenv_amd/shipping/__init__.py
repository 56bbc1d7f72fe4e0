"""The reference's ``shipping`` package surface (shipping/__init__.py:1-2) on the
gfx950 step kernel. ``shippingenv_amd/dropin`` exposes it under the name
``shipping`` so the reference's agents and utils import it unchanged."""
from . import environment, type, util  # noqa: F401
from .environment import Environment
from .type import ShipMove

__all__ = ["Environment", "ShipMove", "environment", "type", "util"]

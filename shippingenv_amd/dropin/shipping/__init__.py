"""Drop-in ``shipping`` package.

Put ``<repo>/shippingenv_amd/dropin`` ahead of the reference on ``sys.path``
(``PYTHONPATH``); ``import shipping``, ``from shipping import Environment,
ShipMove`` and ``from shipping import environment`` (agents/sarsa.py:11,
agents/mcts.py:9) then resolve to the MI355X implementation.
"""
import os
import sys

_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
if _root not in sys.path:
    sys.path.append(_root)

from shippingenv_amd.shipping import environment, type, util  # noqa: E402
from shippingenv_amd.shipping.environment import Environment  # noqa: E402
from shippingenv_amd.shipping.type import ShipMove  # noqa: E402

sys.modules[__name__ + ".environment"] = environment
sys.modules[__name__ + ".type"] = type
sys.modules[__name__ + ".util"] = util

__all__ = ["Environment", "ShipMove", "environment", "type", "util"]

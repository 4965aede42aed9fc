"""Status bitmask <-> the reference's status strings (RLEnv/MSRL_env_ex.py:742-807, 817-879, 890-899)."""
from __future__ import annotations

from . import _lib as L

_TEST = ((L.ST_TEST_ENDPOINT, "|Test ship reaches endpoint|"),
         (L.ST_TEST_HORIZON, "|Test ship hits map horizon|"),
         (L.ST_TEST_TERRAIN, "|Test ship collides with the terrain|"),
         (L.ST_TEST_MECHANICAL, "|Test ship mechanical failure|"),
         (L.ST_TEST_NAVIGATION, "|Test ship navigation failure|"),
         (L.ST_TEST_BLACKOUT, "|Test ship blackout failure|"))
_OBS = ((L.ST_OBS_ENDPOINT, "|Obstacle ship reaches endpoint|"),
        (L.ST_OBS_HORIZON, "|Obstacle ship hits map horizon|"),
        (L.ST_OBS_TERRAIN, "|Obstacle ship collides with the terrain|"),
        (L.ST_OBS_IW_TERMINAL, "|Obstacle ship IW sampled in terminal state|"),
        (L.ST_OBS_NAVIGATION, "|Obstacle ship navigation failure|"))

FAILURE_NAMES = {bit: txt.strip("|") for bit, txt in _TEST + _OBS}
FAILURE_NAMES[L.ST_COLLISION] = "Ship collision"


def status_string(bits: int) -> str:
    """Exactly the string MultiShipRLEnv.step returns for this bitmask."""
    bits = int(bits)
    t = " " + "".join(txt for bit, txt in _TEST if bits & bit)
    if not bits & L.ST_TEST_DONE:
        t += "|Test ship not in terminal state|"
    o = " " + "".join(txt for bit, txt in _OBS if bits & bit)
    if not bits & L.ST_OBS_DONE:
        o += "|Obstacle ship not in terminal state|"
    return t + o + " " + ("|Ship collision|" if bits & L.ST_COLLISION else "")

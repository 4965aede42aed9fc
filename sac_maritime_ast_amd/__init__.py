"""MI355X-native ship-in-transit env step for SAC-AST rollouts (drop-in for the reference's
``MultiShipRLEnv`` hot path).  The compute is the HIP library libsit.so; see include/sit.h."""
from . import _lib
from .config import params, params_from_reference
from .scenario import Scenario, make_scenario
from .status import status_string

__all__ = ["params", "params_from_reference", "Scenario", "make_scenario", "status_string",
           "VecMultiShipRLEnv", "MultiShipRLEnv", "load_library"]


def load_library():
    return _lib.load()


def __getattr__(name):
    if name == "VecMultiShipRLEnv":
        from .env import VecMultiShipRLEnv
        return VecMultiShipRLEnv
    if name == "MultiShipRLEnv":
        from .compat import MultiShipRLEnv
        return MultiShipRLEnv
    raise AttributeError(name)

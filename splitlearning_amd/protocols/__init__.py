from .base import Session, AliceState
from .vanilla import VanillaSession
from .ushape import UShapeSession
from .sisa import SisaSession, ControlSession
from .concat import ConcatSession
from .schedule import run_schedule

SESSIONS = {"vanilla": VanillaSession, "ushape": UShapeSession, "sisa": SisaSession,
            "control": ControlSession, "concat": ConcatSession}


def make_session(args, comm, device) -> Session:
    return SESSIONS[args.mode](args, comm, device)


# Reference-named entry points: `get_alice_and_bob(args)` returned the (alice, bob)
# classes of the selected entity module (split_nn.py:13-23).  Here the session class
# is both roles' API for the selected mode.
def get_alice_and_bob(args):
    cls = SESSIONS[args.mode]
    return cls, cls


__all__ = ["Session", "AliceState", "VanillaSession", "UShapeSession", "SisaSession",
           "ControlSession", "ConcatSession", "run_schedule", "make_session", "SESSIONS",
           "get_alice_and_bob"]

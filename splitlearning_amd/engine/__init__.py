from .slots import OptSlot, adam, sgd_momentum
from .front import FrontEngine
from .tail import TailEngine

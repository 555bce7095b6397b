from .logging import role_logger, NULL
from .metrics import PhaseTimer, sync

__all__ = ["role_logger", "NULL", "PhaseTimer", "sync"]

"""Debug subsystems: exchange race checking and fault injection."""
from .race import ExchangeChecker, RaceError
from .faults import FaultyComm, FaultPlan

__all__ = ["ExchangeChecker", "RaceError", "FaultyComm", "FaultPlan"]

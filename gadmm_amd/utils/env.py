"""Environment switches read on hot host paths (docs/ENV.md).

``os.environ.get`` encodes the key, looks it up and decodes the value on every call (~0.6-1 us); a
D-GADMM or headline solve reads a few dozen A/B switches, so that alone was ~15-30 us of host time per
solve. ``getenv`` reads the same mapping (``os.environ``'s backing dict, which ``os.environ[...] = ``,
``del`` and pytest's ``monkeypatch.setenv`` update) with the key encoded once: same values."""
from __future__ import annotations

import os
from typing import Dict, Optional

_KEYS: Dict[str, bytes] = {}

if isinstance(os.environ, os._Environ) and isinstance(getattr(os.environ, "_data", None), dict):
    _DATA = os.environ._data
    _ENC = os.environ.encodekey
    _DEC = os.environ.decodevalue

    def getenv(name: str, default: Optional[str] = None) -> Optional[str]:
        """``os.environ.get(name, default)``."""
        k = _KEYS.get(name)
        if k is None:
            k = _KEYS[name] = _ENC(name)
        v = _DATA.get(k)
        return default if v is None else _DEC(v)
else:  # not CPython's posix mapping
    def getenv(name: str, default: Optional[str] = None) -> Optional[str]:
        """``os.environ.get(name, default)``."""
        return os.environ.get(name, default)

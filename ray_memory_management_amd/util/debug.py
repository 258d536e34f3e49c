"""Logging helpers. Parity: reference python/ray/util/debug.py (log_once,
disable_log_once_globally, enable_periodic_logging)."""
from __future__ import annotations

import time

_logged = set()
_disabled = False
_periodic_log = False
_last_logged = 0.0


def log_once(key) -> bool:
    """True the first time `key` is seen (or every 60 s with periodic logging on)."""
    global _last_logged
    if _disabled:
        return False
    if key not in _logged:
        _logged.add(key)
        _last_logged = time.time()
        return True
    if _periodic_log and time.time() - _last_logged > 60.0:
        _logged.clear()
        _last_logged = time.time()
        return False
    return False


def disable_log_once_globally():
    global _disabled
    _disabled = True


def enable_periodic_logging():
    global _periodic_log
    _periodic_log = True


def reset_log_once(key=None):
    if key is None:
        _logged.clear()
    else:
        _logged.discard(key)

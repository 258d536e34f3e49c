"""API stability annotations. Parity: reference python/ray/util/annotations.py."""
from __future__ import annotations

import functools
import warnings


def _annotate(obj, tag: str, extra: str = ""):
    doc = obj.__doc__ or ""
    note = f"\n\n    {tag}{(': ' + extra) if extra else ''}"
    try:
        obj.__doc__ = doc + note
    except (AttributeError, TypeError):
        pass
    try:
        obj._annotated = tag
    except (AttributeError, TypeError):
        pass
    return obj


def PublicAPI(*args, **kwargs):
    """Public, stable API (``stability="stable"|"beta"|"alpha"``)."""
    if len(args) == 1 and not kwargs and callable(args[0]):
        return _annotate(args[0], "PublicAPI")
    stability = kwargs.get("stability", "stable")
    return lambda obj: _annotate(obj, f"PublicAPI ({stability})")


def DeveloperAPI(*args, **kwargs):
    if len(args) == 1 and not kwargs and callable(args[0]):
        return _annotate(args[0], "DeveloperAPI")
    return lambda obj: _annotate(obj, "DeveloperAPI")


def Deprecated(*args, **kwargs):
    message = kwargs.get("message", "")

    def wrap(obj):
        if isinstance(obj, type):
            return _annotate(obj, "Deprecated", message)

        @functools.wraps(obj)
        def inner(*a, **k):
            warnings.warn(f"{obj.__name__} is deprecated. {message}", DeprecationWarning, stacklevel=2)
            return obj(*a, **k)

        return _annotate(inner, "Deprecated", message)

    if len(args) == 1 and not kwargs and callable(args[0]):
        return wrap(args[0])
    return wrap

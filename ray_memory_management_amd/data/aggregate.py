"""Aggregations. Parity: reference python/ray/data/aggregate.py (AggregateFn, Count, Sum, Min,
Max, Mean, Std with ignore_nulls) — init / accumulate / merge / finalize protocol so partial
aggregates computed per block combine in any order."""
from __future__ import annotations

import math
from typing import Any, Callable, Optional


def _getter(on):
    if on is None:
        return lambda r: r
    if callable(on):
        return on
    return lambda r: r[on]


def _isnull(v):
    return v is None or (isinstance(v, float) and math.isnan(v))


class AggregateFn:
    def __init__(self, init: Callable[[Any], Any], merge: Callable[[Any, Any], Any],
                 accumulate_row: Optional[Callable[[Any, Any], Any]] = None,
                 finalize: Callable[[Any], Any] = lambda a: a, name: Optional[str] = None,
                 accumulate: Optional[Callable[[Any, Any], Any]] = None):
        if accumulate_row is None:
            accumulate_row = accumulate
        if accumulate_row is None:
            raise ValueError("accumulate_row is required")
        self.init, self.merge, self.accumulate_row, self.finalize = init, merge, accumulate_row, finalize
        self.name = name or "agg"

    def accumulate_rows(self, key, rows):
        a = self.init(key)
        for r in rows:
            a = self.accumulate_row(a, r)
        return a


class _NullAware(AggregateFn):
    """Skips nulls if ignore_nulls else poisons the result with None."""

    def __init__(self, name, on, ignore_nulls, init, acc, merge, finalize=lambda a: a):
        get = _getter(on)
        POISON = "__null__"

        def accumulate(a, r):
            if a is POISON:
                return a
            v = get(r)
            if _isnull(v):
                return a if ignore_nulls else POISON
            return acc(a, v)

        def merge2(a, b):
            if a is POISON or b is POISON:
                return POISON
            return merge(a, b)

        def fin(a):
            return None if a is POISON else finalize(a)

        super().__init__(init=init, merge=merge2, accumulate_row=accumulate, finalize=fin, name=name)


def _label(fn, on):
    return f"{fn}({on})" if isinstance(on, str) else f"{fn}()"


class Count(AggregateFn):
    def __init__(self):
        super().__init__(init=lambda k: 0, accumulate_row=lambda a, r: a + 1, merge=lambda a, b: a + b,
                         name="count()")


class Sum(_NullAware):
    def __init__(self, on=None, ignore_nulls: bool = True):
        super().__init__(_label("sum", on), on, ignore_nulls, lambda k: None,
                         lambda a, v: v if a is None else a + v,
                         lambda a, b: b if a is None else (a if b is None else a + b))


class Min(_NullAware):
    def __init__(self, on=None, ignore_nulls: bool = True):
        super().__init__(_label("min", on), on, ignore_nulls, lambda k: None,
                         lambda a, v: v if a is None else min(a, v),
                         lambda a, b: b if a is None else (a if b is None else min(a, b)))


class Max(_NullAware):
    def __init__(self, on=None, ignore_nulls: bool = True):
        super().__init__(_label("max", on), on, ignore_nulls, lambda k: None,
                         lambda a, v: v if a is None else max(a, v),
                         lambda a, b: b if a is None else (a if b is None else max(a, b)))


class Mean(_NullAware):
    def __init__(self, on=None, ignore_nulls: bool = True):
        super().__init__(_label("mean", on), on, ignore_nulls, lambda k: (0, 0),
                         lambda a, v: (a[0] + v, a[1] + 1), lambda a, b: (a[0] + b[0], a[1] + b[1]),
                         lambda a: a[0] / a[1] if a[1] else None)


class Std(_NullAware):
    """Sample standard deviation (ddof=1) with Chan et al. parallel merge of (count, mean, M2)."""

    def __init__(self, on=None, ddof: int = 1, ignore_nulls: bool = True):
        def acc(a, v):
            n, mean, m2 = a
            n += 1
            d = v - mean
            mean += d / n
            return (n, mean, m2 + d * (v - mean))

        def merge(a, b):
            na, ma, sa = a
            nb, mb, sb = b
            n = na + nb
            if n == 0:
                return (0, 0.0, 0.0)
            d = mb - ma
            return (n, ma + d * nb / n, sa + sb + d * d * na * nb / n)

        def fin(a):
            n, _, m2 = a
            return math.sqrt(m2 / (n - ddof)) if n - ddof > 0 else None

        super().__init__(_label("std", on), on, ignore_nulls, lambda k: (0, 0.0, 0.0), acc, merge, fin)

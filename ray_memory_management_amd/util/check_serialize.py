"""inspect_serializability. Parity: reference python/ray/util/check_serialize.py: walk an object
(function closures and globals, object attributes) and report which members cloudpickle cannot
serialize, so a failing `@remote` definition or argument can be diagnosed."""
from __future__ import annotations

import inspect
from typing import Any, Optional, Set, Tuple

import cloudpickle


class FailureTuple:
    def __init__(self, obj: Any, name: str, parent: Any):
        self.obj, self.name, self.parent = obj, name, parent

    def __repr__(self):
        return f"FailTuple({self.name} [obj={self.obj!r}, parent={self.parent!r}])"

    def __eq__(self, other):
        return isinstance(other, FailureTuple) and (self.name, self.obj) == (other.name, other.obj)

    def __hash__(self):
        return hash(self.name)


def _ok(obj) -> bool:
    try:
        cloudpickle.dumps(obj)
        return True
    except Exception:
        return False


def _inspect(obj, name, parent, failures: Set[FailureTuple], depth: int, seen: set, printer):
    if id(obj) in seen or depth < 0:
        return
    seen.add(id(obj))
    if _ok(obj):
        return
    found_child = False
    children = []
    if inspect.isfunction(obj):
        cv = inspect.getclosurevars(obj)
        children = list(cv.globals.items()) + list(cv.nonlocals.items())
    elif hasattr(obj, "__dict__") and not inspect.isclass(obj):
        children = list(vars(obj).items())
    elif isinstance(obj, dict):
        children = [(str(k), v) for k, v in obj.items()]
    elif isinstance(obj, (list, tuple, set)):
        children = [(f"[{i}]", v) for i, v in enumerate(obj)]
    for cname, child in children:
        if not _ok(child):
            found_child = True
            printer(f"  {'  ' * (3 - depth)}{cname}: {type(child).__name__} is not serializable")
            _inspect(child, cname, obj, failures, depth - 1, seen, printer)
    if not found_child:
        failures.add(FailureTuple(obj, name, parent))


def inspect_serializability(base_obj: Any, name: Optional[str] = None, depth: int = 3, print_file=None,
                            _failure_set=None) -> Tuple[bool, Set[FailureTuple]]:
    """Returns (serializable, failures): the innermost members that cannot be pickled."""
    name = name or getattr(base_obj, "__name__", repr(base_obj))
    lines = []
    printer = lines.append
    if _ok(base_obj):
        return True, set()
    failures: Set[FailureTuple] = set() if _failure_set is None else _failure_set
    printer(f"Checking serializability of {name}: not serializable")
    _inspect(base_obj, name, None, failures, depth, set(), printer)
    if print_file is not None:
        print("\n".join(lines), file=print_file)
    return False, failures

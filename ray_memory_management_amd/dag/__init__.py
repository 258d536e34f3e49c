"""Lazy DAG API (``.bind()`` / ``InputNode`` / ``execute``). Parity: reference python/ray/dag/
(dag_node.py, function_node.py, class_node.py, input_node.py)."""
from __future__ import annotations

import uuid
from typing import Any, Dict, List


class DAGNode:
    def __init__(self, args=(), kwargs=None, options=None):
        self._bound_args = tuple(args)
        self._bound_kwargs = dict(kwargs or {})
        self._bound_options = dict(options or {})
        self._stable_uuid = uuid.uuid4().hex

    def get_args(self):
        return self._bound_args

    def get_kwargs(self):
        return self._bound_kwargs

    def get_options(self):
        return self._bound_options

    def _children(self) -> List["DAGNode"]:
        out = []

        def scan(v):
            if isinstance(v, DAGNode):
                out.append(v)
            elif isinstance(v, (list, tuple)):
                for x in v:
                    scan(x)
            elif isinstance(v, dict):
                for x in v.values():
                    scan(x)

        scan(self._bound_args)
        scan(self._bound_kwargs)
        return out

    def _resolve(self, v, cache, inp):
        if isinstance(v, DAGNode):
            return v._execute(cache, inp)
        if isinstance(v, list):
            return [self._resolve(x, cache, inp) for x in v]
        if isinstance(v, tuple):
            return tuple(self._resolve(x, cache, inp) for x in v)
        if isinstance(v, dict):
            return {k: self._resolve(x, cache, inp) for k, x in v.items()}
        return v

    def _execute(self, cache, inp):
        key = self._stable_uuid
        if key not in cache:
            args = self._resolve(self._bound_args, cache, inp)
            kwargs = self._resolve(self._bound_kwargs, cache, inp)
            cache[key] = self._execute_impl(args, kwargs, cache, inp)
        return cache[key]

    def _execute_impl(self, args, kwargs, cache, inp):
        raise NotImplementedError

    def execute(self, *args, **kwargs):
        return self._execute({}, (args, kwargs))

    def apply_recursive(self, fn):
        return fn(self)


class InputNode(DAGNode):
    def __init__(self):
        super().__init__()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def __getattr__(self, key):
        if key.startswith("_"):
            raise AttributeError(key)
        return InputAttributeNode(self, key)

    def __getitem__(self, key):
        return InputAttributeNode(self, key)

    def _execute(self, cache, inp):
        args, kwargs = inp
        if len(args) == 1 and not kwargs:
            return args[0]
        return _DAGInput(args, kwargs)


class _DAGInput:
    def __init__(self, args, kwargs):
        self.args = args
        self.kwargs = kwargs


class InputAttributeNode(DAGNode):
    def __init__(self, parent: InputNode, key):
        super().__init__()
        self._parent = parent
        self._key = key

    def _execute(self, cache, inp):
        args, kwargs = inp
        if isinstance(self._key, int):
            if len(args) == 1 and not kwargs and not isinstance(args[0], _DAGInput):
                return args[0][self._key]
            return args[self._key]
        if self._key in kwargs:
            return kwargs[self._key]
        v = args[0] if args else None
        if isinstance(v, dict):
            return v[self._key]
        return getattr(v, self._key)


class FunctionNode(DAGNode):
    def __init__(self, remote_fn, args, kwargs, options):
        super().__init__(args, kwargs, options)
        self._remote_fn = remote_fn

    def _execute_impl(self, args, kwargs, cache, inp):
        return self._remote_fn._remote(args, kwargs, self._bound_options)


class ClassNode(DAGNode):
    def __init__(self, actor_cls, args, kwargs, options):
        super().__init__(args, kwargs, options)
        self._actor_cls = actor_cls
        self._handle = None

    def _execute_impl(self, args, kwargs, cache, inp):
        if self._handle is None:
            self._handle = self._actor_cls._remote(args, kwargs, self._bound_options)
        return self._handle

    def __getattr__(self, item):
        if item.startswith("_"):
            raise AttributeError(item)
        node = self

        class _Bindable:
            def bind(self_inner, *a, **k):
                return ClassMethodNode(node, item, a, k, {})

            def options(self_inner, **o):
                class _B:
                    def bind(self2, *a, **k):
                        return ClassMethodNode(node, item, a, k, o)
                return _B()

        return _Bindable()


class ClassMethodNode(DAGNode):
    def __init__(self, target, method_name, args, kwargs, options):
        super().__init__(args, kwargs, options)
        self._target = target
        self._method = method_name

    def _children(self):
        c = super()._children()
        if isinstance(self._target, DAGNode):
            c.append(self._target)
        return c

    def _execute_impl(self, args, kwargs, cache, inp):
        handle = self._target._execute(cache, inp) if isinstance(self._target, DAGNode) else self._target
        m = getattr(handle, self._method)
        if self._bound_options:
            return m.options(**self._bound_options).remote(*args, **kwargs)
        return m.remote(*args, **kwargs)


class MultiOutputNode(DAGNode):
    def __init__(self, outputs):
        super().__init__(tuple(outputs))

    def _execute_impl(self, args, kwargs, cache, inp):
        return list(args)


# reference dag/constants.py keys (used when DAG nodes are serialized / introspected)
PARENT_CLASS_NODE_KEY = "parent_class_node"
PREV_CLASS_METHOD_CALL_KEY = "prev_class_method_call"
DAGNODE_TYPE_KEY = "__dag_node_type__"

DAGInputData = _DAGInput  # reference input_node.py DAGInputData: the (args, kwargs) an InputNode resolves to


def _label(node: DAGNode) -> str:
    for attr in ("_remote_fn", "_cls", "_method_name"):
        v = getattr(node, attr, None)
        if v is not None:
            name = getattr(v, "__name__", None) or getattr(getattr(v, "_function", None), "__name__", None) or str(v)
            return f"{type(node).__name__}\\n{name}"
    return type(node).__name__


def plot(dag: DAGNode, to_file: str = None) -> str:
    """Graphviz DOT text of the DAG (reference dag/vis_utils.py plot, which renders through pydot —
    not installed here — so the DOT source is returned and written to `to_file` when given)."""
    ids, lines, stack, seen = {}, ["digraph G {", "  rankdir=LR;"], [dag], set()
    while stack:
        n = stack.pop()
        if id(n) in seen:
            continue
        seen.add(id(n))
        ids.setdefault(id(n), f"n{len(ids)}")
        lines.append(f'  {ids[id(n)]} [label="{_label(n)}"];')
        children = list(n._children())
        parent = getattr(n, "_parent", None)
        if isinstance(parent, DAGNode):
            children.append(parent)
        for c in children:
            ids.setdefault(id(c), f"n{len(ids)}")
            lines.append(f"  {ids[id(c)]} -> {ids[id(n)]};")
            stack.append(c)
    lines.append("}")
    dot = "\n".join(lines)
    if to_file:
        with open(to_file if to_file.endswith(".dot") else to_file + ".dot", "w") as f:
            f.write(dot)
    return dot


__all__ = ["DAGInputData", "PARENT_CLASS_NODE_KEY", "PREV_CLASS_METHOD_CALL_KEY", "DAGNODE_TYPE_KEY", "plot",
           "DAGNode", "InputNode", "InputAttributeNode", "FunctionNode", "ClassNode", "ClassMethodNode",
           "MultiOutputNode"]

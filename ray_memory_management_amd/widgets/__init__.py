"""Notebook helpers. Parity: reference python/ray/widgets/{__init__.py, util.py} (Template rendering
of the HTML reprs and the `ensure_notebook_deps` decorator that falls back to the plain repr when
ipywidgets is missing — it is not installed in this image, so the fallback is what runs)."""
from __future__ import annotations

import functools
import html
import importlib.util
from typing import Callable, Dict


class Template:
    """Minimal `{{ key }}` HTML template (the reference ships .html.j2 files)."""

    def __init__(self, text: str):
        self.text = text

    def render(self, **kwargs) -> str:
        out = self.text
        for k, v in kwargs.items():
            out = out.replace("{{ " + k + " }}", str(v))
        return out


def make_table_html_repr(obj, title: str = "") -> str:
    rows = "".join(f"<tr><td>{html.escape(str(k))}</td><td>{html.escape(str(v))}</td></tr>"
                   for k, v in (vars(obj) if hasattr(obj, "__dict__") else {}).items())
    return f"<div><b>{html.escape(title)}</b><table>{rows}</table></div>"


def ensure_notebook_deps(*deps) -> Callable:
    """Decorator: run the wrapped `_ipython_display_`-style function only if every (module, version)
    dependency is importable, else fall back to `repr(self)`."""
    names = [d[0] if isinstance(d, (tuple, list)) else d for d in deps]

    def wrap(fn):
        @functools.wraps(fn)
        def inner(self, *a, **kw):
            if all(importlib.util.find_spec(n) is not None for n in names):
                return fn(self, *a, **kw)
            return repr(self)

        return inner

    return wrap


def widgets_available() -> bool:
    return importlib.util.find_spec("ipywidgets") is not None


_DISPLAY: Dict[str, str] = {}

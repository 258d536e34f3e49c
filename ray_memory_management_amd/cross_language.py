"""Cross-language descriptors. Parity: reference python/ray/cross_language.py (java_function,
java_actor_class, cpp_function) and the Language enum. This framework runs Python workers only —
there is no Java or C++ worker runtime on the MI355X stack — so the descriptors exist for API
compatibility and raise a clear error when they would need a foreign-language worker."""
from __future__ import annotations

import enum


class Language(enum.IntEnum):
    PYTHON = 0
    JAVA = 1
    CPP = 2


class _CrossLanguageDescriptor:
    def __init__(self, language: Language, name: str, kind: str):
        self.language, self.name, self.kind = language, name, kind

    def options(self, **_kw) -> "_CrossLanguageDescriptor":
        return self

    def remote(self, *args, **kwargs):
        raise NotImplementedError(f"{self.language.name} {self.kind} {self.name!r}: this framework has no "
                                  f"{self.language.name.title()} worker runtime (Python workers only)")

    def __repr__(self) -> str:
        return f"<{self.language.name} {self.kind} {self.name}>"


def java_function(class_name: str, function_name: str) -> _CrossLanguageDescriptor:
    return _CrossLanguageDescriptor(Language.JAVA, f"{class_name}.{function_name}", "function")


def java_actor_class(class_name: str) -> _CrossLanguageDescriptor:
    return _CrossLanguageDescriptor(Language.JAVA, class_name, "actor class")


def cpp_function(function_name: str) -> _CrossLanguageDescriptor:
    return _CrossLanguageDescriptor(Language.CPP, function_name, "function")

"""Parity: reference python/ray/tune/error.py."""


class TuneError(Exception):
    pass

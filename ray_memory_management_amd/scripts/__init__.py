"""CLI package. Parity: reference python/ray/scripts/."""

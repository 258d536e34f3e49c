"""Record layout of the sort benchmark (gensort / sortbenchmark.org format): 100-byte records whose
first 10 bytes are the key. Parity: reference python/ray/experimental/raysort/constants.py."""
RECORD_SIZE = 100  # bytes
KEY_SIZE = 10      # bytes; the first 8 form the partitioning prefix (big-endian u64)
PREFIX_SIZE = 8

INPUT_MANIFEST_FILE = "input-manifest.csv"
OUTPUT_MANIFEST_FILE = "output-manifest.csv"
DATA_DIR_NAME = "raysort-data"


def bytes_to_records(n_bytes: int) -> int:
    if n_bytes % RECORD_SIZE:
        raise ValueError(f"{n_bytes} bytes is not a whole number of {RECORD_SIZE}-byte records")
    return n_bytes // RECORD_SIZE


def merge_part_ids(reducer_id: int, mapper_round: int) -> int:
    """Id of the first-stage merge output of (reducer, mapper round)."""
    return reducer_id * 1_000_000 + mapper_round

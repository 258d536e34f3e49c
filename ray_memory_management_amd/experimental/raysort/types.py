"""Types of the sort benchmark (reference python/ray/experimental/raysort/types.py)."""
from typing import NamedTuple

ByteCount = int
RecordCount = int
PartId = int
Path = str


class PartInfo(NamedTuple):
    part_id: PartId
    node: str
    path: Path
    num_records: RecordCount = 0

    def __repr__(self):
        return f"Part({self.node}:{self.path})"


class BlockInfo(NamedTuple):
    offset: int
    size: int

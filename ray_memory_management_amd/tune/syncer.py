"""Experiment-directory syncing. Parity: reference python/ray/tune/syncer.py (SyncConfig:
upload_dir, syncer, sync_period, sync_on_checkpoint; the driver syncs the experiment directory to
``upload_dir`` periodically and at the end). Only local paths and ``file://`` URIs are supported
here (no network: cloud URIs raise)."""
from __future__ import annotations

import dataclasses
import os
import shutil
import time
from typing import Optional


@dataclasses.dataclass
class SyncConfig:
    upload_dir: Optional[str] = None
    syncer: Optional[str] = "auto"
    sync_period: float = 300.0
    sync_on_checkpoint: bool = True


def _local_target(uri: str) -> str:
    if uri.startswith("file://"):
        return uri[len("file://"):]
    if "://" in uri:
        raise ValueError(f"upload_dir {uri!r}: only local paths / file:// URIs are supported (no network)")
    return uri


class Syncer:
    """Copies the experiment directory to ``upload_dir/<experiment name>`` (incremental: only files
    that are new or changed since the last sync)."""

    def __init__(self, sync_config: SyncConfig, local_dir: str):
        self.cfg = sync_config
        self.local_dir = local_dir
        self.target = os.path.join(_local_target(sync_config.upload_dir), os.path.basename(local_dir.rstrip("/")))
        self.last_sync = 0.0
        self.num_syncs = 0

    def sync_up(self, force: bool = False) -> bool:
        if not force and time.time() - self.last_sync < self.cfg.sync_period:
            return False
        for root, _, files in os.walk(self.local_dir):
            rel = os.path.relpath(root, self.local_dir)
            dst_dir = os.path.join(self.target, rel) if rel != "." else self.target
            os.makedirs(dst_dir, exist_ok=True)
            for f in files:
                src, dst = os.path.join(root, f), os.path.join(dst_dir, f)
                try:
                    st = os.stat(src)
                    if os.path.exists(dst):
                        dt = os.stat(dst)
                        if dt.st_size == st.st_size and dt.st_mtime >= st.st_mtime:
                            continue
                    shutil.copy2(src, dst)
                except OSError:
                    pass
        self.last_sync = time.time()
        self.num_syncs += 1
        return True

"""Lineage retention and lost-object recovery for the head process.

Parity: reference ``src/ray/core_worker/object_recovery_manager.cc`` (RecoverObject → pin an
existing copy or resubmit the creating task, recursively recovering missing arguments) and the
lineage-pinning half of ``reference_count.cc`` (a task's spec is kept while any of its return
objects is in scope, or while a retained task that consumed one of its returns is kept).

Design here: the head sees every normal task finish, so it is the natural owner of lineage. It
records, per finished reconstructable task (``max_retries != 0``, static ``num_returns``), the spec
and the node its returns were sealed on. Objects are *lost* when

* the virtual node holding them is removed (``cluster_utils.Cluster.remove_node``; the shm store is
  machine-wide, so the head deletes that node's primary copies to reproduce what a real node loss
  does), or
* the process owning a GPU object dies (its HBM arena goes with it).

A lost object that is still referenced is deleted from the store and its creating task resubmitted
(arguments that are gone are recovered first, recursively). When lineage is missing or the retry
budget is spent, the object is replaced by an ``ObjectLostError``/``OwnerDiedError`` so a ``get``
raises instead of hanging. Lineage is bounded (``max_lineage_entries``, oldest evicted first).
"""
from __future__ import annotations

import collections
from typing import Dict, Iterable, List, Optional

from ray_memory_management_amd import exceptions as exc
from ray_memory_management_amd._private import serialization as ser
from ray_memory_management_amd._private.ids import object_id_for_return


class LineageRec:
    __slots__ = ("spec", "returns", "live", "dependents", "parents", "retries_left", "node")

    def __init__(self, spec: dict, returns: List[bytes], node):
        self.spec = spec
        self.returns = returns
        self.live = set(returns)
        self.dependents = 0
        self.parents: List[bytes] = []
        r = spec.get("max_retries", 3)
        self.retries_left = -1 if r is None or r < 0 else int(r)
        self.node = node


class ObjectRecoveryManager:
    def __init__(self, head, max_entries: int = 200_000):
        self.head = head
        self.max_entries = max_entries
        self.lineage: "collections.OrderedDict[bytes, LineageRec]" = collections.OrderedDict()
        self.obj_task: Dict[bytes, bytes] = {}       # return oid -> creating task id (while lineage kept)
        self.obj_node: Dict[bytes, int] = {}         # return oid -> node its primary copy lives on
        self.num_reconstructions = 0
        self.num_lost = 0
        # lost objects whose lineage may still be in flight: a directly submitted task's completion
        # record travels owner -> head separately from the worker's death, so a loss can arrive
        # first; oid -> (deadline, cause, owner_died), settled by task_finished or the deadline
        self.awaiting: Dict[bytes, tuple] = {}
        self.lineage_grace_s = 2.0

    # ------------------------------------------------------------------ recording
    @staticmethod
    def reconstructable(spec: dict) -> bool:
        nr = spec.get("num_returns", 1)
        return (isinstance(nr, int) and nr > 0 and spec.get("max_retries", 3) != 0
                and not spec.get("actor_id") and not spec.get("actor_creation"))

    @staticmethod
    def returns_of(spec: dict) -> List[bytes]:
        nr = spec.get("num_returns", 1)
        if not isinstance(nr, int):
            return []
        return [object_id_for_return(spec["task_id"], i) for i in range(1, nr + 1)]

    def task_finished(self, spec: dict, node) -> None:
        """Called when a normal task finished OK (returns sealed on ``node``)."""
        tid = spec["task_id"]
        rets = self.returns_of(spec)
        for oid in rets:
            self.obj_node[oid] = node
        if not self.reconstructable(spec):
            return
        old = self.lineage.get(tid)
        if old is not None:  # a reconstruction finished: keep the record (and its budget)
            old.node = node
            old.live = {o for o in rets if o in self.head.refcounts}
            return
        rec = LineageRec(spec, rets, node)
        rec.live = {o for o in rets if o in self.head.refcounts}
        late = [o for o in rets if o in self.awaiting]  # lost before this record arrived
        if not rec.live and not late:
            return  # nobody references the outputs any more: nothing to protect
        for r in spec.get("arg_refs", ()):
            ptid = self.obj_task.get(r)
            if ptid is not None and ptid in self.lineage and ptid not in rec.parents:
                self.lineage[ptid].dependents += 1
                rec.parents.append(ptid)
        self.lineage[tid] = rec
        for oid in rets:
            self.obj_task[oid] = tid
        while len(self.lineage) > self.max_entries:
            otid, orec = self.lineage.popitem(last=False)
            self._forget(otid, orec)
        for oid in late:
            _, cause, owner_died = self.awaiting.pop(oid)
            if not self.recover(oid):
                self._lost_error(oid, cause, owner_died)

    def expire_awaiting(self, now: float) -> None:
        """Lost objects whose lineage never arrived within the grace period fail (head housekeeping)."""
        for oid, (deadline, cause, owner_died) in list(self.awaiting.items()):
            if now >= deadline:
                del self.awaiting[oid]
                self._lost_error(oid, cause, owner_died)

    def _lost_error(self, oid: bytes, cause: str, owner_died: bool) -> None:
        err = (exc.OwnerDiedError if owner_died else exc.ObjectLostError)(
            oid.hex(), message=f"Object {oid.hex()} was lost ({cause}) and cannot be reconstructed "
                               "(no lineage, or the task's max_retries is exhausted).")
        self._store_error(oid, err)

    def object_freed(self, oid: bytes) -> None:
        self.obj_node.pop(oid, None)
        tid = self.obj_task.get(oid)
        if tid is None:
            return
        rec = self.lineage.get(tid)
        if rec is None:
            self.obj_task.pop(oid, None)
            return
        rec.live.discard(oid)
        self._maybe_drop(tid, rec)

    def _maybe_drop(self, tid: bytes, rec: LineageRec) -> None:
        stack = [(tid, rec)]
        while stack:
            t, r = stack.pop()
            if r.live or r.dependents > 0 or t not in self.lineage:
                continue
            del self.lineage[t]
            self._forget(t, r)
            for p in r.parents:
                pr = self.lineage.get(p)
                if pr is not None:
                    pr.dependents -= 1
                    stack.append((p, pr))

    def _forget(self, tid: bytes, rec: LineageRec) -> None:
        for oid in rec.returns:
            if self.obj_task.get(oid) == tid:
                del self.obj_task[oid]

    # ------------------------------------------------------------------ loss + recovery
    def node_removed(self, node_id) -> List[bytes]:
        lost = [o for o, n in self.obj_node.items() if n == node_id]
        return self.objects_lost(lost, f"node {node_id} was removed")

    def objects_lost(self, oids: Iterable[bytes], cause: str, owner_died: bool = False) -> List[bytes]:
        """Delete still-referenced lost copies and start recovery. Returns the oids handled."""
        head = self.head
        handled = []
        to_recover = []
        for oid in oids:
            self.obj_node.pop(oid, None)
            if oid not in head.refcounts:
                # unreferenced: just drop the copy
                try:
                    head.store.delete([oid])
                except Exception:
                    pass
                continue
            try:
                if head.store.contains(oid) and not head.store.delete([oid]):
                    continue  # pinned by a live reader: the copy is still usable on this machine
            except Exception:
                continue
            self.num_lost += 1
            handled.append(oid)
            to_recover.append(oid)
        for oid in to_recover:
            if self.recover(oid):
                continue
            if oid not in self.obj_task and self.lineage_grace_s > 0:
                import time

                self.awaiting[oid] = (time.time() + self.lineage_grace_s, cause, owner_died)
                continue
            self._lost_error(oid, cause, owner_died)
        return handled

    def recover(self, oid: bytes, _depth: int = 0) -> bool:
        """Make `oid` available again: already there, being recomputed, or resubmit its task."""
        head = self.head
        if head.store.contains(oid):
            return True
        tid = self.obj_task.get(oid)
        if tid is None:
            return False
        if tid in head.tasks:  # already pending/running (e.g. another return of the same task)
            return True
        rec = self.lineage.get(tid)
        if rec is None or rec.retries_left == 0 or _depth > 1000:
            return False
        if rec.retries_left > 0:
            rec.retries_left -= 1
        spec = dict(rec.spec)
        spec.pop("_key", None)
        spec.pop("_res", None)
        # pin the args first (so a recovered arg is not freed the moment it is sealed), then recover
        # any that are gone
        args = [r for r in spec.get("arg_refs", ())]
        missing = [r for r in args if not (r[:1] == b"\xaa" and r[-3:] == b"\xaa\xaa\xaa")
                   and not head.store.contains(r)]
        for r in missing:
            if not self.recover(r, _depth + 1):
                err = exc.ObjectReconstructionFailedError(
                    oid.hex(), message=f"Object {oid.hex()} cannot be reconstructed: its argument {r.hex()} is lost "
                               "and has no lineage.")
                for o in rec.returns:
                    if o in head.refcounts and not head.store.contains(o):
                        self._store_error(o, err)
                return True  # handled (error stored)
        self.num_reconstructions += 1
        head._resubmit(spec)
        return True

    def _store_error(self, oid: bytes, err: BaseException) -> None:
        data, bufs, _ = ser.serialize(err)
        try:
            if self.head.store.state(oid) == 1:
                self.head.store.abort(oid)
            if not self.head.store.contains(oid):
                self.head.store.put_serialized(oid, data, bufs, ser.TAG_ERROR, True)
        except Exception:
            pass

    def stats(self) -> dict:
        return {"lineage_entries": len(self.lineage), "tracked_objects": len(self.obj_node),
                "num_reconstructions": self.num_reconstructions, "num_lost": self.num_lost}

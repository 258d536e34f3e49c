"""ObjectRecoveryManager unit tests with a stub head: the lineage grace period for objects lost
before their (directly submitted) task's completion record reached the head."""
import pytest

from ray_memory_management_amd._private.object_recovery import ObjectRecoveryManager
from ray_memory_management_amd._private.ids import object_id_for_return


class _Store:
    def __init__(self):
        self.objs, self.errors = set(), {}

    def contains(self, oid):
        return oid in self.objs or oid in self.errors

    def delete(self, oids):
        for o in oids:
            self.objs.discard(o)
        return True

    def state(self, oid):
        return 0

    def abort(self, oid):
        pass

    def put_serialized(self, oid, data, bufs, tag, seal):
        self.errors[oid] = data


class _Head:
    def __init__(self):
        self.store = _Store()
        self.refcounts = {}
        self.tasks = {}
        self.resubmitted = []

    def _resubmit(self, spec):
        self.resubmitted.append(spec["task_id"])


def _spec(tid):
    return {"task_id": tid, "num_returns": 2, "max_retries": 2, "arg_refs": []}


@pytest.fixture
def setup():
    head = _Head()
    rec = ObjectRecoveryManager(head)
    tid = b"\x01" * 24
    rets = [object_id_for_return(tid, i) for i in (1, 2)]
    for o in rets:
        head.refcounts[o] = 1
        head.store.objs.add(o)
    return head, rec, tid, rets


def test_lost_then_lineage_arrives_reconstructs(setup):
    head, rec, tid, rets = setup
    rec.objects_lost([rets[1]], "the worker process owning them died", owner_died=True)
    assert rets[1] in rec.awaiting and not head.store.errors and not head.resubmitted
    rec.task_finished(_spec(tid), node=0)  # the completion record arrives after the loss
    assert head.resubmitted == [tid] and not rec.awaiting and not head.store.errors


def test_lost_without_lineage_fails_after_grace(setup):
    head, rec, tid, rets = setup
    rec.lineage_grace_s = 0.5
    rec.objects_lost([rets[1]], "the worker process owning them died", owner_died=True)
    rec.expire_awaiting(now=0.0)  # before the deadline: still waiting
    assert rets[1] in rec.awaiting and not head.store.errors
    import time

    rec.expire_awaiting(now=time.time() + 1.0)
    assert not rec.awaiting and rets[1] in head.store.errors and not head.resubmitted


def test_known_lineage_reconstructs_at_once(setup):
    head, rec, tid, rets = setup
    rec.task_finished(_spec(tid), node=0)
    rec.objects_lost([rets[0]], "node removed")
    assert head.resubmitted == [tid] and not rec.awaiting


def test_no_grace_fails_at_once(setup):
    head, rec, tid, rets = setup
    rec.lineage_grace_s = 0.0
    rec.objects_lost([rets[0]], "node removed")
    assert rets[0] in head.store.errors and not rec.awaiting

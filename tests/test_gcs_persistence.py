"""GCS fault tolerance with external storage: the head's tables survive a head restart.
Mirrors reference python/ray/tests/test_gcs_fault_tolerance.py (KV and detached actors available
after the GCS restarts with the same storage; the actor comes back with fresh state)."""
import time

import ray_memory_management_amd as ray
from ray_memory_management_amd import internal
from ray_memory_management_amd._private import worker as W


@ray.remote
class Keeper:
    def __init__(self, tag):
        self.tag = tag
        self.n = 0

    def bump(self):
        self.n += 1
        return self.tag, self.n


def test_kv_jobs_and_detached_actor_survive_head_restart(tmp_path):
    cfg = {"gcs_storage_path": str(tmp_path / "gcs"), "gcs_storage_flush_interval_ms": 10}
    ray.init(num_cpus=2, namespace="ft", _system_config=cfg)
    try:
        internal._internal_kv_put(b"model_version", b"7")
        a = Keeper.options(name="keeper", lifetime="detached").remote("hello")
        assert ray.get(a.bump.remote()) == ("hello", 1)
        assert ray.get(a.bump.remote()) == ("hello", 2)
        b = Keeper.options(name="temp").remote("x")  # not detached: dies with the job
        ray.get(b.bump.remote())
        time.sleep(0.2)
    finally:
        ray.shutdown()
    ray.init(num_cpus=2, namespace="ft", _system_config=cfg)
    try:
        assert internal._internal_kv_get(b"model_version") == b"7"
        h = ray.get_actor("keeper")
        assert ray.get(h.bump.remote(), timeout=60) == ("hello", 1)  # recreated: fresh state
        try:
            ray.get_actor("temp")
            raise AssertionError("non-detached actor must not be restored")
        except ValueError:
            pass
        st = W._state("gcs")
        assert st["restored"]["actors"] == 1 and st["restored"]["kv_namespaces"] >= 1
        assert st["restored"]["jobs"] >= 1
        jobs = ray.util.state.list_jobs()
        assert any(not j.get("alive") for j in jobs)  # the previous driver's job, from history
        ray.kill(h)
    finally:
        ray.shutdown()


def test_no_storage_no_snapshot(tmp_path):
    ray.init(num_cpus=1)
    try:
        assert W._state("gcs")["storage_path"] is None
    finally:
        ray.shutdown()


def test_killed_detached_actor_and_deleted_kv_stay_gone(tmp_path):
    cfg = {"gcs_storage_path": str(tmp_path / "gcs"), "gcs_storage_flush_interval_ms": 10}
    ray.init(num_cpus=2, namespace="ft2", _system_config=cfg)
    try:
        internal._internal_kv_put(b"a", b"1")
        internal._internal_kv_put(b"b", b"2")
        internal._internal_kv_del(b"a")
        k = Keeper.options(name="gone", lifetime="detached").remote("g")
        ray.get(k.bump.remote())
        ray.kill(k)
        keep = Keeper.options(name="kept", lifetime="detached").remote("k")
        ray.get(keep.bump.remote())
        time.sleep(0.2)
    finally:
        ray.shutdown()
    ray.init(num_cpus=2, namespace="ft2", _system_config=cfg)
    try:
        assert internal._internal_kv_get(b"a") is None and internal._internal_kv_get(b"b") == b"2"
        try:
            ray.get_actor("gone")
            raise AssertionError("a killed detached actor must not come back")
        except ValueError:
            pass
        h = ray.get_actor("kept")
        assert ray.get(h.bump.remote(), timeout=60) == ("k", 1)
        ray.kill(h)
    finally:
        ray.shutdown()


def test_corrupt_snapshot_is_ignored(tmp_path):
    d = tmp_path / "gcs"
    d.mkdir()
    for name in ("gcs_snapshot.json", "snapshot.json", "gcs.json"):
        (d / name).write_text("{not json")
    ray.init(num_cpus=1, _system_config={"gcs_storage_path": str(d)})
    try:
        assert ray.get(ray.put(3)) == 3  # the head starts with empty tables
        assert W._state("gcs")["storage_path"] == str(d)
    finally:
        ray.shutdown()

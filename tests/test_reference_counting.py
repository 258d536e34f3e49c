"""Distributed reference counting, ported from the reference's python/ray/tests/test_reference_counting.py.
Same workloads. "Pinned" is checked the way the reference checks it: fill the 100 MiB store with short-lived
objects, then ask the store whether the object still exists.

One difference in meaning: the reference evicts unpinned objects under LRU pressure, while here an object is
freed as soon as its last reference goes, so `succeed=False` holds even without the fill. The reference's
owner-died distinction also differs: references are accounted at the head, not by the owning worker, so a
crashed chain surfaces as the crash (WorkerCrashedError), not as OwnerDiedError. Both are RayError.
"""
import asyncio
import copy
import os
import time

import numpy as np
import pytest

import ray_memory_management_amd as ray
from ray_memory_management_amd._private import worker as _w

MB = 1 << 20


@pytest.fixture
def one_worker_100MiB():
    # reference fixture: 1 CPU, 100 MiB store, no spilling (so "still there" means pinned, not spilled)
    yield ray.init(num_cpus=1, object_store_memory=100 * MB,
                   _system_config={"task_retry_delay_ms": 0, "automatic_object_spilling_enabled": False})
    ray.shutdown()


@ray.remote(num_cpus=0)
class SignalActor:
    """reference ray._private.test_utils.SignalActor"""

    def __init__(self):
        self.ev = asyncio.Event()

    async def wait(self):
        await self.ev.wait()

    async def send(self):
        self.ev.set()


def _exists(oid: bytes) -> bool:
    return bool(_w.global_worker.store.contains(oid))


def _wait_for(cond, timeout=10.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if cond():
            return
        time.sleep(0.05)
    raise AssertionError("condition not met in time")


def _fill_object_store_and_get(oid: bytes, succeed=True, object_MiB=20, num_objects=5):
    for _ in range(num_objects):
        ray.put(np.zeros(object_MiB * MB, dtype=np.uint8))
    if succeed:
        _wait_for(lambda: _exists(oid))
    else:
        _wait_for(lambda: not _exists(oid))


def _put_object(obj, use_ray_put):
    """reference test_utils.put_object: a ray.put object, or the same value returned by a task."""
    if use_ray_put:
        return ray.put(obj)

    @ray.remote
    def make():
        return obj

    ref = make.remote()
    ray.get(ref)
    return ref


def _local_refs(ref):
    return _w.global_worker.local_refs.get(ref.binary(), 0)


def test_local_refcounts(one_worker_100MiB):
    r1 = ray.put(None)
    assert _local_refs(r1) == 1
    r1_copy = copy.copy(r1)
    assert _local_refs(r1) == 2
    key = r1.binary()
    del r1
    assert _local_refs(r1_copy) == 1
    del r1_copy
    assert _w.global_worker.local_refs.get(key, 0) == 0


def test_basic_pinning(one_worker_100MiB):
    @ray.remote
    def f(array):
        return np.sum(array)

    @ray.remote
    class Actor:
        def __init__(self):
            # a long-lived reference held by the actor: pinned while the actor is alive
            self.large_object = ray.put(np.zeros(25 * MB, dtype=np.uint8))

        def get_large_object(self):
            return ray.get(self.large_object)

    actor = Actor.remote()
    for _ in range(10):
        ray.get(f.remote(np.zeros(10 * MB, dtype=np.uint8)))
    assert ray.get(actor.get_large_object.remote()).nbytes == 25 * MB


def test_pending_task_dependency_pinning(one_worker_100MiB):
    @ray.remote
    def pending(input1, input2):
        return

    signal = SignalActor.remote()
    obj_ref = pending.remote(np.zeros(20 * MB, dtype=np.uint8), signal.wait.remote())
    for _ in range(2):
        ray.put(np.zeros(20 * MB, dtype=np.uint8))
    ray.get(signal.send.remote())
    ray.get(obj_ref)


def test_out_of_band_serialized_object_ref(one_worker_100MiB):
    import cloudpickle

    obj_ref = ray.put("hello")
    s = cloudpickle.dumps(obj_ref)  # pickled outside the runtime: the object must stay alive for it
    del obj_ref
    assert ray.get(cloudpickle.loads(s)) == "hello"


def test_captured_object_ref(one_worker_100MiB):
    captured_id = ray.put(np.zeros(10 * MB, dtype=np.uint8))

    @ray.remote
    def f(signal):
        ray.get(signal.wait.remote())
        ray.get(captured_id)  # noqa: F821

    signal = SignalActor.remote()
    obj_ref = f.remote(signal)
    cap = captured_id.binary()
    del f
    del captured_id
    ray.get(signal.send.remote())
    ray.get(obj_ref)  # the captured ref was still readable inside the task
    assert _exists(cap)  # captured by the pickled function: pinned though no local reference is left

    captured_id = ray.put(np.zeros(10 * MB, dtype=np.uint8))

    @ray.remote
    class Actor:
        def get(self, signal):
            ray.get(signal.wait.remote())
            return ray.get(captured_id).nbytes  # noqa: F821

    signal = SignalActor.remote()
    actor = Actor.remote()
    obj_ref = actor.get.remote(signal)
    del Actor
    del captured_id
    ray.get(signal.send.remote())
    assert ray.get(obj_ref) == 10 * MB


@pytest.mark.parametrize("use_ray_put,failure", [(False, False), (False, True), (True, False), (True, True)])
def test_basic_serialized_reference(one_worker_100MiB, use_ray_put, failure):
    """A task holds a serialized (nested) reference while pending; the object is freed once it finishes."""
    @ray.remote(max_retries=1)
    def pending(ref, dep):
        ray.get(ref[0])
        if failure:
            os._exit(0)

    array_oid = _put_object(np.zeros(20 * MB, dtype=np.uint8), use_ray_put)
    signal = SignalActor.remote()
    obj_ref = pending.remote([array_oid], signal.wait.remote())
    oid = array_oid.binary()
    del array_oid
    _fill_object_store_and_get(oid)
    ray.get(signal.send.remote())
    try:
        ray.get(obj_ref)
        assert not failure
    except ray.exceptions.WorkerCrashedError:
        assert failure
    _fill_object_store_and_get(oid, succeed=False)


@pytest.mark.parametrize("use_ray_put,failure", [(False, False), (False, True), (True, False), (True, True)])
def test_recursive_serialized_reference(one_worker_100MiB, use_ray_put, failure):
    """A chain of tasks passes a serialized reference to its tail; pinned until the tail finishes."""
    @ray.remote(max_retries=1)
    def recursive(ref, signal, max_depth, depth=0):
        ray.get(ref[0])
        if depth == max_depth:
            ray.get(signal.wait.remote())
            if failure:
                os._exit(0)
            return
        return recursive.remote(ref, signal, max_depth, depth + 1)

    signal = SignalActor.remote()
    max_depth = 5
    array_oid = _put_object(np.zeros(20 * MB, dtype=np.uint8), use_ray_put)
    head_oid = recursive.remote([array_oid], signal, max_depth)
    oid = array_oid.binary()
    del array_oid
    tail_oid = head_oid
    for _ in range(max_depth):
        tail_oid = ray.get(tail_oid)
    _fill_object_store_and_get(oid)
    ray.get(signal.send.remote())
    try:
        assert ray.get(tail_oid) is None
        assert not failure
    except ray.exceptions.RayError:
        assert failure
    _fill_object_store_and_get(oid, succeed=False)


@pytest.mark.parametrize("use_ray_put,failure", [(False, False), (False, True), (True, False), (True, True)])
def test_actor_holding_serialized_reference(one_worker_100MiB, use_ray_put, failure):
    @ray.remote
    class GreedyActor:
        def set_ref1(self, ref):
            self.ref1 = ref

        def add_ref2(self, new_ref):
            self.ref2 = new_ref

        def delete_ref1(self):
            self.ref1 = None

        def delete_ref2(self):
            self.ref2 = None

    array_oid = _put_object(np.zeros(20 * MB, dtype=np.uint8), use_ray_put)
    actor = GreedyActor.remote()
    actor.set_ref1.remote([array_oid])
    ray.get(actor.add_ref2.remote([array_oid]))  # a duplicate reference to the same object
    oid = array_oid.binary()
    del array_oid
    _fill_object_store_and_get(oid)
    ray.get(actor.delete_ref1.remote())  # removing one of the two keeps it pinned
    _fill_object_store_and_get(oid)
    if failure:
        ray.kill(actor)  # the actor exiting releases what it held
        with pytest.raises(ray.exceptions.RayActorError):
            ray.get(actor.delete_ref1.remote(), timeout=10)
    else:
        ray.get(actor.delete_ref2.remote())
    _fill_object_store_and_get(oid, succeed=False)


@pytest.mark.parametrize("use_ray_put,failure", [(False, False), (False, True), (True, False), (True, True)])
def test_worker_holding_serialized_reference(one_worker_100MiB, use_ray_put, failure):
    @ray.remote(max_retries=1)
    def child(dep1, dep2):
        if failure:
            os._exit(0)
        return

    @ray.remote
    class Submitter:
        def launch_pending_task(self, ref, signal):
            return child.remote(ref[0], signal.wait.remote())

    signal = SignalActor.remote()
    array_oid = _put_object(np.zeros(20 * MB, dtype=np.uint8), use_ray_put)
    s = Submitter.remote()
    child_return_id = ray.get(s.launch_pending_task.remote([array_oid], signal))
    oid = array_oid.binary()
    del array_oid
    _fill_object_store_and_get(oid)
    ray.get(signal.send.remote())
    try:
        ray.get(child_return_id)
        assert not failure
    except ray.exceptions.WorkerCrashedError:
        assert failure
    del child_return_id
    _fill_object_store_and_get(oid, succeed=False)


def test_basic_nested_ids(one_worker_100MiB):
    inner_oid = ray.put(np.zeros(20 * MB, dtype=np.uint8))
    outer_oid = ray.put([inner_oid])
    oid = inner_oid.binary()
    del inner_oid
    _fill_object_store_and_get(oid)  # the outer object pins the inner one
    del outer_oid
    _fill_object_store_and_get(oid, succeed=False)


def _all_actors_dead():
    from ray_memory_management_amd.util import state

    return all(a["state"] == "DEAD" for a in state.list_actors())


def test_kill_actor_immediately_after_creation(one_worker_100MiB):
    @ray.remote
    class A:
        pass

    a, b = A.remote(), A.remote()
    ray.kill(a)
    ray.kill(b)
    _wait_for(_all_actors_dead)


def test_remove_actor_immediately_after_creation(one_worker_100MiB):
    @ray.remote
    class A:
        pass

    a, b = A.remote(), A.remote()
    del a
    del b
    _wait_for(_all_actors_dead)


def test_actor_constructor_borrow_cancellation(one_worker_100MiB):
    """A reference borrowed by an actor constructor is freed when the never-scheduled actor goes out of
    scope (reference :559)."""
    @ray.remote(resources={"nonexistent_resource": 1})
    class Actor:
        def __init__(self, obj_containing_ref):
            raise ValueError("the constructor must not run")

    def implicit_cancel():
        ref = ray.put(np.zeros(MB, dtype=np.uint8))
        Actor.remote({"foo": ref})
        return ref.binary()

    oid = implicit_cancel()
    _wait_for(lambda: not _exists(oid))


def test_out_of_band_actor_handle_deserialization(one_worker_100MiB):
    """Reference test_reference_counting_2.py:709: a deepcopy (pickle round trip) of a handle inside a task."""
    @ray.remote
    class Actor:
        def ping(self):
            return 1

    actor = Actor.remote()

    @ray.remote
    def func(config):
        config = copy.deepcopy(config)
        return ray.get(config["actor"].ping.remote())

    assert ray.get(func.remote({"actor": actor})) == 1


def test_out_of_band_actor_handle_bypass_reference_counting(one_worker_100MiB):
    """Reference test_reference_counting_2.py:728: a handle pickled out of band does not keep the actor alive."""
    import pickle

    @ray.remote
    class Actor:
        def ping(self):
            return 1

    actor = Actor.remote()
    ray.get(actor.ping.remote())
    serialized = pickle.dumps({"actor": actor})
    del actor
    _wait_for(_all_actors_dead)
    config = pickle.loads(serialized)
    with pytest.raises(ray.exceptions.RayActorError):
        ray.get(config["actor"].ping.remote(), timeout=10)


# ---------------------------------------------------------------------------------------------------------
# reference python/ray/tests/test_reference_counting_2.py

@pytest.mark.parametrize("use_ray_put,failure", [(False, False), (False, True), (True, False), (True, True)])
def test_recursively_nest_ids(one_worker_100MiB, use_ray_put, failure):
    """:66 An object containing refs pins the inner ids recursively, also for submitted tasks."""
    @ray.remote(max_retries=1)
    def recursive(ref, signal, max_depth, depth=0):
        unwrapped = ray.get(ref[0])
        if depth == max_depth:
            ray.get(signal.wait.remote())
            if failure:
                os._exit(0)
            return
        return recursive.remote(unwrapped, signal, max_depth, depth + 1)

    signal = SignalActor.remote()
    max_depth = 5
    array_oid = _put_object(np.zeros(20 * MB, dtype=np.uint8), use_ray_put)
    nested_oid = array_oid
    for _ in range(max_depth):
        nested_oid = ray.put([nested_oid])
    head_oid = recursive.remote([nested_oid], signal, max_depth)
    oid = array_oid.binary()
    del array_oid, nested_oid
    tail_oid = head_oid
    for _ in range(max_depth):
        tail_oid = ray.get(tail_oid)
    _fill_object_store_and_get(oid)
    ray.get(signal.send.remote())
    if not failure:
        ray.get(tail_oid)
    else:
        with pytest.raises(ray.exceptions.RayError):  # reference: OwnerDiedError (see the module doc)
            ray.get(tail_oid)
    _fill_object_store_and_get(oid, succeed=False)


@pytest.mark.parametrize("use_ray_put,failure", [(False, False), (False, True), (True, False), (True, True)])
def test_return_object_ref(one_worker_100MiB, use_ray_put, failure):
    """:120 A ref returned inside a task's result stays pinned while the caller holds it."""
    @ray.remote
    def return_an_id():
        return [_put_object(np.zeros(20 * MB, dtype=np.uint8), use_ray_put)]

    @ray.remote(max_retries=1)
    def exit():
        os._exit(0)

    outer_oid = return_an_id.remote()
    inner_bytes = ray.get(outer_oid)[0].binary()
    inner_oid = ray.get(outer_oid)[0]
    del outer_oid
    _fill_object_store_and_get(inner_bytes)
    if failure:
        # the reference frees it when its owner (the worker) dies; here the driver's reference keeps it, so
        # the worker crash is checked and then the reference is dropped
        with pytest.raises(ray.exceptions.WorkerCrashedError):
            ray.get(exit.remote())
        _fill_object_store_and_get(inner_bytes)
    del inner_oid
    _fill_object_store_and_get(inner_bytes, succeed=False)


@pytest.mark.parametrize("use_ray_put,failure", [(False, False), (False, True), (True, False), (True, True)])
def test_pass_returned_object_ref(one_worker_100MiB, use_ray_put, failure):
    """:155 A returned ref passed on to another task is pinned by that task until it finishes."""
    @ray.remote
    def return_an_id():
        return [_put_object(np.zeros(20 * MB, dtype=np.uint8), use_ray_put)]

    @ray.remote(max_retries=0)
    def pending(ref, signal):
        ray.get(signal.wait.remote())
        ray.get(ref[0])
        if failure:
            os._exit(0)

    signal = SignalActor.remote()
    outer_oid = return_an_id.remote()
    inner_bytes = ray.get(outer_oid)[0].binary()
    pending_oid = pending.remote([outer_oid], signal)
    del outer_oid
    ray.get(signal.send.remote())
    try:
        ray.get(pending_oid)
        assert not failure
    except ray.exceptions.WorkerCrashedError:
        assert failure
    _wait_for(lambda: not _exists(inner_bytes))


@pytest.mark.parametrize("use_ray_put,failure", [(False, False), (False, True), (True, False), (True, True)])
def test_recursively_pass_returned_object_ref(one_worker_100MiB, use_ray_put, failure):
    """:201 A returned ref passed down a chain of tasks that each return it again."""
    @ray.remote
    def return_an_id():
        return _put_object(np.zeros(20 * MB, dtype=np.uint8), use_ray_put)

    @ray.remote(max_retries=1)
    def recursive(ref, signal, max_depth, depth=0):
        inner_id = ray.get(ref[0])
        if depth == max_depth:
            ray.get(signal.wait.remote())
            if failure:
                os._exit(0)
            return inner_id
        return inner_id, recursive.remote(ref, signal, max_depth, depth + 1)

    max_depth = 5
    outer_oid = return_an_id.remote()
    signal = SignalActor.remote()
    head_oid = recursive.remote([outer_oid], signal, max_depth)
    inner_oid = None
    outer_oid = head_oid
    for _ in range(max_depth):
        inner_oid, outer_oid = ray.get(outer_oid)
    _fill_object_store_and_get(outer_oid.binary(), succeed=False)  # the tail has not returned yet
    ray.get(signal.send.remote())
    try:
        ray.get(outer_oid)
        _fill_object_store_and_get(inner_oid.binary())
        assert not failure
    except ray.exceptions.RayError:
        assert failure
    inner_bytes = inner_oid.binary()
    del inner_oid, head_oid, outer_oid
    _fill_object_store_and_get(inner_bytes, succeed=False)


@pytest.mark.parametrize("use_ray_put", [False, True])
def test_recursively_return_borrowed_object_ref(one_worker_100MiB, use_ray_put):
    """:264 (the failure variant kills the owner to get OwnerDiedError; references are accounted at the head
    here, so the driver's reference keeps the object instead)."""
    @ray.remote
    def recursive(num_tasks_left):
        if num_tasks_left == 0:
            return _put_object(np.zeros(20 * MB, dtype=np.uint8), use_ray_put), os.getpid()
        return ray.get(recursive.remote(num_tasks_left - 1))

    head_oid = recursive.remote(5)
    final_oid, _ = ray.get(head_oid)
    final_bytes = final_oid.binary()
    _fill_object_store_and_get(final_bytes)
    _fill_object_store_and_get(final_bytes)
    del head_oid
    del final_oid
    _fill_object_store_and_get(final_bytes, succeed=False)


def test_borrowed_id(one_worker_100MiB):
    """:304 (no-failure case) a ref handed from one actor to another stays usable by the borrower."""
    @ray.remote
    class Parent:
        def pass_ref(self, ref, borrower):
            self.ref = ref[0]
            ray.get(borrower.receive_ref.remote(ref))

    @ray.remote
    class Borrower:
        def __init__(self):
            self.ref = None

        def receive_ref(self, ref):
            self.ref = ref[0]

        def resolve_ref(self):
            return ray.get(self.ref).nbytes

        def ping(self):
            return

    parent = Parent.remote()
    borrower = Borrower.remote()
    ray.get(borrower.ping.remote())
    obj = ray.put(np.zeros(20 * MB, dtype=np.uint8))
    ray.get(parent.pass_ref.remote([obj], borrower))
    obj_bytes = obj.binary()
    del obj
    _fill_object_store_and_get(obj_bytes)
    assert ray.get(borrower.resolve_ref.remote()) == 20 * MB


def test_inlined_nested_refs(one_worker_100MiB):
    """:554 (single node) a ref created by an actor, returned through a task, passed to another task."""
    @ray.remote
    class Actor:
        def nested(self):
            return ray.put("x")

    @ray.remote
    def nested_nested(a):
        return a.nested.remote()

    @ray.remote
    def foo(ref):
        time.sleep(0.5)
        return ray.get(ref)

    a = Actor.remote()
    nested_nested_ref = nested_nested.remote(a)
    nested_ref = ray.get(nested_nested_ref)
    del nested_nested_ref
    x = foo.remote(nested_ref)
    del nested_ref
    assert ray.get(x) == "x"


def test_return_nested_ids(one_worker_100MiB):
    """:594 (ray issue 17553) refs nested in a returned object survive being echoed through a closure."""
    class Nested:
        def __init__(self, blocks):
            self._blocks = blocks

    @ray.remote
    def echo(fn):
        return fn()

    @ray.remote
    def create_nested():
        return Nested([ray.put(np.random.random(MB // 8)) for _ in range(10)])

    @ray.remote
    def test():
        ref = create_nested.remote()
        result1 = ray.get(ref)
        del ref
        result = echo.remote(lambda: result1)  # noqa: B023
        del result1
        time.sleep(1)
        return ray.get(ray.get(result)._blocks[0]).shape

    assert ray.get(test.remote()) == (MB // 8,)


def test_actor_constructor_borrowed_refs(one_worker_100MiB):
    """:631 the actor's constructor is the only holder of a ref."""
    @ray.remote(num_cpus=0)
    class Borrower:
        def __init__(self, borrowed_refs):
            self.borrowed_refs = borrowed_refs

        def test(self):
            return len(ray.get(self.borrowed_refs))

    ref = ray.put(np.random.random(MB // 8))
    b = Borrower.remote([ref])
    del ref
    for _ in range(3):
        assert ray.get(b.test.remote()) == 1
        time.sleep(0.3)


def test_deep_nested_refs(one_worker_100MiB):
    """:653 a chain of 200 tasks each returning the next one's ref."""
    @ray.remote
    def f(x):
        if x > 200:
            return x
        return f.remote(x + 1)

    r = f.remote(1)
    while isinstance(r, ray.ObjectRef):
        r = ray.get(r)
    assert r == 201


def test_forward_nested_ref(one_worker_100MiB):
    """:672 a ref to a ref, forwarded by a task to an actor that keeps the inner one."""
    @ray.remote
    def nested_ref():
        return ray.put(1)

    @ray.remote
    def nested_nested_ref():
        return nested_ref.remote()

    @ray.remote(num_cpus=0)
    class Borrower:
        def pass_ref(self, middle_ref):
            self.inner_ref = ray.get(middle_ref)

        def check_ref(self):
            return ray.get(self.inner_ref)

    @ray.remote
    def pass_nested_ref(borrower, outer_ref):
        ray.get(borrower.pass_ref.remote(outer_ref[0]))

    b = Borrower.remote()
    outer_ref = nested_nested_ref.remote()
    x = pass_nested_ref.remote(b, [outer_ref])
    del outer_ref
    ray.get(x)
    for _ in range(3):
        assert ray.get(b.check_ref.remote()) == 1
        time.sleep(0.3)

"""joblib backend. Parity: reference python/ray/util/joblib/{__init__.py (register_ray),
ray_backend.py (RayBackend: joblib's MultiprocessingBackend driving ray.util.multiprocessing.Pool,
n_jobs=-1 → every CPU in the cluster)}.

Usage::

    from ray_memory_management_amd.util.joblib import register_ray
    register_ray()
    with joblib.parallel_backend("ray"):
        joblib.Parallel(n_jobs=4)(joblib.delayed(f)(i) for i in range(100))
"""
from __future__ import annotations


def register_ray():
    """Register the "ray" joblib backend (joblib must be importable)."""
    try:
        from joblib.parallel import register_parallel_backend
    except ImportError as e:  # pragma: no cover
        raise ImportError("To use the ray backend you must install joblib") from e
    register_parallel_backend("ray", _backend_class())


def _backend_class():
    from joblib._parallel_backends import MultiprocessingBackend

    from ray_memory_management_amd.util.multiprocessing import Pool

    class RayBackend(MultiprocessingBackend):
        supports_sharedmem = False

        def __init__(self, nesting_level=None, inner_max_num_threads=None, ray_remote_args=None, **kw):
            super().__init__(nesting_level=nesting_level, inner_max_num_threads=inner_max_num_threads, **kw)
            self.ray_remote_args = ray_remote_args

        def effective_n_jobs(self, n_jobs):
            import ray_memory_management_amd as ray

            if not ray.is_initialized():
                ray.init()
            if n_jobs is None:
                n_jobs = 1
            if n_jobs < 0:
                return max(1, int(ray.cluster_resources().get("CPU", 1)) + 1 + n_jobs)
            return max(1, int(n_jobs))

        def configure(self, n_jobs=1, parallel=None, prefer=None, require=None, **memmapping_args):
            n_jobs = self.effective_n_jobs(n_jobs)
            self._pool = Pool(processes=n_jobs, ray_remote_args=self.ray_remote_args)
            self.parallel = parallel
            return n_jobs

        def terminate(self):
            pool = getattr(self, "_pool", None)
            if pool is not None:
                pool.terminate()
                self._pool = None

    return RayBackend


__all__ = ["register_ray"]

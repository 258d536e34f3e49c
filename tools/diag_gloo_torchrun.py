"""Diagnostic: util.collective gloo all-reduce latency between two actors, launched directly or as
rank 0 of torchrun (the other ranks wait at a barrier). Prints one JSON line per tensor kind."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")
    if rank == 0:
        for k in [k for k in os.environ if k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")
                  or k.startswith("TORCHELASTIC_")]:
            os.environ.pop(k)
        import ray_memory_management_amd as ray
        from ray_memory_management_amd.util import collective as col

        ray.init(num_cpus=4, num_gpus=1)

        @ray.remote(num_cpus=1, num_gpus=0.5)
        class A:
            def _collective_init(self, w, r, b, g):
                col.init_collective_group(w, r, b, g)
                return True

            def bench(self, device, n, iters):
                import torch

                t = torch.ones(n, dtype=torch.bfloat16, device=device)
                col.allreduce(t, "g")
                if device == "cuda":
                    torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(iters):
                    col.allreduce(t, "g")
                if device == "cuda":
                    torch.cuda.synchronize()
                return (time.perf_counter() - t0) / iters * 1e3

        acts = [A.remote() for _ in range(2)]
        col.create_collective_group(acts, 2, [0, 1], backend="gloo", group_name="g")
        for dev in ("cpu", "cuda"):
            ms = ray.get([a.bench.remote(dev, 1 << 20, 50) for a in acts])
            print(json.dumps({"launch": "torchrun" if world > 1 else "direct", "device": dev,
                              "allreduce_ms_2MB": [round(x, 3) for x in ms]}), flush=True)
        ray.shutdown()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

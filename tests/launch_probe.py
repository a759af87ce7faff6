"""A tiny `--gpus N` script for tests/test_bench_cpu.py: the same launcher call as bench.py, then a
gloo all-reduce over the ranks it started (CPU only).  argv: gpus [failing_rank]."""
import json
import os
import sys
from datetime import timedelta

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from image_recommender_amd.launch import maybe_spawn
    gpus = int(sys.argv[1])
    fail_rank = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    maybe_spawn(gpus, os.path.abspath(__file__), sys.argv[1:], require_gpu=False,
                visible=int(os.environ.get("PROBE_VISIBLE", "0")))
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        dist.init_process_group("gloo", timeout=timedelta(seconds=60))
    rank = int(os.environ.get("RANK", "0"))
    if rank == fail_rank:
        sys.exit(3)
    t = torch.tensor([rank + 1.0])
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"world_size": world, "sum": float(t.item())}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

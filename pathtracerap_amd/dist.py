"""Sample-sharded multi-GPU rendering (one process per GPU, RCCL over xGMI).

A ray's RNG seed depends on its slot in the globally compacted ray pool of
its iteration, so pixels cannot be split without changing the samples; whole
iterations can.  Each rank renders a contiguous iteration range into its
own float3 accumulator and one all-reduce (sum) combines them.  The
all-reduce runs whenever a process group exists, at world size 1 too, so a
one-rank RCCL group exercises the same ordering (the collective on the torch
stream after the renderer's launches) as the 8-GPU run.
"""
from __future__ import annotations

from typing import Callable, Optional


def shard_iterations(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced split of iterations [0, total): (first, count)."""
    if world <= 0 or not (0 <= rank < world) or total < 0:
        raise ValueError("bad shard arguments")
    base, extra = divmod(total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def render_sharded(scene, cfg, total_iters: int, device=None,
                   render_fn: Optional[Callable] = None):
    """Render ``total_iters`` samples per pixel across the process group and
    return the summed accumulator (a (W*H*3,) float32 tensor on every rank).

    ``render_fn(first, n, image_tensor)`` may replace the GPU renderer (used
    by the CPU tests with the oracle); by default the gfx950 Renderer renders
    straight into ``image_tensor`` on the current stream.
    """
    import torch
    import torch.distributed as dist

    grouped = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size() if grouped else 1
    rank = dist.get_rank() if grouped else 0
    first, n = shard_iterations(total_iters, rank, world)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if render_fn is None else torch.device("cpu")
    image = torch.zeros(cfg.width * cfg.height * 3, dtype=torch.float32, device=device)
    if render_fn is not None:
        render_fn(first, n, image)
    else:
        from . import Renderer
        r = Renderer(cfg)
        r.set_stream(torch.cuda.current_stream(device).cuda_stream)
        r.bind_image(image.data_ptr(), keepalive=image)
        r.allocateOnGPU(scene)
        r.renderLoop(first_iter=first, n_iters=n, sync=False)
    if grouped:
        dist.all_reduce(image, op=dist.ReduceOp.SUM)      # RCCL (nccl backend) over xGMI, or gloo
    if render_fn is None:
        torch.cuda.synchronize(device)
        r.free()
    return image

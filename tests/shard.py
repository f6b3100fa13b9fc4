"""Test helper: host-side mirror of the library's multi-GPU partitioning of a frame.

Every (pixel, sample) is independent (main.cpp:557-588) and the RNG is keyed by the GLOBAL sample
index, so a frame shards by sample range with no data-path exchange.  The library
(render.hip `shard_range`, used by mcpt_render_opts.devices and .comm) gives shard k of n of the job
[begin, end) the samples [begin + len*k//n, begin + len*(k+1)//n); `sample_range` is the same
formula, for callers that shard by hand (e.g. host copies summed over gloo in the tests).
"""


def sample_range(rank, world_size, spp, begin=0):
    """Contiguous, balanced split of [begin, begin + spp) -- rank gets [a, b)."""
    if not (0 <= rank < world_size) or spp < 0:
        raise ValueError("bad rank/world/spp")
    return begin + rank * spp // world_size, begin + (rank + 1) * spp // world_size


def reduce_framebuffers(fb, dist, dst=0):
    """Sum per-rank framebuffers onto `dst` with torch.distributed (host copies over gloo).  The GPU
    path does this inside the library with RCCL (mcpt_render_opts.comm)."""
    dist.reduce(fb, dst=dst, op=dist.ReduceOp.SUM)
    return fb

"""Multi-GPU partitioning of a frame.

Every (pixel, sample) is independent and the RNG is keyed by the GLOBAL sample index, so a frame
shards by sample range with no data-path exchange: rank r renders samples
[r*spp/G, (r+1)*spp/G) of every pixel into its own fp64 framebuffer, and ONE reduce (sum) over
RCCL combines them.  The image is independent of G up to fp64 summation order.
"""


def sample_range(rank, world_size, spp):
    """Contiguous, balanced split of [0, spp) -- rank gets [begin, end)."""
    if not (0 <= rank < world_size) or spp < 0:
        raise ValueError("bad rank/world/spp")
    return rank * spp // world_size, (rank + 1) * spp // world_size


def reduce_framebuffers(fb, dist, dst=0):
    """Sum per-rank framebuffers onto `dst` (torch tensor, any backend: gloo on CPU, nccl=RCCL on GPU)."""
    dist.reduce(fb, dst=dst, op=dist.ReduceOp.SUM)
    return fb

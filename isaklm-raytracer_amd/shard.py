"""spp-slice sharding of one frame across GPUs.

Rank r of N renders its own slice of the passes for every pixel, seeded with
the mt19937 outputs [r*W*H, (r+1)*W*H) — a continuation of the reference's
G_Buffer seeding (rt/screen.cuh:34-45), so rank 0 alone reproduces the
single-GPU reference stream.  The slices meet in ONE reduce (sum) of the
accumulators into rank 0 before the tonemap; over torch.distributed's "nccl"
backend that is an RCCL reduce over xGMI.  No other data-path collective.
"""


def seed_skip(rank, width, height):
    return rank * width * height


def pass_slice(rank, world, total_passes):
    """[begin, end) of the passes rank renders when a job of total_passes is split."""
    return rank * total_passes // world, (rank + 1) * total_passes // world


def reduce_to_root(dist, fb, sq, count, root=0):
    """Sum the frame accumulators (fb f32x3, sq f32, count i32) into `root`."""
    dist.reduce(fb, root)
    dist.reduce(sq, root)
    dist.reduce(count, root)

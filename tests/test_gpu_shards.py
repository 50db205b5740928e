"""Multi-GPU building blocks on one GPU: row-interleaved shards
are bit-identical to the one-GPU frame (adaptive sampling included) and sum
to it; the RCCL reduce of the C-ABI (rt_reduce_shards) on a 1-rank
communicator.  The 2-rank reduce itself is covered by the gloo test
(tests/test_distributed.py) and by the driver's 8-GPU bench."""
import numpy as np
import pytest

import helpers
import rt

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kernel", [rt.KERNEL_MEGA, rt.KERNEL_WAVEFRONT], ids=["mega", "wavefront"])
@pytest.mark.parametrize("adaptive", [False, True], ids=["fixed", "adaptive"])
def test_row_shards_sum_to_full_frame(kernel, adaptive):
    run = helpers.GpuRun("cornell")
    W, H, P, N = 37, 23, 12, 3
    kw = dict(adaptive=adaptive, min_samples=4, kernel=kernel)
    full, _, _ = run.render(W, H, P, calls=2, **kw)
    parts = [run.render(W, H, P, calls=2, shard_id=g, num_shards=N, **kw)[0] for g in range(N)]
    rows = np.arange(W * H) // W
    for g, (fb, sq, cnt, rng) in enumerate(parts):
        own = rows % N == g
        helpers.assert_bitwise((fb[own], sq[own], cnt[own], rng[own]),
                               (full[0][own], full[1][own], full[2][own], full[3][own]), what=f"shard {g}")
        assert not fb[~own].any() and not sq[~own].any() and not cnt[~own].any()  # untouched (zero) rows
    fb = sum(p[0] for p in parts)
    sq = sum(p[1] for p in parts)
    cnt = sum(p[2] for p in parts)
    assert np.array_equal(fb.view(np.uint32), full[0].view(np.uint32))
    assert np.array_equal(sq.view(np.uint32), full[1].view(np.uint32))
    assert np.array_equal(cnt, full[2])


def test_bad_shard_id_rejected():
    run = helpers.GpuRun("cornell")
    with pytest.raises(rt.RtError):
        run.render(8, 8, 1, shard_id=3, num_shards=3)


def test_rccl_reduce_one_rank_is_identity():
    run = helpers.GpuRun("cornell")
    W, H = 24, 16
    before, _, g = run.render(W, H, 3)
    comm = rt.Comm(1, 0, rt.Comm.unique_id())
    try:
        comm.reduce(g.g, W, H, 0)
    finally:
        comm.close()
    after = g.download()
    helpers.assert_bitwise(after, before, what="1-rank reduce")

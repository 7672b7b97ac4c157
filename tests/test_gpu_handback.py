"""The numpy hand-back of samples_ (device.to_host_many: pinned 64 MiB ring, DMA of one chunk
while the host threads copy out the one before): byte-identical to a plain copy for every
dtype the graph produces, sizes below, at and across chunk boundaries, and through the public
Node.sample(), which leaves numpy samples_ on every node as the reference does
(modeling.py:582-583, 614)."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_to_host_many_matches_plain_copies(gpu):
    import torch

    from probabilit_amd import device

    dev = device.device()
    chunk = device._STAGE_BYTES
    g = torch.Generator(device=dev).manual_seed(3)
    ts = [torch.randn(chunk // 8 * 3 + 12345, dtype=torch.float64, device=dev, generator=g),  # 3+ chunks
          torch.randint(-2**31, 2**31 - 1, (chunk // 4,), dtype=torch.int32, device=dev, generator=g),  # exactly 1
          torch.randint(-2**40, 2**40, (5_000_000,), dtype=torch.int64, device=dev, generator=g),  # 40 MB
          torch.rand(3_000_000, device=dev, generator=g) < 0.5,  # bool: plain path
          torch.randn(1000, dtype=torch.float64, device=dev, generator=g),  # small: plain path
          torch.randn(2, 4_000_001, dtype=torch.float64, device=dev, generator=g)]  # 2-D
    outs = device.to_host_many(ts)
    for t, o in zip(ts, outs):
        ref = t.cpu().numpy()
        assert o.dtype == ref.dtype and o.shape == ref.shape
        assert o.tobytes() == ref.tobytes()
    again = device.to_host_many(ts[:1])[0]  # the ring is reused
    assert again.tobytes() == ts[0].cpu().numpy().tobytes()


def test_sample_leaves_numpy_on_every_node(gpu):
    from oracle.pipeline import cfg3_corr, cfg_dists
    from probabilit_amd.modeling import Distribution, NoOp

    ds = [Distribution(name, **kw) for name, kw in cfg_dists(8)]
    root = NoOp(*ds).correlate(*ds, corr_mat=cfg3_corr(8))
    n = 2_000_003
    root.sample(n, random_state=4, method="lhs")
    host = [x.__dict__["_host"] for x in ds]
    assert all(isinstance(h, np.ndarray) and h.shape == (n,) for h in host)
    for x, h in zip(ds, host):
        assert h.tobytes() == x.samples_device.cpu().numpy().tobytes()

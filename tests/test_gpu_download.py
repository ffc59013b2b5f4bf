"""The chunked pinned download of hourly planes (engine.hourly_to_host) equals
the plain gather + copy, in caller order and in device order, for fp64 and
fp32 tiles and a ragged last chunk."""
import numpy as np
import pytest
import torch

from dgen_amd.engine import hourly_agent_major, hourly_to_host

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_hourly_to_host_matches_plain_copy(dtype):
    n = 20_011
    g = torch.Generator(device="cuda").manual_seed(5)
    t = torch.rand((2190, n, 4), device="cuda", dtype=dtype, generator=g)
    perm = np.random.default_rng(3).permutation(n)
    inv = torch.as_tensor(np.argsort(perm), device="cuda")
    ref = hourly_agent_major(t).cpu().numpy()
    got = hourly_to_host(t, None, chunk=3000, threads=4)
    assert np.array_equal(got, ref)
    got = hourly_to_host(t, inv, chunk=3000, threads=4)
    assert np.array_equal(got, ref[np.argsort(perm)])

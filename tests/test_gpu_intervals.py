"""Batched degraded-read reconstruct: many independent
stripes of arbitrary lengths and erasure patterns in one GPU round trip,
bit-exact against the oracle."""
import numpy as np
import pytest

from oracle import corc
from oracle import rs_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["zero_copy", "copies"])
def staging_path(request, gpu):
    """The compact staging is decoded in place by the kernel over PCIe (zero
    copy, default) or copied H2D / D2H around the kernel."""
    import helyim_amd as H
    H.lib.hec_set_host_zero_copy(1 if request.param == "zero_copy" else 0)
    yield request.param
    H.lib.hec_set_host_zero_copy(1)


def _stripe(rng, L):
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(10)]
    full = data + [np.zeros(L, np.uint8) for _ in range(4)]
    corc.CReedSolomon(10, 4).encode(full)
    return full


@pytest.mark.parametrize("data_only", [False, True])
def test_reconstruct_batch_ragged(gpu, data_only):
    import helyim_amd as H
    rng = np.random.default_rng(11 + data_only)
    rs = H.ReedSolomon(10, 4)
    lens = [1, 7, 15, 16, 17, 4095, 4096, 4097, 12000, 65536 + 3] + \
        [int(x) for x in np.exp(rng.uniform(np.log(64), np.log(300000), 300))]
    fulls, stripes, erased = [], [], []
    for L in lens:
        full = _stripe(rng, L)
        e = set(rng.choice(14, int(rng.integers(0, 5)), replace=False).tolist())
        fulls.append(full)
        erased.append(e)
        stripes.append([None if i in e else full[i].copy() for i in range(14)])
    rs.reconstruct_batch(stripes, data_only=data_only)
    for full, st, e in zip(fulls, stripes, erased):
        for i in range(14):
            if data_only and i >= 10 and i in e:
                assert st[i] is None
            else:
                assert np.array_equal(st[i], full[i])


def test_reconstruct_batch_generic_geometry(gpu):
    import helyim_amd as H
    rng = np.random.default_rng(5)
    rs, ors = H.ReedSolomon(6, 3), O.ReedSolomon(6, 3)
    stripes, fulls = [], []
    for L in (3, 100, 5000):
        full = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(6)] + [np.zeros(L, np.uint8)] * 3
        full = [f.copy() for f in full]
        ors.encode(full)
        fulls.append(full)
        stripes.append([None if i in (1, 7) else full[i].copy() for i in range(9)])
    rs.reconstruct_batch(stripes)
    for full, st in zip(fulls, stripes):
        for a, b in zip(full, st):
            assert np.array_equal(a, b)

"""Host-memory batches (zero-copy kernels on pinned memory, or the pinned
H2D -> kernel -> D2H pipeline) vs the oracle."""
import itertools

import numpy as np
import pytest

from oracle import corc
from oracle import rs_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["zero_copy", "copy_pipeline"])
def host_path(request, gpu):
    """Every host-batch test runs on both paths: pinned buffers coded in place
    by the kernel over PCIe (default), and the H2D -> kernel -> D2H pipeline.
    Pageable buffers take the pipeline either way."""
    import helyim_amd as H
    assert H.lib.hec_set_host_zero_copy(1 if request.param == "zero_copy" else 0) == 0
    yield request.param
    H.lib.hec_set_host_zero_copy(1)


def _host_stripes(S, L, pin=True):
    import torch
    t = torch.zeros((S, 14, L), dtype=torch.uint8)
    if pin:
        t = t.pin_memory()
    a = t.numpy()
    for s in range(S):
        a[s, :10] = corc.splitmix64_bytes(O.STRIPE_SEED_BASE + s, 10 * L).reshape(10, L)
    return t


@pytest.mark.parametrize("L,S,pin", [(1, 3, True), (17, 5, True), (4096, 7, True), (65536 + 5, 9, True),
                                     (1 << 20, 40, True), (1000, 4, False), (1 << 20, 40, False),
                                     (65536 + 5, 300, False)])
def test_host_encode_batch(gpu, L, S, pin):
    import helyim_amd as H
    import helyim_amd.batch as B
    rs = H.ReedSolomon(10, 4)
    t = _host_stripes(S, L, pin)
    B.host_encode_batch(rs, t)
    a = t.numpy()
    ref = corc.encode_stripes(np.ascontiguousarray(a[:, :10]))
    assert np.array_equal(a[:, 10:], ref)


@pytest.mark.parametrize("pin", [True, False])
def test_host_reconstruct_every_pattern(gpu, pin):
    import helyim_amd as H
    import helyim_amd.batch as B
    rs = H.ReedSolomon(10, 4)
    pats = [c for e in range(0, 6) for c in itertools.combinations(range(14), e)]
    S, L = len(pats), 512 + 3
    t = _host_stripes(S, L, pin)
    B.host_encode_batch(rs, t)
    good = t.clone()
    a = t.numpy()
    masks = np.full(S, (1 << 14) - 1, dtype=np.uint32)
    for s, p in enumerate(pats):
        for i in p:
            a[s, i] = 0x5A
            masks[s] &= ~np.uint32(1 << i)
    bad = B.host_reconstruct_batch(rs, t, masks)
    n5 = sum(1 for p in pats if len(p) == 5)
    assert bad == n5
    for s, p in enumerate(pats):
        if len(p) <= 4:
            assert np.array_equal(a[s], good.numpy()[s]), p


def test_mixed_workload_lengths(gpu):
    """BASELINE config 5 shape: shard lengths 64 KiB..4 MiB, 0..4 erasures."""
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    rs = H.ReedSolomon(10, 4)
    rng = np.random.default_rng(5)
    for L in (64 << 10, 256 << 10, 1 << 20, 4 << 20):
        S = 3
        t = _host_stripes(S, L)
        B.host_encode_batch(rs, t)
        good = t.clone()
        masks = np.zeros(S, dtype=np.uint32)
        for s in range(S):
            e = int(rng.integers(0, 5))
            drop = rng.choice(14, e, replace=False)
            masks[s] = ((1 << 14) - 1) & ~int(sum(1 << int(i) for i in drop))
            for i in drop:
                t[s, int(i)] = 0
        assert B.host_reconstruct_batch(rs, t, masks) == 0
        assert torch.equal(t, good)
        ref = corc.encode_stripes(np.ascontiguousarray(good.numpy()[:, :10]))
        assert np.array_equal(good.numpy()[:, 10:], ref)


@pytest.mark.parametrize("k,m,pin", [(3, 2, True), (6, 3, False), (12, 4, True), (8, 8, False)])
def test_host_batches_generic_geometry(gpu, k, m, pin):
    """Host batches on geometries other than RS(10,4) (pinned: zero copy or
    pipeline; pageable: pooled staging), seeded per-stripe erasures, against
    the C oracle."""
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    rng = np.random.default_rng(31 * k + m)
    n, S, L = k + m, 6, 4096 + 7
    rs, ors = H.ReedSolomon(k, m), corc.CReedSolomon(k, m)
    t = torch.zeros((S, n, L), dtype=torch.uint8)
    if pin:
        t = t.pin_memory()
    a = t.numpy()
    a[:, :k] = rng.integers(0, 256, (S, k, L), dtype=np.uint8)
    want = a.copy()
    for s in range(S):
        ors.encode([want[s, i] for i in range(n)])
    B.host_encode_batch(rs, t)
    assert np.array_equal(a, want)
    masks = np.full(S, (1 << n) - 1, np.uint32)
    for s in range(S):
        for i in rng.choice(n, int(rng.integers(0, m + 1)), replace=False):
            masks[s] &= ~np.uint32(1 << int(i))
            a[s, int(i)] = 0xC3
    assert B.host_reconstruct_batch(rs, t, masks) == 0
    assert np.array_equal(a, want)


# ---- one host batch over a device set (hec_host_*_batch_multi) -------------
# The 1-GPU box repeats device 0: every range runs concurrently on its own
# host thread, pipeline and streams, which is the code an 8-GPU node runs with
# distinct ids. Range boundaries fall inside ragged stripe counts (S not a
# multiple of the list length) and at one stripe per range.
@pytest.mark.parametrize("devices,S,L,pin", [([0, 0], 7, 4096 + 3, True), ([0, 0, 0], 40, 1 << 20, True),
                                             ([0, 0], 9, 65536 + 5, False), ([0] * 5, 3, 1000, True),
                                             ([0, 0, 0, 0], 5, 17, False)])
def test_host_batch_multi_device_encode_and_every_erasure_count(gpu, devices, S, L, pin):
    import helyim_amd as H
    import helyim_amd.batch as B
    rs = H.ReedSolomon(10, 4)
    t = _host_stripes(S, L, pin)
    B.host_encode_batch(rs, t, devices=devices)
    a = t.numpy()
    want = a.copy()
    want[:, 10:] = corc.encode_stripes(np.ascontiguousarray(a[:, :10]))
    assert np.array_equal(a, want)
    rng = np.random.default_rng(S * 131 + len(devices))
    masks = np.full(S, (1 << 14) - 1, np.uint32)
    for s in range(S):
        e = s % 6  # 0..4 rebuilt, 5 counted as bad
        for i in rng.choice(14, e, replace=False):
            masks[s] &= ~np.uint32(1 << int(i))
            a[s, int(i)] = 0xA5
    bad = B.host_reconstruct_batch(rs, t, masks, devices=devices)
    assert bad == sum(1 for s in range(S) if s % 6 == 5)
    for s in range(S):
        if s % 6 <= 4:
            assert np.array_equal(a[s], want[s]), s


def test_host_batch_multi_device_errors(gpu):
    import ctypes
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    from helyim_amd.errors import DeviceError
    rs = H.ReedSolomon(10, 4)
    t = _host_stripes(4, 4096)
    before = t.clone()
    ndev = torch.cuda.device_count()
    with pytest.raises(DeviceError) as ei:  # a device out of range fails before any work
        B.host_encode_batch(rs, t, devices=[0, ndev])
    assert "device" in str(ei.value)
    assert torch.equal(t, before)
    with pytest.raises(ValueError):
        B.host_encode_batch(rs, t, devices=[])
    devs = (ctypes.c_int * 2)(0, 0)  # no stripes: nothing to do
    base = t.data_ptr()
    assert H.lib.hec_host_encode_batch_multi(rs.handle, devs, 2, base, 14 * 4096, 4096, base + 40960, 14 * 4096,
                                             4096, 4096, 0) == 0
    # the multi-device call and the single-device call agree byte for byte
    u = before.clone().pin_memory()
    B.host_encode_batch(rs, t, devices=[0, 0, 0])
    B.host_encode_batch(rs, u)
    assert torch.equal(t, u)


@pytest.mark.parametrize("k,m", [(3, 2), (6, 3)])
def test_host_batch_multi_device_generic_geometry(gpu, k, m):
    """The multi-device split on geometries other than RS(10,4) (each range
    takes the generic kernels), against the C oracle."""
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    rng = np.random.default_rng(7 * k + m)
    n, S, L = k + m, 5, 4096 + 9
    rs, ors = H.ReedSolomon(k, m), corc.CReedSolomon(k, m)
    t = torch.zeros((S, n, L), dtype=torch.uint8).pin_memory()
    a = t.numpy()
    a[:, :k] = rng.integers(0, 256, (S, k, L), dtype=np.uint8)
    want = a.copy()
    for s in range(S):
        ors.encode([want[s, i] for i in range(n)])
    B.host_encode_batch(rs, t, devices=[0, 0, 0])
    assert np.array_equal(a, want)
    masks = np.full(S, (1 << n) - 1, np.uint32)
    for s in range(S):
        for i in rng.choice(n, int(rng.integers(1, m + 1)), replace=False):
            masks[s] &= ~np.uint32(1 << int(i))
            a[s, int(i)] = 0x3C
    assert B.host_reconstruct_batch(rs, t, masks, devices=[0, 0]) == 0
    assert np.array_equal(a, want)


def _multi_roundtrip(t, devices):
    """encode + 0..4-erasure reconstruct of the host batch t over `devices`,
    byte-compared with the C oracle."""
    import helyim_amd as H
    import helyim_amd.batch as B
    rs = H.ReedSolomon(10, 4)
    S = t.shape[0]
    B.host_encode_batch(rs, t, devices=devices)
    a = t.numpy()
    want = a.copy()
    want[:, 10:] = corc.encode_stripes(np.ascontiguousarray(a[:, :10]))
    assert np.array_equal(a, want)
    rng = np.random.default_rng(S + 17 * len(devices))
    masks = np.full(S, (1 << 14) - 1, np.uint32)
    for s in range(S):
        for i in rng.choice(14, s % 5, replace=False):
            masks[s] &= ~np.uint32(1 << int(i))
            a[s, int(i)] = 0x5A
    assert B.host_reconstruct_batch(rs, t, masks, devices=devices) == 0
    assert np.array_equal(a, want)


@pytest.mark.parametrize("memory", ["hec_host_alloc", "placed", "torch_pinned", "pageable"])
def test_host_batch_multi_distinct_devices(gpu, memory):
    """one host batch over DISTINCT GPUs (each range on its own
    device; pinned memory allocated under device 0 coded zero-copy by the
    others, a per-range placed batch, pageable memory) vs the oracle. Needs
    two or more GPUs: skipped on the one-GPU pool, so distinct-device
    operation stays unverified there."""
    import torch
    import helyim_amd as H
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("needs >= 2 GPUs (the pool's boxes have one)")
    devices = list(range(min(n, 8)))
    S, L = 4 * len(devices) + 3, 65536
    torch.cuda.set_device(0)
    buf = None
    if memory == "hec_host_alloc":
        buf = H.HostBuffer(S * 14 * L)
    elif memory == "placed":
        buf = H.HostBuffer.for_devices(devices, 14 * L, S)
    if buf is not None:
        t = buf.tensor((S, 14, L))
        t.copy_(_host_stripes(S, L, pin=False))
    else:
        t = _host_stripes(S, L, pin=memory == "torch_pinned")
    _multi_roundtrip(t, devices)
    del t
    if buf is not None:
        buf.close()


def test_host_batch_multi_on_a_placed_buffer(gpu):
    """hec_host_alloc_multi's batch (pinned by hipHostRegister, not
    hipHostMalloc) through the _multi calls over a repeated device list, on
    both host paths, vs the oracle."""
    import helyim_amd as H
    S, L = 9, 65536 + 16
    buf = H.HostBuffer.for_devices([0, 0, 0], 14 * L, S)
    t = buf.tensor((S, 14, L))
    assert int(t.sum()) == 0  # zero-filled
    t.copy_(_host_stripes(S, L, pin=False))
    _multi_roundtrip(t, [0, 0, 0])
    del t
    buf.close()


def test_host_pipeline_pool_trims_after_a_burst(gpu, host_path):
    """a burst of concurrent host batches may create up to
    8 pipelines per device, but only the first 2 keep their staging after
    their call; the pinned and device staging left behind is bounded by two
    pipelines' worth (hec_host_staging_stats), and every result is exact."""
    import ctypes
    import threading
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    rs = H.ReedSolomon(10, 4)
    S, L = 16, 1 << 20
    src = _host_stripes(S, L, pin=False)
    want = src.numpy().copy()
    want[:, 10:] = corc.encode_stripes(np.ascontiguousarray(want[:, :10]))
    errors, start = [], threading.Barrier(12)

    def work():
        try:
            t = src.clone()  # pageable: the staging path
            start.wait()
            for _ in range(2):
                B.host_encode_batch(rs, t)
            assert np.array_equal(t.numpy(), want)
        except Exception as ex:  # pragma: no cover - reported below
            errors.append(repr(ex))

    ths = [threading.Thread(target=work) for _ in range(12)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors
    n, pinned, dev = ctypes.c_int(), ctypes.c_uint64(), ctypes.c_uint64()
    assert H.lib.hec_host_staging_stats(ctypes.byref(n), ctypes.byref(pinned), ctypes.byref(dev)) == 0
    # a pipeline's chunk is <= 96 MiB of stripes (host_pipeline.cpp kChunkBytes;
    # every host batch of this suite has 14 L below that), so a warm pipeline
    # holds at most two such pinned slots (pageable path) and three device
    # slots (copy path), sized by the largest batch it has served; the burst's
    # other pipelines hold none. Without the trim: ~8 x 2 x 88 MiB pinned here.
    chunk = 96 << 20
    per_pinned = 2 * chunk + (4 << 20)  # + mask words
    per_dev = 3 * chunk + (4 << 20)
    assert 1 <= n.value <= 8
    assert pinned.value <= 2 * per_pinned, (n.value, pinned.value)
    assert dev.value <= 2 * per_dev, (n.value, dev.value)
    torch.cuda.synchronize()


def test_which_buffers_are_coded_zero_copy(gpu, host_path):
    """hec_host_zero_copy_view: hec_host_alloc, hec_host_alloc_multi
    (hipHostRegister'd, not hipHostMalloc'd) and torch pinned buffers are
    coded in place over PCIe; pageable memory, a range running past a pinned
    allocation, and everything under hec_set_host_zero_copy(0) take staging."""
    import ctypes
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    on = host_path == "zero_copy"
    S, L = 4, 4096
    a = H.HostBuffer(S * 14 * L)
    b = H.HostBuffer.for_devices([0, 0], 14 * L, S)
    ta, tb = a.tensor((S, 14, L)), b.tensor((S, 14, L))
    tp = torch.zeros((S, 14, L), dtype=torch.uint8).pin_memory()
    tq = torch.zeros((S, 14, L), dtype=torch.uint8)
    assert B.host_zero_copy(ta) == on and B.host_zero_copy(tb) == on and B.host_zero_copy(tp) == on
    assert not B.host_zero_copy(tq)
    z = ctypes.c_int(7)
    assert H.lib.hec_host_zero_copy_view(a.ptr, S * 14 * L + (1 << 30), ctypes.byref(z)) == 0
    assert z.value == 0  # runs past the allocation
    del ta, tb
    a.close()
    b.close()


@pytest.mark.parametrize("L", [2048, 2048 * 5, 3 * 8192, 1 << 20, 4096 + 16, 4096 + 1])
def test_host_encode_kernel_choice_over_pcie(gpu, L):
    """Zero-copy host-batch encodes take the 8 B-per-lane table kernel for
    shard lengths that are multiples of 2 KiB and the 16-byte table kernel
    otherwise; every choice, and a batch at an odd host address (unaligned:
    the generic kernel), writes the oracle's parity."""
    import helyim_amd as H
    import helyim_amd.batch as B
    rs = H.ReedSolomon(10, 4)
    lib = H.lib
    S = 6
    name = lib.hec_host_encode_kernel_name(L).decode()
    if L % 2048 == 0:
        assert name.startswith("rs104_narrow_kernel<DEC=false, 8 B per lane>"), name
    else:
        assert name.startswith("rs104_kernel<DEC=false>"), name
    t = _host_stripes(S, L)
    B.host_encode_batch(rs, t)
    a = t.numpy()
    assert np.array_equal(a[:, 10:], corc.encode_stripes(np.ascontiguousarray(a[:, :10])))
    # the same stripes one byte into a pinned buffer: unaligned bases
    import torch
    raw = torch.zeros(S * 14 * L + 1, dtype=torch.uint8).pin_memory()
    u = raw[1:].view(S, 14, L)
    u[:, :10] = t[:, :10]
    B.host_encode_batch(rs, u)
    assert np.array_equal(u.numpy()[:, 10:], a[:, 10:])


@pytest.mark.parametrize("pin", [True, False])
def test_error_return_leaves_nothing_in_flight(gpu, monkeypatch, pin):
    """A host batch that fails part-way returns only once the work it had
    queued onto the caller's buffers has landed (hec.h: nothing in flight on
    error returns). HEC_TEST_HOST_FAIL_AFTER_CHUNK=2 fails a copy-pipeline
    encode right after queueing chunk 2's kernel: at return, chunks 0-1 hold
    the oracle's parity, and chunk 2's (never copied back) and later chunks'
    parity rows are untouched. A 1 MiB stripe is 14 MiB, so a 96 MiB chunk
    holds 6 stripes (host_pipeline.cpp kChunkBytes). The pinned case is the
    one that exercises the drain: its device-to-host copies land in the
    caller's buffer asynchronously (a pageable destination is staged by the
    runtime and lands before the copy call returns)."""
    import helyim_amd as H
    import helyim_amd.batch as B
    assert H.lib.hec_set_host_zero_copy(0) == 0  # the copy pipeline (reset by the host_path fixture)
    rs = H.ReedSolomon(10, 4)
    S, L, C = 24, 1 << 20, 6
    t = _host_stripes(S, L, pin=pin)
    a = t.numpy()
    a[:, 10:] = 0xA5
    ref = corc.encode_stripes(np.ascontiguousarray(a[:, :10]))
    monkeypatch.setenv("HEC_TEST_HOST_FAIL_AFTER_CHUNK", "2")
    with pytest.raises(H.DeviceError, match="test hook: failure after chunk 2"):
        B.host_encode_batch(rs, t)
    assert np.array_equal(a[:2 * C, 10:], ref[:2 * C])
    assert (a[2 * C:, 10:] == 0xA5).all()
    monkeypatch.delenv("HEC_TEST_HOST_FAIL_AFTER_CHUNK")
    B.host_encode_batch(rs, t)  # the pipeline is usable again
    assert np.array_equal(a[:, 10:], ref)

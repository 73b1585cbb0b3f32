"""File-level drop-ins (write_ec_files / rebuild_ec_files) on the GPU against
the committed 30 MB fixture and the oracle's encoder.rs restatement."""
import os

import numpy as np
import pytest

from oracle import rs_oracle as O

pytestmark = pytest.mark.gpu


def _sha(path):
    return O.sha256(open(path, "rb").read())


def test_volume_30mb_encode_rebuild(gpu, golden, tmp_path):
    import helyim_amd as H
    g = golden("volume_30mb.json")
    base = str(tmp_path / "1")
    vol = O.synthetic_volume(g["dat_bytes"])
    open(base + ".dat", "wb").write(vol.tobytes())
    H.write_ec_files(base)
    assert [_sha(base + H.to_ext(i)) for i in range(14)] == g["shard_sha256"]
    for drop in g["drops"]:
        for i in drop:
            os.remove(base + H.to_ext(i))
        assert H.rebuild_ec_files(base) == sorted(drop)
        assert [_sha(base + H.to_ext(i)) for i in range(14)] == g["shard_sha256"]
    assert H.rebuild_ec_files(base) == []


@pytest.mark.parametrize("size", [1, 639, 640, 641, 2000, 6401, 6400 * 2 + 3, 6400 * 3])
def test_small_geometry_vs_oracle(gpu, tmp_path, size):
    """Large-row path exercised with 640-byte 'large' and 32-byte 'small' blocks."""
    import helyim_amd as H
    buf, large, small = 16, 640, 32
    dat = O.splitmix64_bytes(5 + size, size).tobytes()
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    for base in (a, b):
        open(base + ".dat", "wb").write(dat)
    H.generate_ec_files(a, buf, large, small)
    O.write_ec_files(b, buf, large, small)
    for i in range(14):
        assert open(a + H.to_ext(i), "rb").read() == open(b + O.to_ext(i), "rb").read(), i
    # rebuild (1 MiB read rows, encoder.rs:244-307) of a seeded 1-4 shard drop
    rng = np.random.default_rng(size)
    drop = sorted(int(i) for i in rng.choice(14, int(rng.integers(1, 5)), replace=False))
    want = [open(a + H.to_ext(i), "rb").read() for i in range(14)]
    for i in drop:
        os.remove(a + H.to_ext(i))
    assert H.rebuild_ec_files(a) == drop
    assert [open(a + H.to_ext(i), "rb").read() for i in range(14)] == want


def test_unexpected_block_size(gpu, tmp_path):
    import helyim_amd as H
    base = str(tmp_path / "v")
    open(base + ".dat", "wb").write(b"x" * 100)
    with pytest.raises(H.UnexpectedBlockSize) as ei:
        H.generate_ec_files(base, 24, 640, 32)
    # helyim's payload: UnexpectedBlockSize(block_size, buf_size), encoder.rs:140-143
    assert (ei.value.block_size, ei.value.buf_size) == (32, 24)
    assert str(ei.value) == "unexpected block size 32, buffer size 24"


@pytest.mark.parametrize("buf,large,small,size,written", [
    (16, 640, 24, 6400 + 1000, 640),  # one large row coded, then the small rows' check fails
    (24, 640, 32, 6400 + 1000, 0),    # the first large row's check fails: nothing coded
])
def test_unexpected_block_size_leaves_the_reference_bytes(gpu, tmp_path, buf, large, small, size, written):
    """UnexpectedBlockSize is raised by encode_data at the first row of a kind
    whose block the buffer does not divide (encoder.rs:139-144), after the
    rows before it were written: the 14 files hold exactly those rows, byte
    for byte the oracle's encoder.rs restatement, which stops at the same
    point."""
    import helyim_amd as H
    dat = O.splitmix64_bytes(77, size).tobytes()
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    for base in (a, b):
        open(base + ".dat", "wb").write(dat)
    with pytest.raises(H.UnexpectedBlockSize) as ei:
        H.generate_ec_files(a, buf, large, small)
    with pytest.raises(O.UnexpectedBlockSize):
        O.write_ec_files(b, buf, large, small)
    assert (ei.value.block_size, ei.value.buf_size) == ((small if written else large), buf)
    for i in range(14):
        got = open(a + H.to_ext(i), "rb").read()
        assert len(got) == written, (i, len(got))
        assert got == open(b + O.to_ext(i), "rb").read(), i


def test_rebuild_errors(gpu, tmp_path):
    import helyim_amd as H
    base = str(tmp_path / "v")
    vol = O.synthetic_volume(3_000_000)
    open(base + ".dat", "wb").write(vol.tobytes())
    H.write_ec_files(base)
    shas = [_sha(base + H.to_ext(i)) for i in range(14)]
    # too few shards present -> ErasureCoding(TooFewShardsPresent)
    for i in range(5):
        os.rename(base + H.to_ext(i), base + H.to_ext(i) + ".bak")
    with pytest.raises(H.ErasureCoding) as ei:
        H.rebuild_ec_files(base)
    assert isinstance(ei.value.inner, H.TooFewShardsPresent)
    # the missing shards' outputs were created and truncated before decoding,
    # so the failed rebuild leaves them empty, as the reference's does
    # (encoder.rs:96-104 opens them before rebuild_ec_files_inner)
    for i in range(5):
        assert os.path.getsize(base + H.to_ext(i)) == 0, i
    for i in range(5):
        os.replace(base + H.to_ext(i) + ".bak", base + H.to_ext(i))
    # shard 0 one row + 5 bytes long: the second row reads n = 5 != 1 MiB ->
    # UnexpectedEcShardSize after the first row was rebuilt (encoder.rs:275-280)
    os.remove(base + H.to_ext(3))
    with open(base + H.to_ext(0), "r+b") as f:
        f.truncate((1 << 20) + 5)
    with pytest.raises(H.UnexpectedEcShardSize) as ei:
        H.rebuild_ec_files(base)
    assert (ei.value.expected, ei.value.actual) == (1 << 20, 5)
    assert str(ei.value) == "ec shard size expected 1048576 but actually is 5"
    assert _sha(base + H.to_ext(3)) == shas[3]


def test_rebuild_matches_oracle_on_odd_sizes(gpu, tmp_path):
    """Shard files smaller than 1 MiB (row = file size), mirrored by the oracle."""
    import helyim_amd as H
    rs = O.ReedSolomon(10, 4)
    L = 1000
    data = [O.splitmix64_bytes(40 + i, L) for i in range(10)]
    sh = data + [np.zeros(L, np.uint8) for _ in range(4)]
    rs.encode(sh)
    base = str(tmp_path / "w")
    for i in range(14):
        open(base + H.to_ext(i), "wb").write(sh[i].tobytes())
    for i in (2, 11):
        os.remove(base + H.to_ext(i))
    assert H.rebuild_ec_files(base) == [2, 11]
    for i in range(14):
        assert open(base + H.to_ext(i), "rb").read() == sh[i].tobytes()


def _tree(base):
    """{ext: bytes} of every .ecNN file of a volume (absent files left out)."""
    import helyim_amd as H
    return {i: open(base + H.to_ext(i), "rb").read() for i in range(14) if os.path.exists(base + H.to_ext(i))}


def test_zero_byte_dat_gives_14_empty_shards(gpu, tmp_path):
    """A 0-byte .dat (encoder.rs:62: remaining = 0): neither row loop runs
    (:215, :228), so write_ec_files leaves the 14 files open_ec_files created
    and truncated (:111-127) empty; the oracle's restatement agrees."""
    import helyim_amd as H
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    for base in (a, b):
        open(base + ".dat", "wb").close()
        for i in (3, 12):  # stale shard files from an earlier run are truncated
            open(base + H.to_ext(i), "wb").write(b"stale")
    H.write_ec_files(a)
    O.write_ec_files(b)
    assert _tree(a) == _tree(b) == {i: b"" for i in range(14)}
    # and a rebuild over those empty shards (the first present read is 0
    # bytes, encoder.rs:269-271) recreates the missing one, still empty
    os.remove(a + H.to_ext(5))
    assert H.rebuild_ec_files(a) == [5]
    assert _tree(a) == {i: b"" for i in range(14)}


@pytest.mark.parametrize("short", [0, 6, 13])
def test_rebuild_stops_when_a_present_shard_ends_a_row_early(gpu, tmp_path, short):
    """rebuild_ec_files reads row by row in shard order and returns Ok at the
    first present shard whose read is 0 bytes (encoder.rs:268-271), BEFORE
    the size check (:275) and before that row is reconstructed or written:
    with one present shard (the first, a middle or the last present one) a
    whole 1 MiB row shorter than the others, the rebuilt shards hold only the
    rows every present shard has. Exact sizes and bytes, product vs oracle."""
    import helyim_amd as H
    L = 2 << 20  # two 1 MiB rebuild rows
    rs = O.ReedSolomon(10, 4)
    sh = [O.splitmix64_bytes(700 + i, L) for i in range(10)] + [np.zeros(L, np.uint8) for _ in range(4)]
    rs.encode(sh)
    lost = [2, 11] if short not in (2, 11) else [3, 10]
    trees = []
    for name in ("a", "b"):
        base = str(tmp_path / name)
        for i in range(14):
            open(base + H.to_ext(i), "wb").write(sh[i].tobytes())
        os.truncate(base + H.to_ext(short), 1 << 20)
        for i in lost:
            os.remove(base + H.to_ext(i))
        trees.append(base)
    assert H.rebuild_ec_files(trees[0]) == lost
    assert O.rebuild_ec_files(trees[1]) == lost
    got, want = _tree(trees[0]), _tree(trees[1])
    assert got == want
    for i in lost:
        assert len(got[i]) == 1 << 20, (i, len(got[i]))  # row 1 never written
        assert got[i] == sh[i][: 1 << 20].tobytes()


@pytest.mark.parametrize("lost", [[0, 7, 10, 13], list(range(5, 14))])
def test_rebuild_over_all_empty_present_shards(gpu, tmp_path, lost):
    """Every present shard empty: the first read returns 0 bytes at offset 0
    (encoder.rs:269-271), so rebuild_ec_files returns the missing ids with
    their files created (open with create + truncate: :96-103) and empty --
    even with only 5 present, since the loop returns Ok before reconstruct
    could report TooFewShardsPresent (:288)."""
    import helyim_amd as H
    bases = [str(tmp_path / n) for n in ("a", "b")]
    for base in bases:
        for i in range(14):
            if i not in lost:
                open(base + H.to_ext(i), "wb").close()
    assert H.rebuild_ec_files(bases[0]) == lost
    assert O.rebuild_ec_files(bases[1]) == lost
    assert _tree(bases[0]) == _tree(bases[1]) == {i: b"" for i in range(14)}


def test_rebuild_with_every_shard_missing(gpu, tmp_path):
    """No shard file present: nothing is read, so the first row goes straight
    to reconstruct with 0 present shards -> ErasureCoding(TooFewShardsPresent)
    (encoder.rs:262-288), after all 14 outputs were created empty (:96-103)."""
    import helyim_amd as H
    base = str(tmp_path / "none")
    with pytest.raises(H.ErasureCoding) as ei:
        H.rebuild_ec_files(base)
    assert isinstance(ei.value.inner, H.TooFewShardsPresent)
    with pytest.raises(O.TooFewShardsPresent):
        O.rebuild_ec_files(str(tmp_path / "none_oracle"))
    assert _tree(base) == {i: b"" for i in range(14)}
    assert _tree(str(tmp_path / "none_oracle")) == {i: b"" for i in range(14)}


def test_randomised_rebuild_size_rules_vs_oracle(gpu, tmp_path):
    """Seeded sweep of rebuild_ec_files over present shards whose sizes break
    the equal-rows rule in every way the reference's loop distinguishes
    (encoder.rs:262-306, reads in shard order per 1 MiB row): a shard a row
    short, a shard cut mid-row, a shard extended by a few bytes, an empty
    shard, placed first, in the middle or last among the present ones, 1-4
    shards lost. The product and the oracle's restatement must agree on the
    outcome -- the rebuilt ids, or the error and its (expected, actual)
    payload -- and on every byte of every file afterwards."""
    import helyim_amd as H
    rng = np.random.default_rng(2606)
    rs = O.ReedSolomon(10, 4)
    M = 1 << 20
    for case in range(24):
        L = int(rng.choice([M, 2 * M, 3 * M, 2 * M + 4096, M + 17]))
        sh = [O.splitmix64_bytes(1000 * case + i, L) for i in range(10)] + [np.zeros(L, np.uint8) for _ in range(4)]
        rs.encode(sh)
        lost = sorted(int(i) for i in rng.choice(14, int(rng.integers(1, 5)), replace=False))
        present = [i for i in range(14) if i not in lost]
        edits = {}
        for _ in range(int(rng.integers(0, 3))):
            i = int(rng.choice([present[0], present[len(present) // 2], present[-1]]))
            edits[i] = int(rng.choice([max(L - M, 0), L - 5, L + 3, 0, M // 2]))
        bases = [str(tmp_path / f"{n}{case}") for n in ("a", "b")]
        for base in bases:
            for i in present:
                data = sh[i].tobytes()
                if i in edits:
                    n = edits[i]
                    data = data[:n] if n <= L else data + bytes(n - L)
                open(base + H.to_ext(i), "wb").write(data)
        try:
            got = ("ok", H.rebuild_ec_files(bases[0]))
        except H.UnexpectedEcShardSize as e:
            got = ("size", (e.expected, e.actual))
        except H.ErasureCoding as e:
            got = ("rs", type(e.inner).__name__)
        try:
            want = ("ok", O.rebuild_ec_files(bases[1]))
        except O.UnexpectedEcShardSize as e:
            want = ("size", tuple(e.args))
        except O.TooFewShardsPresent:
            want = ("rs", "TooFewShardsPresent")
        assert got == want, (case, L, lost, edits, got, want)
        assert _tree(bases[0]) == _tree(bases[1]), (case, L, lost, edits)


def test_device_selection_and_concurrent_volumes(gpu, golden, tmp_path):
    """hec_set_device per thread (hec.h): volumes encoded and rebuilt
    concurrently from several threads, round-robin over the visible devices
    (all on device 0 on a one-GPU box), each byte-identical to the fixture."""
    import threading
    import helyim_amd as H
    n = H.device_count()
    assert n >= 1 and 0 <= H.get_device() < n
    for bad in (n, -1):
        with pytest.raises(H.DeviceError) as ei:
            H.set_device(bad)
        assert ei.value.code == 66  # HEC_ERR_INVALID_ARGUMENT
    g = golden("volume_30mb.json")
    vol = O.synthetic_volume(g["dat_bytes"]).tobytes()
    bases = [str(tmp_path / str(v)) for v in range(4)]
    for b in bases:
        open(b + ".dat", "wb").write(vol)
    errs, seen = [], {}

    def work(v, b):
        try:
            H.set_device(v % n)
            seen[v] = H.get_device()
            H.write_ec_files(b)
            for i in (1, 4, 11, 13):
                os.remove(b + H.to_ext(i))
            assert H.rebuild_ec_files(b) == [1, 4, 11, 13]
        except BaseException as e:  # surfaced in the main thread
            errs.append(e)

    th = [threading.Thread(target=work, args=(v, b)) for v, b in enumerate(bases)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    assert seen == {v: v % n for v in range(4)}
    for b in bases:
        assert [_sha(b + H.to_ext(i)) for i in range(14)] == g["shard_sha256"]


def test_randomised_file_geometry_vs_oracle(gpu, tmp_path):
    """Seeded sweep of generate_ec_files over block geometries (buffer,
    large and small block sizes) and .dat sizes around the large-row rule
    (large rows only while remaining > 10 large blocks, encoder.rs:215),
    byte-compared with the oracle's encoder.rs restatement, then a seeded
    drop + rebuild round trip."""
    import helyim_amd as H
    rng = np.random.default_rng(42)
    for case in range(24):
        buf = 16 * int(rng.integers(1, 3))
        small = buf * int(rng.integers(1, 5))
        large = small * int(rng.integers(2, 9))
        big = 10 * large
        size = int(rng.choice([int(rng.integers(1, big)), big, big + 1, 2 * big + int(rng.integers(0, big)),
                               3 * big - 1]))
        dat = O.splitmix64_bytes(900 + case, size).tobytes()
        a, b = str(tmp_path / f"a{case}"), str(tmp_path / f"b{case}")
        for base in (a, b):
            open(base + ".dat", "wb").write(dat)
        H.generate_ec_files(a, buf, large, small)
        O.write_ec_files(b, buf, large, small)
        for i in range(14):
            assert open(a + H.to_ext(i), "rb").read() == open(b + O.to_ext(i), "rb").read(), (case, i)
        drop = sorted(int(i) for i in rng.choice(14, int(rng.integers(1, 5)), replace=False))
        want = [open(a + H.to_ext(i), "rb").read() for i in range(14)]
        for i in drop:
            os.remove(a + H.to_ext(i))
        assert H.rebuild_ec_files(a) == drop
        assert [open(a + H.to_ext(i), "rb").read() for i in range(14)] == want, case


def _file_digest(path):
    import hashlib
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(16 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def test_production_geometry_multi_slice_multi_job_vs_oracle(gpu, tmp_path):
    """The file-layer paths a real 30,000 MB volume takes, at a size the C
    oracle finishes in seconds: 48 MiB large blocks (three 16 MiB slices per
    large block, ec_files.cpp kLargeSlice), 1 MiB small blocks, 256 KiB
    buffers (encoder.rs:200-242). .dat = 10 x 48 MiB + 260 MiB + 12,345 B:
    one large row (remaining > 10 large blocks, encoder.rs:215), then 27
    small rows = two 25-row GPU jobs; with the large row's 3 slice jobs that
    is 5 jobs over 3 pipeline slots (out-of-order slot reuse). Shard files are
    75 MiB = 75 one-MiB rebuild rows = three 25-row rebuild jobs
    (encoder.rs:244-307). Every shard file is compared with the oracle's."""
    import helyim_amd as H
    from oracle import corc
    MiB = 1 << 20
    large, small, buf = 48 * MiB, MiB, 256 * 1024
    size = 10 * large + 260 * MiB + 12345
    dat = corc.splitmix64_bytes(0x5EED0000 + 48, size)
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    for base in (a, b):
        with open(base + ".dat", "wb") as f:
            f.write(memoryview(dat))
    del dat
    H.generate_ec_files(a, buf, large, small)
    assert corc.write_ec_files(b, buf, large, small) == 0
    want = [_file_digest(b + O.to_ext(i)) for i in range(14)]
    assert os.path.getsize(a + H.to_ext(0)) == large + 27 * small
    assert [_file_digest(a + H.to_ext(i)) for i in range(14)] == want
    os.remove(b + ".dat")
    # drop 4 (two data, two parity), rebuild on the GPU and in the oracle
    drop = [2, 7, 10, 13]
    for i in drop:
        os.remove(a + H.to_ext(i))
        os.remove(b + O.to_ext(i))
    assert H.rebuild_ec_files(a) == drop
    assert corc.rebuild_ec_files(b) == (0, drop)
    for i in range(14):
        assert _file_digest(a + H.to_ext(i)) == want[i] == _file_digest(b + O.to_ext(i)), i
    # four data shards lost: the decode reads all four parity shards
    for i in (0, 1, 5, 9):
        os.remove(a + H.to_ext(i))
    assert H.rebuild_ec_files(a) == [0, 1, 5, 9]
    assert [_file_digest(a + H.to_ext(i)) for i in range(14)] == want


def _same_file(a, b, chunk=1 << 28):
    """Byte-compare two files in 256 MiB pieces (numpy), sizes first."""
    if os.path.getsize(a) != os.path.getsize(b):
        return False
    with open(a, "rb") as fa, open(b, "rb") as fb:
        while True:
            x, y = fa.read(chunk), fb.read(chunk)
            if x != y:
                return False
            if not x:
                return True


@pytest.mark.parametrize("extra", [0, 4097])
def test_reference_geometry_large_row_threshold(gpu, extra):
    """The reference's own constants (1 GiB large blocks, 1 MiB small blocks,
    256 KiB buffers) at the large-row threshold, encoder.rs:215 (`remaining >
    large_block_size * DATA_SHARDS_COUNT`, strict): a .dat of exactly 10 GiB
    takes NO large row (1024 small rows, 1 GiB shard files); 10 GiB + 4097 B
    takes one large row (each data shard's 1 GiB block in 64 slices of 16 MiB)
    and one zero-padded small row (1 GiB + 1 MiB shard files). Every shard file
    is byte-compared with the C oracle's encoder.rs restatement, then four
    shards (two data, two parity) are rebuilt on both sides and compared.
    Files live in /dev/shm (~40 GB at the peak, removed afterwards)."""
    import shutil
    import tempfile
    import helyim_amd as H
    from oracle import corc
    GiB, MiB = 1 << 30, 1 << 20
    size = 10 * GiB + extra
    d = tempfile.mkdtemp(prefix="hec_refgeom_", dir="/dev/shm")
    try:
        a, b = os.path.join(d, "a"), os.path.join(d, "b")
        with open(a + ".dat", "wb") as f:
            left, part = size, 0
            while left:
                n = min(left, GiB)
                f.write(memoryview(corc.splitmix64_bytes(0x5EED7000 + part, n)))
                left -= n
                part += 1
        os.link(a + ".dat", b + ".dat")  # one copy of the 10 GiB input, read by both encoders
        H.write_ec_files(a)
        assert corc.write_ec_files(b) == 0
        want_len = GiB + (MiB if extra else 0)
        for i in range(14):
            assert os.path.getsize(a + H.to_ext(i)) == want_len, i
            assert _same_file(a + H.to_ext(i), b + O.to_ext(i)), i
        os.remove(a + ".dat")
        os.remove(b + ".dat")
        drop = [3, 9, 10, 12]
        for i in drop:
            os.remove(a + H.to_ext(i))
            os.remove(b + O.to_ext(i))
        assert H.rebuild_ec_files(a) == drop
        assert corc.rebuild_ec_files(b) == (0, drop)
        for i in drop:
            assert _same_file(a + H.to_ext(i), b + O.to_ext(i)), i
    finally:
        shutil.rmtree(d, ignore_errors=True)


def test_write_error_in_the_pipeline_carries_its_errno(gpu, tmp_path):
    """An I/O error inside the file pipeline's writer threads (encoder.rs:194
    `output.write_all(..)?` -> EcShardError::Io) comes back with its errno:
    shard 3's output is /dev/full, so its pwritev fails with ENOSPC after the
    GPU coded the rows, and hec_last_error_values carries 28 out of the
    worker thread (ErrorSlot -> drain)."""
    import errno
    import helyim_amd as H
    if not os.path.exists("/dev/full"):
        pytest.skip("no /dev/full")
    base = str(tmp_path / "v")
    open(base + ".dat", "wb").write(O.synthetic_volume(3_000_000).tobytes())
    os.symlink("/dev/full", base + H.to_ext(3))
    with pytest.raises(H.Io) as ei:
        H.write_ec_files(base)
    assert ei.value.errno == errno.ENOSPC, (ei.value.errno, str(ei.value))
    assert isinstance(ei.value.os_error, OSError) and ei.value.os_error.errno == errno.ENOSPC
    assert "(os error 28)" in str(ei.value)

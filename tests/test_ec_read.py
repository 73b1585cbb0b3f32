"""Needle reads from EC shards: locate_data, the .ecx
lookup and the degraded read (helyim-ec/src/locate.rs,
helyim-store/src/erasure_coding/mod.rs:129-491).

The oracle's read path is pinned against the volume's own .dat bytes (a read
of an intact or degraded volume must return the original data), and
locate_data against intervals derived by hand from locate.rs. CPU tests cover
everything that needs no reconstruction (libhec reads present shards without
touching the GPU); gpu tests rebuild lost intervals and compare with the
oracle."""
import struct

import numpy as np
import pytest

from oracle import corc
from oracle import rs_oracle as O

LARGE, SMALL, BUF = 640, 32, 16


def _volume(tmp_path, size, seed=3, name="v"):
    base = str(tmp_path / name)
    dat = O.splitmix64_bytes(seed, size).tobytes()
    open(base + ".dat", "wb").write(dat)
    assert corc.write_ec_files(base, BUF, LARGE, SMALL) == 0
    return base, dat


def _drop(base, ids):
    import os
    for i in ids:
        os.remove(base + O.to_ext(i))


def _ranges(rng, size, n, maxlen=3000):
    out = []
    for _ in range(n):
        ln = int(rng.integers(1, maxlen))
        off = int(rng.integers(0, max(size - ln, 1)))
        out.append((off, min(ln, size - off)))
    return out


# ---- locate_data ------------------------------------------------------------

# (large, small, data_size, offset, size) -> [(block_index, inner, size, is_large, large_block_rows)]
LOCATE_KAT = [
    # inside the large rows, across one block boundary
    ((640, 32, 19520, 1000, 700), [(1, 360, 280, True, 3), (2, 0, 420, True, 3)]),
    # large -> small transition (block_index wraps to 0 at large_block_rows * 10)
    ((640, 32, 19520, 19100, 150), [(29, 540, 100, True, 3), (0, 0, 32, False, 3), (1, 0, 18, False, 3)]),
    # the two large-row counts disagree (locate.rs:39-40 vs :84): 2 vs 3
    ((640, 32, 18880, 12805, 10), [(0, 5, 10, False, 3)]),
    ((640, 32, 19520, 77, 0), []),
    # real geometry: 1 GiB / 1 MiB blocks, a 30 GB volume
    ((1 << 30, 1 << 20, 30_000_000_000, 21_474_836_480 + 5, 2 << 20),
     [(0, 5, (1 << 20) - 5, False, 2), (1, 0, 1 << 20, False, 2), (2, 0, 5, False, 2)]),
]


@pytest.mark.parametrize("args,want", LOCATE_KAT)
def test_locate_data_known_answers(args, want):
    import helyim_amd as H
    assert O.locate_data(*args) == want
    assert [iv.as_tuple() for iv in H.locate_data(*args)] == want


def test_interval_offsets_known_answers():
    import helyim_amd as H
    ivs = H.locate_data(640, 32, 19520, 19100, 150)
    assert [(iv.shard_id(), iv.offset(640, 32)) for iv in ivs] == [(9, 1820), (0, 1920), (1, 1920)]
    (q,) = H.locate_data(640, 32, 18880, 12805, 10)
    assert (q.shard_id(), q.offset(640, 32)) == (0, 1925)  # mirrors the reference (true place: 1285)


def test_locate_data_random_vs_oracle():
    import helyim_amd as H
    rng = np.random.default_rng(9)
    for _ in range(3000):
        large, small = [(64, 8), (640, 32), (640, 64), (4096, 256), (1 << 30, 1 << 20)][int(rng.integers(0, 5))]
        data_size = int(rng.integers(0, 60 * large))
        offset = int(rng.integers(0, data_size + 1))
        size = int(rng.integers(0, 40 * small + (2 * large if rng.random() < 0.3 else 0)))  # <= ~2k intervals
        want = O.locate_data(large, small, data_size, offset, size)
        got = H.locate_data(large, small, data_size, offset, size)
        assert [iv.as_tuple() for iv in got] == want, (large, small, data_size, offset, size)
        assert [iv.offset(large, small) for iv in got] == [O.interval_offset(w, large, small) for w in want]
        assert [iv.shard_id() for iv in got] == [O.interval_shard_id(w) for w in want]


# ---- .ecx lookup --------------------------------------------------------------

def test_find_needle_from_ecx(tmp_path):
    import helyim_amd as H
    base = str(tmp_path / "v")
    keys = sorted(set(np.random.default_rng(2).integers(1, 1 << 40, 300).tolist()))
    raw = b"".join(struct.pack(">QIi", k, i + 1, (i * 37) % 5000 - (100 if i % 17 == 0 else 0))
                   for i, k in enumerate(keys))
    open(base + ".ecx", "wb").write(raw)
    for i, k in enumerate(keys):
        assert H.find_needle_from_ecx(base, k) == O.find_needle_from_ecx(base, k)
    for k in (0, keys[0] - 1, keys[-1] + 1, keys[10] + 1):
        if k in keys:
            continue
        with pytest.raises(H.Io, match="is not found"):
            H.find_needle_from_ecx(base, k)
        with pytest.raises(O.IoError):
            O.find_needle_from_ecx(base, k)


# ---- reads with every shard present (host only) ------------------------------

@pytest.mark.parametrize("size", [19300, 6400 * 2 + 3, 1000, 32123])
def test_oracle_read_matches_dat(tmp_path, size):
    """Pins the oracle's read path: intact and degraded reads return the .dat."""
    base, dat = _volume(tmp_path, size)
    rng = np.random.default_rng(size)
    ranges = _ranges(rng, size, 40)
    want = b"".join(dat[o:o + n] for o, n in ranges)
    assert O.read_ec_data(base, ranges, LARGE, SMALL) == want
    assert corc.read_ec_data(base, ranges, LARGE, SMALL) == (0, want)
    _drop(base, [0, 3, 11, 13])
    assert O.read_ec_data(base, ranges, LARGE, SMALL) == want
    assert corc.read_ec_data(base, ranges, LARGE, SMALL) == (0, want)


@pytest.mark.parametrize("size", [19300, 32123])
def test_read_present_shards_host_only(tmp_path, size):
    import helyim_amd as H
    base, dat = _volume(tmp_path, size)
    _drop(base, [10, 11, 12, 13])  # parity lost: data reads need no reconstruction
    rng = np.random.default_rng(size + 1)
    ranges = _ranges(rng, size, 60)
    assert H.read_ec_data(base, ranges, LARGE, SMALL) == b"".join(dat[o:o + n] for o, n in ranges)


def test_read_quirk_volume_matches_oracle(tmp_path):
    """locate.rs's two large-row counts disagree for this volume, so reads in
    the small rows land past the shard ends; the product fails like the
    oracle (read_exact_at -> UnexpectedEof) instead of returning bytes."""
    import helyim_amd as H
    base, dat = _volume(tmp_path, 6400 * 2 + 6000)
    with pytest.raises(O.IoError):
        O.read_ec_data(base, [(12800 + 5, 10)], LARGE, SMALL)
    with pytest.raises(H.Io):
        H.read_ec_data(base, [(12800 + 5, 10)], LARGE, SMALL)
    assert H.read_ec_data(base, [(100, 1000)], LARGE, SMALL) == dat[100:1100]  # large rows are fine


def test_read_error_follows_interval_order_host_only(tmp_path):
    """read_ec_shard_intervals walks a range's intervals in order with `?`
    (erasure_coding/mod.rs:311-325), so the FIRST failing interval decides the
    error. On a volume where locate.rs's two large-row counts disagree, every
    small-row interval lands past the shard ends: a range whose first interval
    is on a lost shard fails TooFewShardsPresent (its recovery finds no other
    shard reaching that far, mod.rs:461) even though its next interval, on a
    present shard, would fail Io -- decided before any device work, so no GPU
    is needed. The C oracle agrees."""
    import helyim_amd as H
    base, dat = _volume(tmp_path, 5863, seed=53)  # 608-byte shards, data_size 6080: large_block_rows 1 vs 0
    _drop(base, [8, 11])
    r = (5078, 495)  # block 158 -> shard 8 (lost) first, then shard 9 (present)
    assert corc.read_ec_data(base, [r], LARGE, SMALL)[0] == -4
    with pytest.raises(H.ErasureCoding) as ei:
        H.read_ec_data(base, [r], LARGE, SMALL)
    assert isinstance(ei.value.inner, H.TooFewShardsPresent)
    r2 = (5090, 100)  # block 159 -> shard 9 (present) first: Io, as the oracle
    assert corc.read_ec_data(base, [r2], LARGE, SMALL)[0] == -1
    with pytest.raises(H.Io):
        H.read_ec_data(base, [r2], LARGE, SMALL)


def test_read_errors_host_only(tmp_path):
    import helyim_amd as H
    with pytest.raises(H.ShardNotFound):
        H.read_ec_data(str(tmp_path / "none"), [(0, 1)], LARGE, SMALL)
    base, _ = _volume(tmp_path, 19300)
    with open(base + O.to_ext(4), "r+b") as f:  # a present shard that is too short
        f.truncate(100)
    with pytest.raises(H.Io):
        H.read_ec_data(base, [(4 * 640 + 200, 10)], LARGE, SMALL)


def _needle_volume(tmp_path, n_needles=40, seed=4):
    """A .dat with needles at 8-aligned offsets and its .idx -> .ecx."""
    rng = np.random.default_rng(seed)
    entries, pos = [], 8
    for nid in range(1, n_needles + 1):
        size = int(rng.integers(0, 900))
        body = 16 + size + 4
        actual = body + (8 - body % 8)
        entries.append((nid * 7, pos // 8, size))
        pos += actual
    size = pos + 64
    base, dat = _volume(tmp_path, size, seed=seed)
    raw = b"".join(struct.pack(">QIi", k, o, s) for k, o, s in entries)
    open(base + ".idx", "wb").write(raw)
    O.write_sorted_file_from_index(base)
    open(base + ".ecj", "wb").write(struct.pack(">Q", entries[5][0]))  # needle 6 deleted after EC
    O.rebuild_ecx_file(base)
    return base, dat, entries


def _needle_bytes(dat, off, size):
    body = 16 + size + 4
    return dat[off * 8: off * 8 + body + (8 - body % 8)]


def test_read_needles_host_only(tmp_path):
    import helyim_amd as H
    base, dat, entries = _needle_volume(tmp_path)
    for i, (k, off, size) in enumerate(entries):
        if i == 5:
            with pytest.raises(H.NeedleNotFound):
                H.read_ec_needle(base, k, LARGE, SMALL)
            with pytest.raises(O.NeedleNotFound):
                O.read_ec_needle(base, k, LARGE, SMALL)
            continue
        want = _needle_bytes(dat, off, size)
        assert O.read_ec_needle(base, k, LARGE, SMALL) == want
        assert H.read_ec_needle(base, k, LARGE, SMALL) == want
    with pytest.raises(H.Io):
        H.read_ec_needle(base, 123456789, LARGE, SMALL)


def test_read_needles_batch_host_only(tmp_path):
    import helyim_amd as H
    base, dat, entries = _needle_volume(tmp_path)
    ids = [k for k, _, _ in entries] + [999999, entries[3][0]]
    got = H.read_ec_needles(base, ids, LARGE, SMALL)
    for i, (k, off, size) in enumerate(entries):
        if i == 5:
            assert isinstance(got[i], H.NeedleNotFound)
        else:
            assert got[i] == _needle_bytes(dat, off, size)
    assert isinstance(got[len(entries)], H.Io)
    assert got[-1] == _needle_bytes(dat, entries[3][1], entries[3][2])
    assert H.read_ec_needles(base, [], LARGE, SMALL) == []


def test_default_geometry_entry_points_host_only(tmp_path):
    """hec_read_ec_needle and hec_ec_volume_open take the reference's own
    1 GiB / 1 MiB blocks (ERASURE_CODING_*_BLOCK_SIZE, lib.rs:44-50): on a
    volume coded at those blocks they read what the _ex forms read, and what
    the oracle reads, with every shard present (no GPU)."""
    import ctypes
    import helyim_amd as H
    rng = np.random.default_rng(44)
    base = str(tmp_path / "d")
    entries, pos = [], 8
    for nid in range(1, 30):
        size = int(rng.integers(0, 200_000))
        body = 16 + size + 4
        entries.append((nid * 11, pos // 8, size))
        pos += body + (8 - body % 8)
    dat = O.splitmix64_bytes(77, pos + 8).tobytes()
    open(base + ".dat", "wb").write(dat)
    assert corc.write_ec_files(base, 256 << 10, H.ERASURE_CODING_LARGE_BLOCK_SIZE,
                               H.ERASURE_CODING_SMALL_BLOCK_SIZE) == 0
    open(base + ".idx", "wb").write(b"".join(struct.pack(">QIi", k, o, s) for k, o, s in entries))
    O.write_sorted_file_from_index(base)
    lib = H.lib
    vol = ctypes.c_void_p()
    assert lib.hec_ec_volume_open(base.encode(), ctypes.byref(vol)) == 0
    try:
        for k, off, size in entries:
            want = _needle_bytes(dat, off, size)
            assert O.read_ec_needle(base, k) == want
            buf = ctypes.create_string_buffer(len(want))
            n = ctypes.c_size_t()
            assert lib.hec_read_ec_needle(base.encode(), k, buf, len(want), ctypes.byref(n)) == 0
            assert buf.raw[:n.value] == want
            buf2 = ctypes.create_string_buffer(len(want))
            assert lib.hec_ec_volume_read_needle(vol, k, buf2, len(want), ctypes.byref(n)) == 0
            assert buf2.raw[:n.value] == want
        n = ctypes.c_size_t()
        assert lib.hec_read_ec_needle(base.encode(), 5, None, 0, ctypes.byref(n)) == H.Io.code
        assert lib.hec_ec_volume_read_needle(vol, entries[0][0], None, 0, ctypes.byref(n)) != 0
        assert n.value == len(_needle_bytes(dat, entries[0][1], entries[0][2]))
    finally:
        lib.hec_ec_volume_close(vol)


# ---- degraded reads: lost data shards rebuilt on the GPU ---------------------

@pytest.mark.gpu
@pytest.mark.parametrize("lost", [(0,), (2, 7), (0, 1, 2, 3), (9, 10, 12, 13), (4, 5, 6, 11)])
def test_degraded_read_vs_oracle(gpu, tmp_path, lost):
    import helyim_amd as H
    size = 32123
    base, dat = _volume(tmp_path, size)
    _drop(base, lost)
    rng = np.random.default_rng(sum(lost) + 1)
    ranges = _ranges(rng, size, 300) + [(0, size), (size - 1, 1)]
    want = b"".join(dat[o:o + n] for o, n in ranges)
    got = H.read_ec_data(base, ranges, LARGE, SMALL)
    assert got == want
    assert O.read_ec_data(base, ranges[:40], LARGE, SMALL) == want[:sum(n for _, n in ranges[:40])]


@pytest.mark.gpu
def test_degraded_read_sweep_vs_oracle(gpu, tmp_path):
    """Seeded sweep of the degraded read (erasure_coding/mod.rs:303-491 with
    locate.rs) over volume sizes -- small rows only, large + small rows, and
    sizes where locate.rs's two large-row counts disagree (:39-40 vs :84) --
    and 0-5 lost shards, data and parity: every range is read alone and
    compared with the C oracle's outcome (bytes, Io, TooFewShardsPresent),
    then all the ranges that succeed are read again as one batch (one GPU
    round trip for every lost interval)."""
    import helyim_amd as H
    rng = np.random.default_rng(403491)
    for case in range(12):
        size = int(rng.choice([int(rng.integers(100, 6400)), int(rng.integers(6401, 40000)),
                               6400 * 2 + int(rng.integers(3000, 6400))]))
        base, dat = _volume(tmp_path, size, seed=50 + case, name=f"s{case}")
        lost = sorted(int(i) for i in rng.choice(14, int(rng.integers(0, 6)), replace=False))
        _drop(base, lost)
        ranges = _ranges(rng, size, 40, maxlen=2500)
        ok = []
        for r in ranges:
            rc, want = corc.read_ec_data(base, [r], LARGE, SMALL)
            if rc == 0:
                assert H.read_ec_data(base, [r], LARGE, SMALL) == want == dat[r[0]:r[0] + r[1]], (case, r)
                ok.append(r)
            elif rc == -4:
                with pytest.raises(H.ErasureCoding) as ei:
                    H.read_ec_data(base, [r], LARGE, SMALL)
                assert isinstance(ei.value.inner, H.TooFewShardsPresent), (case, r)
            else:
                assert rc == -1, (case, r, rc)
                with pytest.raises(H.Io):
                    H.read_ec_data(base, [r], LARGE, SMALL)
        if ok:
            assert H.read_ec_data(base, ok, LARGE, SMALL) == b"".join(dat[o:o + n] for o, n in ok), case


def _outcome_h(H, fn):
    try:
        return ("ok", fn())
    except H.NeedleNotFound:
        return ("deleted", None)
    except H.ErasureCoding as e:
        return ("rs", type(e.inner).__name__)
    except H.Io:
        return ("io", None)


def _outcome_o(fn):
    try:
        return ("ok", fn())
    except O.NeedleNotFound:
        return ("deleted", None)
    except O.RSError as e:
        return ("rs", type(e).__name__)
    except O.IoError:
        return ("io", None)


@pytest.mark.gpu
def test_degraded_needle_read_sweep_vs_oracle(gpu, tmp_path):
    """Seeded sweep of read_ec_shard_needle (erasure_coding/mod.rs:129-171):
    needle volumes of several sizes, needles deleted after EC (.ecj applied
    to .ecx), absent ids, 0-5 lost shards. Every needle read alone must give
    the oracle's outcome -- its bytes, NeedleNotFound (deleted), Io (absent
    id or a short read), TooFewShardsPresent -- and the batched read of the
    ids whose reads succeed or are not found must give the same statuses and
    bytes in one call."""
    import helyim_amd as H
    rng = np.random.default_rng(129171)
    for case in range(8):
        vdir = tmp_path / f"n{case}"
        vdir.mkdir()
        base, dat, entries = _needle_volume(vdir, n_needles=int(rng.integers(6, 80)), seed=300 + case)
        dels = [entries[int(i)][0] for i in rng.choice(len(entries), int(rng.integers(0, 4)), replace=False)]
        with open(base + ".ecj", "ab") as f:
            for k in dels:
                f.write(struct.pack(">Q", k))
        O.rebuild_ecx_file(base)
        lost = sorted(int(i) for i in rng.choice(14, int(rng.integers(0, 6)), replace=False))
        _drop(base, lost)
        ids = [k for k, _, _ in entries] + [int(x) for x in rng.integers(1, 10 ** 6, 3)]
        solo = {}
        for k in ids:
            got = _outcome_h(H, lambda: H.read_ec_needle(base, k, LARGE, SMALL))
            want = _outcome_o(lambda: O.read_ec_needle(base, k, LARGE, SMALL))
            assert got == want, (case, lost, k, got[0], want[0])
            solo[k] = got
        for k, off, size in entries:
            if solo[k][0] == "ok":
                assert solo[k][1] == _needle_bytes(dat, off, size), (case, k)
        batch_ids = [k for k in ids if solo[k][0] in ("ok", "deleted") or k not in {e[0] for e in entries}]
        res = H.read_ec_needles(base, batch_ids, LARGE, SMALL)
        for k, r in zip(batch_ids, res):
            kind = solo[k][0]
            if kind == "ok":
                assert r == solo[k][1], (case, k)
            elif kind == "deleted":
                assert isinstance(r, H.NeedleNotFound), (case, k)
            else:
                assert isinstance(r, H.Io), (case, k)


@pytest.mark.gpu
def test_degraded_needle_reads(gpu, tmp_path):
    import helyim_amd as H
    base, dat, entries = _needle_volume(tmp_path, n_needles=120)
    _drop(base, [1, 4, 8, 13])
    for i, (k, off, size) in enumerate(entries):
        if i == 5:
            with pytest.raises(H.NeedleNotFound):
                H.read_ec_needle(base, k, LARGE, SMALL)
            continue
        assert H.read_ec_needle(base, k, LARGE, SMALL) == _needle_bytes(dat, off, size), k


@pytest.mark.gpu
def test_degraded_needle_batch(gpu, tmp_path):
    import helyim_amd as H
    base, dat, entries = _needle_volume(tmp_path, n_needles=300, seed=6)
    _drop(base, [0, 2, 3, 9])
    got = H.read_ec_needles(base, [k for k, _, _ in entries], LARGE, SMALL)
    for i, (k, off, size) in enumerate(entries):
        if i == 5:
            assert isinstance(got[i], H.NeedleNotFound)
        else:
            assert got[i] == _needle_bytes(dat, off, size), k


@pytest.mark.gpu
def test_degraded_read_default_geometry(gpu, tmp_path):
    """1 GiB / 1 MiB blocks on a 3 MB volume (small rows only)."""
    import helyim_amd as H
    base = str(tmp_path / "v")
    vol = O.synthetic_volume(3_000_000).tobytes()
    open(base + ".dat", "wb").write(vol)
    H.write_ec_files(base)
    _drop(base, [0, 5, 9, 12])
    rng = np.random.default_rng(8)
    ranges = _ranges(rng, len(vol), 200, maxlen=300_000)
    assert H.read_ec_data(base, ranges) == b"".join(vol[o:o + n] for o, n in ranges)


@pytest.mark.gpu
def test_degraded_read_too_many_lost(gpu, tmp_path):
    import helyim_amd as H
    base, dat = _volume(tmp_path, 19300)
    _drop(base, [0, 1, 2, 3, 4])
    assert H.read_ec_data(base, [(5 * 640 + 3, 600)], LARGE, SMALL) == dat[5 * 640 + 3:5 * 640 + 603]
    with pytest.raises(H.ErasureCoding) as ei:
        H.read_ec_data(base, [(100, 10)], LARGE, SMALL)
    assert isinstance(ei.value.inner, H.TooFewShardsPresent)
    with pytest.raises(O.RSError):
        O.read_ec_data(base, [(100, 10)], LARGE, SMALL)


# ---- mounted volume handle (EcVolume, helyim-ec/src/volume/mod.rs) ------------

def test_ec_volume_mount_vif_and_ecj(tmp_path):
    """EcVolume::new: .ecj created, .vif written with version 2 when missing or
    when its `files` list is empty (maybe_load_volume_info), kept otherwise."""
    import json
    import os
    import helyim_amd as H
    base, _, _ = _needle_volume(tmp_path)
    twin = str(tmp_path / "twin")
    import shutil
    for ext in (".ecx",):
        shutil.copyfile(base + ext, twin + ext)
    for b in (base, twin):
        for ext in (".ecj", ".vif"):
            if os.path.exists(b + ext):
                os.remove(b + ext)
    with H.EcVolume(base, LARGE, SMALL) as v:
        assert v.version == O.ec_volume_open_version(twin) == 2
        assert v.shard_ids() == list(range(14))
    for ext in (".ecj", ".vif"):
        assert open(base + ext, "rb").read() == open(twin + ext, "rb").read()
    H.save_volume_info(base + ".vif", 3)  # files empty -> rewritten as version 2
    with H.EcVolume(base, LARGE, SMALL) as v:
        assert v.version == 2
    assert open(base + ".vif", "rb").read() == O.volume_info_json(2)
    info = {"files": [{"backend_type": "s3", "key": "k"}], "version": 3, "replication": ""}
    open(base + ".vif", "w").write(json.dumps(info))
    with H.EcVolume(base, LARGE, SMALL) as v:
        assert v.version == 3
    assert json.loads(open(base + ".vif").read()) == info
    _drop(base, [2, 11])
    with H.EcVolume(base, LARGE, SMALL) as v:
        assert v.shard_ids() == [i for i in range(14) if i not in (2, 11)]
    os.remove(base + ".ecx")
    with pytest.raises(H.Io):
        H.EcVolume(base, LARGE, SMALL)


def test_ec_volume_reads_host_only(tmp_path):
    import helyim_amd as H
    base, dat, entries = _needle_volume(tmp_path)
    with H.EcVolume(base, LARGE, SMALL) as v:
        for i, (k, off, size) in enumerate(entries):
            assert v.find_needle_from_ecx(k) == H.find_needle_from_ecx(base, k)
            if i == 5:
                with pytest.raises(H.NeedleNotFound):
                    v.read_needle(k)
                continue
            assert v.read_needle(k) == _needle_bytes(dat, off, size)
        got = v.read_needles([k for k, _, _ in entries] + [999999])
        assert got[:5] + got[6:-1] == [_needle_bytes(dat, o, s) for i, (_, o, s) in enumerate(entries) if i != 5]
        assert isinstance(got[5], H.NeedleNotFound) and isinstance(got[-1], H.Io)
        with pytest.raises(H.Io, match="is not found"):
            v.read_needle(123456789)


def test_ec_volume_delete_needle(tmp_path):
    """delete_needle_from_ecx: .ecx tombstone + .ecj append, byte-identical to
    the oracle; the needle then reads as deleted; an absent id writes nothing."""
    import shutil
    import helyim_amd as H
    base, dat, entries = _needle_volume(tmp_path)
    twin = str(tmp_path / "twin")
    shutil.copyfile(base + ".ecx", twin + ".ecx")
    with H.EcVolume(base, LARGE, SMALL) as v:
        O.ec_volume_open_version(twin)
        for i in (0, 17, 39):
            k = entries[i][0]
            v.delete_needle_from_ecx(k)
            O.ec_volume_delete_needle(twin, k)
            with pytest.raises(H.NeedleNotFound):
                v.read_needle(k)
            assert v.find_needle_from_ecx(k) == (entries[i][1], -1)
        before = (open(base + ".ecx", "rb").read(), open(base + ".ecj", "rb").read())
        with pytest.raises(H.Io, match="is not found"):
            v.delete_needle_from_ecx(424242)
        assert (open(base + ".ecx", "rb").read(), open(base + ".ecj", "rb").read()) == before
        assert v.read_needle(entries[1][0]) == _needle_bytes(dat, entries[1][1], entries[1][2])
    for ext in (".ecx", ".ecj"):
        assert open(base + ext, "rb").read() == open(twin + ext, "rb").read()
    H.rebuild_ecx_file(base)  # replaying the .ecj is idempotent on the tombstones
    O.rebuild_ecx_file(twin)
    assert open(base + ".ecx", "rb").read() == open(twin + ".ecx", "rb").read()


@pytest.mark.gpu
def test_ec_volume_degraded_reads_concurrent(gpu, tmp_path):
    """Degraded reads through one mounted handle from 8 threads at once."""
    import threading
    import helyim_amd as H
    base, dat, entries = _needle_volume(tmp_path, n_needles=200, seed=7)
    _drop(base, [1, 4, 8, 13])
    errors = []
    with H.EcVolume(base, LARGE, SMALL) as v:
        def worker(t):
            try:
                for i in range(t, len(entries), 8):
                    k, off, size = entries[i]
                    if i == 5:
                        continue
                    if v.read_needle(k) != _needle_bytes(dat, off, size):
                        errors.append(k)
                got = v.read_needles([k for k, _, _ in entries[t::8]])
                for (k, off, size), g in zip(entries[t::8], got):
                    if not isinstance(g, Exception) and g != _needle_bytes(dat, off, size):
                        errors.append(k)
            except Exception as e:  # noqa: BLE001
                errors.append(repr(e))
        th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
        for x in th:
            x.start()
        for x in th:
            x.join()
    assert not errors


@pytest.mark.gpu
def test_degraded_read_worker_error_reaches_the_caller(gpu, tmp_path):
    """a survivor read that fails inside the batched
    degraded read runs on a host-pool worker once the interval's 10 survivor
    reads total >= 256 KiB (parallel_io_for); its detail and values must come
    back on the caller's thread, not the caller's stale ones. A 600 KB needle
    in shard 0's block is lost (shard 0 dropped); after mounting, survivor
    shard 5 is truncated, so its read returns short: Io "shard shrank", errno
    0 -- and not the "is not found" Io the same thread raised just before."""
    import helyim_amd as H
    size = 600_000
    body = 16 + size + 4
    actual = body + (8 - body % 8)
    base = str(tmp_path / "big")
    dat = O.splitmix64_bytes(77, 8 + actual + 64).tobytes()
    open(base + ".dat", "wb").write(dat)
    H.write_ec_files(base)
    open(base + ".idx", "wb").write(struct.pack(">QIi", 7, 1, size))
    O.write_sorted_file_from_index(base)
    _drop(base, [0])
    with H.EcVolume(base) as v:
        assert v.read_needle(7) == _needle_bytes(dat, 1, size)  # degraded read, intact survivors
        with open(base + O.to_ext(5), "r+b") as f:
            f.truncate(0)
        with pytest.raises(H.Io, match="is not found"):
            v.read_needle(123456789)  # leaves a stale Io detail on this thread
        with pytest.raises(H.Io) as ei:
            v.read_needle(7)
    assert "shrank" in ei.value.detail and O.to_ext(5) in ei.value.detail, ei.value.detail
    assert ei.value.errno == 0 and ei.value.os_error is None

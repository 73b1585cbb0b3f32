"""EC volume files around the shards: .ecx sorted
index, .ecj tombstones, .vif, and the EC -> volume decoder. Host-side byte
formats in libhec, checked against the oracle's restatement (CPU only)."""
import os
import struct

import numpy as np
import pytest

from oracle import rs_oracle as O


def _idx(rng, n, keys=200):
    """Random .idx journal: sets, re-sets, deletes (offset 0 or size -1)."""
    out = b""
    for _ in range(n):
        k = int(rng.integers(0, keys))
        r = rng.random()
        if r < 0.15:
            out += struct.pack(">QIi", k, 0, int(rng.integers(1, 5000)))
        elif r < 0.3:
            out += struct.pack(">QIi", k, int(rng.integers(1, 1 << 20)), -1)
        else:
            out += struct.pack(">QIi", k, int(rng.integers(1, 1 << 31)), int(rng.integers(0, 1 << 20)))
    return out


@pytest.mark.parametrize("seed", range(5))
def test_sorted_index_and_tombstones(tmp_path, seed):
    import helyim_amd as H
    rng = np.random.default_rng(seed)
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    raw = _idx(rng, 600)
    for base in (a, b):
        open(base + ".idx", "wb").write(raw)
    H.write_sorted_file_from_index(a)
    O.write_sorted_file_from_index(b)
    ecx = open(a + ".ecx", "rb").read()
    assert ecx == open(b + ".ecx", "rb").read()
    keys = [struct.unpack(">Q", ecx[i:i + 8])[0] for i in range(0, len(ecx), 16)]
    assert keys == sorted(set(keys))
    ids = b"".join(struct.pack(">Q", int(k)) for k in rng.integers(0, 260, 50)) + b"\x01\x02\x03"
    for base in (a, b):
        open(base + ".ecj", "wb").write(ids)
    H.rebuild_ecx_file(a)
    O.rebuild_ecx_file(b)
    assert open(a + ".ecx", "rb").read() == open(b + ".ecx", "rb").read()
    assert not os.path.exists(a + ".ecj")
    H.rebuild_ecx_file(a)  # no .ecj: no-op


def test_sorted_index_known_answer(tmp_path):
    import helyim_amd as H
    base = str(tmp_path / "v")
    raw = (struct.pack(">QIi", 9, 10, 100) + struct.pack(">QIi", 3, 20, 5) + struct.pack(">QIi", 9, 30, 7)
           + struct.pack(">QIi", 5, 0, 9) + struct.pack(">QIi", 4, 40, 1) + struct.pack(">QIi", 4, 41, -1))
    open(base + ".idx", "wb").write(raw)
    H.write_sorted_file_from_index(base)
    assert open(base + ".ecx", "rb").read() == struct.pack(">QIi", 3, 20, 5) + struct.pack(">QIi", 9, 30, 7)


def test_partial_index_entry_is_unexpected_eof(tmp_path):
    import helyim_amd as H
    base = str(tmp_path / "v")
    open(base + ".idx", "wb").write(struct.pack(">QIi", 1, 2, 3) + b"\x00" * 5)
    with pytest.raises(H.Io):
        H.write_sorted_file_from_index(base)
    assert not os.path.exists(base + ".ecx")
    with pytest.raises(O.IoError):
        O.write_sorted_file_from_index(base)


def test_volume_info(tmp_path):
    import helyim_amd as H
    p = str(tmp_path / "v.vif")
    H.save_volume_info(p, 3)
    assert open(p, "rb").read() == O.volume_info_json(3) == b'{"files":[],"version":3,"replication":""}'


@pytest.mark.parametrize("seed", range(3))
def test_find_data_filesize_and_index_file(tmp_path, seed):
    import helyim_amd as H
    rng = np.random.default_rng(100 + seed)
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    raw = _idx(rng, 300)
    raw += struct.pack(">QIi", 999, (1 << 29) + 5, 77)  # offset*8 wraps u32 like the reference
    for base in (a, b):
        open(base + ".idx", "wb").write(raw)
        open(base + ".ec00", "wb").write(bytes([3, 0, 1, 4, 0, 0, 0, 0]) + b"x" * 100)
    H.write_sorted_file_from_index(a)
    O.write_sorted_file_from_index(b)
    assert H.find_data_filesize(a) == O.find_data_filesize(b)
    ids = b"".join(struct.pack(">Q", int(k)) for k in rng.integers(0, 200, 20))
    for base in (a, b):
        open(base + ".ecj", "wb").write(ids)
    H.write_index_file_from_ec_index(a)
    O.write_index_file_from_ec_index(b)
    assert open(a + ".idx", "rb").read() == open(b + ".idx", "rb").read()
    open(a + ".ec00", "r+b").write(bytes([3, 0, 1, 9]))  # TTL unit 9: invalid
    with pytest.raises(H.Io):
        H.find_data_filesize(a)


@pytest.mark.parametrize("size", [1, 1000, (1 << 20) * 10 + 17, (1 << 20) * 25])
def test_write_data_file_roundtrip(tmp_path, size):
    """.dat -> shards (oracle file layer) -> write_data_file(.dat size) == original."""
    import helyim_amd as H
    base = str(tmp_path / "v")
    dat = O.splitmix64_bytes(size, size).tobytes()
    open(base + ".dat", "wb").write(dat)
    O.write_ec_files(base)
    os.remove(base + ".dat")
    H.write_data_file(base, size)
    assert open(base + ".dat", "rb").read() == dat
    os.rename(base + ".dat", base + ".h")
    O.write_data_file(base, size)
    assert open(base + ".dat", "rb").read() == dat
    with open(base + ".ec03", "r+b") as f:
        f.truncate(10)
    if size > 3 << 20:
        with pytest.raises(H.Io):
            H.write_data_file(base, size)

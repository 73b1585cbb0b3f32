"""One EC volume through helyim's whole EC-tier lifecycle on the GPU, every
file compared byte for byte with the oracle's restatement of the same step
(the reference's own geometry: 1 GiB large / 1 MiB small blocks):

  VolumeEcShardsGenerate   .idx -> .ecx, .dat -> .ec00-.ec13, .vif
                           (helyim-store/src/server.rs:466-475)
  EcVolume delete          .ecx tombstone + .ecj append (volume/mod.rs:157-171)
  VolumeEcShardsRebuild    lost shards rebuilt, .ecj folded into .ecx
                           (server.rs:497-498)
  degraded needle reads    lost intervals rebuilt from survivors
                           (erasure_coding/mod.rs:129-171, 403-491)
  VolumeEcShardsToVolume   .ec00-.ec09 -> .dat, .ecx + .ecj -> .idx
                           (server.rs:701-724, decoder.rs:22-180)

The GF work runs in libhec's kernels (generate, rebuild, degraded reads); the
.ecx / .ecj / .vif / decoder steps are host byte formats that ride along, so
this is their GPU-box test inside the path that produces their inputs."""
import os
import shutil
import struct

import numpy as np
import pytest

from oracle import corc
from oracle import rs_oracle as O

pytestmark = pytest.mark.gpu


def _make_volume(d, name, n_needles, seed):
    """A .dat (8-byte superblock, version 3, then needle records at 8-aligned
    offsets) and its .idx (16-byte big-endian entries, two later deletions)."""
    rng = np.random.default_rng(seed)
    base = os.path.join(d, name)
    entries, pos, recs = [], 8, [bytes([3, 0, 0, 0, 0, 0, 0, 0])]
    for j in range(n_needles):
        size = int(rng.integers(0, 60000))
        body = 16 + size + 4
        actual = body + (8 - body % 8)
        key = 1000 + 3 * j
        recs.append(rng.integers(0, 256, actual, dtype=np.uint8).tobytes())
        entries.append((key, pos // 8, size))
        pos += actual
    dat = b"".join(recs)
    open(base + ".dat", "wb").write(dat)
    idx = [struct.pack(">QIi", k, o, s) for k, o, s in entries]
    idx.append(struct.pack(">QIi", entries[7][0], 0, -1))  # deleted before EC
    idx.append(struct.pack(">QIi", entries[8][0], entries[8][1], -1))
    open(base + ".idx", "wb").write(b"".join(idx))
    return base, dat, entries


def _needle(dat, off, size):
    body = 16 + size + 4
    return dat[off * 8: off * 8 + body + (8 - body % 8)]


def _files_equal(a, b, exts):
    for ext in exts:
        pa, pb = a + ext, b + ext
        assert os.path.exists(pa) == os.path.exists(pb), ext
        if os.path.exists(pa):
            assert open(pa, "rb").read() == open(pb, "rb").read(), ext


SHARDS = [O.to_ext(i) for i in range(14)]


def test_ec_volume_lifecycle_vs_oracle(gpu, tmp_path):
    import helyim_amd as H
    ours, theirs = tmp_path / "gpu", tmp_path / "oracle"
    ours.mkdir()
    theirs.mkdir()
    base, dat, entries = _make_volume(str(ours), "7", n_needles=150, seed=11)  # ~4.5 MB: 1 small row
    twin = str(theirs / "7")
    for ext in (".dat", ".idx"):
        shutil.copyfile(base + ext, twin + ext)

    # 1. VolumeEcShardsGenerate
    H.volume_ec_shards_generate(base, 3)
    O.write_sorted_file_from_index(twin)
    assert corc.write_ec_files(twin) == 0
    open(twin + ".vif", "wb").write(O.volume_info_json(3))
    _files_equal(base, twin, [".ecx", ".vif"] + SHARDS)

    # 2. deletes through a mounted EcVolume
    gone = [entries[i][0] for i in (0, 33, 149)]
    with H.EcVolume(base) as v:
        # EcVolume::new ignores a .vif whose `files` list is empty -- which is
        # what the generate RPC writes -- and rewrites it as version 2
        # (volume/mod.rs:66-77, volume_info.rs:107-119); so does the oracle
        assert v.version == 2 and v.shard_ids() == list(range(14))
        for k in gone:
            v.delete_needle_from_ecx(k)
    assert O.ec_volume_open_version(twin) == 2
    for k in gone:
        O.ec_volume_delete_needle(twin, k)
    _files_equal(base, twin, [".ecx", ".ecj", ".vif"])

    # 3. VolumeEcShardsRebuild with 4 shards lost (data and parity)
    lost = [0, 3, 11, 13]
    for i in lost:
        os.remove(base + O.to_ext(i))
        os.remove(twin + O.to_ext(i))
    assert H.volume_ec_shards_rebuild(base) == lost
    rc, ids = corc.rebuild_ec_files(twin)
    assert rc == 0 and ids == lost
    O.rebuild_ecx_file(twin)
    _files_equal(base, twin, [".ecx", ".ecj"] + SHARDS)
    assert not os.path.exists(base + ".ecj")

    # 4. degraded needle reads: two data shards lost again, every needle read
    for i in (1, 5):
        shutil.move(base + O.to_ext(i), base + O.to_ext(i) + ".keep")
    deleted = set(gone) | {entries[7][0], entries[8][0]}
    with H.EcVolume(base) as v:
        got = v.read_needles([k for k, _, _ in entries])
    for (k, off, size), g in zip(entries, got):
        if k in deleted:
            assert isinstance(g, (H.NeedleNotFound, H.Io)), k
        else:
            assert g == _needle(dat, off, size), k
    for i in (1, 5):
        shutil.move(base + O.to_ext(i) + ".keep", base + O.to_ext(i))

    # 5. VolumeEcShardsToVolume
    for b in (base, twin):
        os.remove(b + ".dat")
        os.remove(b + ".idx")
    size = H.find_data_filesize(base)
    assert size == O.find_data_filesize(twin)
    H.write_data_file(base, size)
    O.write_data_file(twin, size)
    H.write_index_file_from_ec_index(base)
    O.write_index_file_from_ec_index(twin)
    _files_equal(base, twin, [".dat", ".idx"])
    # the decoded volume is the original up to its last live needle
    assert open(base + ".dat", "rb").read() == dat[:size]

"""The drop-in boundary without a GPU: libhec loads, exports every symbol the
header declares, and its host-side logic (geometry, matrix, argument/error
checks that precede any device work) behaves like upstream."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT, has_gpu
from oracle import rs_oracle as O

HEADER = os.path.join(ROOT, "include", "hec.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hec_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_exports_header():
    import helyim_amd
    from helyim_amd import _lib
    names = declared_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(helyim_amd.lib, n), n
        assert n in _lib.SIGNATURES, n
    assert "gfx950" in helyim_amd.version()


def test_speed_settings_are_the_three_host_path_knobs():
    """hec.h keeps only settings whose non-default value a
    product path uses (the host paths' staging threshold, zero copy or SDMA
    copies, completion-flag threshold); kernel choice has no knob, and the
    removed measurement switches are gone from the library too."""
    import helyim_amd
    setters = [n for n in declared_functions() if n.startswith("hec_set_")]
    assert sorted(setters) == ["hec_set_completion_signal", "hec_set_device", "hec_set_host_staging",
                               "hec_set_host_zero_copy"]
    for gone in ("hec_set_launch_config", "hec_set_kernel_mode", "hec_set_workgroup_size",
                 "hec_set_decode_vector_bytes", "hec_set_encode_vector_bytes", "hec_set_encode_kernel",
                 "hec_set_bitslice_vector_bytes", "hec_set_ragged_encode_remap", "hec_set_host_encode_narrow",
                 "hec_set_xcd_parts", "hec_set_chunk_rotation", "hec_set_file_zero_copy", "hec_file_path_stats"):
        assert not hasattr(helyim_amd.lib, gone), gone


def test_library_is_gfx950_code_object():
    so = os.path.join(ROOT, "helyim_amd", "libhec.so")
    blob = open(so, "rb").read()
    assert b"gfx950" in blob


def test_status_codes_and_strings():
    from helyim_amd import _lib, errors
    assert _lib.strerror(0) == "ok"
    assert "smaller than number of parity shards" in _lib.strerror(errors.TooFewShardsPresent.code)
    assert "ec shard size expected" in _lib.strerror(errors.UnexpectedEcShardSize.code)


def test_rs_new_errors():
    import helyim_amd as H
    with pytest.raises(H.TooFewDataShards):
        H.ReedSolomon(0, 4)
    with pytest.raises(H.TooFewParityShards):
        H.ReedSolomon(10, 0)
    with pytest.raises(H.TooManyShards):
        H.ReedSolomon(250, 7)
    rs = H.ReedSolomon(128, 128)
    assert rs.total_shard_count() == 256


@pytest.mark.parametrize("k,m", [(10, 4), (5, 5), (3, 2), (17, 3), (1, 1), (200, 56)])
def test_matrix_matches_oracle(k, m):
    import helyim_amd as H
    from oracle import rs_oracle as O
    assert np.array_equal(H.ReedSolomon(k, m).matrix(), O.build_matrix(k, k + m))


def test_argument_errors_before_device():
    import helyim_amd as H
    rs = H.ReedSolomon(10, 4)
    L = 64
    sh = [np.zeros(L, np.uint8) for _ in range(14)]
    with pytest.raises(H.TooFewShards):
        rs.encode(sh[:13])
    with pytest.raises(H.TooManyShards):
        rs.encode(sh + [np.zeros(L, np.uint8)])
    with pytest.raises(H.EmptyShard):
        rs.encode([np.zeros(0, np.uint8)] + sh[1:])
    with pytest.raises(H.IncorrectShardSize):
        rs.encode(sh[:13] + [np.zeros(L + 1, np.uint8)])
    with pytest.raises(H.TooFewShardsPresent):
        rs.reconstruct([None] * 5 + sh[5:])
    with pytest.raises(H.IncorrectShardSize):
        rs.reconstruct([None] + sh[1:13] + [np.zeros(3, np.uint8)])
    with pytest.raises(H.TooFewShards):
        rs.reconstruct(sh[:12])
    # all present: upstream no-op, no device work
    rs.reconstruct(list(sh))


@pytest.mark.skipif(has_gpu(), reason="checks the no-GPU error path")
def test_no_cpu_fallback():
    import helyim_amd as H
    rs = H.ReedSolomon(10, 4)
    sh = [np.ones(64, np.uint8) for _ in range(14)]
    with pytest.raises(H.DeviceError) as ei:
        rs.encode(sh)
    assert ei.value.code == 65  # HEC_ERR_NO_DEVICE
    for call in (H.device_count, H.get_device, lambda: H.set_device(0)):
        with pytest.raises(H.DeviceError) as ei:
            call()
        assert ei.value.code == 65


def test_constants_and_ext():
    import helyim_amd as H
    assert (H.DATA_SHARDS_COUNT, H.PARITY_SHARDS_COUNT, H.TOTAL_SHARDS_COUNT) == (10, 4, 14)
    assert H.ERASURE_CODING_LARGE_BLOCK_SIZE == 1 << 30
    assert H.ERASURE_CODING_SMALL_BLOCK_SIZE == 1 << 20
    assert [H.to_ext(i) for i in (0, 9, 13)] == [".ec00", ".ec09", ".ec13"]
    # shard.rs:51-65 naming
    assert H.ec_shard_filename("", "/data", 7) == "/data/7"
    assert H.ec_shard_filename("pics", "/data", 7) == "/data/pics_7"
    assert H.ec_shard_base_filename("", 42) == "42"
    assert H.ec_shard_base_filename("pics", 42) == "pics_42"
    assert H.ec_shard_filename("c", "d", 3) + H.to_ext(13) == "d/c_3.ec13"


def test_file_layer_io_errors(tmp_path):
    """EcShardError::Io carries the io::Error: the errno comes back through
    hec_last_error_values (encoder.rs:58-62 opens the .dat with `?`)."""
    import errno

    import helyim_amd as H
    with pytest.raises(H.Io) as ei:
        H.write_ec_files(str(tmp_path / "missing"))
    assert ei.value.errno == errno.ENOENT
    assert isinstance(ei.value.os_error, FileNotFoundError)
    assert str(ei.value).startswith("Io error: open ") and str(ei.value).endswith("(os error 2)")
    # an unwritable output directory: the first shard file's open fails
    ro = tmp_path / "ro"
    ro.mkdir()
    open(ro / "v.dat", "wb").write(b"x" * 100)
    os.chmod(ro, 0o500)
    try:
        if os.access(ro, os.W_OK):  # root ignores the mode bits
            pytest.skip("running as root: directory permissions are not enforced")
        with pytest.raises(H.Io) as ei:
            H.write_ec_files(str(ro / "v"))
        assert ei.value.errno == errno.EACCES
    finally:
        os.chmod(ro, 0o700)


def test_file_layer_size_errors_carry_helyims_values(tmp_path):
    """UnexpectedBlockSize(block_size, buf_size) (encoder.rs:139-144) and
    UnexpectedEcShardSize(expected, actual) (encoder.rs:272-280) come back with
    both usizes (hec_last_error_values), checked before any device work: the
    large-row block check precedes the first row, and a rebuild whose first
    row already disagrees never reaches the GPU."""
    import helyim_amd as H
    from helyim_amd import _lib
    base = str(tmp_path / "v")
    open(base + ".dat", "wb").write(b"x" * (10 * 640 + 1))  # one large row (strict '>')
    with pytest.raises(H.UnexpectedBlockSize) as ei:
        H.generate_ec_files(base, 24, 640, 32)
    assert ei.value.values == (640, 24) and (ei.value.block_size, ei.value.buf_size) == (640, 24)
    assert str(ei.value) == "unexpected block size 640, buffer size 24"
    assert _lib.last_values() == (640, 24, 0)

    rb = str(tmp_path / "r")
    for i in range(14):
        if i != 2:
            open(rb + H.to_ext(i), "wb").write(bytes(999 if i == 5 else 1000))
    with pytest.raises(H.UnexpectedEcShardSize) as ei:
        H.rebuild_ec_files(rb)
    assert (ei.value.expected, ei.value.actual) == (1000, 999)
    assert str(ei.value) == "ec shard size expected 1000 but actually is 999"
    # a payload-free failure afterwards does not leak the old values into Io
    with pytest.raises(H.Io) as ei:
        H.write_ec_files(str(tmp_path / "missing"))
    assert _lib.last_values() == (0, 0, 2)


def test_underflow_display_mirrors_helyims_format():
    """errors.rs:60 formats Underflow with {0} twice; the mirror keeps that."""
    import helyim_amd as H
    e = H.Underflow(3, 10)
    assert e.values == (3, 10) and str(e) == "Only 3 shards found but 3 required"


def test_reconstruct_batch_validation_before_device():
    import helyim_amd as H
    rs = H.ReedSolomon(10, 4)
    good = [np.zeros(8, np.uint8) for _ in range(14)]
    rs.reconstruct_batch([list(good), list(good)])  # all present: no-op, no device work
    bad = [None] * 5 + [np.zeros(8, np.uint8) for _ in range(9)]
    with pytest.raises(H.TooFewShardsPresent) as ei:
        rs.reconstruct_batch([list(good), bad])
    assert ei.value.stripe == 1
    with pytest.raises(H.IncorrectShardSize) as ei:
        rs.reconstruct_batch([[None] + good[1:13] + [np.zeros(9, np.uint8)]])
    assert ei.value.stripe == 0


def test_kernel_selection_follows_the_shard_length():
    """The encode-kernel report follows the shard length (no device work):
    bit-sliced on multiples of 8 KiB, the 16-byte table kernel on other
    16-byte multiples; the host-zero-copy knob takes 0 and 1."""
    import helyim_amd as H
    lib = H.lib
    assert lib.hec_encode_kernel_name(1 << 20).decode() == "rs104_bs_encode_kernel (bit-sliced)"
    assert lib.hec_encode_kernel_name(8192).decode() == "rs104_bs_encode_kernel (bit-sliced)"
    assert lib.hec_encode_kernel_name(8192 + 16).decode().startswith("rs104_kernel<DEC=false>")
    assert lib.hec_encode_kernel_name(4096).decode().startswith("rs104_kernel<DEC=false>")
    assert lib.hec_encode_kernel_name(17).decode().startswith("rs104_kernel<DEC=false>")
    assert lib.hec_set_host_zero_copy(0) == 0 and lib.hec_set_host_zero_copy(1) == 0


@pytest.mark.parametrize("k,m", [(10, 4), (3, 2)])
def test_argument_errors_match_the_oracle_sweep(k, m):
    """Seeded sweep of the per-call API's argument checks against the
    oracle's restatement of upstream's (slot count, then each present shard
    in index order: EmptyShard, IncorrectShardSize; then all present -> no-op,
    then TooFewShardsPresent): random slot counts, absent slots, empty and
    off-by-one shards, for reconstruct, reconstruct_data, encode and verify.
    Every check precedes device work, so the error (or its absence) is
    compared here without a GPU; where the oracle accepts the input, libhec
    either needs no device (all present) or reports that it has none."""
    import helyim_amd as H
    rng = np.random.default_rng(1000 * k + m)
    n = k + m
    hrs, ors = H.ReedSolomon(k, m), O.ReedSolomon(k, m)
    gpu = has_gpu()
    for case in range(400):
        cnt = int(rng.choice([n, n, n, n - 1, n + 1]))
        L = int(rng.integers(1, 40))
        slots = []
        for _ in range(cnt):
            r = rng.random()
            if r < 0.25:
                slots.append(None)
            elif r < 0.3:
                slots.append(np.zeros(0, np.uint8))
            elif r < 0.35:
                slots.append(np.zeros(L + int(rng.choice([-1, 1])), np.uint8) if L > 1 else np.zeros(L + 1, np.uint8))
            else:
                slots.append(rng.integers(0, 256, L, dtype=np.uint8))
        for op in ("reconstruct", "reconstruct_data", "encode", "verify"):
            if op in ("encode", "verify"):
                arg = [s if s is not None else np.zeros(L, np.uint8) for s in slots]
            else:
                arg = list(slots)
            try:
                getattr(ors, op)([None if s is None else s.copy() for s in arg])
                want = None
            except Exception as e:  # the oracle's upstream error classes
                want = type(e).__name__
            try:
                getattr(hrs, op)([None if s is None else s.copy() for s in arg])
                got = None
            except H.DeviceError:
                got = "no device"
            except H.Error as e:
                got = type(e).__name__
            if want is None:
                assert got is None or (got == "no device" and not gpu), (case, op, got)
            else:
                assert got == want, (case, op, cnt, [None if s is None else len(s) for s in slots], got, want)


def test_strided_batch_geometry_checked_before_device():
    """Overlapping shards/stripes and wrapping extents are refused by the C ABI
    before any device work (fake non-null pointers are never touched)."""
    import helyim_amd as H
    lib, rs = H.lib, H.ReedSolomon(10, 4)
    P, L = 0x1000, 4096
    bad_encode = [
        (P, 14 * L, L - 16, P, 14 * L, L, L, 2),          # data shards overlap
        (P, 14 * L, L, P, 14 * L, L - 1, L, 2),           # parity shards overlap
        (P, L - 1, 10 * L, P, L, 10 * L, L, 2),           # data stripes overlap
        (P, 1 << 62, L, P, 14 * L, L, L, 8),              # extent wraps
    ]
    for args in bad_encode:
        assert lib.hec_gpu_encode_batch(rs.handle, *args, None) == 66, args
        assert lib.hec_host_encode_batch(rs.handle, *args) == 66, args
    masks = (ctypes.c_uint32 * 2)(0x3FFF, 0x3FFF)
    assert lib.hec_gpu_reconstruct_batch(rs.handle, P, 14 * L, L - 1, L, 2, P, None, None) == 66
    assert lib.hec_host_reconstruct_batch(rs.handle, P, 14 * L, L - 1, L, 2, masks, None) == 66
    assert lib.hec_host_reconstruct_batch(rs.handle, P, 1 << 63, L, L, 3, masks, None) == 66
    # the one-call *_multi host batches check the geometry and the device list
    # before starting any thread or device work
    devs = (ctypes.c_int * 2)(0, 0)
    for args in bad_encode:
        assert lib.hec_host_encode_batch_multi(rs.handle, devs, 2, *args) == 66, args
    assert lib.hec_host_reconstruct_batch_multi(rs.handle, devs, 2, P, 14 * L, L - 1, L, 2, masks, None) == 66
    assert lib.hec_host_encode_batch_multi(rs.handle, None, 0, P, 14 * L, L, P, 14 * L, L, L, 2) != 0
    many = (ctypes.c_int * 257)()
    assert lib.hec_host_encode_batch_multi(rs.handle, many, 257, P, 14 * L, L, P, 14 * L, L, L, 2) == 66


def test_decode_kernel_name_follows_dispatch():
    """hec_decode_kernel_name comes from the same choice the launcher makes
    (rs104_pick): 8 B per lane on multiples of 2 KiB, the 16-byte table kernel
    on other 16-byte multiples; there is no width knob (round 6)."""
    import helyim_amd as H
    lib = H.lib
    assert lib.hec_decode_kernel_name(1 << 20).decode() == "rs104_narrow_kernel<DEC=true, 8 B per lane> (table lookup)"
    assert lib.hec_decode_kernel_name(2048).decode().startswith("rs104_narrow_kernel<DEC=true")
    assert lib.hec_decode_kernel_name(2048 + 16).decode().startswith("rs104_kernel<DEC=true>")
    assert not hasattr(lib, "hec_set_decode_vector_bytes")
    assert lib.hec_encode_kernel_name(1 << 20).decode() == "rs104_bs_encode_kernel (bit-sliced)"


def test_kernel_choice_rule_over_many_lengths():
    """The documented rule over a sweep of 16-byte-multiple
    shard lengths: device encode bit-sliced iff L % 8 KiB == 0, else the
    16-byte table kernel; zero-copy host encode and device decode 8 B per
    lane iff L % 2 KiB == 0, else the 16-byte table kernel."""
    import helyim_amd as H
    lib = H.lib
    lens = sorted({16 * i for i in range(1, 600, 7)} | {2048 * i for i in range(1, 40)} |
                  {8192 * i + d for i in range(1, 20) for d in (0, 16, 2048)} | {1 << 20, (1 << 20) + 16, 1 << 30})
    for L in lens:
        enc = lib.hec_encode_kernel_name(L).decode()
        hst = lib.hec_host_encode_kernel_name(L).decode()
        dec = lib.hec_decode_kernel_name(L).decode()
        assert enc == ("rs104_bs_encode_kernel (bit-sliced)" if L % 8192 == 0
                       else "rs104_kernel<DEC=false> (table lookup)"), (L, enc)
        assert hst == ("rs104_narrow_kernel<DEC=false, 8 B per lane> (table lookup)" if L % 2048 == 0
                       else "rs104_kernel<DEC=false> (table lookup)"), (L, hst)
        assert dec == ("rs104_narrow_kernel<DEC=true, 8 B per lane> (table lookup)" if L % 2048 == 0
                       else "rs104_kernel<DEC=true> (table lookup)"), (L, dec)


def test_ragged_kernel_name_follows_the_launch_choice():
    """hec_ragged_kernel_name comes from the ragged launch's own pick
    (ragged_pick in intervals.cpp): bit-sliced only when every length is a
    multiple of 8 KiB; every ragged launch deals each XCD an eighth."""
    import helyim_amd.batch as B
    aligned = [(0, 65536, 65536, 0x3FFF), (14 * 65536, 8192, 8192, 0x3FF0)]
    odd = aligned + [(14 * 65536 + 14 * 8192, 8192, 4096, 0x3FFF)]
    assert B.ragged_kernel_name(aligned, False) == "rs104_bs_ragged_kernel (bit-sliced, XCD eighths)"
    assert B.ragged_kernel_name(odd, False) == "rs104_ragged_kernel<DEC=false> (table lookup, XCD eighths)"
    assert B.ragged_kernel_name(aligned, True) == "rs104_ragged_kernel<DEC=true> (table lookup, XCD eighths)"


def test_host_alloc_multi_arguments_checked_before_device():
    import helyim_amd as H
    lib = H.lib
    p = ctypes.c_void_p()
    devs = (ctypes.c_int * 2)(0, 0)
    assert lib.hec_host_alloc_multi(devs, 2, 4096, 4, None) == 66
    assert lib.hec_host_alloc_multi(None, 0, 4096, 4, ctypes.byref(p)) == 66
    assert lib.hec_host_alloc_multi(devs, 0, 4096, 4, ctypes.byref(p)) == 66
    assert lib.hec_host_alloc_multi(devs, 2, 0, 4, ctypes.byref(p)) == 66
    assert lib.hec_host_alloc_multi(devs, 2, 4096, 0, ctypes.byref(p)) == 66
    assert lib.hec_host_alloc_multi(devs, 2, 1 << 63, 4, ctypes.byref(p)) == 66  # overflows
    many = (ctypes.c_int * 257)()
    assert lib.hec_host_alloc_multi(many, 257, 4096, 4, ctypes.byref(p)) == 66
    assert p.value is None


def test_every_failure_resets_the_detail_and_values(tmp_path):
    """hec_last_error_detail / _values describe the LAST failure: an RS-level
    error after an Io failure leaves neither the old text nor the old errno."""
    import helyim_amd as H
    from helyim_amd import _lib
    with pytest.raises(H.Io):
        H.write_ec_files(str(tmp_path / "missing"))
    assert _lib.last_detail() and _lib.last_values()[2] == 2
    rs = H.ReedSolomon(10, 4)
    with pytest.raises(H.TooFewShards):
        rs.encode([np.zeros(8, np.uint8) for _ in range(13)])
    assert _lib.last_detail() == "" and _lib.last_values() == (0, 0, 0)
    with pytest.raises(H.TooFewShardsPresent):
        rs.reconstruct_batch([[np.zeros(8, np.uint8)] * 14, [None] * 5 + [np.zeros(8, np.uint8)] * 9])
    assert _lib.last_detail() == "stripe 1"


def test_host_encode_kernel_over_pcie():
    """Zero-copy host-batch encodes (the kernel streams host memory over PCIe)
    take the 8-byte-per-lane table encode where the shard length is a
    multiple of 2 KiB; device batches keep the bit-sliced kernel."""
    import helyim_amd as H
    lib = H.lib
    L = 1 << 20
    assert lib.hec_host_encode_kernel_name(L).decode().startswith("rs104_narrow_kernel<DEC=false, 8 B per lane>")
    assert lib.hec_encode_kernel_name(L).decode().startswith("rs104_bs_encode_kernel")
    assert lib.hec_host_encode_kernel_name(4096 + 16).decode().startswith("rs104_kernel<DEC=false>")
    for name in (lib.hec_host_encode_kernel_name(0), lib.hec_encode_kernel_name(0), lib.hec_decode_kernel_name(0)):
        assert name.decode().startswith("none")  # empty shards never launch


def test_batch_base_alignment_helpers():
    """bench.py --base-align: address_alignment is the
    largest power of two dividing an address; empty_stripes refuses a
    base_align that is not a power of two (and negative geometry) before it
    allocates anything."""
    import helyim_amd.batch as B
    assert B.address_alignment(0x4000_0000) == 1 << 30
    assert B.address_alignment(0x7F00_0020_0000) == 1 << 21
    assert B.address_alignment(12) == 4
    assert B.address_alignment(0) == 1 << 40
    with pytest.raises(ValueError, match="power of two"):
        B.empty_stripes(4, 14, 1 << 20, base_align=3 << 20)
    with pytest.raises(ValueError):
        B.empty_stripes(4, 14, 1 << 20, base_align=-1)

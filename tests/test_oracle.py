"""The oracle itself: pinned to the upstream KATs and the committed fixtures,
and the numpy and C restatements cross-checked against each other (CPU)."""
import os

import numpy as np
import pytest

from oracle import corc
from oracle import rs_oracle as O


def test_gf_kats(golden):
    kat = golden("upstream_kat.json")
    for a, b, out in kat["gf_mul"]:
        assert O.gf_mul(a, b) == out
        assert corc.lib().orc_gf_mul(a, b) == out
    for a, b, out in kat["gf_div"]:
        assert O.gf_div(a, b) == out
    for a, n, out in kat["gf_exp"]:
        assert O.gf_exp(a, n) == out
        assert corc.lib().orc_gf_exp(a, n) == out


def test_matrix_kats(golden):
    kat = golden("upstream_kat.json")
    mm = kat["matrix_mul"]
    out = O.mat_mul(np.array(mm["a"], np.uint8), np.array(mm["b"], np.uint8))
    assert out.tolist() == mm["out"]
    for case in kat["matrix_inverse"]:
        m = np.array(case["m"], np.uint8)
        assert O.mat_invert(m).tolist() == case["inv"]
        cinv = np.zeros_like(m)
        assert corc.lib().orc_invert(m.ctypes.data, cinv.ctypes.data, m.shape[0]) == 0
        assert cinv.tolist() == case["inv"]


def test_singular_matrix():
    m = np.array([[1, 2], [2, 4]], np.uint8)
    with pytest.raises(O.SingularMatrix):
        O.mat_invert(m)


def test_rs_5_5_one_encode(golden):
    kat = golden("upstream_kat.json")["rs_5_5_one_encode"]
    for impl in ("py", "c"):
        shards = [np.array(d, np.uint8) for d in kat["data"]] + [np.zeros(2, np.uint8) for _ in range(5)]
        if impl == "py":
            O.ReedSolomon(5, 5).encode(shards)
        else:
            corc.CReedSolomon(5, 5).encode(shards, simd=False)
        assert [s.tolist() for s in shards[5:]] == kat["parity"]


def test_rs_10_4_matrix(golden):
    kat = golden("upstream_kat.json")
    rs = O.ReedSolomon(10, 4)
    assert np.array_equal(rs.matrix[:10], np.eye(10, dtype=np.uint8))
    assert rs.parity_rows.tolist() == kat["rs_10_4_parity_rows"]
    assert corc.CReedSolomon(10, 4).matrix().tolist() == rs.matrix.tolist()
    assert golden("tables.json")["matrix_10_4"] == rs.matrix.tolist()


def test_tables_fixture(golden):
    t = golden("tables.json")
    assert O.sha256(O.EXP_TABLE[:255]) == t["exp_sha256"]
    assert O.sha256(O.LOG_TABLE[1:].astype(np.uint8)) == t["log_sha256"]
    assert O.sha256(O.MUL_TABLE) == t["mul_sha256"]


def test_splitmix_py_vs_c():
    for seed, n in [(0x5EED0000, 1), (0x5EED0000, 13), (0x5EED0007, 4096 + 5), (123, 100000)]:
        assert np.array_equal(O.splitmix64_bytes(seed, n), corc.splitmix64_bytes(seed, n))


@pytest.mark.parametrize("L", [8, 4096, 65536, 1 << 20])
def test_shard_seed_splits_the_stripe_stream(L):
    """batch.shard_seed (the padded batch fill, bench.py's layout): shard i
    filled on its own under shard_seed(seed, i, L) holds the bytes of the
    stripe's one splitmix64 stream at [i * L, (i + 1) * L); seeds near 2^64
    wrap as the C generator's uint64 arithmetic does."""
    from helyim_amd.batch import shard_seed
    for seed in (0x5EED0000, 0x5EED0000 + (3 << 20) + 17, (1 << 64) - 5):
        stream = corc.splitmix64_bytes(seed, 10 * L)
        for i in range(10):
            assert np.array_equal(corc.splitmix64_bytes(shard_seed(seed, i, L), L), stream[i * L:(i + 1) * L]), (seed, i)
    with pytest.raises(ValueError):
        shard_seed(1, 1, 12)


def test_encode_vectors_fixture(golden):
    g = golden("encode_vectors.json")
    rs = O.ReedSolomon(10, 4)
    for L, ent in g["vectors"].items():
        L = int(L)
        if L > 65536:
            continue  # 1 MiB case is covered by the C oracle below
        data = O.stripe_data(0, L)
        assert O.sha256(data) == ent["data_sha256"]
        shards = [data[i].copy() for i in range(10)] + [np.zeros(L, np.uint8) for _ in range(4)]
        rs.encode(shards)
        assert [O.sha256(s) for s in shards[10:]] == ent["parity_sha256"]
        if "parity_hex" in ent:
            assert [s.tobytes().hex() for s in shards[10:]] == ent["parity_hex"]


@pytest.mark.parametrize("simd", [False, True])
def test_c_oracle_encode_vectors(golden, simd):
    g = golden("encode_vectors.json")
    crs = corc.CReedSolomon(10, 4)
    for L, ent in g["vectors"].items():
        L = int(L)
        data = corc.splitmix64_bytes(g["seed"], 10 * L).reshape(10, L)
        shards = [data[i].copy() for i in range(10)] + [np.zeros(L, np.uint8) for _ in range(4)]
        crs.encode(shards, simd=simd)
        assert [O.sha256(s) for s in shards[10:]] == ent["parity_sha256"], L


def test_decode_matrices_fixture(golden):
    rs = O.ReedSolomon(10, 4)
    for key, ent in golden("decode_matrices.json").items():
        pat = [int(x) for x in key.split(",")]
        present = [i for i in range(14) if i not in pat]
        assert present[:10] == ent["valid"]
        assert O.mat_invert(rs.matrix[ent["valid"], :]).tolist() == ent["inverse"]


@pytest.mark.parametrize("k,m", [(10, 4), (5, 5), (3, 2), (17, 3), (4, 6), (1, 1)])
def test_reconstruct_py_vs_c(k, m):
    rng = np.random.default_rng(k * 100 + m)
    L = 257
    rs, crs = O.ReedSolomon(k, m), corc.CReedSolomon(k, m)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    full = data + [np.zeros(L, np.uint8) for _ in range(m)]
    rs.encode(full)
    cfull = [d.copy() for d in data] + [np.zeros(L, np.uint8) for _ in range(m)]
    crs.encode(cfull)
    for a, b in zip(full, cfull):
        assert np.array_equal(a, b)
    n = k + m
    for _ in range(20):
        e = int(rng.integers(1, m + 1))
        erased = sorted(rng.choice(n, e, replace=False).tolist())
        sh = [None if i in erased else full[i].copy() for i in range(n)]
        rs.reconstruct(sh)
        csh = [np.zeros(L, np.uint8) if i in erased else full[i].copy() for i in range(n)]
        assert crs.reconstruct(csh, [i not in erased for i in range(n)]) == 0
        for i in range(n):
            assert np.array_equal(sh[i], full[i])
            assert np.array_equal(csh[i], full[i])


def test_reconstruct_errors_and_data_only():
    rs = O.ReedSolomon(10, 4)
    L = 33
    full = [np.full(L, i, np.uint8) for i in range(10)] + [np.zeros(L, np.uint8) for _ in range(4)]
    rs.encode(full)
    with pytest.raises(O.TooFewShardsPresent):
        rs.reconstruct([None] * 5 + full[5:])
    with pytest.raises(O.TooFewShards):
        rs.reconstruct(full[:13])
    with pytest.raises(O.IncorrectShardSize):
        rs.reconstruct([np.zeros(3, np.uint8)] + full[1:])
    sh = [None, full[1]] + full[2:12] + [None, None]
    rs.reconstruct_data(sh)
    assert np.array_equal(sh[0], full[0]) and sh[12] is None and sh[13] is None
    with pytest.raises(O.TooFewDataShards):
        O.ReedSolomon(0, 4)
    with pytest.raises(O.TooFewParityShards):
        O.ReedSolomon(4, 0)
    with pytest.raises(O.TooManyShards):
        O.ReedSolomon(200, 57)


def _manual_layout(dat: bytes, large: int, small: int):
    """Independent statement of the encoder.rs:200-242 row layout for data shards."""
    rows = []
    remaining, pos = len(dat), 0
    while remaining > large * 10:
        rows.append((pos, large))
        pos += large * 10
        remaining -= large * 10
    while remaining > 0:
        rows.append((pos, small))
        pos += small * 10
        remaining -= small * 10
    shards = [b"" for _ in range(10)]
    for start, block in rows:
        for i in range(10):
            chunk = dat[start + i * block: start + (i + 1) * block]
            shards[i] += chunk + b"\0" * (block - len(chunk))
    return shards


@pytest.mark.parametrize("size", [1, 639, 640, 641, 2000, 6401, 6400 * 2 + 3])
def test_oracle_file_layout(tmp_path, size):
    buf, large, small = 16, 640, 32
    dat = O.splitmix64_bytes(99, size).tobytes()
    base = str(tmp_path / "v")
    open(base + ".dat", "wb").write(dat)
    O.write_ec_files(base, buf, large, small)
    expect = _manual_layout(dat, large, small)
    rs = O.ReedSolomon(10, 4)
    got = [open(base + O.to_ext(i), "rb").read() for i in range(14)]
    for i in range(10):
        assert got[i] == expect[i]
    L = len(got[0])
    shards = [np.frombuffer(g, np.uint8).copy() for g in got]
    assert rs.verify(shards) and all(len(g) == L for g in got)


def test_oracle_block_size_error(tmp_path):
    base = str(tmp_path / "v")
    open(base + ".dat", "wb").write(b"x" * 100)
    with pytest.raises(O.UnexpectedBlockSize):
        O.write_ec_files(base, 24, 640, 32)


def test_volume_fixture(golden, tmp_path):
    g = golden("volume_30mb.json")
    vol = O.synthetic_volume(g["dat_bytes"])
    assert O.sha256(vol) == g["dat_sha256"]
    assert g["shard_bytes"] == [3 * (1 << 20)] * 14


def test_c_oracle_file_layer_vs_fixture(golden, tmp_path):
    g = golden("volume_30mb.json")
    base = str(tmp_path / "1")
    open(base + ".dat", "wb").write(O.synthetic_volume(g["dat_bytes"]).tobytes())
    assert corc.write_ec_files(base) == 0
    shas = [O.sha256(open(base + O.to_ext(i), "rb").read()) for i in range(14)]
    assert shas == g["shard_sha256"]
    for drop in g["drops"]:
        for i in drop:
            os.remove(base + O.to_ext(i))
        rc, ids = corc.rebuild_ec_files(base)
        assert rc == 0 and ids == sorted(drop)
        assert [O.sha256(open(base + O.to_ext(i), "rb").read()) for i in range(14)] == g["shard_sha256"]


@pytest.mark.parametrize("size", [1, 641, 6400 * 2 + 3])
def test_c_oracle_file_layer_small_geometry(tmp_path, size):
    dat = O.splitmix64_bytes(7 + size, size).tobytes()
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    for base in (a, b):
        open(base + ".dat", "wb").write(dat)
    assert corc.write_ec_files(a, 16, 640, 32) == 0
    O.write_ec_files(b, 16, 640, 32)
    for i in range(14):
        assert open(a + O.to_ext(i), "rb").read() == open(b + O.to_ext(i), "rb").read()


# ---- the reference's file-layer edge cases, both restatements ---------------
def _files(base):
    return {i: open(base + O.to_ext(i), "rb").read() for i in range(14) if os.path.exists(base + O.to_ext(i))}


def test_oracles_zero_byte_dat(tmp_path):
    """encoder.rs:62 remaining = 0: no row loop runs (:215, :228); the 14
    files open_ec_files created and truncated (:111-127) stay empty."""
    for k, write in enumerate((lambda b: O.write_ec_files(b), lambda b: corc.write_ec_files(b))):
        base = str(tmp_path / f"z{k}")
        open(base + ".dat", "wb").close()
        open(base + O.to_ext(4), "wb").write(b"stale")
        assert write(base) in (None, 0)
        assert _files(base) == {i: b"" for i in range(14)}


@pytest.mark.parametrize("buf,large,small,written", [(16, 640, 24, 640), (24, 640, 32, 0)])
def test_oracles_block_size_error_after_written_rows(tmp_path, buf, large, small, written):
    """encode_data checks block % buf at each row (encoder.rs:139-144), after
    the rows before it were written: the files hold exactly those rows."""
    dat = O.splitmix64_bytes(77, 7400).tobytes()
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    for base in (a, b):
        open(base + ".dat", "wb").write(dat)
    with pytest.raises(O.UnexpectedBlockSize) as ei:
        O.write_ec_files(a, buf, large, small)
    assert ei.value.args == ((small if written else large), buf)
    assert corc.write_ec_files(b, buf, large, small) == -2
    fa, fb = _files(a), _files(b)
    assert fa == fb and all(len(v) == written for v in fa.values())


@pytest.mark.parametrize("short", [0, 6, 13])
def test_oracles_rebuild_stops_at_a_short_present_shard(tmp_path, short):
    """rebuild_ec_files_inner returns Ok at the first present shard whose
    read is 0 bytes (encoder.rs:268-271), before the size check (:275) and
    before the row is reconstructed or written."""
    L = 2 << 20
    rs = O.ReedSolomon(10, 4)
    sh = [O.splitmix64_bytes(700 + i, L) for i in range(10)] + [np.zeros(L, np.uint8) for _ in range(4)]
    rs.encode(sh)
    lost = [2, 11] if short not in (2, 11) else [3, 10]
    bases = [str(tmp_path / n) for n in ("a", "b")]
    for base in bases:
        for i in range(14):
            open(base + O.to_ext(i), "wb").write(sh[i].tobytes())
        os.truncate(base + O.to_ext(short), 1 << 20)
        for i in lost:
            os.remove(base + O.to_ext(i))
    assert O.rebuild_ec_files(bases[0]) == lost
    assert corc.rebuild_ec_files(bases[1]) == (0, lost)
    fa, fb = _files(bases[0]), _files(bases[1])
    assert fa == fb
    for i in lost:
        assert fa[i] == sh[i][: 1 << 20].tobytes()


@pytest.mark.parametrize("present", [10, 5, 0])
def test_oracles_rebuild_over_empty_or_no_shards(tmp_path, present):
    """Empty present shards: the first read is 0 bytes, so the rebuild
    returns the missing ids with empty outputs -- also with only 5 present
    (Ok comes before reconstruct's TooFewShardsPresent, encoder.rs:269-271 vs
    :288). No shard at all: nothing is read, reconstruct reports
    TooFewShardsPresent, all 14 outputs created empty (:96-103)."""
    bases = [str(tmp_path / n) for n in ("a", "b")]
    lost = list(range(present, 14))
    for base in bases:
        for i in range(present):
            open(base + O.to_ext(i), "wb").close()
    if present:
        assert O.rebuild_ec_files(bases[0]) == lost
        assert corc.rebuild_ec_files(bases[1]) == (0, lost)
    else:
        with pytest.raises(O.TooFewShardsPresent):
            O.rebuild_ec_files(bases[0])
        assert corc.rebuild_ec_files(bases[1])[0] == -4
    for base in bases:
        assert _files(base) == {i: b"" for i in range(14)}


# ---- a third formulation: polynomial interpolation over GF(2^8) -------------
# The construction V x inv(V[0..k]) with V[r][c] = r^c is
# the systematic evaluation code: shard r of a stripe is p(r) for the unique
# polynomial p of degree < k with p(i) = data_i at i = 0..k-1. Lagrange
# interpolation restates that without a matrix inverse (pure-Python GF
# arithmetic from log/exp tables built here, not the oracle's), so encode and
# reconstruct of both oracles are checked against a formulation that shares
# no code with them.
def _gf():
    exp, log = [0] * 512, [0] * 256
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= 0x11D
    for i in range(255, 512):
        exp[i] = exp[i - 255]
    mul = lambda a, b: 0 if a == 0 or b == 0 else exp[log[a] + log[b]]  # noqa: E731
    inv = lambda a: exp[255 - log[a]]  # noqa: E731
    return mul, inv


def _lagrange_eval(xs, ys, x0, mul, inv):
    """p(x0) for the polynomial through (xs[i], ys[i]); addition is XOR."""
    acc = 0
    for i, xi in enumerate(xs):
        num, den = 1, 1
        for j, xj in enumerate(xs):
            if j != i:
                num = mul(num, x0 ^ xj)
                den = mul(den, xi ^ xj)
        acc ^= mul(ys[i], mul(num, inv(den)))
    return acc


@pytest.mark.parametrize("k,m", [(10, 4), (5, 5), (3, 2)])
def test_encode_and_reconstruct_match_interpolation(k, m):
    mul, inv = _gf()
    rng = np.random.default_rng(100 * k + m)
    L = 9
    data = rng.integers(0, 256, (k, L), dtype=np.uint8)
    want = np.zeros((k + m, L), np.uint8)
    want[:k] = data
    for col in range(L):
        for r in range(k, k + m):
            want[r, col] = _lagrange_eval(list(range(k)), [int(v) for v in data[:, col]], r, mul, inv)
    # both oracles' encode
    rs = O.ReedSolomon(k, m)
    sh = [data[i].copy() for i in range(k)] + [np.zeros(L, np.uint8) for _ in range(m)]
    rs.encode(sh)
    assert np.array_equal(np.stack(sh), want)
    csh = [data[i].copy() for i in range(k)] + [np.zeros(L, np.uint8) for _ in range(m)]
    corc.CReedSolomon(k, m).encode(csh)
    assert np.array_equal(np.stack(csh), want)
    # any k surviving shards determine p: interpolate the lost ones back
    for _ in range(6):
        lost = sorted(int(i) for i in rng.choice(k + m, m, replace=False))
        alive = [i for i in range(k + m) if i not in lost][:k]
        for col in range(L):
            for r in lost:
                v = _lagrange_eval(alive, [int(want[i, col]) for i in alive], r, mul, inv)
                assert v == want[r, col]
        got = [None if i in lost else want[i].copy() for i in range(k + m)]
        rs.reconstruct(got)
        assert np.array_equal(np.stack(got), want), lost


def test_random_geometries_three_formulations_agree():
    """Property sweep (hypothesis, seeded): for random geometries (k data, m
    parity; k + m <= 40), shard lengths and erasure sets, the three
    independent formulations agree byte for byte -- the numpy restatement,
    the C restatement (scalar and AVX2 kernels) and Lagrange interpolation
    over GF(2^8) from its own tables (the systematic evaluation code: shard r
    = p(r) for the degree < k polynomial through the data). Reconstruct from
    any k survivors returns the codeword, and verify() flags one flipped
    byte."""
    from hypothesis import given, settings, HealthCheck, strategies as st
    mul, inv = _gf()

    @settings(max_examples=200, deadline=None, derandomize=True,
              suppress_health_check=[HealthCheck.too_slow])
    @given(st.integers(1, 30), st.integers(1, 10), st.integers(1, 24), st.integers(0, 2**32 - 1))
    def check(k, m, L, seed):
        rng = np.random.default_rng(seed)
        n = k + m
        data = rng.integers(0, 256, (k, L), dtype=np.uint8)
        want = np.zeros((n, L), np.uint8)
        want[:k] = data
        for col in range(L):
            ys = [int(v) for v in data[:, col]]
            for r in range(k, n):
                want[r, col] = _lagrange_eval(list(range(k)), ys, r, mul, inv)
        rs, crs = O.ReedSolomon(k, m), corc.CReedSolomon(k, m)
        sh = [data[i].copy() for i in range(k)] + [np.zeros(L, np.uint8) for _ in range(m)]
        rs.encode(sh)
        assert np.array_equal(np.stack(sh), want)
        for simd in (False, True):
            csh = [data[i].copy() for i in range(k)] + [np.zeros(L, np.uint8) for _ in range(m)]
            crs.encode(csh, simd=simd)
            assert np.array_equal(np.stack(csh), want)
        assert rs.verify([want[i].copy() for i in range(n)])
        bad = [want[i].copy() for i in range(n)]
        bad[int(rng.integers(0, n))][int(rng.integers(0, L))] ^= 1 + int(rng.integers(0, 255))
        assert not rs.verify(bad)
        e = int(rng.integers(1, m + 1))
        lost = sorted(int(i) for i in rng.choice(n, e, replace=False))
        got = [None if i in lost else want[i].copy() for i in range(n)]
        rs.reconstruct(got)
        assert np.array_equal(np.stack(got), want)
        cgot = [np.zeros(L, np.uint8) if i in lost else want[i].copy() for i in range(n)]
        assert crs.reconstruct(cgot, [i not in lost for i in range(n)]) == 0
        assert np.array_equal(np.stack(cgot), want)

    check()

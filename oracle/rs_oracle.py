"""CPU oracle for the helyim-ec RS(10,4) hot path -- TEST INFRASTRUCTURE ONLY.

This module is the numpy restatement of the algorithm behind helyim-ec's
erasure coding. It exists to CHECK the HIP product path (helyim_amd/libhec.so);
it is never the thing measured or shipped. Only tests/, __graft_entry__.smoke(),
bench.py's cpu_baseline leg and the measurement tools under tools/ (as the
checker of GPU outputs and as the timed CPU baseline beside them) import it;
the product package helyim_amd/ never does.

Provenance of the algorithm (the reference cannot be built here: Rust toolchain
absent, and the arithmetic lives in the un-vendored git dependency
``reed-solomon-erasure`` 6.0.0, git helyim/reed-solomon-erasure branch main,
feature ``simd-accel`` -- /root/reference/Cargo.toml:72,
/root/reference/helyim-ec/Cargo.toml:26):

* GF(2^8), generating polynomial x^8+x^4+x^3+x^2+1 (0x11D), generator 2
  -- upstream ``galois_8`` (published algorithm; restated here).
* Encoding matrix = Vandermonde(total x data), V[r][c] = exp(r, c), times the
  inverse of its top data x data square -- upstream ``ReedSolomon::new``.
* encode / reconstruct / reconstruct_data / verify semantics -- upstream
  ``ReedSolomon`` (error variants, first-k-present rule, zero-filled missing
  buffers), called from /root/reference/helyim-ec/src/encoder.rs:191,208-209,
  249-250,288 and helyim-store/src/erasure_coding/mod.rs:411-412,426.
* File layout -- /root/reference/helyim-ec/src/encoder.rs:39-307 (restated in
  ``write_ec_files`` / ``rebuild_ec_files`` below, line cites inline).

PARITY UNPINNED (by the reference): helyim has no EC tests, fixtures or golden
vectors, the arithmetic crate is not in /root/reference and Rust
cannot be built here, so nothing the reference itself produced pins this
oracle. What it is checked against instead: the upstream crate's published
known-answer tests (mul/exp/inverse KATs and the RS(5,5) one-encode vector,
committed as data in tests/golden/upstream_kat.json) and the independent C
restatement in oracle/rs_oracle.c.
"""
from __future__ import annotations

import hashlib
import os
from typing import List, Optional, Sequence

import numpy as np

# --------------------------------------------------------------------------
# GF(2^8) -- upstream galois_8 (poly 0x11D = GENERATING_POLYNOMIAL 29 | 0x100)
# --------------------------------------------------------------------------
GF_POLY = 0x11D
FIELD_SIZE = 256


def _build_tables():
    exp = np.zeros(510, dtype=np.uint8)
    log = np.zeros(256, dtype=np.int32)
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= GF_POLY
    for i in range(255, 510):
        exp[i] = exp[i - 255]
    a = np.arange(256)
    la = log[a][:, None] + log[a][None, :]
    mul = exp[la].astype(np.uint8)
    mul[0, :] = 0
    mul[:, 0] = 0
    return exp, log, mul


EXP_TABLE, LOG_TABLE, MUL_TABLE = _build_tables()


def gf_mul(a: int, b: int) -> int:
    return int(MUL_TABLE[a, b])


def gf_div(a: int, b: int) -> int:
    if a == 0:
        return 0
    if b == 0:
        raise ZeroDivisionError("divisor is 0")
    return int(EXP_TABLE[(int(LOG_TABLE[a]) - int(LOG_TABLE[b])) % 255])


def gf_exp(a: int, n: int) -> int:
    """upstream galois_8::exp: exp(a,0)=1, exp(0,n>0)=0."""
    if n == 0:
        return 1
    if a == 0:
        return 0
    return int(EXP_TABLE[(int(LOG_TABLE[a]) * n) % 255])


# --------------------------------------------------------------------------
# Matrices over GF(2^8)
# --------------------------------------------------------------------------
def mat_mul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    rows, inner = a.shape
    inner2, cols = b.shape
    assert inner == inner2
    out = np.zeros((rows, cols), dtype=np.uint8)
    for r in range(rows):
        acc = np.zeros(cols, dtype=np.uint8)
        for k in range(inner):
            acc ^= MUL_TABLE[a[r, k], b[k, :]]
        out[r] = acc
    return out


class SingularMatrix(Exception):
    pass


def mat_invert(m: np.ndarray) -> np.ndarray:
    """Gauss-Jordan inversion over GF(2^8) (upstream matrix.rs invert)."""
    n = m.shape[0]
    assert m.shape == (n, n)
    work = np.concatenate([m.astype(np.uint8), np.eye(n, dtype=np.uint8)], axis=1)
    for r in range(n):
        if work[r, r] == 0:
            for below in range(r + 1, n):
                if work[below, r] != 0:
                    work[[r, below]] = work[[below, r]]
                    break
        if work[r, r] == 0:
            raise SingularMatrix()
        if work[r, r] != 1:
            scale = gf_div(1, int(work[r, r]))
            work[r] = MUL_TABLE[scale, work[r]]
        for other in range(n):
            if other != r and work[other, r] != 0:
                work[other] ^= MUL_TABLE[int(work[other, r]), work[r]]
    return work[:, n:].copy()


def vandermonde(rows: int, cols: int) -> np.ndarray:
    v = np.zeros((rows, cols), dtype=np.uint8)
    for r in range(rows):
        for c in range(cols):
            v[r, c] = gf_exp(r, c)
    return v


def build_matrix(data_shards: int, total_shards: int) -> np.ndarray:
    """upstream ReedSolomon::new: V(total x data) * inv(V[0..data])."""
    v = vandermonde(total_shards, data_shards)
    top = v[:data_shards, :]
    return mat_mul(v, mat_invert(top))


# --------------------------------------------------------------------------
# ReedSolomon -- upstream API semantics (errors mirror reed_solomon_erasure::Error)
# --------------------------------------------------------------------------
class RSError(Exception):
    """Base of the reed_solomon_erasure::Error mirror."""


def _mk(name):
    return type(name, (RSError,), {})


TooFewShards = _mk("TooFewShards")
TooManyShards = _mk("TooManyShards")
TooFewDataShards = _mk("TooFewDataShards")
TooManyDataShards = _mk("TooManyDataShards")
TooFewParityShards = _mk("TooFewParityShards")
TooManyParityShards = _mk("TooManyParityShards")
TooFewBufferShards = _mk("TooFewBufferShards")
TooManyBufferShards = _mk("TooManyBufferShards")
IncorrectShardSize = _mk("IncorrectShardSize")
TooFewShardsPresent = _mk("TooFewShardsPresent")
EmptyShard = _mk("EmptyShard")
InvalidShardFlags = _mk("InvalidShardFlags")
InvalidIndex = _mk("InvalidIndex")


def mul_rows(coefs: np.ndarray, inputs: Sequence[np.ndarray]) -> List[np.ndarray]:
    """out[r] = XOR_i coefs[r,i] * inputs[i] (bytewise GF mul-add)."""
    outs = []
    for r in range(coefs.shape[0]):
        acc = np.zeros_like(inputs[0])
        for i, buf in enumerate(inputs):
            c = int(coefs[r, i])
            if c:
                acc ^= MUL_TABLE[c][buf]
        outs.append(acc)
    return outs


class ReedSolomon:
    def __init__(self, data_shards: int, parity_shards: int):
        if data_shards == 0:
            raise TooFewDataShards()
        if parity_shards == 0:
            raise TooFewParityShards()
        if data_shards + parity_shards > FIELD_SIZE:
            raise TooManyShards()
        self.data_shard_count = data_shards
        self.parity_shard_count = parity_shards
        self.total_shard_count = data_shards + parity_shards
        self.matrix = build_matrix(data_shards, self.total_shard_count)
        self.parity_rows = self.matrix[data_shards:, :]
        self._cache = {}

    # -- checks mirroring upstream check_piece_count!/check_slices! ---------
    def _check_count(self, n):
        if n < self.total_shard_count:
            raise TooFewShards()
        if n > self.total_shard_count:
            raise TooManyShards()

    @staticmethod
    def _check_sizes(bufs):
        size = len(bufs[0])
        if size == 0:
            raise EmptyShard()
        for b in bufs[1:]:
            if len(b) != size:
                raise IncorrectShardSize()

    def encode(self, shards: List[np.ndarray]) -> None:
        self._check_count(len(shards))
        self._check_sizes(shards)
        k = self.data_shard_count
        outs = mul_rows(self.parity_rows, shards[:k])
        for j, o in enumerate(outs):
            shards[k + j][:] = o

    def verify(self, shards: List[np.ndarray]) -> bool:
        self._check_count(len(shards))
        self._check_sizes(shards)
        k = self.data_shard_count
        outs = mul_rows(self.parity_rows, shards[:k])
        return all(np.array_equal(o, shards[k + j]) for j, o in enumerate(outs))

    def decode_matrix(self, valid: Sequence[int], invalid: Sequence[int]) -> np.ndarray:
        key = tuple(invalid)
        if key not in self._cache:
            sub = self.matrix[list(valid), :]
            self._cache[key] = mat_invert(sub)
        return self._cache[key]

    def reconstruct(self, shards: List[Optional[np.ndarray]]) -> None:
        self._reconstruct(shards, data_only=False)

    def reconstruct_data(self, shards: List[Optional[np.ndarray]]) -> None:
        self._reconstruct(shards, data_only=True)

    def _reconstruct(self, shards, data_only):
        self._check_count(len(shards))
        k = self.data_shard_count
        number_present = 0
        shard_len = None
        for s in shards:
            if s is not None:
                if len(s) == 0:
                    raise EmptyShard()
                number_present += 1
                if shard_len is not None and len(s) != shard_len:
                    raise IncorrectShardSize()
                shard_len = len(s)
        if number_present == self.total_shard_count:
            return
        if number_present < k:
            raise TooFewShardsPresent()
        valid, invalid, sub = [], [], []
        for row, s in enumerate(shards):
            if s is not None:
                if len(sub) < k:
                    sub.append(s)
                    valid.append(row)
            else:
                invalid.append(row)
                if not (row >= k and data_only):
                    shards[row] = np.zeros(shard_len, dtype=np.uint8)
        dm = self.decode_matrix(valid, invalid)
        miss_data = [i for i in invalid if i < k]
        if miss_data:
            outs = mul_rows(dm[miss_data, :], sub)
            for i, o in zip(miss_data, outs):
                shards[i][:] = o
        if data_only:
            return
        miss_par = [i for i in invalid if i >= k]
        if miss_par:
            outs = mul_rows(self.parity_rows[[i - k for i in miss_par], :], shards[:k])
            for i, o in zip(miss_par, outs):
                shards[i][:] = o


# --------------------------------------------------------------------------
# Deterministic synthetic data: splitmix64, little-endian bytes
# --------------------------------------------------------------------------
SPLITMIX_GAMMA = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1


def splitmix64_bytes(seed: int, nbytes: int) -> np.ndarray:
    """Byte stream: word n (n>=1) = mix(seed + n*gamma), little-endian."""
    nwords = (nbytes + 7) // 8
    with np.errstate(over="ignore"):
        n = np.arange(1, nwords + 1, dtype=np.uint64)
        z = np.uint64(seed & M64) + n * np.uint64(SPLITMIX_GAMMA)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8)[:nbytes].copy()


STRIPE_SEED_BASE = 0x5EED0000
VOLUME_SEED = 0x5EED0000


def stripe_data(s: int, shard_len: int, k: int = 10, gpu: int = 0) -> np.ndarray:
    """Data shards of synthetic stripe s: [k, L] from seed 0x5EED0000 + gpu*2^20 + s."""
    return splitmix64_bytes(STRIPE_SEED_BASE + gpu * (1 << 20) + s, k * shard_len).reshape(k, shard_len)


def synthetic_volume(nbytes: int) -> np.ndarray:
    """8-byte superblock [2,0,...] followed by splitmix64(VOLUME_SEED) bytes."""
    out = np.empty(nbytes, dtype=np.uint8)
    head = np.array([2, 0, 0, 0, 0, 0, 0, 0], dtype=np.uint8)
    out[: min(8, nbytes)] = head[: min(8, nbytes)]
    if nbytes > 8:
        out[8:] = splitmix64_bytes(VOLUME_SEED, nbytes - 8)
    return out


# --------------------------------------------------------------------------
# File level -- /root/reference/helyim-ec/src/encoder.rs
# --------------------------------------------------------------------------
DATA_SHARDS_COUNT = 10          # helyim-ec/src/lib.rs:46
PARITY_SHARDS_COUNT = 4         # lib.rs:47
TOTAL_SHARDS_COUNT = 14         # lib.rs:48
ERASURE_CODING_LARGE_BLOCK_SIZE = 1024 * 1024 * 1024  # lib.rs:49
ERASURE_CODING_SMALL_BLOCK_SIZE = 1024 * 1024         # lib.rs:50


class UnexpectedBlockSize(Exception):
    pass


class UnexpectedEcShardSize(Exception):
    pass


def to_ext(i: int) -> str:
    return ".ec%02d" % i  # lib.rs:84-86


def write_ec_files(base: str, buf_size: int = 256 * 1024,
                   large: int = ERASURE_CODING_LARGE_BLOCK_SIZE,
                   small: int = ERASURE_CODING_SMALL_BLOCK_SIZE) -> None:
    """encoder.rs:39-46 + 52-71 + 200-242 (generate_ec_files/encode_data_file)."""
    rs = ReedSolomon(DATA_SHARDS_COUNT, PARITY_SHARDS_COUNT)
    with open(base + ".dat", "rb") as f:
        dat = f.read()
    remaining = len(dat)
    outs = [open(base + to_ext(i), "wb") for i in range(TOTAL_SHARDS_COUNT)]
    try:
        processed = 0

        def encode_row(start, block):
            # encoder.rs:129-156 encode_data
            if block % buf_size != 0:
                raise UnexpectedBlockSize(block, buf_size)
            for b in range(block // buf_size):
                off = start + b * buf_size
                bufs = []
                for i in range(DATA_SHARDS_COUNT):  # encoder.rs:169-189 (short read -> zero fill)
                    p = off + block * i
                    chunk = np.frombuffer(dat[p:p + buf_size], dtype=np.uint8)
                    buf = np.zeros(buf_size, dtype=np.uint8)
                    buf[: len(chunk)] = chunk
                    bufs.append(buf)
                bufs += [np.zeros(buf_size, dtype=np.uint8) for _ in range(PARITY_SHARDS_COUNT)]
                rs.encode(bufs)  # encoder.rs:191
                for i in range(TOTAL_SHARDS_COUNT):
                    outs[i].write(bufs[i].tobytes())

        while remaining > large * DATA_SHARDS_COUNT:  # encoder.rs:215 (strict >)
            encode_row(processed, large)
            processed += large * DATA_SHARDS_COUNT
            remaining -= large * DATA_SHARDS_COUNT
        while remaining > 0:  # encoder.rs:228
            encode_row(processed, small)
            processed += small * DATA_SHARDS_COUNT
            remaining -= small * DATA_SHARDS_COUNT
    finally:
        for o in outs:
            o.close()


def rebuild_ec_files(base: str) -> List[int]:
    """encoder.rs:48-50, 73-109, 244-307 (generate_missing_ec_files)."""
    rs = ReedSolomon(DATA_SHARDS_COUNT, PARITY_SHARDS_COUNT)
    has = [os.path.exists(base + to_ext(i)) for i in range(TOTAL_SHARDS_COUNT)]
    rebuilt = [i for i in range(TOTAL_SHARDS_COUNT) if not has[i]]
    inputs = {i: open(base + to_ext(i), "rb") for i in range(TOTAL_SHARDS_COUNT) if has[i]}
    outputs = {i: open(base + to_ext(i), "wb") for i in rebuilt}
    try:
        start = 0
        size = 0
        while True:
            bufs: List[Optional[np.ndarray]] = [None] * TOTAL_SHARDS_COUNT
            for i in range(TOTAL_SHARDS_COUNT):
                if has[i]:
                    inputs[i].seek(start)
                    data = inputs[i].read(ERASURE_CODING_SMALL_BLOCK_SIZE)
                    n = len(data)
                    if n == 0:  # encoder.rs:269-271
                        return rebuilt
                    if size == 0:
                        size = n
                    if size != n:  # encoder.rs:275-280
                        raise UnexpectedEcShardSize(size, n)
                    buf = np.zeros(ERASURE_CODING_SMALL_BLOCK_SIZE, dtype=np.uint8)
                    buf[:n] = np.frombuffer(data, dtype=np.uint8)
                    bufs[i] = buf
            rs.reconstruct(bufs)  # encoder.rs:288 (on full 1 MiB buffers)
            for i in rebuilt:
                outputs[i].seek(start)
                outputs[i].write(bufs[i][:size].tobytes())
            start += size
    finally:
        for f in list(inputs.values()) + list(outputs.values()):
            f.close()


def sha256(b) -> str:
    if isinstance(b, np.ndarray):
        b = b.tobytes()
    return hashlib.sha256(b).hexdigest()


# --------------------------------------------------------------------------
# EC volume files around the shards -- restated from the reference:
#   .idx/.ecx entries: 16 bytes big endian (u64 needle id, u32 offset/8, i32 size)
#   helyim-common/src/types/needle.rs:119-160, helyim-ec/src/needle/mod.rs:12-44
# --------------------------------------------------------------------------
import struct as _struct


class IoError(Exception):
    pass


def _entries(raw: bytes):
    return [_struct.unpack(">QIi", raw[i:i + 16]) for i in range(0, len(raw) - len(raw) % 16, 16)]


def write_sorted_file_from_index(base: str, ext: str = ".ecx") -> None:
    """encoder.rs:21-37 + SortedIndexMap::load_from_index (needle/mod.rs:12-32):
    IndexMap insert / shift_remove replay, then ascending sort by key."""
    with open(base + ".idx", "rb") as f:
        raw = f.read()
    live = {}
    for key, off, size in _entries(raw):
        if off == 0 or size < 0:          # Size::is_deleted: size < 0 || size == -1
            live.pop(key, None)
        else:
            live[key] = (off, size)
    if len(raw) % 16:                     # walk_index_file: read_exact of a partial entry
        raise IoError("UnexpectedEof")
    with open(base + ext, "wb") as f:
        for key in sorted(live):
            f.write(_struct.pack(">QIi", key, *live[key]))


def rebuild_ecx_file(base: str) -> None:
    """lib.rs:95-133 (binary search :54-82, tombstone write :88-93)."""
    ecj = base + ".ecj"
    if not os.path.exists(ecj):
        return
    with open(base + ".ecx", "r+b") as ecx:
        raw = bytearray(ecx.read())
        n = len(raw) // 16
        ids = open(ecj, "rb").read()
        for p in range(0, len(ids) - len(ids) % 8, 8):
            want = _struct.unpack(">Q", ids[p:p + 8])[0]
            lo, hi = 0, n
            while lo < hi:
                mid = (lo + hi) // 2
                key = _struct.unpack(">Q", raw[mid * 16:mid * 16 + 8])[0]
                if key == want:
                    raw[mid * 16 + 12:mid * 16 + 16] = _struct.pack(">i", -1)
                    break
                if key < want:
                    lo = mid + 1
                else:
                    hi = mid
        ecx.seek(0)
        ecx.write(raw)
    os.remove(ecj)


def volume_info_json(version: int) -> bytes:
    """serde_json of VolumeInfo { version, ..Default } (volume.proto:75-79)."""
    return ('{"files":[],"version":%d,"replication":""}' % version).encode()


def find_data_filesize(base: str) -> int:
    """decoder.rs:46-66 (Offset::actual_offset is a wrapping u32 product)."""
    with open(base + ".ec00", "rb") as f:
        sb = f.read(8)
    if len(sb) < 8:
        raise IoError("UnexpectedEof")
    if sb[3] > 6:
        raise IoError("Ttl error: invalid unit")
    size = 0
    for key, off, s in _entries(open(base + ".ecx", "rb").read()):
        if s < 0:
            continue
        body = 16 + s + 4
        stop = ((off * 8) & 0xFFFFFFFF) + body + (8 - body % 8)
        size = max(size, stop)
    return size


def write_data_file(base: str, data_filesize: int) -> None:
    """decoder.rs:142-180 (large rows while size >= 10 GiB, then 1 MiB blocks)."""
    ins = [open(base + to_ext(i), "rb") for i in range(10)]
    try:
        with open(base + ".dat", "wb") as out:
            L, S = ERASURE_CODING_LARGE_BLOCK_SIZE, ERASURE_CODING_SMALL_BLOCK_SIZE
            while data_filesize >= 10 * L:
                for f in ins:
                    b = f.read(L)
                    if len(b) < L:
                        raise IoError("UnexpectedEof")
                    out.write(b)
                    data_filesize -= L
            while data_filesize > 0:
                for f in ins:
                    n = min(data_filesize, S)
                    b = f.read(n)
                    if len(b) < n:
                        raise IoError("UnexpectedEof")
                    out.write(b)
                    data_filesize -= n
    finally:
        for f in ins:
            f.close()


def write_index_file_from_ec_index(base: str) -> None:
    """decoder.rs:22-44: .ecx copied, then a deleted entry per .ecj id."""
    raw = open(base + ".ecx", "rb").read()
    with open(base + ".idx", "wb") as out:
        out.write(raw)
        if os.path.exists(base + ".ecj"):
            ids = open(base + ".ecj", "rb").read()
            for p in range(0, len(ids) - len(ids) % 8, 8):
                out.write(ids[p:p + 8] + _struct.pack(">Ii", 0, -1))


# --------------------------------------------------------------------------
# Needle reads -- restated from the reference:
#   locate_data / Interval      helyim-ec/src/locate.rs:1-100
#   find_needle_from_ecx        helyim-ec/src/volume/mod.rs:153-155, lib.rs:54-82
#   read path                   helyim-store/src/erasure_coding/mod.rs:129-171,303-491
# Shards are the local base.ecNN files; a lost shard is a missing file.
# --------------------------------------------------------------------------
class NeedleNotFound(Exception):
    pass


class ShardNotFound(Exception):
    pass


def _locate_offset(large, small, data_size, offset):
    """locate.rs:74-100 (large-row count = data_size // (large * 10))."""
    large_row_size = large * DATA_SHARDS_COUNT
    large_block_rows = data_size // (large * DATA_SHARDS_COUNT)
    if offset < large_block_rows * large_row_size:
        return offset // large, True, offset % large
    offset -= large_block_rows * large_row_size
    return offset // small, False, offset % small


def locate_data(large, small, data_size, offset, size):
    """locate.rs:29-72. Intervals as (block_index, inner_block_offset, size,
    is_large_block, large_block_rows); note the large-row count here is
    (data_size + small * 10) // (large * 10), unlike _locate_offset."""
    block_index, is_large, inner = _locate_offset(large, small, data_size, offset)
    large_block_rows = (data_size + small * DATA_SHARDS_COUNT) // (large * DATA_SHARDS_COUNT)
    out = []
    while size > 0:
        remaining = (large if is_large else small) - inner
        if size <= remaining:
            out.append((block_index, inner, size, is_large, large_block_rows))
            return out
        out.append((block_index, inner, remaining, is_large, large_block_rows))
        size -= remaining
        block_index += 1
        if is_large and block_index == large_block_rows * DATA_SHARDS_COUNT:
            is_large, block_index = False, 0
        inner = 0
    return out


def interval_shard_id(iv) -> int:
    """Interval::shard_id (locate.rs:12-15)."""
    return iv[0] % DATA_SHARDS_COUNT


def interval_offset(iv, large, small) -> int:
    """Interval::offset (locate.rs:17-27)."""
    block_index, inner, _, is_large, large_block_rows = iv
    row = block_index // DATA_SHARDS_COUNT
    if is_large:
        return inner + row * large
    return inner + large_block_rows * large + row * small


def find_needle_from_ecx(base: str, needle_id: int):
    """search_needle_from_sorted_index (lib.rs:54-82): (offset, size) as stored."""
    raw = open(base + ".ecx", "rb").read()
    lo, hi = 0, len(raw) // 16
    while lo < hi:
        mid = (lo + hi) // 2
        key, off, size = _struct.unpack(">QIi", raw[mid * 16:mid * 16 + 16])
        if key == needle_id:
            return off, size
        if key < needle_id:
            lo = mid + 1
        else:
            hi = mid
    raise IoError("Needle %d is not found" % needle_id)


def read_ec_data(base: str, ranges, large=ERASURE_CODING_LARGE_BLOCK_SIZE,
                 small=ERASURE_CODING_SMALL_BLOCK_SIZE) -> bytes:
    """read_ec_shard_intervals over (offset, size) ranges from the local shard
    files: data_size = first shard file's size * 10 (volume/mod.rs:146); a
    present shard is read exactly (read_exact_at, mod.rs:344); a missing one
    is recovered from every other shard's full-length read of the same range
    (mod.rs:403-491: read == buf_len) with upstream reconstruct."""
    names = [base + to_ext(i) for i in range(TOTAL_SHARDS_COUNT)]
    have = [os.path.exists(n) for n in names]
    if not any(have):
        raise ShardNotFound(base)
    data_size = os.path.getsize(names[have.index(True)]) * DATA_SHARDS_COUNT
    rs = ReedSolomon(DATA_SHARDS_COUNT, PARITY_SHARDS_COUNT)
    out = bytearray()

    def pread(i, off, n):
        with open(names[i], "rb") as f:
            f.seek(off)
            return f.read(n)

    for offset, size in ranges:
        for iv in locate_data(large, small, data_size, offset, size):
            sid, off, n = interval_shard_id(iv), interval_offset(iv, large, small), iv[2]
            if have[sid]:
                b = pread(sid, off, n)
                if len(b) != n:
                    raise IoError("UnexpectedEof")
                out += b
                continue
            bufs = [None] * TOTAL_SHARDS_COUNT
            for i in range(TOTAL_SHARDS_COUNT):
                if i != sid and have[i]:
                    b = pread(i, off, n)
                    if len(b) == n:
                        bufs[i] = np.frombuffer(b, np.uint8).copy()
            rs.reconstruct(bufs)
            out += bufs[sid].tobytes()
    return bytes(out)


def read_ec_needle(base: str, needle_id: int, large=ERASURE_CODING_LARGE_BLOCK_SIZE,
                   small=ERASURE_CODING_SMALL_BLOCK_SIZE) -> bytes:
    """read_ec_shard_needle's data path (mod.rs:129-171 via
    locate_ec_shard_needle, volume/mod.rs:136-151)."""
    off, size = find_needle_from_ecx(base, needle_id)
    if size < 0:
        raise NeedleNotFound(needle_id)
    actual_offset = (off * 8) & 0xFFFFFFFF              # Offset::actual_offset, u32 product
    body = 16 + (size & 0xFFFFFFFF) + 4                 # Size::actual_size
    actual_size = (body + (8 - body % 8)) & 0xFFFFFFFF
    return read_ec_data(base, [(actual_offset, actual_size)], large, small)


# ---- EcVolume (helyim-ec/src/volume/mod.rs:30-171) ---------------------------

def ec_volume_open_version(base: str) -> int:
    """EcVolume::new's .vif step (mod.rs:66-77) with maybe_load_volume_info
    (volume_info.rs:107-119): a missing .vif, or one whose `files` list is
    empty, is (re)written as VolumeInfo{version: 2}; else its version. Also
    creates .ecj (OpenOptions::create, mod.rs:59-64)."""
    import json
    open(base + ".ecj", "ab").close()
    vif = base + ".vif"
    if os.path.exists(vif):
        info = json.loads(open(vif, "rb").read())
        if info.get("files"):
            return int(info.get("version", 0))
    with open(vif, "wb") as f:
        f.write(volume_info_json(2))
    return 2


def ec_volume_delete_needle(base: str, needle_id: int) -> None:
    """delete_needle_from_ecx (mod.rs:157-171): tombstone the entry's size in
    .ecx (mark_needle_deleted, lib.rs:88-93), append the id to .ecj."""
    with open(base + ".ecx", "r+b") as ecx:
        raw = ecx.read()
        lo, hi = 0, len(raw) // 16
        while lo < hi:
            mid = (lo + hi) // 2
            key = _struct.unpack(">Q", raw[mid * 16:mid * 16 + 8])[0]
            if key == needle_id:
                ecx.seek(mid * 16 + 12)
                ecx.write(_struct.pack(">i", -1))
                break
            if key < needle_id:
                lo = mid + 1
            else:
                hi = mid
        else:
            raise IoError("Needle %d is not found" % needle_id)
    with open(base + ".ecj", "ab") as f:
        f.write(_struct.pack(">Q", needle_id))

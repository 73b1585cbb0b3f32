"""Error types mirroring the reference's error enums.

* ``Error`` and its subclasses mirror ``reed_solomon_erasure::Error``
  (upstream crate 6.0.0), codes 1..13 of include/hec.h.
* ``EcShardError`` and subclasses mirror helyim_ec::EcShardError
  (/root/reference/helyim-ec/src/errors.rs:55-66), codes 32..35; an RS error
  raised from the file layer is wrapped as ``EcShardError.ErasureCoding``
  exactly like errors.rs:58-59 (``#[from] reed_solomon_erasure::Error``).
* ``EcVolumeError`` subclasses mirror the needle-read variants of
  helyim_ec::EcVolumeError (errors.rs:31-34), codes 48..49.
* ``DeviceError`` covers this library's own HIP/device failures (64..).
"""
from __future__ import annotations

from . import _lib


class Error(Exception):
    """reed_solomon_erasure::Error"""
    code = -1


class TooFewShards(Error): code = 1
class TooManyShards(Error): code = 2
class TooFewDataShards(Error): code = 3
class TooManyDataShards(Error): code = 4
class TooFewParityShards(Error): code = 5
class TooManyParityShards(Error): code = 6
class TooFewBufferShards(Error): code = 7
class TooManyBufferShards(Error): code = 8
class IncorrectShardSize(Error): code = 9
class TooFewShardsPresent(Error): code = 10
class EmptyShard(Error): code = 11
class InvalidShardFlags(Error): code = 12
class InvalidIndex(Error): code = 13


class EcShardError(Exception):
    """helyim_ec::EcShardError"""
    code = -1


class Io(EcShardError):
    """EcShardError::Io(std::io::Error): ``errno`` is the OS error behind it
    (hec_last_error_values; 0 when there was none, e.g. a short read), and
    ``os_error`` the matching OSError (None without an errno)."""
    code = 32

    def __init__(self, detail: str, errno: int = 0):
        import os as _os
        self.detail, self.errno = detail, errno
        self.os_error = OSError(errno, _os.strerror(errno)) if errno else None
        # thiserror "Io error: {0}" over io::Error's Display "... (os error N)"
        super().__init__(f"Io error: {detail}" + (f" (os error {errno})" if errno else ""))


class _SizePair(EcShardError):
    """The (usize, usize) variants of EcShardError (errors.rs:60-65); str() is
    helyim's thiserror text with the two values filled in."""
    fmt = ""

    def __init__(self, a: int, b: int):
        self.values = (a, b)
        super().__init__(self.fmt.format(a, b))


class Underflow(_SizePair):
    """Underflow(found, required); helyim's format prints {0} twice (errors.rs:60)."""
    code = 33
    fmt = "Only {0} shards found but {0} required"


class UnexpectedEcShardSize(_SizePair):
    """UnexpectedEcShardSize(expected, actual) (encoder.rs:276-279)."""
    code = 34
    fmt = "ec shard size expected {0} but actually is {1}"

    @property
    def expected(self) -> int:
        return self.values[0]

    @property
    def actual(self) -> int:
        return self.values[1]


class UnexpectedBlockSize(_SizePair):
    """UnexpectedBlockSize(block_size, buf_size) (encoder.rs:140-143)."""
    code = 35
    fmt = "unexpected block size {0}, buffer size {1}"

    @property
    def block_size(self) -> int:
        return self.values[0]

    @property
    def buf_size(self) -> int:
        return self.values[1]


class EcVolumeError(Exception):
    """helyim_ec::EcVolumeError (helyim-ec/src/errors.rs:15-35), the variants
    the needle-read path returns."""
    code = -1


class NeedleNotFound(EcVolumeError): code = 48
class ShardNotFound(EcVolumeError): code = 49


class ErasureCoding(EcShardError):
    """EcShardError::ErasureCoding(reed_solomon_erasure::Error)"""

    def __init__(self, inner: Error):
        super().__init__(f"Erasure coding error: {inner}")
        self.inner = inner


class DeviceError(Exception):
    """HIP / device / argument failure inside libhec (no reference counterpart)."""

    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


_RS = {c.code: c for c in (TooFewShards, TooManyShards, TooFewDataShards, TooManyDataShards,
                           TooFewParityShards, TooManyParityShards, TooFewBufferShards,
                           TooManyBufferShards, IncorrectShardSize, TooFewShardsPresent,
                           EmptyShard, InvalidShardFlags, InvalidIndex)}
_EC = {c.code: c for c in (Io, Underflow, UnexpectedEcShardSize, UnexpectedBlockSize, NeedleNotFound,
                           ShardNotFound)}


def _message(code: int) -> str:
    detail = _lib.last_detail()
    text = _lib.strerror(code)
    return f"{text} ({detail})" if detail else text


def check(code: int) -> None:
    """Raise the mirror exception for an RS-level status code."""
    if code == 0:
        return
    if code in _RS:
        raise _RS[code](_lib.strerror(code))
    if code in _EC:
        cls = _EC[code]
        a, b, errno = _lib.last_values()
        if issubclass(cls, _SizePair):
            raise cls(a, b)
        if cls is Io:
            raise Io(_lib.last_detail() or _lib.strerror(code), errno)
        raise cls(_message(code))
    raise DeviceError(code, _message(code))


def check_ec(code: int) -> None:
    """Raise for a file-level status: RS errors wrap into ErasureCoding."""
    if code == 0:
        return
    if code in _RS:
        raise ErasureCoding(_RS[code](_lib.strerror(code)))
    check(code)

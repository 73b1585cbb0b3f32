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


class Io(EcShardError): code = 32
class Underflow(EcShardError): code = 33
class UnexpectedEcShardSize(EcShardError): code = 34
class UnexpectedBlockSize(EcShardError): code = 35


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
        raise _EC[code](_message(code))
    raise DeviceError(code, _message(code))


def check_ec(code: int) -> None:
    """Raise for a file-level status: RS errors wrap into ErasureCoding."""
    if code == 0:
        return
    if code in _RS:
        raise ErasureCoding(_RS[code](_lib.strerror(code)))
    check(code)

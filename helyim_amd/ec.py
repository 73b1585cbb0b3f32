"""helyim_ec crate surface for the hot path (GPU-backed).

Constants mirror /root/reference/helyim-ec/src/lib.rs:44-50 and ``to_ext``
lib.rs:84-86; ``write_ec_files`` / ``rebuild_ec_files`` mirror
encoder.rs:39-50 (called by helyim-store/src/server.rs:468 and :497).
Errors are ``helyim_amd.errors.EcShardError`` subclasses, with RS errors
wrapped as ``ErasureCoding`` like errors.rs:58-59.
"""
from __future__ import annotations

import ctypes
from typing import List

from . import _lib
from .errors import check, check_ec

lib = _lib.lib

DATA_SHARDS_COUNT = 10
PARITY_SHARDS_COUNT = 4
TOTAL_SHARDS_COUNT = DATA_SHARDS_COUNT + PARITY_SHARDS_COUNT
ERASURE_CODING_LARGE_BLOCK_SIZE = 1024 * 1024 * 1024
ERASURE_CODING_SMALL_BLOCK_SIZE = 1024 * 1024


def to_ext(ec_idx: int) -> str:
    return ".ec%02d" % ec_idx


def write_ec_files(base_filename: str) -> None:
    """base.dat -> base.ec00 .. base.ec13 (encoder.rs:39-46)."""
    check_ec(lib.hec_write_ec_files(base_filename.encode()))


def generate_ec_files(base_filename: str, buf_size: int, large_block_size: int,
                      small_block_size: int) -> None:
    """encoder.rs:52-71 with explicit geometry (tests shrink the blocks)."""
    check_ec(lib.hec_write_ec_files_ex(base_filename.encode(), buf_size, large_block_size,
                                       small_block_size))


def rebuild_ec_files(base_filename: str) -> List[int]:
    """Recreate missing .ecNN files; returns the rebuilt shard ids (encoder.rs:48-50)."""
    ids = (ctypes.c_uint32 * TOTAL_SHARDS_COUNT)()
    n = ctypes.c_size_t(0)
    check_ec(lib.hec_rebuild_ec_files(base_filename.encode(), ids, ctypes.byref(n)))
    return [int(ids[i]) for i in range(n.value)]


# --- EC volume files around the shards (helyim-ec host-side byte formats) ---

def write_sorted_file_from_index(base_filename: str, ext: str = ".ecx") -> None:
    """.idx -> sorted .ecx (encoder.rs:21-37). Raises Io like EcVolumeError::Io."""
    check(lib.hec_write_sorted_file_from_index(base_filename.encode(), ext.encode()))


def rebuild_ecx_file(base_filename: str) -> None:
    """Apply .ecj tombstones to .ecx, delete .ecj (lib.rs:95-133)."""
    check(lib.hec_rebuild_ecx_file(base_filename.encode()))


def save_volume_info(filename: str, version: int) -> None:
    """.vif as the generate RPC writes it (server.rs:470-475)."""
    check(lib.hec_save_volume_info(filename.encode(), version))


def find_data_filesize(base_filename: str) -> int:
    """decoder.rs:46-66."""
    out = ctypes.c_uint64(0)
    check(lib.hec_find_data_filesize(base_filename.encode(), ctypes.byref(out)))
    return int(out.value)


def write_data_file(base_filename: str, data_filesize: int) -> None:
    """.ec00-.ec09 -> .dat (decoder.rs:142-180)."""
    check(lib.hec_write_data_file(base_filename.encode(), data_filesize))


def write_index_file_from_ec_index(base_filename: str) -> None:
    """.ecx + .ecj -> .idx (decoder.rs:22-44)."""
    check(lib.hec_write_index_file_from_ec_index(base_filename.encode()))


def volume_ec_shards_generate(base_filename: str, version: int) -> None:
    """The body of the VolumeEcShardsGenerate RPC (helyim-store/src/server.rs:466-475):
    .ecx, then .ec00-.ec13, then .vif."""
    write_sorted_file_from_index(base_filename, ".ecx")
    write_ec_files(base_filename)
    save_volume_info(base_filename + ".vif", version)


def volume_ec_shards_rebuild(base_filename: str) -> List[int]:
    """The body of the VolumeEcShardsRebuild RPC for one location (server.rs:497-498)."""
    ids = rebuild_ec_files(base_filename)
    rebuild_ecx_file(base_filename)
    return ids

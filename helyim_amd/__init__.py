"""helyim_amd -- MI355X-native RS(10,4) erasure coding for helyim's EC tier.

Host mirror of the reference's operator surface for the hot path:

* ``ReedSolomon`` -- reed_solomon_erasure::ReedSolomon<galois_8::Field>
  (new / encode / verify / reconstruct / reconstruct_data);
* ``write_ec_files`` / ``rebuild_ec_files`` / ``to_ext`` and the geometry
  constants -- helyim_ec (helyim-ec/src/lib.rs, encoder.rs);
* ``batch`` -- device-resident stripe batches (torch tensors on ROCm).

All compute runs in helyim_amd/libhec.so (HIP, gfx950). Import fails if the
library is missing; there is no CPU fallback.
"""
from ._lib import LIB_PATH, lib  # noqa: F401  (raises ImportError when not built)
from .errors import (  # noqa: F401
    DeviceError, EcShardError, EcVolumeError, EmptyShard, ErasureCoding, Error, IncorrectShardSize, InvalidIndex,
    InvalidShardFlags, Io, TooFewBufferShards, TooFewDataShards, TooFewParityShards, TooFewShards,
    TooFewShardsPresent, TooManyBufferShards, TooManyDataShards, TooManyParityShards, TooManyShards,
    NeedleNotFound, ShardNotFound, Underflow, UnexpectedBlockSize, UnexpectedEcShardSize,
)
from .rs import ReedSolomon  # noqa: F401
from .device import HostBuffer, bind_host_to_device, device_count, get_device, numa_node, set_device  # noqa: F401
from .ec import (  # noqa: F401
    DATA_SHARDS_COUNT, ERASURE_CODING_LARGE_BLOCK_SIZE, ERASURE_CODING_SMALL_BLOCK_SIZE,
    PARITY_SHARDS_COUNT, TOTAL_SHARDS_COUNT, EcVolume, Interval, find_data_filesize, find_needle_from_ecx, locate_data,
    read_ec_data, read_ec_needle, read_ec_needles, generate_ec_files, rebuild_ec_files,
    rebuild_ecx_file, save_volume_info, to_ext, ec_shard_filename, ec_shard_base_filename, volume_ec_shards_generate, volume_ec_shards_rebuild,
    write_data_file, write_ec_files, write_index_file_from_ec_index, write_sorted_file_from_index,
)


def version() -> str:
    return lib.hec_version().decode()

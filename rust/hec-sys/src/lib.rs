//! Raw bindings to `libhec.so`, one `extern "C"` item per function of
//! `include/hec.h` (the bindgen output a maintainer would check in). Each
//! entry point replaces an interface of the reference (paths relative to
//! /root/reference):
//!
//! * `hec_rs_*` -- `reed_solomon_erasure::ReedSolomon<galois_8::Field>`
//!   {new, encode, verify, reconstruct, reconstruct_data}, called at
//!   helyim-ec/src/encoder.rs:191,208-209,249-250,288 and
//!   helyim-store/src/erasure_coding/mod.rs:411-412,426;
//! * `hec_write_ec_files[_ex]` / `hec_rebuild_ec_files` --
//!   `helyim_ec::{write_ec_files, generate_ec_files, rebuild_ec_files}`
//!   (helyim-ec/src/encoder.rs:39-71), called by helyim-store/src/server.rs:468,497;
//! * the `.ecx`/`.ecj`/`.vif`, decoder and needle-read functions --
//!   helyim-ec/src/{lib,decoder,locate}.rs and erasure_coding/mod.rs:129-491.
//!
//! Status codes: 0 = ok; 1..=13 = `reed_solomon_erasure::Error` in declaration
//! order; 32..=35 = `EcShardError`; 48..=49 = `EcVolumeError`; 64.. = device /
//! argument errors of libhec.
#![allow(non_camel_case_types)]

use std::os::raw::{c_char, c_int, c_void};

#[repr(C)]
pub struct hec_rs_t {
    _p: [u8; 0],
}

#[repr(C)]
pub struct hec_ec_volume_t {
    _p: [u8; 0],
}

/// helyim-ec/src/locate.rs:3-9 `Interval`.
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct hec_interval {
    pub block_index: u64,
    pub inner_block_offset: u64,
    pub size: u64,
    pub large_block_rows: u64,
    pub is_large_block: u32,
    pub reserved: u32,
}

/// One stripe of a ragged device batch.
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct hec_stripe_desc {
    pub offset: u64,
    pub shard_stride: u64,
    pub shard_len: u32,
    pub present_mask: u32,
}

pub const HEC_OK: c_int = 0;
pub const HEC_ERR_TOO_FEW_SHARDS_PRESENT: c_int = 10;
pub const HEC_ERR_IO: c_int = 32;
pub const HEC_ERR_UNDERFLOW: c_int = 33;
pub const HEC_ERR_UNEXPECTED_EC_SHARD_SIZE: c_int = 34;
pub const HEC_ERR_UNEXPECTED_BLOCK_SIZE: c_int = 35;
pub const HEC_ERR_NEEDLE_NOT_FOUND: c_int = 48;
pub const HEC_ERR_SHARD_NOT_FOUND: c_int = 49;
pub const HEC_ERR_HIP: c_int = 64;
pub const HEC_ERR_NO_DEVICE: c_int = 65;
pub const HEC_ERR_INVALID_ARGUMENT: c_int = 66;
pub const HEC_ERR_OUT_OF_MEMORY: c_int = 67;

pub const HEC_DATA_SHARDS_COUNT: u32 = 10;
pub const HEC_PARITY_SHARDS_COUNT: u32 = 4;
pub const HEC_TOTAL_SHARDS_COUNT: u32 = 14;
pub const HEC_LARGE_BLOCK_SIZE: u64 = 1024 * 1024 * 1024;
pub const HEC_SMALL_BLOCK_SIZE: u64 = 1024 * 1024;

extern "C" {
    pub fn hec_strerror(status: c_int) -> *const c_char;
    pub fn hec_last_error_detail() -> *const c_char;
    pub fn hec_last_error_values(a: *mut u64, b: *mut u64, os_errno: *mut c_int) -> c_int;

    // device selection (per calling thread)
    pub fn hec_device_count(count: *mut c_int) -> c_int;
    pub fn hec_set_device(device: c_int) -> c_int;
    pub fn hec_get_device(device: *mut c_int) -> c_int;

    // NUMA placement of the host side of a GPU
    pub fn hec_device_numa_node(device: c_int, node: *mut c_int) -> c_int;
    pub fn hec_bind_thread_to_device(device: c_int, n_cpus: *mut c_int) -> c_int;
    pub fn hec_host_alloc(bytes: usize, out: *mut *mut c_void) -> c_int;
    pub fn hec_host_alloc_multi(devices: *const c_int, n_devices: usize, stripe_stride: u64, n_stripes: u32,
                                out: *mut *mut c_void) -> c_int;
    pub fn hec_host_free(p: *mut c_void) -> c_int;
    pub fn hec_host_numa_node(p: *const c_void, node: *mut c_int) -> c_int;

    // ReedSolomon<galois_8::Field>
    pub fn hec_rs_new(data_shards: usize, parity_shards: usize, out: *mut *mut hec_rs_t) -> c_int;
    pub fn hec_rs_free(rs: *mut hec_rs_t);
    pub fn hec_rs_data_shard_count(rs: *const hec_rs_t) -> usize;
    pub fn hec_rs_parity_shard_count(rs: *const hec_rs_t) -> usize;
    pub fn hec_rs_total_shard_count(rs: *const hec_rs_t) -> usize;
    pub fn hec_rs_matrix(rs: *const hec_rs_t, out: *mut u8, out_len: usize) -> c_int;
    pub fn hec_rs_encode(rs: *const hec_rs_t, shards: *const *mut u8, shard_lens: *const usize,
                         n_shards: usize) -> c_int;
    pub fn hec_rs_verify(rs: *const hec_rs_t, shards: *const *const u8, shard_lens: *const usize,
                         n_shards: usize, ok: *mut c_int) -> c_int;
    pub fn hec_rs_reconstruct(rs: *const hec_rs_t, shards: *const *mut u8, shard_lens: *const usize,
                              present: *const u8, n_shards: usize) -> c_int;
    pub fn hec_rs_reconstruct_data(rs: *const hec_rs_t, shards: *const *mut u8, shard_lens: *const usize,
                                   present: *const u8, n_shards: usize) -> c_int;
    pub fn hec_rs_reconstruct_batch(rs: *const hec_rs_t, shards: *const *mut u8, lens: *const usize,
                                    present: *const u8, n_stripes: usize, data_only: c_int,
                                    bad_index: *mut usize) -> c_int;

    // device-resident and host-memory stripe batches
    pub fn hec_gpu_encode_batch(rs: *const hec_rs_t, d_data: *const u8, data_stripe_stride: u64,
                                data_shard_stride: u64, d_parity: *mut u8, parity_stripe_stride: u64,
                                parity_shard_stride: u64, shard_len: u64, n_stripes: u32,
                                stream: *mut c_void) -> c_int;
    pub fn hec_gpu_reconstruct_batch(rs: *const hec_rs_t, d_shards: *mut u8, stripe_stride: u64,
                                     shard_stride: u64, shard_len: u64, n_stripes: u32,
                                     d_present_masks: *const u32, d_bad_stripes: *mut u32,
                                     stream: *mut c_void) -> c_int;
    pub fn hec_host_encode_batch(rs: *const hec_rs_t, h_data: *const u8, data_stripe_stride: u64,
                                 data_shard_stride: u64, h_parity: *mut u8, parity_stripe_stride: u64,
                                 parity_shard_stride: u64, shard_len: u64, n_stripes: u32) -> c_int;
    pub fn hec_host_reconstruct_batch(rs: *const hec_rs_t, h_shards: *mut u8, stripe_stride: u64,
                                      shard_stride: u64, shard_len: u64, n_stripes: u32,
                                      h_present_masks: *const u32, n_bad_stripes: *mut u32) -> c_int;
    pub fn hec_host_encode_batch_multi(rs: *const hec_rs_t, devices: *const c_int, n_devices: usize,
                                       h_data: *const u8, data_stripe_stride: u64, data_shard_stride: u64,
                                       h_parity: *mut u8, parity_stripe_stride: u64, parity_shard_stride: u64,
                                       shard_len: u64, n_stripes: u32) -> c_int;
    pub fn hec_host_reconstruct_batch_multi(rs: *const hec_rs_t, devices: *const c_int, n_devices: usize,
                                            h_shards: *mut u8, stripe_stride: u64, shard_stride: u64,
                                            shard_len: u64, n_stripes: u32, h_present_masks: *const u32,
                                            n_bad_stripes: *mut u32) -> c_int;
    pub fn hec_gpu_encode_ragged(rs: *const hec_rs_t, d_base: *mut u8, descs: *const hec_stripe_desc,
                                 n_stripes: u32, stream: *mut c_void) -> c_int;
    pub fn hec_gpu_reconstruct_ragged(rs: *const hec_rs_t, d_base: *mut u8, descs: *const hec_stripe_desc,
                                      n_stripes: u32, d_bad_stripes: *mut u32, stream: *mut c_void) -> c_int;
    pub fn hec_gpu_fill_splitmix(d_base: *mut u8, stripe_stride: u64, bytes_per_stripe: u64, n_stripes: u32,
                                 seed_base: u64, stream: *mut c_void) -> c_int;

    // helyim_ec file layer
    pub fn hec_write_ec_files(base_filename: *const c_char) -> c_int;
    pub fn hec_write_ec_files_ex(base_filename: *const c_char, buf_size: u64, large_block_size: u64,
                                 small_block_size: u64) -> c_int;
    pub fn hec_rebuild_ec_files(base_filename: *const c_char, rebuilt_ids: *mut u32, n_rebuilt: *mut usize)
                                -> c_int;
    pub fn hec_write_sorted_file_from_index(base_filename: *const c_char, ext: *const c_char) -> c_int;
    pub fn hec_rebuild_ecx_file(base_filename: *const c_char) -> c_int;
    pub fn hec_save_volume_info(filename: *const c_char, version: u32) -> c_int;
    pub fn hec_find_data_filesize(base_filename: *const c_char, data_filesize: *mut u64) -> c_int;
    pub fn hec_write_data_file(base_filename: *const c_char, data_filesize: i64) -> c_int;
    pub fn hec_write_index_file_from_ec_index(base_filename: *const c_char) -> c_int;

    // needle reads
    pub fn hec_locate_data(large_block_len: u64, small_block_len: u64, data_size: u64, offset: u64, size: u64,
                           out: *mut hec_interval, cap: usize, n_out: *mut usize) -> c_int;
    pub fn hec_interval_shard_id(interval: *const hec_interval) -> u32;
    pub fn hec_interval_offset(interval: *const hec_interval, large_block_size: u64, small_block_size: u64)
                               -> u64;
    pub fn hec_find_needle_from_ecx(base_filename: *const c_char, needle_id: u64, offset: *mut u32,
                                    size: *mut i32) -> c_int;
    pub fn hec_read_ec_data(base_filename: *const c_char, large_block_size: u64, small_block_size: u64,
                            offsets: *const u64, sizes: *const u64, n_ranges: usize, out: *mut u8) -> c_int;
    pub fn hec_read_ec_needle(base_filename: *const c_char, needle_id: u64, out: *mut u8, cap: usize,
                              n_out: *mut usize) -> c_int;
    pub fn hec_read_ec_needle_ex(base_filename: *const c_char, large_block_size: u64, small_block_size: u64,
                                 needle_id: u64, out: *mut u8, cap: usize, n_out: *mut usize) -> c_int;
    pub fn hec_read_ec_needles(base_filename: *const c_char, large_block_size: u64, small_block_size: u64,
                               needle_ids: *const u64, n: usize, out: *mut u8, cap: usize, out_offsets: *mut u64,
                               statuses: *mut c_int) -> c_int;

    // mounted EcVolume
    pub fn hec_ec_volume_open(base_filename: *const c_char, out: *mut *mut hec_ec_volume_t) -> c_int;
    pub fn hec_ec_volume_open_ex(base_filename: *const c_char, large_block_size: u64, small_block_size: u64,
                                 out: *mut *mut hec_ec_volume_t) -> c_int;
    pub fn hec_ec_volume_close(vol: *mut hec_ec_volume_t);
    pub fn hec_ec_volume_version(vol: *const hec_ec_volume_t) -> u32;
    pub fn hec_ec_volume_shard_bits(vol: *const hec_ec_volume_t) -> u32;
    pub fn hec_ec_volume_find_needle(vol: *const hec_ec_volume_t, needle_id: u64, offset: *mut u32,
                                     size: *mut i32) -> c_int;
    pub fn hec_ec_volume_delete_needle(vol: *mut hec_ec_volume_t, needle_id: u64) -> c_int;
    pub fn hec_ec_volume_read_needle(vol: *mut hec_ec_volume_t, needle_id: u64, out: *mut u8, cap: usize,
                                     n_out: *mut usize) -> c_int;
    pub fn hec_ec_volume_read_needles(vol: *mut hec_ec_volume_t, needle_ids: *const u64, n: usize, out: *mut u8,
                                      cap: usize, out_offsets: *mut u64, statuses: *mut c_int) -> c_int;

    // tuning / introspection (speed only)
    pub fn hec_set_host_staging(max_bytes: u64) -> c_int;
    pub fn hec_set_completion_signal(max_bytes: u64) -> c_int;
    pub fn hec_set_host_zero_copy(on: c_int) -> c_int;
    pub fn hec_host_encode_kernel_name(shard_len: u64) -> *const c_char;
    pub fn hec_host_zero_copy_view(p: *const c_void, bytes: u64, zero_copy: *mut c_int) -> c_int;
    pub fn hec_host_staging_stats(n_pipelines: *mut c_int, pinned_bytes: *mut u64, device_bytes: *mut u64) -> c_int;
    pub fn hec_version() -> *const c_char;
    pub fn hec_encode_kernel_name(shard_len: u64) -> *const c_char;
    pub fn hec_decode_kernel_name(shard_len: u64) -> *const c_char;
    pub fn hec_ragged_kernel_name(descs: *const hec_stripe_desc, n_stripes: u32, decode: c_int) -> *const c_char;
}

/*
 * hec.h -- C ABI of the MI355X-native RS(10,4) erasure-coding engine that
 * replaces helyim-ec's CPU path (libhec.so, built for gfx950).
 *
 * Every entry point takes plain pointers and sizes. Each one names the
 * reference interface it replaces (paths relative to /root/reference):
 *
 *  - the arithmetic boundary: reed_solomon_erasure::ReedSolomon<galois_8::Field>
 *    {new, encode, reconstruct} as called at helyim-ec/src/encoder.rs:191,
 *    208-209, 249-250, 288 and helyim-store/src/erasure_coding/mod.rs:411-412,
 *    426 (crate 6.0.0, git helyim/reed-solomon-erasure, Cargo.toml:72);
 *  - the crate API boundary: helyim_ec::write_ec_files / rebuild_ec_files
 *    (helyim-ec/src/encoder.rs:39-50, exported at helyim-ec/src/lib.rs:17),
 *    called by helyim-store/src/server.rs:468 and :497.
 *
 * All compute runs on the GPU through HIP kernels. There is no CPU fallback:
 * without a usable GPU every compute entry point returns HEC_ERR_NO_DEVICE or
 * HEC_ERR_HIP.
 *
 * Threading: a hec_rs_t is immutable after hec_rs_new and may be shared by
 * threads (upstream ReedSolomon is Send + Sync). Device state (tables,
 * decode-pattern cache, staging buffers) is per device and mutex guarded.
 * Host-memory entry points synchronise before returning, on error returns
 * too (no copy or kernel touching caller memory is left in flight); the
 * hec_gpu_* batch entry points are asynchronous on the caller's stream.
 */
#ifndef HEC_H
#define HEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes -------------------------------------------------------
 * 1..13 are 1:1 with reed_solomon_erasure::Error (declaration order);
 * 32..35 with helyim_ec::EcShardError (helyim-ec/src/errors.rs:55-66);
 * 64.. are device / argument errors of this library. */
enum hec_status {
    HEC_OK = 0,
    HEC_ERR_TOO_FEW_SHARDS = 1,
    HEC_ERR_TOO_MANY_SHARDS = 2,
    HEC_ERR_TOO_FEW_DATA_SHARDS = 3,
    HEC_ERR_TOO_MANY_DATA_SHARDS = 4,
    HEC_ERR_TOO_FEW_PARITY_SHARDS = 5,
    HEC_ERR_TOO_MANY_PARITY_SHARDS = 6,
    HEC_ERR_TOO_FEW_BUFFER_SHARDS = 7,
    HEC_ERR_TOO_MANY_BUFFER_SHARDS = 8,
    HEC_ERR_INCORRECT_SHARD_SIZE = 9,
    HEC_ERR_TOO_FEW_SHARDS_PRESENT = 10,
    HEC_ERR_EMPTY_SHARD = 11,
    HEC_ERR_INVALID_SHARD_FLAGS = 12,
    HEC_ERR_INVALID_INDEX = 13,
    HEC_ERR_IO = 32,                      /* EcShardError::Io */
    HEC_ERR_UNDERFLOW = 33,               /* EcShardError::Underflow */
    HEC_ERR_UNEXPECTED_EC_SHARD_SIZE = 34,/* EcShardError::UnexpectedEcShardSize */
    HEC_ERR_UNEXPECTED_BLOCK_SIZE = 35,   /* EcShardError::UnexpectedBlockSize */
    HEC_ERR_NEEDLE_NOT_FOUND = 48,        /* EcVolumeError::NeedleNotFound */
    HEC_ERR_SHARD_NOT_FOUND = 49,         /* EcVolumeError::ShardNotFound */
    HEC_ERR_HIP = 64,                     /* a HIP runtime call failed */
    HEC_ERR_NO_DEVICE = 65,               /* no usable GPU */
    HEC_ERR_INVALID_ARGUMENT = 66,        /* null pointer, bad stride, ... */
    HEC_ERR_OUT_OF_MEMORY = 67
};

/* Static text for a status code (the upstream Display string where one exists). */
const char* hec_strerror(int status);
/* Thread-local detail of the last failure on this thread (e.g. the errno text,
 * the two sizes of UnexpectedEcShardSize). Empty string when none. */
const char* hec_last_error_detail(void);
/* Payload of the last failure on this thread, so a binding can rebuild the
 * reference's error values (helyim-ec/src/errors.rs:55-66), not only its
 * variant: *a / *b = the two usizes of UnexpectedEcShardSize(expected, actual)
 * (encoder.rs:276-279) and UnexpectedBlockSize(block_size, buf_size)
 * (encoder.rs:140-143); *os_errno = the errno behind an HEC_ERR_IO (the
 * io::Error of EcShardError::Io, encoder.rs:175 -- 0 when the failure had no OS
 * error, e.g. a short read). Meaningful right after a call returned one of
 * codes 32..35 (every such return sets all three; 0 where the variant has no
 * such value); other statuses may leave stale values. Null pointers are
 * skipped. Returns HEC_OK. */
int hec_last_error_values(uint64_t* a, uint64_t* b, int* os_errno);

/* ---- device selection (no reference counterpart: helyim has no GPU) -------
 * Every entry point works on the calling thread's current HIP device. A
 * multi-GPU volume server that does not link HIP itself picks the device per
 * call with these, e.g. volume_id % count before hec_write_ec_files (whole
 * volumes per GPU); per-device state is independent, so calls
 * on different devices run concurrently. */
int hec_device_count(int* count);  /* HEC_ERR_NO_DEVICE (and 0) without a GPU */
int hec_set_device(int device);    /* this thread only; HEC_ERR_INVALID_ARGUMENT if out of range */
int hec_get_device(int* device);

/* ---- NUMA placement of the host side of a GPU (no reference
 * counterpart: helyim is CPU-only) -------------------------------------------
 * Every pinned buffer libhec allocates (host-batch and file-layer staging,
 * small-call staging, degraded-read staging) lives on the NUMA node of the
 * device it serves. */
/* sysfs NUMA node of the device's PCI function; -1 when the platform does not
 * say. */
int hec_device_numa_node(int device, int* node);
/* Restrict the calling thread (and threads it creates later) to the CPUs of
 * the device's NUMA node that it is allowed to run on; *n_cpus (optional) =
 * how many. No-op (HEC_OK, 0 CPUs) when the node is unknown or none of its
 * CPUs is in the thread's allowed set. */
int hec_bind_thread_to_device(int device, int* n_cpus);
/* Pinned host memory on the current device's NUMA node, addressable by the
 * GPU (host-batch entry points code it zero-copy). Free with hec_host_free. */
int hec_host_alloc(size_t bytes, void** out);
/* One pinned host batch of n_stripes * stripe_stride bytes for the _multi
 * calls over the same device list: range r = stripes [S*r/R, S*(r+1)/R)
 * (R = min(n_devices, n_stripes), the split hec_host_*_batch_multi uses) has
 * its pages preferred on devices[r]'s NUMA node (mbind before the first
 * touch; a page straddling two ranges goes with the earlier one), so on a
 * two-socket node every GPU's range is read and written on its own socket.
 * Zero-filled, pinned and mapped for every device (zero-copy for any range).
 * Placement is speed only: a node short of memory spills to the others.
 * Free with hec_host_free. Errors: HEC_ERR_INVALID_ARGUMENT (empty list, > 256
 * entries, a device out of range, empty or overflowing batch). */
int hec_host_alloc_multi(const int* devices, size_t n_devices, uint64_t stripe_stride, uint32_t n_stripes,
                         void** out);
int hec_host_free(void* p);
/* NUMA node holding the page at p (diagnostic; HEC_ERR_IO if not resident). */
int hec_host_numa_node(const void* p, int* node);

/* ---- geometry constants (helyim-ec/src/lib.rs:46-50) ---------------------- */
#define HEC_DATA_SHARDS_COUNT 10u
#define HEC_PARITY_SHARDS_COUNT 4u
#define HEC_TOTAL_SHARDS_COUNT 14u
#define HEC_LARGE_BLOCK_SIZE (1024ull * 1024ull * 1024ull)
#define HEC_SMALL_BLOCK_SIZE (1024ull * 1024ull)

/* ---- codec context: replaces ReedSolomon<galois_8::Field> ----------------- */
typedef struct hec_rs hec_rs_t;

/* ReedSolomon::new(data_shards, parity_shards) (encoder.rs:208-209).
 * Errors: TOO_FEW_DATA_SHARDS (0 data), TOO_FEW_PARITY_SHARDS (0 parity),
 * TOO_MANY_SHARDS (data + parity > 256). */
int hec_rs_new(size_t data_shards, size_t parity_shards, hec_rs_t** out);
void hec_rs_free(hec_rs_t* rs);
size_t hec_rs_data_shard_count(const hec_rs_t* rs);
size_t hec_rs_parity_shard_count(const hec_rs_t* rs);
size_t hec_rs_total_shard_count(const hec_rs_t* rs);
/* Copies the (total x data) row-major encoding matrix into out. */
int hec_rs_matrix(const hec_rs_t* rs, uint8_t* out, size_t out_len);

/* ReedSolomon::encode(&mut shards) (encoder.rs:191), host memory.
 * shards[0..data) are read, shards[data..total) receive parity in place.
 * shard_lens[i] is the length of shards[i]. Errors: TOO_FEW_SHARDS /
 * TOO_MANY_SHARDS (n_shards != total), EMPTY_SHARD, INCORRECT_SHARD_SIZE. */
int hec_rs_encode(const hec_rs_t* rs, uint8_t* const* shards, const size_t* shard_lens,
                  size_t n_shards);

/* ReedSolomon::verify(&shards): *ok = 1 when the parity matches the data. */
int hec_rs_verify(const hec_rs_t* rs, const uint8_t* const* shards, const size_t* shard_lens,
                  size_t n_shards, int* ok);

/* ReedSolomon::reconstruct(&mut [Option<Vec<u8>>]) (encoder.rs:288,
 * erasure_coding/mod.rs:426). present[i] != 0 marks Some(shard); shard_lens
 * of absent slots are ignored. Absent slots must point at a caller buffer of
 * the common shard length (upstream allocates vec![0; len]); they are filled.
 * All present -> no-op. Errors: TOO_FEW_SHARDS / TOO_MANY_SHARDS,
 * EMPTY_SHARD, INCORRECT_SHARD_SIZE, TOO_FEW_SHARDS_PRESENT. Decode uses the
 * first data_shards present shards in index order, as upstream does. */
int hec_rs_reconstruct(const hec_rs_t* rs, uint8_t* const* shards, const size_t* shard_lens,
                       const uint8_t* present, size_t n_shards);
/* ReedSolomon::reconstruct_data: as above but absent parity slots are left
 * untouched. */
int hec_rs_reconstruct_data(const hec_rs_t* rs, uint8_t* const* shards, const size_t* shard_lens,
                            const uint8_t* present, size_t n_shards);

/* Batched ReedSolomon::reconstruct over n_stripes independent stripes of any
 * lengths in ONE GPU round trip -- the degraded-read path
 * (helyim-store/src/erasure_coding/mod.rs:403-491 reconstructs one needle
 * interval per call). shards / lens / present are n_stripes * total entries,
 * stripe-major; per stripe the semantics and errors are hec_rs_reconstruct's
 * (reconstruct_data when data_only != 0). Every stripe is validated before
 * any work; on error nothing is written and *bad_index (optional) names the
 * first failing stripe. */
int hec_rs_reconstruct_batch(const hec_rs_t* rs, uint8_t* const* shards, const size_t* lens,
                             const uint8_t* present, size_t n_stripes, int data_only, size_t* bad_index);

/* ---- device-resident batches (no reference counterpart: the GPU form of the
 * encode_data_one_batch loop, encoder.rs:158-198, over many stripes) -------
 * Shard (stripe s, shard i) lives at base + s*stripe_stride + i*shard_stride.
 * Pointers are device pointers on the current HIP device; stream is a
 * hipStream_t (NULL = default stream). Calls are asynchronous.
 * Layout (speed only): with 1 MiB shards, a 64 KiB gap after each shard
 * (shard_stride = shard_len + 65536) runs encode and decode ~1.6% faster than
 * packed shards (the bench's batch is laid out so). */

/* Encode n_stripes stripes: read data shards 0..data from d_data, write parity
 * shards 0..parity to d_parity (shard index relative to each base).
 * All strided batches (device and host) return HEC_ERR_INVALID_ARGUMENT,
 * before any device work, when shards of a stripe overlap (shard stride <
 * shard_len), stripes overlap (stripe stride < shard_len) or the batch's byte
 * extent wraps 64 bits. Buffer sizes themselves cannot be checked here. */
int hec_gpu_encode_batch(const hec_rs_t* rs,
                         const uint8_t* d_data, uint64_t data_stripe_stride, uint64_t data_shard_stride,
                         uint8_t* d_parity, uint64_t parity_stripe_stride, uint64_t parity_shard_stride,
                         uint64_t shard_len, uint32_t n_stripes, void* stream);

/* Reconstruct n_stripes stripes of all total shards in place. d_present_masks
 * (device, n_stripes words): bit i set = shard i present. Stripes with every
 * shard present are left untouched (upstream no-op); stripes with fewer than
 * data_shards present are skipped and counted into *d_bad_stripes (device
 * word, optional, accumulated). Requires total shards <= 16. */
int hec_gpu_reconstruct_batch(const hec_rs_t* rs, uint8_t* d_shards, uint64_t stripe_stride,
                              uint64_t shard_stride, uint64_t shard_len, uint32_t n_stripes,
                              const uint32_t* d_present_masks, uint32_t* d_bad_stripes,
                              void* stream);

/* ---- host-memory batches (the path helyim runs: bytes start and end in host
 * memory, encoder.rs:169-195 / 263-304) -------------------------------------
 * Same strided layout as above but on HOST pointers; synchronous on return.
 * Pinned buffers the GPU can address (hipHostMalloc, torch pin_memory) are
 * coded zero-copy: the kernel reads and writes them over PCIe directly.
 * Pageable memory is copied chunk by chunk (host worker pool) into pinned
 * slots that the kernel codes in place, the copies of one chunk overlapping
 * the kernel of the next. With hec_set_host_zero_copy(0) both go through
 * H2D -> kernel -> D2H over 3 HIP streams. */
int hec_host_encode_batch(const hec_rs_t* rs,
                          const uint8_t* h_data, uint64_t data_stripe_stride, uint64_t data_shard_stride,
                          uint8_t* h_parity, uint64_t parity_stripe_stride, uint64_t parity_shard_stride,
                          uint64_t shard_len, uint32_t n_stripes);
/* Reconstruct in place with per-stripe host masks (bit i = shard i present):
 * only the first data_shards present shards of a stripe cross PCIe H2D and
 * only its erased shards cross D2H. Stripes with fewer than data_shards
 * present are skipped and counted into *n_bad_stripes (optional). Requires
 * total shards <= 16. */
int hec_host_reconstruct_batch(const hec_rs_t* rs, uint8_t* h_shards, uint64_t stripe_stride,
                               uint64_t shard_stride, uint64_t shard_len, uint32_t n_stripes,
                               const uint32_t* h_present_masks, uint32_t* n_bad_stripes);

/* One host batch spread over several GPUs of this process (SURVEY.md §8e:
 * contiguous stripe ranges per GPU; helyim's volume server is one process,
 * helyim-store/src/server.rs:451-506, so without this one call is capped by
 * one GPU's PCIe link). devices[0..n_devices) may repeat a device (two
 * concurrent ranges on it). Range r = stripes [S*r/R, S*(r+1)/R), R =
 * min(n_devices, n_stripes), runs on devices[r] from its own host thread
 * (CPUs bound to that GPU's NUMA node) through hec_host_encode_batch /
 * hec_host_reconstruct_batch, with its own streams and staging. Synchronous:
 * returns when every range is done; on failure the status of the first
 * failing range in list order (hec_last_error_detail names the range).
 * Arguments and results otherwise as the single-device calls;
 * *n_bad_stripes is the sum over ranges. An empty list or a device out of
 * range, or more than 256 entries -> HEC_ERR_INVALID_ARGUMENT before any work. */
int hec_host_encode_batch_multi(const hec_rs_t* rs, const int* devices, size_t n_devices,
                                const uint8_t* h_data, uint64_t data_stripe_stride, uint64_t data_shard_stride,
                                uint8_t* h_parity, uint64_t parity_stripe_stride, uint64_t parity_shard_stride,
                                uint64_t shard_len, uint32_t n_stripes);
int hec_host_reconstruct_batch_multi(const hec_rs_t* rs, const int* devices, size_t n_devices,
                                     uint8_t* h_shards, uint64_t stripe_stride, uint64_t shard_stride,
                                     uint64_t shard_len, uint32_t n_stripes, const uint32_t* h_present_masks,
                                     uint32_t* n_bad_stripes);

/* Ragged device batches (RS(10,4)): every stripe has its own length, shard
 * stride and erasure pattern -- BASELINE config 5's mixed 64 KiB-4 MiB
 * stripes in ONE launch. Stripe j's shard i is at d_base + offset + i *
 * shard_stride (offset, stride and d_base 16-byte aligned, stride >=
 * shard_len). Encode reads shards 0..9 and writes 10..13; reconstruct uses
 * present_mask like hec_gpu_reconstruct_batch. descs are HOST memory; the
 * launch is asynchronous on `stream`. */
typedef struct hec_stripe_desc {
    uint64_t offset;
    uint64_t shard_stride;
    uint32_t shard_len;
    uint32_t present_mask;
} hec_stripe_desc;
int hec_gpu_encode_ragged(const hec_rs_t* rs, uint8_t* d_base, const hec_stripe_desc* descs,
                          uint32_t n_stripes, void* stream);
int hec_gpu_reconstruct_ragged(const hec_rs_t* rs, uint8_t* d_base, const hec_stripe_desc* descs,
                               uint32_t n_stripes, uint32_t* d_bad_stripes, void* stream);

/* Deterministic splitmix64 stripe data (bench / test inputs): stripe s gets
 * bytes_per_stripe bytes at d_base + s*stripe_stride, 64-bit word n (n >= 1)
 * = splitmix64_mix(seed_base + s + n * 0x9E3779B97F4A7C15), little endian. */
int hec_gpu_fill_splitmix(uint8_t* d_base, uint64_t stripe_stride, uint64_t bytes_per_stripe,
                          uint32_t n_stripes, uint64_t seed_base, void* stream);

/* ---- file level: helyim_ec::write_ec_files / rebuild_ec_files ------------ */

/* write_ec_files(base_filename) (encoder.rs:39-46): base.dat -> base.ec00..ec13. */
int hec_write_ec_files(const char* base_filename);
/* generate_ec_files(base, buf_size, large_block_size, small_block_size)
 * (encoder.rs:52-71): same, with explicit geometry (tests use small blocks to
 * exercise the large-row path). */
int hec_write_ec_files_ex(const char* base_filename, uint64_t buf_size, uint64_t large_block_size,
                          uint64_t small_block_size);
/* rebuild_ec_files(base_filename) -> Vec<u32> (encoder.rs:48-50, 73-109,
 * 244-307): recreates every missing .ecNN. rebuilt_ids (capacity 14) receives
 * the rebuilt shard ids in ascending order, *n_rebuilt their count. */
int hec_rebuild_ec_files(const char* base_filename, uint32_t* rebuilt_ids, size_t* n_rebuilt);

/* ---- EC volume files around the shards (host-side byte formats) ----------- */
/* write_sorted_file_from_index(base, ext) (encoder.rs:21-37): replay base.idx
 * (16-byte BE entries; offset 0 or negative size deletes) and write the live
 * entries sorted by needle id to base+ext (".ecx"). */
int hec_write_sorted_file_from_index(const char* base_filename, const char* ext);
/* rebuild_ecx_file(base) (lib.rs:95-133): apply base.ecj tombstones to base.ecx,
 * then delete base.ecj; no .ecj -> HEC_OK. */
int hec_rebuild_ecx_file(const char* base_filename);
/* save_volume_info(filename, VolumeInfo{version}) as the generate RPC writes it
 * (volume_info.rs:121-132, server.rs:470-475). */
int hec_save_volume_info(const char* filename, uint32_t version);
/* find_data_filesize(base) (decoder.rs:46-66). */
int hec_find_data_filesize(const char* base_filename, uint64_t* data_filesize);
/* write_data_file(base, size) (decoder.rs:142-180): .ec00-.ec09 -> base.dat. */
int hec_write_data_file(const char* base_filename, int64_t data_filesize);
/* write_index_file_from_ec_index(base) (decoder.rs:22-44): .ecx + .ecj -> .idx. */
int hec_write_index_file_from_ec_index(const char* base_filename);

/* ---- needle reads from EC shards (locate + degraded read) ----------------- */
/* Interval (helyim-ec/src/locate.rs:3-9). */
typedef struct hec_interval {
    uint64_t block_index;
    uint64_t inner_block_offset;
    uint64_t size;
    uint64_t large_block_rows;
    uint32_t is_large_block;
    uint32_t reserved;
} hec_interval;
/* locate_data(large_block_len, small_block_len, data_size, offset, size)
 * (locate.rs:29-72, with locate_offset :74-100 and its own large-row count).
 * Writes up to cap intervals; *n_out = the number locate_data yields (an
 * HEC_ERR_INVALID_ARGUMENT when it exceeds cap). */
int hec_locate_data(uint64_t large_block_len, uint64_t small_block_len, uint64_t data_size, uint64_t offset,
                    uint64_t size, hec_interval* out, size_t cap, size_t* n_out);
/* Interval::shard_id (locate.rs:12-15) and Interval::offset (:17-27). */
uint32_t hec_interval_shard_id(const hec_interval* interval);
uint64_t hec_interval_offset(const hec_interval* interval, uint64_t large_block_size, uint64_t small_block_size);
/* EcVolume::find_needle_from_ecx (volume/mod.rs:153-155 ->
 * search_needle_from_sorted_index, lib.rs:54-82): binary search of base.ecx.
 * *offset is the stored Offset (units of 8 bytes), *size the stored Size (< 0
 * = deleted). Absent id -> HEC_ERR_IO ("Needle {id} is not found",
 * io::ErrorKind::NotFound). */
int hec_find_needle_from_ecx(const char* base_filename, uint64_t needle_id, uint32_t* offset, int32_t* size);
/* read_ec_shard_intervals (erasure_coding/mod.rs:303-401) over n_ranges
 * (offset, size) ranges of the volume's data, against the local shard files
 * base.ec00..ec13 (data_size = first shard file's size x 10, volume/mod.rs:146).
 * An interval on a present shard is read from it (short read -> HEC_ERR_IO);
 * an interval on a missing shard is rebuilt from the other shards' same range
 * (recover_one_remote_ec_shard_interval, :403-491: full-length reads count as
 * present; fewer than 10 -> HEC_ERR_TOO_FEW_SHARDS_PRESENT). All rebuilt
 * intervals of the call go to the GPU as one batch. out receives the ranges
 * back to back (sum of sizes bytes). No shard file -> HEC_ERR_SHARD_NOT_FOUND. */
int hec_read_ec_data(const char* base_filename, uint64_t large_block_size, uint64_t small_block_size,
                     const uint64_t* offsets, const uint64_t* sizes, size_t n_ranges, uint8_t* out);
/* read_ec_shard_needle's data path (erasure_coding/mod.rs:129-171): look the
 * needle up in base.ecx, HEC_ERR_NEEDLE_NOT_FOUND if deleted, then read its
 * actual_size bytes at actual_offset (Offset * 8 as u32, Size::actual_size)
 * through hec_read_ec_data with the 1 GiB / 1 MiB blocks. *n_out = the
 * needle's byte count; cap smaller than that -> HEC_ERR_INVALID_ARGUMENT.
 * Parsing the needle record is the caller's (Needle::read_bytes). */
int hec_read_ec_needle(const char* base_filename, uint64_t needle_id, uint8_t* out, size_t cap, size_t* n_out);
/* hec_read_ec_needle with explicit block sizes (tests exercise large rows). */
int hec_read_ec_needle_ex(const char* base_filename, uint64_t large_block_size, uint64_t small_block_size,
                          uint64_t needle_id, uint8_t* out, size_t cap, size_t* n_out);
/* Many needle reads of one volume in one call (a server's concurrent reads):
 * every lost interval of every needle is rebuilt in one GPU batch.
 * statuses[i] = HEC_OK, HEC_ERR_IO (id not in .ecx) or HEC_ERR_NEEDLE_NOT_FOUND
 * (deleted); found needles' bytes go back to back into out, needle i at
 * [out_offsets[i], out_offsets[i+1]) (empty when not found); out_offsets has
 * n + 1 entries and is filled even when cap is too small (then
 * HEC_ERR_INVALID_ARGUMENT). A shard read or reconstruct failure fails the
 * whole call with that status. */
int hec_read_ec_needles(const char* base_filename, uint64_t large_block_size, uint64_t small_block_size,
                        const uint64_t* needle_ids, size_t n, uint8_t* out, size_t cap, uint64_t* out_offsets,
                        int* statuses);

/* ---- mounted EC volume (EcVolume, helyim-ec/src/volume/mod.rs:30-171) -------
 * A handle that keeps the volume's files open for a stream of reads, so a
 * needle read costs the lookup and the preads only. */
typedef struct hec_ec_volume hec_ec_volume_t;
/* EcVolume::new (mod.rs:45-92) + add_ec_shard (mod.rs:94-108) for every local
 * base.ecNN: opens base.ecx read-write (missing -> HEC_ERR_IO), opens or
 * creates base.ecj, loads the version from base.vif -- a missing .vif or one
 * whose `files` list is empty (maybe_load_volume_info, volume_info.rs:107-119)
 * is (re)written as the default VolumeInfo with version 2 -- and mounts every
 * shard file present. 1 GiB / 1 MiB blocks (ERASURE_CODING_*_BLOCK_SIZE). */
int hec_ec_volume_open(const char* base_filename, hec_ec_volume_t** out);
/* hec_ec_volume_open with explicit block sizes (tests exercise large rows). */
int hec_ec_volume_open_ex(const char* base_filename, uint64_t large_block_size, uint64_t small_block_size,
                          hec_ec_volume_t** out);
void hec_ec_volume_close(hec_ec_volume_t* vol);
/* EcVolume::version; 0 for a null handle. */
uint32_t hec_ec_volume_version(const hec_ec_volume_t* vol);
/* Bit i set = shard i mounted. */
uint32_t hec_ec_volume_shard_bits(const hec_ec_volume_t* vol);
/* find_needle_from_ecx (mod.rs:153-155), as hec_find_needle_from_ecx. */
int hec_ec_volume_find_needle(const hec_ec_volume_t* vol, uint64_t needle_id, uint32_t* offset, int32_t* size);
/* delete_needle_from_ecx (mod.rs:157-171): the entry's size becomes the
 * tombstone (-1) in .ecx (mark_needle_deleted, lib.rs:88-93) and the id is
 * appended to .ecj (8 bytes, big-endian). Absent id -> HEC_ERR_IO ("Needle {id}
 * is not found"), nothing written. Deletes are serialised per handle. */
int hec_ec_volume_delete_needle(hec_ec_volume_t* vol, uint64_t needle_id);
/* hec_read_ec_needle / hec_read_ec_needles against the mounted files (same
 * arguments, statuses and errors). Reads may run concurrently on one handle. */
int hec_ec_volume_read_needle(hec_ec_volume_t* vol, uint64_t needle_id, uint8_t* out, size_t cap, size_t* n_out);
int hec_ec_volume_read_needles(hec_ec_volume_t* vol, const uint64_t* needle_ids, size_t n, uint8_t* out, size_t cap,
                               uint64_t* out_offsets, int* statuses);

/* ---- tuning / introspection ----------------------------------------------- */
/* Kernel choice has no knob: it follows the shard length, the alignment and
 * where the bytes live (hec_*_kernel_name below report it). The knobs left
 * (process-wide, results identical) are the host paths' thresholds and mode. */
/* Host-memory encode / reconstruct calls whose input (data shards x shard
 * length) is at most max_bytes are packed into pinned staging and moved with
 * one H2D and one D2H copy; larger calls copy each shard directly. 0 disables
 * staging. Default 16 MiB (the measured crossover). Speed only. Returns HEC_OK. */
int hec_set_host_staging(uint64_t max_bytes);
/* Host batches (and the per-call and degraded-read staging): 1 = zero-copy
 * kernels that stream host memory over PCIe themselves (default), 0 = the
 * copy pipeline: DMA copies H2D -> kernel at HBM speed -> D2H over 3 HIP
 * streams, so the CUs are not held for the transfer (a GPU shared with other
 * work) at a lower link rate (41-44 against 51-53 GiB/s of data, DESIGN.md
 * section 5). Identical results. Returns HEC_OK. */
int hec_set_host_zero_copy(int on);
/* Name of the kernel a zero-copy host-batch encode of this shard length runs
 * (static string): over PCIe the 8-byte-per-lane table encode where the shard
 * length is a multiple of 2 KiB (~3.5% faster there than the bit-sliced kernel,
 * profiles/r04/e2e_encode_kernels_{v,w}.jsonl). */
const char* hec_host_encode_kernel_name(uint64_t shard_len);
/* Diagnostic: *zero_copy = 1 when [p, p + bytes) is one pinned range the
 * current device can address, i.e. host batches on it are coded zero-copy
 * (hec_host_alloc, hec_host_alloc_multi, hipHostMalloc, torch pin_memory),
 * 0 when they go through staging copies (pageable memory), or with
 * hec_set_host_zero_copy(0). */
int hec_host_zero_copy_view(const void* p, uint64_t bytes, int* zero_copy);
/* Diagnostic: host-batch pipelines of the current device (at most 8; only
 * the first 2 keep their staging between calls, the others free it when
 * their call ends) and the pinned host / device staging bytes they hold now.
 * Waits for calls in flight on those pipelines. */
int hec_host_staging_stats(int* n_pipelines, uint64_t* pinned_bytes, uint64_t* device_bytes);
/* Host-memory calls coded zero-copy whose input is at most max_bytes learn
 * that the kernel finished from a flag the kernel's last workgroup stores in
 * pinned memory (the caller spins on it, up to 200 us, then falls back to a
 * stream synchronise) instead of hipStreamSynchronize: ~4 us less per small
 * call. 0 disables. Default 1 MiB. Speed only. Returns HEC_OK. */
int hec_set_completion_signal(uint64_t max_bytes);
/* Version string of the library build. */
const char* hec_version(void);
/* Name of the kernel a 16-byte-aligned RS(10,4) device batch encode of this
 * shard length runs (static string;
 * shard_len 0, which fails with HEC_ERR_EMPTY_SHARD before any launch, names
 * no kernel: "none (...)"). */
const char* hec_encode_kernel_name(uint64_t shard_len);
/* Same for a 16-byte-aligned in-place RS(10,4) device batch reconstruct. */
const char* hec_decode_kernel_name(uint64_t shard_len);
/* Kernel hec_gpu_encode_ragged (decode = 0) or hec_gpu_reconstruct_ragged
 * (decode != 0) runs on these descriptors: the same choice the launch makes
 * (static string). */
const char* hec_ragged_kernel_name(const hec_stripe_desc* descs, uint32_t n_stripes, int decode);

#ifdef __cplusplus
}
#endif
#endif /* HEC_H */

// Shared host/device declarations for the gfx950 RS kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "fastdiv.hpp"

namespace hec {

// One coding plan: nout output rows = coefficient matrix (nout x nin) applied
// to the nin input shards of a stripe. Encode is one plan (inputs = data
// shards, outputs = parity shards); decode has one plan per erasure pattern
// (inputs = first nin present shards, outputs = erased shards), matching
// upstream reconstruct's "first data_shard_count present shards" rule.
struct DevPlan {
    uint32_t nin;      // inputs (== data shard count)
    uint32_t nout;     // outputs; 0 = nothing to do (all shards present)
    uint32_t tab_off;  // word offset of this plan's tables: [nin][tab_rows][kTabWords]
    uint32_t idx_off;  // word offset of [nin] input shard ids then [nout] output ids
    uint32_t tab_rows; // table row stride (>= nout; padded rows hold coefficient 0)
    uint32_t pad[3];
};

constexpr uint32_t kNoPlan = 0xFFFFFFFFu;   // mask LUT entry: too few shards present
constexpr int kThreads = 256;               // 4 waves of 64 lanes
// Workgroups per launch: the dispatch packet's grid is 32-bit in work-items,
// so 2^23 workgroups (2^31 work-items at 256 threads) keeps every launch legal.
constexpr uint64_t kMaxLaunchBlocks = 1ull << 23;
constexpr int kVecBytes = 16;               // one dwordx4 per lane per access

struct ApplyArgs {
    const uint8_t* in_base;      // input shard (stripe s, id i) = in_base + s*in_stripe + i*in_shard
    uint64_t in_stripe;
    uint64_t in_shard;
    uint8_t* out_base;           // output shard (stripe s, id j) = out_base + s*out_stripe + j*out_shard
    uint64_t out_stripe;
    uint64_t out_shard;
    uint64_t len;                // shard length in bytes (same for every stripe of the batch)
    uint64_t n_items;            // n_stripes * chunks_per_stripe
    uint32_t chunks_per_stripe;  // ceil(len / chunk_bytes)
    uint32_t n_stripes;
    const DevPlan* plans;
    const uint32_t* tabs;
    const uint32_t* idx;
    const uint32_t* masks;       // optional per-stripe present mask (bit i = shard i present)
    const uint32_t* lut;         // mask -> plan id (used when masks != nullptr)
    uint32_t mask_limit;         // (1 << total shards) - 1: masks are clipped to the LUT
    uint32_t* bad_count;         // optional: stripes skipped for too few present shards
    uint32_t fast104;            // 1: RS(10,4) plan set with 4-row tables; encode = plan 0 at
                                 //    offset 0, decode = tables at lut[mask] * 200 words
    // Launcher-computed workgroup -> chunk map of the RS(10,4) fast paths, so
    // the kernels derive (stripe, chunk) in a few scalar ops with no division:
    uint32_t map_q8, map_r8;     // workgroups / 8 and % 8 (XCD eighths remap)
    uint32_t cps_mul, cps_shift; // item / chunks_per_stripe as a multiply-shift (FastDiv)
    // Optional completion signal (small host calls): the last workgroup of
    // the launch stores done_seq into done_flag (pinned host memory) after a
    // system-scope release, so the host spins on it instead of paying
    // hipStreamSynchronize. done_count: device word, 0 between launches.
    uint32_t* done_count;
    uint32_t* done_flag;
    uint32_t done_seq;
};

// Ragged RS(10,4) batch (every stripe its own length / stride / mask); all
// strides 16-byte aligned. Stripe s has shards at base + off + i*shard_stride
// and owns workgroups [first_block, first_block + ceil(len / 4 KiB)).
struct RaggedItem {
    uint64_t off;          // shard 0 (full layout) or input slot 0 (compact layout)
    uint64_t shard_stride;
    uint32_t len;
    uint32_t mask;         // present mask (decode); ignored by encode
    uint32_t first_block;
    uint32_t pad;
    uint64_t out_off;      // compact decode: output slot 0 (erased shards, ascending)
};

struct RaggedArgs {
    uint8_t* base;
    const RaggedItem* items;
    const uint32_t* block_item;  // workgroup -> stripe index
    uint32_t n_blocks;
    const uint32_t* tabs;        // encode plan tables, or the dense decode set
    const uint32_t* lut;         // decode: mask -> plan id
    uint32_t* bad_count;
    uint32_t compact;            // decode: inputs = slots 0..9 at off (the first 10 present
                                 // shards), outputs = slots 0..e-1 at out_off (erased shards)
    uint32_t block_base;         // launcher-internal: first map entry of this launch
    uint32_t map_q8, map_r8;     // launcher-internal: that launch's workgroups / 8 and % 8
    uint32_t inline_one;         // 1: a single stripe, described by `one` (no items / map in memory)
    RaggedItem one;
    uint32_t* done_count;        // optional completion signal, as ApplyArgs
    uint32_t* done_flag;
    uint32_t done_seq;
};

hipError_t launch_rs104_ragged(const RaggedArgs& a, bool decode, hipStream_t stream);
// Bit-sliced ragged encode: every stripe's length a multiple of kBsChunk bytes;
// the workgroup map has len / kBsChunk entries per stripe.
constexpr uint32_t kBsChunk = 2 * kThreads * kVecBytes;  // 8 KiB
// Column range of one workgroup of the 8-byte-per-lane table kernels.
constexpr uint32_t kNarrowChunk = kThreads * 8;  // 2 KiB
hipError_t launch_rs104_bs_ragged(const RaggedArgs& a, hipStream_t stream);


// Launch one coding pass. nin: number of inputs the caller guarantees (10
// selects the unrolled helyim RS(10,4) path; anything else the generic loop).
// over_pcie: an encode whose operands are host memory the kernel streams over
// PCIe (zero-copy host batches): the 8-byte-per-lane table encode where the
// shard length is a multiple of 2 KiB instead of the bit-sliced one (its
// narrower column range per workgroup ran 50.5-52.9 against 49.4-51.1 GiB/s
// in 7 alternating rounds on two boxes, profiles/r04/e2e_encode_kernels_{v,w}.jsonl).
hipError_t launch_apply(const ApplyArgs& a, int nin, bool aligned, bool over_pcie, hipStream_t stream);

// Name of the kernel an aligned RS(10,4) device encode of one stripe of this
// shard length runs under cfg (introspection for benchmarks and profiles; the
// same choice launch_apply makes, rs_kernels.hip rs104_pick).
const char* encode_kernel_name(uint64_t len, bool over_pcie);
// Same for an aligned in-place RS(10,4) device batch reconstruct.
const char* decode_kernel_name(uint64_t len);

// splitmix64 byte stream per stripe (bench/test data generator):
// stripe s: bytes_per_stripe bytes at base + s*stripe_stride, word n (n>=1) =
// mix(seed_base + s + n*gamma), little endian.
hipError_t launch_fill_splitmix(uint8_t* base, uint64_t stripe_stride, uint64_t bytes_per_stripe,
                                uint32_t n_stripes, uint64_t seed_base, hipStream_t stream);

}  // namespace hec

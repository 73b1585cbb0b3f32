// gfx950 (CDNA4) kernels for the helyim-ec RS(10,4) hot path.
//
// Replaces the arithmetic of upstream reed-solomon-erasure's
// `ReedSolomon::encode` / `reconstruct` (called from
// /root/reference/helyim-ec/src/encoder.rs:191,288 and
// helyim-store/src/erasure_coding/mod.rs:426), whose CPU kernel is a pshufb
// nibble-table loop run 40 times per 256 KiB batch.
//
// Design (see DESIGN.md "Kernels"):
//  * One pass per stripe chunk: every input byte is read from HBM once and
//    every output byte written once (14 L bytes per encoded stripe), instead
//    of the CPU's 10 read-modify-write sweeps per output.
//  * GF(2^8) constant multiply as a byte-sliced SWAR lookup on whole dwords:
//    c*x = T0[x&7] ^ T1[(x>>3)&7] ^ T2[x>>6]; each table is <= 8 bytes, so one
//    v_perm_b32 performs four lookups. Three v_perm + 1.5 v_bitop3 (xor3) per
//    coefficient per dword; selectors are shared by all output rows.
//  * Tables and shard ids are wave-uniform -> scalar loads (SGPRs); only the
//    data is vector traffic: coalesced loads and stores (1 KiB per wave
//    instruction at 16 B per lane), non-temporal since every byte is touched
//    once.
//  * The encode of shard lengths that are a multiple of 8 KiB is bit-sliced
//    (rs104_bs_encode_kernel): the fixed parity matrix as a generated XOR
//    program over bit planes, half the table multiply's VALU work.
//
// Every kernel here is a product path: rs104_pick / ragged_pick choose among
// them by shard length, alignment and where the bytes live. Variants measured
// and not kept (XOR-only twins, the pair kernel, chunk rotation,
// 128/512/1024-thread launches, 4 B and 8 B-load variants, occupancy caps, the
// round-6 32-byte-per-lane table decode) are in git history and
// profiles/r0*/INDEX.md; the math-free stream ceilings live in
// tools/membench.hip.
#include <algorithm>
#include <type_traits>

#include "rs_kernels.hpp"
#include "bitslice.hpp"

namespace hec {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Scalar-cache view of plan metadata: uniform loads through the constant
// address space become s_load (SGPR) instead of per-lane vector loads.
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(4))) T* as_const(const T* p) {
    return (const __attribute__((address_space(4))) T*)(p);
}
typedef const __attribute__((address_space(4))) uint32_t* cu32p;

// Global-address-space views: the nontemporal hint on a flat (generic)
// pointer is dropped by the backend (plain global_load_dwordx4), so the
// streamed shards -- each byte touched exactly once -- are accessed through
// address_space(1) pointers to get `nt` (+2-4%, profiles/r01/tune11_*.jsonl;
// other cache policies through raw buffer instructions measured no better,
// profiles/r02/ab_cache_policy_buffer_*.txt).
typedef const __attribute__((address_space(1))) u32x4* gcu32x4p;
typedef __attribute__((address_space(1))) u32x4* gu32x4p;
typedef const __attribute__((address_space(1))) uint8_t* gcu8p;
typedef __attribute__((address_space(1))) uint8_t* gu8p;

__device__ __forceinline__ u32x4 load_full(const uint8_t* p, bool aligned) {
    if (aligned) return __builtin_nontemporal_load((gcu32x4p)(p));
    u32x4 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}

__device__ __forceinline__ void store_full(uint8_t* p, u32x4 v, bool aligned) {
    if (aligned)
        __builtin_nontemporal_store(v, (gu32x4p)(p));
    else
        __builtin_memcpy(p, &v, 16);
}

// Streamed access at (uniform shard base) + (lane offset): the base is moved
// to the global address space before the offset is added, so a 32-bit offset
// becomes the saddr form (SGPR base + VGPR offset) with no 64-bit VALU math.
template <typename OffT>
__device__ __forceinline__ u32x4 load_at(const uint8_t* base, OffT o) {
    return __builtin_nontemporal_load((gcu32x4p)((gcu8p)(base) + o));
}
template <typename OffT>
__device__ __forceinline__ void store_at(uint8_t* base, OffT o, u32x4 v) {
    __builtin_nontemporal_store(v, (gu32x4p)((gu8p)(base) + o));
}

__device__ __noinline__ u32x4 load_tail(const uint8_t* p, uint64_t avail) {
    uint8_t b[16];
    for (int i = 0; i < 16; ++i) b[i] = (uint64_t(i) < avail) ? p[i] : 0;
    u32x4 v;
    __builtin_memcpy(&v, b, 16);
    return v;
}

__device__ __noinline__ void store_tail(uint8_t* p, u32x4 v, uint64_t avail) {
    uint8_t b[16];
    __builtin_memcpy(b, &v, 16);
    for (int i = 0; i < 16; ++i)
        if (uint64_t(i) < avail) p[i] = b[i];
}

// acc[r] ^= coef(r) * d for R output rows; tab -> [rows][5] words of this input.
template <int R>
__device__ __forceinline__ void gf_mac(u32x4 (&acc)[R], const u32x4 d, cu32p tab) {
    uint32_t s0[4], s1[4], s2[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint32_t x = d[w];
        s0[w] = x & 0x07070707u;
        s1[w] = (x >> 3) & 0x07070707u;
        s2[w] = (x >> 6) & 0x03030303u;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t t0l = tab[r * 5 + 0], t0h = tab[r * 5 + 1];
        const uint32_t t1l = tab[r * 5 + 2], t1h = tab[r * 5 + 3];
        const uint32_t t2 = tab[r * 5 + 4];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const uint32_t a = __builtin_amdgcn_perm(t0h, t0l, s0[w]);
            const uint32_t b = __builtin_amdgcn_perm(t1h, t1l, s1[w]);
            const uint32_t c = __builtin_amdgcn_perm(t2, t2, s2[w]);
            acc[r][w] = __builtin_amdgcn_bitop3_b32(acc[r][w], a, b, 0x96) ^ c;
        }
    }
}

// Two inputs at once: the six lookups of a row are folded into the
// accumulator by three 3-input XORs (v_bitop3) instead of four ops.
// nrows (wave-uniform, <= R): rows at or past it skip their math (a decode
// with e < 4 erasures; scalar branches, the tables keep their 4-row stride).
template <int R, typename V = u32x4>
__device__ __forceinline__ void gf_mac2(V (&acc)[R], const V d0, const V d1, cu32p tab0, cu32p tab1,
                                        uint32_t nrows = R) {
    constexpr int W = int(sizeof(V) / 4);  // dwords per lane vector
    uint32_t s[2][3][W];
#pragma unroll
    for (int w = 0; w < W; ++w) {
        const uint32_t x0 = d0[w], x1 = d1[w];
        s[0][0][w] = x0 & 0x07070707u;
        s[0][1][w] = (x0 >> 3) & 0x07070707u;
        s[0][2][w] = (x0 >> 6) & 0x03030303u;
        s[1][0][w] = x1 & 0x07070707u;
        s[1][1][w] = (x1 >> 3) & 0x07070707u;
        s[1][2][w] = (x1 >> 6) & 0x03030303u;
    }
    // both inputs' table words for every row, requested before the row
    // branches (the empty asm keeps the loads from sinking into them, where
    // each row would wait on its own scalar round trip)
    uint32_t ta[R * 5], tbw[R * 5];
#pragma unroll
    for (int j = 0; j < R * 5; ++j) {
        ta[j] = tab0[j];
        tbw[j] = tab1[j];
    }
    if (R < 4 || nrows < uint32_t(R)) {
#pragma unroll
        for (int j = 0; j < R * 5; ++j) asm volatile("" ::"s"(ta[j]), "s"(tbw[j]));
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (r > 0 && uint32_t(r) >= nrows) break;
        const uint32_t a0l = ta[r * 5 + 0], a0h = ta[r * 5 + 1], a1l = ta[r * 5 + 2], a1h = ta[r * 5 + 3],
                       a2 = ta[r * 5 + 4];
        const uint32_t b0l = tbw[r * 5 + 0], b0h = tbw[r * 5 + 1], b1l = tbw[r * 5 + 2], b1h = tbw[r * 5 + 3],
                       b2 = tbw[r * 5 + 4];
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const uint32_t p0 = __builtin_amdgcn_perm(a0h, a0l, s[0][0][w]);
            const uint32_t p1 = __builtin_amdgcn_perm(a1h, a1l, s[0][1][w]);
            const uint32_t p2 = __builtin_amdgcn_perm(a2, a2, s[0][2][w]);
            const uint32_t q0 = __builtin_amdgcn_perm(b0h, b0l, s[1][0][w]);
            const uint32_t q1 = __builtin_amdgcn_perm(b1h, b1l, s[1][1][w]);
            const uint32_t q2 = __builtin_amdgcn_perm(b2, b2, s[1][2][w]);
            uint32_t x = __builtin_amdgcn_bitop3_b32(acc[r][w], p0, p1, 0x96);
            x = __builtin_amdgcn_bitop3_b32(x, p2, q0, 0x96);
            acc[r][w] = __builtin_amdgcn_bitop3_b32(x, q1, q2, 0x96);
        }
    }
}

// One group of R (<= 4) output rows of a plan, one 16-byte vector per lane.
// K > 0: compile-time input count (all K loads issued before any math);
// K == 0: runtime nin loop. Lanes whose vector crosses the end of the shard
// take the byte-wise tail path (only in the last chunk of a stripe).
template <int K, int R, bool ALIGNED>
__device__ __forceinline__ void apply_group(const ApplyArgs& a, const uint8_t* in_b, uint8_t* out_b,
                                            cu32p in_ids, cu32p out_ids, cu32p tab, uint32_t nin,
                                            uint32_t tab_row_stride, uint64_t chunk_off) {
    const uint64_t o = chunk_off + threadIdx.x * kVecBytes;
    if (o >= a.len) return;
    const uint64_t avail = a.len - o;
    u32x4 acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = u32x4{0, 0, 0, 0};
    if (avail >= kVecBytes) {
        if constexpr (K > 0) {
            u32x4 d[K];
#pragma unroll
            for (int i = 0; i < K; ++i) d[i] = load_full(in_b + uint64_t(in_ids[i]) * a.in_shard + o, ALIGNED);
#pragma unroll
            for (int i = 0; i < K; ++i) gf_mac<R>(acc, d[i], tab + i * tab_row_stride);
        } else {
            for (uint32_t i = 0; i < nin; ++i) {
                const u32x4 d = load_full(in_b + uint64_t(in_ids[i]) * a.in_shard + o, ALIGNED);
                gf_mac<R>(acc, d, tab + i * tab_row_stride);
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) store_full(out_b + uint64_t(out_ids[r]) * a.out_shard + o, acc[r], ALIGNED);
    } else {
        for (uint32_t i = 0; i < nin; ++i) {
            const u32x4 d = load_tail(in_b + uint64_t(in_ids[i]) * a.in_shard + o, avail);
            gf_mac<R>(acc, d, tab + i * tab_row_stride);
        }
        for (int r = 0; r < R; ++r) store_tail(out_b + uint64_t(out_ids[r]) * a.out_shard + o, acc[r], avail);
    }
}

// Completion signal of a launch for a host that spins on pinned memory
// (small host calls): every wave drains its stores, the
// workgroup meets at a barrier, lane 0 releases at system scope and counts
// itself in; the last workgroup resets the counter and stores the sequence
// number into the host flag. Every workgroup of the grid reaches this (the
// kernels call it after their body, early exits included).
__device__ __forceinline__ void signal_done(uint32_t* count, uint32_t* flag, uint32_t seq) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        const uint32_t blocks = gridDim.x * gridDim.y * gridDim.z;
        if (__hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == blocks - 1) {
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __threadfence_system();
            __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// Generic plan interpreter (any k + m <= 256, unaligned bases and strides,
// ad-hoc host plans): grid-stride over (stripe, 4 KiB chunk) items.
template <int K, bool ALIGNED>
__global__ __launch_bounds__(kThreads) void rs_apply_kernel(ApplyArgs a) {
    // XCD-aware chunk mapping: workgroups b, b+8, b+16, ... are dealt to one
    // XCD (MI355X_MICROARCH.md, dispatch), so a bijective remap hands them
    // consecutive chunks. Speed only: correctness never depends on placement.
    const uint32_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = blockIdx.x % 8;
    const uint64_t first = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + blockIdx.x / 8;
    for (uint64_t item = first; item < a.n_items; item += gridDim.x) {
        const uint32_t stripe = uint32_t(item / a.chunks_per_stripe);
        const uint32_t chunk = uint32_t(item - uint64_t(stripe) * a.chunks_per_stripe);
        uint32_t pid = 0;
        if (a.masks) {
            pid = as_const(a.lut)[as_const(a.masks)[stripe] & a.mask_limit];
            if (pid == kNoPlan) {
                if (chunk == 0 && threadIdx.x == 0 && a.bad_count) atomicAdd(a.bad_count, 1u);
                continue;
            }
        }
        const __attribute__((address_space(4))) DevPlan* pp = as_const(a.plans) + pid;
        const DevPlan p{pp->nin, pp->nout, pp->tab_off, pp->idx_off, pp->tab_rows, {0, 0, 0}};
        if (p.nout == 0) continue;
        const uint8_t* in_b = a.in_base + uint64_t(stripe) * a.in_stripe;
        uint8_t* out_b = a.out_base + uint64_t(stripe) * a.out_stripe;
        cu32p in_ids = as_const(a.idx) + p.idx_off;
        cu32p out_ids = in_ids + p.nin;
        cu32p tab = as_const(a.tabs) + p.tab_off;
        const uint32_t row_stride = p.tab_rows * 5;  // words per input
        const uint64_t chunk_off = uint64_t(chunk) * (kThreads * kVecBytes);
        for (uint32_t g = 0; g < p.nout; g += 4) {
            const uint32_t R = p.nout - g < 4 ? p.nout - g : 4;
            cu32p tg = tab + g * 5;
            switch (R) {
                case 4: apply_group<K, 4, ALIGNED>(a, in_b, out_b, in_ids, out_ids + g, tg, p.nin, row_stride, chunk_off); break;
                case 3: apply_group<K, 3, ALIGNED>(a, in_b, out_b, in_ids, out_ids + g, tg, p.nin, row_stride, chunk_off); break;
                case 2: apply_group<K, 2, ALIGNED>(a, in_b, out_b, in_ids, out_ids + g, tg, p.nin, row_stride, chunk_off); break;
                default: apply_group<K, 1, ALIGNED>(a, in_b, out_b, in_ids, out_ids + g, tg, p.nin, row_stride, chunk_off); break;
            }
        }
    }
    if (a.done_flag) signal_done(a.done_count, a.done_flag, a.done_seq);
}

// ---------------------------------------------------------------------------
// RS(10,4) fast paths (k = 10, n = 14, 16-byte aligned strides): the shard ids
// come from kernel arguments (encode) or straight from the stripe's present
// mask with scalar bit scans (decode), so a workgroup issues its ten loads
// after at most ONE scalar load; the coefficient tables (fixed stride of 4
// rows x 5 words per input) arrive in parallel with the data.
// ---------------------------------------------------------------------------
// Workgroup -> (stripe, chunk). Workgroups b, b+8, b+16, ... are dealt to one
// XCD (observed round-robin dispatch; MI355X_MICROARCH.md), so XCD x = b % 8
// takes the contiguous x-th eighth of all chunks (+5-9% over dispatch order):
// item = x*q + min(x, r) + b/8 from the launcher's constants (map_q8 / map_r8),
// then the chunks per stripe as a multiply-shift divisor (FastDiv): a handful
// of scalar ops from blockIdx, no division, so a workgroup reaches its
// stripe's mask load (decode) or its first data load (encode) a few cycles
// after launch. A bijection: speed only, never correctness.
__device__ __forceinline__ void fast_item(const ApplyArgs& a, uint32_t per_stripe, uint32_t& stripe,
                                          uint32_t& chunk) {
    // Every kernel argument the workgroup will need, in SGPRs at entry: one
    // round trip, instead of loads the compiler sinks behind the decode's
    // mask checks (each a further trip).
    asm volatile("" ::"s"(a.in_base), "s"(a.in_stripe), "s"(a.in_shard), "s"(a.out_base), "s"(a.out_stripe),
                 "s"(a.out_shard), "s"(a.len), "s"(a.masks), "s"(a.lut), "s"(a.tabs), "s"(a.map_q8),
                 "s"(a.map_r8), "s"(a.cps_mul), "s"(a.cps_shift), "s"(a.chunks_per_stripe));
    const uint32_t b = blockIdx.x, x = b & 7u, q = a.map_q8, r = a.map_r8;
    const uint32_t item = x * q + (x < r ? x : r) + (b >> 3);
    stripe = fastdiv(item, a.cps_mul, a.cps_shift);
    chunk = item - stripe * per_stripe;
}

// One 4 KiB chunk of one RS(10,4) stripe. Encode (DEC=false): inputs 0..9 at
// in_b, outputs 0..3 at out_b. Decode (DEC=true): in place at in_b == out_b
// (or COMPACT: inputs are slots 0..9 at in_b, outputs slots 0..e-1 at out_b),
// shard ids from the present mask, tables at lut[mask] * 200 words.
// OffT: type of the lane's byte offset in the shard. uint32_t (every ragged
// stripe, and strided batches of shards below 4 GiB) lets each load address
// be a scalar shard base plus a 32-bit lane offset (global_load saddr form:
// no per-load 64-bit VALU address math).
template <bool DEC, bool COMPACT = false, typename OffT = uint64_t>
__device__ __forceinline__ void rs104_chunk(const uint8_t* in_b, uint8_t* out_b, uint64_t in_shard,
                                            uint64_t out_shard, uint64_t len, uint32_t chunk, uint32_t mask_in,
                                            cu32p tab, cu32p lut, uint32_t* bad_count) {
    constexpr int K = 10, N = 14, R = 4;
    uint32_t in_id[K], out_id[R];
    uint32_t nout = R;
    uint32_t mask = 0, plan = 0;
    if constexpr (DEC) {
        mask = mask_in & ((1u << N) - 1);
        const uint32_t present = __builtin_popcount(mask);
        if (present < K) {
            if (chunk == 0 && threadIdx.x == 0 && bad_count) atomicAdd(bad_count, 1u);
            return;
        }
        if (present == N) return;  // upstream: all present -> no-op
        nout = N - present;
        uint32_t m = mask;
#pragma unroll
        for (int i = 0; i < K; ++i) {  // first K present shards, ascending
            in_id[i] = COMPACT ? i : __builtin_ctz(m);
            m &= m - 1;
        }
        uint32_t e = ~mask & ((1u << N) - 1);
#pragma unroll
        for (int r = 0; r < R; ++r) {  // erased shards, ascending
            out_id[r] = COMPACT ? r : (e ? __builtin_ctz(e) : 0);
            e &= e - 1;
        }
        // plan lookup issued now; its value is first needed after the data
        // loads, so the scalar round trip overlaps them
        plan = lut[mask];
    } else {
#pragma unroll
        for (int i = 0; i < K; ++i) in_id[i] = i;
#pragma unroll
        for (int r = 0; r < R; ++r) out_id[r] = r;
    }
    const OffT o = OffT(chunk) * OffT(kThreads * kVecBytes) + OffT(threadIdx.x * kVecBytes);
    if (o >= len) return;
    const uint64_t avail = len - o;
    u32x4 acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = u32x4{0, 0, 0, 0};
    if (avail >= kVecBytes) {
        u32x4 d[K];
#pragma unroll
        for (int i = 0; i < K; ++i) d[i] = load_at(in_b + uint64_t(in_id[i]) * in_shard, o);
        // all ten loads in flight before any math: without this fence the
        // scheduler interleaves them with the table multiply two at a time
        // (36 VGPRs, but one wave then waits on HBM five times per chunk;
        // -5% decode time with it, profiles/r02/ab_loads_first.txt)
        __builtin_amdgcn_sched_barrier(0);
        // opaque here: the table address math (and so the wait for the plan
        // lookup) cannot be hoisted above the data loads
        if constexpr (DEC) {
            asm volatile("" : "+s"(plan));
            tab += plan * (K * R * 5);
        }
#pragma unroll
        for (int i = 0; i < K; i += 2)
            gf_mac2<R>(acc, d[i], d[i + 1], tab + i * (R * 5), tab + (i + 1) * (R * 5), nout);
        // Materialise every row before the uniform `r < nout` store branches:
        // otherwise the compiler sinks each row's math into its branch, keeps
        // all 200 table words live and spills SGPRs (154 VGPRs, 3 waves/SIMD).
#pragma unroll
        for (int r = 0; r < R; ++r) asm volatile("" ::"v"(acc[r]));
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (r < int(nout)) store_at(out_b + uint64_t(out_id[r]) * out_shard, o, acc[r]);
    } else {
        if constexpr (DEC) {
            asm volatile("" : "+s"(plan));
            tab += plan * (K * R * 5);
        }
        for (int i = 0; i < K; ++i) {
            const u32x4 d = load_tail(in_b + uint64_t(in_id[i]) * in_shard + o, avail);
            gf_mac<R>(acc, d, tab + i * (R * 5));
        }
        for (int r = 0; r < R; ++r)
            if (r < int(nout)) store_tail(out_b + uint64_t(out_id[r]) * out_shard + o, acc[r], avail);
    }
}

// 16 bytes per lane, one 4 KiB column range per workgroup: the aligned
// RS(10,4) encodes the bit-sliced kernel does not take and the decodes of
// shard lengths that are not a multiple of 2 KiB. OffT = uint64_t for shards
// of 4 GiB and more.
template <bool DEC, typename OffT>
__global__ __launch_bounds__(kThreads) void rs104_kernel(ApplyArgs a) {
    uint32_t stripe, chunk;
    fast_item(a, a.chunks_per_stripe, stripe, chunk);
    const uint32_t mask = DEC ? as_const(a.masks)[stripe] : 0u;
    rs104_chunk<DEC, false, OffT>(a.in_base + uint64_t(stripe) * a.in_stripe,
                                  a.out_base + uint64_t(stripe) * a.out_stripe, a.in_shard, a.out_shard, a.len,
                                  chunk, mask, as_const(a.tabs), as_const(a.lut), a.bad_count);
    if (a.done_flag) signal_done(a.done_count, a.done_flag, a.done_seq);
}

// RS(10,4) with 8 bytes per lane (2 KiB column range per workgroup, dwordx2
// streams): less math per wave between its loads and its stores, 54 VGPRs
// (8 waves/SIMD) instead of 100. The decode of shard lengths that are a
// multiple of 2 KiB (0.9-1.7% faster than 16 B, profiles/r02/
// ab_decode_bytes_per_lane.jsonl), and the zero-copy host encode over PCIe
// (DEC=false: inputs 0..9, outputs 0..3; profiles/r04/e2e_encode_kernels_*).
// Shards below 4 GiB (32-bit lane offsets).
template <bool DEC>
__device__ __forceinline__ void rs104_narrow_chunk(const uint8_t* in_b, uint8_t* out_b, uint64_t in_shard,
                                                   uint64_t out_shard, uint32_t chunk, uint32_t mask_in, cu32p tabs,
                                                   cu32p lut, uint32_t* bad_count) {
    typedef u32x2 V;
    constexpr int K = 10, N = 14, R = 4, VB = int(sizeof(V));
    uint32_t in_id[K], out_id[R];
    uint32_t nout = R, plan = 0;
    bool work = true;
    if constexpr (DEC) {
        const uint32_t mask = mask_in & ((1u << N) - 1);
        const uint32_t present = __builtin_popcount(mask);
        if (present < K && chunk == 0 && threadIdx.x == 0 && bad_count) atomicAdd(bad_count, 1u);
        work = present >= K && present < N;  // too few: skipped + counted; all present: upstream no-op
        nout = N - present;
        uint32_t m = mask;
#pragma unroll
        for (int i = 0; i < K; ++i) {  // first K present shards, ascending
            in_id[i] = m ? __builtin_ctz(m) : 0;
            m &= m - 1;
        }
        uint32_t e = ~mask & ((1u << N) - 1);
#pragma unroll
        for (int r = 0; r < R; ++r) {  // erased shards, ascending
            out_id[r] = e ? __builtin_ctz(e) : 0;
            e &= e - 1;
        }
        if (work) plan = lut[mask];  // first used after the data loads
    } else {
#pragma unroll
        for (int i = 0; i < K; ++i) in_id[i] = i;
#pragma unroll
        for (int r = 0; r < R; ++r) out_id[r] = r;
    }
    if (work) {
        const uint32_t o = chunk * (kThreads * VB) + threadIdx.x * VB;
        V d[K];
#pragma unroll
        for (int i = 0; i < K; ++i)
            d[i] = __builtin_nontemporal_load(
                (const __attribute__((address_space(1))) V*)((gcu8p)(in_b + uint64_t(in_id[i]) * in_shard) + o));
        __builtin_amdgcn_sched_barrier(0);  // all ten loads in flight before the math
        asm volatile("" : "+s"(plan));
        cu32p tab = tabs + plan * (K * R * 5);
        V acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = V(0u);
#pragma unroll
        for (int i = 0; i < K; i += 2)
            gf_mac2<R, V>(acc, d[i], d[i + 1], tab + i * (R * 5), tab + (i + 1) * (R * 5), nout);
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int w = 0; w < VB / 4; ++w) asm volatile("" ::"v"(acc[r][w]));
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (r < int(nout))
                __builtin_nontemporal_store(
                    acc[r], (__attribute__((address_space(1))) V*)((gu8p)(out_b + uint64_t(out_id[r]) * out_shard) + o));
    }
}

template <bool DEC>
__global__ __launch_bounds__(kThreads) void rs104_narrow_kernel(ApplyArgs a) {
    uint32_t stripe, chunk;
    fast_item(a, a.chunks_per_stripe, stripe, chunk);
    const uint32_t mask = DEC ? as_const(a.masks)[stripe] : 0u;
    rs104_narrow_chunk<DEC>(a.in_base + uint64_t(stripe) * a.in_stripe, a.out_base + uint64_t(stripe) * a.out_stripe,
                            a.in_shard, a.out_shard, chunk, mask, as_const(a.tabs), as_const(a.lut), a.bad_count);
    if (a.done_flag) signal_done(a.done_count, a.done_flag, a.done_seq);
}

// ---------------------------------------------------------------------------
// Bit-sliced RS(10,4) encode (fixed parity matrix). A lane owns 32 bytes of
// every shard (two 16-byte vectors 4 KiB apart, so each load instruction stays
// one contiguous 1 KiB per wave). Its 8 dwords per shard are transposed into 8
// bit planes (plane k = bit k of the 32 bytes), the 80 data planes go through
// the generated XOR program (tools/gen_bitslice.py: 328 three-input XORs for
// all 32 parity planes), and the parity planes are transposed back. Per data
// dword that is ~12.5 VALU ops against ~27 for the table-lookup multiply, so
// the math hides at lower occupancy (170 VGPRs, 2 waves/SIMD).
// ---------------------------------------------------------------------------
// One 8 KiB column range (`chunk`) of one stripe: inputs 0..9 at in_b, parity
// 0..3 at out_b.
template <typename OffT = uint64_t>
__device__ __forceinline__ void rs104_bs_chunk(const uint8_t* in_b, uint8_t* out_b, uint64_t in_shard,
                                               uint64_t out_shard, uint32_t chunk) {
    constexpr int K = 10, R = 4;
    const OffT base = OffT(chunk) * OffT(kBsChunk) + OffT(threadIdx.x * 16);
    uint32_t p[K * 8];
    u32x4 d[K][2];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        d[i][0] = load_at(in_b + uint64_t(i) * in_shard, base);
        d[i][1] = load_at(in_b + uint64_t(i) * in_shard, base + OffT(kThreads * 16));
    }
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            p[8 * i + w] = d[i][0][w];
            p[8 * i + 4 + w] = d[i][1][w];
        }
#pragma unroll
    for (int i = 0; i < K; ++i) transpose8(p + 8 * i);
    uint32_t q[R * 8];
    rs104_encode_planes(p, q);
#pragma unroll
    for (int j = 0; j < R; ++j) {
        transpose8(q + 8 * j);
        store_at(out_b + uint64_t(j) * out_shard, base, u32x4{q[8 * j], q[8 * j + 1], q[8 * j + 2], q[8 * j + 3]});
        store_at(out_b + uint64_t(j) * out_shard, base + OffT(kThreads * 16),
                 u32x4{q[8 * j + 4], q[8 * j + 5], q[8 * j + 6], q[8 * j + 7]});
    }
}

template <typename OffT>
__global__ __launch_bounds__(kThreads) void rs104_bs_encode_kernel(ApplyArgs a) {
    uint32_t stripe, chunk;
    fast_item(a, a.chunks_per_stripe, stripe, chunk);
    rs104_bs_chunk<OffT>(a.in_base + uint64_t(stripe) * a.in_stripe, a.out_base + uint64_t(stripe) * a.out_stripe,
                         a.in_shard, a.out_shard, chunk);
    if (a.done_flag) signal_done(a.done_count, a.done_flag, a.done_seq);
}

// Map entry of this workgroup: XCD x = blockIdx % 8 takes the x-th eighth of
// the launch's entries, so the workgroups sharing an XCD (and its L2) stream
// consecutive chunks, as in the strided kernels. The ragged decode +2% on the
// bench batch (with the no-op skip +10% on the mixed workload,
// profiles/r02/ab_ragged_remap_skip.jsonl); the bit-sliced ragged encode +2%
// at 512 mixed stripes, +7% at 4096 and +9% on uniform 4 MiB stripes
// (profiles/r03/sweep_mixed2.jsonl).
__device__ __forceinline__ uint32_t ragged_block(const RaggedArgs& a) {
    const uint32_t b = blockIdx.x, x = b & 7u;
    return x * a.map_q8 + (x < a.map_r8 ? x : a.map_r8) + (b >> 3) + a.block_base;
}

// Descriptor of the stripe workgroup blk works on: the kernel-argument copy
// for a one-stripe launch, else the workgroup map and item table (scalar loads).
__device__ __forceinline__ RaggedItem ragged_item(const RaggedArgs& a, uint32_t blk) {
    if (a.inline_one) return a.one;
    const __attribute__((address_space(4))) RaggedItem* p = as_const(a.items) + as_const(a.block_item)[blk];
    return RaggedItem{p->off, p->shard_stride, p->len, p->mask, p->first_block, 0, p->out_off};
}

// Ragged encode with every stripe length a multiple of 8 KiB: workgroup ->
// stripe map as rs104_ragged_kernel, one 8 KiB column range per workgroup.
__global__ __launch_bounds__(kThreads) void rs104_bs_ragged_kernel(RaggedArgs a) {
    const uint32_t blk = ragged_block(a);
    const RaggedItem it = ragged_item(a, blk);
    const uint64_t off = it.off, stride = it.shard_stride;
    const uint32_t first = it.first_block;
    const uint8_t* b = a.base + off;
    rs104_bs_chunk<uint32_t>(b, a.base + off + 10 * stride, stride, stride, blk - first);
    if (a.done_flag) signal_done(a.done_count, a.done_flag, a.done_seq);
}

hipError_t launch_rs104_bs_ragged(const RaggedArgs& a, hipStream_t stream) {
    for (uint64_t b0 = 0; b0 < a.n_blocks; b0 += kMaxLaunchBlocks) {  // see kMaxLaunchBlocks
        RaggedArgs r = a;
        r.block_base = uint32_t(b0);
        if (b0 + kMaxLaunchBlocks < a.n_blocks) r.done_flag = nullptr;  // the last launch signals
        const uint32_t nb = uint32_t(std::min<uint64_t>(kMaxLaunchBlocks, a.n_blocks - b0));
        r.map_q8 = nb / 8;
        r.map_r8 = nb % 8;
        hipLaunchKernelGGL(rs104_bs_ragged_kernel, dim3(nb), dim3(kThreads), 0, stream, r);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// Ragged batches: every stripe has its own length, shard stride and mask
// (degraded reads of needle intervals, mixed 64 KiB-4 MiB stripes). The host
// lays stripes out back to back and passes a workgroup -> stripe map.
template <bool DEC, bool COMPACT>
__global__ __launch_bounds__(kThreads) void rs104_ragged_kernel(RaggedArgs a) {
    const uint32_t blk = ragged_block(a);
    // one stripe (a per-call host reconstruct): its descriptor is a kernel
    // argument, so the launch needs no metadata upload and no dependent loads
    const RaggedItem it = ragged_item(a, blk);
    uint8_t* b = a.base + it.off;
    uint8_t* o = COMPACT ? a.base + it.out_off : (DEC ? b : b + 10 * it.shard_stride);
    rs104_chunk<DEC, COMPACT, uint32_t>(b, o, it.shard_stride, it.shard_stride, it.len, blk - it.first_block, it.mask,
                                        as_const(a.tabs), as_const(a.lut), a.bad_count);
    if (a.done_flag) signal_done(a.done_count, a.done_flag, a.done_seq);
}

hipError_t launch_rs104_ragged(const RaggedArgs& a, bool decode, hipStream_t stream) {
    for (uint64_t b0 = 0; b0 < a.n_blocks; b0 += kMaxLaunchBlocks) {  // see kMaxLaunchBlocks
        RaggedArgs r = a;
        r.block_base = uint32_t(b0);
        if (b0 + kMaxLaunchBlocks < a.n_blocks) r.done_flag = nullptr;  // the last launch signals
        const dim3 grid(uint32_t(std::min<uint64_t>(kMaxLaunchBlocks, a.n_blocks - b0)));
        r.map_q8 = grid.x / 8;
        r.map_r8 = grid.x % 8;
        if (decode && a.compact)
            hipLaunchKernelGGL((rs104_ragged_kernel<true, true>), grid, dim3(kThreads), 0, stream, r);
        else if (decode)
            hipLaunchKernelGGL((rs104_ragged_kernel<true, false>), grid, dim3(kThreads), 0, stream, r);
        else
            hipLaunchKernelGGL((rs104_ragged_kernel<false, false>), grid, dim3(kThreads), 0, stream, r);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// The kernel an aligned RS(10,4) batch with the fast plan layout runs, shared
// by launch_apply and the name functions so a reported name is the kernel
// that runs.
enum class Rs104Kind { Apply, Bitslice, Narrow, Table };
static Rs104Kind rs104_pick(uint64_t len, uint64_t n_stripes, bool dec, bool over_pcie) {
    // launch_apply sizes its stripe ranges for 4 KiB chunks; a batch whose
    // chunks would pass one launch's workgroup limit takes the generic kernel
    const uint64_t items = (len + 4095) / 4096 * n_stripes;
    if (items > kMaxLaunchBlocks) return Rs104Kind::Apply;
    const bool off32 = len <= 0xFFFFFFFFull;
    if (!dec && !over_pcie && len % kBsChunk == 0) return Rs104Kind::Bitslice;
    // the decode, and the encode over PCIe: 8 bytes per lane where the shard
    // length is a multiple of 2 KiB
    if ((dec || over_pcie) && off32 && len % kNarrowChunk == 0 && (len / kNarrowChunk) * n_stripes <= kMaxLaunchBlocks)
        return Rs104Kind::Narrow;
    return Rs104Kind::Table;
}

static const char* rs104_name(Rs104Kind k, bool dec) {
    switch (k) {
        case Rs104Kind::Apply: return "rs_apply_kernel<10> (table lookup)";
        case Rs104Kind::Bitslice: return "rs104_bs_encode_kernel (bit-sliced)";
        case Rs104Kind::Narrow:
            return dec ? "rs104_narrow_kernel<DEC=true, 8 B per lane> (table lookup)"
                       : "rs104_narrow_kernel<DEC=false, 8 B per lane> (table lookup)";
        default: return dec ? "rs104_kernel<DEC=true> (table lookup)" : "rs104_kernel<DEC=false> (table lookup)";
    }
}

constexpr const char* kNoLaunch = "none (empty shards: EmptyShard, no launch)";

const char* decode_kernel_name(uint64_t len) {
    if (len == 0) return kNoLaunch;
    return rs104_name(rs104_pick(len, 1, true, false), true);
}

const char* encode_kernel_name(uint64_t len, bool over_pcie) {
    if (len == 0) return kNoLaunch;
    return rs104_name(rs104_pick(len, 1, false, over_pcie), false);
}

// Launch constants of fast_item: the XCD eighths of the grid and the chunks
// per stripe as a multiply-shift divisor.
static void set_fast_map(ApplyArgs& a, uint32_t chunk_bytes, bool round_up) {
    a.chunks_per_stripe = uint32_t(round_up ? (a.len + chunk_bytes - 1) / chunk_bytes : a.len / chunk_bytes);
    a.n_items = uint64_t(a.chunks_per_stripe) * a.n_stripes;
    a.map_q8 = uint32_t(a.n_items / 8);
    a.map_r8 = uint32_t(a.n_items % 8);
    const FastDiv f = make_fastdiv(a.chunks_per_stripe ? a.chunks_per_stripe : 1);
    a.cps_mul = f.mul;
    a.cps_shift = f.shift;
}

template <bool DEC>
static hipError_t launch_rs104(ApplyArgs a, Rs104Kind kind, hipStream_t stream) {
    const bool off32 = a.len <= 0xFFFFFFFFull;
    switch (kind) {
        case Rs104Kind::Bitslice:
            set_fast_map(a, kBsChunk, false);
            if (a.n_items == 0) return hipSuccess;
            if (off32)
                hipLaunchKernelGGL((rs104_bs_encode_kernel<uint32_t>), dim3(uint32_t(a.n_items)), dim3(kThreads), 0,
                                   stream, a);
            else
                hipLaunchKernelGGL((rs104_bs_encode_kernel<uint64_t>), dim3(uint32_t(a.n_items)), dim3(kThreads), 0,
                                   stream, a);
            break;
        case Rs104Kind::Narrow:
            set_fast_map(a, kNarrowChunk, false);
            if (a.n_items == 0) return hipSuccess;
            hipLaunchKernelGGL((rs104_narrow_kernel<DEC>), dim3(uint32_t(a.n_items)), dim3(kThreads), 0, stream, a);
            break;
        default:
            set_fast_map(a, kThreads * kVecBytes, true);
            if (a.n_items == 0) return hipSuccess;
            if (off32)
                hipLaunchKernelGGL((rs104_kernel<DEC, uint32_t>), dim3(uint32_t(a.n_items)), dim3(kThreads), 0,
                                   stream, a);
            else
                hipLaunchKernelGGL((rs104_kernel<DEC, uint64_t>), dim3(uint32_t(a.n_items)), dim3(kThreads), 0,
                                   stream, a);
            break;
    }
    return hipGetLastError();
}

template <int K, bool ALIGNED>
static hipError_t launch_t(ApplyArgs a, hipStream_t stream) {
    const uint64_t chunk = uint64_t(kThreads) * kVecBytes;
    a.chunks_per_stripe = uint32_t((a.len + chunk - 1) / chunk);
    a.n_items = uint64_t(a.chunks_per_stripe) * a.n_stripes;
    if (a.n_items == 0) return hipSuccess;
    const uint64_t grid = std::min<uint64_t>(a.n_items, kMaxLaunchBlocks);  // grid-stride covers the rest
    hipLaunchKernelGGL((rs_apply_kernel<K, ALIGNED>), dim3(uint32_t(grid)), dim3(kThreads), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_apply(const ApplyArgs& a, int nin, bool aligned, bool over_pcie, hipStream_t stream) {
    // RS(10,4) fast path: fixed 4-row table stride, one chunk of >= 2 KiB per
    // workgroup and no grid-stride loop, so one launch takes at most
    // kMaxLaunchBlocks chunks: larger batches (tens of millions of short
    // stripes) go in stripe ranges.
    const uint64_t per_stripe = (a.len + 4095) / 4096;
    const uint64_t items = per_stripe * a.n_stripes;
    if (a.fast104 && items > kMaxLaunchBlocks && a.n_stripes > 1 && per_stripe <= kMaxLaunchBlocks) {
        const uint32_t step = uint32_t(kMaxLaunchBlocks / per_stripe);
        for (uint32_t s0 = 0; s0 < a.n_stripes; s0 += step) {
            ApplyArgs b = a;
            b.n_stripes = std::min(step, a.n_stripes - s0);
            if (s0 + step < a.n_stripes) b.done_flag = nullptr;  // same stream: the last launch signals
            b.in_base += uint64_t(s0) * a.in_stripe;
            b.out_base += uint64_t(s0) * a.out_stripe;
            if (b.masks) b.masks += s0;
            hipError_t e = launch_apply(b, nin, aligned, over_pcie, stream);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    const Rs104Kind kind = rs104_pick(a.len, a.n_stripes, a.masks != nullptr, over_pcie && !a.masks);
    if (a.fast104 && aligned && kind != Rs104Kind::Apply)
        return a.masks ? launch_rs104<true>(a, kind, stream) : launch_rs104<false>(a, kind, stream);
    if (nin == 10) return aligned ? launch_t<10, true>(a, stream) : launch_t<10, false>(a, stream);
    return aligned ? launch_t<0, true>(a, stream) : launch_t<0, false>(a, stream);
}

// ---------------------------------------------------------------------------
// splitmix64 synthetic stripes (deterministic bench / test inputs)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void fill_splitmix_kernel(uint8_t* base, uint64_t stripe_stride,
                                                                  uint64_t bytes_per_stripe,
                                                                  uint32_t n_stripes, uint64_t seed_base) {
    const uint64_t words = (bytes_per_stripe + 7) / 8;
    const uint64_t total = words * n_stripes;
    for (uint64_t t = uint64_t(blockIdx.x) * kThreads + threadIdx.x; t < total;
         t += uint64_t(gridDim.x) * kThreads) {
        const uint64_t s = t / words;
        const uint64_t w = t - s * words;
        uint64_t z = seed_base + s + (w + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        uint8_t* p = base + s * stripe_stride + w * 8;
        const uint64_t left = bytes_per_stripe - w * 8;
        if (left >= 8 && (reinterpret_cast<uintptr_t>(p) & 7) == 0) {
            *reinterpret_cast<uint64_t*>(p) = z;
        } else {
            for (uint64_t b = 0; b < 8 && b < left; ++b) p[b] = uint8_t(z >> (8 * b));
        }
    }
}

hipError_t launch_fill_splitmix(uint8_t* base, uint64_t stripe_stride, uint64_t bytes_per_stripe,
                                uint32_t n_stripes, uint64_t seed_base, hipStream_t stream) {
    const uint64_t total = ((bytes_per_stripe + 7) / 8) * n_stripes;
    if (total == 0) return hipSuccess;
    uint64_t grid = (total + kThreads - 1) / kThreads;
    if (grid > 65536) grid = 65536;
    hipLaunchKernelGGL(fill_splitmix_kernel, dim3(uint32_t(grid)), dim3(kThreads), 0, stream, base,
                       stripe_stride, bytes_per_stripe, n_stripes, seed_base);
    return hipGetLastError();
}

}  // namespace hec

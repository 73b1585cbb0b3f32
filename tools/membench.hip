// HBM ceiling microbenchmark for the RS(10,4) access pattern on MI355X.
//
// Measures, on the same 56 GiB region the bench uses ([4096][14][1 MiB]):
//   copy      : 1 read stream -> 1 write stream (float4), the guide's ceiling
//   read      : read-only (xor-reduce, one store per thread)
//   write     : write-only
//   nRmW      : n input streams -> m output streams at shard stride `stride`
//               (10R4W == the encode pattern with the math removed)
// One workgroup (256 lanes x 16 B) per 4 KiB chunk unless noted.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/membench tools/membench.hip
// Run:   build/membench [pad|mix|calib]  (prints one JSON line per case)
// calib: make build/membench_calib (links libhec; see calib() below)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <string>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e = (x);                                                               \
        if (e != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

__global__ __launch_bounds__(256) void k_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t n) {
    uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    if (i < n) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ src, u32x4* __restrict__ sink, uint64_t n) {
    uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    u32x4 v = __builtin_nontemporal_load(src + i);
    if (v.x == 0x12345678u && v.y == 0x9abcdef0u) sink[threadIdx.x] = v;  // practically never
}

__global__ __launch_bounds__(256) void k_write(u32x4* __restrict__ dst, uint64_t n) {
    uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    if (i < n) __builtin_nontemporal_store(u32x4{uint32_t(i), 1, 2, 3}, dst + i);
}

// n inputs (shards 0..n-1) -> m outputs (shards n..n+m-1) per stripe; chunk = 4 KiB
template <int N, int M>
__global__ __launch_bounds__(256) void k_nrmw(uint8_t* base, uint64_t stripe_stride, uint64_t shard_stride,
                                             uint32_t chunks_per_stripe, int xcd_remap) {
    uint32_t b = blockIdx.x;
    if (xcd_remap) {  // consecutive chunks on one XCD (blocks b, b+8, ... share an XCD)
        const uint32_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = b % 8;
        b = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
    }
    const uint32_t stripe = b / chunks_per_stripe, chunk = b % chunks_per_stripe;
    const uint64_t o = uint64_t(chunk) * 4096 + threadIdx.x * 16;
    uint8_t* s = base + uint64_t(stripe) * stripe_stride;
    u32x4 acc = {0, 0, 0, 0};
    u32x4 d[N > 0 ? N : 1];
#pragma unroll
    for (int i = 0; i < N; ++i) d[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(s + i * shard_stride + o));
#pragma unroll
    for (int i = 0; i < N; ++i) acc ^= d[i];
#pragma unroll
    for (int j = 0; j < M; ++j) {
        u32x4 v = acc;
        v.x ^= j;
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(s + (N + j) * shard_stride + o));
    }
    if (M == 0 && acc.x == 0x12345678u && acc.y == 0x9abcdef0u) *reinterpret_cast<u32x4*>(s) = acc;
}

// 10 reads -> 4 writes; each lane handles V vectors 4 KiB apart, so one
// workgroup covers V*4 KiB contiguous per shard. Dynamic LDS limits blocks/CU.
template <int V>
__global__ __launch_bounds__(256) void k_10r4w_v(uint8_t* base, uint64_t stripe_stride, uint64_t shard_stride,
                                                uint32_t chunks_per_stripe, int xcd_remap) {
    extern __shared__ uint32_t lds_pad[];
    uint32_t b = blockIdx.x;
    if (xcd_remap) {
        const uint32_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = b % 8;
        b = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
    }
    const uint32_t stripe = b / chunks_per_stripe, chunk = b % chunks_per_stripe;
    uint8_t* s = base + uint64_t(stripe) * stripe_stride;
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const uint64_t o = (uint64_t(chunk) * V + v) * 4096 + threadIdx.x * 16;
        u32x4 d[10];
#pragma unroll
        for (int i = 0; i < 10; ++i) d[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(s + i * shard_stride + o));
        u32x4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < 10; ++i) acc ^= d[i];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            u32x4 w = acc;
            w.x ^= j;
            __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(s + (10 + j) * shard_stride + o));
        }
    }
    if (threadIdx.x == 999) lds_pad[0] = 1;
}

// 10 reads -> 4 writes through buffer instructions with explicit cache-policy
// bits (gfx950 CPol: bit0 sc0, bit1 nt, bit4 sc1); eighths XCD remap.
__global__ __launch_bounds__(256) void k_10r4w_pol(uint8_t* base, uint64_t stripe_stride, uint32_t shard_stride,
                                                  uint32_t chunks_per_stripe, int lpol, int spol) {
    const uint32_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = blockIdx.x % 8;
    const uint32_t b = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + blockIdx.x / 8;
    const uint32_t stripe = b / chunks_per_stripe, chunk = b % chunks_per_stripe;
    uint8_t* s = base + uint64_t(stripe) * stripe_stride;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(s, 0, 14 * shard_stride, 0x00020000);
    const uint32_t o = chunk * 4096 + threadIdx.x * 16;
    u32x4 d[10];
#define LD(i, P) d[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (i) * shard_stride + o, 0, P))
#define LOADS(P) { LD(0,P); LD(1,P); LD(2,P); LD(3,P); LD(4,P); LD(5,P); LD(6,P); LD(7,P); LD(8,P); LD(9,P); }
    switch (lpol) { case 0: LOADS(0); break; case 1: LOADS(1); break; case 2: LOADS(2); break; case 16: LOADS(16); break; default: LOADS(3); }
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 10; ++i) acc ^= d[i];
#define ST(j, P) { u32x4 w = acc; w.x ^= j; __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, w), rs, (10 + j) * shard_stride + o, 0, P); }
#define STORES(P) { ST(0,P); ST(1,P); ST(2,P); ST(3,P); }
    switch (spol) {
        case 0: STORES(0); break; case 1: STORES(1); break; case 2: STORES(2); break; case 3: STORES(3); break;
        case 16: STORES(16); break; case 17: STORES(17); break; case 18: STORES(18); break; default: STORES(19);
    }
}

// FETCH_SIZE / WRITE_SIZE calibration: the decode's own
// access pattern with the math removed, over a KNOWN byte count. VB bytes per
// lane (8 = global_load_dwordx2 like rs104_narrow_kernel, 16 = dwordx4), one
// workgroup per 256 * VB byte column range of one stripe, XCD eighths remap,
// reads shards 0..9 non-temporal, then either writes shards 10..13 (W = 4,
// the decode's 4-erasure pattern) or nothing (W = 0: read-only).
template <int VB>
struct VecOf;
template <>
struct VecOf<8> {
    typedef uint32_t T __attribute__((ext_vector_type(2)));
};
template <>
struct VecOf<16> {
    typedef uint32_t T __attribute__((ext_vector_type(4)));
};
template <int VB, int W>
__global__ __launch_bounds__(256) void k_cal(uint8_t* base, uint64_t stripe_stride, uint64_t shard_stride,
                                            uint32_t chunks_per_stripe, uint32_t* sink) {
    typedef typename VecOf<VB>::T V;
    const uint32_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = blockIdx.x % 8;
    const uint32_t b = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + blockIdx.x / 8;
    const uint32_t stripe = b / chunks_per_stripe, chunk = b % chunks_per_stripe;
    uint8_t* s = base + uint64_t(stripe) * stripe_stride;
    const uint64_t o = uint64_t(chunk) * (256 * VB) + threadIdx.x * VB;
    V d[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) d[i] = __builtin_nontemporal_load(reinterpret_cast<const V*>(s + i * shard_stride + o));
    V acc = d[0];
#pragma unroll
    for (int i = 1; i < 10; ++i) acc ^= d[i];
#pragma unroll
    for (int j = 0; j < W; ++j) {
        V w = acc;
        w.x ^= j;
        __builtin_nontemporal_store(w, reinterpret_cast<V*>(s + (10 + j) * shard_stride + o));
    }
    if (W == 0 && acc.x == 0x12345678u && acc.y == 0x9abcdef0u) sink[threadIdx.x] = acc.x;  // practically never
}

struct Timer {
    hipEvent_t a, b;
    Timer() { CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b)); }
    void start() { CHECK(hipEventRecord(a)); }
    float stop() { CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b)); float ms; CHECK(hipEventElapsedTime(&ms, a, b)); return ms; }
};

template <typename F>
static void run(const char* name, const char* extra, double bytes, F f, int reps = 7) {
    Timer t;
    f();
    CHECK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int i = 0; i < reps; ++i) { t.start(); f(); ms.push_back(t.stop()); }
    std::sort(ms.begin(), ms.end());
    printf("{\"case\": \"%s\"%s, \"ms_med\": %.3f, \"TBps_med\": %.3f, \"TBps_best\": %.3f}\n", name, extra,
           ms[reps / 2], bytes / ms[reps / 2] / 1e9, bytes / ms[0] / 1e9);
    fflush(stdout);
}

// Padded layouts: 1 MiB shards at shard stride L + pad, or stripes at
// 14 L + stripe pad (does breaking the 2^20 spacing help the write streams?).
static int pad_sweep() {
    const uint64_t S = 4096, L = 1ull << 20, N = 14, maxpad = 65536;
    uint8_t* buf;
    CHECK(hipMalloc(&buf, S * N * (L + maxpad)));
    CHECK(hipMemset(buf, 0x5a, S * N * (L + maxpad)));
    const uint32_t cps = uint32_t(L / 4096), grid = uint32_t(S * cps);
    char extra[160];
    for (uint64_t pad : {0ull, 256ull, 1024ull, 2048ull, 4096ull, 8192ull, 12288ull, 65536ull}) {
        const uint64_t ss = L + pad;
        snprintf(extra, sizeof extra, ", \"shard_pad\": %llu, \"stripe_pad\": 0, \"xcd_remap\": 1",
                 (unsigned long long)pad);
        run("10r4w", extra, double(S * 14 * L), [&] {
            hipLaunchKernelGGL((k_nrmw<10, 4>), dim3(grid), dim3(256), 0, 0, buf, N * ss, ss, cps, 1);
        });
        run("0r14w", extra, double(S * 14 * L), [&] {
            hipLaunchKernelGGL((k_nrmw<0, 14>), dim3(grid), dim3(256), 0, 0, buf, N * ss, ss, cps, 1);
        });
    }
    for (uint64_t spad : {4096ull, 65536ull, 14ull * 65536ull}) {
        snprintf(extra, sizeof extra, ", \"shard_pad\": 0, \"stripe_pad\": %llu, \"xcd_remap\": 1",
                 (unsigned long long)spad);
        run("10r4w", extra, double(S * 14 * L), [&] {
            hipLaunchKernelGGL((k_nrmw<10, 4>), dim3(grid), dim3(256), 0, 0, buf, N * L + spad, L, cps, 1);
        });
        run("0r14w", extra, double(S * 14 * L), [&] {
            hipLaunchKernelGGL((k_nrmw<0, 14>), dim3(grid), dim3(256), 0, 0, buf, N * L + spad, L, cps, 1);
        });
    }
    CHECK(hipFree(buf));
    return 0;
}

// Read/write mix on the bench's padded layout (shard stride 1 MiB + 64 KiB,
// XCD eighths): 10 reads + m writes per stripe, m = 0..4, and 13r1w, 12r2w.
// Does a mostly-read mix run faster per byte than 10r4w?
static int mix_sweep() {
    const uint64_t S = 4096, L = 1ull << 20, N = 14, ss = L + 65536;
    uint8_t* buf;
    CHECK(hipMalloc(&buf, S * N * ss));
    CHECK(hipMemset(buf, 0x5a, S * N * ss));
    const uint32_t cps = uint32_t(L / 4096), grid = uint32_t(S * cps);
    char extra[96];
    snprintf(extra, sizeof extra, ", \"shard_stride\": %llu, \"xcd_remap\": 1", (unsigned long long)ss);
#define MIX(R, W)                                                                                         \
    run(#R "r" #W "w", extra, double(S * (R + W) * L), [&] {                                              \
        hipLaunchKernelGGL((k_nrmw<R, W>), dim3(grid), dim3(256), 0, 0, buf, N * ss, ss, cps, 1);         \
    })
    for (int round = 0; round < 2; ++round) {
        MIX(10, 0); MIX(10, 1); MIX(10, 2); MIX(10, 3); MIX(10, 4); MIX(13, 1); MIX(12, 2); MIX(14, 0); MIX(0, 14);
    }
#undef MIX
    CHECK(hipFree(buf));
    return 0;
}

// libhec's own batch entry points, for the calibration pass: the decode and
// encode run in the SAME rocprofv3 PMC pass as the calibration streams
// (build: make build/membench_calib, linked against helyim_amd/libhec.so).
#ifdef MEMBENCH_WITH_HEC
#include "../include/hec.h"
#endif

// Calibration pass: known-byte streams at 8 and 16 B per lane, then the
// shipped RS(10,4) encode and 4-erasure decode on the same padded batch
// (shard stride 1 MiB + 64 KiB, as bench.py). Each case runs `reps` times;
// tools/pmc_summary.py divides the known bytes by the counters.
static int calib() {
    const uint64_t S = 4096, L = 1ull << 20, N = 14, ss = L + 65536;
    const int reps = 3;
    uint8_t* buf;
    CHECK(hipMalloc(&buf, S * N * ss));
    CHECK(hipMemset(buf, 0x5a, S * N * ss));
    uint32_t* sink;
    CHECK(hipMalloc(&sink, 4096));
    char extra[160];
#define CAL(VB, W)                                                                                          \
    {                                                                                                       \
        const uint32_t cps = uint32_t(L / (256 * VB));                                                      \
        snprintf(extra, sizeof extra, ", \"bytes_per_lane\": %d, \"read_bytes\": %llu, \"write_bytes\": %llu", \
                 VB, (unsigned long long)(S * 10 * L), (unsigned long long)(S * W * L));                     \
        run("cal_" #VB "B_10r" #W "w", extra, double(S * (10 + W) * L), [&] {                               \
            hipLaunchKernelGGL((k_cal<VB, W>), dim3(uint32_t(S * cps)), dim3(256), 0, 0, buf, N * ss, ss, cps, sink); \
        }, reps);                                                                                           \
    }
    CAL(8, 0); CAL(8, 4); CAL(16, 0); CAL(16, 4);
#undef CAL
#ifdef MEMBENCH_WITH_HEC
    hec_rs_t* rs = nullptr;
    if (hec_rs_new(10, 4, &rs)) { fprintf(stderr, "hec_rs_new failed\n"); return 1; }
    std::vector<uint32_t> masks(S);
    uint64_t z = 0x9E3779B97F4A7C15ull;
    for (uint64_t s = 0; s < S; ++s) {  // 4 distinct erasures per stripe
        uint32_t m = (1u << 14) - 1;
        while (__builtin_popcount(m) > 10) {
            z ^= z << 13, z ^= z >> 7, z ^= z << 17;
            m &= ~(1u << (z % 14));
        }
        masks[s] = m;
    }
    uint32_t* dmask;
    CHECK(hipMalloc(&dmask, S * 4));
    CHECK(hipMemcpy(dmask, masks.data(), S * 4, hipMemcpyHostToDevice));
    snprintf(extra, sizeof extra, ", \"algorithmic_bytes\": %llu, \"kernel\": \"%s\"", (unsigned long long)(S * 14 * L),
             hec_encode_kernel_name(L));
    run("hec_encode", extra, double(S * 14 * L), [&] {
        if (hec_gpu_encode_batch(rs, buf, N * ss, ss, buf + 10 * ss, N * ss, ss, L, uint32_t(S), nullptr)) exit(1);
    }, reps);
    snprintf(extra, sizeof extra, ", \"algorithmic_bytes\": %llu, \"kernel\": \"%s\"", (unsigned long long)(S * 14 * L),
             hec_decode_kernel_name(L));
    run("hec_decode", extra, double(S * 14 * L), [&] {
        if (hec_gpu_reconstruct_batch(rs, buf, N * ss, ss, L, uint32_t(S), dmask, nullptr, nullptr)) exit(1);
    }, reps);
    CHECK(hipFree(dmask));
    hec_rs_free(rs);
#endif
    CHECK(hipFree(sink));
    CHECK(hipFree(buf));
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && std::string(argv[1]) == "calib") return calib();
    if (argc > 1 && std::string(argv[1]) == "pad") return pad_sweep();
    if (argc > 1 && std::string(argv[1]) == "mix") return mix_sweep();
    const uint64_t S = 4096, L = 1ull << 20, N = 14;
    const uint64_t total = S * N * L;  // 56 GiB
    uint8_t* buf;
    CHECK(hipMalloc(&buf, total));
    CHECK(hipMemset(buf, 0x5a, total));
    u32x4* sink;
    CHECK(hipMalloc(&sink, 4096));
    char extra[128];

    {  // copy 28 GiB -> 28 GiB
        const uint64_t n = total / 2 / 16;
        run("copy_1r1w", "", double(total), [&] {
            hipLaunchKernelGGL(k_copy, dim3(uint32_t(n / 256)), dim3(256), 0, 0, (const u32x4*)buf, (u32x4*)(buf + total / 2), n);
        });
    }
    {
        const uint64_t n = total / 16;
        run("read_only", "", double(total), [&] {
            hipLaunchKernelGGL(k_read, dim3(uint32_t(n / 256)), dim3(256), 0, 0, (const u32x4*)buf, sink, n);
        });
        run("write_only", "", double(total), [&] {
            hipLaunchKernelGGL(k_write, dim3(uint32_t(n / 256)), dim3(256), 0, 0, (u32x4*)buf, n);
        });
    }
    // n-read/m-write patterns on the [S][14][L] layout
    const uint32_t cps = uint32_t(L / 4096);
    const uint32_t grid = uint32_t(S * cps);
    for (int remap = 0; remap <= 1; ++remap) {
        snprintf(extra, sizeof extra, ", \"stride\": %llu, \"xcd_remap\": %d", (unsigned long long)L, remap);
        run("10r4w", extra, double(S * 14 * L), [&] {
            hipLaunchKernelGGL((k_nrmw<10, 4>), dim3(grid), dim3(256), 0, 0, buf, N * L, L, cps, remap);
        });
        run("14r0w", extra, double(S * 14 * L), [&] {
            hipLaunchKernelGGL((k_nrmw<14, 0>), dim3(grid), dim3(256), 0, 0, buf, N * L, L, cps, remap);
        });
        run("0r14w", extra, double(S * 14 * L), [&] {
            hipLaunchKernelGGL((k_nrmw<0, 14>), dim3(grid), dim3(256), 0, 0, buf, N * L, L, cps, remap);
        });
        run("7r7w", extra, double(S * 14 * L), [&] {
            hipLaunchKernelGGL((k_nrmw<7, 7>), dim3(grid), dim3(256), 0, 0, buf, N * L, L, cps, remap);
        });
        run("1r1w", extra, double(S * 2 * L * 7), [&] {  // 7 independent 1r1w pairs per stripe
            hipLaunchKernelGGL((k_nrmw<1, 1>), dim3(grid * 7), dim3(256), 0, 0, buf, 2 * L, L, cps, remap);
        });
    }
    // same 10r4w pattern at other shard spacings (stripes re-cut to keep 56 GiB)
    for (uint64_t stride : {4096ull, 65536ull, 262144ull, 1ull << 20, 4ull << 20}) {
        const uint64_t Ls = stride;  // shard length == spacing
        const uint64_t Ss = S * L / Ls;
        const uint32_t c = uint32_t(Ls / 4096);
        snprintf(extra, sizeof extra, ", \"stride\": %llu, \"xcd_remap\": 0", (unsigned long long)stride);
        run("10r4w", extra, double(Ss * 14 * Ls), [&] {
            hipLaunchKernelGGL((k_nrmw<10, 4>), dim3(uint32_t(Ss * c)), dim3(256), 0, 0, buf, N * Ls, Ls, c, 0);
        });
    }
    // chunk-per-workgroup x XCD remap x occupancy (LDS-limited blocks/CU) at 1 MiB shard stride
    for (int V : {1, 2, 4, 8}) {
        for (int remap = 0; remap <= 1; ++remap) {
            for (int lds : {0, 40 * 1024, 80 * 1024}) {
                const uint32_t c = uint32_t(L / (4096 * V));
                snprintf(extra, sizeof extra, ", \"V\": %d, \"xcd_remap\": %d, \"lds\": %d", V, remap, lds);
                auto launch = [&] {
                    switch (V) {
                        case 1: hipLaunchKernelGGL((k_10r4w_v<1>), dim3(uint32_t(S * c)), dim3(256), lds, 0, buf, N * L, L, c, remap); break;
                        case 2: hipLaunchKernelGGL((k_10r4w_v<2>), dim3(uint32_t(S * c)), dim3(256), lds, 0, buf, N * L, L, c, remap); break;
                        case 4: hipLaunchKernelGGL((k_10r4w_v<4>), dim3(uint32_t(S * c)), dim3(256), lds, 0, buf, N * L, L, c, remap); break;
                        default: hipLaunchKernelGGL((k_10r4w_v<8>), dim3(uint32_t(S * c)), dim3(256), lds, 0, buf, N * L, L, c, remap); break;
                    }
                };
                run("10r4w_v", extra, double(S * 14 * L), launch);
            }
        }
    }
    for (uint64_t stride : {16384ull, 32768ull, 65536ull, 131072ull}) {
        const uint64_t Ls = stride, Ss = S * L / Ls;
        const uint32_t c = uint32_t(Ls / 4096);
        snprintf(extra, sizeof extra, ", \"stride\": %llu, \"xcd_remap\": 1", (unsigned long long)stride);
        run("10r4w", extra, double(Ss * 14 * Ls), [&] {
            hipLaunchKernelGGL((k_nrmw<10, 4>), dim3(uint32_t(Ss * c)), dim3(256), 0, 0, buf, N * Ls, Ls, c, 1);
        });
    }
    for (int lp : {2, 0, 1, 16}) {
        for (int sp : {2, 0, 1, 3, 16, 17, 18, 19}) {
            if (lp != 2 && sp != 2) continue;
            snprintf(extra, sizeof extra, ", \"load_pol\": %d, \"store_pol\": %d", lp, sp);
            run("10r4w_pol", extra, double(S * 14 * L), [&] {
                hipLaunchKernelGGL(k_10r4w_pol, dim3(grid), dim3(256), 0, 0, buf, N * L, uint32_t(L), cps, lp, sp);
            });
        }
    }
    CHECK(hipFree(buf));
    return 0;
}

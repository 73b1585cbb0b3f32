// Which physical address bits spread HBM traffic over channels? Reads (or
// writes) confined to the addresses whose bit b equals 0 -- half of a 32 GiB
// span, moved in pieces of G bytes -- against the same amount of traffic on a
// contiguous half (bit 35). A bit that selects between two disjoint halves of
// the channels (with no XOR partner below log2(G), which varies inside every
// piece) halves the rate; a bit the address hash mixes with lower bits does
// not. Measurement only (DESIGN.md "What bounds it").
// Build: hipcc --offload-arch=gfx950 -O3 -o build/chanprobe tools/chanprobe.hip
// Run:   build/chanprobe   (one JSON line per case)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e = (x);                                                               \
        if (e != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

// piece q -> address with bit `bit` forced to 0: the piece index's bits at and
// above (bit - g) move up by one
__device__ __forceinline__ uint64_t piece_addr(uint64_t q, int g, int bit) {
    const int s = bit - g;
    const uint64_t lo = q & ((1ull << s) - 1), hi = q >> s;
    return ((hi << (s + 1)) | lo) << g;
}

// 256 lanes x 16 B per workgroup = 4 KiB = 4096 >> g pieces of 2^g bytes
template <bool WRITE>
__global__ __launch_bounds__(256) void k_sel(uint8_t* base, int g, int bit, u32x4* sink) {
    const uint64_t byte = uint64_t(blockIdx.x) * 4096 + threadIdx.x * 16;  // in the confined stream
    const uint64_t q = byte >> g, in = byte & ((1ull << g) - 1);
    u32x4* p = reinterpret_cast<u32x4*>(base + piece_addr(q, g, bit) + in);
    if constexpr (WRITE) {
        __builtin_nontemporal_store(u32x4{uint32_t(byte), 1, 2, 3}, p);
    } else {
        const u32x4 v = __builtin_nontemporal_load(p);
        if (v.x == 0x12345678u && v.y == 0x9abcdef0u) sink[threadIdx.x] = v;  // practically never
    }
}

int main() {
    const uint64_t span = 1ull << 36;   // 64 GiB allocation
    const uint64_t moved = span / 2;    // every case moves 32 GiB
    uint8_t* buf;
    CHECK(hipMalloc(&buf, span));
    CHECK(hipMemset(buf, 0x5a, span));
    u32x4* sink;
    CHECK(hipMalloc(&sink, 4096));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const uint32_t grid = uint32_t(moved / 4096);
    for (int g : {8, 12}) {
        for (int bit = g; bit <= 35; ++bit) {
            for (int w = 0; w < 2; ++w) {
                auto launch = [&] {
                    if (w) hipLaunchKernelGGL(k_sel<true>, dim3(grid), dim3(256), 0, 0, buf, g, bit, sink);
                    else hipLaunchKernelGGL(k_sel<false>, dim3(grid), dim3(256), 0, 0, buf, g, bit, sink);
                };
                launch();
                CHECK(hipDeviceSynchronize());
                std::vector<float> ms;
                for (int r = 0; r < 3; ++r) {
                    CHECK(hipEventRecord(a));
                    launch();
                    CHECK(hipEventRecord(b));
                    CHECK(hipEventSynchronize(b));
                    float t;
                    CHECK(hipEventElapsedTime(&t, a, b));
                    ms.push_back(t);
                }
                std::sort(ms.begin(), ms.end());
                printf("{\"piece_log2\": %d, \"bit\": %d, \"op\": \"%s\", \"ms_med\": %.3f, \"TBps\": %.3f}\n", g, bit,
                       w ? "write" : "read", ms[1], double(moved) / ms[1] / 1e9);
                fflush(stdout);
            }
        }
    }
    CHECK(hipFree(buf));
    CHECK(hipFree(sink));
    return 0;
}

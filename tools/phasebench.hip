// Read/write phase-separation probe for the RS(10,4) traffic mix on MI355X.
//
// Question: the 10-read / 4-write stream pattern tops out near 6.3 TB/s while
// a pure read stream reaches ~7.1 and a pure write stream ~6.75 (DESIGN.md §4
// "What bounds it"). If the loss is the HBM read/write turnaround of mixed
// traffic, would the chip move the same bytes faster when EVERY CU reads in
// the same time window and writes in the next one? No inter-CU communication
// is needed for that: all CUs read the chip-wide 100 MHz REALTIME counter
// (s_memrealtime) and pick the phase from it.
//
// Kernel: 4 workgroups per CU, each owning 40 MiB of reads and 16 MiB of
// writes (10:4, 56 GiB in all, as one bench launch). A workgroup moves 32 KiB
// batches (8 x 16 B per lane, all in flight): a read batch when the clock is
// in the read window (or its writes are done), a write batch otherwise. It
// never waits, so it always terminates. Mode "mixed" ignores the clock and
// interleaves batches 10:4 (the encode's mix). Bytes are junk (probe only).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o build/phasebench tools/phasebench.hip
// Run:   build/phasebench      (one JSON line per case)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                               \
    do {                                                                                       \
        hipError_t e = (x);                                                                    \
        if (e != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));   \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

constexpr int kBatch = 8;  // 16-byte vectors per lane per batch (32 KiB per 256-lane workgroup)

// period / read_ticks in 100 MHz ticks; period == 0: clock ignored, batches
// interleaved so that reads : writes stay rb : wb.
// interleave 1: batch i of workgroup g sits at (i * grid + g) (the grid sweeps
// one contiguous span per step, as the dispatch-order kernels do); 0: each
// workgroup streams its own contiguous region.
__global__ __launch_bounds__(256) void k_phased(const u32x4* __restrict__ rsrc, u32x4* __restrict__ wdst,
                                                uint32_t rb, uint32_t wb, uint32_t period, uint32_t read_ticks,
                                                u32x4* sink, int interleave) {
    const uint64_t g = blockIdx.x, G = gridDim.x;
    const uint64_t rstep = interleave ? G : 1, wstep = interleave ? G : 1;
    const u32x4* rp = rsrc + (interleave ? g : g * rb) * kBatch * 256 + threadIdx.x;
    u32x4* wp = wdst + (interleave ? g : g * wb) * kBatch * 256 + threadIdx.x;
    uint32_t ri = 0, wi = 0;
    u32x4 acc = {0, 0, 0, 0};
    while (ri < rb || wi < wb) {
        bool do_read;
        if (ri >= rb) {
            do_read = false;
        } else if (wi >= wb) {
            do_read = true;
        } else if (period == 0) {
            do_read = uint64_t(ri) * wb <= uint64_t(wi) * rb;
        } else {
            const uint64_t t = __builtin_amdgcn_s_memrealtime();
            do_read = uint32_t(t % period) < read_ticks;
        }
        if (do_read) {
            u32x4 d[kBatch];
#pragma unroll
            for (int k = 0; k < kBatch; ++k) d[k] = __builtin_nontemporal_load(rp + (uint64_t(ri) * rstep * kBatch + k) * 256);
#pragma unroll
            for (int k = 0; k < kBatch; ++k) acc ^= d[k];
            ++ri;
        } else {
#pragma unroll
            for (int k = 0; k < kBatch; ++k) {
                u32x4 v = acc;
                v.x ^= k;
                __builtin_nontemporal_store(v, wp + (uint64_t(wi) * wstep * kBatch + k) * 256);
            }
            ++wi;
        }
    }
    if (acc.x == 0x12345678u && acc.y == 0x9abcdef0u) sink[threadIdx.x] = acc;  // keeps the loads live
}

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t wgs = uint32_t(cus) * (getenv("PB_WG_PER_CU") ? atoi(getenv("PB_WG_PER_CU")) : 4);
    const uint64_t R = 40ull << 30, W = 16ull << 30;
    const uint64_t batch_bytes = uint64_t(kBatch) * 256 * 16;
    const uint32_t rb = uint32_t(R / wgs / batch_bytes), wb = uint32_t(W / wgs / batch_bytes);
    const double bytes = double(uint64_t(rb) * wgs * batch_bytes + uint64_t(wb) * wgs * batch_bytes);
    uint8_t *r, *w;
    u32x4* sink;
    CHECK(hipMalloc(&r, uint64_t(rb) * wgs * batch_bytes));
    CHECK(hipMalloc(&w, uint64_t(wb) * wgs * batch_bytes));
    CHECK(hipMalloc(&sink, 4096));
    CHECK(hipMemset(r, 0x5a, uint64_t(rb) * wgs * batch_bytes));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    struct Case { const char* name; uint32_t period, read_ticks; };
    std::vector<Case> cases = {{"mixed", 0, 0}};
    for (uint32_t p : {2000u, 4000u, 8000u, 16000u, 32000u})
        for (double f : {0.66, 0.72}) cases.push_back({"phased", p, uint32_t(p * f)});
    cases.push_back({"mixed", 0, 0});
    const int il = getenv("PB_INTERLEAVE") ? atoi(getenv("PB_INTERLEAVE")) : 1;
    for (const Case& c : cases) {
        std::vector<float> ms;
        for (int i = 0; i < 6; ++i) {
            CHECK(hipEventRecord(a));
            hipLaunchKernelGGL(k_phased, dim3(wgs), dim3(256), 0, 0, (const u32x4*)r, (u32x4*)w, rb, wb, c.period,
                               c.read_ticks, sink, il);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float t;
            CHECK(hipEventElapsedTime(&t, a, b));
            if (i) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        printf("{\"wgs\": %u, \"interleave\": %d, \"case\": \"%s\", \"period_us\": %.1f, \"read_frac\": %.2f, \"ms_med\": %.3f, \"TBps_med\": %.3f, "
               "\"TBps_best\": %.3f}\n",
               wgs, il, c.name, c.period / 100.0, c.period ? double(c.read_ticks) / c.period : 10.0 / 14, ms[ms.size() / 2],
               bytes / ms[ms.size() / 2] / 1e9, bytes / ms[0] / 1e9);
        fflush(stdout);
    }
    for (int mode = 0; mode < 2; ++mode) {  // read-only / write-only of the same byte counts
        std::vector<float> ms;
        for (int i = 0; i < 6; ++i) {
            CHECK(hipEventRecord(a));
            hipLaunchKernelGGL(k_phased, dim3(wgs), dim3(256), 0, 0, (const u32x4*)r, (u32x4*)w, mode ? 0 : rb,
                               mode ? wb : 0, 0u, 0u, sink, il);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float t;
            CHECK(hipEventElapsedTime(&t, a, b));
            if (i) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const double by = double(uint64_t(mode ? wb : rb) * wgs * batch_bytes);
        printf("{\"case\": \"%s\", \"ms_med\": %.3f, \"TBps_med\": %.3f}\n", mode ? "write_only" : "read_only",
               ms[ms.size() / 2], by / ms[ms.size() / 2] / 1e9);
        fflush(stdout);
    }
    return 0;
}

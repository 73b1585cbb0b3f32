// Zero-copy probe: the RS(10,4) encode kernel reading data shards straight from
// mapped pinned host memory and writing parity straight back to it (no SDMA
// copies), against the copy pipeline (hec_host_encode_batch). Parity checked
// against a device-resident encode of the same bytes. Measurement only.
// build: hipcc -O2 --offload-arch=gfx950 -I include tools/zerocopy_probe.hip -L helyim_amd -lhec -o build/zerocopy_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "hec.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)
#define HCHECK(x) do { int r_ = (x); if (r_) { std::printf("hec error %d (%s) at %d\n", r_, hec_last_error_detail(), __LINE__); std::exit(1); } } while (0)

int main(int argc, char** argv) {
    const uint32_t S = argc > 1 ? uint32_t(std::atoi(argv[1])) : 512;
    const uint64_t L = 1 << 20, N = 14;
    const uint64_t bytes = S * N * L;
    hec_rs_t* rs;
    HCHECK(hec_rs_new(10, 4, &rs));
    for (unsigned flags : {unsigned(hipHostMallocDefault), unsigned(hipHostMallocMapped | hipHostMallocNonCoherent)}) {
        uint8_t* h;
        CHECK(hipHostMalloc(reinterpret_cast<void**>(&h), bytes, flags));
        uint8_t* hd;
        CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hd), h, 0));
        for (uint64_t i = 0; i < bytes; i += 8) {
            uint64_t z = i * 0x9E3779B97F4A7C15ull;
            z ^= z >> 29;
            std::memcpy(h + i, &z, 8);
        }
        uint8_t* d;
        CHECK(hipMalloc(reinterpret_cast<void**>(&d), bytes));
        CHECK(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice));
        HCHECK(hec_gpu_encode_batch(rs, d, N * L, L, d + 10 * L, N * L, L, L, S, nullptr));
        CHECK(hipDeviceSynchronize());
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        // zero-copy: kernel reads host data, writes host parity
        HCHECK(hec_gpu_encode_batch(rs, hd, N * L, L, hd + 10 * L, N * L, L, L, S, nullptr));  // warm-up
        CHECK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            CHECK(hipEventRecord(a));
            HCHECK(hec_gpu_encode_batch(rs, hd, N * L, L, hd + 10 * L, N * L, L, L, S, nullptr));
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms;
            CHECK(hipEventElapsedTime(&ms, a, b));
            best = ms < best ? ms : best;
        }
        // compare parity with the device-resident encode
        std::vector<uint8_t> ref(bytes);
        CHECK(hipMemcpy(ref.data(), d, bytes, hipMemcpyDeviceToHost));
        bool same = std::memcmp(ref.data(), h, bytes) == 0;
        // copy pipeline for comparison
        auto t0 = std::chrono::steady_clock::now();
        HCHECK(hec_host_encode_batch(rs, h, N * L, L, h + 10 * L, N * L, L, L, S));
        auto t1 = std::chrono::steady_clock::now();
        const double pipe_s = std::chrono::duration<double>(t1 - t0).count();
        const double data = double(S) * 10 * L;
        std::printf("{\"flags\": %u, \"stripes\": %u, \"zero_copy_ms\": %.3f, \"zero_copy_data_GiB_s\": %.2f, "
                    "\"pcie_GB_s\": %.2f, \"copy_pipeline_data_GiB_s\": %.2f, \"identical\": %s}\n",
                    flags, S, best, data / (best * 1e-3) / (1 << 30), data * 1.4 / (best * 1e-3) / 1e9,
                    data / pipe_s / (1 << 30), same ? "true" : "false");
        std::fflush(stdout);
        CHECK(hipFree(d));
        CHECK(hipHostFree(h));
    }
    return 0;
}

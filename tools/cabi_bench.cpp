// The BASELINE device-resident workload driven through the C ABI alone
// (include/hec.h), as a C/Rust consumer would call it: no Python, no PyTorch.
// 4096 x [14][1 MiB] stripes in HBM, splitmix64 data (hec_gpu_fill_splitmix),
// encode (hec_gpu_encode_batch) then a 4-erasure reconstruct
// (hec_gpu_reconstruct_batch), timed with HIP events on the caller's stream.
// Checks: sampled stripes are erased on the device and must come back
// byte-identical. Prints one JSON line.
//
//   make build/cabi_bench && build/cabi_bench [stripes] [steps] [warmup]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/hec.h"

#define HIPCHECK(x)                                                                          \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 2;                                                                        \
        }                                                                                    \
    } while (0)
#define HECCHECK(x)                                                                         \
    do {                                                                                    \
        int rc_ = (x);                                                                      \
        if (rc_ != HEC_OK) {                                                                \
            std::fprintf(stderr, "%s:%d %s: %s (%s)\n", __FILE__, __LINE__, #x, hec_strerror(rc_), \
                         hec_last_error_detail());                                           \
            return 2;                                                                       \
        }                                                                                   \
    } while (0)

static uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main(int argc, char** argv) {
    const uint32_t S = argc > 1 ? uint32_t(std::atoi(argv[1])) : 4096;
    const int steps = argc > 2 ? std::atoi(argv[2]) : 10;
    const int warmup = argc > 3 ? std::atoi(argv[3]) : 3;
    const uint64_t L = 1ull << 20, N = HEC_TOTAL_SHARDS_COUNT, stripe = N * L;
    if (S == 0 || steps <= 0 || warmup < 0) return 1;

    hec_rs_t* rs = nullptr;
    HECCHECK(hec_rs_new(HEC_DATA_SHARDS_COUNT, HEC_PARITY_SHARDS_COUNT, &rs));
    HECCHECK(hec_set_device(0));
    hipStream_t st;
    HIPCHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    uint8_t* d = nullptr;
    uint32_t *d_masks = nullptr, *d_bad = nullptr;
    HIPCHECK(hipMalloc(&d, S * stripe));
    HIPCHECK(hipMalloc(&d_masks, S * 4));
    HIPCHECK(hipMalloc(&d_bad, 4));
    HECCHECK(hec_gpu_fill_splitmix(d, stripe, HEC_DATA_SHARDS_COUNT * L, S, 0x5EED0000ull, st));

    // 4 erasures per stripe, uniform over the 1001 patterns (seeded)
    std::vector<uint32_t> masks(S);
    uint64_t seed = 0xEC0000;
    for (auto& m : masks) {
        int idx[14] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13};
        for (int i = 0; i < 4; ++i) std::swap(idx[i], idx[i + int(splitmix(seed) % (14 - i))]);
        m = 0x3FFF;
        for (int i = 0; i < 4; ++i) m &= ~(1u << idx[i]);
    }
    HIPCHECK(hipMemcpyAsync(d_masks, masks.data(), S * 4, hipMemcpyHostToDevice, st));
    HIPCHECK(hipMemsetAsync(d_bad, 0, 4, st));

    auto encode = [&] {
        return hec_gpu_encode_batch(rs, d, stripe, L, d + HEC_DATA_SHARDS_COUNT * L, stripe, L, L, S, st);
    };
    auto decode = [&] { return hec_gpu_reconstruct_batch(rs, d, stripe, L, L, S, d_masks, d_bad, st); };
    for (int i = 0; i < warmup; ++i) {
        HECCHECK(encode());
        HECCHECK(decode());
    }
    std::vector<hipEvent_t> ev(3 * steps);
    for (auto& e : ev) HIPCHECK(hipEventCreate(&e));
    HIPCHECK(hipStreamSynchronize(st));
    for (int i = 0; i < steps; ++i) {
        HIPCHECK(hipEventRecord(ev[3 * i], st));
        HECCHECK(encode());
        HIPCHECK(hipEventRecord(ev[3 * i + 1], st));
        HECCHECK(decode());
        HIPCHECK(hipEventRecord(ev[3 * i + 2], st));
    }
    HIPCHECK(hipStreamSynchronize(st));
    double enc = 0, dec = 0;
    for (int i = 0; i < steps; ++i) {
        float a, b;
        HIPCHECK(hipEventElapsedTime(&a, ev[3 * i], ev[3 * i + 1]));
        HIPCHECK(hipEventElapsedTime(&b, ev[3 * i + 1], ev[3 * i + 2]));
        enc += a, dec += b;
    }
    enc /= steps, dec /= steps;

    // verification: erase sampled stripes on the device, rebuild, compare
    const uint32_t V = std::min<uint32_t>(S, 16);
    std::vector<uint8_t> want(V * stripe), got(V * stripe);
    HIPCHECK(hipMemcpy(want.data(), d, V * stripe, hipMemcpyDeviceToHost));
    for (uint32_t s = 0; s < V; ++s)
        for (uint64_t i = 0; i < N; ++i)
            if (!((masks[s] >> i) & 1)) HIPCHECK(hipMemsetAsync(d + s * stripe + i * L, 0xA5, L, st));
    HECCHECK(hec_gpu_reconstruct_batch(rs, d, stripe, L, L, V, d_masks, d_bad, st));
    HIPCHECK(hipStreamSynchronize(st));
    HIPCHECK(hipMemcpy(got.data(), d, V * stripe, hipMemcpyDeviceToHost));
    uint32_t bad = 0;
    HIPCHECK(hipMemcpy(&bad, d_bad, 4, hipMemcpyDeviceToHost));
    const bool ok = std::memcmp(want.data(), got.data(), want.size()) == 0 && bad == 0;

    const double bytes = double(S) * stripe;  // encode: 10 L read + 4 L written; decode: 10 + 4
    std::printf("{\"tool\": \"cabi_bench\", \"api\": \"hec_gpu_encode_batch + hec_gpu_reconstruct_batch\", "
                "\"stripes\": %u, \"shard_len\": %llu, \"steps\": %d, \"encode_ms\": %.4f, \"decode_ms\": %.4f, "
                "\"encode_TBps\": %.3f, \"decode_TBps\": %.3f, \"encode_frac\": %.4f, "
                "\"data_GiB_s\": %.1f, \"encode_kernel\": \"%s\", \"verified\": %s}\n",
                S, (unsigned long long)L, steps, enc, dec, bytes / enc / 1e9, bytes / dec / 1e9,
                bytes / enc / 1e9 / 8.0, 2.0 * S * HEC_DATA_SHARDS_COUNT * L / ((enc + dec) * 1e-3) / (1ull << 30),
                hec_encode_kernel_name(L), ok ? "true" : "false");
    for (auto& e : ev) (void)hipEventDestroy(e);
    (void)hipFree(d);
    (void)hipFree(d_masks);
    (void)hipFree(d_bad);
    (void)hipStreamDestroy(st);
    hec_rs_free(rs);
    return ok ? 0 : 3;
}

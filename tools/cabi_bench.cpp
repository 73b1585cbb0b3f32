// The BASELINE device-resident workload driven through the C ABI alone
// (include/hec.h), as a C/Rust consumer would call it: no Python, no PyTorch.
// Per worker: S x [14][1 MiB] stripes in HBM (a 64 KiB gap after every shard,
// as bench.py lays its batch out; argv[5] sets the gap), splitmix64 data
// (hec_gpu_fill_splitmix), encode (hec_gpu_encode_batch) then a 4-erasure
// reconstruct (hec_gpu_reconstruct_batch), timed with HIP events on the
// worker's own stream. Checks: sampled stripes are erased on the device and
// must come back byte-identical. Prints one JSON line.
//
// Workers are threads, worker t on device t % count (hec_set_device): SURVEY
// §8d config 4's "thread + stream per GPU, no collective" form of weak
// scaling. Workers start together after a host barrier; the job time is the
// slowest worker's wall time over the timed steps.
//
//   make build/cabi_bench && build/cabi_bench [stripes] [steps] [warmup] [workers] [shard_gap]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../include/hec.h"

#define HIPCHECK(x)                                                                                 \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) {                                                                     \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 2;                                                                               \
        }                                                                                           \
    } while (0)
#define HECCHECK(x)                                                                                      \
    do {                                                                                                 \
        int rc_ = (x);                                                                                   \
        if (rc_ != HEC_OK) {                                                                             \
            std::fprintf(stderr, "%s:%d %s: %s (%s)\n", __FILE__, __LINE__, #x, hec_strerror(rc_),      \
                         hec_last_error_detail());                                                       \
            return 2;                                                                                    \
        }                                                                                                \
    } while (0)

namespace {

constexpr uint64_t L = 1ull << 20, N = HEC_TOTAL_SHARDS_COUNT;
uint64_t P = L + (64ull << 10);  // shard stride
uint64_t kStripe = N * P;        // stripe stride

uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Host barrier for the workers (every worker reaches it once per phase).
struct Barrier {
    std::mutex mu;
    std::condition_variable cv;
    int n, waiting = 0;
    uint64_t gen = 0;
    explicit Barrier(int n_) : n(n_) {}
    void wait() {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t g = gen;
        if (++waiting == n) {
            waiting = 0;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != g; });
        }
    }
};

struct Result {
    int rc = 1;
    int device = -1;
    double wall_s = 0, enc_ms = 0, dec_ms = 0;
    bool ok = false;
};

int worker(int t, int device, uint32_t S, int steps, int warmup, hec_rs_t* rs, Barrier& bar, Result& res) {
    // Every exit path passes both barriers so the other workers never hang.
    struct Guard {
        Barrier& b;
        int passed = 0;
        ~Guard() {
            while (passed++ < 2) b.wait();
        }
    } guard{bar};
    HECCHECK(hec_set_device(device));
    HECCHECK(hec_get_device(&res.device));
    hipStream_t st;
    HIPCHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    uint8_t* d = nullptr;
    uint32_t *d_masks = nullptr, *d_bad = nullptr;
    HIPCHECK(hipMalloc(&d, S * kStripe));
    HIPCHECK(hipMalloc(&d_masks, S * 4));
    HIPCHECK(hipMalloc(&d_bad, 4));
    // worker t's stripes are seeded like bench.py's rank t
    // shard i holds words i * L / 8 on of its stripe's splitmix64 stream: the
    // bytes a packed batch gets from one hec_gpu_fill_splitmix per stripe
    for (uint64_t i = 0; i < HEC_DATA_SHARDS_COUNT; ++i)
        HECCHECK(hec_gpu_fill_splitmix(d + i * P, kStripe, L, S,
                                       0x5EED0000ull + (uint64_t(t) << 20) + i * (L / 8) * 0x9E3779B97F4A7C15ull, st));

    // 4 erasures per stripe, uniform over the 1001 patterns (seeded per worker)
    std::vector<uint32_t> masks(S);
    uint64_t seed = 0xEC0000 + uint64_t(t);
    for (auto& m : masks) {
        int idx[14] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13};
        for (int i = 0; i < 4; ++i) std::swap(idx[i], idx[i + int(splitmix(seed) % uint64_t(14 - i))]);
        m = 0x3FFF;
        for (int i = 0; i < 4; ++i) m &= ~(1u << idx[i]);
    }
    HIPCHECK(hipMemcpyAsync(d_masks, masks.data(), S * 4, hipMemcpyHostToDevice, st));
    HIPCHECK(hipMemsetAsync(d_bad, 0, 4, st));

    auto encode = [&] {
        return hec_gpu_encode_batch(rs, d, kStripe, P, d + HEC_DATA_SHARDS_COUNT * P, kStripe, P, L, S, st);
    };
    auto decode = [&] { return hec_gpu_reconstruct_batch(rs, d, kStripe, P, L, S, d_masks, d_bad, st); };
    for (int i = 0; i < warmup; ++i) {
        HECCHECK(encode());
        HECCHECK(decode());
    }
    std::vector<hipEvent_t> ev(3 * size_t(steps));
    for (auto& e : ev) HIPCHECK(hipEventCreate(&e));
    HIPCHECK(hipStreamSynchronize(st));
    ++guard.passed;
    bar.wait();  // all workers warmed up: start together
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < steps; ++i) {
        HIPCHECK(hipEventRecord(ev[3 * i], st));
        HECCHECK(encode());
        HIPCHECK(hipEventRecord(ev[3 * i + 1], st));
        HECCHECK(decode());
        HIPCHECK(hipEventRecord(ev[3 * i + 2], st));
    }
    HIPCHECK(hipStreamSynchronize(st));
    res.wall_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    ++guard.passed;
    bar.wait();
    for (int i = 0; i < steps; ++i) {
        float a, b;
        HIPCHECK(hipEventElapsedTime(&a, ev[3 * i], ev[3 * i + 1]));
        HIPCHECK(hipEventElapsedTime(&b, ev[3 * i + 1], ev[3 * i + 2]));
        res.enc_ms += a / steps, res.dec_ms += b / steps;
    }

    // verification: erase sampled stripes on the device, rebuild, compare
    const uint32_t V = std::min<uint32_t>(S, 16);
    std::vector<uint8_t> want(V * kStripe), got(V * kStripe);
    HIPCHECK(hipMemcpy(want.data(), d, V * kStripe, hipMemcpyDeviceToHost));
    for (uint32_t s = 0; s < V; ++s)
        for (uint64_t i = 0; i < N; ++i)
            if (!((masks[s] >> i) & 1)) HIPCHECK(hipMemsetAsync(d + s * kStripe + i * P, 0xA5, L, st));
    HECCHECK(hec_gpu_reconstruct_batch(rs, d, kStripe, P, L, V, d_masks, d_bad, st));
    HIPCHECK(hipStreamSynchronize(st));
    HIPCHECK(hipMemcpy(got.data(), d, V * kStripe, hipMemcpyDeviceToHost));
    uint32_t bad = 0;
    HIPCHECK(hipMemcpy(&bad, d_bad, 4, hipMemcpyDeviceToHost));
    res.ok = std::memcmp(want.data(), got.data(), want.size()) == 0 && bad == 0;

    for (auto& e : ev) (void)hipEventDestroy(e);
    (void)hipFree(d);
    (void)hipFree(d_masks);
    (void)hipFree(d_bad);
    (void)hipStreamDestroy(st);
    res.rc = 0;
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    const uint32_t S = argc > 1 ? uint32_t(std::atoi(argv[1])) : 4096;
    const int steps = argc > 2 ? std::atoi(argv[2]) : 10;
    const int warmup = argc > 3 ? std::atoi(argv[3]) : 3;
    const int workers = argc > 4 ? std::atoi(argv[4]) : 1;
    const long gap = argc > 5 ? std::atol(argv[5]) : 64l << 10;
    if (S == 0 || steps <= 0 || warmup < 0 || workers <= 0 || workers > 64 || gap < 0) return 1;
    P = L + uint64_t(gap);
    kStripe = N * P;
    int count = 0;
    HECCHECK(hec_device_count(&count));
    hec_rs_t* rs = nullptr;  // one immutable context shared by every worker (hec.h threading rules)
    HECCHECK(hec_rs_new(HEC_DATA_SHARDS_COUNT, HEC_PARITY_SHARDS_COUNT, &rs));

    Barrier bar(workers);
    std::vector<Result> res(workers);
    std::vector<std::thread> th;
    for (int t = 0; t < workers; ++t)
        th.emplace_back([&, t] { worker(t, t % count, S, steps, warmup, rs, bar, res[t]); });
    for (auto& x : th) x.join();
    hec_rs_free(rs);

    bool ok = true;
    double wall = 0, enc = 0, dec = 0;
    std::string devs;
    for (int t = 0; t < workers; ++t) {
        ok = ok && res[t].rc == 0 && res[t].ok;
        wall = std::max(wall, res[t].wall_s);
        enc = std::max(enc, res[t].enc_ms);
        dec = std::max(dec, res[t].dec_ms);
        devs += (t ? "," : "") + std::to_string(res[t].device);
    }
    const double bytes = double(S) * N * L;  // per worker and launch: encode 10 L + 4 L, decode 10 + 4
    const double payload = 2.0 * workers * S * HEC_DATA_SHARDS_COUNT * L * steps;
    std::printf("{\"tool\": \"cabi_bench\", \"api\": \"hec_gpu_encode_batch + hec_gpu_reconstruct_batch\", "
                "\"workers\": %d, \"devices\": [%s], \"visible_devices\": %d, \"stripes_per_worker\": %u, "
                "\"shard_len\": %llu, \"shard_stride\": %llu, \"steps\": %d, \"job_data_GiB_s\": %.1f, \"encode_ms\": %.4f, "
                "\"decode_ms\": %.4f, \"encode_TBps\": %.3f, \"decode_TBps\": %.3f, \"encode_frac\": %.4f, "
                "\"encode_kernel\": \"%s\", \"verified\": %s}\n",
                workers, devs.c_str(), count, S, (unsigned long long)L, (unsigned long long)P, steps, payload / wall / double(1ull << 30),
                enc, dec, bytes / enc / 1e9, bytes / dec / 1e9, bytes / enc / 1e9 / 8.0, hec_encode_kernel_name(L),
                ok ? "true" : "false");
    return ok ? 0 : 3;
}

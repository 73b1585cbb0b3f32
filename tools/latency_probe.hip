// Small-call latency floor on MI355X: what one per-call drop-in
// (hec_rs_encode / hec_rs_reconstruct on a 1-4 KiB needle interval) pays
// beyond its bytes. Cases, median of 2000 round trips each (µs):
//   launch_sync      : empty kernel + hipStreamSynchronize
//   launch_event     : empty kernel + hipEventRecord + hipEventSynchronize
//   launch_flag      : kernel stores a flag into pinned host memory (system
//                      scope, after a system fence); the host spins on it
//   zc_sync / zc_flag: a 4 KiB-per-shard zero-copy "stripe" (10 x 4 KiB read
//                      over PCIe by one 256-lane workgroup, 4 x 4 KiB written
//                      back) with either completion
//   launch_query     : empty kernel + hipStreamQuery spin (launch_evquery: on an event)
//   launch_only      : host time of hipLaunchKernelGGL alone
// Build: hipcc --offload-arch=gfx950 -O3 -o build/latency_probe tools/latency_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                             \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                         \
        }                                                                                    \
    } while (0)

__global__ void k_empty() {}

__global__ void k_flag(volatile uint32_t* flag, uint32_t v) {
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(const_cast<uint32_t*>(flag), v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// 10 x 4 KiB in, 4 x 4 KiB out, one workgroup, all over PCIe (zero copy)
__global__ __launch_bounds__(256) void k_zc(const u32x4* in, u32x4* out, volatile uint32_t* flag, uint32_t v) {
    u32x4 d[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) d[i] = in[i * 256 + threadIdx.x];
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 10; ++i) acc ^= d[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        u32x4 w = acc;
        w.x ^= j;
        out[j * 256 + threadIdx.x] = w;
    }
    if (flag) {
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence_system();
            __hip_atomic_store(const_cast<uint32_t*>(flag), v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

using clk = std::chrono::steady_clock;

template <typename F>
static void run(const char* name, F f, int n = 2000) {
    for (int i = 0; i < 50; ++i) f(i);
    std::vector<double> us;
    us.reserve(n);
    for (int i = 0; i < n; ++i) {
        auto t0 = clk::now();
        f(i + 50);
        us.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
    }
    std::sort(us.begin(), us.end());
    printf("{\"case\": \"%s\", \"us_p50\": %.2f, \"us_p10\": %.2f, \"us_p90\": %.2f}\n", name, us[n / 2], us[n / 10],
           us[n * 9 / 10]);
    fflush(stdout);
}

int main() {
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev;
    CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    uint32_t* flag;
    CHECK(hipHostMalloc(reinterpret_cast<void**>(&flag), 4096, hipHostMallocDefault));
    *flag = 0;
    uint32_t* dflag;
    CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dflag), flag, 0));
    uint8_t* hio;
    CHECK(hipHostMalloc(reinterpret_cast<void**>(&hio), 14 * 4096, hipHostMallocDefault));
    uint8_t* dio;
    CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dio), hio, 0));
    auto spin = [&](uint32_t v) {
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != v) {
        }
    };
    run("launch_sync", [&](int) {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
        CHECK(hipStreamSynchronize(s));
    });
    run("launch_event", [&](int) {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
        CHECK(hipEventRecord(ev, s));
        CHECK(hipEventSynchronize(ev));
    });
    run("launch_query", [&](int) {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
        hipError_t e;
        while ((e = hipStreamQuery(s)) == hipErrorNotReady) {
        }
        CHECK(e);
    });
    run("launch_evquery", [&](int) {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
        CHECK(hipEventRecord(ev, s));
        hipError_t e;
        while ((e = hipEventQuery(ev)) == hipErrorNotReady) {
        }
        CHECK(e);
    });
    run("launch_flag", [&](int i) {
        hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, s, dflag, uint32_t(i + 1));
        spin(uint32_t(i + 1));
    });
    CHECK(hipStreamSynchronize(s));
    run("zc_sync", [&](int) {
        hipLaunchKernelGGL(k_zc, dim3(1), dim3(256), 0, s, (const u32x4*)dio, (u32x4*)(dio + 10 * 4096),
                           (volatile uint32_t*)nullptr, 0u);
        CHECK(hipStreamSynchronize(s));
    });
    run("zc_query", [&](int) {
        hipLaunchKernelGGL(k_zc, dim3(1), dim3(256), 0, s, (const u32x4*)dio, (u32x4*)(dio + 10 * 4096),
                           (volatile uint32_t*)nullptr, 0u);
        hipError_t e;
        while ((e = hipStreamQuery(s)) == hipErrorNotReady) {
        }
        CHECK(e);
    });
    run("zc_flag", [&](int i) {
        hipLaunchKernelGGL(k_zc, dim3(1), dim3(256), 0, s, (const u32x4*)dio, (u32x4*)(dio + 10 * 4096),
                           (volatile uint32_t*)dflag, uint32_t(1000000 + i));
        spin(uint32_t(1000000 + i));
    });
    CHECK(hipStreamSynchronize(s));
    {
        std::vector<double> us;
        for (int i = 0; i < 2000; ++i) {
            auto t0 = clk::now();
            hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
            us.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
            if (i % 64 == 63) CHECK(hipStreamSynchronize(s));
        }
        CHECK(hipStreamSynchronize(s));
        std::sort(us.begin(), us.end());
        printf("{\"case\": \"launch_only\", \"us_p50\": %.2f, \"us_p10\": %.2f, \"us_p90\": %.2f}\n", us[1000], us[200],
               us[1800]);
    }
    return 0;
}

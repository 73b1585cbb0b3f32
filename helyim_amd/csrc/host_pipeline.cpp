// Host-memory stripe batches through the GPU: the path helyim actually runs
// (shard bytes start and end in host memory: .dat pages / shard files,
// helyim-ec/src/encoder.rs:169-195, 263-304). Chunks of stripes are pipelined
// over kDepth HIP streams, each with its own device slot, so the H2D copy of
// chunk i+1, the kernel of chunk i and the D2H copy of chunk i-1 overlap
// (PCIe Gen5 x16 is full duplex; the copy engines run beside the kernel).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>

#include "hec_internal.hpp"

namespace hec {
namespace {

constexpr int kDepth = 3;
constexpr uint64_t kChunkBytes = 96ull << 20;  // target bytes of one chunk's 14 shards

struct Pipeline {
    std::mutex mu;
    hipStream_t streams[kDepth] = {};
    uint8_t* slot[kDepth] = {};
    uint32_t* mask_dev[kDepth] = {};
    uint32_t* mask_host[kDepth] = {};  // pinned staging for per-chunk masks
    size_t slot_cap = 0, mask_cap = 0;
    // pinned staging for pageable callers: two slots the kernels code in place
    uint8_t* hslot[2] = {};
    hipEvent_t hdone[2] = {};
    size_t hslot_cap = 0;
    int reserve_host(size_t bytes) {
        if (!hdone[0])
            for (auto& e : hdone) HEC_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        if (bytes <= hslot_cap) return HEC_OK;
        for (auto& h : hslot) {
            if (h) HEC_HIP(hipHostFree(h));
            h = nullptr;
        }
        hslot_cap = 0;
        for (auto& h : hslot) HEC_TRY(pinned_alloc(reinterpret_cast<void**>(&h), bytes));
        hslot_cap = bytes;
        return HEC_OK;
    }
    int init() { return HEC_OK; }  // streams and slots are made on first use (reserve)
    // Staging bytes held (pinned host, device).
    uint64_t pinned_bytes() const {
        return (hslot[0] ? 2 * hslot_cap : 0) + (mask_host[0] ? uint64_t(kDepth) * mask_cap * 4 : 0);
    }
    uint64_t device_bytes() const {
        return (slot[0] ? uint64_t(kDepth) * slot_cap : 0) + (mask_dev[0] ? uint64_t(kDepth) * mask_cap * 4 : 0);
    }
    // Free the large staging (the pageable path's pinned slots and the copy
    // path's device slots); streams, events and mask words stay. The next
    // call on this pipeline reserves again.
    void trim() {  // (the lease has drained the streams)
        for (auto& h : hslot) {
            if (h) (void)hipHostFree(h);
            h = nullptr;
        }
        hslot_cap = 0;
        for (auto& d : slot) {
            if (d) (void)hipFree(d);
            d = nullptr;
        }
        slot_cap = 0;
    }
    ~Pipeline() {
        for (auto& h : hslot) (void)hipHostFree(h);
        for (auto& e : hdone)
            if (e) (void)hipEventDestroy(e);
        for (int i = 0; i < kDepth; ++i) {
            (void)hipFree(slot[i]);
            (void)hipFree(mask_dev[i]);
            (void)hipHostFree(mask_host[i]);
            if (streams[i]) (void)hipStreamDestroy(streams[i]);
        }
    }
    int reserve(size_t slot_bytes, size_t n_masks) {
        if (!streams[0])
            for (int i = 0; i < kDepth; ++i) HEC_HIP(hipStreamCreateWithFlags(&streams[i], hipStreamNonBlocking));
        if (slot_bytes > slot_cap) {
            for (int i = 0; i < kDepth; ++i) {
                if (slot[i]) HEC_HIP(hipFree(slot[i]));
                slot[i] = nullptr;
            }
            slot_cap = 0;
            for (int i = 0; i < kDepth; ++i) HEC_HIP(hipMalloc(reinterpret_cast<void**>(&slot[i]), slot_bytes));
            slot_cap = slot_bytes;
        }
        if (n_masks > mask_cap) {
            for (int i = 0; i < kDepth; ++i) {
                if (mask_dev[i]) HEC_HIP(hipFree(mask_dev[i]));
                if (mask_host[i]) HEC_HIP(hipHostFree(mask_host[i]));
                mask_dev[i] = mask_host[i] = nullptr;
            }
            mask_cap = 0;
            for (int i = 0; i < kDepth; ++i) {
                HEC_HIP(hipMalloc(reinterpret_cast<void**>(&mask_dev[i]), n_masks * 4));
                HEC_TRY(pinned_alloc(reinterpret_cast<void**>(&mask_host[i]), n_masks * 4));
            }
            mask_cap = n_masks;
        }
        return HEC_OK;
    }
};

// Per-device pool of pipelines (SlotPool, hec_internal.hpp): concurrent host
// batches on one device -- other threads, or two ranges of one multi-device
// call on the same GPU -- each lease their own streams and slots. Up to
// kScratchSlots (8) pipelines exist per device, but only the first
// kWarmSlots (2) keep their staging between calls: a pipeline created by a
// burst of concurrent calls frees its large buffers when its call ends
// (PipelineLease), so the steady footprint per device is that of two
// pipelines (INTEGRATION.md §5 states the worst case).
std::mutex& pipeline_reg_mu() {
    static std::mutex* m = new std::mutex();
    return *m;
}
std::map<int, std::unique_ptr<SlotPool<Pipeline>>>& pipeline_reg() {
    static auto* reg = new std::map<int, std::unique_ptr<SlotPool<Pipeline>>>();  // process lifetime
    return *reg;
}

struct PipelineLease {
    Lease<Pipeline> lease;
    bool trim_after = false;
    Pipeline* operator->() const { return lease.sc; }
    ~PipelineLease() {  // still holding the pipeline's mutex
        if (!lease.sc) return;
        // Host batches code caller memory in place (zero copy) or copy into
        // it: an error return between enqueues must not leave that work in
        // flight for the caller's freed buffers (StreamDrain's rule). After
        // a successful call every stream is idle already.
        for (auto st : lease.sc->streams)
            if (st && hipStreamSynchronize(st) != hipSuccess) (void)hipGetLastError();
        if (trim_after) lease.sc->trim();
    }
};

int lease_pipeline(PipelineLease& out) {
    int dev;
    int rc = current_device(&dev);
    if (rc) return rc;
    SlotPool<Pipeline>* pool;
    {
        std::lock_guard<std::mutex> lk(pipeline_reg_mu());
        auto& p = pipeline_reg()[dev];
        if (!p) p.reset(new SlotPool<Pipeline>());
        pool = p.get();
    }
    if ((rc = pool->lease(out.lease))) return rc;
    out.trim_after = out.lease.index >= kWarmSlots;
    return HEC_OK;
}

// Copy `rows` rows of `width` bytes with pitches (2D; 1D when both are dense).
hipError_t copy2d(void* dst, uint64_t dpitch, const void* src, uint64_t spitch, uint64_t width, uint64_t rows,
                  hipMemcpyKind kind, hipStream_t s) {
    if (rows == 0 || width == 0) return hipSuccess;
    if (rows == 1 || (dpitch == width && spitch == width))
        return hipMemcpyAsync(dst, src, width * rows, kind, s);
    return hipMemcpy2DAsync(dst, dpitch, src, spitch, width, rows, kind, s);
}

// Zero-copy: pinned host memory that the GPU can address directly
// (hipHostMalloc / torch pin_memory) is handed to the kernel as is, so the
// kernel's loads and stores cross PCIe themselves -- no staging slots, no SDMA
// copies, both directions at once. Measured 51 GiB/s of data encoded vs 41-44
// for the copy pipeline (profiles/r02/HISTORY.md "host path"). The whole
// [p, p + span) must be one registered host range; anything else (pageable
// memory, device memory, a range running past the allocation) takes the copy
// pipeline. hec_set_host_zero_copy(0) disables it (the CUs then stay free
// while SDMA engines move the bytes).
bool host_device_view(const void* p, uint64_t span, uint8_t** dev) {
    if (!zero_copy_enabled() || span == 0) return false;
    hipPointerAttribute_t a{}, b{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    const void* last = static_cast<const uint8_t*>(p) + (span - 1);
    if (hipPointerGetAttributes(&b, last) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    if (a.type != hipMemoryTypeHost || b.type != hipMemoryTypeHost || !a.devicePointer || !b.devicePointer)
        return false;
    if (static_cast<uint8_t*>(b.devicePointer) - static_cast<uint8_t*>(a.devicePointer) != int64_t(span - 1))
        return false;
    *dev = static_cast<uint8_t*>(a.devicePointer);
    return true;
}

// bytes from the first to the last byte touched by a strided batch
uint64_t batch_span(uint64_t stripe_stride, uint64_t shard_stride, uint32_t shards, uint64_t len, uint32_t stripes) {
    return uint64_t(stripes - 1) * stripe_stride + uint64_t(shards - 1) * shard_stride + len;
}

// Test hook: HEC_TEST_HOST_FAIL_AFTER_CHUNK=i fails a copy-pipeline encode
// right after queueing chunk i's kernel, so a test can check that the work
// queued before an error return has landed when the call returns
// (tests/test_gpu_host_batch.py). Read per call; -1 = off.
int forced_failure_chunk() {
    const char* v = std::getenv("HEC_TEST_HOST_FAIL_AFTER_CHUNK");
    return v && *v ? std::atoi(v) : -1;
}

uint32_t chunk_stripes(uint64_t shard_len, int n, uint32_t n_stripes) {
    uint64_t c = std::max<uint64_t>(1, kChunkBytes / (uint64_t(n) * shard_len));
    return uint32_t(std::min<uint64_t>(c, n_stripes));
}

// One host batch over a device set (contiguous stripe ranges
// per GPU). Range r = stripes [S*r/R, S*(r+1)/R) of R = min(n_devices, S)
// ranges runs on devices[r] from its own host thread: hipSetDevice, CPUs bound
// to that GPU's NUMA node (hec_bind_thread_to_device), and the single-device
// host path, which leases its own pipeline (streams, device slots, pinned
// staging on that node). A device listed twice runs two ranges concurrently on
// two pipelines. Every range runs to its end; the call returns the status of
// the first failing range in list order (its detail prefixed with the range).
constexpr size_t kMaxDeviceRanges = 256;
int run_device_ranges(const int* devices, size_t n_devices, uint32_t n_stripes,
                      const std::function<int(uint32_t s0, uint32_t count, size_t range)>& fn) {
    if (!devices || n_devices == 0) return fail(HEC_ERR_INVALID_ARGUMENT, "empty device list");
    if (n_devices > kMaxDeviceRanges)  // one host thread per entry
        return fail(HEC_ERR_INVALID_ARGUMENT, "more than " + std::to_string(kMaxDeviceRanges) + " device entries");
    int count = 0;
    HEC_TRY(hec_device_count(&count));
    for (size_t r = 0; r < n_devices; ++r)
        if (devices[r] < 0 || devices[r] >= count)
            return fail(HEC_ERR_INVALID_ARGUMENT,
                        "device " + std::to_string(devices[r]) + " of " + std::to_string(count) + " in the list");
    if (n_stripes == 0) return HEC_OK;
    // (Each device's host worker pools bind their workers to that GPU's node,
    // so a range's staging copies run next to its pinned memory.)
    const size_t R = std::min<size_t>(n_devices, n_stripes);
    std::vector<int> rcs(R, HEC_OK);
    std::vector<std::string> details(R);
    std::vector<ErrorValues> values(R);
    std::vector<std::thread> th;
    th.reserve(R);
    try {
        for (size_t r = 0; r < R; ++r) {
            const uint32_t s0 = uint32_t(uint64_t(n_stripes) * r / R);
            const uint32_t s1 = uint32_t(uint64_t(n_stripes) * (r + 1) / R);
            th.emplace_back([&, r, s0, s1] {
                const hipError_t e = hipSetDevice(devices[r]);
                if (e != hipSuccess) {
                    rcs[r] = hip_fail(e, "hipSetDevice");
                } else {
                    (void)hec_bind_thread_to_device(devices[r], nullptr);  // placement only: no-op when unknown
                    rcs[r] = fn(s0, s1 - s0, r);
                }
                if (rcs[r]) {
                    details[r] = hec_last_error_detail();
                    values[r] = last_error_values();
                }
            });
        }
    } catch (const std::exception& ex) {  // no thread for a range: nothing escapes the C ABI
        for (size_t r = th.size(); r < R; ++r) {
            rcs[r] = HEC_ERR_OUT_OF_MEMORY;
            details[r] = std::string("no host thread for the range: ") + ex.what();
        }
    }
    for (auto& t : th) t.join();
    for (size_t r = 0; r < R; ++r)
        if (rcs[r]) {
            const uint32_t s0 = uint32_t(uint64_t(n_stripes) * r / R);
            const uint32_t s1 = uint32_t(uint64_t(n_stripes) * (r + 1) / R);
            return fail_with(rcs[r],
                             "device " + std::to_string(devices[r]) + " stripes [" + std::to_string(s0) + ", " +
                                 std::to_string(s1) + "): " + details[r],
                             values[r]);
        }
    return HEC_OK;
}

}  // namespace
}  // namespace hec

using namespace hec;

extern "C" {

int hec_host_encode_batch(const hec_rs_t* rs, const uint8_t* h_data, uint64_t data_stripe_stride,
                          uint64_t data_shard_stride, uint8_t* h_parity, uint64_t parity_stripe_stride,
                          uint64_t parity_shard_stride, uint64_t shard_len, uint32_t n_stripes) {
    if (!rs || !h_data || !h_parity) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    if (shard_len == 0) return fail(HEC_ERR_EMPTY_SHARD, "");
    if (n_stripes == 0) return HEC_OK;
    int rc;
    if ((rc = check_strided("data", uint32_t(rs->k), data_stripe_stride, data_shard_stride, shard_len, n_stripes)) ||
        (rc = check_strided("parity", uint32_t(rs->m), parity_stripe_stride, parity_shard_stride, shard_len,
                            n_stripes)))
        return rc;
    GeomDevice* gd;
    if ((rc = geom_device(rs, &gd))) return rc;
    PipelineLease lease;
    if ((rc = lease_pipeline(lease))) return rc;
    Pipeline* p = lease.lease.sc;
    const int k = rs->k, m = rs->m;
    uint8_t *zd, *zp;
    if (host_device_view(h_data, batch_span(data_stripe_stride, data_shard_stride, k, shard_len, n_stripes), &zd) &&
        host_device_view(h_parity, batch_span(parity_stripe_stride, parity_shard_stride, m, shard_len, n_stripes),
                         &zp)) {
        if ((rc = p->reserve(0, 1))) return rc;
        if ((rc = run_apply(gd->encode, uint32_t(k), zd, data_stripe_stride, data_shard_stride, zp,
                            parity_stripe_stride, parity_shard_stride, shard_len, n_stripes, nullptr, nullptr,
                            p->streams[0], nullptr, /*over_pcie=*/true)))
            return rc;
        HEC_HIP(hipStreamSynchronize(p->streams[0]));
        return HEC_OK;
    }
    const uint64_t Lp = (shard_len + 255) / 256 * 256;  // device shard pitch
    const uint32_t C = chunk_stripes(Lp, rs->n, n_stripes);
    const uint64_t dstripe = uint64_t(rs->n) * Lp;
    if (zero_copy_enabled()) {
        // Pageable memory: chunks are copied into two pinned slots on the host
        // pool and coded in place by the zero-copy kernel; packing chunk i+1
        // and unpacking chunk i-1 overlap the kernel of chunk i.
        if ((rc = p->reserve(0, 1)) || (rc = p->reserve_host(size_t(C) * dstripe))) return rc;
        uint8_t* zs[2] = {pinned_device_ptr(p->hslot[0]), pinned_device_ptr(p->hslot[1])};
        if (zs[0] && zs[1]) {
            hipStream_t st = p->streams[0];
            auto unpack = [&](uint32_t s0, uint32_t c, int q) {
                parallel_for(size_t(c) * m, uint64_t(c) * m * shard_len, [&](size_t t) {
                    const uint32_t s = uint32_t(t / m);
                    const int j = int(t % m);
                    std::memcpy(h_parity + (s0 + s) * parity_stripe_stride + j * parity_shard_stride,
                                p->hslot[q] + s * dstripe + uint64_t(k + j) * Lp, shard_len);
                });
            };
            uint32_t prev_s0 = 0, prev_c = 0;
            for (uint32_t s0 = 0, it = 0; s0 < n_stripes; s0 += C, ++it) {
                const uint32_t c = std::min(C, n_stripes - s0);
                const int q = int(it % 2);
                uint8_t* h = p->hslot[q];
                parallel_for(size_t(c) * k, uint64_t(c) * k * shard_len, [&](size_t t) {
                    const uint32_t s = uint32_t(t / k);
                    const int i = int(t % k);
                    std::memcpy(h + s * dstripe + uint64_t(i) * Lp,
                                h_data + (s0 + s) * data_stripe_stride + i * data_shard_stride, shard_len);
                });
                if ((rc = run_apply(gd->encode, uint32_t(k), zs[q], dstripe, Lp, zs[q] + uint64_t(k) * Lp, dstripe,
                                    Lp, (shard_len + 15) / 16 * 16, c, nullptr, nullptr, st, nullptr,
                                    /*over_pcie=*/true)))
                    return rc;
                HEC_HIP(hipEventRecord(p->hdone[q], st));
                if (it > 0) {  // chunk it-1 (other slot) is done or nearly: hand its parity back
                    HEC_HIP(hipEventSynchronize(p->hdone[1 - q]));
                    unpack(prev_s0, prev_c, 1 - q);
                }
                prev_s0 = s0, prev_c = c;
            }
            const int last = int(((n_stripes + C - 1) / C - 1) % 2);
            HEC_HIP(hipEventSynchronize(p->hdone[last]));
            unpack(prev_s0, prev_c, last);
            return HEC_OK;
        }
    }
    if ((rc = p->reserve(size_t(C) * rs->n * Lp, 1))) return rc;
    const int fail_at = forced_failure_chunk();
    for (uint32_t s0 = 0, it = 0; s0 < n_stripes; s0 += C, ++it) {
        const uint32_t c = std::min(C, n_stripes - s0);
        const int q = int(it % kDepth);
        hipStream_t st = p->streams[q];
        uint8_t* d = p->slot[q];
        for (uint32_t s = 0; s < c; ++s)  // data shards of stripe s -> [s][0..k)
            HEC_HIP(copy2d(d + s * dstripe, Lp, h_data + (s0 + s) * data_stripe_stride, data_shard_stride,
                           shard_len, uint64_t(k), hipMemcpyHostToDevice, st));
        // len rounded to 16: the pad bytes of the device pitch are computed but never copied back
        if ((rc = run_apply(gd->encode, uint32_t(k), d, dstripe, Lp, d + uint64_t(k) * Lp, dstripe, Lp,
                            (shard_len + 15) / 16 * 16, c, nullptr, nullptr, st)))
            return rc;
        if (int(it) == fail_at) return fail(HEC_ERR_HIP, "test hook: failure after chunk " + std::to_string(it));
        for (uint32_t s = 0; s < c; ++s)
            HEC_HIP(copy2d(h_parity + (s0 + s) * parity_stripe_stride, parity_shard_stride,
                           d + s * dstripe + uint64_t(k) * Lp, Lp, shard_len, uint64_t(m), hipMemcpyDeviceToHost, st));
    }
    for (int q = 0; q < kDepth; ++q) HEC_HIP(hipStreamSynchronize(p->streams[q]));
    return HEC_OK;
}

int hec_host_reconstruct_batch(const hec_rs_t* rs, uint8_t* h_shards, uint64_t stripe_stride, uint64_t shard_stride,
                               uint64_t shard_len, uint32_t n_stripes, const uint32_t* h_present_masks,
                               uint32_t* n_bad_stripes) {
    if (!rs || !h_shards || !h_present_masks) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    if (shard_len == 0) return fail(HEC_ERR_EMPTY_SHARD, "");
    if (n_bad_stripes) *n_bad_stripes = 0;
    if (n_stripes == 0) return HEC_OK;
    int rc;
    if ((rc = check_strided("shards", uint32_t(rs->n), stripe_stride, shard_stride, shard_len, n_stripes))) return rc;
    GeomDevice* gd;
    if ((rc = geom_device(rs, &gd))) return rc;
    PipelineLease lease;
    if ((rc = lease_pipeline(lease))) return rc;
    Pipeline* p = lease.lease.sc;
    const int k = rs->k, n = rs->n;
    const uint32_t full = n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1);
    uint8_t* zs;
    if (host_device_view(h_shards, batch_span(stripe_stride, shard_stride, n, shard_len, n_stripes), &zs)) {
        // masks to the device (the caller's array may be pageable), then one
        // decode over the pinned host shards in place
        if ((rc = p->reserve(0, n_stripes))) return rc;
        if ((rc = ensure_dense_decode(rs, gd, p->streams[0]))) return rc;
        uint32_t bad = 0;
        for (uint32_t s = 0; s < n_stripes; ++s) {
            const uint32_t mask = h_present_masks[s] & full;
            p->mask_host[0][s] = mask;
            bad += __builtin_popcount(mask) < k ? 1u : 0u;
        }
        HEC_HIP(hipMemcpyAsync(p->mask_dev[0], p->mask_host[0], size_t(n_stripes) * 4, hipMemcpyHostToDevice,
                               p->streams[0]));
        if ((rc = run_apply(gd->decode_dense, uint32_t(k), zs, stripe_stride, shard_stride, zs, stripe_stride,
                            shard_stride, shard_len, n_stripes, p->mask_dev[0], nullptr, p->streams[0])))
            return rc;
        HEC_HIP(hipStreamSynchronize(p->streams[0]));
        if (n_bad_stripes) *n_bad_stripes = bad;
        return HEC_OK;
    }
    const uint64_t Lp = (shard_len + 255) / 256 * 256;
    const uint32_t C = chunk_stripes(Lp, n, n_stripes);
    const uint64_t dstripe = uint64_t(n) * Lp;
    if (zero_copy_enabled()) {
        // Pageable memory: the first k present shards of each stripe are copied
        // into two pinned slots on the host pool, decoded in place there by the
        // zero-copy kernel, and only the erased shards are copied back; chunk
        // i+1's copies in and chunk i-1's copies out overlap chunk i's kernel.
        if ((rc = p->reserve(0, C)) || (rc = p->reserve_host(size_t(C) * dstripe))) return rc;
        if ((rc = ensure_dense_decode(rs, gd, p->streams[0]))) return rc;
        uint8_t* hz[2] = {pinned_device_ptr(p->hslot[0]), pinned_device_ptr(p->hslot[1])};
        uint32_t* zm[2] = {reinterpret_cast<uint32_t*>(pinned_device_ptr(p->mask_host[0])),
                           reinterpret_cast<uint32_t*>(pinned_device_ptr(p->mask_host[1]))};
        if (hz[0] && hz[1] && zm[0] && zm[1]) {
            hipStream_t st = p->streams[0];
            uint32_t bad = 0;
            auto unpack = [&](uint32_t s0, uint32_t c, int q) {
                parallel_for(size_t(c) * n, uint64_t(c) * 4 * shard_len, [&](size_t t) {
                    const uint32_t s = uint32_t(t / n);
                    const int i = int(t % n);
                    const uint32_t mask = p->mask_host[q][s];
                    if (__builtin_popcount(mask) < k || ((mask >> i) & 1)) return;
                    std::memcpy(h_shards + (s0 + s) * stripe_stride + uint64_t(i) * shard_stride,
                                p->hslot[q] + s * dstripe + uint64_t(i) * Lp, shard_len);
                });
            };
            uint32_t prev_s0 = 0, prev_c = 0;
            for (uint32_t s0 = 0, it = 0; s0 < n_stripes; s0 += C, ++it) {
                const uint32_t c = std::min(C, n_stripes - s0);
                const int q = int(it % 2);
                for (uint32_t s = 0; s < c; ++s) {
                    const uint32_t mask = h_present_masks[s0 + s] & full;
                    p->mask_host[q][s] = mask;
                    bad += __builtin_popcount(mask) < k ? 1u : 0u;
                }
                uint8_t* h = p->hslot[q];
                parallel_for(size_t(c) * n, uint64_t(c) * k * shard_len, [&](size_t t) {
                    const uint32_t s = uint32_t(t / n);
                    const int i = int(t % n);
                    const uint32_t mask = p->mask_host[q][s];
                    if (__builtin_popcount(mask) < k || __builtin_popcount(mask) == n || !((mask >> i) & 1)) return;
                    if (__builtin_popcount(mask & ((1u << i) - 1)) >= k) return;  // only the first k present
                    std::memcpy(h + s * dstripe + uint64_t(i) * Lp,
                                h_shards + (s0 + s) * stripe_stride + uint64_t(i) * shard_stride, shard_len);
                });
                if ((rc = run_apply(gd->decode_dense, uint32_t(k), hz[q], dstripe, Lp, hz[q], dstripe, Lp,
                                    (shard_len + 15) / 16 * 16, c, zm[q], nullptr, st)))
                    return rc;
                HEC_HIP(hipEventRecord(p->hdone[q], st));
                if (it > 0) {
                    HEC_HIP(hipEventSynchronize(p->hdone[1 - q]));
                    unpack(prev_s0, prev_c, 1 - q);
                }
                prev_s0 = s0, prev_c = c;
            }
            const int last = int(((n_stripes + C - 1) / C - 1) % 2);
            HEC_HIP(hipEventSynchronize(p->hdone[last]));
            unpack(prev_s0, prev_c, last);
            if (n_bad_stripes) *n_bad_stripes = bad;
            return HEC_OK;
        }
    }
    if ((rc = p->reserve(size_t(C) * n * Lp, C))) return rc;
    if ((rc = ensure_dense_decode(rs, gd, p->streams[0]))) return rc;
    uint32_t bad = 0;
    for (uint32_t s0 = 0, it = 0; s0 < n_stripes; s0 += C, ++it) {
        const uint32_t c = std::min(C, n_stripes - s0);
        const int q = int(it % kDepth);
        hipStream_t st = p->streams[q];
        uint8_t* d = p->slot[q];
        // the staging of this slot was last read by the copy issued kDepth chunks ago
        HEC_HIP(hipStreamSynchronize(st));
        for (uint32_t s = 0; s < c; ++s) {
            const uint32_t mask = h_present_masks[s0 + s] & full;
            p->mask_host[q][s] = mask;
            const int present = __builtin_popcount(mask);
            if (present < k) {
                ++bad;
                continue;
            }
            if (present == n) continue;
            // H2D only the first k present shards (the ones the decode reads),
            // merged into runs of adjacent shard ids.
            int used = 0;
            for (int i = 0; i < n && used < k;) {
                if (!((mask >> i) & 1)) {
                    ++i;
                    continue;
                }
                int j = i;
                while (j < n && ((mask >> j) & 1) && used + (j - i) < k) ++j;
                HEC_HIP(copy2d(d + s * dstripe + uint64_t(i) * Lp, Lp,
                               h_shards + (s0 + s) * stripe_stride + uint64_t(i) * shard_stride, shard_stride,
                               shard_len, uint64_t(j - i), hipMemcpyHostToDevice, st));
                used += j - i;
                i = j;
            }
        }
        HEC_HIP(hipMemcpyAsync(p->mask_dev[q], p->mask_host[q], c * 4, hipMemcpyHostToDevice, st));
        if ((rc = run_apply(gd->decode_dense, uint32_t(k), d, dstripe, Lp, d, dstripe, Lp,
                            (shard_len + 15) / 16 * 16, c, p->mask_dev[q], nullptr, st)))
            return rc;
        for (uint32_t s = 0; s < c; ++s) {
            const uint32_t mask = p->mask_host[q][s];
            if (__builtin_popcount(mask) < k) continue;
            for (int i = 0; i < n;) {  // D2H the erased shards, merged into runs
                if ((mask >> i) & 1) {
                    ++i;
                    continue;
                }
                int j = i;
                while (j < n && !((mask >> j) & 1)) ++j;
                HEC_HIP(copy2d(h_shards + (s0 + s) * stripe_stride + uint64_t(i) * shard_stride, shard_stride,
                               d + s * dstripe + uint64_t(i) * Lp, Lp, shard_len, uint64_t(j - i),
                               hipMemcpyDeviceToHost, st));
                i = j;
            }
        }
    }
    for (int q = 0; q < kDepth; ++q) HEC_HIP(hipStreamSynchronize(p->streams[q]));
    if (n_bad_stripes) *n_bad_stripes = bad;
    return HEC_OK;
}

int hec_host_encode_batch_multi(const hec_rs_t* rs, const int* devices, size_t n_devices, const uint8_t* h_data,
                                uint64_t data_stripe_stride, uint64_t data_shard_stride, uint8_t* h_parity,
                                uint64_t parity_stripe_stride, uint64_t parity_shard_stride, uint64_t shard_len,
                                uint32_t n_stripes) {
    if (!rs || !h_data || !h_parity) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    if (shard_len == 0) return fail(HEC_ERR_EMPTY_SHARD, "");
    int rc;
    if ((rc = check_strided("data", uint32_t(rs->k), data_stripe_stride, data_shard_stride, shard_len, n_stripes)) ||
        (rc = check_strided("parity", uint32_t(rs->m), parity_stripe_stride, parity_shard_stride, shard_len,
                            n_stripes)))
        return rc;
    return run_device_ranges(devices, n_devices, n_stripes, [&](uint32_t s0, uint32_t c, size_t) {
        return hec_host_encode_batch(rs, h_data + s0 * data_stripe_stride, data_stripe_stride, data_shard_stride,
                                     h_parity + s0 * parity_stripe_stride, parity_stripe_stride, parity_shard_stride,
                                     shard_len, c);
    });
}

int hec_host_reconstruct_batch_multi(const hec_rs_t* rs, const int* devices, size_t n_devices, uint8_t* h_shards,
                                     uint64_t stripe_stride, uint64_t shard_stride, uint64_t shard_len,
                                     uint32_t n_stripes, const uint32_t* h_present_masks, uint32_t* n_bad_stripes) {
    if (!rs || !h_shards || !h_present_masks) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    if (shard_len == 0) return fail(HEC_ERR_EMPTY_SHARD, "");
    if (n_bad_stripes) *n_bad_stripes = 0;
    int rc;
    if ((rc = check_strided("shards", uint32_t(rs->n), stripe_stride, shard_stride, shard_len, n_stripes))) return rc;
    std::vector<uint32_t> bad(std::max<size_t>(n_devices, 1), 0);
    rc = run_device_ranges(devices, n_devices, n_stripes, [&](uint32_t s0, uint32_t c, size_t r) {
        return hec_host_reconstruct_batch(rs, h_shards + s0 * stripe_stride, stripe_stride, shard_stride, shard_len, c,
                                          h_present_masks + s0, &bad[r]);
    });
    if (rc) return rc;
    if (n_bad_stripes)
        for (uint32_t b : bad) *n_bad_stripes += b;
    return HEC_OK;
}

int hec_host_zero_copy_view(const void* p, uint64_t bytes, int* zero_copy) {
    if (!zero_copy) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    *zero_copy = 0;
    if (!p || bytes == 0) return HEC_OK;
    int dev;
    int rc = current_device(&dev);
    if (rc) return rc;
    uint8_t* d = nullptr;
    *zero_copy = host_device_view(p, bytes, &d) ? 1 : 0;
    return HEC_OK;
}

int hec_host_staging_stats(int* n_pipelines, uint64_t* pinned_bytes, uint64_t* device_bytes) {
    int dev;
    int rc = current_device(&dev);
    if (rc) return rc;
    SlotPool<Pipeline>* pool = nullptr;
    {
        std::lock_guard<std::mutex> lk(pipeline_reg_mu());
        auto it = pipeline_reg().find(dev);
        if (it != pipeline_reg().end()) pool = it->second.get();
    }
    int n = 0;
    uint64_t pinned = 0, devb = 0;
    if (pool) {
        // Slots are never removed from a pool, so their addresses stay valid;
        // the pool mutex is held only to copy them, never while waiting on a
        // slot (that would stall every lease on the device behind one call).
        std::vector<Pipeline*> slots;
        {
            std::lock_guard<std::mutex> g(pool->mu);
            for (auto& sl : pool->slots) slots.push_back(sl.get());
        }
        for (Pipeline* sl : slots) {
            std::lock_guard<std::mutex> l(sl->mu);  // waits for a call in flight on it
            ++n;
            pinned += sl->pinned_bytes();
            devb += sl->device_bytes();
        }
    }
    if (n_pipelines) *n_pipelines = n;
    if (pinned_bytes) *pinned_bytes = pinned;
    if (device_bytes) *device_bytes = devb;
    return HEC_OK;
}

int hec_set_host_zero_copy(int on) {
    zero_copy_enabled() = on != 0;
    return HEC_OK;
}

}  // extern "C"

// Batched reconstruct of many small, independent stripes in one launch: the
// degraded-read path (helyim-store/src/erasure_coding/mod.rs:403-491 calls
// ReedSolomon::reconstruct once per needle interval, bytes to KiB each).
// Stripes are packed back to back into one pinned staging area, copied to the
// GPU once, decoded by rs104_ragged_kernel (one workgroup per 4 KiB chunk of
// each stripe, per-stripe length and erasure pattern), and copied back once.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <map>
#include <memory>
#include <thread>

#include "hec_internal.hpp"

namespace hec {
namespace {

struct RaggedScratch {
    std::mutex mu;
    hipStream_t stream = nullptr;
    hipEvent_t meta_free = nullptr;  // device-API calls: meta buffers reusable once this fires
    uint8_t* host = nullptr;
    uint8_t* dev = nullptr;
    size_t cap = 0;
    uint8_t* hmeta = nullptr;
    uint8_t* dmeta = nullptr;
    size_t mcap = 0;
    int reserve(size_t bytes, size_t meta) {
        if (!stream) HEC_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        if (bytes > cap && bytes > 0) {
            if (host) HEC_HIP(hipHostFree(host));
            if (dev) HEC_HIP(hipFree(dev));
            host = dev = nullptr;
            cap = 0;
            const size_t want = std::max(bytes, size_t(64) << 20);
            HEC_TRY(pinned_alloc(reinterpret_cast<void**>(&host), want));
            HEC_HIP(hipMalloc(reinterpret_cast<void**>(&dev), want));
            cap = want;
        }
        if (meta > mcap) {
            if (hmeta) HEC_HIP(hipHostFree(hmeta));
            if (dmeta) HEC_HIP(hipFree(dmeta));
            hmeta = dmeta = nullptr;
            mcap = 0;
            const size_t want = std::max(meta, size_t(1) << 20);
            HEC_TRY(pinned_alloc(reinterpret_cast<void**>(&hmeta), want));
            HEC_HIP(hipMalloc(reinterpret_cast<void**>(&dmeta), want));
            mcap = want;
        }
        return HEC_OK;
    }
};

int ragged_scratch(RaggedScratch** out) {
    static std::mutex mu;
    static std::map<int, RaggedScratch*>* reg = new std::map<int, RaggedScratch*>();  // process lifetime
    int dev;
    int rc = current_device(&dev);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(mu);
    auto& p = (*reg)[dev];
    if (!p) p = new RaggedScratch();
    *out = p;
    return HEC_OK;
}

}  // namespace

int compact_reconstruct_104(const hec_rs* rs, const std::vector<CompactJob>& jobs, const CompactFill& fill,
                            const CompactTake& take, bool io_bound_fill) {
    const int k = rs->k, n = rs->n;
    struct Lay {
        uint64_t Lp, off, out_off;
    };
    std::vector<Lay> lay(jobs.size());
    uint64_t total = 0;
    for (size_t j = 0; j < jobs.size(); ++j) {
        if (__builtin_popcount(jobs[j].mask) < k || jobs[j].len == 0 || jobs[j].len > 0xFFFFFFFFull)
            return fail(HEC_ERR_INVALID_ARGUMENT, "compact job without k survivors");
        lay[j].Lp = (jobs[j].len + 15) / 16 * 16;
        lay[j].off = total;
        total += (uint64_t(k) * lay[j].Lp + 255) / 256 * 256;  // compact inputs: the first k present shards
    }
    if (jobs.empty()) return HEC_OK;
    const uint64_t in_total = total;
    for (size_t j = 0; j < jobs.size(); ++j) {  // compact outputs: the erased shards, ascending
        lay[j].out_off = total;
        total += (uint64_t(n - __builtin_popcount(jobs[j].mask)) * lay[j].Lp + 255) / 256 * 256;
    }
    GeomDevice* gd;
    int rc = geom_device(rs, &gd);
    if (rc) return rc;
    RaggedScratch* sc;
    if ((rc = ragged_scratch(&sc))) return rc;
    std::lock_guard<std::mutex> lk(sc->mu);
    std::vector<RaggedItem> items(jobs.size());
    std::vector<uint32_t> block_item;
    for (size_t j = 0; j < jobs.size(); ++j) {
        const uint32_t chunks = uint32_t((jobs[j].len + 4095) / 4096);
        items[j] = RaggedItem{lay[j].off, lay[j].Lp, uint32_t(jobs[j].len), jobs[j].mask,
                              uint32_t(block_item.size()), 0, lay[j].out_off};
        block_item.insert(block_item.end(), chunks, uint32_t(j));
    }
    const size_t items_bytes = items.size() * sizeof(RaggedItem);
    const size_t meta = (items_bytes + 255) / 256 * 256 + block_item.size() * 4;
    if ((rc = sc->reserve(total, meta))) return rc;
    if ((rc = ensure_dense_decode(rs, gd, sc->stream))) return rc;
    // survivors the decode reads (the first k present shards) -> slots 0..k-1
    std::atomic<int> first_err{HEC_OK};
    // one task per (job, slot): a single large interval's 10 survivor reads run
    // in parallel too
    auto fill_one = [&](size_t t) {
        const size_t j = t / size_t(k);
        const int want = int(t % size_t(k));
        int used = 0;
        for (int i = 0; i < n; ++i)
            if ((jobs[j].mask >> i) & 1) {
                if (used == want) {
                    const int r = fill(j, used, i, sc->host + lay[j].off + used * lay[j].Lp);
                    if (r) {
                        int expect = HEC_OK;
                        first_err.compare_exchange_strong(expect, r);
                    }
                    return;
                }
                ++used;
            }
    };
    if (io_bound_fill)
        parallel_io_for(jobs.size() * size_t(k), in_total, fill_one);
    else
        parallel_for(jobs.size() * size_t(k), in_total, fill_one);
    if (first_err.load()) return first_err.load();
    std::memcpy(sc->hmeta, items.data(), items_bytes);
    const size_t map_off = (items_bytes + 255) / 256 * 256;
    std::memcpy(sc->hmeta + map_off, block_item.data(), block_item.size() * 4);
    HEC_HIP(hipMemcpyAsync(sc->dmeta, sc->hmeta, meta, hipMemcpyHostToDevice, sc->stream));
    // zero-copy: the kernel reads the packed survivors and writes the rebuilt
    // shards in the pinned staging itself (no H2D / D2H of the payload)
    uint8_t* zh = zero_copy_enabled() ? pinned_device_ptr(sc->host) : nullptr;
    if (!zh) HEC_HIP(hipMemcpyAsync(sc->dev, sc->host, in_total, hipMemcpyHostToDevice, sc->stream));
    RaggedArgs ra{};
    ra.base = zh ? zh : sc->dev;
    ra.items = reinterpret_cast<const RaggedItem*>(sc->dmeta);
    ra.block_item = reinterpret_cast<const uint32_t*>(sc->dmeta + map_off);
    ra.n_blocks = uint32_t(block_item.size());
    ra.tabs = gd->decode_dense.tabs;
    ra.lut = gd->decode_dense.lut;
    ra.compact = 1;
    HEC_HIP(launch_rs104_ragged(ra, true, sc->stream));
    if (!zh)
        HEC_HIP(hipMemcpyAsync(sc->host + in_total, sc->dev + in_total, total - in_total, hipMemcpyDeviceToHost,
                               sc->stream));
    HEC_HIP(hipStreamSynchronize(sc->stream));
    // hand back the erased shards
    parallel_for(jobs.size(), total - in_total, [&](size_t j) {
        int r = 0;
        for (int i = 0; i < n; ++i)
            if (!((jobs[j].mask >> i) & 1)) take(j, i, sc->host + lay[j].out_off + uint64_t(r++) * lay[j].Lp);
    });
    return HEC_OK;
}

}  // namespace hec

using namespace hec;

extern "C" {

int hec_rs_reconstruct_batch(const hec_rs_t* rs, uint8_t* const* shards, const size_t* lens, const uint8_t* present,
                             size_t n_stripes, int data_only, size_t* bad_index) {
    if (!rs || (n_stripes && (!shards || !lens || !present))) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    const int k = rs->k, n = rs->n;
    if (bad_index) *bad_index = n_stripes;
    // 1. validate every stripe first (upstream reconstruct checks, per stripe)
    struct Active {
        size_t s;
        uint64_t L;
        uint32_t mask;
    };
    std::vector<Active> act;
    for (size_t s = 0; s < n_stripes; ++s) {
        const uint8_t* pr = present + s * n;
        uint64_t L = 0;
        int np = 0, err = HEC_OK;
        uint32_t mask = 0;
        for (int i = 0; i < n && !err; ++i) {
            if (!pr[i]) continue;
            const size_t li = lens[s * n + i];
            if (li == 0) err = HEC_ERR_EMPTY_SHARD;
            else if (np && li != L) err = HEC_ERR_INCORRECT_SHARD_SIZE;
            L = li;
            ++np;
            mask |= 1u << i;
        }
        if (!err && np < n && np < k) err = HEC_ERR_TOO_FEW_SHARDS_PRESENT;
        if (!err && np < n)
            for (int i = 0; i < n; ++i)
                if (!pr[i] && !(data_only && i >= k) && !shards[s * n + i])
                    err = fail(HEC_ERR_INVALID_ARGUMENT, "missing shard without a buffer");
        if (err) {
            if (bad_index) *bad_index = s;
            return err;
        }
        if (np == n) continue;  // upstream no-op
        act.push_back({s, L, mask});
    }
    if (act.empty()) return HEC_OK;

    // Other geometries: one host-API reconstruct per stripe (same kernels, generic path).
    if (!(k == 10 && rs->m == 4)) {
        for (const Active& a : act) {
            int rc = data_only ? hec_rs_reconstruct_data(rs, shards + a.s * n, lens + a.s * n, present + a.s * n, n)
                               : hec_rs_reconstruct(rs, shards + a.s * n, lens + a.s * n, present + a.s * n, n);
            if (rc) {
                if (bad_index) *bad_index = a.s;
                return rc;
            }
        }
        return HEC_OK;
    }

    std::vector<CompactJob> jobs(act.size());
    for (size_t j = 0; j < act.size(); ++j) jobs[j] = CompactJob{act[j].L, act[j].mask};
    return compact_reconstruct_104(
        rs, jobs,
        [&](size_t j, int, int shard, uint8_t* dst) {
            std::memcpy(dst, shards[act[j].s * n + shard], act[j].L);
            return HEC_OK;
        },
        [&](size_t j, int shard, const uint8_t* src) {
            if (!(data_only && shard >= k)) std::memcpy(shards[act[j].s * n + shard], src, act[j].L);
        });
}

}  // extern "C"

namespace hec {
namespace {

// Device-resident ragged batches: stripe descriptors come from the host, data
// stays in HBM. Descriptors -> RaggedItems + workgroup map in pinned staging,
// uploaded on the caller's stream ahead of the kernel.
int gpu_ragged(const hec_rs_t* rs, uint8_t* d_base, const hec_stripe_desc* descs, uint32_t n, bool decode,
               uint32_t* d_bad, hipStream_t stream) {
    if (!rs || !d_base || (n && !descs)) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    if (!(rs->k == 10 && rs->m == 4))
        return fail(HEC_ERR_INVALID_ARGUMENT, "ragged device batches are RS(10,4) only");
    std::vector<RaggedItem> items;
    std::vector<uint32_t> block_item;
    items.reserve(n);
    // encode of lengths that are all multiples of 8 KiB: the bit-sliced kernel
    const LaunchConfig cfg = launch_config();
    bool bitslice = !decode && cfg.bitslice != 0 && cfg.mode == 0;
    for (uint32_t j = 0; j < n && bitslice; ++j) bitslice = descs[j].shard_len % kBsChunk == 0;
    const uint32_t chunk_bytes = bitslice ? kBsChunk : 4096;
    for (uint32_t j = 0; j < n; ++j) {
        const hec_stripe_desc& d = descs[j];
        if (d.shard_len == 0) return fail(HEC_ERR_EMPTY_SHARD, "stripe " + std::to_string(j));
        if ((d.offset | d.shard_stride | uint64_t(reinterpret_cast<uintptr_t>(d_base))) % 16 != 0 ||
            d.shard_stride < d.shard_len)
            return fail(HEC_ERR_INVALID_ARGUMENT, "stripe " + std::to_string(j) +
                                                      ": offset/stride must be 16-byte aligned, stride >= len");
        // 64-bit: a shard_len near 2^32 must not wrap to 0 or 1 chunks
        const uint64_t chunks = (uint64_t(d.shard_len) + chunk_bytes - 1) / chunk_bytes;
        if (block_item.size() + chunks > UINT32_MAX)
            return fail(HEC_ERR_INVALID_ARGUMENT, "ragged batch above 2^32 workgroups");
        items.push_back(RaggedItem{d.offset, d.shard_stride, d.shard_len, d.present_mask,
                                   uint32_t(block_item.size()), 0, 0});
        block_item.insert(block_item.end(), chunks, j);
    }
    if (items.empty()) return HEC_OK;
    GeomDevice* gd;
    int rc = geom_device(rs, &gd);
    if (rc) return rc;
    RaggedScratch* sc;
    if ((rc = ragged_scratch(&sc))) return rc;
    std::lock_guard<std::mutex> lk(sc->mu);
    const size_t items_bytes = items.size() * sizeof(RaggedItem);
    const size_t map_off = (items_bytes + 255) / 256 * 256;
    const size_t meta = map_off + block_item.size() * 4;
    if (sc->meta_free) HEC_HIP(hipEventSynchronize(sc->meta_free));  // previous call's kernel done
    if ((rc = sc->reserve(0, meta))) return rc;
    if (!sc->meta_free) HEC_HIP(hipEventCreateWithFlags(&sc->meta_free, hipEventDisableTiming));
    if (decode && (rc = ensure_dense_decode(rs, gd, sc->stream))) return rc;
    std::memcpy(sc->hmeta, items.data(), items_bytes);
    std::memcpy(sc->hmeta + map_off, block_item.data(), block_item.size() * 4);
    HEC_HIP(hipMemcpyAsync(sc->dmeta, sc->hmeta, meta, hipMemcpyHostToDevice, stream));
    RaggedArgs ra{};
    ra.base = d_base;
    ra.items = reinterpret_cast<const RaggedItem*>(sc->dmeta);
    ra.block_item = reinterpret_cast<const uint32_t*>(sc->dmeta + map_off);
    ra.n_blocks = uint32_t(block_item.size());
    ra.tabs = decode ? gd->decode_dense.tabs : gd->encode.tabs;
    ra.lut = decode ? gd->decode_dense.lut : nullptr;
    ra.bad_count = d_bad;
    if (bitslice)
        HEC_HIP(launch_rs104_bs_ragged(ra, stream));
    else
        HEC_HIP(launch_rs104_ragged(ra, decode, stream));
    HEC_HIP(hipEventRecord(sc->meta_free, stream));
    return HEC_OK;
}

}  // namespace
}  // namespace hec

extern "C" {

int hec_gpu_encode_ragged(const hec_rs_t* rs, uint8_t* d_base, const hec_stripe_desc* descs, uint32_t n_stripes,
                          void* stream) {
    return hec::gpu_ragged(rs, d_base, descs, n_stripes, false, nullptr, static_cast<hipStream_t>(stream));
}

int hec_gpu_reconstruct_ragged(const hec_rs_t* rs, uint8_t* d_base, const hec_stripe_desc* descs,
                               uint32_t n_stripes, uint32_t* d_bad_stripes, void* stream) {
    return hec::gpu_ragged(rs, d_base, descs, n_stripes, true, d_bad_stripes, static_cast<hipStream_t>(stream));
}

}  // extern "C"

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

// Metadata (RaggedItems + workgroup map) of one device-resident ragged call:
// pinned staging and its device copy. The calls take slots round-robin, so a
// call waits only for the kernel that used its slot kMetaSlots calls ago, not
// for the previous call's kernel (a back-to-back encode / reconstruct stream
// keeps the GPU fed while the host builds the next map).
struct MetaSlot {
    uint8_t* h = nullptr;
    uint8_t* d = nullptr;
    size_t cap = 0;
    hipEvent_t free = nullptr;  // recorded after the kernel that read this slot
    int reserve(size_t bytes) {
        if (free) HEC_HIP(hipEventSynchronize(free));
        else HEC_HIP(hipEventCreateWithFlags(&free, hipEventDisableTiming));
        if (bytes <= cap) return HEC_OK;
        if (h) HEC_HIP(hipHostFree(h));
        if (d) HEC_HIP(hipFree(d));
        h = d = nullptr;
        cap = 0;
        const size_t want = std::max(bytes, size_t(1) << 20);
        HEC_TRY(pinned_alloc(reinterpret_cast<void**>(&h), want));
        HEC_HIP(hipMalloc(reinterpret_cast<void**>(&d), want));
        cap = want;
        return HEC_OK;
    }
};
constexpr int kMetaSlots = 4;

struct RaggedScratch {
    std::mutex mu;
    hipStream_t stream = nullptr;
    MetaSlot slots[kMetaSlots];  // device-API ragged calls
    unsigned next_slot = 0;
    Completion done;             // small host calls (compact_reconstruct_104)
    uint8_t* host = nullptr;
    uint8_t* dev = nullptr;
    size_t cap = 0;
    uint8_t* hmeta = nullptr;
    uint8_t* dmeta = nullptr;
    size_t mcap = 0;
    int init() {
        HEC_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        return HEC_OK;
    }
    int reserve(size_t bytes, size_t meta) {
        if (bytes > cap && bytes > 0) {
            if (host) HEC_HIP(hipHostFree(host));
            if (dev) HEC_HIP(hipFree(dev));
            host = dev = nullptr;
            cap = 0;
            const size_t want = std::max(bytes, size_t(16) << 20);
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
    // Compact staging above 64 MiB in a burst slot (index >= kWarmSlots) is
    // freed when its call ends (ScratchTrim's rule, hec_internal.hpp).
    void trim_large() {
        constexpr size_t kKeep = size_t(64) << 20;
        if (cap <= kKeep) return;
        (void)hipStreamSynchronize(stream);  // an error return may leave copies in flight
        (void)hipHostFree(host);
        (void)hipFree(dev);
        host = dev = nullptr;
        cap = 0;
    }
};
struct RaggedTrim {
    RaggedScratch* sc;
    bool on;
    ~RaggedTrim() {
        if (on) sc->trim_large();
    }
};

// Per-device pool of ragged scratch slots (see SlotPool, hec_internal.hpp).
int lease_ragged(Lease<RaggedScratch>& out) {
    static std::mutex mu;
    static auto* reg = new std::map<int, std::unique_ptr<SlotPool<RaggedScratch>>>();  // process lifetime
    int dev;
    int rc = current_device(&dev);
    if (rc) return rc;
    SlotPool<RaggedScratch>* pool;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto& p = (*reg)[dev];
        if (!p) p.reset(new SlotPool<RaggedScratch>());
        pool = p.get();
    }
    return pool->lease(out);
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
    Lease<RaggedScratch> lease;
    if ((rc = lease_ragged(lease))) return rc;
    RaggedScratch* sc = lease.sc;
    const RaggedTrim trim{sc, lease.index >= kWarmSlots};  // before the lease lets go
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
    // The fills may run on host-pool workers, whose failure detail and values
    // are thread-local to them: the first failure's (code, detail, values) is
    // captured on its thread and re-raised on the caller's.
    std::mutex err_mu;
    int first_err = HEC_OK;
    std::string err_detail;
    ErrorValues err_values;
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
                        std::lock_guard<std::mutex> g(err_mu);
                        if (first_err == HEC_OK) {
                            first_err = r;
                            err_detail = hec_last_error_detail();
                            err_values = last_error_values();
                        }
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
    if (first_err) return fail_with(first_err, err_detail, err_values);
    // zero-copy: the kernel reads the packed survivors and writes the rebuilt
    // shards in the pinned staging itself (no H2D / D2H of the payload)
    uint8_t* zh = zero_copy_enabled() ? pinned_device_ptr(sc->host) : nullptr;
    if (!zh) HEC_HIP(hipMemcpyAsync(sc->dev, sc->host, in_total, hipMemcpyHostToDevice, sc->stream));
    RaggedArgs ra{};
    ra.base = zh ? zh : sc->dev;
    ra.n_blocks = uint32_t(block_item.size());
    ra.tabs = gd->decode_dense.tabs;
    ra.lut = gd->decode_dense.lut;
    ra.compact = 1;
    if (items.size() == 1) {  // one stripe (a per-call reconstruct): descriptor as a kernel argument
        ra.inline_one = 1;
        ra.one = items[0];
    } else {
        std::memcpy(sc->hmeta, items.data(), items_bytes);
        const size_t map_off = (items_bytes + 255) / 256 * 256;
        std::memcpy(sc->hmeta + map_off, block_item.data(), block_item.size() * 4);
        HEC_HIP(hipMemcpyAsync(sc->dmeta, sc->hmeta, meta, hipMemcpyHostToDevice, sc->stream));
        ra.items = reinterpret_cast<const RaggedItem*>(sc->dmeta);
        ra.block_item = reinterpret_cast<const uint32_t*>(sc->dmeta + map_off);
    }
    // small zero-copy calls: completion from the kernel's own signal
    const bool signal = zh && in_total <= completion_flag_max();
    if (signal && (rc = sc->done.arm(sc->stream, &ra.done_count, &ra.done_flag, &ra.done_seq))) return rc;
    HEC_HIP(launch_rs104_ragged(ra, true, sc->stream));
    if (!zh)
        HEC_HIP(hipMemcpyAsync(sc->host + in_total, sc->dev + in_total, total - in_total, hipMemcpyDeviceToHost,
                               sc->stream));
    if (signal) {
        if ((rc = sc->done.wait(sc->stream))) return rc;
    } else {
        HEC_HIP(hipStreamSynchronize(sc->stream));
    }
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
            if (i < 32) mask |= 1u << i;  // used by the RS(10,4) path only; n may be up to 256
        }
        if (!err && np < n && np < k) err = HEC_ERR_TOO_FEW_SHARDS_PRESENT;
        if (!err && np < n)
            for (int i = 0; i < n; ++i)
                if (!pr[i] && !(data_only && i >= k) && !shards[s * n + i])
                    err = fail(HEC_ERR_INVALID_ARGUMENT, "missing shard without a buffer");
        if (err) {
            if (bad_index) *bad_index = s;
            return err == HEC_ERR_INVALID_ARGUMENT ? err : fail(err, "stripe " + std::to_string(s));
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

// Workgroups of one ragged stripe: none for a decode of a stripe whose 14
// shards are all present (upstream's no-op), so those launch nothing.
uint64_t ragged_chunks(const hec_stripe_desc& d, bool decode, uint32_t chunk_bytes) {
    if (decode && (d.present_mask & 0x3FFFu) == 0x3FFFu) return 0;
    return (uint64_t(d.shard_len) + chunk_bytes - 1) / chunk_bytes;
}

// The kernel of one ragged launch, shared by gpu_ragged and
// hec_ragged_kernel_name so a reported name is the kernel that runs. Both
// ragged kernels deal each XCD a contiguous eighth of the launch's column
// ranges (ragged_block, rs_kernels.hip).
struct RaggedPick {
    bool bitslice;  // encode with every length a multiple of 8 KiB: rs104_bs_ragged_kernel
};
RaggedPick ragged_pick(const hec_stripe_desc* descs, uint32_t n, bool decode) {
    RaggedPick p;
    p.bitslice = !decode;
    for (uint32_t j = 0; j < n && p.bitslice; ++j) p.bitslice = descs[j].shard_len % kBsChunk == 0;
    return p;
}

const char* ragged_name(const RaggedPick& p, bool decode) {
    if (decode) return "rs104_ragged_kernel<DEC=true> (table lookup, XCD eighths)";
    if (p.bitslice) return "rs104_bs_ragged_kernel (bit-sliced, XCD eighths)";
    return "rs104_ragged_kernel<DEC=false> (table lookup, XCD eighths)";
}

// Device-resident ragged batches: stripe descriptors come from the host, data
// stays in HBM. Descriptors -> RaggedItems + workgroup map in pinned staging,
// uploaded on the caller's stream ahead of the kernel.
int gpu_ragged(const hec_rs_t* rs, uint8_t* d_base, const hec_stripe_desc* descs, uint32_t n, bool decode,
               uint32_t* d_bad, hipStream_t stream) {
    if (!rs || !d_base || (n && !descs)) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    if (!(rs->k == 10 && rs->m == 4))
        return fail(HEC_ERR_INVALID_ARGUMENT, "ragged device batches are RS(10,4) only");
    const RaggedPick pick = ragged_pick(descs, n, decode);
    const bool bitslice = pick.bitslice;
    const uint32_t chunk_bytes = bitslice ? kBsChunk : 4096;
    uint64_t n_blocks = 0;
    for (uint32_t j = 0; j < n; ++j) {
        const hec_stripe_desc& d = descs[j];
        if (d.shard_len == 0) return fail(HEC_ERR_EMPTY_SHARD, "stripe " + std::to_string(j));
        if ((d.offset | d.shard_stride | uint64_t(reinterpret_cast<uintptr_t>(d_base))) % 16 != 0 ||
            d.shard_stride < d.shard_len)
            return fail(HEC_ERR_INVALID_ARGUMENT, "stripe " + std::to_string(j) +
                                                      ": offset/stride must be 16-byte aligned, stride >= len");
        // 64-bit: a shard_len near 2^32 must not wrap to 0 or 1 chunks
        n_blocks += ragged_chunks(d, decode, chunk_bytes);
        if (n_blocks > UINT32_MAX) return fail(HEC_ERR_INVALID_ARGUMENT, "ragged batch above 2^32 workgroups");
    }
    if (n == 0) return HEC_OK;
    GeomDevice* gd;
    int rc = geom_device(rs, &gd);
    if (rc) return rc;
    Lease<RaggedScratch> lease;
    if ((rc = lease_ragged(lease))) return rc;
    RaggedScratch* sc = lease.sc;
    const size_t items_bytes = size_t(n) * sizeof(RaggedItem);
    const size_t map_off = (items_bytes + 255) / 256 * 256;
    const size_t meta = map_off + n_blocks * 4;
    MetaSlot& slot = sc->slots[sc->next_slot++ % kMetaSlots];
    if ((rc = slot.reserve(meta))) return rc;  // waits for this slot's previous kernel only
    if (decode && (rc = ensure_dense_decode(rs, gd, sc->stream))) return rc;
    // items and workgroup map written straight into the pinned slot
    RaggedItem* items = reinterpret_cast<RaggedItem*>(slot.h);
    uint32_t* block_item = reinterpret_cast<uint32_t*>(slot.h + map_off);
    uint32_t first = 0;
    for (uint32_t j = 0; j < n; ++j) {
        const hec_stripe_desc& d = descs[j];
        const uint32_t chunks = uint32_t(ragged_chunks(d, decode, chunk_bytes));
        items[j] = RaggedItem{d.offset, d.shard_stride, d.shard_len, d.present_mask, first, 0, 0};
        std::fill(block_item + first, block_item + first + chunks, j);
        first += chunks;
    }
    HEC_HIP(hipMemcpyAsync(slot.d, slot.h, meta, hipMemcpyHostToDevice, stream));
    RaggedArgs ra{};
    ra.base = d_base;
    ra.items = reinterpret_cast<const RaggedItem*>(slot.d);
    ra.block_item = reinterpret_cast<const uint32_t*>(slot.d + map_off);
    ra.n_blocks = uint32_t(n_blocks);
    ra.tabs = decode ? gd->decode_dense.tabs : gd->encode.tabs;
    ra.lut = decode ? gd->decode_dense.lut : nullptr;
    ra.bad_count = d_bad;
    if (n_blocks == 0) {  // every stripe already complete (upstream no-op)
        HEC_HIP(hipEventRecord(slot.free, stream));
        return HEC_OK;
    }
    if (bitslice)
        HEC_HIP(launch_rs104_bs_ragged(ra, stream));
    else
        HEC_HIP(launch_rs104_ragged(ra, decode, stream));
    HEC_HIP(hipEventRecord(slot.free, stream));
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

const char* hec_ragged_kernel_name(const hec_stripe_desc* descs, uint32_t n_stripes, int decode) {
    if (n_stripes && !descs) return "invalid argument";
    return hec::ragged_name(hec::ragged_pick(descs, n_stripes, decode != 0), decode != 0);
}

}  // extern "C"

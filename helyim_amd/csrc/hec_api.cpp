// C ABI of libhec (include/hec.h): the ReedSolomon<galois_8::Field> surface
// helyim-ec calls (encoder.rs:191,208-209,249-250,288;
// helyim-store/src/erasure_coding/mod.rs:411-412,426), the device batch entry
// points, and shared device state. All compute goes through the gfx950
// kernels in rs_kernels.hip; there is no CPU fallback.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <tuple>

#include "hec_internal.hpp"

namespace hec {

static thread_local std::string g_detail;
static thread_local ErrorValues g_values;

void set_detail(const std::string& s) {
    g_detail = s;
    g_values = ErrorValues{};
}

int fail(int code, const std::string& detail) {
    set_detail(detail);
    return code;
}

int fail_values(int code, const std::string& detail, uint64_t a, uint64_t b) {
    set_detail(detail);
    g_values.a = a;
    g_values.b = b;
    return code;
}

int fail_errno(int code, const std::string& what, int err) {
    set_detail(what + ": " + std::strerror(err));
    g_values.os_errno = err;
    return code;
}

int fail_with(int code, const std::string& detail, const ErrorValues& v) {
    g_detail = detail;
    g_values = v;
    return code;
}

ErrorValues last_error_values() { return g_values; }

int hip_fail(hipError_t e, const char* what) {
    set_detail(std::string(what) + ": " + hipGetErrorString(e));
    if (e == hipErrorOutOfMemory) return HEC_ERR_OUT_OF_MEMORY;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return HEC_ERR_NO_DEVICE;
    return HEC_ERR_HIP;
}

// ---------------------------------------------------------------------------
// Persistent host worker pool (parallel_for). One job at a time: the caller
// publishes it, workers and the caller claim indices from an atomic counter,
// the caller returns when all are done. Workers spin briefly after a job so
// back-to-back small calls find them awake, then sleep on the condition.
// ---------------------------------------------------------------------------
namespace {
class HostPool {
   public:
    // Workers of device `dev`'s pool run on that GPU's NUMA node (when the
    // platform says which; they copy into and out of its pinned staging;
    // profiles/r04/host_pool_bind_ab.jsonl).
    HostPool(unsigned n, int dev) {
        for (unsigned i = 0; i < n; ++i)
            th_.emplace_back([this, dev] {
                (void)hec_bind_thread_to_device(dev, nullptr);  // placement only: no-op when unknown
                loop();
            });
    }
    // false if another caller owns the pool (run serially then)
    bool run(size_t n, unsigned max_threads, const std::function<void(size_t)>& fn) {
        std::unique_lock<std::mutex> own(busy_, std::try_to_lock);
        if (!own.owns_lock()) return false;
        {
            std::lock_guard<std::mutex> lk(mu_);
            fn_ = &fn;
            n_ = n;
            next_.store(0);
            done_.store(0);
            helpers_ = max_threads > 1 ? max_threads - 1 : 0;
            ++gen_;
        }
        cv_.notify_all();
        work();
        while (done_.load(std::memory_order_acquire) < n_) std::this_thread::yield();
        std::lock_guard<std::mutex> lk(mu_);
        fn_ = nullptr;
        // a helper still inside work() has seen next_ >= n_; wait for it to leave
        while (active_.load() != 0) std::this_thread::yield();
        return true;
    }

   private:
    void work() {
        for (;;) {
            const size_t i = next_.fetch_add(1);
            if (i >= n_) return;
            (*fn_)(i);
            done_.fetch_add(1, std::memory_order_release);
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                // spin-wait window first (cheap for back-to-back calls), then sleep
                for (int spin = 0; spin < 256 && gen_ == seen; ++spin) {
                    lk.unlock();
                    std::this_thread::yield();
                    lk.lock();
                }
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                if (!fn_ || helpers_ == 0) continue;
                --helpers_;
                active_.fetch_add(1);
            }
            work();
            active_.fetch_sub(1);
        }
    }
    std::vector<std::thread> th_;
    std::mutex busy_, mu_;
    std::condition_variable cv_;
    const std::function<void(size_t)>* fn_ = nullptr;
    size_t n_ = 0;
    unsigned helpers_ = 0;
    uint64_t gen_ = 0;
    std::atomic<size_t> next_{0}, done_{0};
    std::atomic<int> active_{0};
};
}  // namespace

// Pools per device (up to kPoolsPerDevice each, created on first use and
// never destroyed: their threads live for the process). A call takes a free
// pool of its current device, so the ranges of one multi-device host call --
// and concurrent callers on different GPUs -- copy on their own workers
// instead of all but one running serially. Each pool's workers
// bind themselves to their device's NUMA node, whichever thread created it.
constexpr size_t kPoolsPerDevice = 2;
void pool_run(size_t n, unsigned max_threads, const std::function<void(size_t)>& fn) {
    static std::mutex mu;
    static auto* pools = new std::map<int, std::vector<HostPool*>>();
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        (void)hipGetLastError();
        dev = 0;
    }
    std::vector<HostPool*> mine;
    {
        std::lock_guard<std::mutex> lk(mu);
        mine = (*pools)[dev];
    }
    for (HostPool* p : mine)
        if (p->run(n, max_threads, fn)) return;
    HostPool* fresh = nullptr;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto& v = (*pools)[dev];
        if (v.size() < kPoolsPerDevice) {
            fresh = new HostPool(15, dev);
            v.push_back(fresh);
        }
    }
    if (fresh && fresh->run(n, max_threads, fn)) return;
    for (size_t i = 0; i < n; ++i) fn(i);  // every pool of this device busy: this thread alone
}

int current_device(int* dev) {
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count <= 0) {
        (void)hipGetLastError();
        return fail(HEC_ERR_NO_DEVICE, "no HIP device visible (libhec has no CPU fallback)");
    }
    HEC_HIP(hipGetDevice(dev));
    return HEC_OK;
}

// ---------------------------------------------------------------------------
// Plans
// ---------------------------------------------------------------------------
uint32_t HostPlans::add(const Mat& coefs, const std::vector<uint32_t>& in_ids,
                        const std::vector<uint32_t>& out_ids) {
    DevPlan p{};
    p.nin = uint32_t(in_ids.size());
    p.nout = uint32_t(out_ids.size());
    p.tab_off = uint32_t(tabs.size());
    p.idx_off = uint32_t(idx.size());
    p.tab_rows = fixed_rows ? fixed_rows : p.nout;
    for (uint32_t i = 0; i < p.nin; ++i)
        for (uint32_t r = 0; r < p.tab_rows; ++r) {
            uint32_t t[kTabWords];
            perm_tables(r < p.nout ? coefs.at(int(r), int(i)) : uint8_t(0), t);
            tabs.insert(tabs.end(), t, t + kTabWords);
        }
    idx.insert(idx.end(), in_ids.begin(), in_ids.end());
    idx.insert(idx.end(), out_ids.begin(), out_ids.end());
    plans.push_back(p);
    return uint32_t(plans.size() - 1);
}

uint32_t HostPlans::add_noop(uint32_t nin) {
    DevPlan p{nin, 0, uint32_t(tabs.size()), uint32_t(idx.size()), fixed_rows, {0, 0, 0}};
    tabs.insert(tabs.end(), size_t(nin) * fixed_rows * kTabWords, 0u);
    plans.push_back(p);
    return uint32_t(plans.size() - 1);
}

template <typename T>
static int grow_upload(T*& dptr, size_t& cap, const T* src, size_t count, hipStream_t s) {
    if (count == 0) return HEC_OK;
    if (count > cap) {
        if (dptr) HEC_HIP(hipFree(dptr));
        dptr = nullptr;
        cap = 0;
        HEC_HIP(hipMalloc(reinterpret_cast<void**>(&dptr), count * sizeof(T)));
        cap = count;
    }
    HEC_HIP(hipMemcpyAsync(dptr, src, count * sizeof(T), hipMemcpyHostToDevice, s));
    return HEC_OK;
}

int DevicePlanSet::upload(const HostPlans& hp, const std::vector<uint32_t>* lut_host, hipStream_t s) {
    int rc;
    if ((rc = grow_upload(plans, cap_plans, hp.plans.data(), hp.plans.size(), s))) return rc;
    if ((rc = grow_upload(tabs, cap_tabs, hp.tabs.data(), hp.tabs.size(), s))) return rc;
    if ((rc = grow_upload(idx, cap_idx, hp.idx.data(), hp.idx.size(), s))) return rc;
    if (lut_host && (rc = grow_upload(lut, cap_lut, lut_host->data(), lut_host->size(), s))) return rc;
    // Host vectors may be freed by the caller right after: make the copies land.
    HEC_HIP(hipStreamSynchronize(s));
    return HEC_OK;
}

void DevicePlanSet::release() {
    (void)hipFree(plans);
    (void)hipFree(tabs);
    (void)hipFree(idx);
    (void)hipFree(lut);
    plans = nullptr;
    tabs = idx = lut = nullptr;
    cap_plans = cap_tabs = cap_idx = cap_lut = 0;
}

// upstream reconstruct_internal: first k present shards -> sub-matrix ->
// inverse; missing data rows = inverse rows; missing parity rows = parity
// row x inverse (composed, bit-identical to upstream's second pass since the
// reconstructed data bytes are unique).
int decode_plan(const hec_rs* rs, const uint8_t* present, bool data_only, Mat& coefs,
                std::vector<uint32_t>& in_ids, std::vector<uint32_t>& out_ids, bool* noop) {
    const int k = rs->k, n = rs->n;
    int npresent = 0;
    for (int i = 0; i < n; ++i) npresent += present[i] ? 1 : 0;
    *noop = false;
    in_ids.clear();
    out_ids.clear();
    if (npresent == n) {
        *noop = true;
        return HEC_OK;
    }
    if (npresent < k) return fail(HEC_ERR_TOO_FEW_SHARDS_PRESENT, "");
    std::vector<uint32_t> miss;
    for (int i = 0; i < n; ++i) {
        if (present[i]) {
            if (int(in_ids.size()) < k) in_ids.push_back(uint32_t(i));
        } else {
            miss.push_back(uint32_t(i));
        }
    }
    Mat sub(k, k);
    for (int r = 0; r < k; ++r)
        for (int c = 0; c < k; ++c) sub.at(r, c) = rs->matrix.at(int(in_ids[r]), c);
    Mat inv;
    if (!mat_invert(sub, inv)) return fail(HEC_ERR_INVALID_ARGUMENT, "singular decode matrix");
    for (uint32_t i : miss)
        if (!(data_only && int(i) >= k)) out_ids.push_back(i);
    coefs = Mat(int(out_ids.size()), k);
    const Gf& g = gf();
    for (size_t r = 0; r < out_ids.size(); ++r) {
        const int id = int(out_ids[r]);
        if (id < k) {
            for (int c = 0; c < k; ++c) coefs.at(int(r), c) = inv.at(id, c);
        } else {
            for (int c = 0; c < k; ++c) {
                uint8_t acc = 0;
                for (int t = 0; t < k; ++t) acc ^= g.mul[rs->matrix.at(id, t)][inv.at(t, c)];
                coefs.at(int(r), c) = acc;
            }
        }
    }
    if (out_ids.empty()) *noop = true;
    return HEC_OK;
}

// ---------------------------------------------------------------------------
// Per-device geometry state
// ---------------------------------------------------------------------------
static std::mutex g_geom_mu;
static std::map<std::tuple<int, int, int>, std::unique_ptr<GeomDevice>> g_geom;

int geom_device(const hec_rs* rs, GeomDevice** out) {
    int dev;
    int rc = current_device(&dev);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(g_geom_mu);
    auto key = std::make_tuple(dev, rs->k, rs->m);
    auto it = g_geom.find(key);
    if (it != g_geom.end()) {
        *out = it->second.get();
        return HEC_OK;
    }
    std::unique_ptr<GeomDevice> gd(new GeomDevice());
    const bool is104 = rs->k == 10 && rs->m == 4;
    HostPlans hp;
    if (is104) hp.fixed_rows = 4;
    Mat par(rs->m, rs->k);
    for (int r = 0; r < rs->m; ++r)
        for (int c = 0; c < rs->k; ++c) par.at(r, c) = rs->matrix.at(rs->k + r, c);
    std::vector<uint32_t> in_ids, out_ids;
    for (int i = 0; i < rs->k; ++i) in_ids.push_back(uint32_t(i));
    for (int j = 0; j < rs->m; ++j) out_ids.push_back(uint32_t(j));
    hp.add(par, in_ids, out_ids);
    if ((rc = gd->encode.upload(hp, nullptr, nullptr))) return rc;
    gd->encode.fast104 = is104;
    *out = gd.get();
    g_geom[key] = std::move(gd);
    return HEC_OK;
}

int ensure_dense_decode(const hec_rs* rs, GeomDevice* gd, hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_geom_mu);
    if (gd->decode_ready) return HEC_OK;
    const int n = rs->n, k = rs->k;
    if (n > 16) return fail(HEC_ERR_INVALID_ARGUMENT, "device-mask reconstruct needs total shards <= 16");
    HostPlans hp;
    const bool is104 = k == 10 && rs->m == 4;
    if (is104) hp.fixed_rows = 4;
    std::vector<uint32_t> lut(size_t(1) << n, kNoPlan);
    const uint32_t noop = hp.add_noop(uint32_t(k));
    uint8_t present[16];
    Mat coefs;
    std::vector<uint32_t> in_ids, out_ids;
    for (uint32_t mask = 0; mask < (1u << n); ++mask) {
        const int pc = __builtin_popcount(mask);
        if (pc < k) continue;
        if (pc == n) {
            lut[mask] = noop;
            continue;
        }
        for (int i = 0; i < n; ++i) present[i] = (mask >> i) & 1;
        bool is_noop = false;
        int rc = decode_plan(rs, present, false, coefs, in_ids, out_ids, &is_noop);
        if (rc) return rc;
        lut[mask] = hp.add(coefs, in_ids, out_ids);
    }
    int rc = gd->decode_dense.upload(hp, &lut, s);
    if (rc) return rc;
    gd->decode_dense.fast104 = is104;
    gd->decode_dense.lut_bits = uint32_t(n);
    gd->decode_ready = true;
    return HEC_OK;
}

int run_apply(const DevicePlanSet& ps, uint32_t nin, const uint8_t* in_base, uint64_t in_stripe,
              uint64_t in_shard, uint8_t* out_base, uint64_t out_stripe, uint64_t out_shard,
              uint64_t len, uint32_t n_stripes, const uint32_t* masks, uint32_t* bad,
              hipStream_t s, Completion* done, bool over_pcie) {
    ApplyArgs a{};
    if (done) HEC_TRY(done->arm(s, &a.done_count, &a.done_flag, &a.done_seq));
    a.in_base = in_base;
    a.in_stripe = in_stripe;
    a.in_shard = in_shard;
    a.out_base = out_base;
    a.out_stripe = out_stripe;
    a.out_shard = out_shard;
    a.len = len;
    a.n_stripes = n_stripes;
    a.plans = ps.plans;
    a.tabs = ps.tabs;
    a.idx = ps.idx;
    a.masks = masks;
    a.lut = ps.lut;
    a.bad_count = bad;
    a.fast104 = ps.fast104 ? 1u : 0u;
    a.mask_limit = ps.lut_bits ? ((1u << ps.lut_bits) - 1u) : 0u;
    if (masks && !ps.lut) return fail(HEC_ERR_INVALID_ARGUMENT, "per-stripe masks need a decode LUT");
    const uint64_t align = uint64_t(reinterpret_cast<uintptr_t>(in_base)) | in_stripe | in_shard |
                           uint64_t(reinterpret_cast<uintptr_t>(out_base)) | out_stripe | out_shard;
    const bool aligned = (align % 16) == 0;
    HEC_HIP(launch_apply(a, int(nin), aligned, over_pcie && !masks, s));
    return HEC_OK;
}


// ---------------------------------------------------------------------------
// Per-device scratch for host-memory calls
// ---------------------------------------------------------------------------
static std::mutex g_scratch_mu;
static std::map<int, std::unique_ptr<SlotPool<Scratch>>> g_scratch;  // per device, process lifetime

int Scratch::reserve(size_t bytes) {
    if (bytes <= dcap) return HEC_OK;
    if (dbuf) HEC_HIP(hipFree(dbuf));
    dbuf = nullptr;
    dcap = 0;
    size_t want = std::max(bytes, size_t(16) << 20);
    HEC_HIP(hipMalloc(reinterpret_cast<void**>(&dbuf), want));
    dcap = want;
    return HEC_OK;
}

int Scratch::reserve_host(size_t bytes) {
    if (bytes <= hcap) return HEC_OK;
    if (hbuf) HEC_HIP(hipHostFree(hbuf));
    hbuf = nullptr;
    hcap = 0;
    size_t want = std::max(bytes, size_t(16) << 20);
    HEC_TRY(pinned_alloc(reinterpret_cast<void**>(&hbuf), want));
    hcap = want;
    return HEC_OK;
}

std::atomic<bool>& zero_copy_enabled() {
    static std::atomic<bool> on{true};
    return on;
}

uint8_t* pinned_device_ptr(void* host) {
    void* d = nullptr;
    if (!host || hipHostGetDevicePointer(&d, host, 0) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return static_cast<uint8_t*>(d);
}

std::atomic<uint64_t>& host_staging_max() {
    static std::atomic<uint64_t> v{uint64_t(16) << 20};  // measured crossover
    return v;
}

std::atomic<uint64_t>& completion_flag_max() {
    static std::atomic<uint64_t> v{uint64_t(1) << 20};
    return v;
}

int Completion::arm(hipStream_t s, uint32_t** count_out, uint32_t** flag_out, uint32_t* seq_out) {
    if (!host) {
        HEC_HIP(hipHostMalloc(reinterpret_cast<void**>(&host), 64, hipHostMallocCoherent));
        *host = 0;
        HEC_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&dflag), host, 0));
        HEC_HIP(hipMalloc(reinterpret_cast<void**>(&count), 64));
        HEC_HIP(hipMemsetAsync(count, 0, 64, s));  // ordered before the first signalling launch
    }
    if (++seq == 0) seq = 1;  // 0 is the flag's initial value
    *count_out = count;
    *flag_out = dflag;
    *seq_out = seq;
    return HEC_OK;
}

int Completion::wait(hipStream_t s) {
    const auto t0 = std::chrono::steady_clock::now();
    unsigned spins = 0;
    while (__atomic_load_n(host, __ATOMIC_ACQUIRE) != seq) {
        if ((++spins & 255) == 0 &&
            std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(kSpinUs)) {
            const hipError_t e = hipStreamSynchronize(s);
            if (e == hipSuccess && __atomic_load_n(host, __ATOMIC_ACQUIRE) == seq) return HEC_OK;
            // a launch that did not finish every workgroup leaves the arrival
            // count non-zero: clear it so the next signalled call counts right
            (void)hipMemset(count, 0, 64);
            if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize (completion fallback)");
            return fail(HEC_ERR_HIP, "kernel finished without its completion signal");
        }
    }
    return HEC_OK;
}

int Scratch::init() {
    HEC_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    return HEC_OK;
}

// Staging above kScratchKeep in a burst slot (index >= kWarmSlots) is freed
// when its call ends: a burst of large per-call encodes (say 1 GiB shards:
// 14 GiB of HBM each) must not stay resident in up to kScratchSlots slots for
// the life of the process; the warm slots keep theirs.
constexpr size_t kScratchKeep = size_t(64) << 20;
void Scratch::trim_large() {
    if (dcap <= kScratchKeep && hcap <= kScratchKeep) return;
    (void)hipStreamSynchronize(stream);  // an error return may leave copies in flight
    if (dcap > kScratchKeep) {
        (void)hipFree(dbuf);
        dbuf = nullptr;
        dcap = 0;
    }
    if (hcap > kScratchKeep) {
        (void)hipHostFree(hbuf);
        hbuf = nullptr;
        hcap = 0;
    }
}

int lease_scratch(Lease<Scratch>& out) {
    int dev;
    int rc = current_device(&dev);
    if (rc) return rc;
    SlotPool<Scratch>* pool;
    {
        std::lock_guard<std::mutex> lk(g_scratch_mu);
        std::unique_ptr<SlotPool<Scratch>>& p = g_scratch[dev];
        if (!p) p.reset(new SlotPool<Scratch>());
        pool = p.get();
    }
    return pool->lease(out);
}

static uint64_t round_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

// upstream check_piece_count!(all) + check_slices!(multi)
static int check_shards(const hec_rs* rs, const void* shards, const size_t* lens, size_t n_shards) {
    if (!shards || !lens) return fail(HEC_ERR_INVALID_ARGUMENT, "null shards");
    if (n_shards < size_t(rs->n)) return fail(HEC_ERR_TOO_FEW_SHARDS, "");
    if (n_shards > size_t(rs->n)) return fail(HEC_ERR_TOO_MANY_SHARDS, "");
    if (lens[0] == 0) return fail(HEC_ERR_EMPTY_SHARD, "");
    for (size_t i = 1; i < n_shards; ++i)
        if (lens[i] != lens[0]) return fail(HEC_ERR_INCORRECT_SHARD_SIZE, "");
    return HEC_OK;
}

static int encode_host(const hec_rs* rs, const uint8_t* const* data, uint8_t* const* parity_out,
                       std::vector<uint8_t>* parity_vec, size_t L) {
    GeomDevice* gd;
    int rc = geom_device(rs, &gd);
    if (rc) return rc;
    Lease<Scratch> lease;
    if ((rc = lease_scratch(lease))) return rc;
    Scratch* sc = lease.sc;
    const ScratchTrim trim{sc, lease.index >= kWarmSlots};  // before the lease lets go
    const uint64_t Lp = round_up(L, 256);
    if ((rc = sc->reserve(size_t(Lp) * rs->n))) return rc;
    uint8_t* par = sc->dbuf + size_t(rs->k) * Lp;
    auto dst_of = [&](int j) { return parity_out ? parity_out[j] : parity_vec->data() + size_t(j) * L; };
    if (uint64_t(rs->k) * L <= host_staging_max()) {
        // pinned staging: k shards packed -> one H2D, one D2H of the m parity
        // rows. (Splitting the call into column chunks on one or two streams
        // to overlap packing with the copies measured slower at 256 KiB and
        // 1 MiB shards: the extra HIP calls cost more than the overlap saves.)
        if ((rc = sc->reserve_host(size_t(Lp) * rs->n))) return rc;
        parallel_for(size_t(rs->k), uint64_t(rs->k) * L,
                     [&](size_t i) { std::memcpy(sc->hbuf + i * Lp, data[i], L); });
        uint8_t* hpar = sc->hbuf + size_t(rs->k) * Lp;
        uint8_t* zh = zero_copy_enabled() ? pinned_device_ptr(sc->hbuf) : nullptr;
        if (zh) {  // the kernel reads the packed shards and writes parity over PCIe
            Completion* done = uint64_t(rs->k) * L <= completion_flag_max() ? &sc->done : nullptr;
            if ((rc = run_apply(gd->encode, uint32_t(rs->k), zh, 0, Lp, zh + size_t(rs->k) * Lp, 0, Lp,
                                round_up(L, 16), 1, nullptr, nullptr, sc->stream, done)))
                return rc;
            if (done) {
                if ((rc = done->wait(sc->stream))) return rc;
                parallel_for(size_t(rs->m), uint64_t(rs->m) * L,
                             [&](size_t j) { std::memcpy(dst_of(int(j)), hpar + j * Lp, L); });
                return HEC_OK;
            }
        } else {
            HEC_HIP(hipMemcpyAsync(sc->dbuf, sc->hbuf, size_t(rs->k) * Lp, hipMemcpyHostToDevice, sc->stream));
            if ((rc = run_apply(gd->encode, uint32_t(rs->k), sc->dbuf, 0, Lp, par, 0, Lp, round_up(L, 16), 1,
                                nullptr, nullptr, sc->stream)))
                return rc;
            HEC_HIP(hipMemcpyAsync(hpar, par, size_t(rs->m - 1) * Lp + L, hipMemcpyDeviceToHost, sc->stream));
        }
        HEC_HIP(hipStreamSynchronize(sc->stream));
        parallel_for(size_t(rs->m), uint64_t(rs->m) * L,
                     [&](size_t j) { std::memcpy(dst_of(int(j)), hpar + j * Lp, L); });
        return HEC_OK;
    }
    const StreamDrain drain{sc->stream};  // the D2H copies below write caller memory
    for (int i = 0; i < rs->k; ++i)
        HEC_HIP(hipMemcpyAsync(sc->dbuf + i * Lp, data[i], L, hipMemcpyHostToDevice, sc->stream));
    if ((rc = run_apply(gd->encode, uint32_t(rs->k), sc->dbuf, 0, Lp, par, 0, Lp, round_up(L, 16), 1,
                        nullptr, nullptr, sc->stream)))
        return rc;
    for (int j = 0; j < rs->m; ++j)
        HEC_HIP(hipMemcpyAsync(dst_of(j), par + j * Lp, L, hipMemcpyDeviceToHost, sc->stream));
    HEC_HIP(hipStreamSynchronize(sc->stream));
    return HEC_OK;
}

static int reconstruct_host(const hec_rs* rs, uint8_t* const* shards, const size_t* lens,
                            const uint8_t* present, size_t n_shards, bool data_only) {
    if (!shards || !lens || !present) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    if (n_shards < size_t(rs->n)) return fail(HEC_ERR_TOO_FEW_SHARDS, "");
    if (n_shards > size_t(rs->n)) return fail(HEC_ERR_TOO_MANY_SHARDS, "");
    size_t L = 0;
    int npresent = 0;
    for (size_t i = 0; i < n_shards; ++i) {
        if (!present[i]) continue;
        if (lens[i] == 0) return fail(HEC_ERR_EMPTY_SHARD, "");
        if (npresent && lens[i] != L) return fail(HEC_ERR_INCORRECT_SHARD_SIZE, "");
        L = lens[i];
        ++npresent;
    }
    if (npresent == rs->n) return HEC_OK;
    if (npresent < rs->k) return fail(HEC_ERR_TOO_FEW_SHARDS_PRESENT, "");
    if (rs->k == 10 && rs->m == 4 && uint64_t(rs->k) * L <= host_staging_max())
        // one-stripe degraded read: pinned compact staging + the dense-LUT kernel
        return hec_rs_reconstruct_batch(rs, shards, lens, present, 1, data_only ? 1 : 0, nullptr);
    Mat coefs;
    std::vector<uint32_t> in_ids, out_ids;
    bool noop = false;
    int rc = decode_plan(rs, present, data_only, coefs, in_ids, out_ids, &noop);
    if (rc) return rc;
    for (uint32_t id : out_ids)
        if (!shards[id]) return fail(HEC_ERR_INVALID_ARGUMENT, "missing shard without a buffer");
    if (noop) return HEC_OK;
    Lease<Scratch> lease;
    if ((rc = lease_scratch(lease))) return rc;
    Scratch* sc = lease.sc;
    const ScratchTrim trim{sc, lease.index >= kWarmSlots};
    const uint64_t Lp = round_up(L, 256);
    if ((rc = sc->reserve(size_t(Lp) * rs->n))) return rc;
    HostPlans hp;
    hp.add(coefs, in_ids, out_ids);
    if ((rc = sc->adhoc.upload(hp, nullptr, sc->stream))) return rc;
    const StreamDrain drain{sc->stream};  // the D2H copies below write caller memory
    for (uint32_t id : in_ids)
        HEC_HIP(hipMemcpyAsync(sc->dbuf + id * Lp, shards[id], L, hipMemcpyHostToDevice, sc->stream));
    if ((rc = run_apply(sc->adhoc, uint32_t(rs->k), sc->dbuf, 0, Lp, sc->dbuf, 0, Lp, round_up(L, 16), 1,
                        nullptr, nullptr, sc->stream)))
        return rc;
    for (uint32_t id : out_ids)
        HEC_HIP(hipMemcpyAsync(shards[id], sc->dbuf + id * Lp, L, hipMemcpyDeviceToHost, sc->stream));
    HEC_HIP(hipStreamSynchronize(sc->stream));
    return HEC_OK;
}

}  // namespace hec

using namespace hec;

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

const char* hec_strerror(int status) {
    switch (status) {
        case HEC_OK: return "ok";
        // reed_solomon_erasure::Error Display texts (upstream 6.0.0)
        case HEC_ERR_TOO_FEW_SHARDS: return "The number of provided shards is smaller than the one in codec";
        case HEC_ERR_TOO_MANY_SHARDS: return "The number of provided shards is greater than the one in codec";
        case HEC_ERR_TOO_FEW_DATA_SHARDS: return "The number of provided data shards is smaller than the one in codec";
        case HEC_ERR_TOO_MANY_DATA_SHARDS: return "The number of provided data shards is greater than the one in codec";
        case HEC_ERR_TOO_FEW_PARITY_SHARDS: return "The number of provided parity shards is smaller than the one in codec";
        case HEC_ERR_TOO_MANY_PARITY_SHARDS: return "The number of provided parity shards is greater than the one in codec";
        case HEC_ERR_TOO_FEW_BUFFER_SHARDS: return "The number of provided buffer shards is smaller than the number of parity shards in codec";
        case HEC_ERR_TOO_MANY_BUFFER_SHARDS: return "The number of provided buffer shards is greater than the number of parity shards in codec";
        case HEC_ERR_INCORRECT_SHARD_SIZE: return "At least one of the provided shards is not of the correct size";
        case HEC_ERR_TOO_FEW_SHARDS_PRESENT: return "The number of shards present is smaller than number of parity shards, cannot reconstruct missing shards";
        case HEC_ERR_EMPTY_SHARD: return "The first shard provided is of zero length";
        case HEC_ERR_INVALID_SHARD_FLAGS: return "The number of flags does not match the total number of shards";
        case HEC_ERR_INVALID_INDEX: return "The data shard index provided is greater or equal to the number of data shards in codec";
        // helyim_ec::EcShardError (helyim-ec/src/errors.rs:55-66)
        case HEC_ERR_IO: return "Io error";
        case HEC_ERR_UNDERFLOW: return "Only {0} shards found but {0} required";
        case HEC_ERR_UNEXPECTED_EC_SHARD_SIZE: return "ec shard size expected {0} but actually is {1}";
        case HEC_ERR_UNEXPECTED_BLOCK_SIZE: return "unexpected block size {0}, buffer size {1}";
        case HEC_ERR_NEEDLE_NOT_FOUND: return "Needle not found in volume";
        case HEC_ERR_SHARD_NOT_FOUND: return "Shard not found in volume";
        case HEC_ERR_HIP: return "HIP runtime error";
        case HEC_ERR_NO_DEVICE: return "no usable GPU device";
        case HEC_ERR_INVALID_ARGUMENT: return "invalid argument";
        case HEC_ERR_OUT_OF_MEMORY: return "out of device memory";
        default: return "unknown status";
    }
}

const char* hec_last_error_detail(void) { return g_detail.c_str(); }

int hec_last_error_values(uint64_t* a, uint64_t* b, int* os_errno) {
    if (a) *a = g_values.a;
    if (b) *b = g_values.b;
    if (os_errno) *os_errno = g_values.os_errno;
    return HEC_OK;
}

const char* hec_version(void) { return "libhec 0.1.0 (gfx950)"; }

int hec_device_count(int* count) {
    if (!count) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    *count = 0;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        return fail(HEC_ERR_NO_DEVICE, "no HIP device visible (libhec has no CPU fallback)");
    }
    *count = n;
    return HEC_OK;
}

int hec_set_device(int device) {
    int n;
    int rc = hec_device_count(&n);
    if (rc) return rc;
    if (device < 0 || device >= n)
        return fail(HEC_ERR_INVALID_ARGUMENT, "device " + std::to_string(device) + " of " + std::to_string(n));
    HEC_HIP(hipSetDevice(device));
    return HEC_OK;
}

int hec_get_device(int* device) {
    if (!device) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    return current_device(device);
}

const char* hec_encode_kernel_name(uint64_t shard_len) { return encode_kernel_name(shard_len, false); }
const char* hec_decode_kernel_name(uint64_t shard_len) { return decode_kernel_name(shard_len); }


const char* hec_host_encode_kernel_name(uint64_t shard_len) {
    return encode_kernel_name(shard_len, true);
}

int hec_set_host_staging(uint64_t max_bytes) {
    host_staging_max() = max_bytes;
    return HEC_OK;
}

int hec_set_completion_signal(uint64_t max_bytes) {
    completion_flag_max() = max_bytes;
    return HEC_OK;
}

int hec_rs_new(size_t data_shards, size_t parity_shards, hec_rs_t** out) {
    if (!out) return fail(HEC_ERR_INVALID_ARGUMENT, "null out");
    *out = nullptr;
    if (data_shards == 0) return fail(HEC_ERR_TOO_FEW_DATA_SHARDS, "");
    if (parity_shards == 0) return fail(HEC_ERR_TOO_FEW_PARITY_SHARDS, "");
    if (data_shards + parity_shards > 256) return fail(HEC_ERR_TOO_MANY_SHARDS, "");
    hec_rs_t* rs = new hec_rs_t();
    rs->k = int(data_shards);
    rs->m = int(parity_shards);
    rs->n = rs->k + rs->m;
    rs->matrix = build_encoding_matrix(rs->k, rs->n);
    *out = rs;
    return HEC_OK;
}

void hec_rs_free(hec_rs_t* rs) { delete rs; }

size_t hec_rs_data_shard_count(const hec_rs_t* rs) { return rs ? size_t(rs->k) : 0; }
size_t hec_rs_parity_shard_count(const hec_rs_t* rs) { return rs ? size_t(rs->m) : 0; }
size_t hec_rs_total_shard_count(const hec_rs_t* rs) { return rs ? size_t(rs->n) : 0; }

int hec_rs_matrix(const hec_rs_t* rs, uint8_t* out, size_t out_len) {
    if (!rs || !out || out_len < rs->matrix.v.size()) return fail(HEC_ERR_INVALID_ARGUMENT, "bad matrix buffer");
    std::memcpy(out, rs->matrix.v.data(), rs->matrix.v.size());
    return HEC_OK;
}

int hec_rs_encode(const hec_rs_t* rs, uint8_t* const* shards, const size_t* shard_lens, size_t n_shards) {
    if (!rs) return fail(HEC_ERR_INVALID_ARGUMENT, "null codec");
    int rc = check_shards(rs, shards, shard_lens, n_shards);
    if (rc) return rc;
    return encode_host(rs, const_cast<const uint8_t* const*>(shards), shards + rs->k, nullptr, shard_lens[0]);
}

int hec_rs_verify(const hec_rs_t* rs, const uint8_t* const* shards, const size_t* shard_lens, size_t n_shards,
                  int* ok) {
    if (!rs || !ok) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    int rc = check_shards(rs, shards, shard_lens, n_shards);
    if (rc) return rc;
    const size_t L = shard_lens[0];
    std::vector<uint8_t> par(size_t(rs->m) * L);
    if ((rc = encode_host(rs, shards, nullptr, &par, L))) return rc;
    *ok = 1;
    for (int j = 0; j < rs->m; ++j)
        if (std::memcmp(par.data() + size_t(j) * L, shards[rs->k + j], L) != 0) *ok = 0;
    return HEC_OK;
}

int hec_rs_reconstruct(const hec_rs_t* rs, uint8_t* const* shards, const size_t* shard_lens,
                       const uint8_t* present, size_t n_shards) {
    if (!rs) return fail(HEC_ERR_INVALID_ARGUMENT, "null codec");
    return reconstruct_host(rs, shards, shard_lens, present, n_shards, false);
}

int hec_rs_reconstruct_data(const hec_rs_t* rs, uint8_t* const* shards, const size_t* shard_lens,
                            const uint8_t* present, size_t n_shards) {
    if (!rs) return fail(HEC_ERR_INVALID_ARGUMENT, "null codec");
    return reconstruct_host(rs, shards, shard_lens, present, n_shards, true);
}

int hec_gpu_encode_batch(const hec_rs_t* rs, const uint8_t* d_data, uint64_t data_stripe_stride,
                         uint64_t data_shard_stride, uint8_t* d_parity, uint64_t parity_stripe_stride,
                         uint64_t parity_shard_stride, uint64_t shard_len, uint32_t n_stripes, void* stream) {
    if (!rs || !d_data || !d_parity) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    if (shard_len == 0) return fail(HEC_ERR_EMPTY_SHARD, "");
    int rc;
    if ((rc = check_strided("data", uint32_t(rs->k), data_stripe_stride, data_shard_stride, shard_len, n_stripes)) ||
        (rc = check_strided("parity", uint32_t(rs->m), parity_stripe_stride, parity_shard_stride, shard_len,
                            n_stripes)))
        return rc;
    GeomDevice* gd;
    if ((rc = geom_device(rs, &gd))) return rc;
    return run_apply(gd->encode, uint32_t(rs->k), d_data, data_stripe_stride, data_shard_stride, d_parity,
                     parity_stripe_stride, parity_shard_stride, shard_len, n_stripes, nullptr, nullptr,
                     static_cast<hipStream_t>(stream));
}

int hec_gpu_reconstruct_batch(const hec_rs_t* rs, uint8_t* d_shards, uint64_t stripe_stride, uint64_t shard_stride,
                              uint64_t shard_len, uint32_t n_stripes, const uint32_t* d_present_masks,
                              uint32_t* d_bad_stripes, void* stream) {
    if (!rs || !d_shards || !d_present_masks) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    if (shard_len == 0) return fail(HEC_ERR_EMPTY_SHARD, "");
    int rc;
    if ((rc = check_strided("shards", uint32_t(rs->n), stripe_stride, shard_stride, shard_len, n_stripes))) return rc;
    GeomDevice* gd;
    if ((rc = geom_device(rs, &gd))) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if ((rc = ensure_dense_decode(rs, gd, s))) return rc;
    return run_apply(gd->decode_dense, uint32_t(rs->k), d_shards, stripe_stride, shard_stride, d_shards,
                     stripe_stride, shard_stride, shard_len, n_stripes, d_present_masks, d_bad_stripes, s);
}

int hec_gpu_fill_splitmix(uint8_t* d_base, uint64_t stripe_stride, uint64_t bytes_per_stripe, uint32_t n_stripes,
                          uint64_t seed_base, void* stream) {
    if (!d_base) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    int dev;
    int rc = current_device(&dev);
    if (rc) return rc;
    HEC_HIP(launch_fill_splitmix(d_base, stripe_stride, bytes_per_stripe, n_stripes, seed_base,
                                 static_cast<hipStream_t>(stream)));
    return HEC_OK;
}

}  // extern "C"

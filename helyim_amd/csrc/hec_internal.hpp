// Internal declarations shared by the C ABI (hec_api.cpp) and the file layer
// (ec_files.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hec.h"
#include "gf256.hpp"
#include "rs_kernels.hpp"

struct hec_rs {
    int k = 0, m = 0, n = 0;
    hec::Mat matrix;  // n x k
};

namespace hec {

// Thread-local failure detail (hec_last_error_detail) and the payload of the
// failure (hec_last_error_values): helyim's EcShardError variants carry
// (usize, usize) or an io::Error (helyim-ec/src/errors.rs:55-66), which the C
// ABI's status code alone cannot rebuild.
struct ErrorValues {
    uint64_t a = 0, b = 0;  // UnexpectedEcShardSize(expected, actual), UnexpectedBlockSize(block, buf), Underflow
    int os_errno = 0;       // errno behind an HEC_ERR_IO (0: no OS error, e.g. a short read)
};
void set_detail(const std::string& s);
int fail(int code, const std::string& detail);  // clears the values
int fail_values(int code, const std::string& detail, uint64_t a, uint64_t b);
// detail = what + ": " + strerror(err), os_errno = err
int fail_errno(int code, const std::string& what, int err);
// Re-raise a failure captured on another thread with its values.
int fail_with(int code, const std::string& detail, const ErrorValues& v);
ErrorValues last_error_values();

// Strided-batch geometry sanity (the C ABI sees only pointers, so sizes cannot
// be checked): shards of a stripe and stripes of a shard must not overlap,
// and the batch's byte extent must not wrap the address space.
inline int check_strided(const char* what, uint32_t shards, uint64_t stripe_stride, uint64_t shard_stride,
                         uint64_t len, uint32_t n_stripes) {
    if (shards > 1 && shard_stride < len)
        return fail(HEC_ERR_INVALID_ARGUMENT, std::string(what) + ": shard stride below shard length");
    if (n_stripes > 1 && stripe_stride < len)
        return fail(HEC_ERR_INVALID_ARGUMENT, std::string(what) + ": stripe stride below shard length");
    uint64_t a, b, e;
    if (__builtin_mul_overflow(uint64_t(n_stripes ? n_stripes - 1 : 0), stripe_stride, &a) ||
        __builtin_mul_overflow(uint64_t(shards ? shards - 1 : 0), shard_stride, &b) ||
        __builtin_add_overflow(a, b, &e) || __builtin_add_overflow(e, len, &e))
        return fail(HEC_ERR_INVALID_ARGUMENT, std::string(what) + ": batch extent overflows");
    return HEC_OK;
}
int hip_fail(hipError_t e, const char* what);

// One pwrite of exactly n bytes (the .ecx tombstone, the .ecj append); a
// short write is an error with errno EIO (errno would otherwise be stale).
inline bool pwrite_exact(int fd, const void* p, size_t n, off_t off) {
    const ssize_t w = ::pwrite(fd, p, n, off);
    if (w == ssize_t(n)) return true;
    if (w >= 0) errno = EIO;
    return false;
}

// Propagate a non-zero hec status.
#define HEC_TRY(call)            \
    do {                         \
        int rc_ = (call);        \
        if (rc_) return rc_;     \
    } while (0)

// NUMA placement (numa.cpp): node of a GPU's PCI function (-1 unknown), and
// pinned host memory on the current device's node.
int device_numa_node(int device, int* node);
int pinned_alloc(void** p, size_t bytes);

#define HEC_HIP(call)                                          \
    do {                                                       \
        hipError_t e_ = (call);                                \
        if (e_ != hipSuccess) return ::hec::hip_fail(e_, #call); \
    } while (0)

// Host-side plan list, uploaded as one DevicePlanSet.
struct HostPlans {
    std::vector<DevPlan> plans;
    std::vector<uint32_t> tabs;
    std::vector<uint32_t> idx;
    // > 0: every plan (no-ops included) gets exactly nin * fixed_rows table
    // rows, so plan p's tables start at p * nin * fixed_rows * kTabWords.
    uint32_t fixed_rows = 0;
    // Append a plan: out rows = coefs (nout x nin) over inputs in_ids.
    uint32_t add(const Mat& coefs, const std::vector<uint32_t>& in_ids,
                 const std::vector<uint32_t>& out_ids);
    uint32_t add_noop(uint32_t nin);
};

// Device copy of a HostPlans (+ optional mask LUT).
struct DevicePlanSet {
    DevPlan* plans = nullptr;
    uint32_t* tabs = nullptr;
    uint32_t* idx = nullptr;
    uint32_t* lut = nullptr;
    size_t cap_plans = 0, cap_tabs = 0, cap_idx = 0, cap_lut = 0;
    bool fast104 = false;  // RS(10,4) set with fixed 4-row tables (rs104_kernel eligible)
    uint32_t lut_bits = 0; // total shards the LUT covers (2^lut_bits entries)
    int upload(const HostPlans& hp, const std::vector<uint32_t>* lut_host, hipStream_t s);
    void release();
};

// Decode plan of one erasure pattern (upstream reconstruct semantics).
// present: n flags. data_only: skip missing parity. Returns HEC_OK or
// TOO_FEW_SHARDS_PRESENT; *noop = true when every shard is present.
int decode_plan(const hec_rs* rs, const uint8_t* present, bool data_only, Mat& coefs,
                std::vector<uint32_t>& in_ids, std::vector<uint32_t>& out_ids, bool* noop);

// Per-device state shared by all contexts of one geometry.
struct GeomDevice {
    DevicePlanSet encode;        // plan 0 = encode
    DevicePlanSet decode_dense;  // LUT over all 2^n present masks (n <= 16)
    bool decode_ready = false;
};
int geom_device(const hec_rs* rs, GeomDevice** out);
int ensure_dense_decode(const hec_rs* rs, GeomDevice* gd, hipStream_t s);

int current_device(int* dev);

// Completion of one small host call without hipStreamSynchronize: the
// launch's last workgroup stores a sequence number into a pinned host flag
// (signal_done in rs_kernels.hip) and the caller spins on it. Measured on
// MI355X (profiles/r02/latency_completion_signal.jsonl): a one-workgroup zero-copy stripe
// completes in 9.2 us this way against 13.3 us through hipStreamSynchronize.
// Owned by a scratch object, so calls on it are serialised by its mutex.
struct Completion {
    uint32_t* host = nullptr;   // pinned, coherent
    uint32_t* dflag = nullptr;  // device address of host
    uint32_t* count = nullptr;  // device word, 0 between launches
    uint32_t seq = 0;
    // Next sequence number, filling the launch arguments' done fields; the
    // signalling launch must go on stream s (or one ordered after it).
    int arm(hipStream_t s, uint32_t** count_out, uint32_t** flag_out, uint32_t* seq_out);
    // Spin on the flag for up to kSpinUs, then fall back to
    // hipStreamSynchronize (a long call, or a GPU busy with other streams);
    // a stream that completes without the flag set is an error.
    int wait(hipStream_t s);
    static constexpr int kSpinUs = 200;
};
// Small host calls signal completion (input bytes at most this); 0 disables.
std::atomic<uint64_t>& completion_flag_max();

// Per-device scratch for host-memory entry points (serialised by mu).
struct Scratch {
    std::mutex mu;
    hipStream_t stream = nullptr;
    uint8_t* dbuf = nullptr;
    size_t dcap = 0;
    uint8_t* hbuf = nullptr;  // pinned staging for small calls (one H2D + one D2H)
    size_t hcap = 0;
    DevicePlanSet adhoc;
    Completion done;
    int init();
    int reserve(size_t bytes);
    int reserve_host(size_t bytes);
    void trim_large();  // free staging above 64 MiB (end of a call, slot still held)
};
// Slots created beyond the first kWarmSlots of a pool (bursts of concurrent
// calls) free their large staging when their call ends, so the steady
// footprint per device is that of kWarmSlots slots, not kScratchSlots.
constexpr size_t kWarmSlots = 2;
struct ScratchTrim {
    Scratch* sc;
    bool on;
    ~ScratchTrim() {
        if (on) sc->trim_large();
    }
};
// Drains a stream when its scope ends, whatever the return path. For calls
// that queue copies or kernels onto CALLER memory: an error return between
// two enqueues must not leave that work in flight once the caller, told the
// call failed, frees or reuses its buffers. Success paths have synchronised
// already, so the drain finds the stream idle.
struct StreamDrain {
    hipStream_t s;
    ~StreamDrain() {
        if (s && hipStreamSynchronize(s) != hipSuccess) (void)hipGetLastError();
    }
};
// Scratch slots per device: a host call leases one (its own stream, staging
// buffers and completion flag), so concurrent calls from several threads
// overlap on the GPU instead of queueing behind one mutex (SURVEY.md §8b:
// reentrant, a stream per call). Free slots are taken first; a new slot is
// created while fewer than kScratchSlots exist; past that a call waits for
// one. The lease holds the slot's mutex until it is destroyed.
constexpr int kScratchSlots = 8;
template <typename S>
struct Lease {
    S* sc = nullptr;
    std::unique_lock<std::mutex> lk;
    size_t index = 0;  // the slot's creation order in its pool
};
// Per-device pool of S (S has `std::mutex mu` and `int init()`, called once
// when a slot is created).
template <typename S>
struct SlotPool {
    std::mutex mu;
    std::vector<std::unique_ptr<S>> slots;
    unsigned rr = 0;
    int lease(Lease<S>& out) {
        {
            std::lock_guard<std::mutex> g(mu);
            for (size_t i = 0; i < slots.size(); ++i) {
                std::unique_lock<std::mutex> l(slots[i]->mu, std::try_to_lock);
                if (l.owns_lock()) {
                    out.sc = slots[i].get();
                    out.lk = std::move(l);
                    out.index = i;
                    return 0;
                }
            }
            if (slots.size() < size_t(kScratchSlots)) {
                std::unique_ptr<S> s(new S());
                if (int rc = s->init()) return rc;
                out.lk = std::unique_lock<std::mutex>(s->mu);
                out.sc = s.get();
                out.index = slots.size();
                slots.push_back(std::move(s));
                return 0;
            }
            out.index = rr++ % slots.size();
            out.sc = slots[out.index].get();
        }
        out.lk = std::unique_lock<std::mutex>(out.sc->mu);  // every slot busy: wait for one
        return 0;
    }
};
int lease_scratch(Lease<Scratch>& out);

// Zero-copy switch (hec_set_host_zero_copy): pinned host memory the GPU can
// address is coded by the kernels in place over PCIe instead of being copied.
std::atomic<bool>& zero_copy_enabled();
// Device address of a hipHostMalloc'd pinned buffer (nullptr if unavailable).
uint8_t* pinned_device_ptr(void* host);

// Host calls whose k * shard_len input is at most this many bytes go through
// pinned staging (one H2D, one D2H) instead of one pageable copy per shard.
std::atomic<uint64_t>& host_staging_max();

// Batched RS(10,4) reconstruct of independent stripes through pinned compact
// staging and one rs104_ragged_kernel launch (intervals.cpp). Job j has shard
// length len and present mask; the decode reads its first 10 present shards,
// which fill(j, slot, shard, dst) writes (len bytes) straight into staging
// (non-zero return = that status aborts the call); take(j, shard, src) then
// receives every erased shard. fill / take run on up to 16 threads
// (io_bound_fill: fill does preads, worth threads at smaller sizes).
struct CompactJob {
    uint64_t len;
    uint32_t mask;
};
using CompactFill = std::function<int(size_t job, int slot, int shard, uint8_t* dst)>;
using CompactTake = std::function<void(size_t job, int shard, const uint8_t* src)>;
int compact_reconstruct_104(const hec_rs* rs, const std::vector<CompactJob>& jobs, const CompactFill& fill,
                            const CompactTake& take, bool io_bound_fill = false);

// Run fn(i) for i in [0, n) on a persistent host worker pool of the calling
// thread's current device (host memcpy of staging): up to 16 threads, at
// least 1 MiB of `bytes` per thread and 4 MiB in all (below that, waking
// workers costs more than the copy saves: measured at 256 KiB shards,
// tools/bench_latency.py). Each device has up to 2 pools; concurrent callers
// do not wait for each other: a call that finds every pool of its device
// busy runs serially on its own thread.
void pool_run(size_t n, unsigned max_threads, const std::function<void(size_t)>& fn);

// Same pool for I/O-bound tasks (pread / fill callbacks): syscalls gain from
// threads at smaller sizes than memcpy, so >= 128 KiB per thread.
template <typename F>
void parallel_io_for(size_t n, uint64_t bytes, F fn) {
    const unsigned nt = unsigned(std::min<uint64_t>(16, bytes >> 17));
    if (nt <= 1 || n < 2) {
        for (size_t i = 0; i < n; ++i) fn(i);
        return;
    }
    pool_run(n, nt, std::function<void(size_t)>(fn));
}

template <typename F>
void parallel_for(size_t n, uint64_t bytes, F fn) {
    const unsigned nt = unsigned(std::min<uint64_t>(16, std::max<uint64_t>(1, bytes >> 20)));  // >= 1 MiB/thread
    if (nt <= 1 || n < 2 || bytes < (uint64_t(4) << 20)) {
        for (size_t i = 0; i < n; ++i) fn(i);
        return;
    }
    pool_run(n, nt, std::function<void(size_t)>(fn));
}

// Run one plan set over a strided batch (plan 0 for every stripe unless masks).
// done (optional): the launch signals it (Completion::arm) when it finishes.
// over_pcie: an encode whose buffers are host memory (zero copy).
int run_apply(const DevicePlanSet& ps, uint32_t nin, const uint8_t* in_base, uint64_t in_stripe,
              uint64_t in_shard, uint8_t* out_base, uint64_t out_stripe, uint64_t out_shard,
              uint64_t len, uint32_t n_stripes, const uint32_t* masks, uint32_t* bad,
              hipStream_t s, Completion* done = nullptr, bool over_pcie = false);

}  // namespace hec

// File-level drop-ins for helyim_ec::write_ec_files / rebuild_ec_files
// (/root/reference/helyim-ec/src/encoder.rs:39-307), GPU-backed.
//
// Byte layout is exactly the reference's: rows of 10 blocks (1 GiB blocks
// while more than 10 GiB remain -- strict '>' at encoder.rs:215 -- then 1 MiB
// blocks while anything remains, encoder.rs:228), short reads zero-filled
// (encoder.rs:169-189), shard file j = concatenation of block j of every row.
// The reference's 256 KiB buffer only sets its I/O granularity (bytes are
// position-wise independent), so whole batches of rows go through the GPU.
//
// Pipeline (3 slots): for job k the main thread preads (parallel pieces on an
// I/O pool) into slot k%3's pinned buffer, then queues H2D -> kernel -> D2H on
// the slot's stream; a writer thread waits for the slot's event and pwritev()s
// all 14 (or the rebuilt) shard files in parallel on the pool. Reading job
// k+1, the GPU work of job k and the writes of job k-1 overlap.
#include <fcntl.h>
#include <sys/stat.h>
#include <sys/vfs.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cerrno>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <future>
#include <map>
#include <string>
#include <chrono>
#include <thread>

#include "hec_internal.hpp"

namespace hec {
namespace {

constexpr int K = 10, M = 4, N = 14;
constexpr int kSlots = 3;                      // pipeline depth (profiles/r01/ab_file_pipeline_depth.txt)
constexpr uint64_t kBatchBytes = 256ull << 20;  // data bytes per GPU job
constexpr uint64_t kLargeSlice = 16ull << 20;   // per-shard slice of a large row
constexpr int kIoThreads = 16;

std::string shard_name(const std::string& base, int i) {
    char ext[8];
    std::snprintf(ext, sizeof ext, ".ec%02d", i);  // to_ext, helyim-ec/src/lib.rs:84-86
    return base + ext;
}

struct Fd {
    int fd = -1;
    ~Fd() {
        if (fd >= 0) ::close(fd);
    }
};

// ---------------------------------------------------------------------------
// First-error record shared by the pipeline's threads.
// ---------------------------------------------------------------------------
struct ErrorSlot {
    std::mutex mu;
    std::atomic<int> code{HEC_OK};
    std::string detail;
    ErrorValues values;  // hec_last_error_values of the first failure
    void set(int c, const std::string& d, const ErrorValues& v = ErrorValues{}) {
        std::lock_guard<std::mutex> lk(mu);
        if (code.load() == HEC_OK) {
            detail = d;
            values = v;
            code.store(c);
        }
    }
    bool failed() const { return code.load() != HEC_OK; }
};

void io_error(ErrorSlot& e, const std::string& what) {
    const int err = errno;
    ErrorValues v;
    v.os_errno = err;
    e.set(HEC_ERR_IO, what + ": " + std::strerror(err), v);
}

// ---------------------------------------------------------------------------
// Small fixed thread pool with fork/join task groups.
// ---------------------------------------------------------------------------
// The file layer's I/O and writer threads are left unbound: bound to the
// GPU's NUMA node a 12 GiB encode ran 25.3-28.6 GiB/s against 28.9-30.1
// unbound (profiles/r04/file_pool_bind_ab.jsonl) -- the .dat and shard pages
// in the page cache sit on whichever node, and these threads touch them more
// than the pinned slots.
class Pool {
   public:
    explicit Pool(int n) {
        for (int i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    // Run all tasks, return when every one finished.
    void run_all(std::vector<std::function<void()>>& tasks) {
        if (tasks.empty()) return;
        std::mutex dm;
        std::condition_variable dcv;
        size_t left = tasks.size();
        {
            std::lock_guard<std::mutex> lk(mu_);
            for (auto& t : tasks)
                q_.push_back([&, fn = std::move(t)] {
                    fn();
                    std::lock_guard<std::mutex> l2(dm);
                    if (--left == 0) dcv.notify_all();
                });
        }
        cv_.notify_all();
        std::unique_lock<std::mutex> lk(dm);
        dcv.wait(lk, [&] { return left == 0; });
        tasks.clear();
    }

   private:
    void loop() {
        for (;;) {
            std::function<void()> fn;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
                if (stop_ && q_.empty()) return;
                fn = std::move(q_.front());
                q_.pop_front();
            }
            fn();
        }
    }
    std::vector<std::thread> th_;
    std::deque<std::function<void()>> q_;
    std::mutex mu_;
    std::condition_variable cv_;
    bool stop_ = false;
};

// pread that loops over short reads and zero-fills past EOF (encoder.rs:169-189).
bool pread_zero(int fd, uint8_t* dst, uint64_t len, uint64_t off, ErrorSlot& e) {
    uint64_t got = 0;
    while (got < len) {
        ssize_t r = ::pread(fd, dst + got, len - got, off_t(off + got));
        if (r < 0) {
            if (errno == EINTR) continue;
            io_error(e, "read");
            return false;
        }
        if (r == 0) break;
        got += uint64_t(r);
    }
    if (got < len) std::memset(dst + got, 0, len - got);
    return true;
}

// pwritev of a gather list at a file offset, looping over short writes.
bool pwritev_all(int fd, std::vector<iovec> iov, uint64_t off, ErrorSlot& e) {
    size_t first = 0;
    while (first < iov.size()) {
        const int cnt = int(std::min<size_t>(iov.size() - first, 1024));
        ssize_t w = ::pwritev(fd, iov.data() + first, cnt, off_t(off));
        if (w < 0) {
            if (errno == EINTR) continue;
            io_error(e, "write");
            return false;
        }
        if (w == 0) {  // no progress on a non-empty write: fail instead of spinning (write_all's WriteZero)
            errno = EIO;
            io_error(e, "write: wrote zero bytes");
            return false;
        }
        off += uint64_t(w);
        while (w > 0 && first < iov.size()) {
            if (size_t(w) >= iov[first].iov_len) {
                w -= ssize_t(iov[first].iov_len);
                ++first;
            } else {
                iov[first].iov_base = static_cast<uint8_t*>(iov[first].iov_base) + w;
                iov[first].iov_len -= size_t(w);
                w = 0;
            }
        }
    }
    return true;
}

// ---------------------------------------------------------------------------
// One unit of pipelined work.
// ---------------------------------------------------------------------------
struct ReadSeg {
    int fd;
    uint64_t host_off, len, file_off;
};
struct WriteSeg {
    int fd;
    uint64_t file_off;
    std::vector<std::pair<uint64_t, uint64_t>> pieces;  // (host_off, len) in order
};
struct Copy {
    uint64_t host_off, dev_off, len;
};
struct Job {
    std::vector<ReadSeg> reads;
    std::vector<Copy> h2d, d2h;
    std::function<int(uint8_t* dev, hipStream_t)> kernel;
    std::vector<WriteSeg> writes;
    std::shared_future<void> write_gate;  // optional: writes start once it is ready
};

struct Slot {
    uint8_t* host = nullptr;
    uint8_t* dev = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    bool busy = false;
};

// Stage timing of the pipeline (HEC_FILE_TRACE=1: printed to stderr at each
// drain). Measurement only.
struct StageClock {
    std::atomic<int64_t> read_ns{0}, slot_wait_ns{0}, gpu_wait_ns{0}, write_ns{0}, submit_ns{0};
    static int64_t now() {
        return std::chrono::duration_cast<std::chrono::nanoseconds>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
    }
    void reset() { read_ns = slot_wait_ns = gpu_wait_ns = write_ns = submit_ns = 0; }
};

// Persistent per-device pipeline (one per GPU, reused by every file call so
// small volumes do not pay for pinned allocation, streams and threads).
class FilePipeline {
   public:
    FilePipeline() : pool_(kIoThreads) {}
    // Grow the slots to at least these sizes; call only while idle.
    int ensure(uint64_t host_bytes, uint64_t dev_bytes) {
        HEC_HIP(hipGetDevice(&dev_id_));
        for (auto& s : slots_) {
            if (!s.stream) {
                HEC_HIP(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
                HEC_HIP(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
            }
            if (host_bytes > host_cap_) {
                if (s.host) HEC_HIP(hipHostFree(s.host));
                s.host = nullptr;
                HEC_TRY(pinned_alloc(reinterpret_cast<void**>(&s.host), host_bytes));
            }
            if (dev_bytes > dev_cap_) {
                if (s.dev) HEC_HIP(hipFree(s.dev));
                s.dev = nullptr;
                HEC_HIP(hipMalloc(reinterpret_cast<void**>(&s.dev), dev_bytes));
            }
        }
        host_cap_ = std::max(host_cap_, host_bytes);
        dev_cap_ = std::max(dev_cap_, dev_bytes);
        if (!writer_.joinable())
            writer_ = std::thread([this] { writer_loop(); });
        return HEC_OK;
    }
    // Submit one job (blocks while its slot is still being written).
    void submit(Job job) {
        if (err_.failed()) return;
        const int si = int(next_++ % kSlots);
        Slot& s = slots_[si];
        int64_t t0 = StageClock::now();
        {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return !s.busy; });
            s.busy = true;
            ++inflight_;
        }
        int64_t t1 = StageClock::now();
        clk_.slot_wait_ns += t1 - t0;
        if (err_.failed()) return release(si);
        // reads in parallel pieces
        std::vector<std::function<void()>> tasks;
        for (const ReadSeg& r : job.reads)
            tasks.push_back([this, &s, r] {
                if (!err_.failed()) pread_zero(r.fd, s.host + r.host_off, r.len, r.file_off, err_);
            });
        pool_.run_all(tasks);
        int64_t t2 = StageClock::now();
        clk_.read_ns += t2 - t1;
        if (err_.failed()) return release(si);
        int rc = gpu(s, job);
        clk_.submit_ns += StageClock::now() - t2;
        if (rc) {
            err_.set(rc, hec_last_error_detail(), last_error_values());
            return release(si);
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            wq_.emplace_back(si, std::move(job));
        }
        cv_.notify_all();
    }
    // Wait until every submitted job is written; return (and clear) the first error.
    int drain() {
        {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [this] { return inflight_ == 0; });
        }
        static const bool trace = std::getenv("HEC_FILE_TRACE") != nullptr;
        if (trace)
            std::fprintf(stderr, "hec file pipeline: slot_wait %.3f s, read %.3f s, gpu_submit %.3f s, "
                                 "gpu_wait %.3f s, write %.3f s\n",
                         clk_.slot_wait_ns * 1e-9, clk_.read_ns * 1e-9, clk_.submit_ns * 1e-9,
                         clk_.gpu_wait_ns * 1e-9, clk_.write_ns * 1e-9);
        clk_.reset();
        int code = err_.code.load();
        std::string detail = err_.detail;
        const ErrorValues values = err_.values;
        err_.code.store(HEC_OK);
        err_.detail.clear();
        err_.values = ErrorValues{};
        return code ? fail_with(code, detail, values) : HEC_OK;
    }
    ErrorSlot& errors() { return err_; }

   private:
    int gpu(Slot& s, const Job& job) {
        for (const Copy& c : job.h2d)
            HEC_HIP(hipMemcpyAsync(s.dev + c.dev_off, s.host + c.host_off, c.len, hipMemcpyHostToDevice, s.stream));
        int rc = job.kernel(s.dev, s.stream);
        if (rc) return rc;
        for (const Copy& c : job.d2h)
            HEC_HIP(hipMemcpyAsync(s.host + c.host_off, s.dev + c.dev_off, c.len, hipMemcpyDeviceToHost, s.stream));
        HEC_HIP(hipEventRecord(s.done, s.stream));
        return HEC_OK;
    }
    void release(int si) {
        std::lock_guard<std::mutex> lk(mu_);
        slots_[si].busy = false;
        --inflight_;
        cv_.notify_all();
    }
    void writer_loop() {
        (void)hipSetDevice(dev_id_);
        for (;;) {
            std::pair<int, Job> w;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [this] { return !wq_.empty(); });
                w = std::move(wq_.front());
                wq_.pop_front();
            }
            Slot& s = slots_[w.first];
            const int64_t t0 = StageClock::now();
            hipError_t he = hipEventSynchronize(s.done);
            const int64_t t1 = StageClock::now();
            clk_.gpu_wait_ns += t1 - t0;
            if (he != hipSuccess) err_.set(HEC_ERR_HIP, std::string("hipEventSynchronize: ") + hipGetErrorString(he));
            if (w.second.write_gate.valid()) w.second.write_gate.wait();
            if (!err_.failed()) {
                std::vector<std::function<void()>> tasks;
                for (const WriteSeg& ws : w.second.writes)
                    tasks.push_back([this, &s, &ws] {
                        if (err_.failed()) return;
                        std::vector<iovec> iov;
                        for (auto& p : ws.pieces) iov.push_back(iovec{s.host + p.first, p.second});
                        pwritev_all(ws.fd, std::move(iov), ws.file_off, err_);
                    });
                pool_.run_all(tasks);
            }
            clk_.write_ns += StageClock::now() - t1;
            release(w.first);
        }
    }

    Pool pool_;
    Slot slots_[kSlots];
    std::thread writer_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::pair<int, Job>> wq_;
    uint64_t inflight_ = 0;
    uint64_t host_cap_ = 0, dev_cap_ = 0;
    uint64_t next_ = 0;
    int dev_id_ = 0;
    ErrorSlot err_;
    StageClock clk_;
};

// One pipeline per device, created on first use and intentionally never
// destroyed (its threads and HIP resources live for the process; a static
// destructor could run after the HIP runtime is gone).
struct PipelineLease {
    std::unique_lock<std::mutex> lock;
    FilePipeline* pipe = nullptr;
};
int lease_pipeline(uint64_t host_bytes, uint64_t dev_bytes, PipelineLease& out) {
    static std::mutex reg_mu;
    static std::map<int, std::pair<std::mutex*, FilePipeline*>>* reg =
        new std::map<int, std::pair<std::mutex*, FilePipeline*>>();
    int dev;
    int rc = current_device(&dev);
    if (rc) return rc;
    std::pair<std::mutex*, FilePipeline*> e;
    {
        std::lock_guard<std::mutex> lk(reg_mu);
        auto& slot = (*reg)[dev];
        if (!slot.first) slot = {new std::mutex(), new FilePipeline()};
        e = slot;
    }
    out.lock = std::unique_lock<std::mutex>(*e.first);  // one file operation per device at a time
    out.pipe = e.second;
    return e.second->ensure(host_bytes, dev_bytes);
}

struct Rs104 {
    hec_rs_t* rs = nullptr;
    ~Rs104() { hec_rs_free(rs); }
};

// Reserve the final size of freshly created output files, one fallocate per
// file on its own thread, while the first jobs are read and coded: the
// returned future gates the pipeline's writes. FALLOC_FL_KEEP_SIZE leaves the
// visible size to the writes, so a failed call leaves the bytes the reference
// would. Speed only: the filesystem allocates each file in one call instead of
// block by block inside the writes (re-encoding a 4 GiB volume over its old
// shards on the box's overlay filesystem: 0.16 s with, 0.54-0.78 s without).
// Skipped on tmpfs, where fallocate zero-fills the page cache up front and
// the writes then copy over it (12 GiB volume in /dev/shm: 0.37-0.40 s fresh
// without, 0.47-0.65 s with; profiles/r01/ab_prealloc.txt). Filesystems without
// fallocate are skipped silently.
std::shared_future<void> preallocate_async(const int* fds, int n, uint64_t bytes) {
    if (bytes == 0) return {};
    constexpr long kTmpfsMagic = 0x01021994;
    std::vector<int> v;
    for (int i = 0; i < n; ++i) {
        if (fds[i] < 0) continue;
        struct statfs st;
        if (::fstatfs(fds[i], &st) == 0 && long(st.f_type) == kTmpfsMagic) continue;
        v.push_back(fds[i]);
    }
    if (v.empty()) return {};
    return std::async(std::launch::async, [v, bytes] {
               std::vector<std::thread> th;
               for (int fd : v) th.emplace_back([fd, bytes] { (void)::fallocate(fd, FALLOC_FL_KEEP_SIZE, 0, off_t(bytes)); });
               for (auto& t : th) t.join();
           }).share();
}

// Open (create + truncate) the output files in parallel: truncating an
// existing multi-GiB shard file frees its pages, which is slow one file at a
// time. Same files and flags as the reference's sequential opens; on failure
// the lowest-numbered failing file is reported.
int open_outputs(const std::string& base, const bool* which, Fd* out) {
    std::vector<std::thread> th;
    int err[N];
    for (int i = 0; i < N; ++i) {
        err[i] = 0;
        if (which[i])
            th.emplace_back([&, i] {
                out[i].fd = ::open(shard_name(base, i).c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
                if (out[i].fd < 0) err[i] = errno;
            });
    }
    for (auto& t : th) t.join();
    for (int i = 0; i < N; ++i)
        if (which[i] && out[i].fd < 0)
            return fail_errno(HEC_ERR_IO, "open " + shard_name(base, i), err[i]);
    return HEC_OK;
}

// Split [off, off+len) into up to `parts` read pieces of whole `unit`s.
void add_reads(std::vector<ReadSeg>& v, int fd, uint64_t host_off, uint64_t len, uint64_t file_off, uint64_t unit,
               int parts) {
    uint64_t units = (len + unit - 1) / unit;
    uint64_t per = std::max<uint64_t>(1, (units + parts - 1) / parts) * unit;
    for (uint64_t o = 0; o < len; o += per) v.push_back({fd, host_off + o, std::min(per, len - o), file_off + o});
}

// One job of the staged pipeline over b whole small rows at .dat offset
// `processed` (encoder.rs:228-239): whole rows are contiguous in .dat.
Job small_rows_job(int dat_fd, const Fd* out, const DevicePlanSet* enc, uint64_t processed, uint64_t out_off,
                   uint64_t b, uint64_t small, uint64_t data_cap, const std::shared_future<void>& gate) {
    const uint64_t small_row = small * K;
    Job job;
    add_reads(job.reads, dat_fd, 0, b * small_row, processed, small, kIoThreads);
    job.h2d.push_back({0, 0, b * small_row});
    // parity device/host layout [4][b][small]: each parity file gets one contiguous piece
    job.kernel = [=](uint8_t* d, hipStream_t s) {
        return run_apply(*enc, K, d, small_row, small, d + data_cap, small, b * small, small, uint32_t(b),
                         nullptr, nullptr, s);
    };
    job.d2h.push_back({data_cap, data_cap, b * small * M});
    for (int j = 0; j < K; ++j) {
        WriteSeg ws{out[j].fd, out_off, {}};
        for (uint64_t r = 0; r < b; ++r) ws.pieces.push_back({r * small_row + j * small, small});
        job.writes.push_back(std::move(ws));
    }
    for (int j = 0; j < M; ++j) job.writes.push_back({out[K + j].fd, out_off, {{data_cap + j * b * small, b * small}}});
    job.write_gate = gate;
    return job;
}

}  // namespace

static int write_ec_files_impl(const std::string& base, uint64_t buf_size, uint64_t large, uint64_t small) {
    // generate_ec_files: open .dat read-only (encoder.rs:58-62)
    Fd dat;
    dat.fd = ::open((base + ".dat").c_str(), O_RDONLY);
    if (dat.fd < 0) return fail_errno(HEC_ERR_IO, "open " + base + ".dat", errno);
    struct stat st;
    if (::fstat(dat.fd, &st) != 0) return fail_errno(HEC_ERR_IO, "stat .dat", errno);
    int64_t remaining = int64_t(st.st_size);

    Rs104 rs;  // ReedSolomon::new(10, 4) (encoder.rs:208-209)
    int rc = hec_rs_new(K, M, &rs.rs);
    if (rc) return rc;
    if (buf_size == 0) return fail(HEC_ERR_INVALID_ARGUMENT, "zero buffer size");

    Fd out[N];  // open_ec_files(base, false): create + truncate (encoder.rs:111-127)
    {
        bool all[N];
        std::fill(all, all + N, true);
        if ((rc = open_outputs(base, all, out))) return rc;
    }
    const uint64_t large_row = large * K, small_row = small * K;
    // the reference checks block % buf at the first row of each kind (encoder.rs:139-144)
    const bool has_large = remaining > int64_t(large_row);
    if (has_large && large % buf_size != 0)
        return fail_values(HEC_ERR_UNEXPECTED_BLOCK_SIZE,
                           "unexpected block size " + std::to_string(large) + ", buffer size " + std::to_string(buf_size),
                           large, buf_size);
    // rows of each kind, to size the staging buffers no larger than needed
    const uint64_t n_large = has_large ? (uint64_t(remaining) - 1) / large_row : 0;
    const int64_t small_bytes = remaining - int64_t(n_large * large_row);
    const uint64_t n_small = small_bytes > 0 ? (uint64_t(small_bytes) + small_row - 1) / small_row : 0;
    GeomDevice* gd;
    if ((rc = geom_device(rs.rs, &gd))) return rc;
    std::shared_future<void> prealloc;
    {
        int fds[N];
        for (int i = 0; i < N; ++i) fds[i] = out[i].fd;
        prealloc = preallocate_async(fds, N, n_large * large + n_small * small);
    }

    const uint64_t T = n_large ? std::min<uint64_t>(large, kLargeSlice) : 0;                    // large-row slice
    const uint64_t B = std::min(n_small, std::max<uint64_t>(1, kBatchBytes / small_row));  // small rows per job
    const uint64_t data_cap = (std::max(T * K, B * small_row) + 255) / 256 * 256;
    const uint64_t par_cap = std::max<uint64_t>(256, std::max(T * M, B * small * M));
    PipelineLease lease;
    if ((rc = lease_pipeline(data_cap + par_cap, data_cap + par_cap, lease))) return rc;
    FilePipeline& pipe = *lease.pipe;
    const DevicePlanSet* enc = &gd->encode;

    uint64_t out_off = 0;    // current size of every shard file
    uint64_t processed = 0;  // .dat offset of the current row

    // Large rows (encoder.rs:215-226): block j of the row = .dat[row + j*large, +large)
    while (remaining > int64_t(large_row) && !pipe.errors().failed()) {
        for (uint64_t t = 0; t < large; t += T) {
            const uint64_t n = std::min(T, large - t);
            Job job;
            for (int j = 0; j < K; ++j)
                add_reads(job.reads, dat.fd, j * n, n, processed + j * large + t, 1 << 20, 2);
            job.h2d.push_back({0, 0, n * K});
            job.kernel = [=](uint8_t* d, hipStream_t s) {
                return run_apply(*enc, K, d, 0, n, d + data_cap, 0, n, n, 1, nullptr, nullptr, s);
            };
            job.d2h.push_back({data_cap, data_cap, n * M});
            for (int j = 0; j < K; ++j) job.writes.push_back({out[j].fd, out_off + t, {{j * n, n}}});
            for (int j = 0; j < M; ++j) job.writes.push_back({out[K + j].fd, out_off + t, {{data_cap + j * n, n}}});
            job.write_gate = prealloc;
            pipe.submit(std::move(job));
        }
        out_off += large;
        processed += large_row;
        remaining -= int64_t(large_row);
    }

    // Small rows (encoder.rs:228-239): whole rows are contiguous in .dat.
    if (remaining > 0 && small % buf_size != 0 && !pipe.errors().failed()) {
        int frc = pipe.drain();
        if (frc) return frc;
        return fail_values(HEC_ERR_UNEXPECTED_BLOCK_SIZE,
                           "unexpected block size " + std::to_string(small) + ", buffer size " + std::to_string(buf_size),
                           small, buf_size);
    }
    while (remaining > 0 && !pipe.errors().failed()) {
        const uint64_t rows_left = (uint64_t(remaining) + small_row - 1) / small_row;
        const uint64_t b = std::min(rows_left, B);
        pipe.submit(small_rows_job(dat.fd, out, enc, processed, out_off, b, small, data_cap, prealloc));
        out_off += b * small;
        processed += b * small_row;
        remaining -= int64_t(b * small_row);
    }
    return pipe.drain();
}

static int rebuild_ec_files_impl(const std::string& base, uint32_t* ids, size_t* n_ids) {
    // generate_missing_ec_files (encoder.rs:73-109)
    bool has[N];
    Fd in[N], out[N];
    std::vector<uint32_t> rebuilt;
    for (int i = 0; i < N; ++i) {
        const std::string name = shard_name(base, i);
        struct stat st;
        if (::stat(name.c_str(), &st) == 0) {
            has[i] = true;
            in[i].fd = ::open(name.c_str(), O_RDONLY);
            if (in[i].fd < 0) return fail_errno(HEC_ERR_IO, "open " + name, errno);
        } else {
            if (errno != ENOENT) return fail_errno(HEC_ERR_IO, "stat " + name, errno);
            has[i] = false;
            out[i].fd = ::open(name.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
            if (out[i].fd < 0) return fail_errno(HEC_ERR_IO, "open " + name, errno);
            rebuilt.push_back(uint32_t(i));
        }
    }

    // rebuild_ec_files_inner (encoder.rs:244-307). Row sizes are decided by
    // the present files' sizes exactly as the reference's read_at sequence
    // decides them: n = min(1 MiB, size - offset); stop at the first n == 0;
    // every n must equal the first one (UnexpectedEcShardSize).
    Rs104 rs;
    int rc = hec_rs_new(K, M, &rs.rs);
    if (rc) return rc;
    const uint64_t SB = HEC_SMALL_BLOCK_SIZE;
    uint64_t size[N];
    int npresent = 0;
    for (int i = 0; i < N; ++i) {
        size[i] = 0;
        if (!has[i]) continue;
        ++npresent;
        struct stat st;
        if (::fstat(in[i].fd, &st) != 0) return fail_errno(HEC_ERR_IO, "stat shard", errno);
        size[i] = uint64_t(st.st_size);
    }
    uint64_t row_size = 0;  // input_buffer_data_size
    uint64_t rows = 0;
    int end_rc = HEC_OK;
    std::string end_detail;
    uint64_t end_expected = 0, end_actual = 0;  // UnexpectedEcShardSize(expected, actual)
    for (;;) {
        const uint64_t start = rows * (row_size ? row_size : 1);
        bool stop = false;
        for (int i = 0; i < N && !stop && end_rc == HEC_OK; ++i) {
            if (!has[i]) continue;
            const uint64_t n = size[i] > start ? std::min(SB, size[i] - start) : 0;
            if (n == 0) {
                stop = true;
                break;
            }
            if (row_size == 0) row_size = n;
            if (row_size != n) {
                end_rc = HEC_ERR_UNEXPECTED_EC_SHARD_SIZE;
                end_detail = "ec shard size expected " + std::to_string(row_size) + " but actually is " +
                             std::to_string(n);
                end_expected = row_size;
                end_actual = n;
            }
        }
        if (stop || end_rc != HEC_OK) break;
        if (npresent < K) {  // reconstruct -> TooFewShardsPresent (encoder.rs:288)
            end_rc = HEC_ERR_TOO_FEW_SHARDS_PRESENT;
            break;
        }
        ++rows;
    }

    if (rows > 0 && npresent < N) {
        uint8_t present[N];
        for (int i = 0; i < N; ++i) present[i] = has[i] ? 1 : 0;
        Mat coefs;
        std::vector<uint32_t> in_ids, out_ids;
        bool noop = false;
        if ((rc = decode_plan(rs.rs, present, false, coefs, in_ids, out_ids, &noop))) return rc;
        HostPlans hp;
        hp.add(coefs, in_ids, out_ids);
        DevicePlanSet ps;
        struct PsGuard {
            DevicePlanSet& p;
            ~PsGuard() { p.release(); }
        } pg{ps};
        if ((rc = ps.upload(hp, nullptr, nullptr))) return rc;
        std::shared_future<void> prealloc;
        {
            int fds[N];
            for (int i = 0; i < N; ++i) fds[i] = has[i] ? -1 : out[i].fd;
            prealloc = preallocate_async(fds, N, rows * row_size);
        }
        const uint64_t B = std::max<uint64_t>(1, std::min<uint64_t>(rows, kBatchBytes / (K * row_size)));
        const uint64_t slot = B * row_size;  // bytes per shard slot: layout [14][B rows]
        PipelineLease lease;
        if ((rc = lease_pipeline(slot * N, slot * N, lease))) return rc;
        FilePipeline& pipe = *lease.pipe;
        const DevicePlanSet* psp = &ps;
        for (uint64_t r0 = 0; r0 < rows && !pipe.errors().failed(); r0 += B) {
            const uint64_t nr = std::min(B, rows - r0);
            const uint64_t off = r0 * row_size;
            Job job;
            for (uint32_t id : in_ids) {
                add_reads(job.reads, in[id].fd, id * slot, nr * row_size, off, row_size, 1);
                job.h2d.push_back({id * slot, id * slot, nr * row_size});
            }
            job.kernel = [=](uint8_t* d, hipStream_t s) {
                return run_apply(*psp, K, d, row_size, slot, d, row_size, slot, row_size, uint32_t(nr), nullptr,
                                 nullptr, s);
            };
            for (uint32_t id : out_ids) {
                job.d2h.push_back({id * slot, id * slot, nr * row_size});
                job.writes.push_back({out[id].fd, off, {{id * slot, nr * row_size}}});
            }
            job.write_gate = prealloc;
            pipe.submit(std::move(job));
        }
        if ((rc = pipe.drain())) return rc;
    }
    if (end_rc != HEC_OK) return fail_values(end_rc, end_detail, end_expected, end_actual);
    if (n_ids) *n_ids = rebuilt.size();
    if (ids)
        for (size_t i = 0; i < rebuilt.size(); ++i) ids[i] = rebuilt[i];
    return HEC_OK;
}

}  // namespace hec

extern "C" {

int hec_write_ec_files_ex(const char* base_filename, uint64_t buf_size, uint64_t large_block_size,
                          uint64_t small_block_size) {
    if (!base_filename || !large_block_size || !small_block_size)
        return hec::fail(HEC_ERR_INVALID_ARGUMENT, "bad argument");
    return hec::write_ec_files_impl(base_filename, buf_size, large_block_size, small_block_size);
}

int hec_write_ec_files(const char* base_filename) {
    // write_ec_files: buf 256 KiB, large 1 GiB, small 1 MiB (encoder.rs:39-46)
    return hec_write_ec_files_ex(base_filename, 256 * 1024, HEC_LARGE_BLOCK_SIZE, HEC_SMALL_BLOCK_SIZE);
}

int hec_rebuild_ec_files(const char* base_filename, uint32_t* rebuilt_ids, size_t* n_rebuilt) {
    if (!base_filename) return hec::fail(HEC_ERR_INVALID_ARGUMENT, "bad argument");
    return hec::rebuild_ec_files_impl(base_filename, rebuilt_ids, n_rebuilt);
}

}  // extern "C"

// File-level drop-ins for helyim_ec::write_ec_files / rebuild_ec_files
// (/root/reference/helyim-ec/src/encoder.rs:39-307), GPU-backed.
//
// Byte layout is exactly the reference's: rows of 10 blocks (1 GiB blocks
// while more than 10 GiB remain -- strict '>' at encoder.rs:215 -- then 1 MiB
// blocks while anything remains, encoder.rs:228), short reads zero-filled
// (encoder.rs:169-189), shard file j = concatenation of block j of every row.
// The reference's 256 KiB buffer only sets its I/O granularity (bytes are
// position-wise independent), so here whole batches of rows go through the
// GPU at once: pread -> pinned host -> H2D -> kernel -> D2H -> pwrite.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <string>

#include "hec_internal.hpp"

namespace hec {
namespace {

constexpr int K = 10, M = 4, N = 14;
constexpr uint64_t kBatchBytes = 256ull << 20;  // data bytes per GPU batch
constexpr uint64_t kLargeSlice = 16ull << 20;   // per-shard slice of a large row

std::string shard_name(const std::string& base, int i) {
    char ext[8];
    std::snprintf(ext, sizeof ext, ".ec%02d", i);  // to_ext, helyim-ec/src/lib.rs:84-86
    return base + ext;
}

int io_fail(const std::string& what) { return fail(HEC_ERR_IO, what + ": " + std::strerror(errno)); }

struct Fd {
    int fd = -1;
    ~Fd() {
        if (fd >= 0) ::close(fd);
    }
};

struct Pinned {
    uint8_t* p = nullptr;
    ~Pinned() {
        if (p) (void)hipHostFree(p);
    }
};

struct DevBuf {
    uint8_t* p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

// pread that loops over short reads and zero-fills past EOF (encoder.rs:169-189).
int pread_zero(int fd, uint8_t* dst, uint64_t len, uint64_t off) {
    uint64_t got = 0;
    while (got < len) {
        ssize_t r = ::pread(fd, dst + got, len - got, off_t(off + got));
        if (r < 0) {
            if (errno == EINTR) continue;
            return io_fail("read");
        }
        if (r == 0) break;
        got += uint64_t(r);
    }
    if (got < len) std::memset(dst + got, 0, len - got);
    return HEC_OK;
}

int pwrite_all(int fd, const uint8_t* src, uint64_t len, uint64_t off) {
    uint64_t put = 0;
    while (put < len) {
        ssize_t w = ::pwrite(fd, src + put, len - put, off_t(off + put));
        if (w < 0) {
            if (errno == EINTR) continue;
            return io_fail("write");
        }
        put += uint64_t(w);
    }
    return HEC_OK;
}

struct Rs104 {
    hec_rs_t* rs = nullptr;
    ~Rs104() { hec_rs_free(rs); }
};

}  // namespace

static int write_ec_files_impl(const std::string& base, uint64_t buf_size, uint64_t large, uint64_t small) {
    // generate_ec_files: open .dat read-only (encoder.rs:58-62)
    Fd dat;
    dat.fd = ::open((base + ".dat").c_str(), O_RDONLY);
    if (dat.fd < 0) return io_fail("open " + base + ".dat");
    struct stat st;
    if (::fstat(dat.fd, &st) != 0) return io_fail("stat .dat");
    int64_t remaining = int64_t(st.st_size);

    Rs104 rs;  // ReedSolomon::new(10, 4) (encoder.rs:208-209)
    int rc = hec_rs_new(K, M, &rs.rs);
    if (rc) return rc;
    if (buf_size == 0) return fail(HEC_ERR_INVALID_ARGUMENT, "zero buffer size");

    Fd out[N];  // open_ec_files(base, false): create + truncate (encoder.rs:111-127)
    for (int i = 0; i < N; ++i) {
        out[i].fd = ::open(shard_name(base, i).c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
        if (out[i].fd < 0) return io_fail("open " + shard_name(base, i));
    }
    GeomDevice* gd;
    if ((rc = geom_device(rs.rs, &gd))) return rc;
    hipStream_t s;
    HEC_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    struct StreamGuard {
        hipStream_t s;
        ~StreamGuard() { (void)hipStreamDestroy(s); }
    } sg{s};

    // Host/device staging sized for one batch (whole small rows, or a slice
    // of one large row).
    const uint64_t per_shard_cap = std::max<uint64_t>(small, std::min<uint64_t>(large, kLargeSlice));
    uint64_t small_rows_per_batch = std::max<uint64_t>(1, kBatchBytes / (uint64_t(K) * small));
    uint64_t data_cap = std::max<uint64_t>(per_shard_cap * K, small_rows_per_batch * K * small);
    Pinned hdata, hpar;
    DevBuf ddata, dpar;
    HEC_HIP(hipHostMalloc(reinterpret_cast<void**>(&hdata.p), data_cap, hipHostMallocDefault));
    HEC_HIP(hipHostMalloc(reinterpret_cast<void**>(&hpar.p), data_cap / K * M, hipHostMallocDefault));
    HEC_HIP(hipMalloc(reinterpret_cast<void**>(&ddata.p), data_cap));
    HEC_HIP(hipMalloc(reinterpret_cast<void**>(&dpar.p), data_cap / K * M));

    uint64_t out_off = 0;      // current size of every shard file
    uint64_t processed = 0;    // .dat offset of the current row
    const uint64_t large_row = large * K, small_row = small * K;

    // Large rows (encoder.rs:215-226): block j of the row = .dat[row + j*large, +large)
    while (remaining > int64_t(large_row)) {
        if (large % buf_size != 0) return fail(HEC_ERR_UNEXPECTED_BLOCK_SIZE,
                                               "unexpected block size " + std::to_string(large) +
                                                   ", buffer size " + std::to_string(buf_size));
        for (uint64_t t = 0; t < large; t += per_shard_cap) {
            const uint64_t T = std::min(per_shard_cap, large - t);
            for (int j = 0; j < K; ++j)
                if ((rc = pread_zero(dat.fd, hdata.p + j * T, T, processed + j * large + t))) return rc;
            HEC_HIP(hipMemcpyAsync(ddata.p, hdata.p, T * K, hipMemcpyHostToDevice, s));
            if ((rc = run_apply(gd->encode, K, ddata.p, 0, T, dpar.p, 0, T, T, 1, nullptr, nullptr, s))) return rc;
            HEC_HIP(hipMemcpyAsync(hpar.p, dpar.p, T * M, hipMemcpyDeviceToHost, s));
            HEC_HIP(hipStreamSynchronize(s));
            for (int j = 0; j < K; ++j)
                if ((rc = pwrite_all(out[j].fd, hdata.p + j * T, T, out_off + t))) return rc;
            for (int j = 0; j < M; ++j)
                if ((rc = pwrite_all(out[K + j].fd, hpar.p + j * T, T, out_off + t))) return rc;
        }
        out_off += large;
        processed += large_row;
        remaining -= int64_t(large_row);
    }

    // Small rows (encoder.rs:228-239): whole rows are contiguous in .dat.
    while (remaining > 0) {
        if (small % buf_size != 0) return fail(HEC_ERR_UNEXPECTED_BLOCK_SIZE,
                                               "unexpected block size " + std::to_string(small) +
                                                   ", buffer size " + std::to_string(buf_size));
        const uint64_t rows_left = (uint64_t(remaining) + small_row - 1) / small_row;
        const uint64_t B = std::min(rows_left, small_rows_per_batch);
        if ((rc = pread_zero(dat.fd, hdata.p, B * small_row, processed))) return rc;
        HEC_HIP(hipMemcpyAsync(ddata.p, hdata.p, B * small_row, hipMemcpyHostToDevice, s));
        if ((rc = run_apply(gd->encode, K, ddata.p, small_row, small, dpar.p, small * M, small, small,
                            uint32_t(B), nullptr, nullptr, s)))
            return rc;
        HEC_HIP(hipMemcpyAsync(hpar.p, dpar.p, B * small * M, hipMemcpyDeviceToHost, s));
        HEC_HIP(hipStreamSynchronize(s));
        for (uint64_t r = 0; r < B; ++r) {
            for (int j = 0; j < K; ++j)
                if ((rc = pwrite_all(out[j].fd, hdata.p + r * small_row + j * small, small, out_off + r * small)))
                    return rc;
            for (int j = 0; j < M; ++j)
                if ((rc = pwrite_all(out[K + j].fd, hpar.p + (r * M + j) * small, small, out_off + r * small)))
                    return rc;
        }
        out_off += B * small;
        processed += B * small_row;
        remaining -= int64_t(B * small_row);
    }
    return HEC_OK;
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
            if (in[i].fd < 0) return io_fail("open " + name);
        } else {
            if (errno != ENOENT) return io_fail("stat " + name);
            has[i] = false;
            out[i].fd = ::open(name.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
            if (out[i].fd < 0) return io_fail("open " + name);
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
        if (::fstat(in[i].fd, &st) != 0) return io_fail("stat shard");
        size[i] = uint64_t(st.st_size);
    }
    uint64_t row_size = 0;  // input_buffer_data_size
    uint64_t rows = 0;
    int end_rc = HEC_OK;
    std::string end_detail;
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
            }
        }
        if (stop || end_rc != HEC_OK) break;
        if (npresent < K) {  // reconstruct -> TooFewShardsPresent (encoder.rs:288)
            end_rc = HEC_ERR_TOO_FEW_SHARDS_PRESENT;
            break;
        }
        ++rows;
        if (npresent == N) {
            // reconstruct is a no-op; the loop only re-checks sizes.
            continue;
        }
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
        hipStream_t s;
        HEC_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        struct StreamGuard {
            hipStream_t s;
            ~StreamGuard() { (void)hipStreamDestroy(s); }
        } sg{s};
        DevicePlanSet ps;
        struct PsGuard {
            DevicePlanSet& p;
            ~PsGuard() { p.release(); }
        } pg{ps};
        if ((rc = ps.upload(hp, nullptr, s))) return rc;
        const uint64_t B = std::max<uint64_t>(1, std::min<uint64_t>(rows, kBatchBytes / (K * row_size)));
        const uint64_t slot = B * row_size;  // bytes per shard slot
        Pinned host;
        DevBuf dev;
        HEC_HIP(hipHostMalloc(reinterpret_cast<void**>(&host.p), slot * N, hipHostMallocDefault));
        HEC_HIP(hipMalloc(reinterpret_cast<void**>(&dev.p), slot * N));
        for (uint64_t r0 = 0; r0 < rows; r0 += B) {
            const uint64_t nr = std::min(B, rows - r0);
            const uint64_t off = r0 * row_size;
            for (uint32_t id : in_ids) {
                if ((rc = pread_zero(in[id].fd, host.p + id * slot, nr * row_size, off))) return rc;
                HEC_HIP(hipMemcpyAsync(dev.p + id * slot, host.p + id * slot, nr * row_size,
                                       hipMemcpyHostToDevice, s));
            }
            if ((rc = run_apply(ps, K, dev.p, row_size, slot, dev.p, row_size, slot, row_size, uint32_t(nr),
                                nullptr, nullptr, s)))
                return rc;
            for (uint32_t id : out_ids)
                HEC_HIP(hipMemcpyAsync(host.p + id * slot, dev.p + id * slot, nr * row_size,
                                       hipMemcpyDeviceToHost, s));
            HEC_HIP(hipStreamSynchronize(s));
            for (uint32_t id : out_ids)
                if ((rc = pwrite_all(out[id].fd, host.p + id * slot, nr * row_size, off))) return rc;
        }
    }
    if (end_rc != HEC_OK) return fail(end_rc, end_detail);
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

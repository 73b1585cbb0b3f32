// On-disk EC volume helpers around the hot path:
// host-side byte formats that the generate / rebuild / to-volume RPCs write
// next to the shard files. No GF arithmetic; plain POSIX I/O.
//
//   .ecx  sorted needle index   <- helyim-ec/src/encoder.rs:21-37 (write_sorted_file_from_index)
//                                  helyim-ec/src/needle/mod.rs:12-44 (SortedIndexMap)
//                                  helyim-common/src/types/needle.rs:119-160 (16-byte BE entries)
//   .ecj  deletion journal      <- helyim-ec/src/lib.rs:54-133 (rebuild_ecx_file)
//   .vif  volume info JSON      <- helyim-ec/src/volume_info.rs:121-132, helyim-store/src/server.rs:470-475
//   .dat / .idx from shards     <- helyim-ec/src/decoder.rs:22-180
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "hec_internal.hpp"

namespace hec {
namespace {

constexpr uint64_t kEntry = 16;  // NEEDLE_ENTRY_SIZE: u64 id, u32 offset/8, i32 size, big endian

int io(const std::string& what) { return fail_errno(HEC_ERR_IO, what, errno); }
int eof(const std::string& what) { return fail(HEC_ERR_IO, what + ": failed to fill whole buffer"); }

struct File {
    int fd = -1;
    ~File() {
        if (fd >= 0) ::close(fd);
    }
};

uint64_t be64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
    return v;
}
uint32_t be32(const uint8_t* p) { return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3]; }
void put_be64(uint8_t* p, uint64_t v) {
    for (int i = 7; i >= 0; --i, v >>= 8) p[i] = uint8_t(v);
}
void put_be32(uint8_t* p, uint32_t v) {
    for (int i = 3; i >= 0; --i, v >>= 8) p[i] = uint8_t(v);
}

bool read_all(int fd, std::vector<uint8_t>& out) {
    struct stat st;
    if (::fstat(fd, &st) != 0) return false;
    out.resize(size_t(st.st_size));
    size_t got = 0;
    while (got < out.size()) {
        ssize_t r = ::pread(fd, out.data() + got, out.size() - got, off_t(got));
        if (r < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        if (r == 0) break;
        got += size_t(r);
    }
    out.resize(got);
    return true;
}


bool write_all(int fd, const uint8_t* p, size_t n) {
    while (n) {
        ssize_t w = ::write(fd, p, n);
        if (w < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        if (w == 0) {  // no progress: fail (write_all's WriteZero) instead of spinning
            errno = EIO;
            return false;
        }
        p += w;
        n -= size_t(w);
    }
    return true;
}

bool exists(const std::string& name, int* err) {
    struct stat st;
    if (::stat(name.c_str(), &st) == 0) return true;
    *err = errno == ENOENT ? 0 : errno;
    return false;
}

// Size::is_deleted (helyim-common/src/types/needle.rs:62-65)
bool size_deleted(int32_t s) { return s < 0; }

// Size::actual_size: header 16 + size + checksum 4 + padding, where padding is
// 8 - ((16 + size + 4) % 8), i.e. 8 (not 0) when already aligned (needle.rs:67-74).
uint64_t actual_size(int32_t s) {
    const uint32_t body = 16u + uint32_t(s) + 4u;
    return uint64_t(body + (8u - body % 8u));
}

}  // namespace
}  // namespace hec

using namespace hec;

extern "C" {

// write_sorted_file_from_index(base, ext) (encoder.rs:21-37): replay base.idx
// (walk_index_file: whole 16-byte entries or UnexpectedEof; offset 0 or a
// deleted size removes the key, anything else sets it) and write the live
// entries sorted by needle id to base+ext.
int hec_write_sorted_file_from_index(const char* base_filename, const char* ext) {
    if (!base_filename || !ext) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    const std::string base(base_filename);
    File idx;
    idx.fd = ::open((base + ".idx").c_str(), O_RDONLY);
    if (idx.fd < 0) return io("open " + base + ".idx");
    std::vector<uint8_t> buf;
    if (!read_all(idx.fd, buf)) return io("read .idx");
    std::map<uint64_t, std::pair<uint32_t, int32_t>> live;
    const size_t whole = buf.size() / kEntry;
    for (size_t e = 0; e < whole; ++e) {
        const uint8_t* p = buf.data() + e * kEntry;
        const uint64_t key = be64(p);
        const uint32_t off = be32(p + 8);
        const int32_t size = int32_t(be32(p + 12));
        if (off == 0 || size_deleted(size))
            live.erase(key);
        else
            live[key] = {off, size};
    }
    if (buf.size() % kEntry) return eof("read .idx entry");
    File out;
    out.fd = ::open((base + ext).c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (out.fd < 0) return io("open " + base + ext);
    std::vector<uint8_t> o(live.size() * kEntry);
    size_t i = 0;
    for (auto& kv : live) {
        put_be64(&o[i], kv.first);
        put_be32(&o[i + 8], kv.second.first);
        put_be32(&o[i + 12], uint32_t(kv.second.second));
        i += kEntry;
    }
    if (!write_all(out.fd, o.data(), o.size())) return io("write " + base + ext);
    return HEC_OK;
}

// rebuild_ecx_file(base) (lib.rs:95-133): for every 8-byte BE needle id of
// base.ecj, binary-search base.ecx and overwrite the entry's size with the
// tombstone -1 (search_needle_from_sorted_index :54-82, mark_needle_deleted
// :88-93); ids not found are ignored; finally delete base.ecj. No .ecj -> Ok.
int hec_rebuild_ecx_file(const char* base_filename) {
    if (!base_filename) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    const std::string base(base_filename);
    const std::string ecj = base + ".ecj";
    int err = 0;
    if (!exists(ecj, &err)) {
        if (err) {
            errno = err;
            return io("stat " + ecj);
        }
        return HEC_OK;
    }
    File ecx, j;
    ecx.fd = ::open((base + ".ecx").c_str(), O_RDWR);
    if (ecx.fd < 0) return io("open " + base + ".ecx");
    struct stat st;
    if (::fstat(ecx.fd, &st) != 0) return io("stat .ecx");
    const uint64_t n_entries = uint64_t(st.st_size) / kEntry;
    j.fd = ::open(ecj.c_str(), O_RDWR);
    if (j.fd < 0) return io("open " + ecj);
    std::vector<uint8_t> ids;
    if (!read_all(j.fd, ids)) return io("read .ecj");
    uint8_t e[kEntry], tomb[4];
    put_be32(tomb, uint32_t(int32_t(-1)));  // TOMBSTONE_FILE_SIZE
    for (size_t p = 0; p + 8 <= ids.size(); p += 8) {  // a trailing partial id ends the loop
        const uint64_t want = be64(&ids[p]);
        uint64_t lo = 0, hi = n_entries;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) / 2;
            ssize_t r = ::pread(ecx.fd, e, kEntry, off_t(mid * kEntry));
            if (r != ssize_t(kEntry)) return r < 0 ? io("read .ecx") : eof("read .ecx");
            const uint64_t key = be64(e);
            if (key == want) {
                if (!pwrite_exact(ecx.fd, tomb, 4, off_t(mid * 16 + 8 + 4))) return io("write .ecx");
                break;
            }
            if (key < want)
                lo = mid + 1;
            else
                hi = mid;
        }
    }
    if (::unlink(ecj.c_str()) != 0) return io("remove " + ecj);
    return HEC_OK;
}

// save_volume_info(base.vif, VolumeInfo { version, ..Default }) as written by
// the generate RPC (server.rs:470-475): serde_json of the prost message
// (volume.proto:75-79), fields in declaration order.
int hec_save_volume_info(const char* filename, uint32_t version) {
    if (!filename) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    File f;
    f.fd = ::open(filename, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (f.fd < 0) return io(std::string("open ") + filename);
    const std::string json = "{\"files\":[],\"version\":" + std::to_string(version) + ",\"replication\":\"\"}";
    if (!write_all(f.fd, reinterpret_cast<const uint8_t*>(json.data()), json.size())) return io("write .vif");
    return HEC_OK;
}

// find_data_filesize(base) (decoder.rs:46-66): parse the superblock of .ec00
// (SuperBlock::parse: the TTL unit byte must be 0..6), then the largest
// offset*8 + actual_size over the live entries of .ecx.
int hec_find_data_filesize(const char* base_filename, uint64_t* out) {
    if (!base_filename || !out) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    const std::string base(base_filename);
    File ec0;
    ec0.fd = ::open((base + ".ec00").c_str(), O_RDONLY);
    if (ec0.fd < 0) return io("open " + base + ".ec00");
    uint8_t sb[8];
    ssize_t r = ::pread(ec0.fd, sb, 8, 0);
    if (r != 8) return r < 0 ? io("read superblock") : eof("read superblock");
    if (sb[3] > 6) return fail(HEC_ERR_IO, "Ttl error: invalid unit");
    File ecx;
    ecx.fd = ::open((base + ".ecx").c_str(), O_RDONLY);
    if (ecx.fd < 0) return io("open " + base + ".ecx");
    std::vector<uint8_t> buf;
    if (!read_all(ecx.fd, buf)) return io("read .ecx");
    uint64_t size = 0;
    for (size_t p = 0; p + kEntry <= buf.size(); p += kEntry) {  // iterate_ecx_file stops at EOF
        const int32_t s = int32_t(be32(&buf[p + 12]));
        if (size_deleted(s)) continue;
        // Offset::actual_offset is a u32 product (needle.rs:49-51); the release
        // profile (Cargo.toml:99-100) wraps it, so offsets >= 2^29 wrap here too.
        const uint64_t stop = uint64_t(uint32_t(be32(&buf[p + 8]) * 8u)) + actual_size(s);
        size = std::max(size, stop);
    }
    *out = size;
    return HEC_OK;
}

// write_data_file(base, size) (decoder.rs:142-180): .dat = data blocks of
// .ec00-.ec09 row by row. Large rows while size >= 10 GiB (note: >=, the
// encoder uses >), then 1 MiB blocks while size > 0, each read exactly.
int hec_write_data_file(const char* base_filename, int64_t data_filesize) {
    if (!base_filename) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    const std::string base(base_filename);
    File dat;
    dat.fd = ::open((base + ".dat").c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (dat.fd < 0) return io("open " + base + ".dat");
    File in[10];
    for (int i = 0; i < 10; ++i) {
        char ext[8];
        std::snprintf(ext, sizeof ext, ".ec%02d", i);
        in[i].fd = ::open((base + ext).c_str(), O_RDONLY);
        if (in[i].fd < 0) return io("open " + base + ext);
    }
    uint64_t pos[10] = {0};
    std::vector<uint8_t> buf(size_t(16) << 20);
    auto copy = [&](int i, uint64_t n) -> int {
        while (n) {
            const size_t c = size_t(std::min<uint64_t>(n, buf.size()));
            size_t got = 0;
            while (got < c) {
                ssize_t r = ::pread(in[i].fd, buf.data() + got, c - got, off_t(pos[i] + got));
                if (r < 0) {
                    if (errno == EINTR) continue;
                    return io("read shard");
                }
                if (r == 0) return eof("read shard");  // read_exact
                got += size_t(r);
            }
            if (!write_all(dat.fd, buf.data(), c)) return io("write .dat");
            pos[i] += c;
            n -= c;
        }
        return HEC_OK;
    };
    int rc;
    const int64_t L = int64_t(HEC_LARGE_BLOCK_SIZE), S = int64_t(HEC_SMALL_BLOCK_SIZE);
    while (data_filesize >= 10 * L) {
        for (int i = 0; i < 10; ++i) {
            if ((rc = copy(i, uint64_t(L)))) return rc;
            data_filesize -= L;
        }
    }
    while (data_filesize > 0) {
        for (int i = 0; i < 10; ++i) {
            const int64_t n = std::min(data_filesize, S);
            if (n > 0 && (rc = copy(i, uint64_t(n)))) return rc;
            data_filesize -= std::max<int64_t>(n, 0);
        }
    }
    return HEC_OK;
}

// write_index_file_from_ec_index(base) (decoder.rs:22-44): .idx = copy of
// .ecx followed by one deleted entry (offset 0, size -1) per .ecj id.
int hec_write_index_file_from_ec_index(const char* base_filename) {
    if (!base_filename) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    const std::string base(base_filename);
    File ecx, idx;
    ecx.fd = ::open((base + ".ecx").c_str(), O_RDONLY);
    if (ecx.fd < 0) return io("open " + base + ".ecx");
    idx.fd = ::open((base + ".idx").c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (idx.fd < 0) return io("open " + base + ".idx");
    std::vector<uint8_t> buf;
    if (!read_all(ecx.fd, buf)) return io("read .ecx");
    if (!write_all(idx.fd, buf.data(), buf.size())) return io("write .idx");
    const std::string ecj = base + ".ecj";
    int err = 0;
    if (!exists(ecj, &err)) {
        if (err) {
            errno = err;
            return io("stat " + ecj);
        }
        return HEC_OK;
    }
    File j;
    j.fd = ::open(ecj.c_str(), O_RDONLY);
    if (j.fd < 0) return io("open " + ecj);
    std::vector<uint8_t> ids;
    if (!read_all(j.fd, ids)) return io("read .ecj");
    std::vector<uint8_t> o;
    for (size_t p = 0; p + 8 <= ids.size(); p += 8) {
        uint8_t e[kEntry];
        put_be64(e, be64(&ids[p]));
        put_be32(e + 8, 0);
        put_be32(e + 12, uint32_t(int32_t(-1)));  // NeedleValue::deleted()
        o.insert(o.end(), e, e + kEntry);
    }
    if (!write_all(idx.fd, o.data(), o.size())) return io("write .idx");
    return HEC_OK;
}

}  // extern "C"

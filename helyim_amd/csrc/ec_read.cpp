// Needle reads from an EC volume: locate_data, the .ecx
// needle lookup and the degraded read that rebuilds intervals of lost shards.
//
//   locate_data / Interval        <- helyim-ec/src/locate.rs:1-100
//   find_needle_from_ecx          <- helyim-ec/src/volume/mod.rs:153-155, lib.rs:54-82
//   locate_ec_shard_needle        <- helyim-ec/src/volume/mod.rs:136-151
//   read_ec_shard_needle / _intervals / read_one_ec_shard_interval /
//   recover_one_remote_ec_shard_interval
//                                 <- helyim-store/src/erasure_coding/mod.rs:129-171,303-491
//
// The reference fetches other shards' intervals over gRPC; here the shards are
// the local base.ecNN files (a lost shard is a missing file), which is the
// same arithmetic with the network taken out. Every interval that needs
// recovery in one call is rebuilt in one GPU batch (hec_rs_reconstruct_batch).
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <memory>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "hec_internal.hpp"

namespace hec {
namespace {

constexpr uint64_t kDataShards = 10;  // DATA_SHARDS_COUNT
constexpr int kTotalShards = 14;
constexpr uint64_t kEntry = 16;  // NEEDLE_ENTRY_SIZE

int io(const std::string& what) { return fail_errno(HEC_ERR_IO, what, errno); }


uint64_t be64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
    return v;
}
uint32_t be32(const uint8_t* p) { return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3]; }

std::string shard_name(const std::string& base, int id) {
    char ext[8];
    std::snprintf(ext, sizeof ext, ".ec%02d", id);
    return base + ext;
}

// The base.ecNN files of one volume, opened once per call (missing = -1).
struct Shards {
    int fd[kTotalShards];
    uint64_t size[kTotalShards];
    Shards() {
        for (int i = 0; i < kTotalShards; ++i) fd[i] = -1, size[i] = 0;
    }
    ~Shards() {
        for (int f : fd)
            if (f >= 0) ::close(f);
    }
    int open(const std::string& base) {
        for (int i = 0; i < kTotalShards; ++i) {
            const std::string name = shard_name(base, i);
            fd[i] = ::open(name.c_str(), O_RDONLY);
            if (fd[i] < 0) {
                if (errno == ENOENT) continue;
                return io("open " + name);
            }
            struct stat st;
            if (::fstat(fd[i], &st) != 0) return io("stat " + name);
            size[i] = uint64_t(st.st_size);
        }
        return HEC_OK;
    }
    // EcVolume::shards[0].ecd_filesize: the first loaded shard, ids ascending
    int first() const {
        for (int i = 0; i < kTotalShards; ++i)
            if (fd[i] >= 0) return i;
        return -1;
    }
};

// pread until n bytes or EOF; returns bytes read or -1
ssize_t pread_full(int fd, uint8_t* p, size_t n, uint64_t off) {
    size_t got = 0;
    while (got < n) {
        ssize_t r = ::pread(fd, p + got, n - got, off_t(off + got));
        if (r < 0) {
            if (errno == EINTR) continue;
            return -1;
        }
        if (r == 0) break;
        got += size_t(r);
    }
    return ssize_t(got);
}

// locate_offset (locate.rs:74-94) + locate_offset_within_blocks (:96-100)
void locate_offset(uint64_t large, uint64_t small, uint64_t data_size, uint64_t offset, uint64_t* block_index,
                   bool* is_large, uint64_t* inner) {
    const uint64_t large_row_size = large * kDataShards;
    const uint64_t large_block_rows = data_size / (large * kDataShards);  // note: not locate_data's formula
    if (offset < large_block_rows * large_row_size) {
        *block_index = offset / large;
        *inner = offset % large;
        *is_large = true;
        return;
    }
    offset -= large_block_rows * large_row_size;
    *block_index = offset / small;
    *inner = offset % small;
    *is_large = false;
}

// locate_data (locate.rs:29-72)
int locate(uint64_t large, uint64_t small, uint64_t data_size, uint64_t offset, uint64_t size,
           std::vector<hec_interval>& out) {
    if (large == 0 || small == 0) return fail(HEC_ERR_INVALID_ARGUMENT, "block sizes must be > 0");
    uint64_t block_index, inner;
    bool is_large;
    locate_offset(large, small, data_size, offset, &block_index, &is_large, &inner);
    const uint64_t large_block_rows = (data_size + small * kDataShards) / (large * kDataShards);
    while (size > 0) {
        hec_interval iv{block_index, inner, 0, large_block_rows, is_large ? 1u : 0u, 0u};
        const uint64_t block_remaining = (is_large ? large : small) - inner;
        if (size <= block_remaining) {
            iv.size = size;
            out.push_back(iv);
            return HEC_OK;
        }
        iv.size = block_remaining;
        out.push_back(iv);
        size -= block_remaining;
        block_index += 1;
        if (is_large && block_index == large_block_rows * kDataShards) {
            is_large = false;
            block_index = 0;
        }
        inner = 0;
    }
    return HEC_OK;
}

uint64_t interval_offset(const hec_interval& iv, uint64_t large, uint64_t small) {
    uint64_t off = iv.inner_block_offset;
    const uint64_t row = iv.block_index / kDataShards;
    if (iv.is_large_block)
        off += row * large;
    else
        off += iv.large_block_rows * large + row * small;
    return off;
}

// base.ecx opened for lookups: search_needle_from_sorted_index (lib.rs:54-82).
struct Ecx {
    int fd = -1;
    uint64_t n = 0;
    std::string name;
    ~Ecx() {
        if (fd >= 0) ::close(fd);
    }
    int open(const std::string& base, bool writable = false) {
        name = base + ".ecx";
        fd = ::open(name.c_str(), writable ? O_RDWR : O_RDONLY);
        if (fd < 0) return io("open " + name);
        struct stat st;
        if (::fstat(fd, &st) != 0) return io("stat " + name);
        n = uint64_t(st.st_size) / kEntry;
        return HEC_OK;
    }
    // HEC_OK with the stored offset/size, -1 when absent, or an I/O status;
    // *entry = the matching entry's index
    int find(uint64_t id, uint32_t* offset, int32_t* size, uint64_t* entry = nullptr) const {
        uint64_t lo = 0, hi = n;
        uint8_t e[kEntry];
        while (lo < hi) {
            const uint64_t mid = (lo + hi) / 2;
            const ssize_t got = pread_full(fd, e, kEntry, mid * kEntry);
            if (got != ssize_t(kEntry))
                return got < 0 ? io("read " + name) : fail(HEC_ERR_IO, "read " + name + ": failed to fill whole buffer");
            const uint64_t key = be64(e);
            if (key == id) {
                *offset = be32(e + 8);
                *size = int32_t(be32(e + 12));
                if (entry) *entry = mid;
                return HEC_OK;
            }
            if (key < id)
                lo = mid + 1;
            else
                hi = mid;
        }
        return -1;
    }
};

// Offset::actual_offset (u32 product) and Size::actual_size (needle.rs:49-74)
uint64_t actual_offset(uint32_t off) { return uint64_t(uint32_t(off * 8u)); }
uint64_t actual_size(int32_t sz) {
    const uint32_t body = 16u + uint32_t(sz) + 4u;
    return uint64_t(uint32_t(body + (8u - body % 8u)));
}

const hec_rs* rs104() {
    static hec_rs_t* rs = [] {
        hec_rs_t* r = nullptr;
        hec_rs_new(10, 4, &r);
        return r;
    }();
    return rs;
}

// read_ec_shard_intervals over a list of (offset, size) ranges of the volume's
// data: ranges are located, local intervals pread, lost ones rebuilt in one
// batch. out receives the ranges' bytes back to back.
int read_ranges(const std::string& base, const Shards& sh, uint64_t large, uint64_t small, const uint64_t* offsets,
                const uint64_t* sizes, size_t n, uint8_t* out) {
    int rc;
    const int f = sh.first();
    if (f < 0) return fail(HEC_ERR_SHARD_NOT_FOUND, "no .ecNN shard file for " + base);
    const uint64_t data_size = sh.size[f] * kDataShards;  // volume/mod.rs:146
    struct Lost {
        int shard;
        uint64_t off, size;
        uint8_t* dst;
    };
    std::vector<Lost> lost;
    std::vector<CompactJob> jobs;
    std::vector<hec_interval> ivs;
    uint8_t* dst = out;
    // Intervals in the reference's order (read_ec_shard_intervals walks them
    // one by one with `?`, erasure_coding/mod.rs:311-325): the first interval
    // that fails decides the error. A local interval is read here; a lost one
    // is checked here -- recover_one_remote_ec_shard_interval counts another
    // shard as present when its read of the same range returns the full
    // length, i.e. its file reaches off + size (mod.rs:461), and fails with
    // TooFewShardsPresent below 10 -- and rebuilt later in one GPU batch.
    for (size_t r = 0; r < n; ++r) {
        ivs.clear();
        if ((rc = locate(large, small, data_size, offsets[r], sizes[r], ivs))) return rc;
        for (const hec_interval& iv : ivs) {
            const int id = int(iv.block_index % kDataShards);
            const uint64_t off = interval_offset(iv, large, small);
            if (sh.fd[id] >= 0) {  // local shard: read_exact_at
                const ssize_t got = pread_full(sh.fd[id], dst, iv.size, off);
                if (got < 0) return io("read " + shard_name(base, id));
                if (uint64_t(got) != iv.size)
                    return fail(HEC_ERR_IO, "read " + shard_name(base, id) + ": failed to fill whole buffer");
            } else {
                uint32_t mask = 0;
                for (int i = 0; i < kTotalShards; ++i)
                    if (i != id && sh.fd[i] >= 0 && sh.size[i] >= off + iv.size) mask |= 1u << i;
                if (__builtin_popcount(mask) < int(kDataShards))
                    return fail(HEC_ERR_TOO_FEW_SHARDS_PRESENT, "recovering shard " + std::to_string(id) +
                                                                    " interval at " + std::to_string(off) + ": " +
                                                                    std::to_string(__builtin_popcount(mask)) +
                                                                    " shards present");
                lost.push_back({id, off, iv.size, dst});
                jobs.push_back(CompactJob{iv.size, mask});
            }
            dst += iv.size;
        }
    }
    if (lost.empty()) return HEC_OK;
    // The decode reads the first 10 present shards of each lost interval,
    // pread straight into pinned staging; the rebuilt interval is copied to its
    // place in out.
    return compact_reconstruct_104(
        rs104(), jobs,
        [&](size_t j, int, int shard, uint8_t* dst) {
            const ssize_t got = pread_full(sh.fd[shard], dst, lost[j].size, lost[j].off);
            if (got == ssize_t(lost[j].size)) return int(HEC_OK);
            return got < 0 ? io("read " + shard_name(base, shard))
                           : fail(HEC_ERR_IO, "read " + shard_name(base, shard) + ": shard shrank during the read");
        },
        [&](size_t j, int shard, const uint8_t* src) {
            if (shard == lost[j].shard) std::memcpy(lost[j].dst, src, lost[j].size);
        },
        /*io_bound_fill=*/true);
}

int read_ranges(const std::string& base, uint64_t large, uint64_t small, const uint64_t* offsets,
                const uint64_t* sizes, size_t n, uint8_t* out) {
    Shards sh;
    int rc = sh.open(base);
    if (rc) return rc;
    return read_ranges(base, sh, large, small, offsets, sizes, n, out);
}

// read_ec_shard_needle's data path for one needle (erasure_coding/mod.rs:129-171)
int read_needle(const std::string& base, const Ecx& ecx, const Shards& sh, uint64_t large, uint64_t small,
                uint64_t needle_id, uint8_t* out, size_t cap, size_t* n_out) {
    *n_out = 0;
    uint32_t off;
    int32_t sz;
    int rc = ecx.find(needle_id, &off, &sz);
    if (rc < 0) return fail(HEC_ERR_IO, "Needle " + std::to_string(needle_id) + " is not found");
    if (rc) return rc;
    if (sz < 0)  // Size::is_deleted
        return fail(HEC_ERR_NEEDLE_NOT_FOUND, "Needle " + std::to_string(needle_id) + " not found");
    const uint64_t a_off = actual_offset(off), a_size = actual_size(sz);
    *n_out = size_t(a_size);
    if (a_size > cap)
        return fail(HEC_ERR_INVALID_ARGUMENT, "needle needs " + std::to_string(a_size) + " bytes, cap " +
                                                  std::to_string(cap));
    if (!out) return fail(HEC_ERR_INVALID_ARGUMENT, "null out");
    return read_ranges(base, sh, large, small, &a_off, &a_size, 1, out);
}

// Many needles: lookups, then every range in one read_ranges (one GPU batch).
int read_needles(const std::string& base, const Ecx& ecx, const Shards& sh, uint64_t large, uint64_t small,
                 const uint64_t* needle_ids, size_t n, uint8_t* out, size_t cap, uint64_t* out_offsets,
                 int* statuses) {
    std::vector<uint64_t> offs, sizes;
    uint64_t total = 0;
    for (size_t i = 0; i < n; ++i) {
        uint32_t off;
        int32_t sz;
        out_offsets[i] = total;
        int rc = ecx.find(needle_ids[i], &off, &sz);
        if (rc > 0) return rc;  // I/O error on .ecx
        if (rc < 0) {
            statuses[i] = HEC_ERR_IO;  // not in .ecx (io::ErrorKind::NotFound)
            continue;
        }
        if (sz < 0) {
            statuses[i] = HEC_ERR_NEEDLE_NOT_FOUND;
            continue;
        }
        statuses[i] = HEC_OK;
        offs.push_back(actual_offset(off));
        sizes.push_back(actual_size(sz));
        total += sizes.back();
    }
    out_offsets[n] = total;
    if (total > cap)
        return fail(HEC_ERR_INVALID_ARGUMENT, "needles need " + std::to_string(total) + " bytes, cap " +
                                                  std::to_string(cap));
    if (offs.empty()) return HEC_OK;
    if (!out) return fail(HEC_ERR_INVALID_ARGUMENT, "null out");
    return read_ranges(base, sh, large, small, offs.data(), sizes.data(), offs.size(), out);
}

// maybe_load_volume_info (helyim-ec/src/volume_info.rs:107-119): absent file
// -> none; a VolumeInfo whose `files` list is empty -> none; else its version.
// The JSON is the serde form hec_save_volume_info writes; only the two fields
// the decision needs are read.
int maybe_load_version(const std::string& filename, bool* found, uint32_t* version) {
    *found = false;
    const int fd = ::open(filename.c_str(), O_RDONLY);
    if (fd < 0) {
        if (errno == ENOENT) return HEC_OK;
        return io("open " + filename);
    }
    std::string text;
    char buf[4096];
    for (;;) {
        const ssize_t r = ::read(fd, buf, sizeof buf);
        if (r < 0 && errno == EINTR) continue;
        if (r < 0) {
            ::close(fd);
            return io("read " + filename);
        }
        if (r == 0) break;
        text.append(buf, size_t(r));
    }
    ::close(fd);
    auto skip_ws = [&](size_t i) {
        while (i < text.size() && (text[i] == ' ' || text[i] == '\n' || text[i] == '\t' || text[i] == '\r')) ++i;
        return i;
    };
    auto value_at = [&](const char* key) -> size_t {  // index of the value of "key", or npos
        const size_t k = text.find(std::string("\"") + key + "\"");
        if (k == std::string::npos) return k;
        size_t i = skip_ws(k + std::strlen(key) + 2);
        if (i >= text.size() || text[i] != ':') return std::string::npos;
        return skip_ws(i + 1);
    };
    const size_t fi = skip_ws(0);
    if (fi >= text.size() || text[fi] != '{') return fail(HEC_ERR_IO, filename + ": not a JSON object");
    const size_t files = value_at("files");
    if (files == std::string::npos || text.compare(files, 1, "[") != 0 ||
        (skip_ws(files + 1) < text.size() && text[skip_ws(files + 1)] == ']'))
        return HEC_OK;  // files empty (or defaulted): none
    const size_t v = value_at("version");
    uint32_t ver = 0;
    for (size_t i = v; v != std::string::npos && i < text.size() && text[i] >= '0' && text[i] <= '9'; ++i)
        ver = ver * 10 + uint32_t(text[i] - '0');
    *found = true;
    *version = ver;
    return HEC_OK;
}

}  // namespace
}  // namespace hec

using namespace hec;

// A mounted EC volume (EcVolume, helyim-ec/src/volume/mod.rs:30-171): .ecx
// and .ecj held open, every local base.ecNN mounted, block geometry fixed.
struct hec_ec_volume {
    std::string base;
    uint64_t large = 0, small = 0;
    Shards shards;
    Ecx ecx;
    int ecj_fd = -1;
    uint32_t version = 2;
    std::mutex mu;  // serialises deletes (.ecx tombstone + .ecj append)
    ~hec_ec_volume() {
        if (ecj_fd >= 0) ::close(ecj_fd);
    }
};

extern "C" {

int hec_locate_data(uint64_t large_block_len, uint64_t small_block_len, uint64_t data_size, uint64_t offset,
                    uint64_t size, hec_interval* out, size_t cap, size_t* n_out) {
    if (!n_out || (cap && !out)) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    std::vector<hec_interval> ivs;
    int rc = locate(large_block_len, small_block_len, data_size, offset, size, ivs);
    if (rc) return rc;
    *n_out = ivs.size();
    if (ivs.size() > cap)
        return fail(HEC_ERR_INVALID_ARGUMENT, "need " + std::to_string(ivs.size()) + " intervals, cap " +
                                                  std::to_string(cap));
    std::copy(ivs.begin(), ivs.end(), out);
    return HEC_OK;
}

uint32_t hec_interval_shard_id(const hec_interval* iv) { return iv ? uint32_t(iv->block_index % kDataShards) : 0; }

uint64_t hec_interval_offset(const hec_interval* iv, uint64_t large_block_size, uint64_t small_block_size) {
    return iv ? interval_offset(*iv, large_block_size, small_block_size) : 0;
}

int hec_find_needle_from_ecx(const char* base_filename, uint64_t needle_id, uint32_t* offset, int32_t* size) {
    if (!base_filename || !offset || !size) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    Ecx ecx;
    int rc = ecx.open(base_filename);
    if (rc) return rc;
    rc = ecx.find(needle_id, offset, size);
    if (rc < 0) return fail(HEC_ERR_IO, "Needle " + std::to_string(needle_id) + " is not found");  // ErrorKind::NotFound
    return rc;
}

int hec_read_ec_data(const char* base_filename, uint64_t large_block_size, uint64_t small_block_size,
                     const uint64_t* offsets, const uint64_t* sizes, size_t n_ranges, uint8_t* out) {
    if (!base_filename || (n_ranges && (!offsets || !sizes || !out)))
        return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    return read_ranges(base_filename, large_block_size, small_block_size, offsets, sizes, n_ranges, out);
}

int hec_read_ec_needle_ex(const char* base_filename, uint64_t large_block_size, uint64_t small_block_size,
                          uint64_t needle_id, uint8_t* out, size_t cap, size_t* n_out) {
    if (!base_filename || !n_out) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    *n_out = 0;
    Ecx ecx;
    int rc = ecx.open(base_filename);
    if (rc) return rc;
    Shards sh;
    if ((rc = sh.open(base_filename))) return rc;
    return read_needle(base_filename, ecx, sh, large_block_size, small_block_size, needle_id, out, cap, n_out);
}

int hec_read_ec_needles(const char* base_filename, uint64_t large_block_size, uint64_t small_block_size,
                        const uint64_t* needle_ids, size_t n, uint8_t* out, size_t cap, uint64_t* out_offsets,
                        int* statuses) {
    if (!base_filename || !out_offsets || !statuses || (n && !needle_ids))
        return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    Ecx ecx;
    int rc = ecx.open(base_filename);
    if (rc) return rc;
    Shards sh;
    if ((rc = sh.open(base_filename))) return rc;
    return read_needles(base_filename, ecx, sh, large_block_size, small_block_size, needle_ids, n, out, cap,
                        out_offsets, statuses);
}

int hec_ec_volume_open_ex(const char* base_filename, uint64_t large_block_size, uint64_t small_block_size,
                          hec_ec_volume_t** out) {
    if (!base_filename || !out) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    if (large_block_size == 0 || small_block_size == 0)
        return fail(HEC_ERR_INVALID_ARGUMENT, "block sizes must be > 0");
    std::unique_ptr<hec_ec_volume> v(new hec_ec_volume());
    v->base = base_filename;
    v->large = large_block_size;
    v->small = small_block_size;
    // EcVolume::new (volume/mod.rs:45-92): .ecx read-write, .ecj read-write + create
    int rc = v->ecx.open(v->base, true);
    if (rc) return rc;
    v->ecj_fd = ::open((v->base + ".ecj").c_str(), O_RDWR | O_CREAT, 0644);
    if (v->ecj_fd < 0) return fail_errno(HEC_ERR_IO, "open " + v->base + ".ecj", errno);
    // .vif: load the version, or write the default VolumeInfo (version 2)
    bool found = false;
    uint32_t ver = 0;
    if ((rc = maybe_load_version(v->base + ".vif", &found, &ver))) return rc;
    if (found) {
        v->version = ver;
    } else {
        struct stat st;
        if (::stat((v->base + ".vif").c_str(), &st) == 0 && !(st.st_mode & 0200))  // check_file: not writable
            return fail(HEC_ERR_IO, v->base + ".vif not writable.");
        if ((rc = hec_save_volume_info((v->base + ".vif").c_str(), 2))) return rc;
        v->version = 2;
    }
    // add_ec_shard for every local shard file (mounted by the store)
    if ((rc = v->shards.open(v->base))) return rc;
    *out = v.release();
    return HEC_OK;
}

int hec_ec_volume_open(const char* base_filename, hec_ec_volume_t** out) {
    return hec_ec_volume_open_ex(base_filename, uint64_t(1) << 30, uint64_t(1) << 20, out);
}

void hec_ec_volume_close(hec_ec_volume_t* vol) { delete vol; }

uint32_t hec_ec_volume_version(const hec_ec_volume_t* vol) { return vol ? vol->version : 0; }

uint32_t hec_ec_volume_shard_bits(const hec_ec_volume_t* vol) {
    uint32_t bits = 0;
    for (int i = 0; vol && i < kTotalShards; ++i)
        if (vol->shards.fd[i] >= 0) bits |= 1u << i;
    return bits;
}

int hec_ec_volume_find_needle(const hec_ec_volume_t* vol, uint64_t needle_id, uint32_t* offset, int32_t* size) {
    if (!vol || !offset || !size) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    const int rc = vol->ecx.find(needle_id, offset, size);
    if (rc < 0) return fail(HEC_ERR_IO, "Needle " + std::to_string(needle_id) + " is not found");
    return rc;
}

int hec_ec_volume_delete_needle(hec_ec_volume_t* vol, uint64_t needle_id) {
    if (!vol) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    std::lock_guard<std::mutex> lk(vol->mu);
    // delete_needle_from_ecx (volume/mod.rs:157-171): tombstone the size in .ecx
    // (mark_needle_deleted, lib.rs:88-93), then append the id to .ecj
    uint32_t off;
    int32_t sz;
    uint64_t entry = 0;
    int rc = vol->ecx.find(needle_id, &off, &sz, &entry);
    if (rc < 0) return fail(HEC_ERR_IO, "Needle " + std::to_string(needle_id) + " is not found");
    if (rc) return rc;
    const uint8_t tomb[4] = {0xFF, 0xFF, 0xFF, 0xFF};  // TOMBSTONE_FILE_SIZE = -1, big-endian
    if (!pwrite_exact(vol->ecx.fd, tomb, 4, off_t(entry * kEntry + 12))) return io("write " + vol->ecx.name);
    struct stat st;
    if (::fstat(vol->ecj_fd, &st) != 0) return io("stat " + vol->base + ".ecj");
    uint8_t id[8];
    for (int i = 0; i < 8; ++i) id[i] = uint8_t(needle_id >> (56 - 8 * i));
    if (!pwrite_exact(vol->ecj_fd, id, 8, st.st_size)) return io("write " + vol->base + ".ecj");
    return HEC_OK;
}

int hec_ec_volume_read_needle(hec_ec_volume_t* vol, uint64_t needle_id, uint8_t* out, size_t cap, size_t* n_out) {
    if (!vol || !n_out) return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    return read_needle(vol->base, vol->ecx, vol->shards, vol->large, vol->small, needle_id, out, cap, n_out);
}

int hec_ec_volume_read_needles(hec_ec_volume_t* vol, const uint64_t* needle_ids, size_t n, uint8_t* out, size_t cap,
                               uint64_t* out_offsets, int* statuses) {
    if (!vol || !out_offsets || !statuses || (n && !needle_ids))
        return fail(HEC_ERR_INVALID_ARGUMENT, "null argument");
    return read_needles(vol->base, vol->ecx, vol->shards, vol->large, vol->small, needle_ids, n, out, cap,
                        out_offsets, statuses);
}

int hec_read_ec_needle(const char* base_filename, uint64_t needle_id, uint8_t* out, size_t cap, size_t* n_out) {
    return hec_read_ec_needle_ex(base_filename, uint64_t(1) << 30, uint64_t(1) << 20, needle_id, out, cap, n_out);
}

}  // extern "C"

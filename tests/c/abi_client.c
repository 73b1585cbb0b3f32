/* Standalone C client of libhec: the C ABI (include/hec.h) driven from a
 * process with no Python and no PyTorch, the way a Rust `-sys` binding would
 * (INTEGRATION.md §1). Checked against the C oracle (oracle/rs_oracle.c, test
 * infrastructure only). Built and run by tests/test_c_client.py:
 *
 *   abi_client nogpu  -- no device: metadata calls work, compute calls fail
 *                        with a device status (HEC_ERR_NO_DEVICE / HEC_ERR_HIP)
 *   abi_client gpu D  -- bit-exact parity with the oracle: encode/verify over
 *                        ragged lengths, reconstruct / reconstruct_data of every
 *                        1..4-erasure pattern, the batched degraded read, one
 *                        host batch split over a repeated device list
 *                        (pageable and hec_host_alloc'd), and
 *                        write_ec_files / rebuild_ec_files in directory D, and
 *                        helyim's EcShardError payloads (hec_last_error_values).
 * Exit status 0 = all checks passed; prints one line per failed check. */
#define _POSIX_C_SOURCE 200809L /* truncate */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include "../../include/hec.h"

/* oracle/rs_oracle.c */
void* orc_rs_new(int k, int m);
void orc_rs_free(void* p);
void orc_encode(void* p, uint8_t* const* shards, size_t len, int simd);
int orc_reconstruct(void* p, uint8_t* const* shards, const uint8_t* present, size_t len, int data_only, int simd);
void orc_splitmix64_fill(uint64_t seed, uint8_t* out, size_t nbytes);
int orc_write_ec_files(const char* base, uint64_t buf_size, uint64_t large, uint64_t small, int simd);

static int g_fail = 0;
#define CHECK(cond, ...)                                   \
    do {                                                   \
        if (!(cond)) {                                     \
            ++g_fail;                                      \
            printf("FAIL %s:%d: ", __FILE__, __LINE__);    \
            printf(__VA_ARGS__);                           \
            printf(" [%s]\n", hec_last_error_detail());    \
        }                                                  \
    } while (0)

enum { K = 10, M = 4, N = 14 };

static uint8_t** alloc_stripe(size_t len) {
    uint8_t** s = calloc(N, sizeof *s);
    for (int i = 0; i < N; ++i) s[i] = calloc(len ? len : 1, 1);
    return s;
}
static void free_stripe(uint8_t** s) {
    for (int i = 0; i < N; ++i) free(s[i]);
    free(s);
}

static void check_metadata(hec_rs_t* rs) {
    CHECK(hec_rs_data_shard_count(rs) == K, "data_shard_count");
    CHECK(hec_rs_parity_shard_count(rs) == M, "parity_shard_count");
    CHECK(hec_rs_total_shard_count(rs) == N, "total_shard_count");
    CHECK(strstr(hec_version(), "gfx950") != NULL, "version %s", hec_version());
    CHECK(strcmp(hec_strerror(HEC_ERR_TOO_FEW_SHARDS_PRESENT),
                 "The number of shards present is smaller than number of parity shards, cannot reconstruct "
                 "missing shards") == 0, "strerror");
    hec_rs_t* bad = NULL;
    CHECK(hec_rs_new(0, 4, &bad) == HEC_ERR_TOO_FEW_DATA_SHARDS && !bad, "new(0,4)");
    CHECK(hec_rs_new(4, 0, &bad) == HEC_ERR_TOO_FEW_PARITY_SHARDS && !bad, "new(4,0)");
    CHECK(hec_rs_new(200, 57, &bad) == HEC_ERR_TOO_MANY_SHARDS && !bad, "new(200,57)");
    /* argument validation happens before any device work */
    uint8_t** s = alloc_stripe(8);
    size_t lens[N];
    for (int i = 0; i < N; ++i) lens[i] = 8;
    CHECK(hec_rs_encode(rs, s, lens, N - 1) == HEC_ERR_TOO_FEW_SHARDS, "encode 13 shards");
    CHECK(hec_rs_encode(rs, s, lens, N + 1) == HEC_ERR_TOO_MANY_SHARDS, "encode 15 shards");
    lens[3] = 7;
    CHECK(hec_rs_encode(rs, s, lens, N) == HEC_ERR_INCORRECT_SHARD_SIZE, "encode ragged");
    lens[3] = 8;
    lens[0] = 0;
    CHECK(hec_rs_encode(rs, s, lens, N) == HEC_ERR_EMPTY_SHARD, "encode empty");
    free_stripe(s);
}

static int run_nogpu(void) {
    hec_rs_t* rs = NULL;
    CHECK(hec_rs_new(K, M, &rs) == HEC_OK && rs, "new(10,4)");
    check_metadata(rs);
    uint8_t** s = alloc_stripe(64);
    size_t lens[N];
    for (int i = 0; i < N; ++i) lens[i] = 64;
    const int rc = hec_rs_encode(rs, s, lens, N);
    CHECK(rc == HEC_ERR_NO_DEVICE || rc == HEC_ERR_HIP, "encode without a device returned %d", rc);
    free_stripe(s);
    hec_rs_free(rs);
    return g_fail ? 1 : 0;
}

static void check_encode_reconstruct(hec_rs_t* rs, void* ors, size_t len, uint64_t seed) {
    uint8_t** ref = alloc_stripe(len);
    uint8_t** got = alloc_stripe(len);
    size_t lens[N];
    for (int i = 0; i < K; ++i) orc_splitmix64_fill(seed + i, ref[i], len);
    orc_encode(ors, ref, len, 0);
    for (int i = 0; i < N; ++i) {
        lens[i] = len;
        memcpy(got[i], ref[i], len);
        if (i >= K) memset(got[i], 0, len);
    }
    CHECK(hec_rs_encode(rs, got, lens, N) == HEC_OK, "encode len %zu", len);
    for (int i = K; i < N; ++i) CHECK(memcmp(got[i], ref[i], len) == 0, "parity %d len %zu", i, len);
    int ok = 0;
    CHECK(hec_rs_verify(rs, (const uint8_t* const*)got, lens, N, &ok) == HEC_OK && ok == 1, "verify");
    got[K + 1][len - 1] ^= 1;
    CHECK(hec_rs_verify(rs, (const uint8_t* const*)got, lens, N, &ok) == HEC_OK && ok == 0, "verify corrupt");
    got[K + 1][len - 1] ^= 1;

    /* every erasure pattern of 1..4 shards (1470), reconstruct and reconstruct_data */
    int patterns = 0;
    for (uint32_t mask = 0; mask < (1u << N); ++mask) {
        const int e = __builtin_popcount(mask);
        if (e < 1 || e > M) continue;
        ++patterns;
        uint8_t present[N];
        size_t plens[N];
        for (int i = 0; i < N; ++i) {
            present[i] = !((mask >> i) & 1);
            plens[i] = present[i] ? len : 0;
            if (!present[i]) memset(got[i], 0xA5, len);
        }
        const int data_only = patterns & 1;
        int rc = data_only ? hec_rs_reconstruct_data(rs, got, plens, present, N)
                           : hec_rs_reconstruct(rs, got, plens, present, N);
        CHECK(rc == HEC_OK, "reconstruct mask %#x rc %d", mask, rc);
        for (int i = 0; i < N; ++i) {
            if (data_only && i >= K && !present[i]) {
                uint8_t* want = calloc(len, 1);
                memset(want, 0xA5, len);
                CHECK(memcmp(got[i], want, len) == 0, "reconstruct_data touched parity %d", i);
                free(want);
                memcpy(got[i], ref[i], len);
            } else {
                CHECK(memcmp(got[i], ref[i], len) == 0, "mask %#x shard %d len %zu", mask, i, len);
            }
        }
    }
    CHECK(patterns == 1470, "pattern count %d", patterns);
    uint8_t present[N];
    size_t plens[N];
    for (int i = 0; i < N; ++i) {
        present[i] = i >= 5;
        plens[i] = present[i] ? len : 0;
    }
    CHECK(hec_rs_reconstruct(rs, got, plens, present, N) == HEC_ERR_TOO_FEW_SHARDS_PRESENT, "5 erasures");
    free_stripe(ref);
    free_stripe(got);
}

/* hec_rs_reconstruct_batch: S stripes of different lengths and patterns in one call */
static void check_batch(hec_rs_t* rs, void* ors) {
    enum { S = 37 };
    uint8_t** ref[S];
    uint8_t* bufs[S * N];
    size_t lens[S * N];
    uint8_t present[S * N];
    for (int s = 0; s < S; ++s) {
        const size_t len = 1 + (size_t)s * 997 + (s % 5) * 4096;
        ref[s] = alloc_stripe(len);
        for (int i = 0; i < K; ++i) orc_splitmix64_fill(1000 + 31 * s + i, ref[s][i], len);
        orc_encode(ors, ref[s], len, 0);
        const uint32_t mask = (0x1u << (s % N)) | (s % 3 ? 0x2000u >> (s % 7) : 0u);
        for (int i = 0; i < N; ++i) {
            present[s * N + i] = !((mask >> i) & 1);
            lens[s * N + i] = present[s * N + i] ? len : 0;
            bufs[s * N + i] = malloc(len);
            if (present[s * N + i]) memcpy(bufs[s * N + i], ref[s][i], len);
            else memset(bufs[s * N + i], 0, len);
        }
    }
    size_t bad = 12345;
    CHECK(hec_rs_reconstruct_batch(rs, bufs, lens, present, S, 0, &bad) == HEC_OK, "batch");
    for (int s = 0; s < S; ++s) {
        const size_t len = 1 + (size_t)s * 997 + (s % 5) * 4096;
        for (int i = 0; i < N; ++i) CHECK(memcmp(bufs[s * N + i], ref[s][i], len) == 0, "batch %d/%d", s, i);
    }
    /* a bad stripe in the middle: error names it, nothing written */
    present[20 * N + 0] = present[20 * N + 1] = present[20 * N + 2] = present[20 * N + 3] = present[20 * N + 4] = 0;
    CHECK(hec_rs_reconstruct_batch(rs, bufs, lens, present, S, 0, &bad) == HEC_ERR_TOO_FEW_SHARDS_PRESENT &&
              bad == 20, "batch bad index %zu", bad);
    for (int s = 0; s < S; ++s) {
        free_stripe(ref[s]);
        for (int i = 0; i < N; ++i) free(bufs[s * N + i]);
    }
}

/* hec_host_*_batch_multi: one [S][14][L] host batch split over the device
 * list {0,0,0} (three concurrent ranges on one GPU, each on its own host
 * thread and pipeline; an 8-GPU server lists 0..7), once in pageable memory
 * (pooled pinned staging), in hec_host_alloc'd memory and in one
 * hec_host_alloc_multi batch (ranges placed per device; both zero copy);
 * parity and a 0..5-erasure reconstruct against the C oracle. */
static void check_host_batch_multi(void* ors) {
    enum { S = 11 };
    const size_t L = 65536 + 5, stripe = (size_t)N * L;
    const int devs[3] = {0, 0, 0};
    hec_rs_t* rs = NULL;
    CHECK(hec_rs_new(K, M, &rs) == HEC_OK, "new");
    for (int pinned = 0; pinned < 3; ++pinned) {  /* pageable, hec_host_alloc, hec_host_alloc_multi */
        uint8_t* h = NULL;
        if (pinned == 1) CHECK(hec_host_alloc(S * stripe, (void**)&h) == HEC_OK && h, "host_alloc");
        else if (pinned == 2)
            CHECK(hec_host_alloc_multi(devs, 3, stripe, S, (void**)&h) == HEC_OK && h, "host_alloc_multi");
        else h = malloc(S * stripe);
        if (!h) return;
        uint8_t* want = malloc(S * stripe);
        for (int s = 0; s < S; ++s) {
            uint8_t* p[N];
            for (int i = 0; i < N; ++i) p[i] = want + s * stripe + i * L;
            for (int i = 0; i < K; ++i) orc_splitmix64_fill(7000 + 31 * s + i, p[i], L);
            orc_encode(ors, p, L, 0);
        }
        memcpy(h, want, S * stripe);
        for (int s = 0; s < S; ++s) memset(h + s * stripe + K * L, 0xEE, M * L);
        CHECK(hec_host_encode_batch_multi(rs, devs, 3, h, stripe, L, h + K * L, stripe, L, L, S) == HEC_OK,
              "encode_multi (pinned %d)", pinned);
        CHECK(memcmp(h, want, S * stripe) == 0, "encode_multi bytes (pinned %d)", pinned);
        uint32_t masks[S];
        for (int s = 0; s < S; ++s) {
            masks[s] = 0x3FFFu;
            for (int e = 0; e < s % 6; ++e) {  /* s % 6 erasures: 5 = too few present */
                const int i = (3 * s + 5 * e) % N;
                masks[s] &= ~(1u << i);
                memset(h + s * stripe + i * L, 0xA5, L);
            }
        }
        uint32_t bad = 99;
        CHECK(hec_host_reconstruct_batch_multi(rs, devs, 2, h, stripe, L, L, S, masks, &bad) == HEC_OK,
              "reconstruct_multi (pinned %d)", pinned);
        int want_bad = 0;
        for (int s = 0; s < S; ++s) {
            if (__builtin_popcount(masks[s]) < K) {
                ++want_bad;
                continue;
            }
            CHECK(memcmp(h + s * stripe, want + s * stripe, stripe) == 0, "reconstruct_multi stripe %d", s);
        }
        CHECK(bad == (uint32_t)want_bad, "bad stripes %u, want %d", bad, want_bad);
        const int bad_dev[2] = {0, 1 << 20};
        CHECK(hec_host_encode_batch_multi(rs, bad_dev, 2, h, stripe, L, h + K * L, stripe, L, L, S) ==
                  HEC_ERR_INVALID_ARGUMENT, "device out of range");
        if (pinned) hec_host_free(h);
        else free(h);
        free(want);
    }
    hec_rs_free(rs);
}

/* The call shape INTEGRATION.md §3 gives the degraded read
 * (helyim-store/src/erasure_coding/mod.rs:403-491): one needle read spans
 * several intervals, each on a shard that is gone; the reader fans in the
 * other shards' same ranges (a shard whose remote read fails stays None,
 * mod.rs:461-474) and, instead of one ReedSolomon::reconstruct per interval
 * (mod.rs:426), makes ONE hec_rs_reconstruct_batch over all of the needle's
 * intervals, then copies each interval's recovered shard out (mod.rs:486-488).
 * Checked against the C oracle's per-interval reconstruct. */
static void check_degraded_read_shape(hec_rs_t* rs, void* ors) {
    enum { NI = 5 };
    const size_t ilen[NI] = {1, 4096, 65536 + 3, 512, 1u << 20};
    const int lost[NI] = {3, 0, 9, 12, 5};      /* shard_id_to_recover */
    const int unavailable[NI] = {-1, 13, -1, 1, 10}; /* a survivor whose remote read failed */
    uint8_t* bufs[NI * N];
    size_t lens[NI * N];
    uint8_t present[NI * N];
    uint8_t* want[NI];
    for (int j = 0; j < NI; ++j) {
        uint8_t** full = alloc_stripe(ilen[j]);
        for (int i = 0; i < K; ++i) orc_splitmix64_fill(7000 + 19 * j + i, full[i], ilen[j]);
        orc_encode(ors, full, ilen[j], 0);
        want[j] = malloc(ilen[j]);
        memcpy(want[j], full[lost[j]], ilen[j]);
        for (int i = 0; i < N; ++i) {
            const int p = i != lost[j] && i != unavailable[j];
            present[j * N + i] = (uint8_t)p;
            lens[j * N + i] = p ? ilen[j] : 0;
            bufs[j * N + i] = calloc(1, ilen[j]);  /* upstream: vec![0; len] for None slots */
            if (p) memcpy(bufs[j * N + i], full[i], ilen[j]);
        }
        free_stripe(full);
    }
    size_t bad = 0;
    CHECK(hec_rs_reconstruct_batch(rs, bufs, lens, present, NI, 0, &bad) == HEC_OK, "degraded-read batch");
    for (int j = 0; j < NI; ++j) {
        /* buf.copy_from_slice(data[shard_id_to_recover]) */
        CHECK(memcmp(bufs[j * N + lost[j]], want[j], ilen[j]) == 0, "interval %d shard %d", j, lost[j]);
        /* and the same bytes as the oracle's per-interval reconstruct */
        uint8_t* o[N];
        uint8_t op[N];
        for (int i = 0; i < N; ++i) {
            o[i] = calloc(1, ilen[j]);
            op[i] = present[j * N + i];
            if (op[i]) memcpy(o[i], bufs[j * N + i], ilen[j]);
        }
        CHECK(orc_reconstruct(ors, o, op, ilen[j], 0, 0) == 0, "oracle reconstruct %d", j);
        for (int i = 0; i < N; ++i) {
            CHECK(memcmp(o[i], bufs[j * N + i], ilen[j]) == 0, "interval %d shard %d vs oracle", j, i);
            free(o[i]);
        }
        free(want[j]);
        for (int i = 0; i < N; ++i) free(bufs[j * N + i]);
    }
}

static int read_file(const char* path, uint8_t** out, size_t* n) {
    FILE* f = fopen(path, "rb");
    if (!f) return -1;
    fseek(f, 0, SEEK_END);
    *n = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    *out = malloc(*n ? *n : 1);
    const size_t got = fread(*out, 1, *n, f);
    fclose(f);
    return got == *n ? 0 : -1;
}

static void write_dat(const char* base, size_t size) {
    char p[4096];
    snprintf(p, sizeof p, "%s.dat", base);
    uint8_t* d = malloc(size);
    orc_splitmix64_fill(77, d, size);
    FILE* f = fopen(p, "wb");
    fwrite(d, 1, size, f);
    fclose(f);
    free(d);
}

static void check_files(const char* dir) {
    char a[4096], b[4096], pa[4200], pb[4200];
    snprintf(a, sizeof a, "%s/a", dir);
    snprintf(b, sizeof b, "%s/b", dir);
    const size_t size = 3 * 640 * 10 + 6400 * 2 + 123; /* large rows + small rows + tail */
    write_dat(a, size);
    write_dat(b, size);
    CHECK(hec_write_ec_files_ex(a, 16, 640, 32) == HEC_OK, "write_ec_files_ex");
    CHECK(orc_write_ec_files(b, 16, 640, 32, 0) == 0, "oracle write_ec_files");
    uint8_t* want[N];
    size_t want_n[N];
    for (int i = 0; i < N; ++i) {
        uint8_t* x;
        size_t nx;
        snprintf(pa, sizeof pa, "%s.ec%02d", a, i);
        snprintf(pb, sizeof pb, "%s.ec%02d", b, i);
        CHECK(read_file(pa, &x, &nx) == 0 && read_file(pb, &want[i], &want_n[i]) == 0, "read ec%02d", i);
        CHECK(nx == want_n[i] && memcmp(x, want[i], nx) == 0, "ec%02d differs", i);
        free(x);
    }
    /* lose four shards, rebuild them */
    const int lost[4] = {1, 6, 10, 13};
    for (int j = 0; j < 4; ++j) {
        snprintf(pa, sizeof pa, "%s.ec%02d", a, lost[j]);
        unlink(pa);
    }
    uint32_t ids[N];
    size_t n_ids = 0;
    CHECK(hec_rebuild_ec_files(a, ids, &n_ids) == HEC_OK && n_ids == 4, "rebuild n=%zu", n_ids);
    for (size_t j = 0; j < n_ids && j < 4; ++j) CHECK(ids[j] == (uint32_t)lost[j], "rebuilt id %u", ids[j]);
    for (int i = 0; i < N; ++i) {
        uint8_t* x;
        size_t nx;
        snprintf(pa, sizeof pa, "%s.ec%02d", a, i);
        CHECK(read_file(pa, &x, &nx) == 0 && nx == want_n[i] && memcmp(x, want[i], nx) == 0, "rebuilt ec%02d", i);
        free(x);
        free(want[i]);
    }
}

/* helyim's EcShardError payloads through hec_last_error_values
 * (helyim-ec/src/errors.rs:55-66): Io's errno, UnexpectedBlockSize(block, buf)
 * (encoder.rs:139-144) on the large-row and the small-row check, and -- with
 * a device -- UnexpectedEcShardSize(expected, actual) (encoder.rs:272-280)
 * from a rebuild whose third row is short after two rows were rebuilt. */
static void check_values(int code, uint64_t want_a, uint64_t want_b, int want_errno, const char* what) {
    uint64_t a = 7, b = 7;
    int e = 7;
    CHECK(hec_last_error_values(&a, &b, &e) == HEC_OK, "last_error_values");
    CHECK(a == want_a && b == want_b && e == want_errno, "%s (code %d): values (%llu, %llu, errno %d), want (%llu, %llu, %d)",
          what, code, (unsigned long long)a, (unsigned long long)b, e, (unsigned long long)want_a,
          (unsigned long long)want_b, want_errno);
}

static void check_file_errors(const char* dir, int with_gpu) {
    char base[4096], p[4200];
    snprintf(base, sizeof base, "%s/missing", dir);
    int rc = hec_write_ec_files(base);
    CHECK(rc == HEC_ERR_IO, "write_ec_files(missing) = %d", rc);
    check_values(rc, 0, 0, 2 /* ENOENT */, "missing .dat");

    snprintf(base, sizeof base, "%s/blk", dir);
    write_dat(base, 10 * 640 + 1); /* one large row (strict '>', encoder.rs:215) */
    rc = hec_write_ec_files_ex(base, 24, 640, 32);
    CHECK(rc == HEC_ERR_UNEXPECTED_BLOCK_SIZE, "large-row block size: %d", rc);
    check_values(rc, 640, 24, 0, "large-row UnexpectedBlockSize");
    if (!with_gpu) return;

    write_dat(base, 100); /* small rows only: checked after the pipeline is set up */
    rc = hec_write_ec_files_ex(base, 24, 640, 32);
    CHECK(rc == HEC_ERR_UNEXPECTED_BLOCK_SIZE, "small-row block size: %d", rc);
    check_values(rc, 32, 24, 0, "small-row UnexpectedBlockSize");

    snprintf(base, sizeof base, "%s/trunc", dir);
    write_dat(base, 25000000); /* 3 rows of 1 MiB blocks: shard files of 3 MiB */
    CHECK(hec_write_ec_files(base) == HEC_OK, "write_ec_files(25 MB)");
    uint8_t* want3;
    size_t n3 = 0;
    snprintf(p, sizeof p, "%s.ec03", base);
    CHECK(read_file(p, &want3, &n3) == 0 && n3 == 3u << 20, "read ec03 (%zu)", n3);
    unlink(p);
    snprintf(p, sizeof p, "%s.ec00", base);
    CHECK(truncate(p, (2 << 20) + 5) == 0, "truncate ec00");
    uint32_t ids[N];
    size_t n_ids = 0;
    rc = hec_rebuild_ec_files(base, ids, &n_ids);
    CHECK(rc == HEC_ERR_UNEXPECTED_EC_SHARD_SIZE, "rebuild of a truncated shard: %d", rc);
    check_values(rc, 1u << 20, 5, 0, "UnexpectedEcShardSize");
    /* the two full rows were rebuilt before the short one was read, as upstream */
    uint8_t* got;
    size_t ng = 0;
    snprintf(p, sizeof p, "%s.ec03", base);
    CHECK(read_file(p, &got, &ng) == 0 && ng == 2u << 20 && memcmp(got, want3, ng) == 0,
          "rows rebuilt before the error (%zu bytes)", ng);
    free(got);
    free(want3);
}

int main(int argc, char** argv) {
    if (argc >= 2 && strcmp(argv[1], "nogpu") == 0) {
        if (argc >= 3) check_file_errors(argv[2], 0);
        return run_nogpu();
    }
    if (argc < 3 || strcmp(argv[1], "gpu") != 0) {
        fprintf(stderr, "usage: %s nogpu | gpu <tmpdir>\n", argv[0]);
        return 2;
    }
    hec_rs_t* rs = NULL;
    CHECK(hec_rs_new(K, M, &rs) == HEC_OK, "new(10,4)");
    void* ors = orc_rs_new(K, M);
    check_metadata(rs);
    const size_t lens[] = {1, 17, 4096, 65536 + 7};
    for (size_t j = 0; j < sizeof lens / sizeof lens[0]; ++j) check_encode_reconstruct(rs, ors, lens[j], 100 * j);
    check_batch(rs, ors);
    check_degraded_read_shape(rs, ors);
    check_host_batch_multi(ors);
    check_files(argv[2]);
    check_file_errors(argv[2], 1);
    orc_rs_free(ors);
    hec_rs_free(rs);
    printf("%s: %d failed checks\n", argv[0], g_fail);
    return g_fail ? 1 : 0;
}

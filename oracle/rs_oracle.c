/*
 * CPU oracle for the helyim-ec RS(10,4) hot path -- TEST INFRASTRUCTURE ONLY.
 *
 * Independent plain-C restatement of the arithmetic behind helyim-ec
 * (/root/reference/helyim-ec/src/encoder.rs:191,208-209,249-250,288), which
 * lives in the un-vendored crate reed-solomon-erasure 6.0.0 (git
 * helyim/reed-solomon-erasure, branch main, feature simd-accel;
 * /root/reference/Cargo.toml:72). Used by tests/ (bit-exact checker on the GPU
 * box), by bench.py's cpu_baseline leg (the timed CPU path, kind "port") and
 * by the measurement tools under tools/ (checker and CPU baseline).
 * Never linked into or called by the product library helyim_amd/libhec.so.
 *
 * Two encode kernels, selected by the caller:
 *   simd = 0 : scalar 256x256 MUL_TABLE lookups (upstream's non-SIMD path)
 *   simd = 1 : AVX2 16-entry low/high nibble product tables + vpshufb, the
 *              same algorithm class as upstream simd_c/reedsolomon.c
 *              (reedsolomon_gal_mul / reedsolomon_gal_mul_xor).
 * Loop order follows upstream code_some_slices: input-major, each output
 * slice mul (first input) or mul-xor (later inputs) over the whole slice.
 *
 * PARITY UNPINNED by the reference (it holds no EC tests or vectors and
 * cannot be built here). Checked against the upstream crate's published KATs
 * (tests/golden/upstream_kat.json) and cross-checked against
 * oracle/rs_oracle.py on the fixtures under tests/golden/.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <immintrin.h>

static uint8_t EXP[510];
static int LOG[256];
static uint8_t MUL[256][256];
static int g_init = 0;

static void init_tables(void) {
    if (g_init) return;
    int x = 1;
    for (int i = 0; i < 255; i++) {
        EXP[i] = (uint8_t)x;
        LOG[x] = i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    for (int i = 255; i < 510; i++) EXP[i] = EXP[i - 255];
    for (int a = 0; a < 256; a++)
        for (int b = 0; b < 256; b++)
            MUL[a][b] = (a && b) ? EXP[LOG[a] + LOG[b]] : 0;
    g_init = 1;
}

uint8_t orc_gf_mul(uint8_t a, uint8_t b) { init_tables(); return MUL[a][b]; }

uint8_t orc_gf_exp(uint8_t a, unsigned n) {
    init_tables();
    if (n == 0) return 1;
    if (a == 0) return 0;
    return EXP[(LOG[a] * (unsigned long)n) % 255];
}

static uint8_t gf_inv(uint8_t a) { return EXP[(255 - LOG[a]) % 255]; }

/* Gauss-Jordan over GF(2^8); returns 0 on success, -1 if singular. */
static int invert(const uint8_t* m, uint8_t* out, int n) {
    uint8_t* w = (uint8_t*)malloc((size_t)n * 2 * n);
    for (int r = 0; r < n; r++)
        for (int c = 0; c < 2 * n; c++)
            w[r * 2 * n + c] = c < n ? m[r * n + c] : (uint8_t)(c - n == r);
    for (int r = 0; r < n; r++) {
        uint8_t* row = w + r * 2 * n;
        if (row[r] == 0) {
            for (int b = r + 1; b < n; b++) {
                uint8_t* rb = w + b * 2 * n;
                if (rb[r]) {
                    for (int c = 0; c < 2 * n; c++) { uint8_t t = row[c]; row[c] = rb[c]; rb[c] = t; }
                    break;
                }
            }
        }
        if (row[r] == 0) { free(w); return -1; }
        if (row[r] != 1) {
            uint8_t s = gf_inv(row[r]);
            for (int c = 0; c < 2 * n; c++) row[c] = MUL[s][row[c]];
        }
        for (int o = 0; o < n; o++) {
            if (o == r) continue;
            uint8_t* ro = w + o * 2 * n;
            uint8_t f = ro[r];
            if (f) for (int c = 0; c < 2 * n; c++) ro[c] ^= MUL[f][row[c]];
        }
    }
    for (int r = 0; r < n; r++) memcpy(out + r * n, w + r * 2 * n + n, n);
    free(w);
    return 0;
}

typedef struct {
    int k, m, n;
    uint8_t* matrix; /* n x k */
} orc_rs;

void* orc_rs_new(int k, int m) {
    init_tables();
    if (k <= 0 || m <= 0 || k + m > 256) return NULL;
    orc_rs* rs = (orc_rs*)calloc(1, sizeof(orc_rs));
    rs->k = k; rs->m = m; rs->n = k + m;
    int n = k + m;
    uint8_t* v = (uint8_t*)malloc((size_t)n * k);
    for (int r = 0; r < n; r++)
        for (int c = 0; c < k; c++) v[r * k + c] = orc_gf_exp((uint8_t)r, (unsigned)c);
    uint8_t* inv = (uint8_t*)malloc((size_t)k * k);
    invert(v, inv, k);
    rs->matrix = (uint8_t*)malloc((size_t)n * k);
    for (int r = 0; r < n; r++)
        for (int c = 0; c < k; c++) {
            uint8_t acc = 0;
            for (int t = 0; t < k; t++) acc ^= MUL[v[r * k + t]][inv[t * k + c]];
            rs->matrix[r * k + c] = acc;
        }
    free(v); free(inv);
    return rs;
}

void orc_rs_free(void* p) {
    orc_rs* rs = (orc_rs*)p;
    if (!rs) return;
    free(rs->matrix);
    free(rs);
}

void orc_rs_matrix(void* p, uint8_t* out) {
    orc_rs* rs = (orc_rs*)p;
    memcpy(out, rs->matrix, (size_t)rs->n * rs->k);
}

int orc_invert(const uint8_t* m, uint8_t* out, int n) { init_tables(); return invert(m, out, n); }

/* ---- slice kernels -------------------------------------------------------- */
static void mul_slice_scalar(uint8_t c, const uint8_t* in, uint8_t* out, size_t len, int do_xor) {
    const uint8_t* t = MUL[c];
    if (do_xor) for (size_t i = 0; i < len; i++) out[i] ^= t[in[i]];
    else        for (size_t i = 0; i < len; i++) out[i] = t[in[i]];
}

__attribute__((target("avx2")))
static void mul_slice_avx2(uint8_t c, const uint8_t* in, uint8_t* out, size_t len, int do_xor) {
    uint8_t lo[16], hi[16];
    for (int x = 0; x < 16; x++) { lo[x] = MUL[c][x]; hi[x] = MUL[c][x << 4]; }
    const __m256i tlo = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)lo));
    const __m256i thi = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)hi));
    const __m256i mask = _mm256_set1_epi8(0x0f);
    size_t i = 0;
    for (; i + 32 <= len; i += 32) {
        __m256i v = _mm256_loadu_si256((const __m256i*)(in + i));
        __m256i l = _mm256_and_si256(v, mask);
        __m256i h = _mm256_and_si256(_mm256_srli_epi64(v, 4), mask);
        __m256i p = _mm256_xor_si256(_mm256_shuffle_epi8(tlo, l), _mm256_shuffle_epi8(thi, h));
        if (do_xor) p = _mm256_xor_si256(p, _mm256_loadu_si256((const __m256i*)(out + i)));
        _mm256_storeu_si256((__m256i*)(out + i), p);
    }
    if (i < len) mul_slice_scalar(c, in + i, out + i, len - i, do_xor);
}

static int g_have_avx2 = -1;
static int have_avx2(void) {
    if (g_have_avx2 < 0) g_have_avx2 = __builtin_cpu_supports("avx2") ? 1 : 0;
    return g_have_avx2;
}

int orc_have_avx2(void) { return have_avx2(); }

/* out[r] = XOR_i coefs[r*ncols + i] * in[i], upstream code_some_slices order. */
void orc_code_some_slices(const uint8_t* coefs, int nrows, int ninputs,
                          const uint8_t* const* in, uint8_t* const* out, size_t len, int simd) {
    init_tables();
    int use_avx = simd && have_avx2();
    for (int i = 0; i < ninputs; i++)
        for (int r = 0; r < nrows; r++) {
            uint8_t c = coefs[r * ninputs + i];
            if (use_avx) mul_slice_avx2(c, in[i], out[r], len, i != 0);
            else         mul_slice_scalar(c, in[i], out[r], len, i != 0);
        }
}

/* encode: shards[0..k) data, shards[k..n) parity written in place. */
void orc_encode(void* p, uint8_t* const* shards, size_t len, int simd) {
    orc_rs* rs = (orc_rs*)p;
    orc_code_some_slices(rs->matrix + (size_t)rs->k * rs->k, rs->m, rs->k,
                         (const uint8_t* const*)shards, shards + rs->k, len, simd);
}

/* reconstruct (upstream semantics): present[i] != 0 marks valid shards; every
 * missing slot must point to a caller buffer of len bytes (upstream allocates
 * vec![0; len]). Returns 0, or -1 if fewer than k shards are present.
 * data_only = 1 mirrors reconstruct_data (missing parity untouched). */
int orc_reconstruct(void* p, uint8_t* const* shards, const uint8_t* present, size_t len,
                    int data_only, int simd) {
    orc_rs* rs = (orc_rs*)p;
    int k = rs->k, n = rs->n;
    int npresent = 0;
    for (int i = 0; i < n; i++) npresent += present[i] ? 1 : 0;
    if (npresent == n) return 0;
    if (npresent < k) return -1;
    int valid[256], invalid[256], nv = 0, ni = 0;
    const uint8_t* sub[256];
    for (int i = 0; i < n; i++) {
        if (present[i]) { if (nv < k) { sub[nv] = shards[i]; valid[nv++] = i; } }
        else invalid[ni++] = i;
    }
    uint8_t* a = (uint8_t*)malloc((size_t)k * k);
    uint8_t* inv = (uint8_t*)malloc((size_t)k * k);
    for (int r = 0; r < k; r++) memcpy(a + r * k, rs->matrix + (size_t)valid[r] * k, k);
    invert(a, inv, k);
    uint8_t* rows = (uint8_t*)malloc((size_t)n * k);
    uint8_t* outs[256];
    int nr = 0;
    for (int t = 0; t < ni; t++)
        if (invalid[t] < k) {
            memset(shards[invalid[t]], 0, len);
            memcpy(rows + nr * k, inv + (size_t)invalid[t] * k, k);
            outs[nr++] = shards[invalid[t]];
        }
    if (nr) orc_code_some_slices(rows, nr, k, sub, outs, len, simd);
    if (!data_only) {
        nr = 0;
        for (int t = 0; t < ni; t++)
            if (invalid[t] >= k) {
                memcpy(rows + nr * k, rs->matrix + (size_t)invalid[t] * k, k);
                outs[nr++] = shards[invalid[t]];
            }
        if (nr) orc_code_some_slices(rows, nr, k, (const uint8_t* const*)shards, outs, len, simd);
    }
    free(a); free(inv); free(rows);
    return 0;
}

/* splitmix64 byte stream: word n (n >= 1) = mix(seed + n*gamma), little endian. */
void orc_splitmix64_fill(uint64_t seed, uint8_t* out, size_t nbytes) {
    size_t nw = nbytes / 8;
    for (size_t w = 0; w < nw + 1; w++) {
        uint64_t z = seed + (uint64_t)(w + 1) * 0x9E3779B97F4A7C15ULL;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        z ^= z >> 31;
        for (int b = 0; b < 8; b++) {
            size_t o = w * 8 + b;
            if (o >= nbytes) return;
            out[o] = (uint8_t)(z >> (8 * b));
        }
    }
}

/* ---- file layer: restatement of helyim-ec/src/encoder.rs ------------------
 * orc_write_ec_files  <- write_ec_files / generate_ec_files / encode_data_file
 *                        (encoder.rs:39-46, 52-71, 129-242): rows of 10 blocks
 *                        (large while remaining > 10*large, strict), 256 KiB
 *                        batches, short reads zero-filled, 14 sequential writes.
 * orc_rebuild_ec_files <- rebuild_ec_files / generate_missing_ec_files /
 *                        rebuild_ec_files_inner (encoder.rs:48-50, 73-109, 244-307).
 * Return 0, or: -1 io, -2 UnexpectedBlockSize, -3 UnexpectedEcShardSize,
 * -4 TooFewShardsPresent. Single thread, like helyim. */
#include <fcntl.h>
#include <stdio.h>
#include <sys/stat.h>
#include <unistd.h>

static int read_full(int fd, uint8_t* buf, size_t n, off_t off, size_t* got) {
    size_t g = 0;
    while (g < n) {
        ssize_t r = pread(fd, buf + g, n - g, off + (off_t)g);
        if (r < 0) return -1;
        if (r == 0) break;
        g += (size_t)r;
    }
    *got = g;
    return 0;
}

static int write_full(int fd, const uint8_t* buf, size_t n) {
    size_t p = 0;
    while (p < n) {
        ssize_t w = write(fd, buf + p, n - p);
        if (w < 0) return -1;
        p += (size_t)w;
    }
    return 0;
}

int orc_write_ec_files(const char* base, uint64_t buf_size, uint64_t large, uint64_t small, int simd) {
    char name[4096];
    snprintf(name, sizeof name, "%s.dat", base);
    int dat = open(name, O_RDONLY);
    if (dat < 0) return -1;
    struct stat st;
    if (fstat(dat, &st) != 0) { close(dat); return -1; }
    int64_t remaining = (int64_t)st.st_size;
    void* rs = orc_rs_new(10, 4);
    uint8_t* bufs[14];
    for (int i = 0; i < 14; i++) bufs[i] = (uint8_t*)malloc(buf_size);
    int out[14];
    for (int i = 0; i < 14; i++) {
        snprintf(name, sizeof name, "%s.ec%02d", base, i);
        out[i] = open(name, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    }
    int rc = 0;
    uint64_t processed = 0;
    for (int phase = 0; phase < 2 && rc == 0; phase++) {
        uint64_t block = phase == 0 ? large : small;
        while (rc == 0 && (phase == 0 ? remaining > (int64_t)(large * 10) : remaining > 0)) {
            if (block % buf_size != 0) { rc = -2; break; }
            for (uint64_t b = 0; b < block / buf_size && rc == 0; b++) {
                uint64_t start = processed + b * buf_size;
                for (int i = 0; i < 10; i++) {
                    size_t got = 0;
                    if (read_full(dat, bufs[i], buf_size, (off_t)(start + block * i), &got)) { rc = -1; break; }
                    if (got < buf_size) memset(bufs[i] + got, 0, buf_size - got);
                }
                if (rc) break;
                orc_encode(rs, bufs, buf_size, simd);
                for (int i = 0; i < 14; i++)
                    if (write_full(out[i], bufs[i], buf_size)) { rc = -1; break; }
            }
            processed += block * 10;
            remaining -= (int64_t)(block * 10);
        }
    }
    for (int i = 0; i < 14; i++) { close(out[i]); free(bufs[i]); }
    close(dat);
    orc_rs_free(rs);
    return rc;
}

int orc_rebuild_ec_files(const char* base, uint32_t* ids, size_t* n_ids, int simd) {
    char name[4096];
    int in[14], out[14];
    uint8_t has[14];
    size_t nr = 0;
    for (int i = 0; i < 14; i++) {
        snprintf(name, sizeof name, "%s.ec%02d", base, i);
        struct stat st;
        in[i] = out[i] = -1;
        if (stat(name, &st) == 0) {
            has[i] = 1;
            in[i] = open(name, O_RDONLY);
        } else {
            has[i] = 0;
            out[i] = open(name, O_WRONLY | O_CREAT | O_TRUNC, 0644);
            ids[nr++] = (uint32_t)i;
        }
    }
    *n_ids = nr;
    void* rs = orc_rs_new(10, 4);
    const size_t SB = 1 << 20;
    uint8_t* bufs[14];
    for (int i = 0; i < 14; i++) bufs[i] = (uint8_t*)calloc(1, SB);
    int rc = 0;
    uint64_t start = 0;
    size_t size = 0;
    for (;;) {
        int stop = 0;
        for (int i = 0; i < 14 && !stop && rc == 0; i++) {
            if (!has[i]) continue;
            size_t got = 0;
            if (read_full(in[i], bufs[i], SB, (off_t)start, &got)) { rc = -1; break; }
            if (got == 0) { stop = 1; break; }
            if (size == 0) size = got;
            if (size != got) rc = -3;
        }
        if (stop || rc) break;
        int npres = 0;
        for (int i = 0; i < 14; i++) npres += has[i];
        if (npres < 10) { rc = -4; break; }
        if (npres < 14) {
            orc_reconstruct(rs, bufs, has, SB, 0, simd);
            for (int i = 0; i < 14; i++)
                if (!has[i] && pwrite(out[i], bufs[i], size, (off_t)start) != (ssize_t)size) { rc = -1; break; }
        }
        if (rc) break;
        start += size;
    }
    for (int i = 0; i < 14; i++) {
        if (in[i] >= 0) close(in[i]);
        if (out[i] >= 0) close(out[i]);
        free(bufs[i]);
    }
    orc_rs_free(rs);
    return rc;
}

/* orc_read_ec_data <- read_ec_shard_intervals / read_one_ec_shard_interval /
 * recover_one_remote_ec_shard_interval (helyim-store/src/erasure_coding/
 * mod.rs:303-491) with locate_data (helyim-ec/src/locate.rs:29-100), against
 * the local base.ecNN files, one interval at a time like helyim: a present
 * shard is read exactly; a missing one reads the same range from every other
 * shard (full-length reads count as present) and runs upstream reconstruct.
 * data_size = first shard file's size * 10 (volume/mod.rs:146).
 * Returns 0, -1 io / short read, -4 TooFewShardsPresent, -5 no shard file. */
int orc_read_ec_data(const char* base, uint64_t large, uint64_t small, const uint64_t* offsets,
                     const uint64_t* sizes, size_t n, uint8_t* out, int simd) {
    char name[4096];
    int fd[14];
    uint64_t data_size = 0;
    int first = -1;
    for (int i = 0; i < 14; i++) {
        snprintf(name, sizeof name, "%s.ec%02d", base, i);
        fd[i] = open(name, O_RDONLY);
        if (fd[i] >= 0 && first < 0) {
            struct stat st;
            fstat(fd[i], &st);
            data_size = (uint64_t)st.st_size * 10;
            first = i;
        }
    }
    if (first < 0) return -5;
    void* rs = orc_rs_new(10, 4);
    int rc = 0;
    for (size_t r = 0; r < n && rc == 0; r++) {
        /* locate_offset: its own large-row count (locate.rs:84) */
        uint64_t off = offsets[r], size = sizes[r];
        const uint64_t lrows_off = data_size / (large * 10);
        uint64_t block, inner;
        int is_large;
        if (off < lrows_off * large * 10) {
            block = off / large; inner = off % large; is_large = 1;
        } else {
            off -= lrows_off * large * 10;
            block = off / small; inner = off % small; is_large = 0;
        }
        const uint64_t lrows = (data_size + small * 10) / (large * 10); /* locate.rs:39-40 */
        while (size > 0 && rc == 0) {
            const uint64_t remaining = (is_large ? large : small) - inner;
            const uint64_t take = size <= remaining ? size : remaining;
            const int sid = (int)(block % 10);
            const uint64_t row = block / 10;
            const uint64_t at = is_large ? inner + row * large : inner + lrows * large + row * small;
            if (fd[sid] >= 0) {
                size_t got = 0;
                if (read_full(fd[sid], out, take, (off_t)at, &got) || got != take) rc = -1;
            } else {
                uint8_t* bufs[14];
                uint8_t pres[14];
                for (int i = 0; i < 14; i++) {
                    bufs[i] = (uint8_t*)calloc(1, take);
                    pres[i] = 0;
                    if (i == sid || fd[i] < 0) continue;
                    size_t got = 0;
                    if (read_full(fd[i], bufs[i], take, (off_t)at, &got) == 0 && got == take) pres[i] = 1;
                }
                if (orc_reconstruct(rs, bufs, pres, take, 0, simd)) rc = -4;
                else memcpy(out, bufs[sid], take);
                for (int i = 0; i < 14; i++) free(bufs[i]);
            }
            out += take;
            size -= take;
            if (size == 0) break;
            block += 1;
            if (is_large && block == lrows * 10) { is_large = 0; block = 0; }
            inner = 0;
        }
    }
    for (int i = 0; i < 14; i++)
        if (fd[i] >= 0) close(fd[i]);
    orc_rs_free(rs);
    return rc;
}

// GF(2^8) arithmetic and coding-matrix construction for the product library.
//
// Field: x^8+x^4+x^3+x^2+1 (0x11D), generator 2 -- the field of the upstream
// crate reed-solomon-erasure 6.0.0 `galois_8` that helyim-ec links
// (/root/reference/Cargo.toml:72, helyim-ec/Cargo.toml:26). Matrix: the
// systematic Vandermonde construction of upstream `ReedSolomon::new`, called
// at /root/reference/helyim-ec/src/encoder.rs:208-209,249-250.
//
// Host-side only: this builds the small coefficient matrices and the v_perm
// lookup tables the gfx950 kernels consume. No bulk data is touched here.
#pragma once
#include <cstdint>
#include <cstring>
#include <vector>

namespace hec {

struct Gf {
    uint8_t exp[510];
    uint8_t log[256];
    uint8_t mul[256][256];
    Gf() {
        unsigned x = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = uint8_t(x);
            log[x] = uint8_t(i);
            x <<= 1;
            if (x & 0x100) x ^= 0x11D;
        }
        log[0] = 0;
        for (int i = 255; i < 510; ++i) exp[i] = exp[i - 255];
        for (int a = 0; a < 256; ++a)
            for (int b = 0; b < 256; ++b)
                mul[a][b] = (a && b) ? exp[log[a] + log[b]] : 0;
    }
    uint8_t inv(uint8_t a) const { return exp[(255 - log[a]) % 255]; }
    // upstream galois_8::exp semantics: exp(a,0)=1, exp(0,n>0)=0
    uint8_t pow(uint8_t a, unsigned n) const {
        if (n == 0) return 1;
        if (a == 0) return 0;
        return exp[(unsigned(log[a]) * n) % 255];
    }
};

const Gf& gf();

// Row-major byte matrix.
struct Mat {
    int rows = 0, cols = 0;
    std::vector<uint8_t> v;
    Mat() = default;
    Mat(int r, int c) : rows(r), cols(c), v(size_t(r) * c, 0) {}
    uint8_t& at(int r, int c) { return v[size_t(r) * cols + c]; }
    uint8_t at(int r, int c) const { return v[size_t(r) * cols + c]; }
    const uint8_t* row(int r) const { return v.data() + size_t(r) * cols; }
};

Mat mat_mul(const Mat& a, const Mat& b);
// Gauss-Jordan inversion; returns false when singular.
bool mat_invert(const Mat& m, Mat& out);
// upstream ReedSolomon::new: V(total x data) * inv(V[0..data]), V[r][c] = r^c
Mat build_encoding_matrix(int data_shards, int total_shards);

// Per-coefficient lookup tables for the gfx950 v_perm_b32 kernel.
// c*x = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6]
// word 0/1: T0 bytes 0-3 / 4-7, word 2/3: T1 bytes 0-3 / 4-7, word 4: T2.
constexpr int kTabWords = 5;
inline void perm_tables(uint8_t c, uint32_t out[kTabWords]) {
    const Gf& g = gf();
    uint8_t t0[8], t1[8], t2[4];
    for (int v = 0; v < 8; ++v) {
        t0[v] = g.mul[c][v];
        t1[v] = g.mul[c][v << 3];
    }
    for (int v = 0; v < 4; ++v) t2[v] = g.mul[c][v << 6];
    std::memcpy(&out[0], t0, 8);
    std::memcpy(&out[2], t1, 8);
    std::memcpy(&out[4], t2, 4);
}

}  // namespace hec

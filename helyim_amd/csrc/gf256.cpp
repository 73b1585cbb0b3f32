// GF(2^8) matrices for the product library (host side). See gf256.hpp.
#include "gf256.hpp"

namespace hec {

const Gf& gf() {
    static const Gf g;
    return g;
}

Mat mat_mul(const Mat& a, const Mat& b) {
    const Gf& g = gf();
    Mat out(a.rows, b.cols);
    for (int r = 0; r < a.rows; ++r)
        for (int c = 0; c < b.cols; ++c) {
            uint8_t acc = 0;
            for (int t = 0; t < a.cols; ++t) acc ^= g.mul[a.at(r, t)][b.at(t, c)];
            out.at(r, c) = acc;
        }
    return out;
}

bool mat_invert(const Mat& m, Mat& out) {
    const Gf& g = gf();
    const int n = m.rows;
    if (m.cols != n) return false;
    Mat w(n, 2 * n);
    for (int r = 0; r < n; ++r) {
        for (int c = 0; c < n; ++c) w.at(r, c) = m.at(r, c);
        w.at(r, n + r) = 1;
    }
    for (int r = 0; r < n; ++r) {
        if (w.at(r, r) == 0) {
            for (int b = r + 1; b < n; ++b)
                if (w.at(b, r) != 0) {
                    for (int c = 0; c < 2 * n; ++c) std::swap(w.at(r, c), w.at(b, c));
                    break;
                }
        }
        if (w.at(r, r) == 0) return false;
        if (w.at(r, r) != 1) {
            const uint8_t s = g.inv(w.at(r, r));
            for (int c = 0; c < 2 * n; ++c) w.at(r, c) = g.mul[s][w.at(r, c)];
        }
        for (int o = 0; o < n; ++o) {
            if (o == r) continue;
            const uint8_t f = w.at(o, r);
            if (!f) continue;
            for (int c = 0; c < 2 * n; ++c) w.at(o, c) ^= g.mul[f][w.at(r, c)];
        }
    }
    out = Mat(n, n);
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) out.at(r, c) = w.at(r, n + c);
    return true;
}

Mat build_encoding_matrix(int data_shards, int total_shards) {
    const Gf& g = gf();
    Mat v(total_shards, data_shards);
    for (int r = 0; r < total_shards; ++r)
        for (int c = 0; c < data_shards; ++c) v.at(r, c) = g.pow(uint8_t(r), unsigned(c));
    Mat top(data_shards, data_shards);
    for (int r = 0; r < data_shards; ++r)
        for (int c = 0; c < data_shards; ++c) top.at(r, c) = v.at(r, c);
    Mat inv;
    mat_invert(top, inv);  // Vandermonde top square with distinct points: always invertible
    return mat_mul(v, inv);
}

}  // namespace hec

// Exhaustive-by-sampling check of hec::FastDiv (helyim_amd/csrc/fastdiv.hpp),
// the multiply-shift division the RS(10,4) fast kernels use to split a
// workgroup's chunk index into (stripe, chunk). Exits non-zero on the first
// mismatch. Divisors: 1..70000, every power of two and its neighbours, and
// random 32-bit values; dividends: edges (0, 1, d-1, d, d+1, multiples near
// 2^32) plus a random sample per divisor.
#include <cstdint>
#include <cstdio>

#include "fastdiv.hpp"

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t next32() {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return uint32_t(rng >> 16);
}

static int check(uint32_t d, uint32_t n) {
    const hec::FastDiv f = hec::make_fastdiv(d);
    const uint32_t got = hec::fastdiv(n, f.mul, f.shift);
    if (got != n / d) {
        std::printf("MISMATCH d=%u n=%u got=%u want=%u\n", d, n, got, n / d);
        return 1;
    }
    return 0;
}

static int check_divisor(uint32_t d, int samples) {
    const uint32_t edges[] = {0u, 1u, d - 1, d, d + 1, 2 * d - 1, 2 * d, 0xFFFFFFFFu, 0xFFFFFFFEu, 0x80000000u,
                              0x7FFFFFFFu, (0xFFFFFFFFu / d) * d, (0xFFFFFFFFu / d) * d - 1};
    for (uint32_t n : edges)
        if (check(d, n)) return 1;
    for (int i = 0; i < samples; ++i)
        if (check(d, next32())) return 1;
    return 0;
}

int main() {
    long checked = 0;
    for (uint32_t d = 1; d <= 70000; ++d, ++checked)
        if (check_divisor(d, 512)) return 1;
    for (int s = 0; s < 32; ++s)
        for (int64_t dd = -2; dd <= 2; ++dd) {
            const int64_t d = (int64_t(1) << s) + dd;
            if (d < 1 || d > 0xFFFFFFFFll) continue;
            if (check_divisor(uint32_t(d), 4096)) return 1;
            ++checked;
        }
    for (int i = 0; i < 20000; ++i, ++checked) {
        const uint32_t d = (next32() | 0x80000000u) >> (i % 32);  // every bit length 1..32
        if (check_divisor(d, 64)) return 1;
    }
    std::printf("ok %ld divisors\n", checked);
    return 0;
}

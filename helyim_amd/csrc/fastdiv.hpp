// Unsigned 32-bit division by a launch constant d >= 1 as a multiply and a
// shift (Granlund-Montgomery with the 33-bit magic 2^32 + mul):
//   n / d = (n + mulhi(n, mul)) >> shift,  shift = ceil(log2 d),
//   mul = floor(2^32 (2^shift - d) / d) + 1,
// exact for every 32-bit n. The RS(10,4) fast kernels use it to split a
// workgroup's chunk index into (stripe, chunk) in scalar ops. Plain C++ (no
// HIP headers) so tests/c/fastdiv_check.cpp checks it with g++.
#pragma once
#include <cstdint>

#ifdef __HIPCC__
#define HEC_HD __host__ __device__
#else
#define HEC_HD
#endif

namespace hec {

struct FastDiv {
    uint32_t mul, shift;
};

inline FastDiv make_fastdiv(uint32_t d) {
    uint32_t s = 0;
    while (s < 32 && (uint64_t(1) << s) < d) ++s;
    const uint64_t m = ((uint64_t(1) << 32) * ((uint64_t(1) << s) - d)) / d + 1;
    return FastDiv{uint32_t(m), s};
}

HEC_HD inline uint32_t fastdiv(uint32_t n, uint32_t mul, uint32_t shift) {
    const uint32_t hi = uint32_t((uint64_t(n) * mul) >> 32);
    return uint32_t((uint64_t(n) + hi) >> shift);
}

}  // namespace hec

// Bit-sliced RS(10,4) syndrome decode of one lane's 32 byte columns
// (rs104_bs_decode_kernel in rs_kernels.hip; host-tested by
// tests/test_bitslice_decode.py through the HEC_* hooks of bitslice.hpp).
//
// Upstream reconstruct (reed-solomon-erasure 6.0.0, called at
// /root/reference/helyim-ec/src/encoder.rs:288 and
// helyim-store/src/erasure_coding/mod.rs:426) inverts the rows of the first
// 10 present shards: every present data shard plus the first e_d present
// parity rows ("selected"), e_d = erased data shards. Its answer is the unique
// solution of those 10 equations, so it can be reached another way with the
// same bytes:
//
//   1. P'_j = the parity the FIXED encode program (rs104_bitslice.inc) gives
//      with the erased data shards taken as zero;
//   2. syndrome S_j = P'_j ^ P_j for each selected parity row j
//      (= sum over erased data m of M[10+j][m] * d_m);
//   3. erased data d_m = sum_j A[m][j] * S_j, A = inverse of that e_d x e_d
//      block of the parity matrix (host-computed per erasure pattern);
//   4. erased parity P_j = P'_j ^ sum_j' G[j][j'] * S_j', G = M[10+j, erased
//      data] * A -- parity of the full data, as upstream's second pass.
//
// Steps 1-2 are the bit-sliced XOR program (~4 ops per data dword); only the
// small e_d-input table multiply of steps 3-4 is pattern specific. The table
// decode multiplies all 10 survivors into 4 rows (40 lookups per column).
//
// Table words of one pattern (kSynWords = 160, rs_kernels.hpp): coefficient (row, j) at
// ((row * 4) + j) * kTabWords, rows 0-3 = erased data shards ascending, rows
// 4-7 = parity rows 0-3; j = parity row of the syndrome; unused slots zero.
#pragma once
#include "bitslice.hpp"

#ifndef HEC_PERM
#define HEC_PERM(a, b, sel) __builtin_amdgcn_perm((a), (b), (sel))
#endif

namespace hec {

// acc[w] ^= c * x[w] for 8 dwords (4 bytes each): three 3-bit-index v_perm
// lookups (c*x = T0[x&7] ^ T1[(x>>3)&7] ^ T2[x>>6]), tables tab[0..4].
template <typename TabPtr>
HEC_DEVICE void syn_mac8(uint32_t* acc, const uint32_t (&s0)[8], const uint32_t (&s1)[8], const uint32_t (&s2)[8],
                         TabPtr tab) {
    const uint32_t t0l = tab[0], t0h = tab[1], t1l = tab[2], t1h = tab[3], t2 = tab[4];
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        const uint32_t a = HEC_PERM(t0h, t0l, s0[w]);
        const uint32_t b = HEC_PERM(t1h, t1l, s1[w]);
        const uint32_t c = HEC_PERM(t2, t2, s2[w]);
        acc[w] = HEC_BITOP3(acc[w], a, b, 0x96) ^ c;
    }
}

// Selected parity rows: the first ed present ones (bit j = parity row j).
HEC_DEVICE uint32_t syn_selected(uint32_t mask, uint32_t ed) {
    uint32_t pres = (mask >> 10) & 0xFu, sel = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t)
        if (uint32_t(t) < ed) {
            const uint32_t lo = pres & (0u - pres);
            sel |= lo;
            pres ^= lo;
        }
    return sel;
}

// Phase 1 (steps 1-2 up to the syndromes' P' half): p = data planes (80
// words: 8 dwords of data shard i at p[8i..], zero for an erased shard;
// transposed in place); q = P' (bytes) for every parity row the solve uses.
HEC_DEVICE void rs104_syndrome_phase1(uint32_t (&p)[80], uint32_t mask, uint32_t sel, uint32_t (&q)[32]) {
    const uint32_t erased = ~mask & 0x3FFFu;
#pragma unroll
    for (int i = 0; i < 10; ++i)
        if ((mask >> i) & 1u) transpose8(p + 8 * i);  // erased shards: zero planes stay zero
    rs104_encode_planes(p, q);
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (((sel | (erased >> 10)) >> j) & 1u) transpose8(q + 8 * j);  // P'_j back to bytes where used
}

// Phase 2 (steps 2-4): pp = the selected parity rows' bytes (8 dwords per
// row; other rows ignored). Out: dd[8r..] = erased data shard r (ascending)
// for r < ed; q[8j..] = parity row j for every erased parity row j (bytes).
template <typename TabPtr>
HEC_DEVICE void rs104_syndrome_phase2(uint32_t (&q)[32], const uint32_t (&pp)[32], uint32_t mask, uint32_t ed,
                                      uint32_t sel, TabPtr syn, uint32_t (&dd)[32]) {
    const uint32_t erased = ~mask & 0x3FFFu;
#pragma unroll
    for (int k = 0; k < 32; ++k) dd[k] = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (!((sel >> j) & 1u)) continue;
        uint32_t s0[8], s1[8], s2[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            const uint32_t s = q[8 * j + w] ^ pp[8 * j + w];  // syndrome S_j
            s0[w] = s & 0x07070707u;
            s1[w] = (s >> 3) & 0x07070707u;
            s2[w] = (s >> 6) & 0x03030303u;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (uint32_t(r) < ed) syn_mac8(dd + 8 * r, s0, s1, s2, syn + (r * 4 + j) * 5);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
            if ((erased >> (10 + jj)) & 1u) syn_mac8(q + 8 * jj, s0, s1, s2, syn + ((4 + jj) * 4 + j) * 5);
    }
}

// Both phases: mask = present mask (10..13 of 14 present).
template <typename TabPtr>
HEC_DEVICE void rs104_syndrome_decode_lane(uint32_t (&p)[80], const uint32_t (&pp)[32], uint32_t mask,
                                           TabPtr syn, uint32_t (&dd)[32], uint32_t (&q)[32]) {
    const uint32_t ed = __builtin_popcount(~mask & 0x3FFu);
    const uint32_t sel = syn_selected(mask, ed);
    rs104_syndrome_phase1(p, mask, sel, q);
    rs104_syndrome_phase2(q, pp, mask, ed, sel, syn, dd);
}

}  // namespace hec

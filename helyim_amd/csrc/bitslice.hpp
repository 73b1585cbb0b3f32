// Bit-slicing helpers for the RS(10,4) encode kernel (rs_kernels.hip):
// 8 x 8 bit transposes between bytes and bit planes, and the generated XOR
// program over the planes (rs104_bitslice.inc, tools/gen_bitslice.py).
//
// HEC_DEVICE / HEC_BITOP3 default to the gfx950 device forms; the host-side
// test harness (tests/test_bitslice_program.py) defines them before including
// this header to run the same code on the CPU against the oracle.
#pragma once
#include <cstdint>

#ifndef HEC_DEVICE
#define HEC_DEVICE __device__ __forceinline__
#endif
#ifndef HEC_BITOP3
#define HEC_BITOP3(a, b, c, tt) __builtin_amdgcn_bitop3_b32((a), (b), (c), (tt))
#endif

namespace hec {

// v_bitop3_b32 truth table 0x96 = a ^ b ^ c
HEC_DEVICE uint32_t hec_xor3(uint32_t a, uint32_t b, uint32_t c) { return HEC_BITOP3(a, b, c, 0x96); }

// Swap the off-diagonal s x s blocks of the 8x8 bit matrices (one per byte
// lane) held in rows a (low) and b (high): two shifts and two bit-selects
// (truth table 0xCA = S0 ? S1 : S2 per bit; an intrinsic, so the stages are not
// re-associated into extra ands).
template <int S, uint32_t M>
HEC_DEVICE void swap_blocks(uint32_t& a, uint32_t& b) {
    const uint32_t na = HEC_BITOP3(M, a, b << S, 0xCA);
    const uint32_t nb = HEC_BITOP3(M, a >> S, b, 0xCA);
    a = na;
    b = nb;
}

// In-place 8x8 bit transpose of every byte lane: afterwards r[k] bit (8L+i)
// is bit k of byte L of the original r[i]. An involution.
HEC_DEVICE void transpose8(uint32_t* r) {
#pragma unroll
    for (int i = 0; i < 4; ++i) swap_blocks<4, 0x0F0F0F0Fu>(r[i], r[i + 4]);
#pragma unroll
    for (int i = 0; i < 8; i += 4) {
        swap_blocks<2, 0x33333333u>(r[i], r[i + 2]);
        swap_blocks<2, 0x33333333u>(r[i + 1], r[i + 3]);
    }
#pragma unroll
    for (int i = 0; i < 8; i += 2) swap_blocks<1, 0x55555555u>(r[i], r[i + 1]);
}

#include "rs104_bitslice.inc"

}  // namespace hec

// gf256.h -- GF(2^8) with reduction polynomial x^8+x^4+x^3+x+1 (0x11B), the
// field of the reference's erasure code (crt/nk8.c:54-74).  Host + device.
//
// Device kernels never carry the reference's two 64 KiB tables
// (gf_log = products, gf_alog = quotients, nk8.c:4-8).  They use
//   * a 256-byte log table and a 768-byte antilog table (generator 3; note
//     2 is NOT a generator of 0x11B, it has order 51), staged in LDS, for
//     coefficient arithmetic and the generic kernels; and
//   * per-stripe packed product tables built in LDS from eight basis
//     products (multiplication by a constant is GF(2)-linear) for the
//     streaming kernels -- see nk8_kernels.hip.
#pragma once
#include <stdint.h>

#ifndef __HIPCC__
#define NKFS_HD
#else
#define NKFS_HD __host__ __device__
#endif

namespace nkfs {

// Carry-less 8x8 product reduced by 0x11B (same value as gf_mult_direct).
NKFS_HD inline constexpr uint8_t gf_mul_slow(uint8_t a, uint8_t b)
{
    uint32_t acc = 0;
    for (int bit = 0; bit < 8; ++bit)
        if (b & (1u << bit))
            acc ^= uint32_t(a) << bit;
    for (int bit = 14; bit >= 8; --bit)
        if (acc & (1u << bit))
            acc ^= 0x11Bu << (bit - 8);
    return uint8_t(acc);
}

// x * 2 in the field, applied to the four bytes of a 32-bit word at once.
NKFS_HD inline constexpr uint32_t gf_xtime4(uint32_t v)
{
    uint32_t hi = (v >> 7) & 0x01010101u;
    return ((v << 1) & 0xFEFEFEFEu) ^ (hi * 0x1Bu);
}

// Log/antilog layout shared by host and device (GfTables lives in device
// memory, built once by k_gf_init at nk8_init time).
//   exp[i] = 3^i for i in [0, 510): exp[la + lb] needs no modulo.
//   exp[510..767] = 0 so that exp[LOG_ZERO + anything <= 257] == 0.
//   log[x] = discrete log of x (x != 0); log[0] = LOG_ZERO.
constexpr int LOG_ZERO = 510;
//   inv[x] = x^-1 (inv[0] = 0).
struct GfTables {
    uint16_t log[256];
    uint8_t exp[768];
    uint8_t inv[256];
};

}  // namespace nkfs

// key160.hpp -- 160-bit OverlayKey arithmetic for gfx950 kernels and the C++ host.
//
// Semantics follow src/common/OverlayKey.cc (keyLength = 160): keys are
// unsigned 160-bit integers, arithmetic is mod 2^160 (trim(), 835-838), and the
// ring-interval predicates reproduce the reference's equal-endpoint rules
// exactly (isBetween 587-599, isBetweenR 602-614, isBetweenL 617-629,
// isBetweenLR 632-644).  Device representation: five u32 words, w[0] least
// significant; compares are done on (w4, w3:w2, w1:w0) as u32/u64 pairs so a
// compare is 3 integer compares and no branches.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define OVS_HD __host__ __device__ __forceinline__
#else
#define OVS_HD inline
#endif

namespace ovs {

struct K160 {
    uint32_t w[5];
};

// Node record in HBM: 24 B = key + one aux word (Chord: finger-row offset).
struct alignas(8) KeyRec {
    uint32_t w[5];
    uint32_t aux;
};

OVS_HD uint64_t lo64(const K160& a) { return (uint64_t)a.w[0] | ((uint64_t)a.w[1] << 32); }
OVS_HD uint64_t mid64(const K160& a) { return (uint64_t)a.w[2] | ((uint64_t)a.w[3] << 32); }

OVS_HD K160 key_of(const KeyRec& r)
{
    K160 k;
    k.w[0] = r.w[0]; k.w[1] = r.w[1]; k.w[2] = r.w[2]; k.w[3] = r.w[3]; k.w[4] = r.w[4];
    return k;
}

OVS_HD bool k_eq(const K160& a, const K160& b)
{
    return ((a.w[0] ^ b.w[0]) | (a.w[1] ^ b.w[1]) | (a.w[2] ^ b.w[2]) | (a.w[3] ^ b.w[3]) |
            (a.w[4] ^ b.w[4])) == 0;
}

// a < b as unsigned 160-bit integers (mpn_cmp order, OverlayKey.cc:842-847)
OVS_HD bool k_lt(const K160& a, const K160& b)
{
    const uint64_t am = mid64(a), bm = mid64(b), al = lo64(a), bl = lo64(b);
    return (a.w[4] < b.w[4]) | ((a.w[4] == b.w[4]) & ((am < bm) | ((am == bm) & (al < bl))));
}
OVS_HD bool k_le(const K160& a, const K160& b) { return !k_lt(b, a); }
OVS_HD bool k_gt(const K160& a, const K160& b) { return k_lt(b, a); }
OVS_HD bool k_ge(const K160& a, const K160& b) { return !k_lt(a, b); }

// (a - b) mod 2^160 (OverlayKey::operator-, 256-262)
OVS_HD K160 k_sub(const K160& a, const K160& b)
{
    const uint64_t al = lo64(a), bl = lo64(b), am = mid64(a), bm = mid64(b);
    const uint64_t rl = al - bl;
    const uint64_t c0 = al < bl;
    const uint64_t rm1 = am - bm;
    const uint64_t c1 = am < bm;
    const uint64_t rm = rm1 - c0;
    const uint64_t c2 = rm1 < c0;
    const uint32_t rh = a.w[4] - b.w[4] - (uint32_t)(c1 | c2);
    K160 r;
    r.w[0] = (uint32_t)rl; r.w[1] = (uint32_t)(rl >> 32);
    r.w[2] = (uint32_t)rm; r.w[3] = (uint32_t)(rm >> 32);
    r.w[4] = rh;
    return r;
}

// (a + b) mod 2^160 (OverlayKey::operator+, 247-253)
OVS_HD K160 k_add(const K160& a, const K160& b)
{
    const uint64_t al = lo64(a), bl = lo64(b), am = mid64(a), bm = mid64(b);
    const uint64_t rl = al + bl;
    const uint64_t c0 = rl < al;
    const uint64_t rm1 = am + bm;
    const uint64_t c1 = rm1 < am;
    const uint64_t rm = rm1 + c0;
    const uint64_t c2 = rm < rm1;
    const uint32_t rh = a.w[4] + b.w[4] + (uint32_t)(c1 | c2);
    K160 r;
    r.w[0] = (uint32_t)rl; r.w[1] = (uint32_t)(rl >> 32);
    r.w[2] = (uint32_t)rm; r.w[3] = (uint32_t)(rm >> 32);
    r.w[4] = rh;
    return r;
}

OVS_HD K160 k_xor(const K160& a, const K160& b)
{
    K160 r;
    for (int i = 0; i < 5; ++i) r.w[i] = a.w[i] ^ b.w[i];
    return r;
}

OVS_HD int clz32(uint32_t x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __clz((int)x);
#else
    return x ? __builtin_clz(x) : 32;
#endif
}

// index of the most significant set bit, -1 for zero (OverlayKey::log_2, 558-578)
OVS_HD int k_msb(const K160& a)
{
    for (int i = 4; i >= 0; --i)
        if (a.w[i]) return i * 32 + 31 - clz32(a.w[i]);
    return -1;
}

// word i of a key, 0 above the top word (select chain: no dynamic register indexing)
OVS_HD uint32_t k_word(const K160& a, int i)
{
    return i == 0 ? a.w[0] : i == 1 ? a.w[1] : i == 2 ? a.w[2] : i == 3 ? a.w[3] : i == 4 ? a.w[4] : 0u;
}

// Order-preserving 64-bit code of a 160-bit value v (a floating-point-like
// summary used to decide ring-interval tests without the full key):
//   code(0) = 0;  otherwise code(v) = (msb(v) + 1) << 56 | the 56 bits below msb(v).
// a < b  =>  code(a) <= code(b);   code(a) < code(b)  =>  a < b.
// Equal codes decide nothing: callers fall back to the exact 160-bit compare.
// code(v) >> 32 is the same construction with a 24-bit mantissa.
OVS_HD uint64_t k_code64(const K160& v)
{
    const int e = k_msb(v);
    if (e < 0) return 0;
    uint64_t top;   // the 64-bit window of v whose msb is bit e
    if (e >= 63) {
        const int s = e - 63, q = s >> 5, r = s & 31;
        const uint32_t a0 = k_word(v, q), a1 = k_word(v, q + 1), a2 = k_word(v, q + 2);
        const uint32_t lo = r ? (a0 >> r) | (a1 << (32 - r)) : a0;
        const uint32_t hi = r ? (a1 >> r) | (a2 << (32 - r)) : a1;
        top = (uint64_t)lo | ((uint64_t)hi << 32);
    } else {
        top = lo64(v) << (63 - e);
    }
    return ((uint64_t)(e + 1) << 56) | ((top << 1) >> 8);
}

// 2^e (OverlayKey::pow2, 704-717)
OVS_HD K160 k_pow2(int e)
{
    K160 r;
    for (int i = 0; i < 5; ++i) r.w[i] = (e >> 5) == i ? (1u << (e & 31)) : 0u;
    return r;
}

// x in (a, b)   -- OverlayKey::isBetween (587-599); keys never unspecified here
OVS_HD bool between_open(const K160& x, const K160& a, const K160& b)
{
    if (k_eq(x, a)) return false;
    if (k_lt(a, b)) return k_gt(x, a) & k_lt(x, b);
    return k_gt(x, a) | k_lt(x, b);
}
// x in (a, b]   -- isBetweenR (602-614)
OVS_HD bool between_R(const K160& x, const K160& a, const K160& b)
{
    if (k_eq(a, b) & k_eq(x, a)) return true;
    if (k_le(a, b)) return k_gt(x, a) & k_le(x, b);
    return k_gt(x, a) | k_le(x, b);
}
// x in [a, b)   -- isBetweenL (617-629)
OVS_HD bool between_L(const K160& x, const K160& a, const K160& b)
{
    if (k_eq(a, b) & k_eq(x, a)) return true;
    if (k_le(a, b)) return k_ge(x, a) & k_lt(x, b);
    return k_ge(x, a) | k_lt(x, b);
}
// x in [a, b]   -- isBetweenLR (632-644)
OVS_HD bool between_LR(const K160& x, const K160& a, const K160& b)
{
    if (k_eq(a, b) & k_eq(x, a)) return true;
    if (k_le(a, b)) return k_ge(x, a) & k_le(x, b);
    return k_ge(x, a) | k_le(x, b);
}

}  // namespace ovs

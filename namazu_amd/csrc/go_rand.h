// Go math/rand (Go 1.10 src/math/rand/rng.go, rand.go) restated for gfx950.
//
// rand.New(rand.NewSource(seed)) seeds a 607-word additive lagged-Fibonacci
// state from the Park-Miller LCG x_{n+1} = 48271 x_n mod (2^31-1):
//     vec[i] = (x_{21+3i} << 40) ^ (x_{22+3i} << 20) ^ x_{23+3i} ^ rngCooked[i]
// and the k-th Uint64 output (k = 0, 1, ...) is y_k = y_{k-607} + y_{k-273},
// where y_s (s < 0) is the seeded vec[(333 - s) mod 607]. Since
// x_n = s * 48271^n mod (2^31-1), any vec entry costs 3 modular multiplies by
// constants, so a decision never materialises the 607-word state (the
// reference re-seeds it per event: util/queue/impl.go:39).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "go_rng_cooked.h"

namespace nmz {
namespace gorand {

constexpr uint32_t M31 = 0x7fffffffu;
constexpr uint32_t A = 48271u;
constexpr int LEN = 607;

constexpr uint32_t pow_a(uint32_t n) {
    uint64_t r = 1, b = A;
    while (n) {
        if (n & 1) r = (r * b) % M31;
        b = (b * b) % M31;
        n >>= 1;
    }
    return (uint32_t)r;
}

struct PowTable {
    uint32_t v[3 * LEN + 21];
};
constexpr PowTable make_pow_table() {
    PowTable t{};
    uint64_t r = 1;
    for (int n = 0; n < 3 * LEN + 21; ++n) {
        t.v[n] = (uint32_t)r;
        r = (r * A) % M31;
    }
    return t;
}

// a * b mod (2^31 - 1) for a, b < 2^31 (Mersenne folding). With a * b = Q * 2^31 + R (R < 2^31), the product
// p = a * 2b is Q * 2^32 + 2R, so its high word is Q and its low word shifted right by one is R; Q + R < 2M
// and Q + R = a * b (mod M). For a compile-time b this is v_mad_u64_u32 + lshr + add + a conditional
// subtract: no mask with a literal and no v_alignbit (both half rate on gfx950). `nm` is -M (mod 2^32); a hot
// loop passes it in a VGPR the compiler cannot see through, so that the subtract is a full-rate VGPR-VGPR add
// instead of an add with a literal.
constexpr uint32_t NEG_M31 = 0u - M31;
__host__ __device__ __forceinline__ uint32_t modmul(uint32_t a, uint32_t b, uint32_t nm = NEG_M31) {
    const uint64_t p = (uint64_t)a * (2u * b);
    const uint32_t r = (uint32_t)(p >> 32) + ((uint32_t)p >> 1);
    uint32_t t;
    const bool borrow = __builtin_sub_overflow(r, 0u - nm, &t);
    return borrow ? r : t;
}

// (a * b mod (2^31 - 1)) << 8 for a, b in [1, 2^31 - 1): only the low 24 bits of the residue survive the shift.
// r = Q + R (as in modmul) is never M, because a * b is not 0 mod the prime M; so the residue is r when r < 2^31
// and r - M = r + 1 - 2^31 otherwise, and its low 24 bits are those of r + (r >> 31). No compare, no select.
__host__ __device__ __forceinline__ uint32_t modmul_shl8(uint32_t a, uint32_t b) {
    const uint64_t p = (uint64_t)a * (2u * b);
    const uint32_t r = (uint32_t)(p >> 32) + ((uint32_t)p >> 1);
    return (r + (r >> 31)) << 8;
}

// Go's `seed % int32max; if seed < 0 { seed += int32max }; if seed == 0 { seed = 89482311 }`
__host__ __device__ inline uint32_t seed_reduce(int64_t seed) {
    int64_t s = seed % (int64_t)M31;
    if (s < 0) s += M31;
    if (s == 0) s = 89482311;
    return (uint32_t)s;
}

// seeded vec[i] for a compile-time index
template <int I>
__host__ __device__ __forceinline__ uint64_t vec_c(uint32_t s, uint32_t nm = NEG_M31) {
    constexpr uint32_t ca = pow_a(21 + 3 * I), cb = pow_a(22 + 3 * I), cc = pow_a(23 + 3 * I);
    constexpr uint64_t ck = NMZ_GO_RNG_COOKED[I];
    const uint32_t xb = modmul(s, cb, nm), xc = modmul(s, cc, nm);
    const uint32_t lo = (xb << 20) ^ xc ^ (uint32_t)ck;
    const uint32_t hi = modmul_shl8(s, ca) ^ (xb >> 12) ^ (uint32_t)(ck >> 32);
    return ((uint64_t)hi << 32) | lo;
}

// high word of the seeded vec[I] (only x_{21+3I} and x_{22+3I} enter it)
template <int I>
__host__ __device__ __forceinline__ uint32_t vec_hi(uint32_t s, uint32_t nm = NEG_M31) {
    constexpr uint32_t ca = pow_a(21 + 3 * I), cb = pow_a(22 + 3 * I);
    constexpr uint64_t ck = NMZ_GO_RNG_COOKED[I];
    return modmul_shl8(s, ca) ^ (modmul(s, cb, nm) >> 12) ^ (uint32_t)(ck >> 32);
}

// outputs 0 and 1 after Seed (no state)
__host__ __device__ __forceinline__ uint64_t out0(uint32_t s, uint32_t nm = NEG_M31) {
    return vec_c<333>(s, nm) + vec_c<606>(s, nm);
}
__host__ __device__ __forceinline__ uint64_t out1(uint32_t s, uint32_t nm = NEG_M31) {
    return vec_c<332>(s, nm) + vec_c<605>(s, nm);
}

}  // namespace gorand
}  // namespace nmz

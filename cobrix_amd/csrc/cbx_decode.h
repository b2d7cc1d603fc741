// cbx_decode.h -- per-field decoders of the Cobrix hot path, written for gfx950 lanes.
//
// Each function decodes ONE field value held in (LDS-staged) bytes and returns the value the
// reference produces after Spark's schema conversion, or "invalid" (null).  They are
// arithmetic restatements of the reference's string-building decoders:
//   BCD     -> BCDNumberDecoders.scala:29-168 + DecoderSelector.scala:259-281
//   binary  -> BinaryNumberDecoders.scala:21-135, BinaryUtils.scala:194-276
//   zoned   -> StringDecoders.scala:154-346 (decodeEbcdicNumber + Int/Long/BigNumber/BigDecimal)
//   floats  -> FloatingPointDecoders.scala:33-180 (incl. the IBM-single exponent-mask behaviour)
//   strings -> StringDecoders.scala:44-89, StringTools.scala:28-61
//   decimal conversion -> Spark Decimal.toPrecision (HALF_UP, null on overflow)
// (paths under /root/reference/cobol-parser/src/main/scala/za/co/absa/cobrix/cobol/parser/decoders/)
//
// All functions are __host__ __device__ so tests/native can fuzz the exact device arithmetic
// against the oracle on a CPU; the product only runs them inside the HIP kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cobrix_hip.h"

#define CBX_HD __host__ __device__ __forceinline__

namespace cbx {

// ------------------------------------------------------------------------------------------
// 128-bit unsigned helpers (no __int128 division on the device)
// ------------------------------------------------------------------------------------------
struct U128 {
    uint64_t lo, hi;
};

CBX_HD U128 u128(uint64_t lo, uint64_t hi = 0) { return U128{lo, hi}; }

CBX_HD uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

// a * m + add, m < 2^32; returns false on overflow past 128 bits
CBX_HD bool u128_muladd(U128& a, uint32_t m, uint32_t add) {
    uint64_t lo = a.lo * m;
    uint64_t carry = mulhi64(a.lo, m);
    uint64_t hi_lo = a.hi * m;
    uint64_t hi_hi = mulhi64(a.hi, m);
    uint64_t nlo = lo + add;
    carry += (nlo < lo);
    uint64_t nhi = hi_lo + carry;
    bool ovf = hi_hi != 0 || nhi < hi_lo;
    a.lo = nlo;
    a.hi = nhi;
    return !ovf;
}

CBX_HD bool u128_lt(U128 a, U128 b) { return a.hi < b.hi || (a.hi == b.hi && a.lo < b.lo); }
CBX_HD bool u128_is_zero(U128 a) { return (a.lo | a.hi) == 0; }

// a /= d (d < 2^32), returns remainder
CBX_HD uint32_t u128_divmod32(U128& a, uint32_t d) {
    uint64_t r = 0;
    uint32_t limbs[4] = {(uint32_t)(a.hi >> 32), (uint32_t)a.hi, (uint32_t)(a.lo >> 32), (uint32_t)a.lo};
    uint32_t q[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint64_t cur = (r << 32) | limbs[i];
        q[i] = (uint32_t)(cur / d);
        r = cur % d;
    }
    a.hi = ((uint64_t)q[0] << 32) | q[1];
    a.lo = ((uint64_t)q[2] << 32) | q[3];
    return (uint32_t)r;
}

CBX_HD U128 u128_neg(U128 a) {
    U128 r;
    r.lo = ~a.lo + 1;
    r.hi = ~a.hi + (r.lo == 0 ? 1 : 0);
    return r;
}

// multiply by 10^k; false on overflow
CBX_HD bool u128_mul_pow10(U128& a, int k) {
    bool ok = true;
    while (k >= 9) { ok &= u128_muladd(a, 1000000000u, 0); k -= 9; }
    uint32_t m = 1;
    while (k > 0) { m *= 10; k--; }
    if (m != 1) ok &= u128_muladd(a, m, 0);
    return ok;
}

// number of decimal digits of a (0 -> 1), as Java's BigInteger.toString().length
CBX_HD int u128_ndigits(U128 a) {
    int n = 0;
    if (a.hi == 0) {
        uint64_t x = a.lo;
        do { n++; x /= 10; } while (x);
        return n;
    }
    while (!u128_is_zero(a)) { u128_divmod32(a, 10); n++; }
    return n;
}

// ------------------------------------------------------------------------------------------
// Device-side field descriptor (derived from cbx_field by the plan)
// ------------------------------------------------------------------------------------------
struct Field {
    int32_t kind, out_type, offset, size;
    int32_t precision, scale, sf, out_p, out_s;
    int32_t flags, trim, n_dims;
    int32_t dim_count[CBX_MAX_DIMS];
    int32_t dim_stride[CBX_MAX_DIMS];
    int32_t dim_array[CBX_MAX_DIMS];
    int32_t segment, column;
    int32_t n_slots;        // product of dim_count
    int32_t window;         // LDS window the field (all its elements) is staged in, -1 = global
    uint64_t lim_lo, lim_hi;  // 10^out_p (decimal overflow bound)
};

// cbx_field (ABI) -> Field (device), host side
inline Field make_field(const cbx_field& f) {
    Field d{};
    d.kind = f.kind; d.out_type = f.out_type; d.offset = f.offset; d.size = f.size;
    d.precision = f.precision; d.scale = f.scale; d.sf = f.scale_factor;
    d.out_p = f.out_precision; d.out_s = f.out_scale; d.flags = f.flags; d.trim = f.trim;
    d.n_dims = f.n_dims;
    d.n_slots = 1;
    for (int k = 0; k < CBX_MAX_DIMS; k++) {
        d.dim_count[k] = f.dim_count[k]; d.dim_stride[k] = f.dim_stride[k]; d.dim_array[k] = f.dim_array[k];
        if (k < f.n_dims) d.n_slots *= f.dim_count[k];
    }
    d.segment = f.segment; d.column = f.column;
    unsigned __int128 lim = 1;
    for (int i = 0; i < f.out_precision; i++) lim *= 10;
    d.lim_lo = (uint64_t)lim; d.lim_hi = (uint64_t)(lim >> 64);
    d.window = -1;
    return d;
}

struct Val {
    uint64_t lo, hi;  // two's complement 128-bit value, or float/double bits in lo
    bool valid;
};

CBX_HD Val null_val() { return Val{0, 0, false}; }

// Spark Decimal.toPrecision(P, S, HALF_UP): magnitude M at scale vs -> unscaled at S, null when
// it needs more than P digits.
CBX_HD Val finalize_decimal(U128 M, bool m_ovf, int vs, bool neg, const Field& f) {
    const int S = f.out_s;
    if (m_ovf) return null_val();
    if (vs < S) {
        if (!u128_mul_pow10(M, S - vs)) return null_val();
    } else if (vs > S) {
        int k = vs - S;
        // drop k digits, HALF_UP on the first dropped digit (the rest only matter for ties >= .5,
        // which the first digit >= 5 already decides)
        int j = k - 1;
        while (j >= 9) { u128_divmod32(M, 1000000000u); j -= 9; }
        uint32_t d = 1;
        while (j > 0) { d *= 10; j--; }
        if (d != 1) u128_divmod32(M, d);
        uint32_t first = u128_divmod32(M, 10);
        if (first >= 5) u128_muladd(M, 1, 1);
    }
    if (!u128_lt(M, U128{f.lim_lo, f.lim_hi})) return null_val();
    U128 v = neg ? u128_neg(M) : M;
    return Val{v.lo, v.hi, true};
}

// ------------------------------------------------------------------------------------------
// COMP-3  (BCDNumberDecoders.decodeBCDIntegralNumber / decodeBigBCDNumber)
// ------------------------------------------------------------------------------------------
CBX_HD Val decode_bcd(const Field& f, const uint8_t* p) {
    const int n = f.size;
    U128 M = u128(0);
    bool ovf = false;
    bool bad = false;
    int sig = 0;
    for (int i = 0; i < n; i++) {
        uint32_t b = p[i];
        uint32_t hi = b >> 4, lo = b & 15;
        bad |= hi > 9;
        sig += (sig > 0 || hi != 0);
        ovf |= !u128_muladd(M, 10, hi);
        if (i + 1 < n) {
            bad |= lo > 9;
            sig += (sig > 0 || lo != 0);
            ovf |= !u128_muladd(M, 10, lo);
        }
    }
    uint32_t sn = p[n - 1] & 15;
    bad |= !(sn == 0xC || sn == 0xD || sn == 0xF);
    if (bad) return null_val();
    bool neg = sn == 0xD;
    if ((f.flags & CBX_F_INTEGRAL) && f.precision <= 18) {
        // Java long arithmetic wraps (19 digits at p = 18)
        uint64_t v = neg ? (uint64_t)0 - M.lo : M.lo;
        return Val{v, (uint64_t)((int64_t)v >> 63), true};
    }
    (void)sig;
    if (f.flags & CBX_F_INTEGRAL) return finalize_decimal(M, ovf, 0, neg, f);
    if (f.sf == 0) return finalize_decimal(M, ovf, f.scale, neg, f);
    if (f.sf > 0) {
        ovf |= !u128_mul_pow10(M, f.sf);
        return finalize_decimal(M, ovf, 0, neg, f);
    }
    return finalize_decimal(M, ovf, -f.sf + 2 * n - 1, neg, f);
}

// ------------------------------------------------------------------------------------------
// COMP / COMP-4 / COMP-5 / COMP-9
// ------------------------------------------------------------------------------------------
CBX_HD Val decode_binary(const Field& f, const uint8_t* p) {
    const int n = f.size;
    const bool be = (f.flags & CBX_F_BIG_ENDIAN) != 0;
    const bool sgn = (f.flags & CBX_F_SIGNED) != 0;
    // two's complement / unsigned value of up to 16 bytes
    U128 v = u128(0);
    for (int i = 0; i < n; i++) {
        uint32_t b = p[be ? i : n - 1 - i];
        v.hi = (v.hi << 8) | (v.lo >> 56);
        v.lo = (v.lo << 8) | b;
    }
    bool neg = false;
    if (sgn && n < 16 && n > 0) {
        uint32_t top = p[be ? 0 : n - 1];
        if (top & 0x80) {
            // sign-extend from n bytes
            int bits = 8 * n;
            if (bits < 64) {
                v.lo |= ~(uint64_t)0 << bits;
                v.hi = ~(uint64_t)0;
            } else {
                v.hi |= ~(uint64_t)0 << (bits - 64);
            }
            neg = true;
        }
    } else if (sgn && n == 16) {
        neg = (v.hi >> 63) != 0;
    }
    if (f.flags & CBX_F_INTEGRAL) {
        if (n == 1 || n == 2 || n == 4) {
            if (!sgn && n == 4 && (v.lo & 0x80000000u)) return null_val();
            return Val{v.lo, v.hi, true};
        }
        if (n == 8) {
            if (!sgn && (v.lo >> 63)) return null_val();
            return Val{v.lo, (uint64_t)((int64_t)v.lo >> 63), true};
        }
        U128 M = neg ? u128_neg(v) : v;
        return finalize_decimal(M, false, 0, neg, f);
    }
    U128 M = neg ? u128_neg(v) : v;
    if (f.sf == 0) return finalize_decimal(M, false, f.scale, neg, f);
    if (f.sf > 0) {
        bool ok = u128_mul_pow10(M, f.sf);
        return finalize_decimal(M, !ok, 0, neg, f);
    }
    return finalize_decimal(M, false, -f.sf + u128_ndigits(M), neg, f);
}

// ------------------------------------------------------------------------------------------
// EBCDIC DISPLAY numbers (decodeEbcdicNumber + the Int/Long/BigNumber/BigDecimal wrappers)
// ------------------------------------------------------------------------------------------
// Java-level result of decodeEbcdicNumber summarised: sign (0 none, 1 '+', 2 '-'), digit count,
// dot count, digits after the first dot, digit magnitude (38 significant digits max, ovf beyond).
CBX_HD Val zoned_finish(const Field& f, bool malformed, int sign, int nd, int ndots, int after, U128 D,
                        bool ovf) {
    const bool neg = sign == 2;
    if (malformed || (neg && !(f.flags & CBX_F_SIGNED))) return null_val();
    if (f.flags & CBX_F_INTEGRAL) {
        if (f.precision <= 18) {
            // Integer.parseInt / Long.parseLong
            if (ndots != 0 || nd == 0 || ovf || D.hi != 0) return null_val();
            uint64_t lim = f.precision <= 9 ? (neg ? 0x80000000ull : 0x7FFFFFFFull)
                                            : (neg ? 0x8000000000000000ull : 0x7FFFFFFFFFFFFFFFull);
            if (D.lo > lim) return null_val();
            uint64_t v = neg ? (uint64_t)0 - D.lo : D.lo;
            return Val{v, (uint64_t)((int64_t)v >> 63), true};
        }
        // decodeEbcdicBigNumber(_, unsigned) = BigDecimal(S)
        if (ndots > 1 || nd == 0) return null_val();
        return finalize_decimal(D, ovf, ndots ? after : 0, neg, f);
    }
    if (f.flags & CBX_F_EXPLICIT_DOT) {
        if (ndots > 1 || nd == 0) return null_val();
        return finalize_decimal(D, ovf, ndots ? after : 0, neg, f);
    }
    if (f.sf == 0) {
        // addDecimalPoint(S, scale, 0): any dot -> two dots; "+d" shorter than the scale -> "0.+d"
        if (ndots != 0 || (sign == 1 && nd < f.scale)) return null_val();
        return finalize_decimal(D, ovf, f.scale, neg, f);
    }
    if (f.sf > 0) {
        if (ndots > 1) return null_val();
        ovf |= !u128_mul_pow10(D, f.sf);
        return finalize_decimal(D, ovf, ndots ? after + f.sf : 0, neg, f);
    }
    if (ndots != 0) return null_val();
    return finalize_decimal(D, ovf, -f.sf + nd, neg, f);
}

CBX_HD Val decode_zoned(const Field& f, const uint8_t* p) {
    const int n = f.size;
    bool malformed = false;
    int sign = 0;  // 0 none, 1 '+', 2 '-'
    int nd = 0, ndots = 0, after = 0, sig = 0;
    U128 D = u128(0);
    bool ovf = false;
    for (int i = 0; i < n; i++) {
        uint32_t c = p[i];
        uint32_t hi = c >> 4, lo = c & 15;
        bool dig = lo <= 9 && (hi == 0xF || (sign == 0 && (hi == 0xC || hi == 0xD)));
        bool sch = sign == 0 && (c == 0x60 || c == 0x4E);
        bool dot = c == 0x4B || c == 0x6B;
        bool spc = c == 0x40 || c == 0;
        if (sign == 0 && dig && hi != 0xF) sign = hi == 0xD ? 2 : 1;
        if (sch) sign = c == 0x60 ? 2 : 1;
        malformed |= !(dig || sch || dot || spc);
        if (dig) {
            nd++;
            after += ndots > 0;
            bool s = sig > 0 || lo != 0;
            sig += s;
            if (sig <= 38) u128_muladd(D, 10, lo);
            else ovf = true;
        }
        ndots += dot;
    }
    return zoned_finish(f, malformed, sign, nd, ndots, after, D, ovf);
}

// ------------------------------------------------------------------------------------------
// COMP-1 / COMP-2
// ------------------------------------------------------------------------------------------
// decodeIbmSingleBigEndian, restated bit for bit (the exponent mask is the sign bit)
CBX_HD uint32_t ibm_single_bits(uint32_t mant) {
    int32_t m = (int32_t)mant;
    int32_t sign = m & (int32_t)0x80000000;
    int32_t frac = m & 0x00FFFFFF;
    int32_t expo = (m & (int32_t)0x80000000) >> 22;
    if (frac == 0) return 0u;
    int32_t top = frac & 0x00F00000;
    if (top == 0) {
        // leading zero nibbles of the 24-bit fraction (the reference's shift-by-4 loop)
        int zn = (__builtin_clz((uint32_t)frac << 8)) >> 2;
        frac <<= 4 * zn; expo -= 4 * zn; top = frac & 0x00F00000;
    }
    int32_t lz = (int32_t)((0x000055AFu >> (top >> 19)) & 3);
    frac <<= lz;
    int32_t ce = expo + 131 - lz;
    if (ce >= 0 && ce < 254) return (uint32_t)sign + ((uint32_t)ce << 23) + (uint32_t)frac;
    if (ce > 254) return 0x7F800000u;
    if (ce >= -32) {
        int32_t mask = ~(int32_t)(0xFFFFFFFDu << (-1 - ce));
        int32_t ru = (frac & mask) > 0 ? 1 : 0;
        int32_t cf = ((frac >> (-1 - ce)) + ru) >> 1;
        return (uint32_t)sign + (uint32_t)cf;
    }
    return 0u;
}

// decodeIbmDoubleBigEndian (ibm2ieee), restated bit for bit
CBX_HD uint64_t ibm_double_bits(uint64_t m) {
    uint64_t sign = m & 0x8000000000000000ull;
    int64_t frac = (int64_t)(m & 0x00FFFFFFFFFFFFFFull);
    int64_t expo = (int64_t)((m & 0x7F00000000000000ull) >> 54);
    if (frac == 0) return 0ull;
    int64_t top = frac & 0x00F0000000000000ll;
    if (top == 0) {
        int zn = (__builtin_clzll((uint64_t)frac << 8)) >> 2;
        frac <<= 4 * zn; expo -= 4 * zn; top = frac & 0x00F0000000000000ll;
    }
    int64_t lz = (int64_t)((0x000055AFull >> (top >> 51)) & 3);
    frac <<= lz;
    int64_t ce = expo + 765 - lz;
    int64_t ru = (frac & 0xb) > 0 ? 1 : 0;
    int64_t cf = ((frac >> 2) + ru) >> 1;
    return sign + ((uint64_t)ce << 52) + (uint64_t)cf;
}

CBX_HD Val decode_float(const Field& f, const uint8_t* p) {
    const bool le = (f.flags & CBX_F_LITTLE_ENDIAN_FP) != 0;
    uint32_t w = 0;
    for (int i = 0; i < 4; i++) w = (w << 8) | p[le ? 3 - i : i];
    uint32_t bits = (f.flags & CBX_F_IBM) ? ibm_single_bits(w) : w;
    return Val{bits, 0, true};
}

CBX_HD Val decode_double(const Field& f, const uint8_t* p) {
    const bool le = (f.flags & CBX_F_LITTLE_ENDIAN_FP) != 0;
    uint64_t w = 0;
    for (int i = 0; i < 8; i++) w = (w << 8) | p[le ? 7 - i : i];
    uint64_t bits = (f.flags & CBX_F_IBM) ? ibm_double_bits(w) : w;
    return Val{bits, 0, true};
}

CBX_HD Val decode_numeric(const Field& f, const uint8_t* p) {
    switch (f.kind) {
    case CBX_K_BCD: return decode_bcd(f, p);
    case CBX_K_BINARY: return decode_binary(f, p);
    case CBX_K_ZONED: return decode_zoned(f, p);
    case CBX_K_FLOAT: return decode_float(f, p);
    case CBX_K_DOUBLE: return decode_double(f, p);
    default: return null_val();
    }
}

// ------------------------------------------------------------------------------------------
// Width-specialised decoders over field bytes held in registers (the hot path).
// FB<N>: byte j of the field sits in bits 8*(j&3) of w[j>>2]; loaded from the LDS image with
// dword reads + alignbyte, so a field costs ceil((N+6)/4) ds_read_b32 whatever its alignment.
// ------------------------------------------------------------------------------------------
template <int N>
struct FB {
    uint32_t w[(N + 3) / 4];
    CBX_HD uint32_t byte(int j) const { return (w[j >> 2] >> (8 * (j & 3))) & 0xFFu; }
};

CBX_HD uint32_t align_bytes(uint32_t hi, uint32_t lo, uint32_t sh) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (sh & 3)));
#endif
}

// buf: LDS image (or any byte buffer) with >= 8 readable bytes past the field
template <int N>
CBX_HD FB<N> load_field(const uint8_t* buf, uint32_t addr) {
    constexpr int NW = (N + 3) / 4;
    const uint32_t* p = (const uint32_t*)(buf + (addr & ~3u));
    const uint32_t sh = addr & 3u;
    uint32_t r[NW + 1];
#pragma unroll
    for (int k = 0; k <= NW; k++) r[k] = p[k];
    FB<N> b;
#pragma unroll
    for (int k = 0; k < NW; k++) b.w[k] = align_bytes(r[k + 1], r[k], sh);
    return b;
}

// big-endian value of bytes [i, i + k), k <= 8 (i, k compile-time after unrolling)
template <int N>
CBX_HD uint64_t fb_be(const FB<N>& b, int i, int k) {
    uint64_t v = 0;
#pragma unroll
    for (int j = 0; j < 16; j++)
        if (j < k) v = (v << 8) | b.byte(i + j);
    return v;
}

// 8 valid packed-BCD digits -> binary
CBX_HD uint32_t bcd8_bin(uint32_t x) {
    uint32_t t1 = ((x >> 4) & 0x0F0F0F0Fu) * 10u + (x & 0x0F0F0F0Fu);
    uint32_t t2 = ((t1 >> 8) & 0x00FF00FFu) * 100u + (t1 & 0x00FF00FFu);
    return (t2 >> 16) * 10000u + (t2 & 0xFFFFu);
}
CBX_HD uint64_t bcd16_bin(uint64_t x) {
    return (uint64_t)bcd8_bin((uint32_t)(x >> 32)) * 100000000ull + bcd8_bin((uint32_t)x);
}
// every nibble of x is a decimal digit
CBX_HD bool bcd_ok(uint64_t x) {
    uint64_t lo = x & 0x0F0F0F0F0F0F0F0Full, hi = (x >> 4) & 0x0F0F0F0F0F0F0F0Full;
    return (((lo + 0x0606060606060606ull) | (hi + 0x0606060606060606ull)) & 0x1010101010101010ull) == 0;
}

template <int N>
CBX_HD Val decode_bcd_n(const Field& f, const FB<N>& b) {
    constexpr int NL = N < 8 ? N : 8;      // bytes in the low part (carries the sign nibble)
    constexpr int NH = N - NL;             // leading bytes (digits only)
    const uint64_t lo = fb_be(b, NH, NL);
    const uint32_t sn = (uint32_t)lo & 15u;
    const uint64_t dlo = lo >> 4;          // 2*NL - 1 digits
    bool ok = bcd_ok(dlo) && (sn == 0xC || sn == 0xD || sn == 0xF);
    uint64_t hi = 0;
    if (NH > 0) { hi = fb_be(b, 0, NH); ok &= bcd_ok(hi); }
    if (!ok) return null_val();
    const bool neg = sn == 0xD;
    U128 M = u128(bcd16_bin(dlo));
    if (NH > 0) {
        // M = hi_value * 10^15 + lo_value
        uint64_t hv = bcd16_bin(hi);
        const uint64_t P15 = 1000000000000000ull;
        uint64_t plo = hv * P15, phi = mulhi64(hv, P15);
        uint64_t s = plo + M.lo;
        M.hi = phi + (s < plo);
        M.lo = s;
    }
    if ((f.flags & CBX_F_INTEGRAL) && f.precision <= 18) {
        uint64_t v = neg ? (uint64_t)0 - M.lo : M.lo;  // Java long arithmetic wraps
        return Val{v, (uint64_t)((int64_t)v >> 63), true};
    }
    if (f.flags & CBX_F_INTEGRAL) return finalize_decimal(M, false, 0, neg, f);
    if (f.sf == 0) return finalize_decimal(M, false, f.scale, neg, f);
    if (f.sf > 0) {
        bool okm = u128_mul_pow10(M, f.sf);
        return finalize_decimal(M, !okm, 0, neg, f);
    }
    return finalize_decimal(M, false, -f.sf + 2 * N - 1, neg, f);
}

template <int N>
CBX_HD Val decode_binary_n(const Field& f, const FB<N>& b) {
    const bool be = (f.flags & CBX_F_BIG_ENDIAN) != 0;
    const bool sgn = (f.flags & CBX_F_SIGNED) != 0;
    U128 v = u128(0);
#pragma unroll
    for (int i = 0; i < N; i++) {
        uint32_t x = be ? b.byte(i) : b.byte(N - 1 - i);
        v.hi = (v.hi << 8) | (v.lo >> 56);
        v.lo = (v.lo << 8) | x;
    }
    const uint32_t top = be ? b.byte(0) : b.byte(N - 1);
    bool neg = false;
    if (sgn && (top & 0x80)) {
        if (8 * N < 64) { v.lo |= ~(uint64_t)0 << (8 * N); v.hi = ~(uint64_t)0; }
        else if (8 * N < 128) v.hi |= ~(uint64_t)0 << (8 * N - 64);
        neg = true;
    }
    if (f.flags & CBX_F_INTEGRAL) {
        if (N == 1 || N == 2 || N == 4) {
            if (!sgn && N == 4 && (v.lo & 0x80000000u)) return null_val();
            return Val{v.lo, v.hi, true};
        }
        if (N == 8) {
            if (!sgn && (v.lo >> 63)) return null_val();
            return Val{v.lo, (uint64_t)((int64_t)v.lo >> 63), true};
        }
        U128 M = neg ? u128_neg(v) : v;
        return finalize_decimal(M, false, 0, neg, f);
    }
    U128 M = neg ? u128_neg(v) : v;
    if (f.sf == 0) return finalize_decimal(M, false, f.scale, neg, f);
    if (f.sf > 0) {
        bool ok = u128_mul_pow10(M, f.sf);
        return finalize_decimal(M, !ok, 0, neg, f);
    }
    return finalize_decimal(M, false, -f.sf + u128_ndigits(M), neg, f);
}

// Zoned: fast path for the common layout (F-zone digits, last byte optionally C/D overpunch);
// anything else (spaces, separate signs, dots, malformed bytes) takes the general state machine.
template <int N>
CBX_HD Val decode_zoned_n(const Field& f, const FB<N>& b, const uint8_t* buf, uint32_t addr) {
    bool fast = true;
    uint64_t acc = 0;
#pragma unroll
    for (int j = 0; j < N; j++) {
        uint32_t c = b.byte(j);
        uint32_t lo = c & 15u, hi = c >> 4;
        fast &= lo <= 9u;
        if (j + 1 < N) fast &= hi == 0xFu;
        else fast &= hi == 0xFu || hi == 0xCu || hi == 0xDu;
        acc = acc * 10u + lo;
    }
    if (fast) {
        uint32_t last = b.byte(N - 1) >> 4;
        int sign = last == 0xD ? 2 : (last == 0xC ? 1 : 0);
        // digits are all significant-or-leading-zero; N <= 18 keeps acc exact
        return zoned_finish(f, false, sign, N, 0, 0, u128(acc), false);
    }
    Field g = f;
    g.size = N;
    return decode_zoned(g, buf + addr);
}

template <int N>
CBX_HD Val decode_float_n(const Field& f, const FB<N>& b) {
    const bool le = (f.flags & CBX_F_LITTLE_ENDIAN_FP) != 0;
    if (N == 4) {
        uint32_t w = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) w = (w << 8) | b.byte(le ? 3 - i : i);
        return Val{(f.flags & CBX_F_IBM) ? ibm_single_bits(w) : w, 0, true};
    }
    uint64_t w = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) w = (w << 8) | b.byte(le ? 7 - i : i);
    return Val{(f.flags & CBX_F_IBM) ? ibm_double_bits(w) : w, 0, true};
}

#define CBX_SIZE_CASES_16(M) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15) M(16)
#define CBX_SIZE_CASES_18(M) CBX_SIZE_CASES_16(M) M(17) M(18)

// Numeric field whose bytes start at buf[addr] (bounds already checked by the caller).
CBX_HD Val decode_numeric_at(const Field& f, const uint8_t* buf, uint32_t addr) {
    switch (f.kind) {
    case CBX_K_BCD:
        switch (f.size) {
#define CBX_BCD_CASE(n) case n: return decode_bcd_n<n>(f, load_field<n>(buf, addr));
            CBX_SIZE_CASES_16(CBX_BCD_CASE)
#undef CBX_BCD_CASE
        default: return decode_bcd(f, buf + addr);
        }
    case CBX_K_BINARY:
        switch (f.size) {
#define CBX_BIN_CASE(n) case n: return decode_binary_n<n>(f, load_field<n>(buf, addr));
            CBX_SIZE_CASES_16(CBX_BIN_CASE)
#undef CBX_BIN_CASE
        default: return decode_binary(f, buf + addr);
        }
    case CBX_K_ZONED:
        switch (f.size) {
#define CBX_ZON_CASE(n) case n: return decode_zoned_n<n>(f, load_field<n>(buf, addr), buf, addr);
            CBX_SIZE_CASES_18(CBX_ZON_CASE)
#undef CBX_ZON_CASE
        default: return decode_zoned(f, buf + addr);
        }
    case CBX_K_FLOAT: return decode_float_n<4>(f, load_field<4>(buf, addr));
    case CBX_K_DOUBLE: return decode_float_n<8>(f, load_field<8>(buf, addr));
    default: return null_val();
    }
}

// ------------------------------------------------------------------------------------------
// Strings: trimmed range + UTF-8 length, then the write
// ------------------------------------------------------------------------------------------
struct StrSpan {
    int begin, end;   // kept byte range of the field (after trim)
    int utf8_len;
};

// lut: code page entries (cbx_plan_options.lut)
CBX_HD uint32_t ascii_lut(uint32_t b) {
    // decodeAsciiString: Java signed bytes < 32 (incl. >= 0x80) become ' '
    uint32_t c = (b < 32 || b >= 128) ? 0x20u : b;
    return c | (1u << 24) | (c <= 0x20 ? 0x80000000u : 0u);
}

template <typename LutFn>
CBX_HD StrSpan string_span(const Field& f, const uint8_t* p, int n, LutFn lut) {
    StrSpan s{0, n, 0};
    if (f.kind == CBX_K_HEX) { s.utf8_len = 2 * n; return s; }
    if (f.kind == CBX_K_RAW) { s.utf8_len = n; return s; }
    const bool tl = f.trim == CBX_TRIM_LEFT || f.trim == CBX_TRIM_BOTH;
    const bool tr = f.trim == CBX_TRIM_RIGHT || f.trim == CBX_TRIM_BOTH;
    int b = 0, e = n;
    if (tl) while (b < e && (lut(p[b]) >> 31)) b++;
    if (tr) while (e > b && (lut(p[e - 1]) >> 31)) e--;
    int len = 0;
    for (int i = b; i < e; i++) len += (lut(p[i]) >> 24) & 3;
    s.begin = b; s.end = e; s.utf8_len = len;
    return s;
}

template <typename LutFn>
CBX_HD void string_write(const Field& f, const uint8_t* p, const StrSpan& s, uint8_t* out, LutFn lut) {
    if (f.kind == CBX_K_HEX) {
        const char* H = "0123456789ABCDEF";
        for (int i = s.begin; i < s.end; i++) {
            out[2 * (i - s.begin)] = (uint8_t)H[p[i] >> 4];
            out[2 * (i - s.begin) + 1] = (uint8_t)H[p[i] & 15];
        }
        return;
    }
    if (f.kind == CBX_K_RAW) {
        for (int i = s.begin; i < s.end; i++) out[i - s.begin] = p[i];
        return;
    }
    int k = 0;
    for (int i = s.begin; i < s.end; i++) {
        uint32_t e = lut(p[i]);
        uint32_t l = (e >> 24) & 3;
        out[k] = (uint8_t)e;
        if (l > 1) out[k + 1] = (uint8_t)(e >> 8);
        if (l > 2) out[k + 2] = (uint8_t)(e >> 16);
        k += l;
    }
}

}  // namespace cbx

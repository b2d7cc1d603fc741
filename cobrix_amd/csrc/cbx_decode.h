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
    while (top == 0) { frac <<= 4; expo -= 4; top = frac & 0x00F00000; }
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
    while (top == 0) { frac <<= 4; expo -= 4; top = frac & 0x00F0000000000000ll; }
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

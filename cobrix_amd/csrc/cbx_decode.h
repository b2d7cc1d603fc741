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
// Two layers:
//   * generic byte-loop decoders (decode_bcd / decode_binary / decode_zoned / decode_float /
//     decode_double): any width, any flag combination -- the specification the fast paths are
//     fuzzed against;
//   * runtime-width SWAR fast paths over an LDS record image (decode_value): a field ending at
//     image byte `end` is read as the 8 or 16 bytes before `end` (three dword reads + alignbyte
//     per 8 bytes, whatever the alignment) and decoded with packed-nibble / packed-byte arithmetic.
//     One code path per (kind, width class) instead of one per width keeps the kernel small.
// All functions are __host__ __device__ so tests/native can fuzz the exact device arithmetic
// against the oracle on a CPU; the product only runs them inside the HIP kernels.
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif   /* hipRTC (cbx_jit.h) provides the runtime and the fixed-width types */

#include "cobrix_hip.h"

#define CBX_HD __host__ __device__ __forceinline__
#define CBX_HD_NOINLINE __host__ __device__ __attribute__((noinline))

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
// decoder variant per field (chosen by the plan from kind / width / flags)
enum Variant : int32_t {
    V_GENERIC = 0,   // byte-loop decoder (wide or unusual numerics): deferred to the fixup kernel
    V_BCD8 = 1,      // COMP-3, 1..8 bytes (<= 15 digits): one 64-bit packed-nibble conversion
    V_BCD16 = 2,     // COMP-3, 9..16 bytes (<= 31 digits): two conversions, 128-bit result
    V_BIN8 = 3,      // COMP/COMP-4/5/9 of 1, 2, 4 or 8 bytes (integral, or decimal without P-scaling)
    V_ZONED16 = 4,   // DISPLAY, <= 16 bytes: SWAR fast path (F-zone digits, last-byte overpunch);
                     // any other form (spaces, separate signs, dots, bad bytes) is deferred
    V_FP = 5,        // COMP-1 / COMP-2 (IBM hex or IEEE-754, either byte order)
    V_STRING = 6,    // EBCDIC / ASCII / HEX / RAW strings
    V_RECORD_ID = 7, // generated Record_Id
    V_FILE_ID = 8    // generated File_Id
};

struct Field {
    int32_t kind, out_type, offset, size;
    int32_t precision, scale, sf, out_p, out_s;
    int32_t flags, trim, n_dims;
    int32_t dim_count[CBX_MAX_DIMS];
    int32_t dim_stride[CBX_MAX_DIMS];
    int32_t dim_array[CBX_MAX_DIMS];
    int32_t segment, column;
    int32_t n_slots;        // product of dim_count
    int32_t variant;        // Variant
    int32_t seq;            // strings: index of the (column, slot 0) string sequence, -1 otherwise
    int32_t max_utf8;       // strings: max output bytes per input byte (LUT width, HEX 2)
    int32_t defer;          // numerics that may need the byte-loop decoder: first deferral sequence, else -1
    int32_t fin;            // fast paths: 0 two's-complement integral, 1 decimal (x 10^E after a bound check)
    int32_t plus_null;      // zoned fast path: a '+' overpunch yields null (addDecimalPoint quirk)
    int32_t e_mul;          // fast paths: E = Spark scale - raw scale of the decoded digits (0..19)
    int32_t e_lim;          // fast paths: magnitude bound exponent out_p - E (0..38)
    uint64_t lim_lo, lim_hi;  // 10^out_p (decimal overflow bound, byte-loop decoders)
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
    d.seq = -1;
    d.defer = -1;
    d.max_utf8 = 1;
    // Fast-path finish: a raw digit magnitude M at raw scale r becomes M * 10^E at the Spark
    // scale (E = out_s - r) after the bound check M < 10^(out_p - E); E < 0 would need HALF_UP
    // rounding, so such fields stay on the byte-loop decoder (V_GENERIC, deferred).
    auto fast_dec = [&](int r) -> bool {
        const int E = f.out_scale - r;
        if (E < 0 || E > 19 || f.out_precision - E < 0 || f.out_precision - E > 38) return false;
        d.fin = 1;
        d.e_mul = E;
        d.e_lim = f.out_precision - E;
        return true;
    };
    const bool integral = (f.flags & CBX_F_INTEGRAL) != 0;
    switch (f.kind) {
    case CBX_K_BCD:
        d.variant = f.size <= 8 ? V_BCD8 : (f.size <= 16 ? V_BCD16 : V_GENERIC);
        if (d.variant != V_GENERIC) {
            if (integral && f.precision <= 18) d.fin = 0;
            else if (!fast_dec(integral ? 0 : f.scale_factor == 0 ? f.scale
                               : f.scale_factor > 0 ? -f.scale_factor : -f.scale_factor + 2 * f.size - 1))
                d.variant = V_GENERIC;
        }
        break;
    case CBX_K_BINARY:
        d.variant = (f.size == 1 || f.size == 2 || f.size == 4 || f.size == 8) && (integral || f.scale_factor >= 0) ? V_BIN8 : V_GENERIC;
        if (d.variant == V_BIN8) {
            if (integral) d.fin = 0;
            else if (!fast_dec(f.scale_factor == 0 ? f.scale : -f.scale_factor)) d.variant = V_GENERIC;
        }
        break;
    case CBX_K_ZONED:
        d.variant = f.size <= 16 && !(f.flags & CBX_F_EXPLICIT_DOT) &&
                    (!integral || f.size <= (f.precision <= 9 ? 9 : 18)) ? V_ZONED16 : V_GENERIC;
        if (d.variant == V_ZONED16) {
            if (integral) d.fin = 0;
            else if (!fast_dec(f.scale_factor == 0 ? f.scale : f.scale_factor > 0 ? -f.scale_factor : -f.scale_factor + f.size))
                d.variant = V_GENERIC;
            d.plus_null = !integral && f.scale_factor == 0 && f.size < f.scale;
        }
        break;
    case CBX_K_ASCII_NUM: d.variant = V_GENERIC; break;   // byte-loop decoder (fixup kernel)
    case CBX_K_FLOAT: case CBX_K_DOUBLE: d.variant = V_FP; break;
    case CBX_K_STRING: case CBX_K_STRING_ASCII: case CBX_K_HEX: case CBX_K_RAW:
    case CBX_K_UTF16_BE: case CBX_K_UTF16_LE:
        d.variant = V_STRING;
        // UTF-16: a 2-byte unit -> <= 3 UTF-8 bytes, a 4-byte pair -> 4, a lone tail byte -> U+FFFD (3)
        d.max_utf8 = f.kind == CBX_K_HEX ? 2 : (f.kind == CBX_K_UTF16_BE || f.kind == CBX_K_UTF16_LE) ? 3 : 1;
        break;
    case CBX_K_RECORD_ID: d.variant = V_RECORD_ID; break;
    case CBX_K_FILE_ID: d.variant = V_FILE_ID; break;
    default: d.variant = V_GENERIC; break;
    }
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
template <typename BP>
CBX_HD Val decode_bcd(const Field& f, BP p) {
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
template <typename BP>
CBX_HD Val decode_binary(const Field& f, BP p) {
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

template <typename BP>
CBX_HD Val decode_zoned(const Field& f, BP p) {
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
// ASCII DISPLAY numbers (StringDecoders.decodeAsciiNumber, StringDecoders.scala:221-243, and the
// decodeAsciiInt / Long / BigNumber / BigDecimal wrappers, :259-361).  decodeAsciiNumber keeps
// the LAST '+'/'-' byte as the sign (wherever it is), maps '.' and ',' to '.', appends every
// other byte as a Java char (a signed byte >= 0x80 becomes U+FF80..U+FFFF: no digit, no space)
// and returns sign + buf.trim.  Integer/Long parsing is streamed; the BigDecimal wrappers build
// the Java string (<= kAsciiNumMax bytes, a plan limit) and parse it.
// ------------------------------------------------------------------------------------------
constexpr int kAsciiNumMax = 64;

// Integer.parseInt / Long.parseLong of decodeAsciiNumber(bytes): after the sign bytes are taken
// out, the trimmed rest must be one non-empty run of '0'..'9'.
template <typename BP>
CBX_HD Val ascii_integral(const Field& f, BP p) {
    const int n = f.size;
    int sign = 0, phase = 0, nd = 0;   // phase 0 leading spaces, 1 digits, 2 trailing spaces
    bool bad = false, big = false;
    uint64_t v = 0;
    for (int i = 0; i < n; i++) {
        const uint32_t c = p[i];
        if (c == '+' || c == '-') { sign = c == '-' ? 2 : 1; continue; }
        if (c <= 0x20) { phase = phase == 1 ? 2 : phase; continue; }
        if (phase == 2 || c < '0' || c > '9') { bad = true; continue; }
        phase = 1;
        nd++;
        big |= v > 1844674407370955160ull;
        v = v * 10 + (c - '0');
    }
    const bool neg = sign == 2;
    if (bad || nd == 0 || big || (neg && !(f.flags & CBX_F_SIGNED))) return null_val();
    const uint64_t lim = f.precision <= 9 ? (neg ? 0x80000000ull : 0x7FFFFFFFull)
                                          : (neg ? 0x8000000000000000ull : 0x7FFFFFFFFFFFFFFFull);
    if (v > lim) return null_val();
    v = neg ? (uint64_t)0 - v : v;
    return Val{v, (uint64_t)((int64_t)v >> 63), true};
}

// Spark Decimal.toPrecision of the exact BigDecimal  (M * 10^-vs), M holding the leading <= 38
// significant digits and `first_cut` the first digit cut off after them (-1: none cut, vs
// already counts the cut digits out).  HALF_UP needs only the first dropped digit.
CBX_HD Val finalize_decimal_wide(U128 M, int64_t vs, int first_cut, bool neg, const Field& f) {
    const int S = f.out_s;
    if (u128_is_zero(M) && first_cut <= 0) return Val{0, 0, true};
    if (vs == S) {
        if (first_cut >= 5) u128_muladd(M, 1, 1);
        if (!u128_lt(M, U128{f.lim_lo, f.lim_hi})) return null_val();
        const U128 v = neg ? u128_neg(M) : M;
        return Val{v.lo, v.hi, true};
    }
    if (vs < S && S - vs > 38) return null_val();      // a non-zero M times >= 10^39
    if (vs > S && vs - S > 40) return Val{0, 0, true};   // every digit dropped, the first a 0
    return finalize_decimal(M, false, (int)vs, neg, f);
}

// java.math.BigDecimal(String) (significand [+-]?digits[.digits] | .digits, exponent [eE][+-]?digits)
// then the Spark conversion.
template <typename BP>
CBX_HD Val parse_java_bigdecimal(const Field& f, BP s, int n) {
    int i = 0;
    bool neg = false;
    if (i < n && (s[i] == '+' || s[i] == '-')) { neg = s[i] == '-'; i++; }
    int nd = 0, sig = 0, cut = 0, first_cut = -1;
    bool dot = false;
    int64_t scale = 0;
    U128 M = u128(0);
    for (; i < n; i++) {
        const uint32_t c = s[i];
        if (c >= '0' && c <= '9') {
            nd++;
            scale += dot;
            if (sig > 0 || c != '0') {
                if (sig < 38) { u128_muladd(M, 10, c - '0'); sig++; }
                else { if (cut == 0) first_cut = (int)(c - '0'); cut++; }
            }
        } else if (c == '.' && !dot) {
            dot = true;
        } else if (c == 'e' || c == 'E') {
            i++;
            bool eneg = false;
            if (i < n && (s[i] == '+' || s[i] == '-')) { eneg = s[i] == '-'; i++; }
            if (i >= n) return null_val();
            int64_t ex = 0;
            int ed = 0;
            for (; i < n; i++) {
                if (s[i] < '0' || s[i] > '9') return null_val();
                ex = ex * 10 + (s[i] - '0');
                ed += ex > 0;
                if (ed > 10) return null_val();
            }
            scale -= eneg ? -ex : ex;
            if (scale > 2147483647ll || scale < -2147483648ll) return null_val();
            break;
        } else {
            return null_val();
        }
    }
    if (nd == 0) return null_val();
    return finalize_decimal_wide(M, scale - cut, first_cut, neg, f);
}

template <typename BP>
CBX_HD Val decode_ascii_num(const Field& f, BP p) {
    if ((f.flags & CBX_F_INTEGRAL) && f.precision <= 18) return ascii_integral(f, p);
    const int n = f.size < kAsciiNumMax ? f.size : kAsciiNumMax;
    // decodeAsciiNumber -> s = [sign] + buf.trim
    uint8_t buf[kAsciiNumMax];
    int bl = 0, sign = 0;
    for (int i = 0; i < n; i++) {
        const uint32_t c = p[i];
        if (c == '+' || c == '-') sign = c == '-' ? 2 : 1;
        else buf[bl++] = (uint8_t)(c == ',' ? '.' : c >= 0x80 ? 0xFF : c);   // 0xFF: a U+FFxx char
    }
    if (sign == 2 && !(f.flags & CBX_F_SIGNED)) return null_val();
    int b = 0, e = bl;
    while (b < e && buf[b] <= 0x20) b++;
    while (e > b && buf[e - 1] <= 0x20) e--;
    uint8_t s[2 * kAsciiNumMax + 48];
    int sl = 0;
    if (sign) s[sl++] = sign == 2 ? '-' : '+';
    for (int i = b; i < e; i++) s[sl++] = buf[i];
    if ((f.flags & CBX_F_INTEGRAL) || (f.flags & CBX_F_EXPLICIT_DOT) || (f.scale == 0 && f.sf == 0))
        return parse_java_bigdecimal(f, s, sl);   // BigDecimal(s) == BigDecimal(addDecimalPoint(s, 0, 0))
    // BinaryUtils.addDecimalPoint(s, scale, scaleFactor) (BinaryUtils.scala:194-238)
    uint8_t t[2 * kAsciiNumMax + 48];
    int tl = 0;
    const bool is_neg = sl > 0 && s[0] == '-';
    if (f.sf == 0) {
        const int sc = f.scale;
        if (is_neg ? sl - 1 > sc : sl > sc) {
            for (int i = 0; i < sl - sc; i++) t[tl++] = s[i];
            t[tl++] = '.';
            for (int i = sl - sc; i < sl; i++) t[tl++] = s[i];
        } else {
            if (is_neg) t[tl++] = '-';
            t[tl++] = '0';
            t[tl++] = '.';
            for (int z = 0; z < sc - sl + (is_neg ? 1 : 0); z++) t[tl++] = '0';
            for (int i = is_neg ? 1 : 0; i < sl; i++) t[tl++] = s[i];
        }
    } else if (f.sf < 0) {
        if (is_neg) t[tl++] = '-';
        t[tl++] = '0';
        t[tl++] = '.';
        for (int z = 0; z < -f.sf; z++) t[tl++] = '0';
        for (int i = (sl > 0 && (s[0] == '-' || s[0] == '+')) ? 1 : 0; i < sl; i++) t[tl++] = s[i];
    } else {
        for (int i = 0; i < sl; i++) t[tl++] = s[i];
        for (int z = 0; z < f.sf; z++) t[tl++] = '0';
    }
    return parse_java_bigdecimal(f, t, tl);
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

template <typename BP>
CBX_HD Val decode_float(const Field& f, BP p) {
    const bool le = (f.flags & CBX_F_LITTLE_ENDIAN_FP) != 0;
    uint32_t w = 0;
    for (int i = 0; i < 4; i++) w = (w << 8) | p[le ? 3 - i : i];
    uint32_t bits = (f.flags & CBX_F_IBM) ? ibm_single_bits(w) : w;
    return Val{bits, 0, true};
}

template <typename BP>
CBX_HD Val decode_double(const Field& f, BP p) {
    const bool le = (f.flags & CBX_F_LITTLE_ENDIAN_FP) != 0;
    uint64_t w = 0;
    for (int i = 0; i < 8; i++) w = (w << 8) | p[le ? 7 - i : i];
    uint64_t bits = (f.flags & CBX_F_IBM) ? ibm_double_bits(w) : w;
    return Val{bits, 0, true};
}

template <typename BP>
CBX_HD Val decode_numeric(const Field& f, BP p) {
    switch (f.kind) {
    case CBX_K_BCD: return decode_bcd(f, p);
    case CBX_K_BINARY: return decode_binary(f, p);
    case CBX_K_ZONED: return decode_zoned(f, p);
    case CBX_K_ASCII_NUM: return decode_ascii_num(f, p);
    case CBX_K_FLOAT: return decode_float(f, p);
    case CBX_K_DOUBLE: return decode_double(f, p);
    default: return null_val();
    }
}

// ------------------------------------------------------------------------------------------
// Runtime-width fast paths over a record image.  `img` is an LDS (or host) byte image with at
// least 16 readable guard bytes before and 8 after every field; a field occupies
// img[addr, addr + size).  Callers have already applied the Primitive.decodeTypeValue bounds rule.
// ------------------------------------------------------------------------------------------
CBX_HD uint32_t align_bytes(uint32_t hi, uint32_t lo, uint32_t sh) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (sh & 3)));
#endif
}

// bytes [end - 8, end) as a little-endian u64 (byte end-8 in bits 0..7)
CBX_HD uint64_t img_le64_ending(const uint8_t* img, uint32_t end) {
    const uint32_t s = end - 8;
    const uint32_t* p = (const uint32_t*)(img + (s & ~3u));
    const uint32_t sh = s & 3u;
    const uint32_t r0 = p[0], r1 = p[1], r2 = p[2];
    return ((uint64_t)align_bytes(r2, r1, sh) << 32) | align_bytes(r1, r0, sh);
}

// mask keeping the low n bytes (n in 0..8)
CBX_HD uint64_t low_bytes_mask(int n) { return n >= 8 ? ~0ull : (n <= 0 ? 0ull : ((1ull << (8 * n)) - 1)); }
// mask keeping the high n bytes (n in 0..8)
CBX_HD uint64_t high_bytes_mask(int n) { return n >= 8 ? ~0ull : (n <= 0 ? 0ull : ~0ull << (8 * (8 - n))); }

// big-endian unsigned value of the n <= 8 bytes ending at `end`
CBX_HD uint64_t img_be(const uint8_t* img, uint32_t end, int n) {
    return __builtin_bswap64(img_le64_ending(img, end)) & low_bytes_mask(n);
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
// 8 digit bytes (0..9, most significant digit in the LOWEST byte) -> binary
CBX_HD uint32_t digits8_bin(uint64_t d) {
    d = d * 10u + (d >> 8);                                                     // byte 2j: pair value
    d = (d & 0x000000FF000000FFull) * 100u + ((d >> 16) & 0x000000FF000000FFull);  // dword j: quad value
    return (uint32_t)(d & 0xFFFFu) * 10000u + (uint32_t)((d >> 32) & 0xFFFFu);
}

// ------------------------------------------------------------------------------------------
// Numeric ops: one pre-resolved record per (field, slot) -- what the kernels' hot loop reads
// with a single scalar load (the plan flattens the descriptor tables into them).
// ------------------------------------------------------------------------------------------
enum NumFlags : uint32_t {
    NF_SIGNED = 1, NF_BIG_ENDIAN = 2, NF_INT = 4 /* fin == 0 */, NF_IBM = 8, NF_LE_FP = 16,
    NF_PLUS_NULL = 32, NF_FLOAT = 64 /* COMP-1 (else COMP-2) */
};

struct NumOp {
    int32_t eo;                       // element offset in the record (slot resolved, before start_off)
    uint8_t variant, size, out_type, flags;
    uint8_t n_odo, shift, run, run_odo; // shift: 64 - 8 * min(size, 8) (binary sign extension);
                                      // run: elements r = 0..run-1 of the field's innermost OCCURS
                                      // dimension share this record (0 / 1: a single element) at
                                      // eo + r * run_stride, slot + r, defer + r, and -- run_odo --
                                      // ODO index odo_idx[n_odo - 1] + r
    int32_t column;
    int32_t slot;
    int32_t defer;                    // deferral sequence of this element, -1 if never deferred
    int32_t segment;                  // segment-redefine group, -1 none
    int32_t run_stride;
    // plan-time constants of the fast paths (no table lookups or shifts by size in the kernel)
    uint64_t mask;                    // BCD8 / BIN8: low `size` bytes (after bswap); BCD16: low size-8
                                      // bytes of the leading word; ZONED16: high min(size, 8) bytes
    uint64_t mask0;                   // ZONED16: high size-8 bytes of the preceding word
    uint64_t mul;                     // 10^E (decimal fast finish)
    uint64_t lim_lo, lim_hi;          // 10^(out_p - E): magnitude bound
    uint64_t lim64;                   // the bound saturated to 64 bits (magnitudes that fit 64 bits)
    int16_t odo_arr[CBX_MAX_DIMS];    // OCCURS DEPENDING ON levels: element index odo_idx[j] must be
    int16_t odo_idx[CBX_MAX_DIMS];    // < the record's count of array odo_arr[j]
};
static_assert(sizeof(NumOp) == 96, "NumOp is a 96-byte scalar-load record");

inline NumOp make_numop(const Field& d, int slot, int eo, const int16_t* odo_arr, const int16_t* odo_idx, int n_odo) {
    NumOp o{};
    o.eo = eo;
    o.variant = (uint8_t)d.variant;
    o.size = (uint8_t)(d.size < 255 ? d.size : 255);
    o.out_type = (uint8_t)d.out_type;
    uint32_t fl = 0;
    if (d.flags & CBX_F_SIGNED) fl |= NF_SIGNED;
    if (d.flags & CBX_F_BIG_ENDIAN) fl |= NF_BIG_ENDIAN;
    if (d.fin == 0) fl |= NF_INT;
    if (d.flags & CBX_F_IBM) fl |= NF_IBM;
    if (d.flags & CBX_F_LITTLE_ENDIAN_FP) fl |= NF_LE_FP;
    if (d.plus_null) fl |= NF_PLUS_NULL;
    if (d.kind == CBX_K_FLOAT) fl |= NF_FLOAT;
    o.flags = (uint8_t)fl;
    o.n_odo = (uint8_t)n_odo;
    const int n8 = d.size < 8 ? d.size : 8;
    o.shift = (uint8_t)(64 - 8 * n8);
    switch (d.variant) {
    case V_BCD16: o.mask = low_bytes_mask(d.size - 8); break;
    case V_ZONED16: o.mask = high_bytes_mask(d.size); o.mask0 = high_bytes_mask(d.size - 8); break;
    default: o.mask = low_bytes_mask(d.size); break;
    }
    unsigned __int128 mul = 1, lim = 1;
    for (int i = 0; i < d.e_mul; i++) mul *= 10;
    for (int i = 0; i < d.e_lim; i++) lim *= 10;
    o.mul = (uint64_t)mul;
    o.lim_lo = (uint64_t)lim;
    o.lim_hi = (uint64_t)(lim >> 64);
    o.lim64 = o.lim_hi ? ~0ull : o.lim_lo;
    o.column = d.column;
    o.slot = slot;
    o.defer = d.defer >= 0 ? d.defer + slot : -1;
    o.segment = d.segment;
    for (int j = 0; j < CBX_MAX_DIMS; j++) {
        o.odo_arr[j] = j < n_odo ? odo_arr[j] : 0;
        o.odo_idx[j] = j < n_odo ? odo_idx[j] : 0;
    }
    return o;
}

// 10^k, k = 0..38, as 128-bit (lo, hi) words
#if defined(__HIP_DEVICE_COMPILE__)
__constant__ const uint64_t kPow10Lo[39] = {
    0x0000000000000001ull, 0x000000000000000aull, 0x0000000000000064ull,
    0x00000000000003e8ull, 0x0000000000002710ull, 0x00000000000186a0ull,
    0x00000000000f4240ull, 0x0000000000989680ull, 0x0000000005f5e100ull,
    0x000000003b9aca00ull, 0x00000002540be400ull, 0x000000174876e800ull,
    0x000000e8d4a51000ull, 0x000009184e72a000ull, 0x00005af3107a4000ull,
    0x00038d7ea4c68000ull, 0x002386f26fc10000ull, 0x016345785d8a0000ull,
    0x0de0b6b3a7640000ull, 0x8ac7230489e80000ull, 0x6bc75e2d63100000ull,
    0x35c9adc5dea00000ull, 0x19e0c9bab2400000ull, 0x02c7e14af6800000ull,
    0x1bcecceda1000000ull, 0x161401484a000000ull, 0xdcc80cd2e4000000ull,
    0x9fd0803ce8000000ull, 0x3e25026110000000ull, 0x6d7217caa0000000ull,
    0x4674edea40000000ull, 0xc0914b2680000000ull, 0x85acef8100000000ull,
    0x38c15b0a00000000ull, 0x378d8e6400000000ull, 0x2b878fe800000000ull,
    0xb34b9f1000000000ull, 0x00f436a000000000ull, 0x098a224000000000ull};
__constant__ const uint64_t kPow10Hi[39] = {
    0x0000000000000000ull, 0x0000000000000000ull, 0x0000000000000000ull,
    0x0000000000000000ull, 0x0000000000000000ull, 0x0000000000000000ull,
    0x0000000000000000ull, 0x0000000000000000ull, 0x0000000000000000ull,
    0x0000000000000000ull, 0x0000000000000000ull, 0x0000000000000000ull,
    0x0000000000000000ull, 0x0000000000000000ull, 0x0000000000000000ull,
    0x0000000000000000ull, 0x0000000000000000ull, 0x0000000000000000ull,
    0x0000000000000000ull, 0x0000000000000000ull, 0x0000000000000005ull,
    0x0000000000000036ull, 0x000000000000021eull, 0x000000000000152dull,
    0x000000000000d3c2ull, 0x0000000000084595ull, 0x000000000052b7d2ull,
    0x00000000033b2e3cull, 0x00000000204fce5eull, 0x00000001431e0faeull,
    0x0000000c9f2c9cd0ull, 0x0000007e37be2022ull, 0x000004ee2d6d415bull,
    0x0000314dc6448d93ull, 0x0001ed09bead87c0ull, 0x0013426172c74d82ull,
    0x00c097ce7bc90715ull, 0x0785ee10d5da46d9ull, 0x4b3b4ca85a86c47aull};
CBX_HD U128 pow10_u128(int k) { return U128{kPow10Lo[k], kPow10Hi[k]}; }
#else
inline U128 pow10_u128(int k) {
    unsigned __int128 x = 1;
    for (int i = 0; i < k; i++) x *= 10;
    return U128{(uint64_t)x, (uint64_t)(x >> 64)};
}
#endif

// Fast-path result typing (DecoderSelector.scala:104-281 + Spark Decimal.toPrecision) for a
// digit magnitude M: integral -> two's complement (BCD wraps as a Java long, as the reference);
// decimal -> null from 10^(out_p - E) on, else M * 10^E.  Branch-free apart from uniform tests
// on the op: every lane computes, `valid` selects.  W = output bytes (0: any): for W <= 8 only
// the low 64 bits are produced (a valid decimal of <= 18 digits fits them).
template <int W>
CBX_HD Val fast_finish(const NumOp& op, U128 M, bool neg, bool valid) {
    if (op.flags & NF_INT) {
        const uint64_t v = neg ? (uint64_t)0 - M.lo : M.lo;
        return Val{v, (uint64_t)((int64_t)v >> 63), valid};
    }
    if (W == 4 || W == 8) {
        valid &= M.hi == 0 && M.lo < op.lim64;
        const uint64_t r = M.lo * op.mul;
        const uint64_t v = neg ? (uint64_t)0 - r : r;
        return Val{v, (uint64_t)((int64_t)v >> 63), valid};
    }
    valid &= u128_lt(M, U128{op.lim_lo, op.lim_hi});
    U128 R;
    R.lo = M.lo * op.mul;
    R.hi = mulhi64(M.lo, op.mul) + M.hi * op.mul;
    if (neg) R = u128_neg(R);
    return Val{R.lo, R.hi, valid};
}

// The *_raw decoders take the 8 bytes ending at the element's end (r1 = img_le64_ending(img,
// end)) and, for 16-byte classes, the 8 before them (r0 = img_le64_ending(img, end - 8)).
template <int W>
CBX_HD Val bcd8_raw(const NumOp& op, uint64_t r1) {
    const uint64_t be = __builtin_bswap64(r1) & op.mask;
    const uint32_t sn = (uint32_t)be & 15u;
    const uint64_t dg = be >> 4;
    const bool valid = bcd_ok(dg) && (sn == 0xC || sn == 0xD || sn == 0xF);
    return fast_finish<W>(op, u128(bcd16_bin(dg)), sn == 0xD, valid);
}

template <int W>
CBX_HD Val bcd16_raw(const NumOp& op, uint64_t r1, uint64_t r0) {
    const uint64_t lo = __builtin_bswap64(r1);
    const uint64_t hi = __builtin_bswap64(r0) & op.mask;
    const uint32_t sn = (uint32_t)lo & 15u;
    const uint64_t dlo = lo >> 4;   // 15 digits
    const bool valid = bcd_ok(dlo) && bcd_ok(hi) && (sn == 0xC || sn == 0xD || sn == 0xF);
    const uint64_t hv = bcd16_bin(hi);
    const uint64_t P15 = 1000000000000000ull;
    const uint64_t plo = hv * P15, phi = mulhi64(hv, P15);
    U128 M;
    M.lo = plo + bcd16_bin(dlo);
    M.hi = phi + (M.lo < plo);
    return fast_finish<W>(op, M, sn == 0xD, valid);
}

template <int W>
CBX_HD Val bin8_raw(const NumOp& op, uint64_t le) {
    const int sh = op.shift;
    uint64_t v = (op.flags & NF_BIG_ENDIAN) ? (__builtin_bswap64(le) & op.mask) : (le >> sh);
    bool neg = false;
    if (op.flags & NF_SIGNED) {
        v = (uint64_t)((int64_t)(v << sh) >> sh);
        neg = (int64_t)v < 0;
    }
    if (op.flags & NF_INT) {
        // unsigned 4- and 8-byte values with the top bit set are null (BinaryNumberDecoders.scala:81-82, 111-112)
        const int n = op.size;
        const bool bad = !(op.flags & NF_SIGNED) && ((n == 4 && (v & 0x80000000ull)) || (n == 8 && (v >> 63)));
        return Val{v, neg ? ~0ull : 0ull, !bad};
    }
    // binary decimal (BinaryUtils.decodeBinaryNumber + addDecimalPoint), scale factor >= 0
    return fast_finish<W>(op, u128(neg ? (uint64_t)0 - v : v), neg, true);
}

template <int W>
CBX_HD Val zoned16_raw(const NumOp& op, uint64_t r1, uint64_t r0, bool& defer) {
    const uint64_t Z = 0xF0F0F0F0F0F0F0F0ull, L = 0x0F0F0F0F0F0F0F0Full;
    uint64_t b1 = r1;   // field bytes end-8 .. end-1 (last in the top byte)
    uint64_t b0 = r0;   // end-16 .. end-9
    // bytes in front of the field read as '0' digits (0xF0): leading zeros change nothing
    b1 = (b1 & op.mask) | (Z & ~op.mask);
    b0 = (b0 & op.mask0) | (Z & ~op.mask0);
    const uint32_t lastz = (uint32_t)(b1 >> 60);
    const uint64_t d0 = b0 & L, d1 = b1 & L;
    const bool fast = (b0 & Z) == Z && (((b1 & Z) | 0xF000000000000000ull) == Z) &&
                      (lastz == 0xF || lastz == 0xC || lastz == 0xD) &&
                      (((d0 + 0x0606060606060606ull) | (d1 + 0x0606060606060606ull)) & 0x1010101010101010ull) == 0;
    defer = !fast;
    const bool neg = lastz == 0xD;
    const bool valid = fast && !(neg && !(op.flags & NF_SIGNED)) && !(lastz == 0xC && (op.flags & NF_PLUS_NULL));
    const uint64_t v = (uint64_t)digits8_bin(d0) * 100000000ull + digits8_bin(d1);
    return fast_finish<W>(op, u128(v), neg, valid);
}

CBX_HD Val fp_raw(const NumOp& op, uint64_t le) {
    const bool lef = (op.flags & NF_LE_FP) != 0;
    if (op.flags & NF_FLOAT) {
        uint32_t w = (uint32_t)(le >> 32);
        if (!lef) w = __builtin_bswap32(w);
        return Val{(op.flags & NF_IBM) ? ibm_single_bits(w) : w, 0, true};
    }
    const uint64_t w = lef ? le : __builtin_bswap64(le);
    return Val{(op.flags & NF_IBM) ? ibm_double_bits(w) : w, 0, true};
}

// Numeric element at img[addr, addr + size) (bounds already checked by the caller).  Sets
// `defer` (result null) when the value needs the byte-loop decoder: the kernels record it in
// a deferral bitmap and the fixup kernel decodes it with decode_numeric.
template <int W = 0>
CBX_HD Val decode_value(const NumOp& op, const uint8_t* img, uint32_t addr, bool& defer) {
    const uint32_t end = addr + op.size;
    switch (op.variant) {
    case V_BCD8: return bcd8_raw<W>(op, img_le64_ending(img, end));
    case V_BCD16: return bcd16_raw<W>(op, img_le64_ending(img, end), img_le64_ending(img, end - 8));
    case V_BIN8: return bin8_raw<W>(op, img_le64_ending(img, end));
    case V_ZONED16: return zoned16_raw<W>(op, img_le64_ending(img, end), img_le64_ending(img, end - 8), defer);
    case V_FP: return fp_raw(op, img_le64_ending(img, end));
    default: defer = true; return null_val();
    }
}

// OCCURS DEPENDING ON source (integral, precision <= 18, RecordExtractors.scala:126-134): the
// value as a Java long (BCD wraps; zoned follows Integer/Long.parseInt; binary <= 8 bytes).
template <typename BP>
CBX_HD Val decode_count_int(const Field& f, BP p) {
    const int n = f.size;
    if (f.kind == CBX_K_BCD) {
        uint64_t v = 0;
        for (int i = 0; i < n; i++) {
            const uint32_t b = p[i], hi = b >> 4, lo = b & 15;
            if (hi > 9) return null_val();
            v = v * 10 + hi;
            if (i + 1 < n) {
                if (lo > 9) return null_val();
                v = v * 10 + lo;
            }
        }
        const uint32_t sn = p[n - 1] & 15;
        if (!(sn == 0xC || sn == 0xD || sn == 0xF)) return null_val();
        if (sn == 0xD) v = (uint64_t)0 - v;
        return Val{v, (uint64_t)((int64_t)v >> 63), true};
    }
    if (f.kind == CBX_K_BINARY) {
        const bool be = (f.flags & CBX_F_BIG_ENDIAN) != 0;
        uint64_t v = 0;
        for (int i = 0; i < n && i < 8; i++) v = (v << 8) | p[be ? i : n - 1 - i];
        if (f.flags & CBX_F_SIGNED) {
            const int sh = 64 - 8 * n;
            v = (uint64_t)((int64_t)(v << sh) >> sh);
        } else if ((n == 4 && (v & 0x80000000ull)) || (n == 8 && (v >> 63))) {
            return null_val();
        }
        return Val{v, (uint64_t)((int64_t)v >> 63), true};
    }
    if (f.kind == CBX_K_ASCII_NUM) return ascii_integral(f, p);
    if (f.kind == CBX_K_ZONED) {
        int sign = 0, nd = 0, ndots = 0;
        bool malformed = false, big = false;
        uint64_t v = 0;
        for (int i = 0; i < n; i++) {
            const uint32_t c = p[i], hi = c >> 4, lo = c & 15;
            const bool dig = lo <= 9 && (hi == 0xF || (sign == 0 && (hi == 0xC || hi == 0xD)));
            const bool sch = sign == 0 && (c == 0x60 || c == 0x4E);
            const bool dot = c == 0x4B || c == 0x6B;
            const bool spc = c == 0x40 || c == 0;
            if (sign == 0 && dig && hi != 0xF) sign = hi == 0xD ? 2 : 1;
            if (sch) sign = c == 0x60 ? 2 : 1;
            malformed |= !(dig || sch || dot || spc);
            if (dig) {
                nd++;
                big |= v > 1000000000000000000ull;
                v = v * 10 + lo;
            }
            ndots += dot;
        }
        const bool neg = sign == 2;
        if (malformed || (neg && !(f.flags & CBX_F_SIGNED)) || ndots != 0 || nd == 0 || big) return null_val();
        const uint64_t lim = f.precision <= 9 ? (neg ? 0x80000000ull : 0x7FFFFFFFull)
                                              : (neg ? 0x8000000000000000ull : 0x7FFFFFFFFFFFFFFFull);
        if (v > lim) return null_val();
        v = neg ? (uint64_t)0 - v : v;
        return Val{v, (uint64_t)((int64_t)v >> 63), true};
    }
    return null_val();
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

// UTF-16 (StringDecoders.decodeUtf16String, StringDecoders.scala:98-114): `new String(bytes,
// UTF_16BE|LE)` decodes with the JDK UnicodeDecoder under REPLACE -- U+FFFE and an unpaired low
// surrogate are malformed(2), a high surrogate followed by a non-low unit is malformed(4) (both
// units), a high surrogate or a lone byte at the end is malformed(rest); each malformed run is
// one U+FFFD.  One token at byte `pos` of p[0, n): returns its byte length, code point in cp.
template <typename BP>
CBX_HD int utf16_token(BP p, int pos, int n, bool be, uint32_t& cp) {
    const int r = n - pos;
    cp = 0xFFFDu;
    if (r < 2) return r;
    const uint32_t u = be ? (uint32_t)p[pos] << 8 | p[pos + 1] : (uint32_t)p[pos + 1] << 8 | p[pos];
    if (u >= 0xD800u && u <= 0xDBFFu) {
        if (r < 4) return r;
        const uint32_t u2 = be ? (uint32_t)p[pos + 2] << 8 | p[pos + 3] : (uint32_t)p[pos + 3] << 8 | p[pos + 2];
        if (u2 >= 0xDC00u && u2 <= 0xDFFFu) cp = 0x10000u + ((u - 0xD800u) << 10) + (u2 - 0xDC00u);
        return 4;
    }
    if (!(u == 0xFFFEu || (u >= 0xDC00u && u <= 0xDFFFu))) cp = u;
    return 2;
}
CBX_HD int utf8_width(uint32_t cp) { return cp < 0x80u ? 1 : cp < 0x800u ? 2 : cp < 0x10000u ? 3 : 4; }

// Trimmed span (token boundaries) + UTF-8 length of a UTF-16 field; trimming drops chars <= U+0020.
template <typename BP>
CBX_HD StrSpan utf16_span(int kind, int trim, BP p, int n) {
    const bool be = kind == CBX_K_UTF16_BE;
    int pos = 0, first = -1, last_end = 0, run = 0, u8_first = 0, u8_last = 0;
    while (pos < n) {
        uint32_t cp;
        const int len = utf16_token(p, pos, n, be, cp);
        const int w = utf8_width(cp);
        if (cp > 0x20u) {
            if (first < 0) { first = pos; u8_first = run; }
            last_end = pos + len;
            u8_last = run + w;
        }
        run += w;
        pos += len;
    }
    const bool tl = trim == CBX_TRIM_LEFT || trim == CBX_TRIM_BOTH;
    const bool tr = trim == CBX_TRIM_RIGHT || trim == CBX_TRIM_BOTH;
    StrSpan s;
    int u0 = 0, u1 = run;
    s.begin = 0;
    s.end = n;
    if (tl) { s.begin = first < 0 ? n : first; u0 = first < 0 ? run : u8_first; }
    if (tr) { s.end = first < 0 ? s.begin : last_end; u1 = first < 0 ? u0 : u8_last; }
    s.utf8_len = u1 - u0;
    return s;
}

template <typename BP, typename LutFn>
CBX_HD StrSpan string_span(int kind, int trim, BP p, int n, LutFn lut) {
    StrSpan s{0, n, 0};
    if (kind == CBX_K_HEX) { s.utf8_len = 2 * n; return s; }
    if (kind == CBX_K_RAW) { s.utf8_len = n; return s; }
    if (kind == CBX_K_UTF16_BE || kind == CBX_K_UTF16_LE) return utf16_span(kind, trim, p, n);
    const bool tl = trim == CBX_TRIM_LEFT || trim == CBX_TRIM_BOTH;
    const bool tr = trim == CBX_TRIM_RIGHT || trim == CBX_TRIM_BOTH;
    int b = 0, e = n;
    if (tl) while (b < e && (lut(p[b]) >> 31)) b++;
    if (tr) while (e > b && (lut(p[e - 1]) >> 31)) e--;
    int len = 0;
    for (int i = b; i < e; i++) len += (lut(p[i]) >> 24) & 3;
    s.begin = b; s.end = e; s.utf8_len = len;
    return s;
}

template <typename BP, typename LutFn>
CBX_HD void string_write(int kind, BP p, const StrSpan& s, uint8_t* out, LutFn lut) {
    if (kind == CBX_K_HEX) {
        const char* H = "0123456789ABCDEF";
        for (int i = s.begin; i < s.end; i++) {
            out[2 * (i - s.begin)] = (uint8_t)H[p[i] >> 4];
            out[2 * (i - s.begin) + 1] = (uint8_t)H[p[i] & 15];
        }
        return;
    }
    if (kind == CBX_K_RAW) {
        for (int i = s.begin; i < s.end; i++) out[i - s.begin] = p[i];
        return;
    }
    if (kind == CBX_K_UTF16_BE || kind == CBX_K_UTF16_LE) {
        // s.begin / s.end are token boundaries of the tokenisation over the whole field, so
        // re-tokenising [begin, end) yields the same tokens
        int k = 0;
        for (int pos = s.begin; pos < s.end;) {
            uint32_t cp;
            pos += utf16_token(p, pos, s.end, kind == CBX_K_UTF16_BE, cp);
            if (cp < 0x80u) {
                out[k++] = (uint8_t)cp;
            } else if (cp < 0x800u) {
                out[k++] = (uint8_t)(0xC0u | cp >> 6); out[k++] = (uint8_t)(0x80u | (cp & 63u));
            } else if (cp < 0x10000u) {
                out[k++] = (uint8_t)(0xE0u | cp >> 12); out[k++] = (uint8_t)(0x80u | ((cp >> 6) & 63u));
                out[k++] = (uint8_t)(0x80u | (cp & 63u));
            } else {
                out[k++] = (uint8_t)(0xF0u | cp >> 18); out[k++] = (uint8_t)(0x80u | ((cp >> 12) & 63u));
                out[k++] = (uint8_t)(0x80u | ((cp >> 6) & 63u)); out[k++] = (uint8_t)(0x80u | (cp & 63u));
            }
        }
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

// ------------------------------------------------------------------------------------------
// Strings of at most kStrFastBytes bytes: the element's bytes are read from the record image
// as dwords, each byte's LUT entry is looked up once, and trimming / UTF-8 length become bit
// operations over per-byte masks (ctz / clz / popcount) -- no data-dependent loops.
// ------------------------------------------------------------------------------------------
constexpr int kStrFastBytes = 32;

// bytes img[addr, addr + size) as 8 little-endian dwords (size <= 32; reads up to 36 bytes)
CBX_HD void img_bytes32(const uint8_t* img, uint32_t addr, int size, uint32_t w[8]) {
    const uint32_t* p = (const uint32_t*)(img + (addr & ~3u));
    const uint32_t sh = addr & 3u;
    uint32_t r[9];
#pragma unroll
    for (int k = 0; k < 9; k++) r[k] = 4 * k < size + 3 ? p[k] : 0u;
#pragma unroll
    for (int k = 0; k < 8; k++) w[k] = align_bytes(r[k + 1], r[k], sh);
}

CBX_HD uint32_t ctz32(uint32_t x) { return (uint32_t)__builtin_ctz(x); }
CBX_HD uint32_t clz32(uint32_t x) { return (uint32_t)__builtin_clz(x); }
CBX_HD uint32_t popc32(uint32_t x) { return (uint32_t)__builtin_popcount(x); }
CBX_HD uint32_t bits_below(int k) { return k >= 32 ? 0xFFFFFFFFu : ((1u << k) - 1u); }

// LUT entries of the size (<= 32) bytes held in w (one LDS lookup per byte, shared by the span
// and the write).
template <typename LutFn>
CBX_HD void lut_entries32(const uint32_t w[8], int size, LutFn lut, uint32_t ev[kStrFastBytes]) {
#pragma unroll
    for (int j = 0; j < kStrFastBytes; j++) ev[j] = j < size ? lut((w[j >> 2] >> (8 * (j & 3))) & 0xFFu) : 0u;
}

// Trimmed span + UTF-8 length (StringDecoders.decodeEbcdicString / decodeAsciiString +
// StringTools.trim*) of the first n (<= size <= 32) bytes, from their LUT entries.
CBX_HD StrSpan string_span32e(int trim, const uint32_t ev[kStrFastBytes], int n, int size) {
    uint32_t keep = 0, m2 = 0, m3 = 0;   // bit j: byte j not trimmable / 2-byte / 3-byte UTF-8
#pragma unroll
    for (int j = 0; j < kStrFastBytes; j++) {
        if (j < size) {
            const uint32_t e = ev[j];
            const uint32_t l = (e >> 24) & 3u;
            const uint32_t bit = 1u << j;
            keep |= (e >> 31) ? 0u : bit;
            m2 |= l == 2 ? bit : 0u;
            m3 |= l == 3 ? bit : 0u;
        }
    }
    keep &= bits_below(n);
    const bool tl = trim == CBX_TRIM_LEFT || trim == CBX_TRIM_BOTH;
    const bool tr = trim == CBX_TRIM_RIGHT || trim == CBX_TRIM_BOTH;
    int b = 0, e = n;
    if (tl) b = keep ? (int)ctz32(keep) : n;
    if (tr) e = keep ? 32 - (int)clz32(keep) : b;
    const uint32_t range = bits_below(e) & ~bits_below(b);
    StrSpan s;
    s.begin = b;
    s.end = e;
    s.utf8_len = (e - b) + (int)popc32(m2 & range) + 2 * (int)popc32(m3 & range);
    return s;
}

template <typename LutFn>
CBX_HD StrSpan string_span32(int trim, const uint32_t w[8], int n, int size, LutFn lut) {
    uint32_t ev[kStrFastBytes];
    lut_entries32(w, size, lut, ev);
    return string_span32e(trim, ev, n, size);
}

// UTF-8 bytes of the span into out[0, utf8_len); writes of bytes outside the span (and of the
// unused 2nd / 3rd bytes of a character) go to `dump` instead of branching per lane.
// width: the code page's widest UTF-8 encoding (1..3) -- only that many stores per byte.  `dump`
// should be private to the lane (a shared dump address serialises the wave's LDS stores).
CBX_HD void string_write32e(const uint32_t ev[kStrFastBytes], const StrSpan& s, uint8_t* out, uint8_t* dump, int size,
                            int width) {
    int k = 0;
#pragma unroll
    for (int j = 0; j < kStrFastBytes; j++) {
        if (j < size) {
            const bool in = j >= s.begin && j < s.end;
            const uint32_t e = ev[j];
            *(in ? out + k : dump) = (uint8_t)e;
            if (width > 1) {
                const uint32_t l = (e >> 24) & 3u;
                *(in && l > 1 ? out + k + 1 : dump) = (uint8_t)(e >> 8);
                if (width > 2) *(in && l > 2 ? out + k + 2 : dump) = (uint8_t)(e >> 16);
                k += in ? (int)l : 0;
            } else {
                k += in ? 1 : 0;
            }
        }
    }
}

template <typename LutFn>
CBX_HD void string_write32(const uint32_t w[8], const StrSpan& s, uint8_t* out, uint8_t* dump, int size,
                           int width, LutFn lut) {
    uint32_t ev[kStrFastBytes];
    lut_entries32(w, size, lut, ev);
    string_write32e(ev, s, out, dump, size, width);
}

}  // namespace cbx

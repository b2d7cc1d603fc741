/*
 * cobrix_oracle.c -- TEST INFRASTRUCTURE ONLY (see cobrix_oracle.h).
 *
 * A deliberately literal CPU restatement of the reference's string-based decoders: values are
 * built as the JVM builds them (character buffers -> BigDecimal/Integer parsing) so that every
 * null/edge rule comes out the same way.  It is the checker for the HIP kernels, never the
 * product.  Citations: CP = /root/reference/cobol-parser/src/main/scala/za/co/absa/cobrix/cobol/
 */
#include "cobrix_oracle.h"

#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef __int128 i128;

/* ------------------------------------------------------------------------------------------ */
/* Java-level values                                                                          */
/* ------------------------------------------------------------------------------------------ */
enum { JNULL = 0, JINT, JLONG, JBIGDEC, JFLOAT, JDOUBLE, JSTRING, JBYTES };

#define MAXS 512

typedef struct {
    int type;
    int32_t i;
    int64_t l;
    /* BigDecimal: sign, digit string (no leading zeros except "0"), scale */
    int neg;
    char digits[MAXS];
    int scale;
    uint32_t fbits;
    uint64_t dbits;
    uint16_t str[MAXS];  /* UTF-16 code units */
    int slen;
    uint8_t bytes[MAXS];
    int blen;
} jvalue;

/* Java BigDecimal(String) (exponent-free subset, which is all the decoders produce).
 * Returns 1 on success. */
static int parse_bigdecimal(const char* s, jvalue* v) {
    int i = 0, n = (int)strlen(s);
    v->neg = 0;
    if (i < n && (s[i] == '+' || s[i] == '-')) { v->neg = (s[i] == '-'); i++; }
    int nd = 0, dot = -1, scale = 0;
    char buf[MAXS];
    for (; i < n; i++) {
        char c = s[i];
        if (c >= '0' && c <= '9') {
            if (nd < MAXS - 1) buf[nd++] = c; else return 0;
            if (dot >= 0) scale++;
        } else if (c == '.') {
            if (dot >= 0) return 0;
            dot = i;
        } else if (c == 'e' || c == 'E') {
            /* java.math.BigDecimal(String) exponent: [eE][+-]?digits, scale -= exponent; an
             * exponent past 10 digits (or a scale outside int) -> NumberFormatException */
            i++;
            int eneg = 0;
            if (i < n && (s[i] == '+' || s[i] == '-')) { eneg = s[i] == '-'; i++; }
            if (i >= n) return 0;
            long long ex = 0;
            int ed = 0;
            for (; i < n; i++) {
                if (s[i] < '0' || s[i] > '9') return 0;
                ex = ex * 10 + (s[i] - '0');
                if (ex > 0 || s[i] != '0') ed++;
                if (ed > 10) return 0;
            }
            long long sc = (long long)scale - (eneg ? -ex : ex);
            if (sc > 2147483647LL || sc < -2147483648LL) return 0;
            scale = (int)sc;
            break;
        } else {
            return 0;
        }
    }
    if (nd == 0) return 0;
    buf[nd] = 0;
    int k = 0;
    while (k < nd - 1 && buf[k] == '0') k++;
    memmove(v->digits, buf + k, (size_t)(nd - k + 1));
    v->scale = scale;
    v->type = JBIGDEC;
    if (strcmp(v->digits, "0") == 0) v->neg = 0;
    return 1;
}

/* java.lang.Integer.parseInt / Long.parseLong (radix 10) */
static int parse_java_long(const char* s, int64_t lo_lim_neg_abs_hi, int64_t* out, int is_int) {
    (void)lo_lim_neg_abs_hi;
    int n = (int)strlen(s), i = 0, neg = 0;
    if (n == 0) return 0;
    if (s[0] == '-' || s[0] == '+') { neg = s[0] == '-'; i = 1; if (n == 1) return 0; }
    u128 acc = 0;
    for (; i < n; i++) {
        if (s[i] < '0' || s[i] > '9') return 0;
        acc = acc * 10 + (u128)(s[i] - '0');
        if (acc > ((u128)1 << 64)) return 0;
    }
    u128 lim = is_int ? ((u128)1 << 31) : ((u128)1 << 63);
    if (neg) { if (acc > lim) return 0; *out = (int64_t)(-(i128)acc); }
    else { if (acc > lim - 1) return 0; *out = (int64_t)acc; }
    return 1;
}

/* ------------------------------------------------------------------------------------------ */
/* String decoders  (CP/parser/decoders/StringDecoders.scala, StringTools.scala)              */
/* ------------------------------------------------------------------------------------------ */

/* String.trim / StringTools.trimLeft / trimRight over UTF-16 units (char <= ' ') */
static void apply_trim(uint16_t* s, int* len, int trimming) {
    int st = 0, e = *len;
    if (trimming == ORA_TRIM_LEFT || trimming == ORA_TRIM_BOTH)
        while (st < e && s[st] <= 0x20) st++;
    if (trimming == ORA_TRIM_RIGHT || trimming == ORA_TRIM_BOTH)
        while (st < e && s[e - 1] <= 0x20) e--;
    if (st > 0) memmove(s, s + st, (size_t)(e - st) * 2);
    *len = e - st;
}

/* StringDecoders.decodeEbcdicString (StringDecoders.scala:44-61) */
static void decode_ebcdic_string(const uint8_t* b, int n, int trimming, const uint16_t* lut, jvalue* v) {
    v->type = JSTRING;
    v->slen = 0;
    for (int i = 0; i < n && i < MAXS; i++) v->str[v->slen++] = lut[b[i]];
    apply_trim(v->str, &v->slen, trimming);
}

/* StringDecoders.decodeAsciiString (StringDecoders.scala:70-89): Java bytes are signed */
static void decode_ascii_string(const uint8_t* b, int n, int trimming, jvalue* v) {
    v->type = JSTRING;
    v->slen = 0;
    for (int i = 0; i < n && i < MAXS; i++) {
        int8_t sb = (int8_t)b[i];
        v->str[v->slen++] = sb < 32 ? 0x20 : (uint16_t)sb;
    }
    apply_trim(v->str, &v->slen, trimming);
}

/* StringDecoders.decodeUtf16String (StringDecoders.scala:98-114): `new String(bytes, UTF_16BE/LE)`
 * with the JDK 8 sun.nio.cs.UnicodeDecoder.decodeLoop under CodingErrorAction.REPLACE (what
 * String(byte[], Charset) uses): U+FFFE, an unpaired low surrogate -> malformed(2); a high
 * surrogate not followed by a low one -> malformed(4) (both units); a high surrogate or an odd
 * byte at the end -> underflow, then malformed(remaining) at end of input.  Every malformed run
 * becomes ONE U+FFFD.  Then String.trim / StringTools.trimLeft / trimRight. */
static void decode_utf16_string(const uint8_t* b, int n, int trimming, int big_endian, jvalue* v) {
    v->type = JSTRING;
    v->slen = 0;
    int pos = 0;
    while (pos < n && v->slen < MAXS - 2) {
        int mark = pos;
        int malformed = 0;
        if (n - pos < 2) {
            malformed = n - pos;                                 /* end of input, odd byte */
        } else {
            uint16_t c = big_endian ? (uint16_t)(b[pos] << 8 | b[pos + 1]) : (uint16_t)(b[pos + 1] << 8 | b[pos]);
            pos += 2;
            if (c == 0xFFFE) malformed = 2;
            else if (c >= 0xD800 && c <= 0xDBFF) {
                if (n - pos < 2) malformed = n - mark;           /* UNDERFLOW -> malformed(remaining) */
                else {
                    uint16_t c2 = big_endian ? (uint16_t)(b[pos] << 8 | b[pos + 1]) : (uint16_t)(b[pos + 1] << 8 | b[pos]);
                    pos += 2;
                    if (c2 >= 0xDC00 && c2 <= 0xDFFF) { v->str[v->slen++] = c; v->str[v->slen++] = c2; continue; }
                    malformed = 4;
                }
            } else if (c >= 0xDC00 && c <= 0xDFFF) malformed = 2;
            else { v->str[v->slen++] = c; continue; }
        }
        v->str[v->slen++] = 0xFFFD;
        pos = mark + malformed;
    }
    apply_trim(v->str, &v->slen, trimming);
}

/* AsciiStringDecoderWrapper.apply (AsciiStringDecoderWrapper.scala:43-67): bytes 0..31 -> 32,
 * then `new String(buf, charset)` for a single-byte charset (table from the harness), then trim */
static void decode_charset_string(const uint8_t* b, int n, int trimming, const uint16_t* table, jvalue* v) {
    v->type = JSTRING;
    v->slen = 0;
    for (int i = 0; i < n && i < MAXS; i++) v->str[v->slen++] = table[b[i] < 32 ? 32 : b[i]];
    apply_trim(v->str, &v->slen, trimming);
}

/* StringDecoders.decodeHex (StringDecoders.scala:122-132) */
static void decode_hex(const uint8_t* b, int n, jvalue* v) {
    static const char* H = "0123456789ABCDEF";
    v->type = JSTRING;
    v->slen = 0;
    for (int i = 0; i < n && 2 * i + 1 < MAXS; i++) {
        v->str[v->slen++] = (uint16_t)H[b[i] >> 4];
        v->str[v->slen++] = (uint16_t)H[b[i] & 15];
    }
}

/* StringDecoders.decodeEbcdicNumber (StringDecoders.scala:154-212). Returns 0 for null. */
static int decode_ebcdic_number(const uint8_t* b, int n, int is_unsigned, char* out) {
    char buf[MAXS];
    int bl = 0;
    char sign = ' ';
    int malformed = 0;
    for (int i = 0; i < n; i++) {
        int c = b[i];
        char ch = ' ';
        if (sign != ' ') {
            if (c >= 0xF0 && c <= 0xF9) ch = (char)(c - 0xF0 + '0');
            else if (c == 0x4B || c == 0x6B) ch = '.';
            else if (c == 0x40 || c == 0) ch = ' ';
            else malformed = 1;
        } else if (c >= 0xF0 && c <= 0xF9) {
            ch = (char)(c - 0xF0 + '0');
        } else if (c >= 0xC0 && c <= 0xC9) {
            ch = (char)(c - 0xC0 + '0'); sign = '+';
        } else if (c >= 0xD0 && c <= 0xD9) {
            ch = (char)(c - 0xD0 + '0'); sign = '-';
        } else if (c == 0x60) {
            sign = '-';
        } else if (c == 0x4E) {
            sign = '+';
        } else if (c == 0x4B || c == 0x6B) {
            ch = '.';
        } else if (c == 0x40 || c == 0) {
            ch = ' ';
        } else {
            malformed = 1;
        }
        if (ch != ' ' && bl < MAXS - 2) buf[bl++] = ch;
    }
    buf[bl] = 0;
    if (malformed) return 0;
    if (sign != ' ') {
        if (sign == '-' && is_unsigned) return 0;
        out[0] = sign;
        memcpy(out + 1, buf, (size_t)bl + 1);  /* buf.toString.trim: buf holds no spaces */
        return 1;
    }
    memcpy(out, buf, (size_t)bl + 1);
    return 1;
}

/* StringDecoders.decodeAsciiNumber (StringDecoders.scala:221-243) */
static void java_trim_ascii(char* s) {
    int n = (int)strlen(s), st = 0, e = n;
    while (st < e && (unsigned char)s[st] <= 0x20) st++;
    while (st < e && (unsigned char)s[e - 1] <= 0x20) e--;
    memmove(s, s + st, (size_t)(e - st));
    s[e - st] = 0;
}

static int decode_ascii_number(const uint8_t* b, int n, int is_unsigned, char* out) {
    char buf[MAXS];
    int bl = 0;
    char sign = ' ';
    for (int i = 0; i < n && bl < MAXS - 2; i++) {
        /* bytes(i).toChar on a signed byte: values >= 0x80 become U+FF80..U+FFFF, which are
         * neither digits nor '.' nor trimmed, so any such byte makes the later parse fail;
         * stand it in with '#' (same properties) */
        int8_t sb = (int8_t)b[i];
        char c = sb < 0 ? '#' : (char)sb;
        /* U+0000 is an ordinary (trimmable) Java char; stand it in with U+0001 (same
         * properties) so that it does not end the C string */
        if (c == 0) c = 1;
        if (c == '-' || c == '+') sign = c;
        else if (c == '.' || c == ',') buf[bl++] = '.';
        else buf[bl++] = c;
    }
    buf[bl] = 0;
    java_trim_ascii(buf);
    if (sign != ' ') {
        if (sign == '-' && is_unsigned) return 0;
        out[0] = sign;
        strcpy(out + 1, buf);
        return 1;
    }
    strcpy(out, buf);
    return 1;
}

/* BinaryUtils.addDecimalPoint (BinaryUtils.scala:194-238) */
static void add_decimal_point(const char* iv, int scale, int sf, char* out) {
    int len = (int)strlen(iv);
    int is_neg = len > 0 && iv[0] == '-';
    if (sf == 0) {
        if (scale == 0) { strcpy(out, iv); return; }
        if (is_neg) {
            if (len - 1 > scale) {
                int k = len - scale;
                memcpy(out, iv, (size_t)k); out[k] = '.'; strcpy(out + k + 1, iv + k);
            } else {
                int p = 0;
                out[p++] = '-'; out[p++] = '0'; out[p++] = '.';
                for (int z = 0; z < scale - len + 1; z++) out[p++] = '0';
                strcpy(out + p, iv + 1);
            }
        } else {
            if (len > scale) {
                int k = len - scale;
                memcpy(out, iv, (size_t)k); out[k] = '.'; strcpy(out + k + 1, iv + k);
            } else {
                int p = 0;
                out[p++] = '0'; out[p++] = '.';
                for (int z = 0; z < scale - len; z++) out[p++] = '0';
                strcpy(out + p, iv);
            }
        }
    } else if (sf < 0) {
        int p = 0;
        if (is_neg) out[p++] = '-';
        out[p++] = '0'; out[p++] = '.';
        for (int z = 0; z < -sf; z++) out[p++] = '0';
        const char* ns = (len > 0 && (iv[0] == '-' || iv[0] == '+')) ? iv + 1 : iv;
        strcpy(out + p, ns);
    } else {
        int p = len;
        strcpy(out, iv);
        for (int z = 0; z < sf; z++) out[p++] = '0';
        out[p] = 0;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* BCD (CP/parser/decoders/BCDNumberDecoders.scala)                                           */
/* ------------------------------------------------------------------------------------------ */

/* decodeBCDIntegralNumber (:29-73): Java long arithmetic wraps */
static int decode_bcd_integral(const uint8_t* b, int n, int64_t* out) {
    if (n < 1) return 0;
    int64_t sign = 1;
    uint64_t acc = 0;
    for (int i = 0; i < n; i++) {
        int lo = b[i] & 15, hi = (b[i] >> 4) & 15;
        if (hi < 10) acc = acc * 10 + (uint64_t)hi; else return 0;
        if (i + 1 == n) {
            if (lo == 0x0C || lo == 0x0F) sign = 1;
            else if (lo == 0x0D) sign = -1;
            else return 0;
        } else {
            if (lo < 10) acc = acc * 10 + (uint64_t)lo; else return 0;
        }
    }
    *out = (int64_t)((uint64_t)sign * acc);
    return 1;
}

/* decodeBigBCDNumber (:83-160) */
static int decode_big_bcd_number(const uint8_t* b, int n, int scale, int sf, char* out) {
    if (n < 1) return 0;
    const char* sign = "";
    int intended = n * 2 - (scale + 1);
    int additional = intended <= 0 ? -intended + 1 : 0;
    char chars[MAXS];
    int cl = 0;
    int dpp = n * 2 - (scale + 1) + additional;
    for (int i = 0; i < additional; i++) chars[cl++] = '0';
    for (int i = 0; i < n; i++) {
        int lo = b[i] & 15, hi = (b[i] >> 4) & 15;
        if (hi < 10) chars[cl++] = (char)('0' + hi); else return 0;
        if (i + 1 == n) {
            if (lo == 0x0C || lo == 0x0F) sign = "";
            else if (lo == 0x0D) sign = "-";
            else return 0;
        } else {
            if (lo < 10) chars[cl++] = (char)('0' + lo); else return 0;
        }
    }
    chars[cl] = 0;
    if (sf == 0) {
        char tmp[MAXS];
        if (scale > 0) {
            memcpy(tmp, chars, (size_t)dpp); tmp[dpp] = '.'; strcpy(tmp + dpp + 1, chars + dpp);
        } else {
            strcpy(tmp, chars);
        }
        strcpy(out, sign);
        strcat(out, tmp);
    } else if (sf < 0) {
        int p = 0;
        strcpy(out, sign); p = (int)strlen(out);
        out[p++] = '0'; out[p++] = '.';
        for (int z = 0; z < -sf; z++) out[p++] = '0';
        strcpy(out + p, chars);
    } else {
        strcpy(out, sign);
        strcat(out, chars);
        int p = (int)strlen(out);
        for (int z = 0; z < sf; z++) out[p++] = '0';
        out[p] = 0;
    }
    return 1;
}

/* ------------------------------------------------------------------------------------------ */
/* Binary (CP/parser/decoders/BinaryNumberDecoders.scala, BinaryUtils.decodeBinaryNumber)     */
/* ------------------------------------------------------------------------------------------ */

static void u128_to_str(u128 v, char* out) {
    char t[64];
    int k = 0;
    if (v == 0) t[k++] = '0';
    while (v) { t[k++] = (char)('0' + (int)(v % 10)); v /= 10; }
    for (int i = 0; i < k; i++) out[i] = t[k - 1 - i];
    out[k] = 0;
}

/* BigInt(bytes) / BigInt(1, bytes) -> decimal string; arbitrary width up to 32 bytes */
static void bigint_to_str(const uint8_t* be, int n, int is_signed, char* out) {
    /* base-256 big-endian magnitude -> decimal via repeated division */
    uint8_t mag[64];
    int neg = is_signed && n > 0 && (be[0] & 0x80);
    memcpy(mag, be, (size_t)n);
    if (neg) { /* two's complement negate */
        int carry = 1;
        for (int i = n - 1; i >= 0; i--) {
            int x = (uint8_t)(~mag[i]) + carry;
            mag[i] = (uint8_t)x; carry = x >> 8;
        }
    }
    char digs[200];
    int nd = 0;
    int allzero = 1;
    for (int i = 0; i < n; i++) if (mag[i]) { allzero = 0; break; }
    if (allzero) { strcpy(out, "0"); return; }
    while (1) {
        int rem = 0, nz = 0;
        for (int i = 0; i < n; i++) {
            int cur = rem * 256 + mag[i];
            mag[i] = (uint8_t)(cur / 10); rem = cur % 10;
            if (mag[i]) nz = 1;
        }
        digs[nd++] = (char)('0' + rem);
        if (!nz) break;
    }
    int p = 0;
    if (neg) out[p++] = '-';
    for (int i = nd - 1; i >= 0; i--) out[p++] = digs[i];
    out[p] = 0;
}

/* BinaryUtils.decodeBinaryNumber (:245-276) -> string then addDecimalPoint */
static void decode_binary_number_str(const uint8_t* b, int n, int big_endian, int is_signed,
                                     int scale, int sf, char* out) {
    char iv[MAXS];
    if (n == 0) { strcpy(out, "0"); return; }
    uint8_t be[64];
    for (int i = 0; i < n; i++) be[i] = big_endian ? b[i] : b[n - 1 - i];
    if (is_signed && (n == 1 || n == 2 || n == 4 || n == 8)) {
        int64_t v = (be[0] & 0x80) ? -1 : 0;
        for (int i = 0; i < n; i++) v = (int64_t)(((uint64_t)v << 8) | be[i]);
        if (v < 0) { iv[0] = '-'; u128_to_str((u128)(-(i128)v), iv + 1); }
        else u128_to_str((u128)v, iv);
    } else if (!is_signed && (n == 1 || n == 2 || n == 4)) {
        uint64_t v = 0;
        for (int i = 0; i < n; i++) v = (v << 8) | be[i];
        u128_to_str((u128)v, iv);
    } else {
        bigint_to_str(be, n, is_signed, iv);
    }
    add_decimal_point(iv, scale, sf, out);
}

/* ------------------------------------------------------------------------------------------ */
/* Floating point (CP/parser/decoders/FloatingPointDecoders.scala)                            */
/* ------------------------------------------------------------------------------------------ */

/* decodeIbmSingleBigEndian (:75-114), including the reference's exponent-mask behaviour */
static uint32_t ibm_single(const uint8_t* b) {
    int32_t mant = (int32_t)(((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3]);
    int32_t sign = mant & (int32_t)0x80000000;
    int32_t frac = mant & 0x00FFFFFF;
    int32_t expo = (mant & (int32_t)0x80000000) >> 22;  /* arithmetic shift as in the JVM */
    if (frac == 0) return 0u;
    int32_t top = frac & 0x00F00000;
    while (top == 0) { frac <<= 4; expo -= 4; top = frac & 0x00F00000; }
    int32_t lz = (int32_t)((0x000055AFL >> (top >> 19)) & 3);
    frac <<= lz;
    int32_t ce = expo + 131 - lz;
    if (ce >= 0 && ce < 254) {
        return (uint32_t)sign + ((uint32_t)ce << 23) + (uint32_t)frac;
    } else if (ce > 254) {
        return 0x7F800000u;
    } else if (ce >= -32) {
        int32_t mask = ~(int32_t)(0xFFFFFFFDu << (-1 - ce));
        int32_t ru = (frac & mask) > 0 ? 1 : 0;
        int32_t cf = ((frac >> (-1 - ce)) + ru) >> 1;
        return (uint32_t)sign + (uint32_t)cf;
    }
    return 0u;
}

/* decodeIbmDoubleBigEndian (:127-170) */
static uint64_t ibm_double(const uint8_t* b) {
    uint64_t m = 0;
    for (int i = 0; i < 8; i++) m = (m << 8) | b[i];
    uint64_t sign = m & 0x8000000000000000ULL;
    int64_t frac = (int64_t)(m & 0x00FFFFFFFFFFFFFFULL);
    int64_t expo = (int64_t)((m & 0x7F00000000000000ULL) >> 54);
    if (frac == 0) return 0ull;
    int64_t top = frac & 0x00F0000000000000LL;
    while (top == 0) { frac <<= 4; expo -= 4; top = frac & 0x00F0000000000000LL; }
    int64_t lz = (0x000055AFLL >> (top >> 51)) & 3;
    frac <<= lz;
    int64_t ce = expo + 765 - lz;
    int64_t ru = (frac & 0xb) > 0 ? 1 : 0;
    int64_t cf = ((frac >> 2) + ru) >> 1;
    return sign + ((uint64_t)ce << 52) + (uint64_t)cf;
}

/* ------------------------------------------------------------------------------------------ */
/* Decoder selection (CP/parser/decoders/DecoderSelector.scala:54-290)                        */
/* ------------------------------------------------------------------------------------------ */

static void set_bigdec_or_null(const char* s, jvalue* v) {
    if (!parse_bigdecimal(s, v)) v->type = JNULL;
}

static void decode_value(const ora_node* nd, const ora_options* opt, const uint8_t* b, int n, jvalue* v) {
    char s[MAXS * 2], t[MAXS * 2];
    v->type = JNULL;
    int is_unsigned = !nd->is_signed;
    if (nd->tclass == ORA_ALPHA) {
        switch (nd->enc) {
        case ORA_EBCDIC: decode_ebcdic_string(b, n, opt->trimming, opt->lut, v); return;
        case ORA_ASCII:
            if (opt->ascii_lut) decode_charset_string(b, n, opt->trimming, opt->ascii_lut, v);
            else decode_ascii_string(b, n, opt->trimming, v);
            return;
        case ORA_HEX: decode_hex(b, n, v); return;
        case ORA_RAW: v->type = JBYTES; v->blen = n < MAXS ? n : MAXS; memcpy(v->bytes, b, (size_t)v->blen); return;
        case ORA_UTF16: decode_utf16_string(b, n, opt->trimming, opt->utf16_big_endian, v); return;
        default: v->type = JNULL; return;
        }
    }
    int ebc = nd->enc == ORA_EBCDIC;
    if (nd->tclass == ORA_DECIMAL) {
        switch (nd->compact) {
        case ORA_DISPLAY: {
            int ok = ebc ? decode_ebcdic_number(b, n, is_unsigned, s) : decode_ascii_number(b, n, is_unsigned, s);
            if (!ok) return;
            if (nd->explicit_decimal) { set_bigdec_or_null(s, v); return; }
            add_decimal_point(s, nd->scale, nd->scale_factor, t);
            set_bigdec_or_null(t, v);
            return;
        }
        case ORA_COMP1: {
            if (n < 4) return;
            uint8_t r[4];
            int le = opt->float_format == ORA_FP_IBM_LE || opt->float_format == ORA_FP_IEEE_LE;
            for (int i = 0; i < 4; i++) r[i] = le ? b[3 - i] : b[i];
            v->type = JFLOAT;
            if (opt->float_format == ORA_FP_IBM || opt->float_format == ORA_FP_IBM_LE) v->fbits = ibm_single(r);
            else v->fbits = ((uint32_t)r[0] << 24) | ((uint32_t)r[1] << 16) | ((uint32_t)r[2] << 8) | r[3];
            return;
        }
        case ORA_COMP2: {
            if (n < 8) return;
            uint8_t r[8];
            int le = opt->float_format == ORA_FP_IBM_LE || opt->float_format == ORA_FP_IEEE_LE;
            for (int i = 0; i < 8; i++) r[i] = le ? b[7 - i] : b[i];
            v->type = JDOUBLE;
            if (opt->float_format == ORA_FP_IBM || opt->float_format == ORA_FP_IBM_LE) v->dbits = ibm_double(r);
            else { uint64_t m = 0; for (int i = 0; i < 8; i++) m = (m << 8) | r[i]; v->dbits = m; }
            return;
        }
        case ORA_COMP3:
            if (!decode_big_bcd_number(b, n, nd->scale, nd->scale_factor, s)) return;
            set_bigdec_or_null(s, v);
            return;
        case ORA_COMP4: case ORA_COMP5: case ORA_COMP9:
            decode_binary_number_str(b, n, nd->compact != ORA_COMP9, nd->is_signed, nd->scale, nd->scale_factor, s);
            set_bigdec_or_null(s, v);
            return;
        }
        return;
    }
    /* Integral */
    switch (nd->compact) {
    case ORA_DISPLAY: {
        int ok = ebc ? decode_ebcdic_number(b, n, is_unsigned, s) : decode_ascii_number(b, n, is_unsigned, s);
        if (nd->precision <= 9) {
            int64_t x;
            if (ok && parse_java_long(s, 0, &x, 1)) { v->type = JINT; v->i = (int32_t)x; }
        } else if (nd->precision <= 18) {
            int64_t x;
            if (ok && parse_java_long(s, 0, &x, 0)) { v->type = JLONG; v->l = x; }
        } else {
            if (!ok) return;
            add_decimal_point(s, 0, 0, t);
            set_bigdec_or_null(t, v);
        }
        return;
    }
    case ORA_COMP3: {
        if (nd->precision <= 18) {
            int64_t x;
            if (!decode_bcd_integral(b, n, &x)) return;
            if (nd->precision <= 9) { v->type = JINT; v->i = (int32_t)x; }
            else { v->type = JLONG; v->l = x; }
        } else {
            if (!decode_big_bcd_number(b, n, 0, 0, s)) return;
            set_bigdec_or_null(s, v);
        }
        return;
    }
    case ORA_COMP4: case ORA_COMP5: case ORA_COMP9: {
        /* getBinaryEncodedIntegralDecoder (DecoderSelector.scala:230-256) */
        int be = nd->compact != ORA_COMP9;
        int nb = n;  /* == getBytesCount for the field */
        uint8_t r[64];
        if (nb > 64) return;
        for (int i = 0; i < nb; i++) r[i] = be ? b[i] : b[nb - 1 - i];
        if (nb == 1 || nb == 2 || nb == 4) {
            if (nd->is_signed) {
                int32_t x = (r[0] & 0x80) ? -1 : 0;
                for (int i = 0; i < nb; i++) x = (int32_t)(((uint32_t)x << 8) | r[i]);
                v->type = JINT; v->i = x;
            } else {
                uint32_t x = 0;
                for (int i = 0; i < nb; i++) x = (x << 8) | r[i];
                if (nb == 4 && (int32_t)x < 0) return;
                v->type = JINT; v->i = (int32_t)x;
            }
            if (nd->precision > 9) { v->type = JLONG; v->l = v->i; } /* not reachable by size rules */
        } else if (nb == 8) {
            uint64_t x = 0;
            for (int i = 0; i < 8; i++) x = (x << 8) | r[i];
            if (!nd->is_signed && (int64_t)x < 0) return;
            v->type = JLONG; v->l = (int64_t)x;
        } else {
            /* decodeBinaryAribtraryPrecision (BinaryNumberDecoders.scala:123-135) */
            bigint_to_str(r, nb, nd->is_signed, s);
            set_bigdec_or_null(s, v);
        }
        return;
    }
    }
}

/* ------------------------------------------------------------------------------------------ */
/* Spark conversion (SC/schema/CobolSchema.scala:144-173 + Catalyst Decimal.toPrecision)      */
/* ------------------------------------------------------------------------------------------ */

int32_t ora_spark_type(const ora_node* nd, int32_t* precision, int32_t* scale) {
    *precision = 0; *scale = 0;
    if (nd->tclass == ORA_ALPHA) return nd->enc == ORA_RAW ? ORA_ST_BINARY : ORA_ST_STRING;
    if (nd->tclass == ORA_DECIMAL) {
        if (nd->compact == ORA_COMP1) return ORA_ST_FLOAT;
        if (nd->compact == ORA_COMP2) return ORA_ST_DOUBLE;
        int sf = nd->scale_factor;
        int ep = nd->precision + (sf < 0 ? -sf : sf);
        *precision = ep;
        *scale = sf > 0 ? 0 : (sf < 0 ? ep : nd->scale);
        return ORA_ST_DECIMAL;
    }
    if (nd->precision > 18) { *precision = nd->precision; *scale = 0; return ORA_ST_DECIMAL; }
    if (nd->precision > 9) return ORA_ST_LONG;
    return ORA_ST_INT;
}

/* BigDecimal.setScale(S, HALF_UP) then precision check (null when precision > P) */
static int to_precision(const jvalue* v, int P, int S, i128* out) {
    char d[MAXS * 2];
    int nd = (int)strlen(v->digits);
    int sc = v->scale;
    strcpy(d, v->digits);
    if (strcmp(d, "0") == 0) { *out = 0; return 1; }   /* zero at any scale */
    if ((long long)S - sc > 40) return 0;              /* >= 10^41 unscaled: needs > 38 digits */
    if ((long long)sc - S > nd + 1) { *out = 0; return 1; }  /* every digit dropped, first dropped is 0 */
    if (S >= sc) {
        for (int z = 0; z < S - sc; z++) d[nd++] = '0';
        d[nd] = 0;
    } else {
        int drop = sc - S;
        int keep = nd - drop;
        int round_up = 0;
        if (keep >= 0) round_up = d[keep] >= '5';
        else round_up = 0;  /* all kept digits dropped with at least one leading zero: < 0.5 */
        if (keep <= 0) { d[0] = '0'; nd = 1; d[1] = 0; if (round_up) { d[0] = '1'; } }
        else {
            nd = keep; d[nd] = 0;
            if (round_up) {
                int i = nd - 1;
                while (i >= 0 && d[i] == '9') { d[i] = '0'; i--; }
                if (i >= 0) d[i]++;
                else { memmove(d + 1, d, (size_t)nd + 1); d[0] = '1'; nd++; }
            }
        }
    }
    int k = 0;
    while (k < nd - 1 && d[k] == '0') k++;
    int prec = nd - k;
    if (prec > P) return 0;
    u128 acc = 0;
    for (int i = k; i < nd; i++) acc = acc * 10 + (u128)(d[i] - '0');
    *out = v->neg ? -(i128)acc : (i128)acc;
    return 1;
}

static int put_heap(uint8_t* heap, int64_t cap, int64_t* len, const uint8_t* src, int n, int64_t* off) {
    if (*len + n > cap) return 0;
    memcpy(heap + *len, src, (size_t)n);
    *off = *len;
    *len += n;
    return 1;
}

static int utf16_to_utf8(const uint16_t* s, int n, uint8_t* o) {
    int k = 0;
    for (int i = 0; i < n; i++) {
        uint32_t c = s[i];
        if (c >= 0xD800 && c <= 0xDBFF && i + 1 < n && s[i + 1] >= 0xDC00 && s[i + 1] <= 0xDFFF) {
            c = 0x10000 + ((c - 0xD800) << 10) + (s[i + 1] - 0xDC00u);
            i++;
            o[k++] = (uint8_t)(0xF0 | (c >> 18)); o[k++] = (uint8_t)(0x80 | ((c >> 12) & 63));
            o[k++] = (uint8_t)(0x80 | ((c >> 6) & 63)); o[k++] = (uint8_t)(0x80 | (c & 63));
            continue;
        }
        if (c < 0x80) o[k++] = (uint8_t)c;
        else if (c < 0x800) { o[k++] = (uint8_t)(0xC0 | (c >> 6)); o[k++] = (uint8_t)(0x80 | (c & 63)); }
        else { o[k++] = (uint8_t)(0xE0 | (c >> 12)); o[k++] = (uint8_t)(0x80 | ((c >> 6) & 63)); o[k++] = (uint8_t)(0x80 | (c & 63)); }
    }
    return k;
}

/* Java value -> Spark row value, written as an event payload. Returns 0 on heap overflow. */
static int to_event(const ora_node* nd, const jvalue* v, ora_event* e, uint8_t* heap, int64_t cap, int64_t* hl) {
    int32_t P, S;
    e->stype = ora_spark_type(nd, &P, &S);
    e->lo = e->hi = 0;
    e->isnull = v->type == JNULL;
    if (e->isnull) return 1;
    switch (e->stype) {
    case ORA_ST_INT: e->lo = v->i; e->hi = v->i < 0 ? -1 : 0; break;
    case ORA_ST_LONG: e->lo = v->l; e->hi = v->l < 0 ? -1 : 0; break;
    case ORA_ST_DECIMAL: {
        i128 u;
        if (!to_precision(v, P, S, &u)) { e->isnull = 1; break; }
        e->lo = (int64_t)(uint64_t)u; e->hi = (int64_t)(u >> 64);
        break;
    }
    case ORA_ST_FLOAT: e->lo = (int64_t)v->fbits; break;
    case ORA_ST_DOUBLE: e->lo = (int64_t)v->dbits; break;
    case ORA_ST_STRING: {
        uint8_t u8[MAXS * 3];
        int k = utf16_to_utf8(v->str, v->slen, u8);
        int64_t off;
        if (!put_heap(heap, cap, hl, u8, k, &off)) return 0;
        e->lo = off; e->hi = k;
        break;
    }
    case ORA_ST_BINARY: {
        int64_t off;
        if (!put_heap(heap, cap, hl, v->bytes, v->blen, &off)) return 0;
        e->lo = off; e->hi = v->blen;
        break;
    }
    }
    return 1;
}

/* Primitive.decodeTypeValue (CP/parser/ast/Primitive.scala:102-128) */
static void decode_type_value(const ora_node* nd, const ora_options* opt, int off, const uint8_t* rec,
                              int rec_len, jvalue* v) {
    int bc = nd->data_size;
    if (nd->tclass == ORA_ALPHA) {
        if (off > rec_len) { v->type = JNULL; return; }
    } else {
        if (off + bc > rec_len) { v->type = JNULL; return; }
    }
    int n = off + bc > rec_len ? rec_len - off : bc;
    decode_value(nd, opt, rec + off, n, v);
}

/* ------------------------------------------------------------------------------------------ */
/* extractRecord (CP/reader/extractors/record/RecordExtractors.scala:49-183)                  */
/* ------------------------------------------------------------------------------------------ */

#define MAX_DEPS 256

typedef struct {
    const ora_node* nodes;
    const ora_handler* handlers;
    const ora_options* opt;
    const uint8_t* data;
    int data_len;
    int active_seg;
    uint32_t rec;
    ora_event* ev;
    int64_t ev_cap, n_ev;
    uint8_t* heap;
    int64_t heap_cap, heap_len;
    int err;
    /* dependFields: name id -> Left(int) / Right(string) */
    int ndeps;
    int dep_name[MAX_DEPS];
    int dep_is_str[MAX_DEPS];
    int dep_int[MAX_DEPS];
    uint16_t dep_str[MAX_DEPS][64];
    int dep_slen[MAX_DEPS];
    int depth;
    int idx_stack[16], max_stack[16];
    /* extractHierarchicalRecord only: the walk's hierarchical state; mute = decode without events */
    struct hier_ctx* hier;
    int mute;
    ora_event dummy;
} walk_ctx;

static ora_event* new_event(walk_ctx* c) {
    if (c->mute) { memset(&c->dummy, 0, sizeof(c->dummy)); return &c->dummy; }
    if (c->n_ev >= c->ev_cap) { c->err = -1; return NULL; }
    ora_event* e = &c->ev[c->n_ev++];
    memset(e, 0, sizeof(*e));
    e->rec = c->rec;
    return e;
}

static int dep_find(walk_ctx* c, int name_id) {
    for (int i = 0; i < c->ndeps; i++) if (c->dep_name[i] == name_id) return i;
    return -1;
}

static int java_int_value(const jvalue* v, int* out) {
    switch (v->type) {
    case JINT: *out = v->i; return 1;
    case JLONG: *out = (int32_t)v->l; return 1;       /* Number.intValue */
    case JFLOAT: { float f; memcpy(&f, &v->fbits, 4); *out = f != f ? 0 : (f >= 2147483647.0f ? 2147483647 : (f <= -2147483648.0f ? (-2147483647 - 1) : (int)f)); return 1; }
    case JDOUBLE: { double d; memcpy(&d, &v->dbits, 8); *out = d != d ? 0 : (d >= 2147483647.0 ? 2147483647 : (d <= -2147483648.0 ? (-2147483647 - 1) : (int)d)); return 1; }
    case JBIGDEC: {
        /* BigDecimal.intValue: integer part, low 32 bits */
        int nd = (int)strlen(v->digits);
        int ip = nd - v->scale;
        uint64_t acc = 0;
        for (int i = 0; i < ip && i < nd; i++) acc = acc * 10 + (uint64_t)(v->digits[i] - '0');
        for (int i = nd; i < ip; i++) acc = acc * 10;
        uint32_t lo = (uint32_t)acc;
        *out = v->neg ? (int32_t)(0u - lo) : (int32_t)lo;
        return 1;
    }
    default: return 0;
    }
}

static void walk_group(walk_ctx* c, int gid, int offset, int* size_out);

/* flattened element index over the enclosing arrays (mixed radix of arrayMaxSize) */
static int cur_slot(const walk_ctx* c) {
    int s = 0;
    for (int k = 0; k < c->depth; k++) s = s * c->max_stack[k] + c->idx_stack[k];
    return s;
}

static void emit_value(walk_ctx* c, int nid, const jvalue* v, int slot) {
    if (c->mute) return;
    ora_event* e = new_event(c);
    if (!e) return;
    e->node = nid;
    e->kind = ORA_EV_VALUE;
    e->slot = slot;
    if (!to_event(&c->nodes[nid], v, e, c->heap, c->heap_cap, &c->heap_len)) c->err = -2;
}

/* extractArray (:66-114) */
static int extract_array(walk_ctx* c, int nid, int use_offset) {
    const ora_node* f = &c->nodes[nid];
    int array_size = f->occurs_max;
    int actual = array_size;
    if (f->depending_on_id >= 0) {
        int dv = array_size;
        int k = dep_find(c, f->depending_on_id);
        if (k >= 0) {
            if (!c->dep_is_str[k]) dv = c->dep_int[k];
            else {
                dv = array_size;
                for (int h = f->handlers_begin; h < f->handlers_end; h++) {
                    const ora_handler* hd = &c->handlers[h];
                    if (hd->key_len == c->dep_slen[k] && memcmp(hd->key, c->dep_str[k], (size_t)hd->key_len * 2) == 0) {
                        dv = hd->value; break;
                    }
                }
            }
        }
        actual = (dv >= f->occurs_min && dv <= array_size) ? dv : array_size;
    }
    ora_event* e = new_event(c);
    if (!e) return 0;
    int base = cur_slot(c);
    e->node = nid; e->kind = ORA_EV_ARRAY; e->lo = actual; e->slot = base;
    int offset = use_offset;
    for (int i = 0; i < actual; i++) {
        if (f->kind == ORA_GROUP) {
            int sz;
            if (c->depth >= 16) { c->err = -5; return 0; }
            c->max_stack[c->depth] = array_size; c->idx_stack[c->depth] = i; c->depth++;
            walk_group(c, nid, offset, &sz);
            c->depth--;
            offset += sz;
        } else {
            jvalue v;
            decode_type_value(f, c->opt, offset, c->data, c->data_len, &v);
            offset += f->data_size;
            emit_value(c, nid, &v, base * array_size + i);
        }
        if (c->err) return 0;
    }
    return c->opt->variable_size_occurs ? offset - use_offset : f->actual_size;
}

/* extractValue (:116-137) */
static int extract_value(walk_ctx* c, int nid, int use_offset) {
    const ora_node* f = &c->nodes[nid];
    if (f->kind == ORA_GROUP) {
        if (f->is_segment_redefine && c->active_seg != ORA_ALL_SEGMENTS && f->name_upper_id != c->active_seg) {
            ora_event* e = new_event(c);
            if (e) { e->node = nid; e->kind = ORA_EV_SEGNULL; e->slot = cur_slot(c); }
            return f->actual_size;
        }
        int sz;
        walk_group(c, nid, use_offset, &sz);
        return sz;
    }
    jvalue v;
    decode_type_value(f, c->opt, use_offset, c->data, c->data_len, &v);
    if (v.type != JNULL && f->is_dependee) {
        int k = dep_find(c, f->name_id);
        if (k < 0) {
            if (c->ndeps >= MAX_DEPS) { c->err = -3; return 0; }
            k = c->ndeps++;
            c->dep_name[k] = f->name_id;
        }
        if (v.type == JSTRING) {
            c->dep_is_str[k] = 1;
            c->dep_slen[k] = v.slen < 64 ? v.slen : 64;
            memcpy(c->dep_str[k], v.str, (size_t)c->dep_slen[k] * 2);
        } else {
            int iv;
            if (!java_int_value(&v, &iv)) { c->err = -3; return 0; }
            c->dep_is_str[k] = 0;
            c->dep_int[k] = iv;
        }
    }
    emit_value(c, nid, &v, cur_slot(c));
    return f->actual_size;
}

static void hier_children(walk_ctx* c, int gid);

/* getGroupValues (:139-172; the hierarchical form :324-369 also mutes child-segment fields and
 * appends the group's children) */
static void walk_group(walk_ctx* c, int gid, int offset, int* size_out);

typedef struct hier_ctx {
    int32_t n;
    const uint8_t* const* datas;
    const int32_t* lens;
    const int32_t* seg_group;
    const int32_t* seg_key;
    const int32_t* child_begin;
    const int32_t* child_end;
    const int32_t* children;
    const int32_t* node_offset;
    const int32_t* is_child_seg;
    uint32_t rec_base;
    int cur;            /* currentIndex: the record whose group is being walked */
    int path[64];       /* parentSegmentIds of that walk */
    int path_len;
} hier_ctx;

static void walk_group(walk_ctx* c, int gid, int offset, int* size_out) {
    int bit_offset = offset;
    for (int ch = c->nodes[gid].first_child; ch >= 0; ch = c->nodes[ch].next_sibling) {
        const ora_node* f = &c->nodes[ch];
        const int saved_mute = c->mute;
        if (c->hier && c->hier->is_child_seg[ch]) c->mute = 1;
        if (f->is_array) {
            int sz = extract_array(c, ch, bit_offset);
            c->mute = saved_mute;
            if (c->err) return;
            if (!f->is_redefined) bit_offset += sz;
        } else {
            int sz = extract_value(c, ch, bit_offset);
            c->mute = saved_mute;
            if (c->err) return;
            if (!f->is_redefined) {
                if (f->has_redefines) bit_offset += f->actual_size;
                else bit_offset += sz;
            }
        }
    }
    *size_out = bit_offset - offset;
    if (c->hier && c->nodes[gid].is_segment_redefine) hier_children(c, gid);
}

static int hier_in_path(const hier_ctx* h, int key) {
    for (int i = 0; i < h->path_len; i++) if (h->path[i] == key) return 1;
    return 0;
}

/* extractChildren (:300-322) for each child segment of gid, in parentChildMap order */
static void hier_children(walk_ctx* c, int gid) {
    hier_ctx* h = c->hier;
    for (int k = h->child_begin[gid]; k < h->child_end[gid]; k++) {
        const int field = h->children[k];
        const int from = h->cur + 1;
        int cnt = 0;
        for (int i = from; i < h->n; i++) {
            if (h->seg_group[i] == field) cnt++;
            else if (hier_in_path(h, h->seg_key[i])) break;
        }
        ora_event* e = new_event(c);
        if (!e) return;
        e->node = field; e->kind = ORA_EV_CHILDREN; e->lo = cnt; e->slot = 0;
        const uint8_t* sdata = c->data;
        const int slen = c->data_len, scur = h->cur, sdepth = c->depth;
        const uint32_t srec = c->rec;
        for (int i = from; i < h->n; i++) {
            if (h->seg_group[i] == field) {
                if (h->path_len >= 64) { c->err = -5; return; }
                c->data = h->datas[i]; c->data_len = h->lens[i]; c->rec = h->rec_base + (uint32_t)i;
                h->cur = i;
                memmove(h->path + 1, h->path, sizeof(int) * (size_t)h->path_len);   /* segmentId :: parentSegmentIds */
                h->path[0] = h->seg_key[i];
                h->path_len++;
                c->depth = 0;
                int sz;
                walk_group(c, field, h->node_offset[field], &sz);
                h->path_len--;
                memmove(h->path, h->path + 1, sizeof(int) * (size_t)h->path_len);
                c->depth = sdepth;
                h->cur = scur;
                if (c->err) return;
            } else if (hier_in_path(h, h->seg_key[i])) {
                break;
            }
        }
        c->data = sdata; c->data_len = slen; c->rec = srec;
    }
}

int ora_extract_hier(const ora_node* nodes, int32_t root, const ora_handler* handlers, const ora_options* opt,
                     int32_t n_records, const uint8_t* const* datas, const int32_t* lens,
                     const int32_t* seg_group, const int32_t* seg_key, const int32_t* child_begin,
                     const int32_t* child_end, const int32_t* children, const int32_t* node_offset,
                     const int32_t* is_child_seg, const int32_t* has_parent_seg, int32_t offset_bytes,
                     uint32_t rec_base, ora_event* ev, int64_t ev_cap, int64_t* n_ev,
                     uint8_t* heap, int64_t heap_cap, int64_t* heap_len) {
    if (n_records <= 0) return 0;
    walk_ctx* c = (walk_ctx*)calloc(1, sizeof(walk_ctx));
    hier_ctx* h = (hier_ctx*)calloc(1, sizeof(hier_ctx));
    if (!c || !h) { free(c); free(h); return -4; }
    h->n = n_records; h->datas = datas; h->lens = lens; h->seg_group = seg_group; h->seg_key = seg_key;
    h->child_begin = child_begin; h->child_end = child_end; h->children = children;
    h->node_offset = node_offset; h->is_child_seg = is_child_seg; h->rec_base = rec_base;
    h->cur = 0; h->path[0] = seg_key[0]; h->path_len = 1;   /* segmentsData(0)._1 :: Nil */
    c->nodes = nodes; c->handlers = handlers; c->opt = opt; c->data = datas[0]; c->data_len = lens[0];
    c->active_seg = ORA_ALL_SEGMENTS; c->rec = rec_base;
    c->ev = ev; c->ev_cap = ev_cap; c->n_ev = *n_ev;
    c->heap = heap; c->heap_cap = heap_cap; c->heap_len = *heap_len;
    c->hier = h;
    /* ast.children.collect { case grp: Group if grp.parentSegment.isEmpty => getGroupValues(nextOffset, ...) } */
    int next_offset = offset_bytes;
    for (int r = nodes[root].first_child; r >= 0; r = nodes[r].next_sibling) {
        if (nodes[r].kind != ORA_GROUP || has_parent_seg[r]) continue;
        int sz;
        walk_group(c, r, next_offset, &sz);
        if (c->err) break;
        next_offset += sz;
    }
    int err = c->err;
    *n_ev = c->n_ev;
    *heap_len = c->heap_len;
    free(h);
    free(c);
    return err;
}

int ora_extract_record(const ora_node* nodes, int32_t root, const ora_handler* handlers,
                       const ora_options* opt, const uint8_t* data, int32_t data_len,
                       int32_t offset_bytes, int32_t active_segment_upper_id, uint32_t rec,
                       ora_event* ev, int64_t ev_cap, int64_t* n_ev,
                       uint8_t* heap, int64_t heap_cap, int64_t* heap_len) {
    walk_ctx* c = (walk_ctx*)calloc(1, sizeof(walk_ctx));
    if (!c) return -4;
    c->nodes = nodes; c->handlers = handlers; c->opt = opt; c->data = data; c->data_len = data_len;
    c->active_seg = active_segment_upper_id; c->rec = rec;
    c->ev = ev; c->ev_cap = ev_cap; c->n_ev = *n_ev;
    c->heap = heap; c->heap_cap = heap_cap; c->heap_len = *heap_len;
    int next_offset = offset_bytes;
    for (int r = nodes[root].first_child; r >= 0; r = nodes[r].next_sibling) {
        int sz;
        if (nodes[r].kind == ORA_GROUP) walk_group(c, r, next_offset, &sz);
        else { sz = extract_value(c, r, next_offset); }
        if (c->err) break;
        next_offset += sz;
    }
    int err = c->err;
    *n_ev = c->n_ev;
    *heap_len = c->heap_len;
    free(c);
    return err;
}

/* FixedLenNestedRowIterator.getSegmentId (:89-99): extractPrimitiveField + toString.trim */
static int segment_of(const ora_node* nodes, const ora_options* opt, int seg_field, const uint8_t* rec,
                      int rec_len, int base, const ora_handler* keys, int n_keys) {
    const ora_node* f = &nodes[seg_field];
    /* slice(offset, offset + actualSize) then decodeTypeValue(0, slice) */
    int start = base;
    int end = base + f->actual_size;
    if (start > rec_len) start = rec_len;
    if (end > rec_len) end = rec_len;
    jvalue v;
    decode_type_value(f, opt, 0, rec + start, end - start, &v);
    uint16_t s[MAXS];
    int sl = 0;
    if (v.type == JSTRING) { memcpy(s, v.str, (size_t)v.slen * 2); sl = v.slen; }
    else if (v.type == JINT || v.type == JLONG) {
        char t[32]; char* p = t;
        int64_t x = v.type == JINT ? v.i : v.l;
        if (x < 0) { *p++ = '-'; u128_to_str((u128)(-(i128)x), p); } else u128_to_str((u128)x, p);
        for (sl = 0; t[sl]; sl++) s[sl] = (uint16_t)t[sl];
    } else if (v.type == JBIGDEC) {
        char t[MAXS]; int p = 0, nd = (int)strlen(v.digits);
        if (v.neg) t[p++] = '-';
        if (v.scale == 0) { strcpy(t + p, v.digits); }
        else if (nd > v.scale) { memcpy(t + p, v.digits, (size_t)(nd - v.scale)); p += nd - v.scale; t[p++] = '.'; strcpy(t + p, v.digits + nd - v.scale); }
        else { t[p++] = '0'; t[p++] = '.'; for (int z = 0; z < v.scale - nd; z++) t[p++] = '0'; strcpy(t + p, v.digits); }
        for (sl = 0; t[sl]; sl++) s[sl] = (uint16_t)t[sl];
    }
    apply_trim(s, &sl, ORA_TRIM_BOTH);
    for (int k = 0; k < n_keys; k++)
        if (keys[k].key_len == sl && memcmp(keys[k].key, s, (size_t)sl * 2) == 0) return keys[k].value;
    return -1;
}

int ora_decode_fixed(const ora_node* nodes, int32_t root, const ora_handler* handlers,
                     const ora_options* opt, const uint8_t* data, int64_t n_rec, int32_t stride,
                     int32_t start_offset, int32_t seg_field, int32_t seg_field_offset,
                     const ora_handler* seg_keys, int32_t n_seg_keys,
                     ora_event* ev, int64_t ev_cap, int64_t* n_ev,
                     uint8_t* heap, int64_t heap_cap, int64_t* heap_len) {
    for (int64_t i = 0; i < n_rec; i++) {
        const uint8_t* rec = data + i * (int64_t)stride;
        int active = -1;
        if (seg_field >= 0)
            active = segment_of(nodes, opt, seg_field, rec, stride, start_offset + seg_field_offset, seg_keys, n_seg_keys);
        int r = ora_extract_record(nodes, root, handlers, opt, rec, stride, start_offset, active,
                                   (uint32_t)i, ev, ev_cap, n_ev, heap, heap_cap, heap_len);
        if (r) return r;
    }
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* RDW framing + sparse index                                                                  */
/* ------------------------------------------------------------------------------------------ */

#define MAX_RDW (100 * 1024 * 1024)

/* one VRLRecordReader.fetchRecordUsingRdwHeaders step over an in-memory stream */
typedef struct { int64_t pos, size; } stream_t;

/* returns: 1 record (payload off/len, valid flag), 0 end of file, <0 error */
static int rdw_next(const uint8_t* d, stream_t* s, int be, int adj, int fhb, int ffb,
                    int64_t* off, int32_t* len, int* valid, int64_t* err_off) {
    int64_t hdr_avail = s->size - s->pos;
    int64_t hl = hdr_avail < 4 ? hdr_avail : 4;
    const uint8_t* h = d + s->pos;
    s->pos += hl;                     /* dataStream.next(4) */
    int64_t file_offset = s->pos;     /* dataStream.offset after the header read */
    int64_t rlen;
    int ok;
    if (fhb > 4 && file_offset == 4) { rlen = fhb - 4; ok = 0; }
    else if (s->size > 0 && ffb > 0 && s->size - file_offset <= ffb) { rlen = s->size - file_offset; ok = 0; }
    else {
        if (hl < 4) { rlen = -1; ok = 0; }
        else {
            rlen = be ? (int64_t)h[1] + 256 * (int64_t)h[0] + adj : (int64_t)h[2] + 256 * (int64_t)h[3] + adj;
            if (rlen > 0) {
                if (rlen > MAX_RDW) { *err_off = file_offset; return -3; }
                ok = 1;
            } else { *err_off = file_offset; return -2; }
        }
    }
    if (rlen > 0) {
        int64_t avail = s->size - s->pos;
        int64_t got = rlen < avail ? rlen : avail;
        *off = s->pos; *len = (int32_t)got;
        s->pos += got;
        *valid = ok;
        return 1;
    }
    return 0;
}

int64_t ora_frame_rdw(const uint8_t* data, int64_t n_bytes, int32_t big_endian, int32_t adjustment,
                      int32_t file_header_bytes, int32_t file_footer_bytes,
                      int64_t* rec_off, int32_t* rec_len, int64_t cap, int64_t* err_offset) {
    stream_t s = {0, n_bytes};
    int64_t n = 0;
    while (1) {
        int64_t off; int32_t len; int valid;
        int r = rdw_next(data, &s, big_endian, adjustment, file_header_bytes, file_footer_bytes, &off, &len, &valid, err_offset);
        if (r < 0) return r;
        if (r == 0) break;
        if (!valid) continue;
        if (n >= cap) return -1;
        rec_off[n] = off; rec_len[n] = len; n++;
    }
    return n;
}

/* IndexGenerator.sparseIndexGenerator (CP/reader/index/IndexGenerator.scala:33-127), record
 * header parser branch.  is_root[k] (k = record index incl. invalid records) enables the
 * hierarchical "cut only at root segments" rule; NULL for flat files. */
int64_t ora_sparse_index(const uint8_t* data, int64_t n_bytes, int32_t big_endian, int32_t adjustment,
                         int32_t file_header_bytes, int32_t file_footer_bytes,
                         int64_t records_per_entry, int64_t size_per_entry_mb,
                         const int32_t* is_root,
                         int64_t* out_from, int64_t* out_to, int64_t* out_rec, int64_t cap) {
    const int64_t MB = 1048576;
    int split_by_size = records_per_entry <= 0 && size_per_entry_mb > 0;
    int64_t bytes_per = (size_per_entry_mb > 0 ? size_per_entry_mb : 100) * MB;
    int64_t byte_index = 0, records_in_chunk = 0, bytes_in_chunk = 0, record_index = 0;
    int64_t n = 0;
    if (cap < 1) return -1;
    out_from[0] = 0; out_to[0] = -1; out_rec[0] = 0; n = 1;
    stream_t s = {0, n_bytes};
    while (1) {
        int64_t before = s.pos;
        int64_t off; int32_t len; int valid = 0, err;
        int64_t eo;
        err = rdw_next(data, &s, big_endian, adjustment, file_header_bytes, file_footer_bytes, &off, &len, &valid, &eo);
        if (err < 0) return err;
        int64_t record_size = s.pos - byte_index;
        (void)before;
        int has_more = record_size > 0;
        int eos = s.pos >= s.size;
        if (eos || !has_more) break;
        if (valid && err == 1) {
            int need = records_per_entry > 0 ? records_in_chunk >= records_per_entry : bytes_in_chunk >= bytes_per;
            if (need && (!is_root || is_root[record_index])) {
                if (n >= cap) return -1;
                out_to[n - 1] = byte_index;
                out_from[n] = byte_index; out_to[n] = -1; out_rec[n] = record_index; n++;
                records_in_chunk = 0;
                if (split_by_size) bytes_in_chunk -= size_per_entry_mb * MB;
                else bytes_in_chunk = 0;
            }
        }
        record_index++;
        records_in_chunk++;
        byte_index += record_size;
        bytes_in_chunk += record_size;
    }
    return n;
}

int ora_decode_field(const ora_node* node, const ora_options* opt, const uint8_t* bytes,
                     int32_t n, ora_event* out, uint8_t* heap, int64_t heap_cap, int64_t* heap_len) {
    jvalue v;
    memset(out, 0, sizeof(*out));
    decode_value(node, opt, bytes, n, &v);
    out->kind = ORA_EV_VALUE;
    return to_event(node, &v, out, heap, heap_cap, heap_len) ? 0 : -2;
}

/* Batch of variable-length records (VarLenNestedIterator.fetchNext over framed payloads):
 * record i = data[rec_off[i], rec_off[i] + rec_len[i]), active segment id act[i] (or -1). */
int ora_extract_var(const ora_node* nodes, int32_t root, const ora_handler* handlers,
                    const ora_options* opt, const uint8_t* data, const int64_t* rec_off,
                    const int32_t* rec_len, const int32_t* act, int64_t n, int32_t offset_bytes,
                    ora_event* ev, int64_t ev_cap, int64_t* n_ev,
                    uint8_t* heap, int64_t heap_cap, int64_t* heap_len) {
    for (int64_t i = 0; i < n; i++) {
        int r = ora_extract_record(nodes, root, handlers, opt, data + rec_off[i], rec_len[i], offset_bytes,
                                   act ? act[i] : -1, (uint32_t)i, ev, ev_cap, n_ev, heap, heap_cap, heap_len);
        if (r != 0) return r;
    }
    return 0;
}

/* Text records (is_text): TextRecordExtractor (CP/reader/extractors/raw/TextRecordExtractor.scala:26-108)
 * restated over a SimpleStream of n_bytes (isEndOfStream = offset >= size, SimpleStream.scala:28;
 * next(k) returns min(k, remaining) bytes).  The window buffer is simulated literally, including
 * ensureBytesRead (:98-107) setting bytesSize to the full window after a short read: bytes past
 * the data then read as the buffer's zero fill.  Records are written as (offset, payload length)
 * in stream coordinates; *virtual_bytes = the end of the last window. */
int64_t ora_frame_text(const uint8_t* data, int64_t n_bytes, int32_t record_size, int64_t* off, int32_t* len,
                       int64_t cap, int64_t* virtual_bytes) {
    const int64_t M = (int64_t)record_size + 2;   /* maxRecordSize (:28) */
    int64_t base = 0;      /* stream offset of bytes(0) */
    int64_t size = 0;      /* bytesSize */
    int64_t pos = 0;       /* inputStream.offset */
    int64_t vend = 0;      /* end of the filled window */
    int32_t last_footer = 1;   /* lastFooterSize (:31) */
    int64_t k = 0;
#define TB(i) ((base + (i)) < n_bytes ? data[base + (i)] : (uint8_t)0)
    while (pos < n_bytes || size > 0) {   /* hasNext (:33) */
        /* ensureBytesRead(maxRecordSize) (:98-107) */
        const int64_t want = M - size;
        if (want > 0) {
            const int64_t got = (n_bytes - pos) < want ? (n_bytes - pos) : want;
            if (got > 0) {
                pos += got;
                size = M;
                if (base + M > vend) vend = base + M;
            }
        }
        /* findEol (:46-95); buffer bytes past bytesSize are zero (fill at :89) */
        int64_t rec_len = 0, payload = 0;
        for (int64_t i = 0; rec_len == 0 && i < size; i++) {
            const uint8_t b = (base + i) < vend ? TB(i) : 0;
            if (b == 0x0D) {
                if (i + 1 < M && ((base + i + 1) < vend && i + 1 < size ? TB(i + 1) : 0) == 0x0A) {
                    rec_len = i + 2;
                    payload = i;
                }
            } else if (b == 0x0A) {
                rec_len = i + 1;
                payload = i;
            }
        }
        if (rec_len == 0) {
            if (pos >= n_bytes) { rec_len = size; payload = size; }                       /* last record */
            else { rec_len = size - last_footer; payload = size - last_footer; }         /* no line break */
        }
        if (k < cap) { off[k] = base; len[k] = (int32_t)payload; }
        k++;
        base += rec_len;
        size -= rec_len;
        last_footer = (int32_t)(rec_len - payload);
    }
#undef TB
    *virtual_bytes = vend > n_bytes ? vend : n_bytes;
    return k;
}

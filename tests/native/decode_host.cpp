// TEST SHIM: runs the device field decoders (cobrix_amd/csrc/cbx_decode.h) on the host so the
// exact GPU arithmetic can be fuzzed against the C oracle without a GPU.  Built by
// tests/native/Makefile with hipcc (host path of __host__ __device__ functions); never part of
// the product library.
#include "cbx_decode.h"

using namespace cbx;

extern "C" int cbxh_decode(const cbx_field* cf, const uint8_t* p, int n_avail, const uint32_t* lut,
                           uint64_t* lo, uint64_t* hi, uint8_t* sbuf, int32_t* slen) {
    Field f = make_field(*cf);
    *lo = *hi = 0;
    *slen = 0;
    const bool is_str = f.out_type == CBX_O_STRING || f.out_type == CBX_O_BINARY;
    if (!is_str) {
        if (n_avail < f.size) return 0;  // Primitive.decodeTypeValue numeric bounds
        // the kernels' path: width-specialised decoders reading a (padded) byte image
        alignas(16) uint8_t img[16 + 64 + 16];
        for (int i = 0; i < (int)sizeof img; i++) img[i] = (uint8_t)(0x5A ^ i);   // guard garbage
        const int at = 16 + (int)(reinterpret_cast<uintptr_t>(p) & 3);           // vary alignment
        for (int i = 0; i < f.size && i < 64; i++) img[i + at] = p[i];
        bool defer = false;
        const NumOp op = make_numop(f, 0, 0, nullptr, nullptr, 0);
        Val v = f.size <= 64 ? decode_value(op, img, at, defer) : decode_numeric(f, p);
        if (f.size <= 64 && f.out_type != CBX_O_DEC128) {
            // the kernels' narrow-output (<= 8 bytes) specialisation must agree on the low word
            bool d8 = false;
            const Val v8 = decode_value<8>(op, img, at, d8);
            if (d8 != defer || v8.valid != v.valid || (v.valid && v8.lo != v.lo)) return -1;
        }
        Val g = decode_numeric(f, p);   // generic byte-loop decoder must agree
        if (defer) {
            if (v.valid) return -1;    // a deferred value is left null for the fixup pass
            v = g;                     // ... which decodes it with the byte-loop decoder
        }
        if (f.flags & CBX_F_DEPENDEE) {   // OCCURS DEPENDING ON decoder must agree as well
            Val c = decode_count_int(f, p);
            if (f.precision <= 18 && (f.flags & CBX_F_INTEGRAL) &&
                (c.valid != g.valid || (g.valid && (int32_t)c.lo != (int32_t)g.lo))) return -1;
        }
        if (g.valid != v.valid || (v.valid && (g.lo != v.lo || g.hi != v.hi))) return -1;
        *lo = v.lo;
        *hi = v.hi;
        return v.valid ? 1 : 0;
    }
    if (n_avail < 0) return 0;
    int n = f.size < n_avail ? f.size : n_avail;
    auto lutf = [&](uint32_t b) -> uint32_t { return f.kind == CBX_K_STRING_ASCII ? ascii_lut(b) : lut[b]; };
    StrSpan s = string_span(f.kind, f.trim, p, n, lutf);
    string_write(f.kind, p, s, sbuf, lutf);
    if ((f.kind == CBX_K_STRING || f.kind == CBX_K_STRING_ASCII) && f.size <= kStrFastBytes) {
        // the kernels' register path must agree with the byte loop
        alignas(16) uint8_t img[16 + 64 + 16];
        for (int i = 0; i < (int)sizeof img; i++) img[i] = (uint8_t)(0xA5 ^ (3 * i));
        const int at = 16 + (int)(reinterpret_cast<uintptr_t>(p) & 3);
        for (int i = 0; i < n; i++) img[at + i] = p[i];
        uint32_t w[8];
        img_bytes32(img, at, f.size, w);
        StrSpan s2 = string_span32(f.trim, w, n, f.size, lutf);
        if (s2.begin != s.begin || s2.end != s.end || s2.utf8_len != s.utf8_len) return -1;
        uint8_t out2[4 * kStrFastBytes + 8], dump[4];
        string_write32(w, s2, out2, dump, f.size, 3, lutf);
        for (int i = 0; i < s.utf8_len; i++) if (out2[i] != sbuf[i]) return -1;
    }
    *slen = s.utf8_len;
    return 1;
}

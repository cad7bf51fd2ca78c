// jpeg_decode.cpp — JPEG texture decode (ITU-T T.81 baseline + progressive Huffman, 8-bit).
//
// Texture::load (RTBase/Imaging.h:50-61) calls stbi_load; on x86-64 the vendored stb_image
// v2.30 selects its SSE2 kernels, so the bits of a decoded texel are fixed by:
//   * coefficient decode: T.81 Annex F (sequential) and G (progressive); coefficients are kept
//     as 16-bit, dequantized by a 16-bit multiply (truncated to short);
//   * the IDCT: the islow 2-D integer IDCT with 12-bit fixed-point rotations, column pass
//     rounded (+512) and >>10 then saturated to 16 bit, row pass biased by 65536 + (128<<17),
//     >>17 and saturated to 0..255; the 16-bit sums of coefficient pairs wrap, the rotations are
//     16x16->32-bit dot products (what stbi__idct_simd computes);
//   * chroma upsampling: the "fancy" triangle filter (3:1 vertical then 3:1 horizontal, +8 >>4)
//     for 2x2, 3:1 +2 >>2 for the 2x1 / 1x2 cases, nearest for other factors;
//   * YCbCr -> RGB: 20-bit fixed point with 12-bit coefficients (<<8), the Cb term of green
//     truncated to its high 16 bits, rounding bias 1<<19, clamp (3-channel output path).
// Written from the standard; only the numeric conventions above are taken from stb's behaviour.
#include "image_io.h"

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace rth {
namespace {

const uint8_t kZigzag[64 + 16] = {  // natural index of the k-th zigzag coefficient (+ guard)
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

struct Huffman {
    bool defined = false;
    int mincode[17] = {}, maxcode[18] = {}, valptr[17] = {};
    uint8_t vals[256] = {};
    void build(const uint8_t counts[16], const uint8_t* symbols, int nsym) {
        std::memcpy(vals, symbols, nsym);
        int code = 0, k = 0;
        for (int l = 1; l <= 16; ++l) {
            valptr[l] = k;
            mincode[l] = code;
            code += counts[l - 1];
            k += counts[l - 1];
            maxcode[l] = counts[l - 1] ? code - 1 : -1;
            code <<= 1;
        }
        maxcode[17] = 0x7fffffff;
        defined = true;
    }
};

struct Component {
    int id = 0, h = 1, v = 1, tq = 0;
    int td = 0, ta = 0;    // Huffman table selectors of the current scan
    int dc_pred = 0;
    int x = 0, y = 0;      // component size in samples
    int bw = 0, bh = 0;    // blocks covering x, y
    int w2 = 0, h2 = 0;    // plane size (whole MCUs)
    int cw = 0;            // blocks per coefficient row (whole MCUs)
    std::vector<uint8_t> plane;
    std::vector<int16_t> coef;  // progressive only
};

struct Decoder {
    const uint8_t* p = nullptr;
    const uint8_t* end = nullptr;
    std::string err;
    // bit reader
    uint32_t acc = 0;
    int nbits = 0;
    int marker = -1;  // marker met inside entropy-coded data (-1: none)

    Huffman dc[4], ac[4];
    uint16_t quant[4][64] = {};  // natural order
    Component comp[4];
    int ncomp = 0, img_x = 0, img_y = 0, hmax = 1, vmax = 1, mcux = 0, mcuy = 0;
    bool progressive = false, jfif = false;
    int app14 = -1, restart_interval = 0, eobrun = 0;
    // current scan
    int scomp[4] = {}, sn = 0, ss = 0, se = 63, ah = 0, al = 0;

    bool fail(const char* m) { if (err.empty()) err = m; return false; }
    int u8() { return p < end ? *p++ : 0; }
    int u16() { int a = u8(); return (a << 8) | u8(); }

    // ---- entropy-coded segment bits (byte stuffing 0xFF00; a marker stops the stream)
    void fill() {
        while (nbits <= 24) {
            int b = 0;
            if (marker < 0 && p < end) {
                b = *p++;
                if (b == 0xFF) {
                    int c = p < end ? *p : 0;
                    while (c == 0xFF && p + 1 < end) { ++p; c = *p; }
                    if (c == 0) {
                        ++p;
                    } else {
                        marker = c;
                        ++p;
                        b = 0;
                    }
                }
            }
            acc |= (uint32_t)b << (24 - nbits);
            nbits += 8;
        }
    }
    int bits(int n) {
        if (n == 0) return 0;
        if (nbits < n) fill();
        int v = (int)(acc >> (32 - n));
        acc <<= n;
        nbits -= n;
        return v;
    }
    int bit() { return bits(1); }
    int decode(const Huffman& hf) {
        int code = 0;
        for (int l = 1; l <= 16; ++l) {
            code = (code << 1) | bit();
            if (code <= hf.maxcode[l]) return hf.vals[hf.valptr[l] + code - hf.mincode[l]];
        }
        return -1;
    }
    int extend(int s) {  // receive s bits, sign-extend per T.81 F.2.2.1
        if (s == 0) return 0;
        int v = bits(s);
        return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v;
    }
    void reset_bits() { acc = 0; nbits = 0; marker = -1; }

    // ---- marker segments
    bool read_dqt() {
        int len = u16() - 2;
        while (len > 0) {
            int pq_tq = u8();
            int pq = pq_tq >> 4, tq = pq_tq & 15;
            if (tq > 3 || pq > 1) return fail("bad DQT");
            for (int i = 0; i < 64; ++i) quant[tq][kZigzag[i]] = (uint16_t)(pq ? u16() : u8());
            len -= 1 + 64 * (pq ? 2 : 1);
        }
        return len == 0 || fail("bad DQT length");
    }
    bool read_dht() {
        int len = u16() - 2;
        while (len > 0) {
            int tc_th = u8();
            int tc = tc_th >> 4, th = tc_th & 15;
            if (tc > 1 || th > 3) return fail("bad DHT");
            uint8_t counts[16];
            int n = 0;
            for (int i = 0; i < 16; ++i) { counts[i] = (uint8_t)u8(); n += counts[i]; }
            if (n > 256) return fail("bad DHT count");
            uint8_t sym[256];
            for (int i = 0; i < n; ++i) sym[i] = (uint8_t)u8();
            (tc ? ac[th] : dc[th]).build(counts, sym, n);
            len -= 17 + n;
        }
        return len == 0 || fail("bad DHT length");
    }
    bool read_sof() {
        int len = u16();
        if (u8() != 8) return fail("only 8-bit JPEG");
        img_y = u16();
        img_x = u16();
        ncomp = u8();
        if (img_x <= 0 || img_y <= 0) return fail("bad JPEG size");
        if (ncomp != 1 && ncomp != 3 && ncomp != 4) return fail("bad component count");
        if (len != 8 + 3 * ncomp) return fail("bad SOF length");
        // stb_image's stbi__mad3sizes_valid(x, y, n): x * y * n within an int (stb_image.h:3298); the
        // sample planes below are sized from the header, so a corrupt one fails before allocating
        if ((int64_t)img_x * img_y * ncomp > (int64_t)INT32_MAX) return fail("JPEG too large to decode");
        hmax = vmax = 1;
        for (int i = 0; i < ncomp; ++i) {
            comp[i].id = u8();
            int hv = u8();
            comp[i].h = hv >> 4;
            comp[i].v = hv & 15;
            comp[i].tq = u8();
            if (comp[i].h < 1 || comp[i].h > 4 || comp[i].v < 1 || comp[i].v > 4 || comp[i].tq > 3)
                return fail("bad component");
            hmax = std::max(hmax, comp[i].h);
            vmax = std::max(vmax, comp[i].v);
        }
        for (int i = 0; i < ncomp; ++i)
            if (hmax % comp[i].h || vmax % comp[i].v) return fail("unsupported sampling factors");
        mcux = (img_x + 8 * hmax - 1) / (8 * hmax);
        mcuy = (img_y + 8 * vmax - 1) / (8 * vmax);
        for (int i = 0; i < ncomp; ++i) {
            Component& c = comp[i];
            c.x = (img_x * c.h + hmax - 1) / hmax;
            c.y = (img_y * c.v + vmax - 1) / vmax;
            c.bw = (c.x + 7) >> 3;
            c.bh = (c.y + 7) >> 3;
            c.w2 = mcux * c.h * 8;
            c.h2 = mcuy * c.v * 8;
            c.cw = mcux * c.h;
            c.plane.assign((size_t)c.w2 * c.h2, 0);
            if (progressive) c.coef.assign((size_t)c.w2 * c.h2, 0);
        }
        return true;
    }
    bool read_sos() {
        int len = u16();
        sn = u8();
        if (sn < 1 || sn > 4 || len != 6 + 2 * sn) return fail("bad SOS");
        for (int i = 0; i < sn; ++i) {
            int id = u8(), t = u8();
            int k = 0;
            while (k < ncomp && comp[k].id != id) ++k;
            if (k == ncomp) return fail("SOS component not in frame");
            scomp[i] = k;
            comp[k].td = t >> 4;
            comp[k].ta = t & 15;
            if (comp[k].td > 3 || comp[k].ta > 3) return fail("bad table selector");
        }
        ss = u8();
        se = u8();
        int a = u8();
        ah = a >> 4;
        al = a & 15;
        if (progressive) {
            if (ss > 63 || se > 63 || ss > se || ah > 13 || al > 13) return fail("bad progressive scan");
            if (ss == 0 && se != 0) return fail("bad progressive DC scan");
            if (ss != 0 && sn != 1) return fail("interleaved AC scan");
        } else if (ss != 0 || se != 63 || ah != 0 || al != 0) {
            return fail("bad sequential scan");
        }
        return true;
    }

    // ---- block decoders
    bool block_seq(int16_t out[64], Component& c) {
        const Huffman& hd = dc[c.td];
        const Huffman& ha = ac[c.ta];
        if (!hd.defined || !ha.defined) return fail("missing Huffman table");
        std::memset(out, 0, 64 * sizeof(int16_t));
        int t = decode(hd);
        if (t < 0 || t > 15) return fail("bad DC code");
        int dcv = c.dc_pred + extend(t);
        c.dc_pred = dcv;
        const uint16_t* q = quant[c.tq];
        out[0] = (int16_t)(dcv * q[0]);
        for (int k = 1; k < 64;) {
            int rs = decode(ha);
            if (rs < 0) return fail("bad AC code");
            int r = rs >> 4, s = rs & 15;
            if (s == 0) {
                if (r != 15) break;
                k += 16;
                continue;
            }
            k += r;
            if (k > 63) return fail("AC index overflow");
            int z = kZigzag[k++];
            out[z] = (int16_t)(extend(s) * q[z]);
        }
        return true;
    }
    bool block_dc_prog(int16_t* out, Component& c) {
        if (ah == 0) {
            if (!dc[c.td].defined) return fail("missing Huffman table");
            int t = decode(dc[c.td]);
            if (t < 0 || t > 15) return fail("bad DC code");
            int dcv = c.dc_pred + extend(t);
            c.dc_pred = dcv;
            out[0] = (int16_t)(dcv * (1 << al));
        } else if (bit()) {
            out[0] = (int16_t)(out[0] + (1 << al));
        }
        return true;
    }
    bool block_ac_first(int16_t* out, Component& c) {
        if (eobrun > 0) { --eobrun; return true; }
        const Huffman& ha = ac[c.ta];
        if (!ha.defined) return fail("missing Huffman table");
        for (int k = ss; k <= se;) {
            int rs = decode(ha);
            if (rs < 0) return fail("bad AC code");
            int r = rs >> 4, s = rs & 15;
            if (s == 0) {
                if (r < 15) {
                    eobrun = (1 << r) - 1;
                    if (r) eobrun += bits(r);
                    break;
                }
                k += 16;
                continue;
            }
            k += r;
            if (k > 63) return fail("AC index overflow");
            out[kZigzag[k++]] = (int16_t)(extend(s) * (1 << al));
        }
        return true;
    }
    // correction bit for an already-nonzero coefficient (T.81 G.1.2.3)
    void refine(int16_t& v, int p1) {
        if (bit() && (v & p1) == 0) v = (int16_t)(v >= 0 ? v + p1 : v - p1);
    }
    bool block_ac_refine(int16_t* out, Component& c) {
        const int p1 = 1 << al;
        int k = ss;
        if (eobrun <= 0) {
            const Huffman& ha = ac[c.ta];
            if (!ha.defined) return fail("missing Huffman table");
            for (; k <= se;) {
                int rs = decode(ha);
                if (rs < 0) return fail("bad AC code");
                int r = rs >> 4, s = rs & 15, val = 0;
                if (s == 0) {
                    if (r < 15) {
                        eobrun = 1 << r;
                        if (r) eobrun += bits(r);
                        break;  // the rest of this band is refined below as part of the EOB run
                    }
                    // r == 15: skip 16 zero-history coefficients (refining nonzero ones on the way)
                } else {
                    if (s != 1) return fail("bad refinement magnitude");
                    val = bit() ? p1 : -p1;
                }
                while (k <= se) {
                    int16_t& z = out[kZigzag[k]];
                    if (z != 0) {
                        refine(z, p1);
                    } else {
                        if (r == 0) {
                            if (val) z = (int16_t)val;
                            ++k;
                            break;
                        }
                        --r;
                    }
                    ++k;
                }
            }
        }
        if (eobrun > 0) {
            for (; k <= se; ++k) {
                int16_t& z = out[kZigzag[k]];
                if (z != 0) refine(z, p1);
            }
            --eobrun;
        }
        return true;
    }

    // ---- scans
    // After each restart interval the bit reader must be standing on RSTn (the padding bits of
    // the interval are dropped); any other marker ends the scan. Returns false to stop the scan.
    bool restart_if_due(int& todo) {
        if (restart_interval == 0 || --todo > 0) return true;
        if (nbits < 24) fill();
        if (!(marker >= 0xD0 && marker <= 0xD7)) return false;
        reset_bits();
        for (int i = 0; i < ncomp; ++i) comp[i].dc_pred = 0;
        eobrun = 0;
        todo = restart_interval;
        return true;
    }
    bool scan() {
        reset_bits();
        eobrun = 0;
        for (int i = 0; i < ncomp; ++i) comp[i].dc_pred = 0;
        int todo = restart_interval;
        int16_t blk[64];
        if (sn == 1) {
            Component& c = comp[scomp[0]];
            for (int by = 0; by < c.bh; ++by)
                for (int bx = 0; bx < c.bw; ++bx) {
                    if (!one_block(c, bx, by, blk)) return false;
                    if (!restart_if_due(todo)) return err.empty();
                }
        } else {
            for (int my = 0; my < mcuy; ++my)
                for (int mx = 0; mx < mcux; ++mx) {
                    for (int i = 0; i < sn; ++i) {
                        Component& c = comp[scomp[i]];
                        for (int y = 0; y < c.v; ++y)
                            for (int x = 0; x < c.h; ++x)
                                if (!one_block(c, mx * c.h + x, my * c.v + y, blk)) return false;
                    }
                    if (!restart_if_due(todo)) return err.empty();
                }
        }
        return true;
    }
    bool one_block(Component& c, int bx, int by, int16_t* tmp) {
        if (!progressive) {
            if (!block_seq(tmp, c)) return false;
            idct(tmp, &c.plane[(size_t)by * 8 * c.w2 + (size_t)bx * 8], c.w2);
            return true;
        }
        int16_t* out = &c.coef[64 * ((size_t)by * c.cw + bx)];
        if (ss == 0) return block_dc_prog(out, c);
        return ah == 0 ? block_ac_first(out, c) : block_ac_refine(out, c);
    }
    void finish_progressive() {
        for (int n = 0; n < ncomp; ++n) {
            Component& c = comp[n];
            const uint16_t* q = quant[c.tq];
            for (int by = 0; by < c.bh; ++by)
                for (int bx = 0; bx < c.bw; ++bx) {
                    int16_t* d = &c.coef[64 * ((size_t)by * c.cw + bx)];
                    for (int i = 0; i < 64; ++i) d[i] = (int16_t)(d[i] * q[i]);
                    idct(d, &c.plane[(size_t)by * 8 * c.w2 + (size_t)bx * 8], c.w2);
                }
        }
    }

    // ---- IDCT (see header). 16-bit lane semantics: wrap for pair sums, saturate between passes.
    static int f2f(float x) { return (int)((x * 4096) + 0.5); }
    static int16_t sat16(int32_t v) { return (int16_t)(v < -32768 ? -32768 : (v > 32767 ? 32767 : v)); }
    static int16_t w16(int32_t v) { return (int16_t)(uint16_t)(uint32_t)v; }
    static int32_t dot(int16_t a, int16_t b, int ca, int cb) {
        return (int32_t)((uint32_t)((int32_t)a * (int16_t)ca) + (uint32_t)((int32_t)b * (int16_t)cb));
    }
    static void pass1d(const int16_t r[8], int32_t bias, int shift, int32_t o[8]) {
        static const int r00a = f2f(0.5411961f), r00b = f2f(0.5411961f) + f2f(-1.847759065f);
        static const int r01a = f2f(0.5411961f) + f2f(0.765366865f), r01b = f2f(0.5411961f);
        static const int r10a = f2f(1.175875602f) + f2f(-0.899976223f), r10b = f2f(1.175875602f);
        static const int r11a = f2f(1.175875602f), r11b = f2f(1.175875602f) + f2f(-2.562915447f);
        static const int r20a = f2f(-1.961570560f) + f2f(0.298631336f), r20b = f2f(-1.961570560f);
        static const int r21a = f2f(-1.961570560f), r21b = f2f(-1.961570560f) + f2f(3.072711026f);
        static const int r30a = f2f(-0.390180644f) + f2f(2.053119869f), r30b = f2f(-0.390180644f);
        static const int r31a = f2f(-0.390180644f), r31b = f2f(-0.390180644f) + f2f(1.501321110f);
        auto add = [](int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); };
        auto sub = [](int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); };
        // even part
        int32_t t2e = dot(r[2], r[6], r00a, r00b), t3e = dot(r[2], r[6], r01a, r01b);
        int32_t t0e = (int32_t)w16(r[0] + r[4]) * 4096, t1e = (int32_t)w16(r[0] - r[4]) * 4096;
        int32_t x0 = add(t0e, t3e), x3 = sub(t0e, t3e), x1 = add(t1e, t2e), x2 = sub(t1e, t2e);
        // odd part
        int32_t y0 = dot(r[7], r[3], r20a, r20b), y2 = dot(r[7], r[3], r21a, r21b);
        int32_t y1 = dot(r[5], r[1], r30a, r30b), y3 = dot(r[5], r[1], r31a, r31b);
        int16_t s17 = w16(r[1] + r[7]), s35 = w16(r[3] + r[5]);
        int32_t y4 = dot(s17, s35, r10a, r10b), y5 = dot(s17, s35, r11a, r11b);
        int32_t x4 = add(y0, y4), x5 = add(y1, y5), x6 = add(y2, y5), x7 = add(y3, y4);
        x0 = add(x0, bias); x1 = add(x1, bias); x2 = add(x2, bias); x3 = add(x3, bias);
        o[0] = add(x0, x7) >> shift; o[7] = sub(x0, x7) >> shift;
        o[1] = add(x1, x6) >> shift; o[6] = sub(x1, x6) >> shift;
        o[2] = add(x2, x5) >> shift; o[5] = sub(x2, x5) >> shift;
        o[3] = add(x3, x4) >> shift; o[4] = sub(x3, x4) >> shift;
    }
    static void idct(const int16_t* d, uint8_t* out, int stride) {
        int16_t mid[64];  // [row][col]
        for (int col = 0; col < 8; ++col) {
            int16_t r[8];
            int32_t o[8];
            for (int k = 0; k < 8; ++k) r[k] = d[k * 8 + col];
            pass1d(r, 512, 10, o);
            for (int k = 0; k < 8; ++k) mid[k * 8 + col] = sat16(o[k]);
        }
        for (int row = 0; row < 8; ++row) {
            int32_t o[8];
            pass1d(&mid[row * 8], 65536 + (128 << 17), 17, o);
            for (int k = 0; k < 8; ++k) {
                int v = sat16(o[k]);
                out[(size_t)row * stride + k] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
            }
        }
    }

    // ---- top level
    bool parse(const uint8_t* data, size_t n) {
        p = data;
        end = data + n;
        if (u8() != 0xFF || u8() != 0xD8) return fail("not a JPEG");
        bool have_frame = false;
        for (;;) {
            // next marker (skipping fill bytes)
            int m;
            if (marker >= 0) {
                m = marker;
                marker = -1;
            } else {
                int b = u8();
                while (b != 0xFF && p < end) b = u8();
                m = u8();
                while (m == 0xFF && p < end) m = u8();
            }
            if (p >= end && m != 0xD9) return have_frame ? finish_eoi() : fail("truncated JPEG");
            if (m == 0xD9) return finish_eoi();
            if (m >= 0xD0 && m <= 0xD7) continue;
            switch (m) {
                case 0xC0: case 0xC1: case 0xC2: {
                    if (have_frame) return fail("multiple frames");
                    progressive = m == 0xC2;
                    if (!read_sof()) return false;
                    have_frame = true;
                    break;
                }
                case 0xC4: if (!read_dht()) return false; break;
                case 0xDB: if (!read_dqt()) return false; break;
                case 0xDD: {
                    if (u16() != 4) return fail("bad DRI");
                    restart_interval = u16();
                    break;
                }
                case 0xDA: {
                    if (!have_frame) return fail("scan before frame");
                    if (!read_sos()) return false;
                    if (!scan()) return false;
                    if (marker < 0) {  // the scan ended without a marker inside the bit stream
                        while (p + 1 < end && !(p[0] == 0xFF && p[1] != 0 && !(p[1] >= 0xD0 && p[1] <= 0xD7))) ++p;
                    }
                    break;
                }
                case 0xE0: {  // APP0: JFIF?
                    int len = u16();
                    const uint8_t* q = p;
                    if (len >= 7 && end - q >= 5 && std::memcmp(q, "JFIF\0", 5) == 0) jfif = true;
                    p = q + std::max(0, len - 2);
                    break;
                }
                case 0xEE: {  // APP14: Adobe colour transform
                    int len = u16();
                    const uint8_t* q = p;
                    if (len >= 14 && end - q >= 12 && std::memcmp(q, "Adobe", 5) == 0) app14 = q[11];
                    p = q + std::max(0, len - 2);
                    break;
                }
                default: {
                    if ((m >= 0xC3 && m <= 0xCF) && m != 0xC4 && m != 0xC8 && m != 0xCC)
                        return fail("unsupported JPEG process (lossless / arithmetic / hierarchical)");
                    int len = u16();
                    p += std::max(0, len - 2);
                    break;
                }
            }
            if (p > end) return fail("truncated JPEG segment");
        }
    }
    bool finish_eoi() {
        if (img_x == 0) return fail("no frame");
        if (progressive) finish_progressive();
        return true;
    }
};

inline uint8_t div4(int x) { return (uint8_t)(x >> 2); }
inline uint8_t div16(int x) { return (uint8_t)(x >> 4); }

// one output row of an upsampled component (near = closer source row, far = the other one)
void upsample_row(uint8_t* out, const uint8_t* near, const uint8_t* far, int w, int hs, int vs) {
    if (hs == 1 && vs == 1) {
        std::memcpy(out, near, w);
    } else if (hs == 1 && vs == 2) {
        for (int i = 0; i < w; ++i) out[i] = div4(3 * near[i] + far[i] + 2);
    } else if (hs == 2 && vs == 1) {
        if (w == 1) { out[0] = out[1] = near[0]; return; }
        out[0] = near[0];
        out[1] = div4(near[0] * 3 + near[1] + 2);
        int i = 1;
        for (; i < w - 1; ++i) {
            int n = 3 * near[i] + 2;
            out[i * 2] = div4(n + near[i - 1]);
            out[i * 2 + 1] = div4(n + near[i + 1]);
        }
        out[i * 2] = div4(near[w - 2] * 3 + near[w - 1] + 2);
        out[i * 2 + 1] = near[w - 1];
    } else if (hs == 2 && vs == 2) {
        if (w == 1) { out[0] = out[1] = div4(3 * near[0] + far[0] + 2); return; }
        int t1 = 3 * near[0] + far[0];
        out[0] = div4(t1 + 2);
        for (int i = 1; i < w; ++i) {
            int t0 = t1;
            t1 = 3 * near[i] + far[i];
            out[i * 2 - 1] = div16(3 * t0 + t1 + 8);
            out[i * 2] = div16(3 * t1 + t0 + 8);
        }
        out[w * 2 - 1] = div4(t1 + 2);
    } else {
        for (int i = 0; i < w; ++i)
            for (int j = 0; j < hs; ++j) out[i * hs + j] = near[i];
    }
}

inline int fixed20(float x) { return ((int)((x * 4096.0f) + 0.5f)) << 8; }

void ycc_to_rgb(uint8_t* out, const uint8_t* y, const uint8_t* cb, const uint8_t* cr, int n) {
    static const int kR = fixed20(1.40200f), kG1 = fixed20(0.71414f), kG2 = fixed20(0.34414f), kB = fixed20(1.77200f);
    for (int i = 0; i < n; ++i) {
        int yf = (y[i] << 20) + (1 << 19);
        int c_r = cr[i] - 128, c_b = cb[i] - 128;
        int r = yf + c_r * kR;
        int g = (int)((uint32_t)(yf + c_r * -kG1) + ((uint32_t)(c_b * -kG2) & 0xffff0000u));
        int b = yf + c_b * kB;
        r >>= 20;
        g >>= 20;
        b >>= 20;
        out[i * 3 + 0] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
        out[i * 3 + 1] = (uint8_t)(g < 0 ? 0 : (g > 255 ? 255 : g));
        out[i * 3 + 2] = (uint8_t)(b < 0 ? 0 : (b > 255 ? 255 : b));
    }
}

}  // namespace

bool decode_jpeg_mem(const uint8_t* data, size_t n, Image8& img, std::string& err) {
    Decoder d;
    if (!d.parse(data, n)) { err = "JPEG: " + d.err; return false; }
    if (d.ncomp == 4) { err = "JPEG: 4-component (CMYK/YCCK) images are not supported"; return false; }
    const int W = d.img_x, H = d.img_y, nc = d.ncomp;
    const int outc = nc >= 3 ? 3 : 1;
    int rgb_ids = 0;
    if (nc == 3)
        for (int i = 0; i < 3; ++i) rgb_ids += d.comp[i].id == "RGB"[i];
    const bool is_rgb = nc == 3 && (rgb_ids == 3 || (d.app14 == 0 && !d.jfif));
    img.width = W;
    img.height = H;
    img.channels = outc;
    img.data.assign((size_t)W * H * outc, 0);
    struct Rs { int hs, vs, ystep, ypos, wl; const uint8_t* l0; const uint8_t* l1; std::vector<uint8_t> buf; };
    Rs rs[3];
    for (int k = 0; k < nc; ++k) {
        Component& c = d.comp[k];
        rs[k].hs = d.hmax / c.h;
        rs[k].vs = d.vmax / c.v;
        rs[k].ystep = rs[k].vs >> 1;
        rs[k].ypos = 0;
        rs[k].wl = (W + rs[k].hs - 1) / rs[k].hs;
        rs[k].l0 = rs[k].l1 = c.plane.data();
        rs[k].buf.assign((size_t)W + 3 + 2 * rs[k].hs, 0);
    }
    std::vector<uint8_t> row((size_t)W * 3);
    for (int j = 0; j < H; ++j) {
        const uint8_t* co[3] = {nullptr, nullptr, nullptr};
        for (int k = 0; k < nc; ++k) {
            Rs& r = rs[k];
            const bool ybot = r.ystep >= (r.vs >> 1);
            upsample_row(r.buf.data(), ybot ? r.l1 : r.l0, ybot ? r.l0 : r.l1, r.wl, r.hs, r.vs);
            co[k] = r.buf.data();
            if (++r.ystep >= r.vs) {
                r.ystep = 0;
                r.l0 = r.l1;
                if (++r.ypos < d.comp[k].y) r.l1 += d.comp[k].w2;
            }
        }
        uint8_t* out = &img.data[(size_t)j * W * outc];
        if (nc == 3) {
            if (is_rgb) {
                for (int i = 0; i < W; ++i) {
                    out[i * 3] = co[0][i];
                    out[i * 3 + 1] = co[1][i];
                    out[i * 3 + 2] = co[2][i];
                }
            } else {
                ycc_to_rgb(out, co[0], co[1], co[2], W);
            }
        } else {
            std::memcpy(out, co[0], W);
        }
    }
    return true;
}

bool decode_jpeg(const std::string& path, Image8& img, std::string& err) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) { err = "cannot read " + path; return false; }
    std::vector<uint8_t> buf;
    std::fseek(f, 0, SEEK_END);
    long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    if (n > 0) {
        buf.resize((size_t)n);
        if (std::fread(buf.data(), 1, (size_t)n, f) != (size_t)n) buf.clear();
    }
    std::fclose(f);
    if (buf.empty()) { err = "cannot read " + path; return false; }
    return decode_jpeg_mem(buf.data(), buf.size(), img, err);
}

}  // namespace rth

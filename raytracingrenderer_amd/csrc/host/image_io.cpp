// image_io.cpp — texture decode and film output for the host front-end.
//
// Semantics follow what RTBase gets from its vendored stb libraries:
//   Texture::load (RTBase/Imaging.h:32-71) uses stbi_loadf for names containing ".hdr" and
//   stbi_load for everything else; Film::save (Imaging.h:262-271) writes RLE RGBE via
//   stbi_write_hdr. The decoders/encoder below are written from the file-format specs
//   (PNG: ISO/IEC 15948; Radiance RGBE) and reproduce stb's conversions where they matter
//   for bits: 16-bit PNG samples keep the high byte, RGBE -> float is mantissa * 2^(e-136),
//   float -> RGBE uses frexp(max)*256/max, and scanline RLE only for 8 <= width < 32768.
#include "image_io.h"

#include <cstdint>

#include <zlib.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace rth {

static bool read_file(const std::string& path, std::vector<uint8_t>& out) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    if (n < 0) { std::fclose(f); return false; }
    out.resize((size_t)n);
    size_t got = n ? std::fread(out.data(), 1, (size_t)n, f) : 0;
    std::fclose(f);
    return got == (size_t)n;
}

static uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

static int paeth(int a, int b, int c) {
    int p = a + b - c;
    int pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    if (pa <= pb && pa <= pc) return a;
    if (pb <= pc) return b;
    return c;
}

bool decode_ldr(const std::string& path, Image8& img, std::string& err) {
    uint8_t head[8] = {};
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) { err = "cannot read " + path; return false; }
    size_t n = std::fread(head, 1, sizeof(head), f);
    std::fclose(f);
    if (n >= 2 && head[0] == 0xFF && head[1] == 0xD8) return decode_jpeg(path, img, err);
    return decode_png(path, img, err);
}

// ---------------------------------------------------------------- PNG (non-interlaced)
bool decode_png(const std::string& path, Image8& img, std::string& err) {
    std::vector<uint8_t> f;
    if (!read_file(path, f)) { err = "cannot read " + path; return false; }
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    if (f.size() < 8 || std::memcmp(f.data(), sig, 8) != 0) { err = "not a PNG: " + path; return false; }
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = 0, interlace = 0;
    std::vector<uint8_t> idat, plte, trns;
    size_t pos = 8;
    while (pos + 8 <= f.size()) {
        uint32_t len = be32(&f[pos]);
        const char* type = (const char*)&f[pos + 4];
        if (pos + 12 + (size_t)len > f.size()) { err = "truncated PNG chunk"; return false; }
        const uint8_t* d = &f[pos + 8];
        if (!std::memcmp(type, "IHDR", 4)) {
            w = be32(d); h = be32(d + 4); depth = d[8]; ctype = d[9]; interlace = d[12];
        } else if (!std::memcmp(type, "PLTE", 4)) {
            plte.assign(d, d + len);
        } else if (!std::memcmp(type, "tRNS", 4)) {
            trns.assign(d, d + len);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            idat.insert(idat.end(), d, d + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            break;
        }
        pos += 12 + len;
    }
    if (!w || !h) { err = "PNG without IHDR"; return false; }
    if (interlace) { err = "interlaced PNG not supported: " + path; return false; }
    int samples = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 3 ? 1 : ctype == 4 ? 2 : ctype == 6 ? 4 : 0;
    // stb_image's size limits (stb_image.h:5109-5126, STBI_MAX_DIMENSIONS = 1 << 24): a header the
    // reference rejects is rejected here before anything is allocated
    if (w > (1u << 24) || h > (1u << 24)) { err = "PNG too large (corrupt?): " + path; return false; }
    if (samples && (1u << 30) / w / (ctype == 3 ? 4u : (unsigned)samples) < h) { err = "PNG too large to decode: " + path; return false; }
    if (!samples || !(depth == 8 || depth == 16 || (depth < 8 && (ctype == 0 || ctype == 3)))) {
        err = "unsupported PNG format in " + path;
        return false;
    }
    size_t bits_pp = (size_t)samples * depth;
    size_t row_bytes = (w * bits_pp + 7) / 8;
    size_t bpp = (bits_pp + 7) / 8;  // filter unit
    std::vector<uint8_t> raw(h * (row_bytes + 1));
    uLongf raw_len = (uLongf)raw.size();
    if (uncompress(raw.data(), &raw_len, idat.data(), (uLong)idat.size()) != Z_OK || raw_len != raw.size()) {
        err = "PNG inflate failed: " + path;
        return false;
    }
    std::vector<uint8_t> px(h * row_bytes);
    for (uint32_t y = 0; y < h; ++y) {
        const uint8_t* src = &raw[y * (row_bytes + 1)];
        uint8_t* cur = &px[y * row_bytes];
        const uint8_t* prev = y ? &px[(y - 1) * row_bytes] : nullptr;
        int ft = src[0];
        ++src;
        for (size_t i = 0; i < row_bytes; ++i) {
            int a = i >= bpp ? cur[i - bpp] : 0, b = prev ? prev[i] : 0, c = (prev && i >= bpp) ? prev[i - bpp] : 0;
            int v = src[i];
            switch (ft) {
            case 0: break;
            case 1: v += a; break;
            case 2: v += b; break;
            case 3: v += (a + b) >> 1; break;
            case 4: v += paeth(a, b, c); break;
            default: err = "bad PNG filter"; return false;
            }
            cur[i] = (uint8_t)v;
        }
    }
    // expand to 8-bit channels like stbi_load(req_comp = 0)
    int out_n = samples;
    if (ctype == 3) out_n = trns.empty() ? 3 : 4;
    img.width = (int)w;
    img.height = (int)h;
    img.channels = out_n;
    img.data.assign((size_t)w * h * out_n, 0);
    for (uint32_t y = 0; y < h; ++y) {
        const uint8_t* row = &px[y * row_bytes];
        for (uint32_t x = 0; x < w; ++x) {
            uint8_t* o = &img.data[((size_t)y * w + x) * out_n];
            if (ctype == 3) {
                int idx;
                if (depth == 8) idx = row[x];
                else { int per = 8 / depth; idx = (row[x / per] >> ((per - 1 - x % per) * depth)) & ((1 << depth) - 1); }
                for (int c = 0; c < 3; ++c) o[c] = (size_t)idx * 3 + c < plte.size() ? plte[idx * 3 + c] : 0;
                if (out_n == 4) o[3] = (size_t)idx < trns.size() ? trns[idx] : 255;
            } else if (depth == 8) {
                std::memcpy(o, row + (size_t)x * samples, samples);
            } else if (depth == 16) {
                for (int c = 0; c < samples; ++c) o[c] = row[((size_t)x * samples + c) * 2];  // high byte
            } else {  // 1/2/4-bit grey, scaled to 0..255 like stb
                int per = 8 / depth;
                int v = (row[x / per] >> ((per - 1 - x % per) * depth)) & ((1 << depth) - 1);
                int scale = depth == 1 ? 0xff : depth == 2 ? 0x55 : 0x11;
                o[0] = (uint8_t)(v * scale);
            }
        }
    }
    return true;
}

static void put_be32(std::vector<uint8_t>& v, uint32_t x) {
    v.push_back(x >> 24); v.push_back(x >> 16); v.push_back(x >> 8); v.push_back(x);
}
static void png_chunk(std::vector<uint8_t>& out, const char* type, const std::vector<uint8_t>& data) {
    put_be32(out, (uint32_t)data.size());
    size_t start = out.size();
    out.insert(out.end(), type, type + 4);
    out.insert(out.end(), data.begin(), data.end());
    uLong crc = crc32(0L, out.data() + start, (uInt)(out.size() - start));
    put_be32(out, (uint32_t)crc);
}

bool encode_png(const std::string& path, int w, int h, int channels, const uint8_t* rgb, std::string& err) {
    if (channels != 3 && channels != 4) { err = "encode_png: 3 or 4 channels"; return false; }
    std::vector<uint8_t> raw;
    for (int y = 0; y < h; ++y) {
        raw.push_back(0);
        raw.insert(raw.end(), rgb + (size_t)y * w * channels, rgb + (size_t)(y + 1) * w * channels);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 9) != Z_OK) { err = "deflate failed"; return false; }
    z.resize(zlen);
    std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::vector<uint8_t> ihdr;
    put_be32(ihdr, (uint32_t)w); put_be32(ihdr, (uint32_t)h);
    ihdr.push_back(8); ihdr.push_back(channels == 3 ? 2 : 6); ihdr.push_back(0); ihdr.push_back(0); ihdr.push_back(0);
    png_chunk(out, "IHDR", ihdr);
    png_chunk(out, "IDAT", z);
    png_chunk(out, "IEND", {});
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) { err = "cannot write " + path; return false; }
    bool ok = std::fwrite(out.data(), 1, out.size(), f) == out.size();
    std::fclose(f);
    return ok;
}

// ---------------------------------------------------------------- Radiance RGBE
static inline void rgbe_to_float(const uint8_t* e, float* o) {
    if (e[3] != 0) {
        float f1 = (float)std::ldexp(1.0f, e[3] - (int)(128 + 8));
        o[0] = e[0] * f1;
        o[1] = e[1] * f1;
        o[2] = e[2] * f1;
    } else {
        o[0] = o[1] = o[2] = 0;
    }
}

bool decode_hdr(const std::string& path, ImageF& img, std::string& err) {
    std::vector<uint8_t> f;
    if (!read_file(path, f)) { err = "cannot read " + path; return false; }
    size_t pos = 0;
    auto line = [&](std::string& s) {
        s.clear();
        while (pos < f.size() && f[pos] != '\n') s.push_back((char)f[pos++]);
        if (pos < f.size()) ++pos;
    };
    std::string s;
    line(s);
    if (s != "#?RADIANCE" && s != "#?RGBE") { err = "not a Radiance file: " + path; return false; }
    bool fmt_ok = false;
    for (;;) {
        line(s);
        if (s.empty()) break;
        if (s == "FORMAT=32-bit_rle_rgbe") fmt_ok = true;
        if (pos >= f.size()) break;
    }
    if (!fmt_ok) { err = "unsupported HDR format in " + path; return false; }
    line(s);
    int h = 0, w = 0;
    if (std::sscanf(s.c_str(), "-Y %d +X %d", &h, &w) != 2 || w <= 0 || h <= 0) {
        err = "unsupported HDR orientation in " + path;
        return false;
    }
    // stb_image's limits (stb_image.h:7197-7207): dimensions <= 1 << 24, w * h * 3 floats < 2^31 B
    if (w > (1 << 24) || h > (1 << 24) || (uint64_t)w * (uint64_t)h * 12u > (uint64_t)INT32_MAX) {
        err = "HDR image too large: " + path;
        return false;
    }
    img.width = w;
    img.height = h;
    img.data.assign((size_t)w * h * 3, 0.0f);
    auto flat = [&](size_t from_pixel) -> bool {
        for (size_t i = from_pixel; i < (size_t)w * h; ++i) {
            if (pos + 4 > f.size()) { err = "truncated HDR"; return false; }
            rgbe_to_float(&f[pos], &img.data[i * 3]);
            pos += 4;
        }
        return true;
    };
    if (w < 8 || w >= 32768) return flat(0);
    std::vector<uint8_t> line_buf((size_t)w * 4);
    for (int y = 0; y < h; ++y) {
        if (pos + 4 > f.size()) { err = "truncated HDR"; return false; }
        uint8_t c1 = f[pos], c2 = f[pos + 1], len_hi = f[pos + 2];
        if (c1 != 2 || c2 != 2 || (len_hi & 0x80)) return flat((size_t)y * w);  // old-style: flat from here
        int len = (f[pos + 2] << 8) | f[pos + 3];
        if (len != w) { err = "invalid RLE scanline width"; return false; }
        pos += 4;
        for (int k = 0; k < 4; ++k) {
            int x = 0;
            while (x < w) {
                if (pos >= f.size()) { err = "truncated HDR"; return false; }
                int count = f[pos++];
                if (count > 128) {
                    count -= 128;
                    if (pos >= f.size() || x + count > w) { err = "bad RLE run"; return false; }
                    uint8_t v = f[pos++];
                    for (int i = 0; i < count; ++i) line_buf[(size_t)(x++) * 4 + k] = v;
                } else {
                    if (count == 0 || x + count > w || pos + count > f.size()) { err = "bad RLE dump"; return false; }
                    for (int i = 0; i < count; ++i) line_buf[(size_t)(x++) * 4 + k] = f[pos++];
                }
            }
        }
        for (int x = 0; x < w; ++x) rgbe_to_float(&line_buf[(size_t)x * 4], &img.data[((size_t)y * w + x) * 3]);
    }
    return true;
}

static inline void float_to_rgbe(const float* lin, uint8_t* e) {
    float m = lin[1] > lin[2] ? lin[1] : lin[2];
    m = lin[0] > m ? lin[0] : m;
    if (m < 1e-32f) {
        e[0] = e[1] = e[2] = e[3] = 0;
        return;
    }
    int ex;
    float scale = (float)std::frexp(m, &ex) * 256.0f / m;
    e[0] = (uint8_t)(lin[0] * scale);
    e[1] = (uint8_t)(lin[1] * scale);
    e[2] = (uint8_t)(lin[2] * scale);
    e[3] = (uint8_t)(ex + 128);
}

// One component plane of one scanline, RLE-coded: literal dumps of <=128 bytes, runs (>=3 equal
// bytes) of <=127.
static void rle_plane(std::vector<uint8_t>& out, const uint8_t* c, int w) {
    int x = 0;
    while (x < w) {
        int r = x;
        while (r + 2 < w && !(c[r] == c[r + 1] && c[r] == c[r + 2])) ++r;
        bool has_run = r + 2 < w;
        if (!has_run) r = w;
        while (x < r) {
            int n = r - x < 128 ? r - x : 128;
            out.push_back((uint8_t)n);
            out.insert(out.end(), c + x, c + x + n);
            x += n;
        }
        if (has_run) {
            while (r < w && c[r] == c[x]) ++r;
            while (x < r) {
                int n = r - x < 127 ? r - x : 127;
                out.push_back((uint8_t)(n + 128));
                out.push_back(c[x]);
                x += n;
            }
        }
    }
}

bool encode_hdr(const std::string& path, int w, int h, const float* rgb, std::string& err) {
    if (w <= 0 || h <= 0 || !rgb) { err = "encode_hdr: empty image"; return false; }
    std::vector<uint8_t> out;
    const char* head = "#?RADIANCE\n# Written by stb_image_write.h\nFORMAT=32-bit_rle_rgbe\n";
    out.insert(out.end(), head, head + std::strlen(head));
    char buf[128];
    int n = std::snprintf(buf, sizeof(buf), "EXPOSURE=          1.0000000000000\n\n-Y %d +X %d\n", h, w);
    out.insert(out.end(), buf, buf + n);
    std::vector<uint8_t> planes((size_t)w * 4);
    for (int y = 0; y < h; ++y) {
        const float* row = rgb + (size_t)y * w * 3;
        if (w < 8 || w >= 32768) {
            for (int x = 0; x < w; ++x) {
                uint8_t e[4];
                float_to_rgbe(row + (size_t)x * 3, e);
                out.insert(out.end(), e, e + 4);
            }
            continue;
        }
        for (int x = 0; x < w; ++x) {
            uint8_t e[4];
            float_to_rgbe(row + (size_t)x * 3, e);
            for (int k = 0; k < 4; ++k) planes[(size_t)k * w + x] = e[k];
        }
        out.push_back(2); out.push_back(2); out.push_back((uint8_t)((w >> 8) & 0xff)); out.push_back((uint8_t)(w & 0xff));
        for (int k = 0; k < 4; ++k) rle_plane(out, &planes[(size_t)k * w], w);
    }
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) { err = "cannot write " + path; return false; }
    bool ok = std::fwrite(out.data(), 1, out.size(), f) == out.size();
    std::fclose(f);
    return ok;
}

}  // namespace rth

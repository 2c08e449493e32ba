// png_io.cpp — see png_io.h.  PNG (ISO/IEC 15948) chunk parsing, zlib inflate,
// scanline unfiltering (None/Sub/Up/Average/Paeth), Adam7, sample expansion.
#include "png_io.h"

#include <zlib.h>

#include <cstdio>
#include <cstring>

namespace asw_host {
namespace {

const uint8_t kSig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};

uint32_t be32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
void put32(std::vector<uint8_t> &v, uint32_t x) {
    v.push_back((uint8_t)(x >> 24));
    v.push_back((uint8_t)(x >> 16));
    v.push_back((uint8_t)(x >> 8));
    v.push_back((uint8_t)x);
}

int paeth(int a, int b, int c) {
    const int p = a + b - c;
    const int pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p, pc = p > c ? p - c : c - p;
    if (pa <= pb && pa <= pc) return a;
    return pb <= pc ? b : c;
}

// Reverses the filter of one scanline in place; prev = previous unfiltered line or null.
bool unfilter(uint8_t type, uint8_t *cur, const uint8_t *prev, size_t len, size_t bpp) {
    switch (type) {
        case 0:
            return true;
        case 1:
            for (size_t i = bpp; i < len; ++i) cur[i] = (uint8_t)(cur[i] + cur[i - bpp]);
            return true;
        case 2:
            if (prev)
                for (size_t i = 0; i < len; ++i) cur[i] = (uint8_t)(cur[i] + prev[i]);
            return true;
        case 3:
            for (size_t i = 0; i < len; ++i) {
                const int a = i >= bpp ? cur[i - bpp] : 0, b = prev ? prev[i] : 0;
                cur[i] = (uint8_t)(cur[i] + ((a + b) >> 1));
            }
            return true;
        case 4:
            for (size_t i = 0; i < len; ++i) {
                const int a = i >= bpp ? cur[i - bpp] : 0, b = prev ? prev[i] : 0;
                const int c = (prev && i >= bpp) ? prev[i - bpp] : 0;
                cur[i] = (uint8_t)(cur[i] + paeth(a, b, c));
            }
            return true;
        default:
            return false;
    }
}

struct Header {
    unsigned w, h;
    int depth, ctype, interlace;
    int channels() const { return ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 3 ? 1 : ctype == 4 ? 2 : 4; }
    size_t bits_pp() const { return (size_t)channels() * depth; }
};

// sample j of an unfiltered row (any depth), as an integer of `depth` bits
unsigned sample(const uint8_t *row, size_t j, int depth) {
    if (depth == 8) return row[j];
    if (depth == 16) return (unsigned)row[2 * j] << 8 | row[2 * j + 1];
    const size_t bit = j * depth;
    const unsigned byte = row[bit >> 3];
    const int shift = 8 - depth - (int)(bit & 7);
    return (byte >> shift) & ((1u << depth) - 1);
}

uint8_t to8(unsigned v, int depth) {
    if (depth == 16) return (uint8_t)(v >> 8);
    if (depth == 8) return (uint8_t)v;
    return (uint8_t)(v * 255u / ((1u << depth) - 1));  // 1/2/4-bit grey: exact scaling
}

}  // namespace

std::string png_decode(const std::vector<uint8_t> &f, Image &out) {
    out = Image{};
    if (f.size() < 8 || std::memcmp(f.data(), kSig, 8) != 0) return "not a PNG file";
    Header hd{};
    bool have_hdr = false;
    std::vector<uint8_t> idat, plte, trns;
    size_t pos = 8;
    bool end = false;
    while (!end) {
        if (pos + 12 > f.size()) return "truncated chunk";
        const uint32_t len = be32(&f[pos]);
        if (len > f.size() - pos - 12) return "chunk length out of range";
        const char *type = reinterpret_cast<const char *>(&f[pos + 4]);
        const uint8_t *data = &f[pos + 8];
        const uint32_t crc = be32(&f[pos + 8 + len]);
        if ((uint32_t)crc32(0, reinterpret_cast<const Bytef *>(type), 4 + len) != crc) return "CRC mismatch";
        if (!std::memcmp(type, "IHDR", 4)) {
            if (len != 13) return "bad IHDR";
            hd.w = be32(data);
            hd.h = be32(data + 4);
            hd.depth = data[8];
            hd.ctype = data[9];
            hd.interlace = data[12];
            if (data[10] != 0 || data[11] != 0 || hd.interlace > 1) return "unsupported compression/filter/interlace";
            const int d = hd.depth, c = hd.ctype;
            const bool ok = (c == 0 && (d == 1 || d == 2 || d == 4 || d == 8 || d == 16)) ||
                            (c == 3 && (d == 1 || d == 2 || d == 4 || d == 8)) ||
                            ((c == 2 || c == 4 || c == 6) && (d == 8 || d == 16));
            if (!ok) return "invalid colour type / bit depth";
            if (hd.w == 0 || hd.h == 0 || hd.w > (1u << 16) || hd.h > (1u << 16)) return "image size out of range";
            have_hdr = true;
        } else if (!std::memcmp(type, "PLTE", 4)) {
            plte.assign(data, data + len);
        } else if (!std::memcmp(type, "tRNS", 4)) {
            trns.assign(data, data + len);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            idat.insert(idat.end(), data, data + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            end = true;
        } else if (!(type[0] & 0x20)) {
            return std::string("unknown critical chunk ") + std::string(type, 4);
        }
        pos += 12 + len;
    }
    if (!have_hdr) return "missing IHDR";
    if (hd.ctype == 3 && (plte.empty() || plte.size() % 3)) return "missing PLTE";

    // pass geometry (Adam7 or one pass)
    struct Pass {
        unsigned x0, y0, dx, dy;
    };
    const Pass adam7[7] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4}, {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};
    const Pass single = {0, 0, 1, 1};
    const int npass = hd.interlace ? 7 : 1;
    size_t raw_size = 0;
    for (int k = 0; k < npass; ++k) {
        const Pass &ps = hd.interlace ? adam7[k] : single;
        const size_t pw = hd.w > ps.x0 ? (hd.w - ps.x0 + ps.dx - 1) / ps.dx : 0;
        const size_t ph = hd.h > ps.y0 ? (hd.h - ps.y0 + ps.dy - 1) / ps.dy : 0;
        if (pw && ph) raw_size += ph * (1 + (pw * hd.bits_pp() + 7) / 8);
    }
    std::vector<uint8_t> raw(raw_size);
    {
        z_stream zs{};
        if (inflateInit(&zs) != Z_OK) return "inflateInit failed";
        zs.next_in = idat.data();
        zs.avail_in = (uInt)idat.size();
        zs.next_out = raw.data();
        zs.avail_out = (uInt)raw.size();
        const int r = inflate(&zs, Z_FINISH);
        const size_t got = raw.size() - zs.avail_out;
        inflateEnd(&zs);
        if ((r != Z_STREAM_END && r != Z_BUF_ERROR) || got != raw.size()) return "corrupt image data (zlib)";
    }

    out.width = hd.w;
    out.height = hd.h;
    out.rgba.assign((size_t)hd.w * hd.h * 4, 255);
    const size_t bpp = (hd.bits_pp() + 7) / 8;
    size_t off = 0;
    for (int k = 0; k < npass; ++k) {
        const Pass &ps = hd.interlace ? adam7[k] : single;
        const size_t pw = hd.w > ps.x0 ? (hd.w - ps.x0 + ps.dx - 1) / ps.dx : 0;
        const size_t ph = hd.h > ps.y0 ? (hd.h - ps.y0 + ps.dy - 1) / ps.dy : 0;
        if (!pw || !ph) continue;
        const size_t stride = (pw * hd.bits_pp() + 7) / 8;
        const uint8_t *prev = nullptr;
        for (size_t r = 0; r < ph; ++r) {
            uint8_t *line = &raw[off + r * (stride + 1)];
            if (!unfilter(line[0], line + 1, prev, stride, bpp)) {
                out = Image{};
                return "bad filter type";
            }
            const uint8_t *row = line + 1;
            prev = row;
            const size_t y = ps.y0 + r * ps.dy;
            for (size_t j = 0; j < pw; ++j) {
                uint8_t *o = &out.rgba[(y * hd.w + ps.x0 + j * ps.dx) * 4];
                const int d = hd.depth;
                switch (hd.ctype) {
                    case 0: {
                        const unsigned g = sample(row, j, d);
                        o[0] = o[1] = o[2] = to8(g, d);
                        if (trns.size() >= 2 && g == ((unsigned)trns[0] << 8 | trns[1])) o[3] = 0;
                        break;
                    }
                    case 2: {
                        unsigned c[3];
                        for (int ch = 0; ch < 3; ++ch) {
                            c[ch] = sample(row, j * 3 + ch, d);
                            o[ch] = to8(c[ch], d);
                        }
                        if (trns.size() >= 6 && c[0] == ((unsigned)trns[0] << 8 | trns[1]) &&
                            c[1] == ((unsigned)trns[2] << 8 | trns[3]) && c[2] == ((unsigned)trns[4] << 8 | trns[5]))
                            o[3] = 0;
                        break;
                    }
                    case 3: {
                        const unsigned i = sample(row, j, d);
                        if (3 * i + 2 >= plte.size()) {
                            out = Image{};
                            return "palette index out of range";
                        }
                        o[0] = plte[3 * i];
                        o[1] = plte[3 * i + 1];
                        o[2] = plte[3 * i + 2];
                        o[3] = i < trns.size() ? trns[i] : 255;
                        break;
                    }
                    case 4:
                        o[0] = o[1] = o[2] = to8(sample(row, j * 2, d), d);
                        o[3] = to8(sample(row, j * 2 + 1, d), d);
                        break;
                    default:
                        for (int ch = 0; ch < 4; ++ch) o[ch] = to8(sample(row, j * 4 + ch, d), d);
                }
            }
        }
        off += ph * (stride + 1);
    }
    return {};
}

std::string png_load(const std::string &path, Image &out) {
    FILE *fp = std::fopen(path.c_str(), "rb");
    if (!fp) return "cannot open " + path;
    std::vector<uint8_t> buf;
    uint8_t tmp[1 << 16];
    size_t n;
    while ((n = std::fread(tmp, 1, sizeof tmp, fp)) > 0) buf.insert(buf.end(), tmp, tmp + n);
    std::fclose(fp);
    const std::string e = png_decode(buf, out);
    return e.empty() ? e : path + ": " + e;
}

namespace {
// rows of bytes, `channels` = bytes per pixel (the filter's left neighbour
// distance), colour type `ctype` at bit depth `depth`
std::string encode_bytes(const uint8_t *data, unsigned w, unsigned h, int channels, int ctype, int depth,
                         std::vector<uint8_t> &out) {
    const size_t stride = (size_t)w * channels;
    // per row: the filter (None or Paeth) with the smaller sum of |signed residuals|
    std::vector<uint8_t> raw(h * (stride + 1));
    std::vector<uint8_t> paeth_row(stride);
    for (unsigned y = 0; y < h; ++y) {
        const uint8_t *cur = data + y * stride, *prev = y ? data + (y - 1) * stride : nullptr;
        long s_none = 0, s_paeth = 0;
        for (size_t i = 0; i < stride; ++i) {
            const int a = i >= (size_t)channels ? cur[i - channels] : 0, b = prev ? prev[i] : 0;
            const int c = (prev && i >= (size_t)channels) ? prev[i - channels] : 0;
            paeth_row[i] = (uint8_t)(cur[i] - paeth(a, b, c));
            s_none += cur[i] < 128 ? cur[i] : 256 - cur[i];
            s_paeth += paeth_row[i] < 128 ? paeth_row[i] : 256 - paeth_row[i];
        }
        uint8_t *dst = &raw[y * (stride + 1)];
        if (s_paeth < s_none) {
            dst[0] = 4;
            std::memcpy(dst + 1, paeth_row.data(), stride);
        } else {
            dst[0] = 0;
            std::memcpy(dst + 1, cur, stride);
        }
    }
    uLongf zlen = compressBound(raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), raw.size(), 6) != Z_OK) return "zlib compress failed";
    z.resize(zlen);

    out.assign(kSig, kSig + 8);
    auto chunk = [&](const char *type, const uint8_t *d, size_t n) {
        put32(out, (uint32_t)n);
        const size_t at = out.size();
        out.insert(out.end(), type, type + 4);
        if (n) out.insert(out.end(), d, d + n);
        put32(out, (uint32_t)crc32(0, &out[at], (uInt)(4 + n)));
    };
    uint8_t ihdr[13];
    const uint32_t ww = w, hh = h;
    for (int i = 0; i < 4; ++i) {
        ihdr[i] = (uint8_t)(ww >> (24 - 8 * i));
        ihdr[4 + i] = (uint8_t)(hh >> (24 - 8 * i));
    }
    ihdr[8] = (uint8_t)depth;
    ihdr[9] = (uint8_t)ctype;
    ihdr[10] = ihdr[11] = ihdr[12] = 0;
    chunk("IHDR", ihdr, 13);
    chunk("IDAT", z.data(), z.size());
    chunk("IEND", nullptr, 0);
    return {};
}
}  // namespace

std::string png_encode(const uint8_t *data, unsigned w, unsigned h, int channels, std::vector<uint8_t> &out) {
    if (!data || !w || !h || (channels != 1 && channels != 4)) return "bad image";
    return encode_bytes(data, w, h, channels, channels == 4 ? 6 : 0, 8, out);
}

std::string png_encode16(const uint16_t *data, unsigned w, unsigned h, std::vector<uint8_t> &out) {
    if (!data || !w || !h) return "bad image";
    std::vector<uint8_t> be((size_t)w * h * 2);  // PNG samples are big-endian
    for (size_t i = 0; i < (size_t)w * h; ++i) {
        be[2 * i] = (uint8_t)(data[i] >> 8);
        be[2 * i + 1] = (uint8_t)(data[i] & 255);
    }
    return encode_bytes(be.data(), w, h, 2, 0, 16, out);
}

std::string png_save16(const std::string &path, const uint16_t *data, unsigned w, unsigned h) {
    std::vector<uint8_t> buf;
    std::string e = png_encode16(data, w, h, buf);
    if (!e.empty()) return e;
    FILE *fp = std::fopen(path.c_str(), "wb");
    if (!fp) return "cannot write " + path;
    const bool ok = std::fwrite(buf.data(), 1, buf.size(), fp) == buf.size();
    std::fclose(fp);
    return ok ? std::string() : "short write " + path;
}

std::string png_save(const std::string &path, const uint8_t *data, unsigned w, unsigned h, int channels) {
    std::vector<uint8_t> buf;
    std::string e = png_encode(data, w, h, channels, buf);
    if (!e.empty()) return e;
    FILE *fp = std::fopen(path.c_str(), "wb");
    if (!fp) return "cannot write " + path;
    const bool ok = std::fwrite(buf.data(), 1, buf.size(), fp) == buf.size();
    std::fclose(fp);
    return ok ? std::string() : "short write " + path;
}

}  // namespace asw_host

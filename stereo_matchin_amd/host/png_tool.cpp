// png_tool — exercises png_io from the CPU tests (tests/test_host.py):
//   png_tool decode IN.png OUT.raw   -> "W H" on stdout, RGBA8 bytes to OUT.raw
//   png_tool encode IN.raw W H C OUT.png   (C = 1 grey8 or 4 RGBA8)
//   png_tool encode16 IN.raw W H OUT.png   (host-order uint16 grey)
//   png_tool fuzz SEED.png N S            -> decodes N mutants of SEED.png (seed S);
//     run under the sanitizer build (make ASAN=1) a decoder bug aborts the process
#include <zlib.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "png_io.h"

namespace {

// splitmix64: the fuzzer's only randomness (reproducible from the seed)
struct Rng {
    uint64_t s;
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return z ^ (z >> 31);
    }
    uint32_t below(uint32_t n) { return n ? (uint32_t)(next() % n) : 0; }
};

struct Chunk {
    std::string type;
    std::vector<uint8_t> data;
};

uint32_t rd32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
void wr32(std::vector<uint8_t> &v, uint32_t x) {
    for (int k = 3; k >= 0; --k) v.push_back((uint8_t)(x >> (8 * k)));
}

std::vector<Chunk> split(const std::vector<uint8_t> &f) {
    std::vector<Chunk> out;
    size_t p = 8;
    while (p + 12 <= f.size()) {
        const uint32_t n = rd32(&f[p]);
        if (n > f.size() - p - 12) break;
        out.push_back({std::string(reinterpret_cast<const char *>(&f[p + 4]), 4),
                       std::vector<uint8_t>(f.begin() + (long)p + 8, f.begin() + (long)p + 8 + n)});
        p += 12 + n;
    }
    return out;
}

std::vector<uint8_t> join(const std::vector<Chunk> &cs, bool fix_crc, Rng &rng) {
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::vector<uint8_t> f(sig, sig + 8);
    for (const Chunk &c : cs) {
        wr32(f, (uint32_t)c.data.size());
        const size_t t0 = f.size();
        f.insert(f.end(), c.type.begin(), c.type.end());
        f.insert(f.end(), c.data.begin(), c.data.end());
        uint32_t crc = (uint32_t)crc32(0, &f[t0], (uInt)(f.size() - t0));
        if (!fix_crc && rng.below(2)) crc ^= 1u << rng.below(32);
        wr32(f, crc);
    }
    return f;
}

// one mutant of the seed file: structured edits of IHDR / PLTE / tRNS / IDAT (CRCs
// recomputed so the decoder gets past the chunk layer), raw byte flips, truncation
std::vector<uint8_t> mutate(const std::vector<uint8_t> &seed, Rng &rng) {
    std::vector<Chunk> cs = split(seed);
    const int edits = 1 + (int)rng.below(4);
    for (int e = 0; e < edits && !cs.empty(); ++e) {
        Chunk &c = cs[rng.below((uint32_t)cs.size())];
        switch (rng.below(9)) {
            case 0:  // IHDR field: width / height / depth / colour type / interlace
                if (c.type == "IHDR" && c.data.size() == 13) {
                    const uint32_t k = rng.below(7);
                    if (k < 2) {
                        const uint32_t v = rng.below(4) == 0 ? (uint32_t)rng.next() : rng.below(70);
                        for (int b = 0; b < 4; ++b) c.data[4 * k + b] = (uint8_t)(v >> (24 - 8 * b));
                    } else {
                        c.data[8 + (k - 2)] = (uint8_t)(rng.below(3) ? rng.below(17) : rng.next());
                    }
                }
                break;
            case 1:  // chunk data byte flips
                for (int k = 0, n = 1 + (int)rng.below(8); k < n && !c.data.empty(); ++k)
                    c.data[rng.below((uint32_t)c.data.size())] ^= (uint8_t)(1 + rng.below(255));
                break;
            case 2: {  // resize a chunk (PLTE / tRNS / IDAT lengths off by a little or a lot)
                const long n = (long)c.data.size();
                const long m = rng.below(3) ? n + (long)rng.below(9) - 4 : (long)rng.below(1024);
                c.data.resize(m < 0 ? 0 : (size_t)m);
                break;
            }
            case 3: {  // IDAT = zlib of random scanline bytes (bad filter types, short / long rows)
                if (c.type != "IDAT") break;
                std::vector<uint8_t> raw(rng.below(4096));
                for (uint8_t &b : raw) b = (uint8_t)(rng.below(4) ? rng.below(6) : rng.next());
                uLongf n = compressBound((uLong)raw.size());
                std::vector<uint8_t> z(n);
                if (compress(z.data(), &n, raw.data(), (uLong)raw.size()) == Z_OK) {
                    z.resize(n);
                    c.data = z;
                }
                break;
            }
            case 4:  // drop a chunk
                if (cs.size() > 1) cs.erase(cs.begin() + rng.below((uint32_t)cs.size()));
                break;
            case 5:  // duplicate a chunk (second IHDR / PLTE, split IDAT)
                cs.insert(cs.begin() + rng.below((uint32_t)cs.size() + 1), c);
                break;
            case 6:  // swap two chunks (PLTE after IDAT, IEND first ...)
                std::swap(c, cs[rng.below((uint32_t)cs.size())]);
                break;
            case 7:  // rename a chunk type
                if (!c.type.empty()) c.type[rng.below(4)] ^= (char)(1 + rng.below(63));
                break;
            default:  // truncate the zlib stream
                if (!c.data.empty()) c.data.resize(rng.below((uint32_t)c.data.size()));
                break;
        }
    }
    std::vector<uint8_t> f = join(cs, rng.below(8) != 0, rng);
    if (rng.below(8) == 0 && !f.empty()) f.resize(rng.below((uint32_t)f.size()));        // file truncation
    if (rng.below(8) == 0)
        for (int k = 0; k < 4 && !f.empty(); ++k) f[rng.below((uint32_t)f.size())] ^= 0xFF;  // raw flips
    return f;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc == 5 && !std::strcmp(argv[1], "fuzz")) {
        FILE *f = std::fopen(argv[2], "rb");
        if (!f) return 1;
        std::vector<uint8_t> seed;
        for (int c; (c = std::fgetc(f)) != EOF;) seed.push_back((uint8_t)c);
        std::fclose(f);
        const long n = std::atol(argv[3]);
        Rng rng{(uint64_t)std::atoll(argv[4])};
        long ok = 0;
        for (long i = 0; i < n; ++i) {
            asw_host::Image im;
            if (asw_host::png_decode(mutate(seed, rng), im).empty()) {
                ++ok;
                if (im.rgba.size() != (size_t)im.width * im.height * 4) return 3;  // inconsistent success
            }
        }
        std::printf("%ld %ld\n", n, ok);  // mutants, decoded without error
        return 0;
    }
    if (argc == 4 && !std::strcmp(argv[1], "decode")) {
        asw_host::Image im;
        const std::string e = asw_host::png_load(argv[2], im);
        if (!e.empty()) {
            std::fprintf(stderr, "%s\n", e.c_str());
            return 1;
        }
        FILE *f = std::fopen(argv[3], "wb");
        if (!f) return 1;
        std::fwrite(im.rgba.data(), 1, im.rgba.size(), f);
        std::fclose(f);
        std::printf("%u %u\n", im.width, im.height);
        return 0;
    }
    if (argc == 7 && !std::strcmp(argv[1], "encode")) {
        const unsigned w = (unsigned)std::atoi(argv[3]), h = (unsigned)std::atoi(argv[4]);
        const int c = std::atoi(argv[5]);
        std::vector<uint8_t> buf((size_t)w * h * c);
        FILE *f = std::fopen(argv[2], "rb");
        if (!f || std::fread(buf.data(), 1, buf.size(), f) != buf.size()) return 1;
        std::fclose(f);
        const std::string e = asw_host::png_save(argv[6], buf.data(), w, h, c);
        if (!e.empty()) {
            std::fprintf(stderr, "%s\n", e.c_str());
            return 1;
        }
        return 0;
    }
    if (argc == 6 && !std::strcmp(argv[1], "encode16")) {
        const unsigned w = (unsigned)std::atoi(argv[3]), h = (unsigned)std::atoi(argv[4]);
        std::vector<uint16_t> buf((size_t)w * h);
        FILE *f = std::fopen(argv[2], "rb");
        if (!f || std::fread(buf.data(), 2, buf.size(), f) != buf.size()) return 1;
        std::fclose(f);
        const std::string e = asw_host::png_save16(argv[5], buf.data(), w, h);
        if (!e.empty()) {
            std::fprintf(stderr, "%s\n", e.c_str());
            return 1;
        }
        return 0;
    }
    std::fprintf(stderr, "usage: png_tool decode IN.png OUT.raw | encode IN.raw W H C OUT.png | encode16 IN.raw W H OUT.png\n");
    return 2;
}

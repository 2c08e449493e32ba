// png_tool — exercises png_io from the CPU tests (tests/test_host.py):
//   png_tool decode IN.png OUT.raw   -> "W H" on stdout, RGBA8 bytes to OUT.raw
//   png_tool encode IN.raw W H C OUT.png   (C = 1 grey8 or 4 RGBA8)
//   png_tool encode16 IN.raw W H OUT.png   (host-order uint16 grey)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "png_io.h"

int main(int argc, char **argv) {
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

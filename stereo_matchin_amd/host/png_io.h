// png_io.h — minimal PNG reader/writer for the ASW host driver.
//
// The reference host decodes its inputs with lodepng::decode into RGBA8 and
// writes its outputs with lodepng::encode (stereo_matching/main.cpp:183-186,
// 621-631).  This is an independent implementation over zlib, sized to what the
// driver needs: every non-interlaced and Adam7 PNG of colour types 0/2/3/4/6 at
// bit depths 1-16 decodes to RGBA8 (16-bit samples keep their high byte, tRNS
// honoured); RGBA8, grey8 and grey16 images encode with a per-row filter choice.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace asw_host {

struct Image {
    unsigned width = 0, height = 0;
    std::vector<uint8_t> rgba;  // [height][width][4]
};

// Returns an empty string on success, else a message (the image is then empty).
std::string png_decode(const std::vector<uint8_t> &file, Image &out);
std::string png_load(const std::string &path, Image &out);

// channels = 4 (RGBA8) or 1 (grey8); data is [h][w][channels].
std::string png_encode(const uint8_t *data, unsigned w, unsigned h, int channels, std::vector<uint8_t> &out);
std::string png_save(const std::string &path, const uint8_t *data, unsigned w, unsigned h, int channels);
// 16-bit grey (colour type 0, depth 16): disparity maps past 256 levels
std::string png_encode16(const uint16_t *data, unsigned w, unsigned h, std::vector<uint8_t> &out);
std::string png_save16(const std::string &path, const uint16_t *data, unsigned w, unsigned h);

}  // namespace asw_host

// png_io.h -- 8-bit RGB PNG encode/decode (zlib).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace ipt {
bool png_write_rgb8(const std::string &path, int W, int H, const uint8_t *rgb, std::string *err);
bool png_read_rgb8(const std::string &path, int *W, int *H, std::vector<uint8_t> *rgb, std::string *err);
}  // namespace ipt

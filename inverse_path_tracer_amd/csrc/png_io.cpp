// png_io.cpp -- 8-bit PNG encode/decode on zlib.
//
// Stands in for the reference's (un-vendored) stb_image_write / stb_image:
// createImage writes an RGB8 PNG (path_trace.cu:233 stbi_write_png) and
// createGraph loads the target as RGB8 (inv_scene.h:56 stbi_load(..., 3)).
// Decoding accepts 8-bit greyscale, grey+alpha, RGB, RGBA and palette images
// (non-interlaced) and returns RGB, like stbi_load with req_comp = 3.
#include "png_io.h"

#include <zlib.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <vector>

namespace ipt {
namespace {

void put_u32(std::vector<uint8_t> &b, uint32_t v) {
  b.push_back((uint8_t)(v >> 24));
  b.push_back((uint8_t)(v >> 16));
  b.push_back((uint8_t)(v >> 8));
  b.push_back((uint8_t)v);
}
uint32_t get_u32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
void chunk(std::vector<uint8_t> &out, const char *type, const std::vector<uint8_t> &data) {
  put_u32(out, (uint32_t)data.size());
  const size_t start = out.size();
  out.insert(out.end(), type, type + 4);
  out.insert(out.end(), data.begin(), data.end());
  const uLong crc = crc32(0L, out.data() + start, (uInt)(out.size() - start));
  put_u32(out, (uint32_t)crc);
}
const uint8_t kSig[8] = {137, 80, 78, 71, 13, 10, 26, 10};

int paeth(int a, int b, int c) {
  const int p = a + b - c;
  const int pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p, pc = p > c ? p - c : c - p;
  if (pa <= pb && pa <= pc) return a;
  return pb <= pc ? b : c;
}

}  // namespace

bool png_write_rgb8(const std::string &path, int W, int H, const uint8_t *rgb, std::string *err) {
  if (W <= 0 || H <= 0) {
    *err = "png: bad size";
    return false;
  }
  std::vector<uint8_t> raw((size_t)H * (1 + (size_t)W * 3));
  for (int r = 0; r < H; ++r) {
    uint8_t *row = raw.data() + (size_t)r * (1 + (size_t)W * 3);
    row[0] = 0;
    std::memcpy(row + 1, rgb + (size_t)r * W * 3, (size_t)W * 3);
  }
  uLongf zlen = compressBound((uLong)raw.size());
  std::vector<uint8_t> z(zlen);
  if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) {
    *err = "png: deflate failed";
    return false;
  }
  z.resize(zlen);
  std::vector<uint8_t> out(kSig, kSig + 8), ihdr;
  put_u32(ihdr, (uint32_t)W);
  put_u32(ihdr, (uint32_t)H);
  ihdr.push_back(8);  // bit depth
  ihdr.push_back(2);  // colour type RGB
  ihdr.push_back(0);
  ihdr.push_back(0);
  ihdr.push_back(0);
  chunk(out, "IHDR", ihdr);
  chunk(out, "IDAT", z);
  chunk(out, "IEND", {});
  std::ofstream f(path, std::ios::binary);
  if (!f) {
    *err = "png: cannot open " + path + " for writing";
    return false;
  }
  f.write(reinterpret_cast<const char *>(out.data()), (std::streamsize)out.size());
  return (bool)f;
}

bool png_read_rgb8(const std::string &path, int *W, int *H, std::vector<uint8_t> *rgb, std::string *err) {
  std::ifstream f(path, std::ios::binary);
  if (!f) {
    *err = "png: cannot open " + path;
    return false;
  }
  std::vector<uint8_t> b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  if (b.size() < 8 || std::memcmp(b.data(), kSig, 8) != 0) {
    *err = "png: not a PNG file: " + path;
    return false;
  }
  uint32_t w = 0, h = 0;
  int depth = 0, ctype = -1, interlace = 0;
  std::vector<uint8_t> idat, plte;
  size_t pos = 8;
  while (pos + 12 <= b.size()) {
    const uint32_t len = get_u32(&b[pos]);
    if (pos + 12 + (size_t)len > b.size()) break;
    const char *type = reinterpret_cast<const char *>(&b[pos + 4]);
    const uint8_t *data = &b[pos + 8];
    if (!std::memcmp(type, "IHDR", 4) && len >= 13) {
      w = get_u32(data);
      h = get_u32(data + 4);
      depth = data[8];
      ctype = data[9];
      interlace = data[12];
    } else if (!std::memcmp(type, "PLTE", 4)) {
      plte.assign(data, data + len);
    } else if (!std::memcmp(type, "IDAT", 4)) {
      idat.insert(idat.end(), data, data + len);
    } else if (!std::memcmp(type, "IEND", 4)) {
      break;
    }
    pos += 12 + len;
  }
  int ch = 0;
  switch (ctype) {
    case 0: ch = 1; break;
    case 2: ch = 3; break;
    case 3: ch = 1; break;
    case 4: ch = 2; break;
    case 6: ch = 4; break;
    default: *err = "png: unsupported colour type"; return false;
  }
  if (depth != 8 || interlace != 0 || w == 0 || h == 0) {
    *err = "png: only non-interlaced 8-bit images are supported";
    return false;
  }
  const size_t stride = (size_t)w * ch;
  std::vector<uint8_t> raw((stride + 1) * h);
  uLongf rl = (uLongf)raw.size();
  if (uncompress(raw.data(), &rl, idat.data(), (uLong)idat.size()) != Z_OK || rl != raw.size()) {
    *err = "png: inflate failed";
    return false;
  }
  std::vector<uint8_t> img(stride * h);
  for (uint32_t r = 0; r < h; ++r) {
    const uint8_t ft = raw[r * (stride + 1)];
    const uint8_t *src = &raw[r * (stride + 1) + 1];
    uint8_t *cur = &img[r * stride];
    const uint8_t *prev = r ? &img[(r - 1) * stride] : nullptr;
    for (size_t i = 0; i < stride; ++i) {
      const int a = i >= (size_t)ch ? cur[i - ch] : 0;
      const int up = prev ? prev[i] : 0;
      const int c = (prev && i >= (size_t)ch) ? prev[i - ch] : 0;
      int v = src[i];
      switch (ft) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += up; break;
        case 3: v += (a + up) >> 1; break;
        case 4: v += paeth(a, up, c); break;
        default: *err = "png: bad filter"; return false;
      }
      cur[i] = (uint8_t)v;
    }
  }
  rgb->resize((size_t)w * h * 3);
  for (size_t i = 0; i < (size_t)w * h; ++i) {
    uint8_t *o = &(*rgb)[3 * i];
    const uint8_t *s = &img[i * ch];
    if (ctype == 3) {
      const size_t pi = (size_t)s[0] * 3;
      if (pi + 2 >= plte.size()) {
        *err = "png: palette index out of range";
        return false;
      }
      o[0] = plte[pi];
      o[1] = plte[pi + 1];
      o[2] = plte[pi + 2];
    } else if (ch <= 2) {
      o[0] = o[1] = o[2] = s[0];
    } else {
      o[0] = s[0];
      o[1] = s[1];
      o[2] = s[2];
    }
  }
  *W = (int)w;
  *H = (int)h;
  return true;
}

}  // namespace ipt

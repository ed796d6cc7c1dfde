// png_write.hpp — RGB8 PNG writer (zlib), the output side of the drop-in CLI.
// Writes what stbi_write_png(name, W, H, 3, data, 3W) writes in the reference
// (/root/reference/source.cpp:224-229): 8-bit truecolour, non-interlaced, same pixels; zlib
// level 8 as stb (stb_image_write.h:69).  Byte streams differ (filter choice), pixels do not.
#pragma once

#include <zlib.h>

#include <cstdint>
#include <cstdio>
#include <vector>

namespace ykpng {

inline void put32(std::vector<uint8_t>& b, uint32_t v) {
  b.push_back(uint8_t(v >> 24));
  b.push_back(uint8_t(v >> 16));
  b.push_back(uint8_t(v >> 8));
  b.push_back(uint8_t(v));
}

inline void chunk(std::vector<uint8_t>& out, const char* type, const std::vector<uint8_t>& data) {
  put32(out, (uint32_t)data.size());
  const size_t start = out.size();
  out.insert(out.end(), type, type + 4);
  out.insert(out.end(), data.begin(), data.end());
  put32(out, (uint32_t)crc32(0, out.data() + start, (uInt)(out.size() - start)));
}

// Returns true on success (stbi_write_png returns nonzero on success).
inline bool write_rgb(const char* path, uint32_t w, uint32_t h, const uint8_t* rgb) {
  std::vector<uint8_t> raw;
  raw.reserve((size_t)h * (3 * w + 1));
  for (uint32_t y = 0; y < h; ++y) {
    raw.push_back(0);  // filter: none
    raw.insert(raw.end(), rgb + (size_t)y * 3 * w, rgb + (size_t)(y + 1) * 3 * w);
  }
  uLongf zlen = compressBound((uLong)raw.size());
  std::vector<uint8_t> z(zlen);
  if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 8) != Z_OK) return false;
  z.resize(zlen);
  std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  std::vector<uint8_t> ihdr;
  put32(ihdr, w);
  put32(ihdr, h);
  ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});
  chunk(out, "IHDR", ihdr);
  chunk(out, "IDAT", z);
  chunk(out, "IEND", {});
  FILE* f = std::fopen(path, "wb");
  if (!f) return false;
  const bool ok = std::fwrite(out.data(), 1, out.size(), f) == out.size();
  return (std::fclose(f) == 0) && ok;
}

}  // namespace ykpng

// Image files -> 8-bit pixel arrays with the semantics of the reference's
// stbi_load (stb_image v2.19, vendored at Raytracing_n/stb_image.h and called by
// every scene builder, e.g. Raytracing_n.cpp:269, :614, :631, :636) -- and the
// PPM / PNG writers for the output image.  See imageio.cpp.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace srr {

struct Image {
  int w = 0, h = 0;
  int n = 0;                // channels in px (the file's own count, or req_comp)
  int file_n = 0;           // what stbi_load reports through *comp
  std::vector<uint8_t> px;  // row-major, top row first, n bytes per pixel
};

// Decodes PNG, baseline JPEG or TGA by content (like stbi_load's format probe).
// req_comp 0 keeps the file's channels; 1..4 converts like stbi__convert_format.
int load_image(const std::string& path, int req_comp, Image& out, std::string& err);
int decode_image(const uint8_t* data, size_t len, int req_comp, Image& out, std::string& err);

// PNG encoder (zlib deflate, filter 0 rows), for the output image.
int encode_png(const uint8_t* px, int w, int h, int n, std::vector<uint8_t>& out, std::string& err);

}  // namespace srr

// srr scene description v1 -- tokenizer shared by the oracle consumers
// (oracle/ref/harness.cpp, which builds REFERENCE objects, and
// oracle/restate.cpp, the CPU restatement).  TEST INFRASTRUCTURE ONLY.
//
// The format itself is specified in DESIGN.md §3 ("Scene description").  Each
// non-empty, non-comment line is one construction command; a consumer replays
// the commands in file order, which is also the order in which the reference's
// scene builders (Raytracing_n.cpp:108-711) would call the constructors.
#pragma once
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace srr_text {

struct Cmd {
  int line = 0;
  std::vector<std::string> tok;
  const std::string& at(size_t i) const {
    if (i >= tok.size())
      throw std::runtime_error("scene line " + std::to_string(line) + ": missing token " + std::to_string(i));
    return tok[i];
  }
  float f(size_t i) const { return std::strtof(at(i).c_str(), nullptr); }
  double d(size_t i) const { return std::strtod(at(i).c_str(), nullptr); }
  long long i(size_t k) const { return std::strtoll(at(k).c_str(), nullptr, 10); }
  unsigned long long u(size_t k) const { return std::strtoull(at(k).c_str(), nullptr, 10); }
};

inline std::vector<Cmd> parse(const std::string& text) {
  std::vector<Cmd> out;
  std::istringstream is(text);
  std::string line;
  int ln = 0;
  while (std::getline(is, line)) {
    ++ln;
    size_t h = line.find('#');
    if (h != std::string::npos) line.resize(h);
    std::istringstream ls(line);
    Cmd c;
    c.line = ln;
    std::string t;
    while (ls >> t) c.tok.push_back(t);
    if (!c.tok.empty()) out.push_back(std::move(c));
  }
  if (out.empty() || out[0].tok[0] != "srr_scene" || out[0].i(1) != 1)
    throw std::runtime_error("not an srr_scene v1 description");
  return out;
}

inline std::string read_file(const char* path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error(std::string("cannot open ") + path);
  std::ostringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

// 48-bit LCG state of the reference's global drand48 after perlin.h's static
// initialisers consumed 1,533 draws from seed = 1 (mathf.h:12, perlin.h:94-97;
// SURVEY Q14).  Scene-build draws (bvh axis picks) start here by default.
constexpr unsigned long long kPostPerlinSeed = 24561125610955ULL;

// Per-path RNG seeding (SURVEY §8(d) "RNG seeds"): FNV-1a-64 over the bytes of
// the 32-bit little-endian words (x, y, s); the 48-bit LCG takes the low 48 bits,
// PCG32 starts at PCG32_DEFAULT_STATE ^ (lcg << 16) on the default stream.
inline unsigned long long path_seed(unsigned x, unsigned y, unsigned s, unsigned long long base = 0) {
  unsigned long long h = 0xcbf29ce484222325ULL ^ base;
  const unsigned w[3] = {x, y, s};
  for (int k = 0; k < 3; ++k)
    for (int b = 0; b < 4; ++b) {
      h ^= (w[k] >> (8 * b)) & 0xffu;
      h *= 0x100000001b3ULL;
    }
  return h & 0xFFFFFFFFFFFFULL;
}

// `tex <id> image_raw w h path`: an already decoded RGB8 image, w*h*3 bytes,
// row 0 = top (what stbi_load returns for the reference's RGB assets).
inline std::vector<unsigned char> read_raw_image(const std::string& path, int w, int h) {
  std::string b = read_file(path.c_str());
  if (w <= 0 || h <= 0 || b.size() != (size_t)w * h * 3)
    throw std::runtime_error("image_raw " + path + ": expected " + std::to_string((size_t)w * h * 3) + " bytes");
  return std::vector<unsigned char>(b.begin(), b.end());
}

// Synthetic RGB8 images (`tex <id> image_gen w h seed kind`), integer-only so
// every consumer produces identical bytes.  kind: 0 sky, 1 wood, 2 checker.
inline unsigned hash32(unsigned a) {
  a ^= a >> 16; a *= 0x7feb352dU; a ^= a >> 15; a *= 0x846ca68bU; a ^= a >> 16;
  return a;
}
inline std::vector<unsigned char> gen_image(int w, int h, unsigned seed, int kind) {
  std::vector<unsigned char> px((size_t)w * h * 3);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      unsigned n = hash32(seed * 0x9E3779B9u ^ hash32((unsigned)(y * w + x)));
      int r, g, b;
      if (kind == 0) {          // sky: vertical gradient + hashed speckle (row 0 = top)
        int t = (y * 255) / (h > 1 ? h - 1 : 1);
        r = 90 + (t * 120) / 255 + (int)(n & 15);
        g = 140 + (t * 90) / 255 + (int)((n >> 4) & 15);
        b = 235 - (t * 60) / 255 + (int)((n >> 8) & 15);
      } else if (kind == 1) {   // wood: banded rings along x with hashed grain
        int band = ((x * 7 + (int)((n >> 3) & 7)) / 13) & 15;
        r = 110 + band * 6 + (int)(n & 7);
        g = 70 + band * 4 + (int)((n >> 5) & 7);
        b = 40 + band * 2 + (int)((n >> 9) & 7);
      } else {                  // checker, 8 px cells
        int c = ((x >> 3) ^ (y >> 3)) & 1;
        r = g = b = c ? 230 : 25;
      }
      unsigned char* p = &px[((size_t)y * w + x) * 3];
      p[0] = (unsigned char)(r > 255 ? 255 : r);
      p[1] = (unsigned char)(g > 255 ? 255 : g);
      p[2] = (unsigned char)(b > 255 ? 255 : b);
    }
  return px;
}

}  // namespace srr_text

// Bit-exactness check of csrc/glibc_mathf.h against the host libm (glibc):
// every float input for expf / logf / sinf / cosf, and sampled pairs for powf.
//   g++ -std=c++17 -O2 -mfma -ffp-contract=off -pthread tools/check_glibc_mathf.cpp -o /tmp/chk && /tmp/chk
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "../simple-raytracing-render_amd/csrc/glibc_mathf.h"

using namespace srr::gm;

static bool same(float a, float b) {
  if (a != a && b != b) return true;
  uint32_t x, y;
  std::memcpy(&x, &a, 4);
  std::memcpy(&y, &b, 4);
  return x == y;
}

template <class F, class G>
static void exhaustive(const char* name, F ours, G ref) {
  const int T = std::max(1u, std::thread::hardware_concurrency());
  std::vector<unsigned long long> bad(T, 0), first(T, ~0ull);
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      for (uint64_t u = t; u < (1ull << 32); u += T) {
        float x;
        uint32_t v = (uint32_t)u;
        std::memcpy(&x, &v, 4);
        if (!same(ours(x), ref(x))) {
          if (!bad[t]) first[t] = u;
          ++bad[t];
        }
      }
    });
  for (auto& x : th) x.join();
  unsigned long long n = 0, f = ~0ull;
  for (int t = 0; t < T; ++t) n += bad[t], f = std::min(f, first[t]);
  if (n) {
    float x;
    uint32_t v = (uint32_t)f;
    std::memcpy(&x, &v, 4);
    printf("%s: %llu mismatches over 2^32 inputs (first x=%a ours=%a libm=%a)\n", name, n, x, ours(x), ref(x));
  } else {
    printf("%s: bit-exact over all 2^32 inputs\n", name);
  }
}

int main() {
  exhaustive("expf", [](float x) { return expf_(x); }, [](float x) { return ::expf(x); });
  exhaustive("logf", [](float x) { return logf_(x); }, [](float x) { return ::logf(x); });
  exhaustive("sinf", [](float x) { return sinf_(x); }, [](float x) { return ::sinf(x); });
  exhaustive("cosf", [](float x) { return cosf_(x); }, [](float x) { return ::cosf(x); });
  exhaustive("sincosf (sine)", [](float x) { float s, c; sincosf_(x, s, c); return s; }, [](float x) { return ::sinf(x); });
  exhaustive("sincosf (cosine)", [](float x) { float s, c; sincosf_(x, s, c); return c; }, [](float x) { return ::cosf(x); });
  exhaustive("acosf", [](float x) { return acosf_(x); }, [](float x) { return ::acosf(x); });
  exhaustive("asinf", [](float x) { return asinf_(x); }, [](float x) { return ::asinf(x); });
  exhaustive("atanf", [](float x) { return atanf_(x); }, [](float x) { return ::atanf(x); });
  std::mt19937_64 g(7);
  std::uniform_real_distribution<float> ux(1e-7f, 4.0f), uy(-8.0f, 8.0f), u01(0.0f, 1.0f);
  unsigned long long n = 0, bad = 0;
  for (int i = 0; i < 50000000; ++i) {
    float x = (i & 1) ? ux(g) : 1.0f - std::fmax(u01(g), 1e-6f);  // the Beckmann sampler's pow(1 - u, fit)
    float y = (i & 1) ? uy(g) : 1.0f + u01(g) * (-0.876f + u01(g) * 0.4265f);
    ++n;
    if (!same(powf_(x, y), ::powf(x, y))) {
      if (bad < 5) printf("powf mismatch x=%a y=%a ours=%a libm=%a\n", x, y, powf_(x, y), ::powf(x, y));
      ++bad;
    }
  }
  printf("powf: %llu mismatches in %llu sampled pairs\n", bad, n);
  std::uniform_real_distribution<float> us(-1.0f, 1.0f);
  bad = 0;
  for (int i = 0; i < 20000000; ++i) {  // get_sphere_uv's atan2f(p.z, p.x) on unit vectors, and general pairs
    float y = us(g), x = us(g);
    if (i & 1) y *= 1000.0f;
    if (!same(atan2f_(y, x), ::atan2f(y, x))) ++bad;
  }
  printf("atan2f: %llu mismatches in 20000000 sampled pairs\n", bad);
  return 0;
}

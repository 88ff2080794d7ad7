// Bit-exactness check of include/srr/glibc_math64.h (glibc's dbl-64 sin / cos / acos /
// atan2, restated) against the host libm, which the reference's brdf.h calls.
// Sampled, since the inputs are 64-bit: uniform over each function's whole
// domain by bit pattern, uniform by value over the reference's angle ranges,
// every branch boundary of the restatement +-4096 ulps, and the MERL lookup's
// own near-degenerate atan2 arguments (residues ~1e-17 against ~1).
//   g++ -std=c++17 -O2 -mfma -ffp-contract=off -pthread tools/check_glibc_math64.cpp -o /tmp/chk64 && /tmp/chk64 [M]
// (M: millions of samples per family, default 20)
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "../include/srr/glibc_math64.h"

namespace g = srr::gm64;

static uint64_t B(double x) {
  uint64_t u;
  std::memcpy(&u, &x, 8);
  return u;
}
static double D(uint64_t u) {
  double x;
  std::memcpy(&x, &u, 8);
  return x;
}
static bool same(double a, double b) { return (a != a && b != b) || B(a) == B(b); }

struct Tally {
  std::atomic<unsigned long long> n{0}, bad{0};
  std::atomic<uint64_t> first_a{0}, first_b{0};
};

template <class Gen, class F, class R>
static void run1(const char* name, long long count, Gen gen, F ours, R ref) {
  const int T = std::max(1u, std::thread::hardware_concurrency());
  Tally t;
  std::vector<std::thread> th;
  for (int k = 0; k < T; ++k)
    th.emplace_back([&, k] {
      std::mt19937_64 rng(0x5eed0000ull + 7919ull * k + std::hash<std::string>()(name));
      for (long long i = k; i < count; i += T) {
        const double x = gen(rng);
        const double a = ours(x), b = ref(x);
        ++t.n;
        if (!same(a, b) && t.bad++ == 0) t.first_a = B(x);
      }
    });
  for (auto& x : th) x.join();
  printf("%-34s %12llu samples  %llu differ", name, t.n.load(), t.bad.load());
  if (t.bad) printf("  (first x = %a)", D(t.first_a.load()));
  printf("\n");
  if (t.bad) std::exit(1);
}

template <class Gen, class F, class R>
static void run2(const char* name, long long count, Gen gen, F ours, R ref) {
  const int T = std::max(1u, std::thread::hardware_concurrency());
  Tally t;
  std::vector<std::thread> th;
  for (int k = 0; k < T; ++k)
    th.emplace_back([&, k] {
      std::mt19937_64 rng(0xa7a20000ull + 104729ull * k + std::hash<std::string>()(name));
      for (long long i = k; i < count; i += T) {
        double y, x;
        gen(rng, y, x);
        const double a = ours(y, x), b = ref(y, x);
        ++t.n;
        if (!same(a, b) && t.bad++ == 0) {
          t.first_a = B(y);
          t.first_b = B(x);
        }
      }
    });
  for (auto& x : th) x.join();
  printf("%-34s %12llu samples  %llu differ", name, t.n.load(), t.bad.load());
  if (t.bad) printf("  (first y = %a, x = %a)", D(t.first_a.load()), D(t.first_b.load()));
  printf("\n");
  if (t.bad) std::exit(1);
}

int main(int argc, char** argv) {
  const long long M = (argc > 1 ? atoll(argv[1]) : 20) * 1000000LL;
  auto sinf_ = [](double x) { return g::sin(x); };
  auto cosf_ = [](double x) { return g::cos(x); };
  auto acosf_ = [](double x) { return g::acos(x); };
  auto rsin = [](double x) { return ::sin(x); };
  auto rcos = [](double x) { return ::cos(x); };
  auto racos = [](double x) { return ::acos(x); };
  auto ratan2 = [](double y, double x) { return ::atan2(y, x); };
  auto atan2_ = [](double y, double x) { return g::atan2(y, x); };

  // sin / cos: by value over the reference's angles, and by bit pattern below 105414350
  auto ang = [](std::mt19937_64& r) { return std::uniform_real_distribution<double>(-7.0, 7.0)(r); };
  auto bitsin = [](std::mt19937_64& r) {
    for (;;) {
      const double x = D(r());
      if (std::fabs(x) < 105414335.0) return x;  // below __branred (hi word 0x419921fb)
    }
  };
  const double sin_edges[] = {0x1p-26, 0x1p-27, 0.126, 0.855469, 0.85546875, 2.426265, 2.4262650203704834, 105414335.0,
                              1.5707963267948966, 3.141592653589793, 4.71238898038469, 6.283185307179586};
  auto edge = [&](const double* e, int ne) {
    return [=](std::mt19937_64& r) {
      const double c = e[r() % ne];
      double v = D(B(c) + (int64_t)(r() % 8193) - 4096);
      if (v >= 105414336.0) v = 105414335.0;  // (sin / cos: __branred's range is not restated)
      return (r() & 1) ? -v : v;
    };
  };
  run1("sin  angles [-7, 7]", M, ang, sinf_, rsin);
  run1("cos  angles [-7, 7]", M, ang, cosf_, rcos);
  run1("sin  bit patterns |x| < 1.05e8", M, bitsin, sinf_, rsin);
  run1("cos  bit patterns |x| < 1.05e8", M, bitsin, cosf_, rcos);
  run1("sin  branch edges", M / 4, edge(sin_edges, 12), sinf_, rsin);
  run1("cos  branch edges", M / 4, edge(sin_edges, 12), cosf_, rcos);

  // sincos (glibc's non-FMA s_sincos.c), both outputs
  auto sc_s = [](double x) { double s, c; g::sincos(x, s, c); return s; };
  auto sc_c = [](double x) { double s, c; g::sincos(x, s, c); return c; };
  auto rsc_s = [](double x) { double s, c; ::sincos(x, &s, &c); return s; };
  auto rsc_c = [](double x) { double s, c; ::sincos(x, &s, &c); return c; };
  run1("sincos.sin angles [-7, 7]", M, ang, sc_s, rsc_s);
  run1("sincos.cos angles [-7, 7]", M, ang, sc_c, rsc_c);
  run1("sincos.sin bit patterns", M, bitsin, sc_s, rsc_s);
  run1("sincos.cos bit patterns", M, bitsin, sc_c, rsc_c);
  run1("sincos.sin branch edges", M / 4, edge(sin_edges, 12), sc_s, rsc_s);
  run1("sincos.cos branch edges", M / 4, edge(sin_edges, 12), sc_c, rsc_c);

  // acos: by value over [-1, 1], by bit pattern (all doubles), edges, near +-1
  auto unit = [](std::mt19937_64& r) { return std::uniform_real_distribution<double>(-1.0, 1.0)(r); };
  auto anyd = [](std::mt19937_64& r) { return D(r()); };
  auto near1 = [](std::mt19937_64& r) {
    const double v = 1.0 - std::ldexp(std::uniform_real_distribution<double>(0.0, 1.0)(r), -(int)(r() % 60));
    return (r() & 1) ? -v : v;
  };
  const double acos_edges[] = {0x1p-55, 0.125, 0.25, 0.5, 0.75, 0.921875, 0.953125, 0.96875, 1.0};
  run1("acos [-1, 1]", M, unit, acosf_, racos);
  run1("acos bit patterns", M, anyd, acosf_, racos);
  run1("acos near +-1", M, near1, acosf_, racos);
  run1("acos branch edges", M / 4, edge(acos_edges, 9), acosf_, racos);

  // atan2: unit-circle directions (the half vector), all bit patterns, ratio edges,
  // and brdf's degenerate difference vectors: (residue, residue) with residues ~1e-17
  auto circle = [](std::mt19937_64& r, double& y, double& x) {
    const double t = std::uniform_real_distribution<double>(-3.2, 3.2)(r);
    const double s = std::uniform_real_distribution<double>(0.0, 2.0)(r);
    y = s * std::sin(t);
    x = s * std::cos(t);
  };
  auto anyd2 = [](std::mt19937_64& r, double& y, double& x) {
    y = D(r());
    x = D(r());
  };
  auto residue = [](std::mt19937_64& r, double& y, double& x) {
    auto one = [&] {
      const double v = std::ldexp(std::uniform_real_distribution<double>(0.5, 1.0)(r), -50 - (int)(r() % 20));
      return (r() & 1) ? -v : v;
    };
    y = (r() % 16) ? one() : 0.0;
    x = (r() % 16) ? one() : 0.0;
  };
  auto ratio = [](std::mt19937_64& r, double& y, double& x) {  // u = small/large around 1/16 and the cij rows
    const double u = (r() & 1) ? D(B(0.0625) + (int64_t)(r() % 8193) - 4096)
                               : std::uniform_real_distribution<double>(0.0, 1.0)(r);
    const double l = std::ldexp(1.0, (int)(r() % 40) - 20);
    double a = u * l, b = l;
    if (r() & 1) std::swap(a, b);
    y = (r() & 1) ? -a : a;
    x = (r() & 1) ? -b : b;
  };
  run2("atan2 directions", M, circle, atan2_, ratan2);
  run2("atan2 bit patterns", M, anyd2, atan2_, ratan2);
  run2("atan2 ~1e-17 residues", M, residue, atan2_, ratan2);
  run2("atan2 ratios (1/16, cij rows)", M, ratio, atan2_, ratan2);
  const double sp[] = {0.0, -0.0, 1.0, -1.0, INFINITY, -INFINITY, NAN, 0x1p-1074, -0x1p-1074, 0x1.fffffffffffffp+1023};
  unsigned bad = 0;
  for (double y : sp)
    for (double x : sp) bad += !same(g::atan2(y, x), ::atan2(y, x));
  printf("atan2 special operand pairs: %u of 100 differ\n", bad);
  return bad ? 1 : 0;
}

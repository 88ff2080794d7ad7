"""k_paths' invariant divisors (csrc/kernels.h make_udiv31): the refill turns a
path index into (pixel, sample) and a pixel into (i, j) with (n * m) >> p instead
of integer divisions.  The magic must equal floor(n / d) for every numerator the
kernel can see (n < 2^31: window paths and frame pixels are checked below that)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SRC = r"""
#include <cstdio>
#include <cstdint>
#include <random>
#include "kernels.h"
using namespace srr;
static uint32_t div31(uint32_t n, UDiv31 v) { return (uint32_t)(((uint64_t)n * v.m) >> v.p); }
int main() {
  std::mt19937_64 g(7);
  long bad = 0, checks = 0;
  auto check = [&](uint32_t d, uint32_t n) {
    const UDiv31 v = make_udiv31(d);
    ++checks;
    if (div31(n, v) != n / d) { if (bad++ < 5) printf("d=%u n=%u\n", d, n); }
  };
  for (uint32_t d = 1; d <= 70000; ++d) {  // every spp window and image width in use
    const uint32_t edge[] = {0u, 1u, d - 1, d, d + 1, 2 * d - 1, 2 * d, 0x7ffffffeu, 0x7fffffffu,
                             (0x7fffffffu / d) * d, (0x7fffffffu / d) * d - 1};
    for (uint32_t n : edge) if (n < 0x80000000u) check(d, n);
    for (int k = 0; k < 16; ++k) check(d, (uint32_t)(g() & 0x7fffffffu));
  }
  for (int k = 0; k < 2000000; ++k) {
    const uint32_t d = 1 + (uint32_t)(g() % 0x7fffffffu);
    check(d, (uint32_t)(g() & 0x7fffffffu));
    check(d, (uint32_t)((0x7fffffffu / d) * d));
  }
  printf("%ld checks, %ld wrong\n", checks, bad);
  return bad != 0;
}
"""


def test_udiv31_matches_integer_division(tmp_path):
    src = tmp_path / "udiv.cpp"
    src.write_text(SRC)
    exe = tmp_path / "udiv"
    subprocess.run(["g++", "-std=c++17", "-O2", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    "-I", os.path.join(ROOT, "simple-raytracing-render_amd", "csrc"), str(src), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert " 0 wrong" in out.stdout

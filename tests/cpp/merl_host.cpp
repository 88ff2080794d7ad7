// Host build of the product's MERL lookup (include/srr/merl.h with glibc_math64.h,
// the same source the device kernel k_merl_lookup compiles): reads n queries
// (theta_in, fi_in, theta_out, fi_out as doubles) from argv[1], writes n cells
// (int32) and n x 3 RGB doubles to argv[2].  tests/test_merl.py builds it with g++
// and checks it against the reference's KAT records.
#include <cstdio>
#include <vector>

#include "../../include/srr/merl.h"

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 3;
  std::vector<double> a;
  double v;
  while (fread(&v, 8, 1, f) == 1) a.push_back(v);
  fclose(f);
  const size_t n = a.size() / 4;
  // the synthetic table of oracle/ref/kat.inc merl_table()
  std::vector<double> tab(3 * (size_t)srr::merl::kCells);
  for (size_t k = 0; k < tab.size(); ++k)
    tab[k] = (k % 97 == 0) ? -1.0 : (double)(((unsigned long long)k * 2654435761ULL) % 1000003ULL) / 1000.0;
  std::vector<int> cell(n);
  std::vector<double> rgb(3 * n);
  for (size_t i = 0; i < n; ++i) {
    cell[i] = srr::merl::cell_of(a[4 * i], a[4 * i + 1], a[4 * i + 2], a[4 * i + 3]);
    srr::merl::rgb_of(tab.data(), cell[i], rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2]);
  }
  FILE* o = fopen(argv[2], "wb");
  if (!o) return 4;
  fwrite(cell.data(), 4, n, o);
  fwrite(rgb.data(), 8, 3 * n, o);
  fclose(o);
  return 0;
}

// Force-included shim for compiling the reference translation unit
// (/root/reference/Raytracing_n/Raytracing_n.cpp, MSVC v142 code) with g++ 11 in
// the development container.  TEST INFRASTRUCTURE ONLY: nothing under oracle/
// is linked into, or called by, the product path.
//
// Adaptations, zero edits to reference files:
//  * pre-include every std header the TU needs, because mathf.h:6-8 defines the
//    object-like macros __m/__c/__a which break libstdc++ headers parsed after;
//  * rename drand48/srand48 (glibc declares them with a different contract);
//  * MSVC-only names: errno_t, fopen_s (brdf.h:159), std::fmaxf (reflection.h:12),
//    _CrtDumpMemoryLeaks (Raytracing_n.cpp:950);
//  * malloc -> calloc so beckmann_pdf's pdf_value (pdf.h:122) starts at 0
//    (SURVEY Q11 build definition).
#pragma once
#include <immintrin.h>
#include <cassert>
#include <cstdarg>
#include <climits>
#include <cstddef>
#include <cstdint>
#include <atomic>
#include <iostream>
#include <fstream>
#include <sstream>
#include <vector>
#include <map>
#include <unordered_map>
#include <set>
#include <thread>
#include <mutex>
#include <chrono>
#include <algorithm>
#include <random>
#include <limits>
#include <memory>
#include <functional>
#include <exception>
#include <stdexcept>
#include <new>
#include <ctime>
#include <cstdlib>
#include <cstdio>
#include <cerrno>
#include <cmath>
#include <cfloat>
#include <cstring>
#include <string>
#include <math.h>
#include <stdlib.h>
#include <float.h>

namespace std { using ::fmaxf; }
typedef int errno_t;
static inline errno_t fopen_s(FILE** f, const char* n, const char* m) {
  *f = fopen(n, m);
  return *f ? 0 : errno;
}
#define drand48 ref_drand48
#define srand48 ref_srand48
#define _CrtDumpMemoryLeaks() 0
#define malloc(x) calloc(1, (x))

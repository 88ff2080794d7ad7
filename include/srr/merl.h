// MERL isotropic measured-BRDF table lookup (the reference's brdf.h): the
// table index of an (in, out) direction pair in half/difference-angle
// coordinates (Rusinkiewicz), and the scaled RGB value stored there.  Host and
// device share this code; every operation is double precision in the
// reference's order (kernels are built with -ffp-contract=off), and its double
// cos / sin / acos / atan2 are glibc 2.35's own algorithms (glibc_math64.h), so
// the cell of every query -- out == in included, where phi_diff is atan2 of
// ~1e-17 residues -- is the one the ORACLE PORT computes: the reference's
// brdf.h compiled here by g++ -O2 against glibc 2.35 on an FMA-capable x86-64
// (oracle/ref).  The reference itself is an MSVC v142 project
// (Raytracing_n.vcxproj) whose UCRT libm is a different implementation: for
// out == in, parity with that build is unpinned; other queries can
// differ only where an angle lies within a few ulps of a cell boundary.
//
// Reference: brdf.h:7-15 (resolution, channel scales), :17-61 (index
// functions), :70-154 (vector helpers, std_coords_to_half_diff_coords),
// :190-214 (lookup_brdf_val).  brdfmaterial (material.h:201-241) is dead code
// in the reference; only the lookup is reproduced.
#pragma once

#include <cmath>
#include <cstdint>

#include "glibc_math64.h"

#if defined(__HIPCC__)
#define SRR_HD __device__ inline  // (glibc_math64.h's tables live in device memory)
#else
#define SRR_HD inline
#endif

namespace srr {
namespace merl {

constexpr int kResThetaH = 90;
constexpr int kResThetaD = 90;
constexpr int kResPhiD = 360;
constexpr int kCells = kResThetaH * kResThetaD * kResPhiD / 2;  // doubles per channel (1,458,000)
constexpr double kPiD = 3.1415926535897932384626433832795;     // brdf.h's own M_PI

// theta_half in [0, pi/2] -> [0, 89], square-root spaced (brdf.h:17-30)
SRR_HD int theta_half_index(double theta_half) {
  if (theta_half <= 0.0) return 0;
  const double deg = (theta_half / (kPiD / 2.0)) * kResThetaH;
  const int k = (int)sqrt(deg * kResThetaH);
  return k < 0 ? 0 : (k >= kResThetaH ? kResThetaH - 1 : k);
}

// theta_diff in [0, pi/2] -> [0, 89] (brdf.h:34-43)
SRR_HD int theta_diff_index(double theta_diff) {
  const int k = int(theta_diff / (kPiD * 0.5) * kResThetaD);
  return k < 0 ? 0 : (k < kResThetaD - 1 ? k : kResThetaD - 1);
}

// phi_diff folded to [0, pi] by reciprocity -> [0, 179] (brdf.h:46-61)
SRR_HD int phi_diff_index(double phi_diff) {
  if (phi_diff < 0.0) phi_diff += kPiD;
  const int k = int(phi_diff / kPiD * kResPhiD / 2);
  return k < 0 ? 0 : (k < kResPhiD / 2 - 1 ? k : kResPhiD / 2 - 1);
}

SRR_HD void unit3(double* v) {  // brdf::normalize
  const double len = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  v[0] = v[0] / len;
  v[1] = v[1] / len;
  v[2] = v[2] / len;
}

// Rodrigues rotation of v about a unit axis (brdf::rotate_vector), summed in the
// reference's order: v cos, + axis (axis.v)(1 - cos), + (axis x v) sin
SRR_HD void rotate(const double* v, const double* axis, double angle, double* out) {
  const double c = gm64::cos(angle), s = gm64::sin(angle);
  for (int k = 0; k < 3; ++k) out[k] = v[k] * c;
  double d = axis[0] * v[0] + axis[1] * v[1] + axis[2] * v[2];
  d = d * (1.0 - c);
  for (int k = 0; k < 3; ++k) out[k] += axis[k] * d;
  const double x[3] = {axis[1] * v[2] - axis[2] * v[1], axis[2] * v[0] - axis[0] * v[2],
                       axis[0] * v[1] - axis[1] * v[0]};
  for (int k = 0; k < 3; ++k) out[k] += x[k] * s;
}

// brdf::std_coords_to_half_diff_coords (brdf.h:109-154).  The half vector is
// built from the unnormalised spherical vectors (as the reference does), the
// difference vector from the normalised incoming one.
SRR_HD void half_diff(double theta_in, double fi_in, double theta_out, double fi_out, double& theta_half,
                      double& fi_half, double& theta_diff, double& fi_diff) {
  // (the oracle port's g++ -O2 build merges each of the four angles' sin and cos
  // into one glibc sincos() call -- a different, non-FMA build of the algorithm --
  // while rotate()'s cos / sin stay separate calls)
  double ip, iz, sfi, cfi;
  gm64::sincos(theta_in, ip, iz);
  gm64::sincos(fi_in, sfi, cfi);
  const double ix = ip * cfi, iy = ip * sfi;
  double in[3] = {ix, iy, iz};
  unit3(in);
  double op, oz, sfo, cfo;
  gm64::sincos(theta_out, op, oz);
  gm64::sincos(fi_out, sfo, cfo);
  const double ox = op * cfo, oy = op * sfo;
  double out[3] = {ox, oy, oz};
  unit3(out);  // (unused afterwards, as in the reference)
  double h[3] = {(ix + ox) / 2.0, (iy + oy) / 2.0, (iz + oz) / 2.0};
  unit3(h);
  theta_half = gm64::acos(h[2]);
  fi_half = gm64::atan2(h[1], h[0]);
  const double binormal[3] = {0.0, 1.0, 0.0}, normal[3] = {0.0, 0.0, 1.0};
  double tmp[3], diff[3];
  rotate(in, normal, -fi_half, tmp);
  rotate(tmp, binormal, -theta_half, diff);
  theta_diff = gm64::acos(diff[2]);
  fi_diff = gm64::atan2(diff[1], diff[0]);
}

// lookup_brdf_val's table cell (brdf.h:199-203): phi_half is ignored (isotropic)
SRR_HD int cell_of(double theta_in, double fi_in, double theta_out, double fi_out) {
  double th, fh, td, fd;
  half_diff(theta_in, fi_in, theta_out, fi_out, th, fh, td, fd);
  return phi_diff_index(fd) + theta_diff_index(td) * (kResPhiD / 2) +
         theta_half_index(th) * (kResPhiD / 2) * kResThetaD;
}

// the scaled RGB of a cell; the table is channel-major, kCells doubles each
// (brdf.h:205-207 with RED/GREEN/BLUE_SCALE, :11-13)
SRR_HD void rgb_of(const double* table, int cell, double& r, double& g, double& b) {
  r = table[cell] * (1.0 / 1500.0);
  g = table[cell + kCells] * (1.15 / 1500.0);
  b = table[cell + 2 * kCells] * (1.66 / 1500.0);
}

}  // namespace merl
}  // namespace srr

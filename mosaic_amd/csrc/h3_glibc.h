// H3 v3.7 geoToH3 with the reference's arithmetic (platform glibc libm, x87 long double),
// host only: the near-tie points' second opinion (h3_glibc.cpp).
#pragma once
#include <stdint.h>

namespace mgpu {
namespace h3 {
struct IJK;
}
namespace h3glibc {
// (face, ijk) of the point as H3-Java computes it (H3IndexSystem.scala:168-170 ->
// H3Core.geoToH3(lat, lon, res)); false for non-finite input or a bad resolution
bool face_ijk(double lon_deg, double lat_deg, int res, int* face, h3::IJK* ijk);
// the cell id (0 on invalid input, as H3's geoToH3 returns H3_NULL)
uint64_t point_to_cell(double lon_deg, double lat_deg, int res);
// h3::lattice_key of the route's (face, ijk) (0 on invalid input)
uint64_t lattice_key(double lon_deg, double lat_deg, int res);
}  // namespace h3glibc
}  // namespace mgpu

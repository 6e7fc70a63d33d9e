// face_ijk_to_h3_fast (the kernels' H3 digit encoding) == face_ijk_to_h3 (the
// restated _faceIjkToH3) on random lattice positions of every face and resolution,
// pentagon base cells included.  Built by __graft_entry__.build(), run by
// tests/test_cpp_host.py.
#include "../../mosaic_amd/csrc/h3_core.h"
#include <cstdio>
#include <random>
using namespace mgpu::h3;
int main() {
  std::mt19937_64 g(3);
  long bad = 0, tot = 0, pent = 0, valid = 0;
  for (int res = 0; res <= 15; res++)
    for (int face = 0; face < 20; face++) {
      int R = 2; for (int q = 0; q < res; q++) R = R * 7 / 2 + 3; if (R > 2000000) R = 2000000;
      std::uniform_int_distribution<int> u(-R, R);
      for (int it = 0; it < 20000; it++) {
        IJK c{u(g), u(g), 0}; ijk_normalize(c);
        uint64_t a = face_ijk_to_h3(face, c, res), b = face_ijk_to_h3_fast(face, c, res);
        tot++; if (a != b) { if (bad < 5) printf("res %d face %d ijk %d %d %d: %llx vs %llx\n", res, face, c.i, c.j, c.k, (unsigned long long)a, (unsigned long long)b); bad++; }
        if (a) valid++;
        if (a && H3T_BASE_CELL_DATA[(a >> 45) & 127][4]) pent++;
      }
    }
  printf("tested %ld (valid %ld, pentagon %ld), mismatches %ld\n", tot, valid, pent, bad);
  return (bad != 0 || valid < tot / 10 || pent < 1000) ? 1 : 0;
}

// Tests of the C++ host mirror (include/mosaic_index_system.hpp) -- the reference's
// IndexSystem plugin interface and hot-path functions in a compiled host language.
//   --cpu   resolution validation, exception classes, H3/BNG format <-> parse (no GPU)
//   --gpu   pointToIndex known answers, tessellate + pipJoin + st_contains on MI355X
// Known answers come from the reference's own tests and docs:
//   docs/source/api/spatial-indexing.rst:54-59  (lon 30, lat 10, res 10) -> 623385352048508927
//   TestBNGIndexSystem.scala:12-75               (538825, 179111) res 3 -> 1050138790, res -4 -> 10501373
//   TestBNGIndexSystem.scala:77-95               "TQ" <-> 105010 ...
//   ST_ContainsBehaviors.scala:22-36             two-hole polygon: (35 25) in, (25 25) out
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "mosaic_index_system.hpp"

using namespace mosaic;

static int fails = 0;
#define EXPECT(cond)                                                        \
  do {                                                                      \
    if (!(cond)) {                                                          \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);       \
      fails++;                                                              \
    }                                                                       \
  } while (0)

template <class E, class F>
static bool throws(F f) {
  try {
    f();
  } catch (const E&) {
    return true;
  } catch (...) {
    return false;
  }
  return false;
}

static void cpu_tests() {
  H3IndexSystem h3;
  BNGIndexSystem bng;
  // getResolution (H3IndexSystem.scala:45-60, BNGIndexSystem.scala:349-360)
  EXPECT(h3.getResolution(9) == 9);
  EXPECT(h3.getResolution(std::string("12")) == 12);
  EXPECT(throws<IllegalStateException>([&] { h3.getResolution(16); }));
  EXPECT(throws<IllegalStateException>([&] { h3.getResolution(-1); }));
  EXPECT(throws<IllegalArgumentException>([&] { h3.getResolution(std::string("nine")); }));
  EXPECT(bng.getResolution(-4) == -4);
  EXPECT(bng.getResolution(std::string("100m")) == 4);
  EXPECT(bng.getResolution(std::string("500km")) == -1);
  EXPECT(throws<IllegalStateException>([&] { bng.getResolution(0); }));
  EXPECT(throws<IllegalStateException>([&] { bng.getResolution(7); }));
  EXPECT(throws<IllegalStateException>([&] { bng.getResolution(std::string("2km")); }));
  // factory
  EXPECT(getIndexSystem("h3")->name() == "H3");
  EXPECT(getIndexSystem("BNG")->crsID() == 27700);
  EXPECT(throws<IllegalArgumentException>([&] { getIndexSystem("S2"); }));
  // format / parse
  EXPECT(h3.format(623385352048508927LL) == "8a6b5acc3087fff");
  EXPECT(h3.parse("8a6b5acc3087fff") == 623385352048508927LL);
  EXPECT(bng.format(105010) == "TQ");
  EXPECT(bng.parse("TQ") == 105010);
  EXPECT(bng.format(1050138790) == "TQ3879");
  EXPECT(bng.parse("TQ3879") == 1050138790);
  EXPECT(bng.parse(bng.format(10501373)) == 10501373);
  EXPECT(throws<IllegalArgumentException>([&] { bng.parse("XX"); }));
  EXPECT(h3.getCellIdDataType() == CellIdType::Long && bng.getCellIdDataType() == CellIdType::String);
}

static void gpu_tests() {
  GpuContext ctx(0);
  H3IndexSystem h3;
  BNGIndexSystem bng;
  EXPECT(h3.pointToIndex(ctx, 30.0, 10.0, 10) == 623385352048508927LL);
  EXPECT(bng.pointToIndex(ctx, 538825.0, 179111.0, 3) == 1050138790LL);
  EXPECT(bng.pointToIndex(ctx, 538825.0, 179111.0, -3) == 10501373LL);
  EXPECT(bng.pointToIndex(ctx, 538825.0, 179111.0, -4) == 1050138794LL);
  EXPECT(throws<IllegalArgumentException>([&] { h3.pointToIndex(ctx, 0.0 / 0.0, 1.0, 9); }));
  EXPECT(throws<IllegalStateException>([&] { bng.pointToIndex(ctx, 0.0 / 0.0, 1.0, 3); }));

  // ST_ContainsBehaviors' polygon with two holes, scaled by 1/100 and moved to
  // (lon -74.5, lat 40) so that it lies on one icosahedron face (this tessellator's limit)
  auto S = [](double x, double y) { return std::make_pair(-74.5 + x / 100.0, 40.0 + y / 100.0); };
  Polygons P;
  P.add(7, {{{S(10, 10), S(110, 10), S(110, 110), S(10, 110), S(10, 10)},
             {S(20, 20), S(20, 30), S(30, 30), S(30, 20), S(20, 20)},
             {S(50, 20), S(50, 30), S(60, 30), S(60, 20), S(50, 20)}}});
  ChipTable c = grid_tessellateexplode(P, h3, 6);
  EXPECT(c.size() > 0);
  DeviceChips chips(ctx, c);
  const auto in = S(35, 25), hole = S(25, 25), far = S(200, 5), inside2 = S(40, 80);
  JoinResult r = pipJoin(ctx, chips, h3, 6, {in.first, hole.first, far.first}, {in.second, hole.second, far.second});
  EXPECT(r.point_id.size() == 1 && r.point_id[0] == 0 && r.polygon_id[0] == 7);
  // explicit point ids
  std::vector<int64_t> ids = {1000, 2000, 3000};
  r = pipJoin(ctx, chips, h3, 6, {in.first, hole.first, inside2.first}, {in.second, hole.second, inside2.second}, &ids);
  EXPECT(r.point_id.size() == 2 && r.point_id[0] == 1000 && r.point_id[1] == 3000);
  EXPECT(throws<IllegalStateException>([&] { pipJoin(ctx, chips, h3, 16, {1.0}, {1.0}); }));
  // a polygon across icosahedron faces is refused with a message
  Polygons Q;
  Q.add(1, {{{{10, 10}, {110, 10}, {110, 70}, {10, 70}, {10, 10}}}});
  EXPECT(throws<IllegalArgumentException>([&] { grid_tessellateexplode(Q, h3, 2); }));
}

int main(int argc, char** argv) {
  const bool gpu = argc > 1 && !strcmp(argv[1], "--gpu");
  cpu_tests();
  if (gpu) gpu_tests();
  printf("%s: %d failure(s)\n", gpu ? "cpu+gpu" : "cpu", fails);
  return fails ? 1 : 0;
}

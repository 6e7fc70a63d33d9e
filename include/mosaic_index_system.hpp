// mosaic_index_system.hpp -- C++ host mirror of the reference's IndexSystem plugin
// interface and hot-path functions, over the C ABI in mosaic_gpu.h.
//
// The reference's host is Scala (JVM, no JDK in this image; the JNI binding is in
// INTEGRATION.md).  This header is the compiled-language host: same class and method
// names as the Scala sources, same argument meaning, same exception classes.
//
//   IndexSystem            core/index/IndexSystem.scala:15-318
//     getResolution        H3IndexSystem.scala:45-60, BNGIndexSystem.scala:349-360
//     pointToIndex         IndexSystem.scala:237; H3IndexSystem.scala:168-170; BNGIndexSystem.scala:284-298
//     format / parse       H3IndexSystem.scala:218-228; BNGIndexSystem.scala:119-134, 440-442
//     formatCellId         IndexSystem.scala:48-57
//   IndexSystemFactory     core/index/IndexSystemFactory.scala:31-63
//   grid_tessellateexplode MosaicExplode.scala:70-79 -> Mosaic.getChips (core/Mosaic.scala:22-99)
//   st_contains            ST_Contains.scala:21-44 -> MosaicGeometryJTS.contains (MosaicGeometryJTS.scala:197)
//   pipJoin                the user-level join cell == index_id AND (is_core OR st_contains)
//                          (notebooks/examples/python/Quickstart/QuickstartNotebook.ipynb:1835)
//
// Batch methods take device pointers (HBM) and a hipStream_t (as void*); the scalar
// forms of the reference run as a batch of one through the host-pointer entry points.
// Link with -lmosaic_gpu.  Header-only, C++17.
#ifndef MOSAIC_INDEX_SYSTEM_HPP
#define MOSAIC_INDEX_SYSTEM_HPP

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "mosaic_gpu.h"

namespace mosaic {

// java.lang.IllegalArgumentException / IllegalStateException, as the reference throws
struct IllegalArgumentException : std::invalid_argument {
  using std::invalid_argument::invalid_argument;
};
struct IllegalStateException : std::logic_error {
  using std::logic_error::logic_error;
};
struct ParseException : std::runtime_error {  // JTS ParseException (bad chip WKB)
  using std::runtime_error::runtime_error;
};
struct CapacityError : std::length_error {  // output arrays too small; `required` pairs
  int64_t required;
  CapacityError(const std::string& m, int64_t r) : std::length_error(m), required(r) {}
};
struct DeviceError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// status -> the reference's exception class
inline void check(int32_t st, int64_t required = 0) {
  if (st == MGPU_OK) return;
  const std::string msg = mgpu_last_error();
  switch (st) {
    case MGPU_E_RESOLUTION:
    case MGPU_E_NAN:
    case MGPU_E_INTERNAL:
      throw IllegalStateException(msg);
    case MGPU_E_WKB:
      throw ParseException(msg);
    case MGPU_E_CAPACITY:
      throw CapacityError(msg, required);
    case MGPU_E_DEVICE:
      throw DeviceError(msg);
    default:
      throw IllegalArgumentException(msg);
  }
}

// One per GPU / executor thread (mgpu_ctx): workspace + events.
class GpuContext {
 public:
  explicit GpuContext(int device = 0) { check(mgpu_ctx_create(device, &ctx_)); }
  ~GpuContext() { mgpu_ctx_destroy(ctx_); }
  GpuContext(const GpuContext&) = delete;
  GpuContext& operator=(const GpuContext&) = delete;
  void reserve(int64_t max_points) { check(mgpu_ctx_reserve(ctx_, max_points)); }
  mgpu_ctx* get() const { return ctx_; }

 private:
  mgpu_ctx* ctx_ = nullptr;
};

enum class CellIdType { Long, String };

// abstract class IndexSystem(var cellIdType: DataType)   (IndexSystem.scala:15)
class IndexSystem {
 public:
  virtual ~IndexSystem() = default;
  virtual std::string name() const = 0;
  virtual int32_t code() const = 0;  // MGPU_H3 / MGPU_BNG
  virtual int crsID() const = 0;
  virtual std::vector<int> resolutions() const = 0;
  CellIdType getCellIdDataType() const { return cell_id_type_; }
  void setCellIdDataType(CellIdType t) { cell_id_type_ = t; }

  virtual int getResolution(int res) const {
    check(mgpu_check_resolution(code(), res));
    return res;
  }
  virtual int getResolution(const std::string& res) const = 0;

  // pointToIndex(lon, lat, resolution): Long -- scalar form (a batch of one)
  int64_t pointToIndex(GpuContext& ctx, double lon, double lat, int resolution) const {
    const int r = getResolution(resolution);
    int64_t out = 0;
    check(mgpu_points_to_cells_host(ctx.get(), code(), r, &lon, &lat, 1, &out));
    return out;
  }
  // the batch form over device columns (x = lon / eastings, y = lat / northings)
  void pointsToIndex(GpuContext& ctx, const double* x_dev, const double* y_dev, int64_t n, int resolution,
                     int64_t* out_dev, void* stream = nullptr, mgpu_stats* stats = nullptr) const {
    const int r = getResolution(resolution);
    check(mgpu_points_to_cells(ctx.get(), code(), r, x_dev, y_dev, n, out_dev, stream, stats));
  }

  virtual std::string format(int64_t id) const = 0;
  virtual int64_t parse(const std::string& id) const = 0;

  // formatCellId(cellId, dt) for a Long cell id   (IndexSystem.scala:48-57)
  std::string formatCellIdString(int64_t id) const { return format(id); }
  int64_t formatCellIdLong(const std::string& id) const { return parse(id); }

 protected:
  explicit IndexSystem(CellIdType t) : cell_id_type_(t) {}

 private:
  CellIdType cell_id_type_;
};

// object H3IndexSystem extends IndexSystem(LongType)   (H3IndexSystem.scala:24)
class H3IndexSystem : public IndexSystem {
 public:
  H3IndexSystem() : IndexSystem(CellIdType::Long) {}
  std::string name() const override { return "H3"; }
  int32_t code() const override { return MGPU_H3; }
  int crsID() const override { return 4326; }
  std::vector<int> resolutions() const override {
    std::vector<int> r;
    for (int i = 0; i <= 15; i++) r.push_back(i);
    return r;
  }
  using IndexSystem::getResolution;
  int getResolution(const std::string& res) const override {
    size_t used = 0;
    int r = 0;
    try {
      r = std::stoi(res, &used);
    } catch (const std::exception&) {
      throw IllegalArgumentException("Resolution must be an Int or String.");
    }
    if (used != res.size()) throw IllegalArgumentException("Resolution must be an Int or String.");
    return getResolution(r);
  }
  // the H3 address string (lower-case hex), as h3.geoToH3Address
  std::string format(int64_t id) const override {
    char buf[32];
    snprintf(buf, sizeof buf, "%llx", (unsigned long long)id);
    return buf;
  }
  int64_t parse(const std::string& id) const override {
    size_t used = 0;
    unsigned long long v = 0;
    try {
      v = std::stoull(id, &used, 16);
    } catch (const std::exception&) {
      throw IllegalArgumentException("not an H3 address: " + id);
    }
    if (used != id.size()) throw IllegalArgumentException("not an H3 address: " + id);
    return (int64_t)v;
  }
};

// object BNGIndexSystem extends IndexSystem(StringType)   (BNGIndexSystem.scala:30)
class BNGIndexSystem : public IndexSystem {
 public:
  BNGIndexSystem() : IndexSystem(CellIdType::String) {}
  std::string name() const override { return "BNG"; }
  int32_t code() const override { return MGPU_BNG; }
  int crsID() const override { return 27700; }
  std::vector<int> resolutions() const override { return {1, -1, 2, -2, 3, -3, 4, -4, 5, -5, 6, -6}; }
  using IndexSystem::getResolution;
  // resolutionMap (BNGIndexSystem.scala:46-60)
  int getResolution(const std::string& res) const override {
    static const char* names[] = {"500km", "100km", "50km", "10km", "5km", "1km",
                                  "500m",  "100m",  "50m",  "10m",  "5m",  "1m"};
    static const int values[] = {-1, 1, -2, 2, -3, 3, -4, 4, -5, 5, -6, 6};
    for (int k = 0; k < 12; k++)
      if (res == names[k]) return values[k];
    throw IllegalStateException("BNG resolution not supported; found " + res);
  }
  std::string format(int64_t id) const override {
    char buf[32];
    int64_t off[2] = {0, 0};
    check(mgpu_bng_format(&id, 1, buf, sizeof buf, off));
    return std::string(buf + off[0], buf + off[1]);
  }
  int64_t parse(const std::string& id) const override {
    int64_t off[2] = {0, (int64_t)id.size()}, out = 0;
    check(mgpu_bng_parse(id.data(), off, 1, &out));
    return out;
  }
};

// IndexSystemFactory.getIndexSystem(name)   (IndexSystemFactory.scala:31-63)
inline std::unique_ptr<IndexSystem> getIndexSystem(const std::string& name) {
  std::string n;
  for (char c : name) n += (char)toupper((unsigned char)c);
  if (n == "H3") return std::make_unique<H3IndexSystem>();
  if (n == "BNG") return std::make_unique<BNGIndexSystem>();
  throw IllegalArgumentException("Index system " + name + " not supported by the MI355X path (H3, BNG)");
}

// Rows of grid_tessellateexplode: ChipType (is_core, index_id, wkb) + owning polygon id
struct ChipTable {
  int32_t index_system = MGPU_H3;
  std::vector<int64_t> cell;
  std::vector<int32_t> polygon_id;
  std::vector<uint8_t> is_core;
  std::vector<int64_t> wkb_offsets{0};
  std::vector<uint8_t> wkb;
  size_t size() const { return cell.size(); }
};

// Polygons as flat rings (mgpu_tessellate's layout)
struct Polygons {
  std::vector<int32_t> polygon_id;
  std::vector<int64_t> poly_part_off{0}, part_ring_off{0}, ring_off{0};
  std::vector<double> xy;
  // add a polygon given as parts -> rings -> closed (x, y) rings
  void add(int32_t id, const std::vector<std::vector<std::vector<std::pair<double, double>>>>& parts) {
    polygon_id.push_back(id);
    for (const auto& part : parts) {
      for (const auto& ring : part) {
        for (const auto& p : ring) {
          xy.push_back(p.first);
          xy.push_back(p.second);
        }
        ring_off.push_back((int64_t)xy.size() / 2);
      }
      part_ring_off.push_back((int64_t)ring_off.size() - 1);
    }
    poly_part_off.push_back((int64_t)part_ring_off.size() - 1);
  }
};

// grid_tessellateexplode(geometry, resolution, keepCoreGeometries)
inline ChipTable grid_tessellateexplode(const Polygons& P, const IndexSystem& is, int resolution,
                                        bool keep_core_geometries = true) {
  const int r = is.getResolution(resolution);
  mgpu_tess* t = nullptr;
  check(mgpu_tessellate(is.code(), r, (int64_t)P.polygon_id.size(), P.polygon_id.data(), P.poly_part_off.data(),
                        P.part_ring_off.data(), P.ring_off.data(), P.xy.data(), keep_core_geometries ? 1 : 0, &t));
  int64_t n = 0, bytes = 0;
  check(mgpu_tess_result_sizes(t, &n, &bytes));
  ChipTable c;
  c.index_system = is.code();
  c.cell.resize(n);
  c.polygon_id.resize(n);
  c.is_core.resize(n);
  c.wkb_offsets.resize(n + 1);
  c.wkb.resize(bytes);
  const int32_t st = mgpu_tess_result_copy(t, c.cell.data(), c.polygon_id.data(), c.is_core.data(),
                                           c.wkb_offsets.data(), c.wkb.data());
  mgpu_tess_destroy(t);
  check(st);
  return c;
}

// The uploaded chip table (WKB parsed once, cell index built)
class DeviceChips {
 public:
  DeviceChips(GpuContext& ctx, const ChipTable& c) {
    check(mgpu_chips_upload(ctx.get(), c.index_system, (int64_t)c.size(), c.cell.data(), c.polygon_id.data(),
                            c.is_core.data(), c.wkb_offsets.data(), c.wkb.data(), &chips_));
  }
  ~DeviceChips() { mgpu_chips_destroy(chips_); }
  DeviceChips(const DeviceChips&) = delete;
  DeviceChips& operator=(const DeviceChips&) = delete;
  const mgpu_chips* get() const { return chips_; }

 private:
  mgpu_chips* chips_ = nullptr;
};

// st_contains(chip.wkb, point) for explicit (chip row, point) pairs; device pointers
inline void st_contains(GpuContext& ctx, const DeviceChips& chips, const int64_t* chip_row_dev, const double* x_dev,
                        const double* y_dev, int64_t n, int8_t* out_dev, void* stream = nullptr) {
  check(mgpu_st_contains(ctx.get(), chips.get(), chip_row_dev, x_dev, y_dev, n, out_dev, stream));
}

struct JoinResult {
  std::vector<int64_t> point_id;
  std::vector<int32_t> polygon_id;
};

// The join over host columns (points copied in, pairs out; resized once on capacity)
inline JoinResult pipJoin(GpuContext& ctx, const DeviceChips& chips, const IndexSystem& is, int resolution,
                          const std::vector<double>& x, const std::vector<double>& y,
                          const std::vector<int64_t>* point_id = nullptr) {
  const int r = is.getResolution(resolution);
  const int64_t n = (int64_t)x.size();
  if ((int64_t)y.size() != n || (point_id && (int64_t)point_id->size() != n))
    throw IllegalArgumentException("coordinate / id columns differ in length");
  JoinResult res;
  int64_t cap = n + n / 8 + 16;
  for (int attempt = 0; attempt < 2; attempt++) {
    res.point_id.resize(cap);
    res.polygon_id.resize(cap);
    int64_t cnt = 0;
    const int32_t st = mgpu_pip_join_host(ctx.get(), chips.get(), is.code(), r, x.data(), y.data(),
                                          point_id ? point_id->data() : nullptr, n, cap, &cnt, res.point_id.data(),
                                          res.polygon_id.data());
    if (st == MGPU_E_CAPACITY && attempt == 0) {
      cap = cnt;
      continue;
    }
    check(st, cnt);
    res.point_id.resize(cnt);
    res.polygon_id.resize(cnt);
    return res;
  }
  throw DeviceError("pipJoin: capacity retry failed");
}

}  // namespace mosaic

#endif  // MOSAIC_INDEX_SYSTEM_HPP

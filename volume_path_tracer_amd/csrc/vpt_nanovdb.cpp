// vpt_nanovdb.cpp — NanoGrid<float> buffers and .nvdb files -> vpt_grid_desc (host C++).
//
// The reference keeps its volumes as nanovdb::GridHandle<HostBuffer> (include/vpt/volume_grids.hpp:12-33),
// read by nanovdb::io::readGrid(path, "density" | "temperature") (src/volume_grids.cpp:38-67).  The
// integrator's C ABI takes a flattened vpt_grid_desc; vpt_grid_from_nanovdb builds it from the grid's
// own memory (GridHandle::data(), i.e. &grid, grid.gridSize() bytes), so the reference side passes
// its grid unchanged.  NanoVDB is not in the reference tree (empty external/openvdb submodule), so
// the layout below is restated from NanoVDB 32.x (NanoVDB.h; float grids, NANOVDB_USE_SINGLE_ROOT_KEY),
// as volume_path_tracer_amd/nvdb.py does in Python -- parity with the real library is unpinned:
//
//   GridData     672 B  magic u64 @0, version u32 @16 (major = bits 21+, must be 32), gridSize u64 @32, Map {mMatF 9f, mInvMatF 9f, mVecF 3f} @296,
//                       gridClass u32 @632, gridType u32 @636 (1 = float)
//   TreeData      64 B  @672: node offsets i64 [leaf, lower, upper, root] from TreeData
//   RootData      64 B  bbox 6 i32, tableSize u32 @24, background f32 @28; then tableSize tiles of 32 B:
//                       key u64 (21 bits per axis of origin >> 12, x high), child i64 (from RootData,
//                       0 = tile), state u32, value f32
//   upper node  InternalData<.,5>: valueMask 4096 B @32, childMask 4096 B @4128, table of 32768 x 8 B
//                       @8256 (f32 value or i64 child offset from the node), slot n = i<<10 | j<<5 | k
//   lower node  InternalData<.,4>: valueMask 512 B @32, childMask 512 B @544, table 4096 x 8 B @1088,
//                       slot n = i<<8 | j<<4 | k
//   leaf        2144 B: valueMask 64 B @16, min/max/avg/std f32 @80, 512 f32 values @96 (n = x<<6|y<<3|z)
//
// A non-child slot of an internal node becomes a tile when it is active or its value differs from the
// background (ReadAccessor::getValue returns the slot value either way; probeValue reports the active
// bit).  Every offset is bounds-checked: a malformed buffer is VPT_E_INVALID, never a wild read.
#include <zlib.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "vpt_internal.h"

namespace vpt {

namespace {

constexpr uint64_t kMagicNumber = 0x304244566F6E614EULL;  // "NanoVDB0"
constexpr uint64_t kMagicGrid = 0x314244566F6E614EULL;    // "NanoVDB1"
constexpr uint64_t kMagicFile = 0x324244566F6E614EULL;    // "NanoVDB2"
constexpr uint32_t kGridTypeFloat = 1;
constexpr size_t kGridData = 672, kTreeData = 64, kRootData = 64, kRootTile = 32;
constexpr size_t kUpperMasks = 32, kUpperTable = 8256, kUpperSize = 8256 + 32768 * 8;
constexpr size_t kLowerMasks = 32, kLowerTable = 1088, kLowerSize = 1088 + 4096 * 8;
constexpr size_t kLeafMask = 16, kLeafMax = 84, kLeafValues = 96, kLeafSize = 96 + 512 * 4;
constexpr uint64_t kMaxGridBytes = 1ULL << 40;  // 1 TiB: larger is not a grid this host could hold

struct Buf {
  const uint8_t* p;
  size_t n;
  template <class T>
  T at(size_t off) const {
    T v;
    std::memcpy(&v, p + off, sizeof v);
    return v;
  }
  bool has(int64_t off, size_t len) const { return off >= 0 && (uint64_t)off <= n && len <= n - (size_t)off; }
  // base + rel when that stays inside the buffer with len bytes after it (offsets are untrusted)
  bool child(int64_t base, int64_t rel, size_t len, int64_t& out) const {
    return !__builtin_add_overflow(base, rel, &out) && has(out, len);
  }
  bool bit(size_t mask_off, uint32_t i) const { return (p[mask_off + (i >> 3)] >> (i & 7)) & 1; }
};

int bad(const std::string& m) { return set_error(VPT_E_INVALID, "NanoVDB grid buffer: " + m); }

void add_tile(OwnedGrid& o, int32_t x, int32_t y, int32_t z, int32_t level, float v, bool active) {
  o.tile_origin.insert(o.tile_origin.end(), {x, y, z});
  o.tile_level.push_back(level);
  o.tile_value.push_back(v);
  o.tile_active.push_back(active ? 1 : 0);
}

int flatten(const Buf& b, OwnedGrid& o) {
  if (b.n < kGridData + kTreeData) return bad("shorter than GridData + TreeData");
  const uint64_t magic = b.at<uint64_t>(0);
  if (magic != kMagicNumber && magic != kMagicGrid) return bad("bad magic");
  if ((b.at<uint32_t>(16) >> 21) != 32)  // GridData::mVersion: the layout above is NanoVDB 32.x's
    return bad("unsupported NanoVDB major version " + std::to_string(b.at<uint32_t>(16) >> 21));
  if (b.at<uint32_t>(636) != kGridTypeFloat) return bad("grid type is not float");
  const uint64_t grid_size = b.at<uint64_t>(32);
  if (grid_size > b.n) return bad("gridSize exceeds the buffer");
  vpt_grid_desc& d = o.d;
  std::memcpy(d.map_mat, b.p + 296, 36);
  std::memcpy(d.map_inv_mat, b.p + 332, 36);
  std::memcpy(d.map_vec, b.p + 368, 12);
  int64_t root;
  if (!b.child((int64_t)kGridData, b.at<int64_t>(kGridData + 24), kRootData, root)) return bad("root outside the buffer");
  for (int a = 0; a < 3; ++a) {
    d.index_bbox_min[a] = b.at<int32_t>(root + 4 * a);
    d.index_bbox_max[a] = b.at<int32_t>(root + 12 + 4 * a);
  }
  const uint32_t table = b.at<uint32_t>(root + 24);
  d.background = b.at<float>(root + 28);
  if (!b.has(root + (int64_t)kRootData, (size_t)table * kRootTile)) return bad("root table outside the buffer");
  if (table > (1u << 20)) return bad("implausible root table size");
  const float bg = d.background;
  {  // TreeData::mNodeCount[0], the leaf count: room for the leaves' copies up front (capped by the buffer)
    const uint64_t leaves = std::min<uint64_t>(b.at<uint32_t>(kGridData + 32), b.n / kLeafSize);
    o.leaf_values.reserve(leaves * 512);
    o.leaf_mask.reserve(leaves * 8);
    o.leaf_max.reserve(leaves);
    o.leaf_origin.reserve(leaves * 3);
  }
  for (uint32_t t = 0; t < table; ++t) {
    const int64_t e = root + (int64_t)kRootData + (int64_t)t * kRootTile;
    const uint64_t key = b.at<uint64_t>(e);
    const int64_t child = b.at<int64_t>(e + 8);
    const uint32_t state = b.at<uint32_t>(e + 16);
    const float value = b.at<float>(e + 20);
    int32_t org[3];
    for (int a = 0; a < 3; ++a) org[a] = (int32_t)(uint32_t)(((key >> (42 - 21 * a)) & 0x1FFFFF) << 12);
    if (child == 0) {
      add_tile(o, org[0], org[1], org[2], 3, value, state != 0);
      continue;
    }
    int64_t up;
    if (!b.child(root, child, kUpperSize, up)) return bad("upper node outside the buffer");
    o.upper_origin.insert(o.upper_origin.end(), {org[0], org[1], org[2]});
    const size_t uvm = (size_t)up + kUpperMasks, ucm = uvm + 4096;
    for (uint32_t n = 0; n < 32768; ++n) {
      if (b.bit(ucm, n)) continue;
      const float v = b.at<float>(up + kUpperTable + 8 * n);
      const bool act = b.bit(uvm, n);
      if (act || v != bg)
        add_tile(o, org[0] + (int32_t)((n >> 10) << 7), org[1] + (int32_t)(((n >> 5) & 31) << 7),
                 org[2] + (int32_t)((n & 31) << 7), 2, v, act);
    }
    for (uint32_t n = 0; n < 32768; ++n) {
      if (!b.bit(ucm, n)) continue;
      int64_t lo;
      if (!b.child(up, b.at<int64_t>(up + kUpperTable + 8 * n), kLowerSize, lo)) return bad("lower node outside the buffer");
      const int32_t lorg[3] = {org[0] + (int32_t)((n >> 10) << 7), org[1] + (int32_t)(((n >> 5) & 31) << 7),
                               org[2] + (int32_t)((n & 31) << 7)};
      o.lower_origin.insert(o.lower_origin.end(), {lorg[0], lorg[1], lorg[2]});
      const size_t lvm = (size_t)lo + kLowerMasks, lcm = lvm + 512;
      for (uint32_t m = 0; m < 4096; ++m) {
        if (b.bit(lcm, m)) continue;
        const float v = b.at<float>(lo + kLowerTable + 8 * m);
        const bool act = b.bit(lvm, m);
        if (act || v != bg)
          add_tile(o, lorg[0] + (int32_t)((m >> 8) << 3), lorg[1] + (int32_t)(((m >> 4) & 15) << 3),
                   lorg[2] + (int32_t)((m & 15) << 3), 1, v, act);
      }
      for (uint32_t m = 0; m < 4096; ++m) {
        if (!b.bit(lcm, m)) continue;
        int64_t lf;
        if (!b.child(lo, b.at<int64_t>(lo + kLowerTable + 8 * m), kLeafSize, lf)) return bad("leaf outside the buffer");
        o.leaf_origin.insert(o.leaf_origin.end(), {lorg[0] + (int32_t)((m >> 8) << 3),
                                                   lorg[1] + (int32_t)(((m >> 4) & 15) << 3),
                                                   lorg[2] + (int32_t)((m & 15) << 3)});
        const size_t v0 = o.leaf_values.size();
        o.leaf_values.resize(v0 + 512);
        std::memcpy(o.leaf_values.data() + v0, b.p + lf + kLeafValues, 512 * 4);
        const size_t m0 = o.leaf_mask.size();
        o.leaf_mask.resize(m0 + 8);
        std::memcpy(o.leaf_mask.data() + m0, b.p + lf + kLeafMask, 64);
        o.leaf_max.push_back(b.at<float>(lf + kLeafMax));
      }
    }
  }
  o.finish();
  return VPT_OK;
}

// One grid blob of a .nvdb file: codec NONE (raw) or ZIP (u64 compressed size + zlib stream).
int read_blob(const std::vector<uint8_t>& f, size_t& pos, uint16_t codec, uint64_t grid_size, const std::string& name,
              std::vector<uint8_t>* out) {
  if (codec == 0) {
    if (grid_size > f.size() - pos) return set_error(VPT_E_INVALID, "nvdb: grid '" + name + "' truncated");
    if (out) out->assign(f.begin() + (ptrdiff_t)pos, f.begin() + (ptrdiff_t)(pos + grid_size));
    pos += grid_size;
    return VPT_OK;
  }
  if (codec != 1) return set_error(VPT_E_INVALID, "nvdb: grid '" + name + "': codec " + std::to_string(codec) + " (BLOSC) is not supported");
  if (f.size() - pos < 8) return set_error(VPT_E_INVALID, "nvdb: grid '" + name + "' truncated");
  uint64_t n;
  std::memcpy(&n, f.data() + pos, 8);
  if (n > f.size() - pos - 8) return set_error(VPT_E_INVALID, "nvdb: grid '" + name + "' truncated");
  // gridSize comes from the file: bound it before allocating (deflate expands at most ~1032:1)
  if (out && (grid_size > kMaxGridBytes || grid_size > 1032 * (n + 64)))
    return set_error(VPT_E_INVALID, "nvdb: grid '" + name + "': implausible gridSize " + std::to_string(grid_size));
  if (out) {
    out->resize(grid_size);
    uLongf len = (uLongf)grid_size;
    if (uncompress(out->data(), &len, f.data() + pos + 8, (uLong)n) != Z_OK || len != grid_size)
      return set_error(VPT_E_INVALID, "nvdb: grid '" + name + "': bad zlib stream");
  }
  pos += 8 + n;
  return VPT_OK;
}

}  // namespace
}  // namespace vpt

extern "C" int vpt_grid_from_nanovdb(const void* grid_buffer, size_t bytes, vpt_grid_desc** out) {
  if (!grid_buffer || !out) return vpt::set_error(VPT_E_INVALID, "vpt_grid_from_nanovdb: null argument");
  *out = nullptr;
  try {  // no C++ exception crosses the C ABI (allocation failures of a huge grid)
    std::unique_ptr<vpt::OwnedGrid> o(vpt::owned_grid_new());
    const int rc = vpt::flatten(vpt::Buf{static_cast<const uint8_t*>(grid_buffer), bytes}, *o);
    if (rc) return rc;
    *out = &o.release()->d;
    return VPT_OK;
  } catch (const std::bad_alloc&) {
    return vpt::set_error(VPT_E_NOMEM, "vpt_grid_from_nanovdb: out of host memory");
  } catch (const std::exception& e) {
    return vpt::set_error(VPT_E_INVALID, std::string("vpt_grid_from_nanovdb: ") + e.what());
  }
}

// nanovdb::io::readGrid(path, name) for float grids (src/volume_grids.cpp:38-46): file segments
// (FileHeader 16 B: magic, version, gridCount u16, codec u16; gridCount x (FileMetaData 176 B: gridSize
// @0, gridType @32, nameSize @136, codec @168; name); then the grid blobs).
static int read_nvdb(const char* path, const char* grid_name, vpt_grid_desc** out);

extern "C" int vpt_grid_read_nvdb(const char* path, const char* grid_name, vpt_grid_desc** out) {
  if (!path || !grid_name || !out) return vpt::set_error(VPT_E_INVALID, "vpt_grid_read_nvdb: null argument");
  *out = nullptr;
  try {  // no C++ exception crosses the C ABI
    return read_nvdb(path, grid_name, out);
  } catch (const std::bad_alloc&) {
    return vpt::set_error(VPT_E_NOMEM, "vpt_grid_read_nvdb: out of host memory");
  } catch (const std::exception& e) {
    return vpt::set_error(VPT_E_INVALID, std::string("vpt_grid_read_nvdb: ") + e.what());
  }
}

static int read_nvdb(const char* path, const char* grid_name, vpt_grid_desc** out) {
  std::ifstream in(path, std::ios::binary);
  if (!in) return vpt::set_error(VPT_E_IO, std::string("vpt_grid_read_nvdb: cannot open ") + path);
  std::vector<uint8_t> f((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  size_t pos = 0;
  bool first = true;
  while (f.size() - pos >= 16) {
    uint64_t magic;
    uint32_t version;
    uint16_t count, codec;
    std::memcpy(&magic, f.data() + pos, 8);
    std::memcpy(&version, f.data() + pos + 8, 4);
    std::memcpy(&count, f.data() + pos + 12, 2);
    std::memcpy(&codec, f.data() + pos + 14, 2);
    if (magic != vpt::kMagicNumber && magic != vpt::kMagicFile) {
      if (first) return vpt::set_error(VPT_E_INVALID, std::string("vpt_grid_read_nvdb: not a NanoVDB file: ") + path);
      break;
    }
    if ((version >> 21) != 32)
      return vpt::set_error(VPT_E_INVALID, "vpt_grid_read_nvdb: unsupported NanoVDB major version " + std::to_string(version >> 21));
    first = false;
    pos += 16;
    struct Meta {
      std::string name;
      uint64_t size;
      uint32_t type;
      uint16_t codec;
    };
    std::vector<Meta> metas;
    for (uint16_t g = 0; g < count; ++g) {
      if (f.size() - pos < 176) return vpt::set_error(VPT_E_INVALID, "vpt_grid_read_nvdb: truncated metadata");
      Meta m;
      uint32_t name_size;
      std::memcpy(&m.size, f.data() + pos, 8);
      std::memcpy(&m.type, f.data() + pos + 32, 4);
      std::memcpy(&name_size, f.data() + pos + 136, 4);
      std::memcpy(&m.codec, f.data() + pos + 168, 2);
      pos += 176;
      if (name_size > f.size() - pos) return vpt::set_error(VPT_E_INVALID, "vpt_grid_read_nvdb: truncated name");
      m.name.assign(reinterpret_cast<const char*>(f.data() + pos), strnlen(reinterpret_cast<const char*>(f.data() + pos), name_size));
      pos += name_size;
      metas.push_back(m);
    }
    for (const Meta& m : metas) {
      const bool want = m.name == grid_name;
      std::vector<uint8_t> blob;
      int rc = vpt::read_blob(f, pos, m.codec, m.size, m.name, want ? &blob : nullptr);
      if (rc) return rc;
      if (!want) continue;
      if (m.type != vpt::kGridTypeFloat)
        return vpt::set_error(VPT_E_INVALID, "vpt_grid_read_nvdb: grid '" + m.name + "' is not a float grid");
      return vpt_grid_from_nanovdb(blob.data(), blob.size(), out);
    }
  }
  return VPT_OK;  // no grid of that name: *out stays NULL (the reference's nanovdb_try_read_grid)
}

extern "C" void vpt_grid_free(vpt_grid_desc* d) { delete reinterpret_cast<vpt::OwnedGrid*>(d); }

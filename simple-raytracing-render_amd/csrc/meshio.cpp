// Mesh files -> triangles with the semantics of the reference's model loader
// (model.h:27-102, geometry.h:24-90, assimp with aiProcess_Triangulate |
// JoinIdenticalVertices | SortByPType [| FlipUVs] [| FlipWindingOrder]):
//   * only the first mesh is used (model::genhitablemodel returns mesh 0);
//   * positions are scaled component-wise;
//   * UVs come from channel 0 (uv.z = 0); FlipUVs maps v -> 1 - v;
//   * FlipWindingOrder reverses each face's index order;
//   * polygons are triangulated as a fan from their first corner (convex faces);
//   * build definition: the reference reads normals only when the
//     file has UVs and otherwise indexes an empty vector (undefined); here a
//     face without file normals gets its face normal, like the teapot (Q5).
// The assimp binaries the reference ships are Win32 only, so no parity vector
// pins these loaders; tests/test_meshio.py checks them on synthetic files.
#include "meshio.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>

namespace srr {

namespace {

struct PlyProp {
  std::string name;
  std::string type;       // scalar type, or list item type
  std::string list_type;  // count type for lists, "" for scalars
};

struct PlyElement {
  std::string name;
  long long count = 0;
  std::vector<PlyProp> props;
};

int type_size(const std::string& t) {
  if (t == "char" || t == "int8" || t == "uchar" || t == "uint8") return 1;
  if (t == "short" || t == "int16" || t == "ushort" || t == "uint16") return 2;
  if (t == "int" || t == "int32" || t == "uint" || t == "uint32" || t == "float" || t == "float32") return 4;
  if (t == "double" || t == "float64") return 8;
  return 0;
}

double read_binary(const unsigned char* p, const std::string& t, bool big) {
  unsigned char b[8];
  const int n = type_size(t);
  for (int i = 0; i < n; ++i) b[i] = big ? p[n - 1 - i] : p[i];
  if (t == "char" || t == "int8") return (double)(int8_t)b[0];
  if (t == "uchar" || t == "uint8") return (double)b[0];
  if (t == "short" || t == "int16") { int16_t v; std::memcpy(&v, b, 2); return v; }
  if (t == "ushort" || t == "uint16") { uint16_t v; std::memcpy(&v, b, 2); return v; }
  if (t == "int" || t == "int32") { int32_t v; std::memcpy(&v, b, 4); return v; }
  if (t == "uint" || t == "uint32") { uint32_t v; std::memcpy(&v, b, 4); return v; }
  if (t == "float" || t == "float32") { float v; std::memcpy(&v, b, 4); return v; }
  double v;
  std::memcpy(&v, b, 8);
  return v;
}

}  // namespace

int load_ply(const std::string& path, MeshData& out, std::string& err) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return err = "cannot open " + path, -1;
  std::string line;
  std::getline(f, line);
  if (line.rfind("ply", 0) != 0) return err = path + ": not a PLY file", -1;
  std::string format;
  std::vector<PlyElement> elems;
  for (;;) {
    if (!std::getline(f, line)) return err = path + ": truncated header", -1;
    if (!line.empty() && line.back() == '\r') line.pop_back();
    std::istringstream ls(line);
    std::string kw;
    ls >> kw;
    if (kw == "format") {
      ls >> format;
    } else if (kw == "element") {
      PlyElement e;
      ls >> e.name >> e.count;
      elems.push_back(e);
    } else if (kw == "property") {
      if (elems.empty()) return err = path + ": property before element", -1;
      PlyProp p;
      std::string t;
      ls >> t;
      if (t == "list") ls >> p.list_type >> p.type >> p.name;
      else { p.type = t; ls >> p.name; }
      if (!type_size(p.type) || (!p.list_type.empty() && !type_size(p.list_type)))
        return err = path + ": unsupported property type in '" + line + "'", -1;
      elems.back().props.push_back(p);
    } else if (kw == "end_header") {
      break;
    }
  }
  const bool ascii = format == "ascii";
  const bool big = format == "binary_big_endian";
  if (!ascii && format != "binary_little_endian" && !big) return err = path + ": unknown format " + format, -1;
  std::vector<float> pos, nrm, uv;
  bool has_n = false, has_uv = false;
  std::vector<std::vector<int>> faces;
  std::vector<unsigned char> buf;
  auto read_value = [&](const std::string& t, double& v) -> bool {
    if (ascii) return (bool)(f >> v);
    const int n = type_size(t);
    unsigned char b[8];
    if (!f.read((char*)b, n)) return false;
    v = read_binary(b, t, big);
    return true;
  };
  for (const PlyElement& e : elems) {
    const bool is_v = e.name == "vertex", is_f = e.name == "face";
    int ix = -1, iy = -1, iz = -1, inx = -1, iny = -1, inz = -1, iu = -1, iv = -1, ilist = -1;
    for (size_t k = 0; k < e.props.size(); ++k) {
      const std::string& n = e.props[k].name;
      if (n == "x") ix = (int)k;
      else if (n == "y") iy = (int)k;
      else if (n == "z") iz = (int)k;
      else if (n == "nx") inx = (int)k;
      else if (n == "ny") iny = (int)k;
      else if (n == "nz") inz = (int)k;
      else if (n == "u" || n == "s" || n == "texture_u" || n == "texture_s") iu = (int)k;
      else if (n == "v" || n == "t" || n == "texture_v" || n == "texture_t") iv = (int)k;
      else if (n == "vertex_indices" || n == "vertex_index") ilist = (int)k;
    }
    if (is_v) {
      has_n = inx >= 0 && iny >= 0 && inz >= 0;
      has_uv = iu >= 0 && iv >= 0;
      if (ix < 0 || iy < 0 || iz < 0) return err = path + ": vertex element without x y z", -1;
    }
    std::vector<double> vals(e.props.size());
    for (long long r = 0; r < e.count; ++r) {
      std::vector<int> idx;
      for (size_t k = 0; k < e.props.size(); ++k) {
        const PlyProp& p = e.props[k];
        if (!p.list_type.empty()) {
          double cnt;
          if (!read_value(p.list_type, cnt)) return err = path + ": truncated " + e.name, -1;
          for (long long q = 0; q < (long long)cnt; ++q) {
            double x;
            if (!read_value(p.type, x)) return err = path + ": truncated " + e.name, -1;
            if ((int)k == ilist) idx.push_back((int)x);
          }
        } else if (!read_value(p.type, vals[k])) {
          return err = path + ": truncated " + e.name, -1;
        }
      }
      if (is_v) {
        pos.insert(pos.end(), {(float)vals[ix], (float)vals[iy], (float)vals[iz]});
        if (has_n) nrm.insert(nrm.end(), {(float)vals[inx], (float)vals[iny], (float)vals[inz]});
        if (has_uv) uv.insert(uv.end(), {(float)vals[iu], (float)vals[iv], 0.f});
      } else if (is_f) {
        faces.push_back(idx);
      }
    }
  }
  out = MeshData{};
  const long long nv = (long long)pos.size() / 3;
  for (const std::vector<int>& face : faces) {
    for (int v : face)
      if (v < 0 || v >= nv) return err = path + ": face index out of range", -1;
    for (size_t k = 1; k + 1 < face.size(); ++k) {  // fan triangulation
      const int c[3] = {face[0], face[k], face[k + 1]};
      MeshData::Corner tri[3];
      for (int j = 0; j < 3; ++j) {
        std::memcpy(tri[j].p, &pos[3 * (size_t)c[j]], 12);
        if (has_n) std::memcpy(tri[j].n, &nrm[3 * (size_t)c[j]], 12);
        if (has_uv) std::memcpy(tri[j].uv, &uv[3 * (size_t)c[j]], 12);
      }
      out.tris.push_back({tri[0], tri[1], tri[2]});
    }
  }
  out.has_normals = has_n;
  out.has_uvs = has_uv;
  return 0;
}

int load_mesh_file(const std::string& path, MeshData& out, std::string& err) {
  std::string ext;
  const size_t dot = path.find_last_of('.');
  if (dot != std::string::npos) ext = path.substr(dot + 1);
  std::transform(ext.begin(), ext.end(), ext.begin(), ::tolower);
  if (ext == "ply") return load_ply(path, out, err);
  if (ext == "fbx") return load_fbx(path, out, err);
  err = path + ": unsupported mesh format (PLY and FBX are)";
  return -1;
}

void apply_model_semantics(MeshData& m, bool flip_uvs, bool flip_winding, const float scale[3]) {
  for (auto& t : m.tris) {
    if (flip_winding) std::swap(t[0], t[2]);  // aiProcess_FlipWindingOrder
    for (auto& c : t) {
      for (int a = 0; a < 3; ++a) c.p[a] = c.p[a] * scale[a];  // geometry.h:65
      if (flip_uvs) c.uv[1] = 1.0f - c.uv[1];                   // aiProcess_FlipUVs
    }
  }
}

}  // namespace srr

// Binary FBX (7.x) geometry reader for the reference's model loader path
// (model.h:27-60 through assimp's FBX importer).
//
// Format: a 27-byte header ("Kaydara FBX Binary  \0\x1a\0" + uint32 version),
// then node records {end offset, property count, property bytes, name, properties,
// nested records} with 32-bit fields before version 7500 and 64-bit after; a
// nested list ends with an all-zero record.  Array properties (f d l i b) may be
// zlib-deflated.
//
// Mesh selection follows assimp's converter: models are visited depth-first from
// the scene root along the "OO" connections in file order, and the first
// Geometry attached to a model is mesh 0 (model::genhitablemodel uses mesh 0
// only).  A mesh whose polygons carry several materials is split by material in
// assimp; mesh 0 is then the lowest material index.  Per-corner attributes follow
// the layer mapping (ByPolygonVertex / ByVertice / ByPolygon / AllSame) and
// reference mode (Direct / IndexToDirect).
#include <zlib.h>

#include <algorithm>
#include <cstring>
#include <fstream>
#include <functional>
#include <map>
#include <memory>

#include "meshio.h"

namespace srr {

namespace {

struct FbxProp {
  char type = 0;
  int64_t i = 0;
  double d = 0;
  std::string s;
  std::vector<double> arr_d;   // f d arrays
  std::vector<int64_t> arr_i;  // i l b arrays
};

struct FbxNode {
  std::string name;
  std::vector<FbxProp> props;
  std::vector<std::unique_ptr<FbxNode>> kids;
  const FbxNode* child(const char* n) const {
    for (auto& k : kids)
      if (k->name == n) return k.get();
    return nullptr;
  }
};

struct Reader {
  const std::vector<unsigned char>& b;
  size_t pos = 0;
  bool wide = false;  // version >= 7500: 64-bit record fields
  std::string err;
  explicit Reader(const std::vector<unsigned char>& buf) : b(buf) {}
  bool need(size_t n) {
    if (pos + n > b.size()) {
      err = "truncated FBX";
      return false;
    }
    return true;
  }
  template <class T>
  bool get(T& v) {
    if (!need(sizeof(T))) return false;
    std::memcpy(&v, &b[pos], sizeof(T));
    pos += sizeof(T);
    return true;
  }
  bool array(char t, FbxProp& p) {
    uint32_t len, enc, clen;
    if (!get(len) || !get(enc) || !get(clen) || !need(clen)) return false;
    const int es = (t == 'd' || t == 'l') ? 8 : (t == 'b' ? 1 : 4);
    std::vector<unsigned char> raw((size_t)len * es);
    if (enc == 0) {
      if (clen != raw.size()) return err = "FBX array length mismatch", false;
      std::memcpy(raw.data(), &b[pos], clen);
    } else if (enc == 1) {
      uLongf out = (uLongf)raw.size();
      if (uncompress(raw.data(), &out, &b[pos], clen) != Z_OK || out != raw.size())
        return err = "FBX array inflate failed", false;
    } else {
      return err = "FBX array encoding unknown", false;
    }
    pos += clen;
    for (uint32_t k = 0; k < len; ++k) {
      const unsigned char* e = &raw[(size_t)k * es];
      if (t == 'f') { float v; std::memcpy(&v, e, 4); p.arr_d.push_back(v); }
      else if (t == 'd') { double v; std::memcpy(&v, e, 8); p.arr_d.push_back(v); }
      else if (t == 'i') { int32_t v; std::memcpy(&v, e, 4); p.arr_i.push_back(v); }
      else if (t == 'l') { int64_t v; std::memcpy(&v, e, 8); p.arr_i.push_back(v); }
      else p.arr_i.push_back(e[0]);
    }
    return true;
  }
  bool prop(FbxProp& p) {
    if (!get(p.type)) return false;
    switch (p.type) {
      case 'Y': { int16_t v; if (!get(v)) return false; p.i = v; return true; }
      case 'C': { uint8_t v; if (!get(v)) return false; p.i = v; return true; }
      case 'I': { int32_t v; if (!get(v)) return false; p.i = v; return true; }
      case 'L': { int64_t v; if (!get(v)) return false; p.i = v; return true; }
      case 'F': { float v; if (!get(v)) return false; p.d = v; return true; }
      case 'D': { double v; if (!get(v)) return false; p.d = v; return true; }
      case 'f': case 'd': case 'l': case 'i': case 'b': return array(p.type, p);
      case 'S': case 'R': {
        uint32_t n;
        if (!get(n) || !need(n)) return false;
        p.s.assign((const char*)&b[pos], n);
        pos += n;
        return true;
      }
    }
    err = std::string("FBX property type '") + p.type + "' unknown";
    return false;
  }
  // one node record; returns false on error; *null set for the list terminator
  bool node(FbxNode& n, bool& null) {
    uint64_t end, nprops, plen;
    uint8_t nlen;
    if (wide) {
      if (!get(end) || !get(nprops) || !get(plen)) return false;
    } else {
      uint32_t e32, n32, p32;
      if (!get(e32) || !get(n32) || !get(p32)) return false;
      end = e32, nprops = n32, plen = p32;
    }
    if (!get(nlen)) return false;
    null = end == 0;
    if (null) return true;
    if (!need(nlen)) return false;
    n.name.assign((const char*)&b[pos], nlen);
    pos += nlen;
    for (uint64_t k = 0; k < nprops; ++k) {
      FbxProp p;
      if (!prop(p)) return false;
      n.props.push_back(std::move(p));
    }
    while (pos < end) {
      auto kid = std::make_unique<FbxNode>();
      bool kn;
      if (!node(*kid, kn)) return false;
      if (kn) break;
      n.kids.push_back(std::move(kid));
    }
    if (end > b.size()) return err = "FBX record past end of file", false;
    pos = end;
    return true;
  }
};

std::string str_prop(const FbxNode* n, size_t k = 0) {
  return n && n->props.size() > k ? n->props[k].s : std::string();
}

}  // namespace

int load_fbx(const std::string& path, MeshData& out, std::string& err) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return err = "cannot open " + path, -1;
  std::vector<unsigned char> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  static const char kMagic[] = "Kaydara FBX Binary  ";
  if (buf.size() < 27 || std::memcmp(buf.data(), kMagic, 20) != 0)
    return err = path + ": not a binary FBX file", -1;
  uint32_t version;
  std::memcpy(&version, &buf[23], 4);
  Reader rd(buf);
  rd.pos = 27;
  rd.wide = version >= 7500;
  FbxNode root;
  for (;;) {
    auto n = std::make_unique<FbxNode>();
    bool null;
    if (!rd.node(*n, null)) return err = path + ": " + rd.err, -1;
    if (null) break;
    root.kids.push_back(std::move(n));
    if (rd.pos >= buf.size()) break;
  }
  const FbxNode* objects = root.child("Objects");
  if (!objects) return err = path + ": no Objects section", -1;
  std::map<int64_t, const FbxNode*> geometry, model;
  for (auto& o : objects->kids) {
    if (o->props.empty()) continue;
    if (o->name == "Geometry" && str_prop(o.get(), 2) == "Mesh") geometry[o->props[0].i] = o.get();
    if (o->name == "Model") model[o->props[0].i] = o.get();
  }
  // object graph: parent -> children in file order ("C", "OO", child, parent)
  std::map<int64_t, std::vector<int64_t>> kids;
  if (const FbxNode* con = root.child("Connections"))
    for (auto& c : con->kids)
      if (c->name == "C" && c->props.size() >= 3 && c->props[0].s == "OO") kids[c->props[2].i].push_back(c->props[1].i);
  const FbxNode* geo = nullptr;
  std::function<void(int64_t)> visit = [&](int64_t id) {
    auto it = kids.find(id);
    if (it == kids.end() || geo) return;
    for (int64_t k : it->second)  // the model's own geometry first, then child models
      if (!geo && model.count(id) && geometry.count(k)) geo = geometry[k];
    for (int64_t k : it->second)
      if (!geo && model.count(k)) visit(k);
  };
  visit(0);
  if (!geo && !geometry.empty()) geo = geometry.begin()->second;
  if (!geo) return err = path + ": no mesh geometry", -1;

  const FbxNode* vn = geo->child("Vertices");
  const FbxNode* pn = geo->child("PolygonVertexIndex");
  if (!vn || !pn || vn->props.empty() || pn->props.empty()) return err = path + ": geometry without vertices", -1;
  const std::vector<double>& V = vn->props[0].arr_d;
  const std::vector<int64_t>& PI = pn->props[0].arr_i;
  // polygons: corner ranges in PolygonVertexIndex (negative index closes a polygon)
  std::vector<std::pair<size_t, size_t>> polys;
  for (size_t k = 0, s = 0; k < PI.size(); ++k)
    if (PI[k] < 0) {
      polys.emplace_back(s, k + 1);
      s = k + 1;
    }
  auto vertex_of = [&](size_t corner) { return PI[corner] < 0 ? -PI[corner] - 1 : PI[corner]; };
  // a layer element's value for (polygon, corner, vertex)
  struct Layer {
    std::string mapping, ref;
    const std::vector<double>* data = nullptr;
    const std::vector<int64_t>* index = nullptr;
    int width = 0;
  };
  auto layer = [&](const char* elem, const char* dname, const char* iname, int width) {
    Layer L;
    const FbxNode* e = geo->child(elem);
    if (!e) return L;
    L.mapping = str_prop(e->child("MappingInformationType"));
    L.ref = str_prop(e->child("ReferenceInformationType"));
    const FbxNode* d = e->child(dname);
    const FbxNode* ix = e->child(iname);
    if (d && !d->props.empty()) L.data = &d->props[0].arr_d;
    if (ix && !ix->props.empty()) L.index = &ix->props[0].arr_i;
    L.width = width;
    return L;
  };
  auto fetch = [&](const Layer& L, size_t poly, size_t corner, int64_t vtx, float* o) {
    if (!L.data) return false;
    int64_t k = (L.mapping == "ByPolygonVertex") ? (int64_t)corner
                : (L.mapping == "ByVertice" || L.mapping == "ByVertex") ? vtx
                : (L.mapping == "ByPolygon") ? (int64_t)poly : 0;
    if (L.ref == "IndexToDirect" || L.ref == "Index") {
      if (!L.index || k < 0 || k >= (int64_t)L.index->size()) return false;
      k = (*L.index)[(size_t)k];
    }
    if (k < 0 || (size_t)(k + 1) * L.width > L.data->size()) return false;
    for (int a = 0; a < L.width; ++a) o[a] = (float)(*L.data)[(size_t)k * L.width + a];
    return true;
  };
  const Layer nl = layer("LayerElementNormal", "Normals", "NormalsIndex", 3);
  const Layer ul = layer("LayerElementUV", "UV", "UVIndex", 2);
  // material split (assimp: one mesh per material; mesh 0 = lowest index)
  std::vector<int64_t> pmat(polys.size(), 0);
  if (const FbxNode* me = geo->child("LayerElementMaterial")) {
    const FbxNode* m = me->child("Materials");
    const std::string mapping = str_prop(me->child("MappingInformationType"));
    if (m && !m->props.empty() && mapping == "ByPolygon")
      for (size_t p = 0; p < polys.size() && p < m->props[0].arr_i.size(); ++p) pmat[p] = m->props[0].arr_i[p];
  }
  int64_t mesh_mat = polys.empty() ? 0 : *std::min_element(pmat.begin(), pmat.end());
  out = MeshData{};
  out.has_normals = nl.data != nullptr;
  out.has_uvs = ul.data != nullptr;
  const int64_t nvert = (int64_t)V.size() / 3;
  for (size_t p = 0; p < polys.size(); ++p) {
    if (pmat[p] != mesh_mat) continue;
    auto corner = [&](size_t c) {
      MeshData::Corner k{};
      const int64_t v = vertex_of(c);
      if (v >= 0 && v < nvert)
        for (int a = 0; a < 3; ++a) k.p[a] = (float)V[(size_t)v * 3 + a];
      float t[3] = {0, 0, 0};
      if (fetch(nl, p, c, v, t)) std::memcpy(k.n, t, 12);
      float uv[2] = {0, 0};
      if (fetch(ul, p, c, v, uv)) { k.uv[0] = uv[0]; k.uv[1] = uv[1]; }
      return k;
    };
    const size_t s = polys[p].first, e = polys[p].second;
    for (size_t c = s + 1; c + 1 < e; ++c) {  // fan from the polygon's first corner
      for (size_t q : {s, c, c + 1})
        if (vertex_of(q) < 0 || vertex_of(q) >= nvert) return err = path + ": vertex index out of range", -1;
      out.tris.push_back({corner(s), corner(c), corner(c + 1)});
    }
  }
  return 0;
}

}  // namespace srr

// Mesh files (PLY, binary FBX) -> triangle corners, with the reference model
// loader's semantics (model.h, geometry.h); see meshio.cpp and fbx.cpp.
#pragma once
#include <array>
#include <string>
#include <vector>

namespace srr {

struct MeshData {
  struct Corner {
    float p[3] = {0, 0, 0};
    float n[3] = {0, 0, 0};
    float uv[3] = {0, 0, 0};  // uv.z = 0 (assimp's 2-component channels)
  };
  std::vector<std::array<Corner, 3>> tris;
  bool has_normals = false, has_uvs = false;
};

int load_ply(const std::string& path, MeshData& out, std::string& err);
int load_fbx(const std::string& path, MeshData& out, std::string& err);
int load_mesh_file(const std::string& path, MeshData& out, std::string& err);  // by extension
void apply_model_semantics(MeshData& m, bool flip_uvs, bool flip_winding, const float scale[3]);

}  // namespace srr

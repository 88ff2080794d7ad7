// Link stub for the three Assimp::Importer symbols model.h references.  The
// vendored assimp binaries are Win32-only, so model.h-based scenes (FBX/PLY
// import) are unavailable to the oracle; ReadFile returns nullptr.
// TEST INFRASTRUCTURE ONLY (see oracle/ref/shim.h).
#include <assimp/Importer.hpp>

namespace Assimp {
Importer::Importer() : pimpl(nullptr) {}
Importer::~Importer() {}
const aiScene* Importer::ReadFile(const char*, unsigned int) { return nullptr; }
}  // namespace Assimp

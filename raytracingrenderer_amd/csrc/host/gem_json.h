// gem_json.h — scene.json and .gem readers with RTBase's GEMLoader semantics
// (RTBase/GEMLoader.h:40-750; MIT-licensed course loader, re-implemented here).
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace rth {

// GEMProperty (GEMLoader.h:40-115): a name and the string form of a JSON value.
struct Property {
    std::string name, value;
    bool present = false;
    std::string str() const { return value; }
    float as_float(float dflt) const;   // std::stof with fallback
    int as_int(int dflt) const;         // std::stoi with fallback
    void as_vec3(float& x, float& y, float& z, float dflt = 0.0f) const;  // split on ' '
};

struct PropertyList {
    std::vector<Property> props;
    Property find(const std::string& name) const;  // first match, else empty "not found"
};

struct Instance {
    float world[16] = {0};
    std::string mesh;
    PropertyList material;
};

struct SceneFile {
    std::vector<Instance> instances;
    PropertyList properties;
};

bool parse_scene_json(const std::string& path, SceneFile& out, std::string& err);

struct GemVertex {  // GEMStaticVertex, 44 bytes on disk
    float pos[3], normal[3], tangent[3], u, v;
};
struct GemMesh {
    std::vector<GemVertex> vertices;
    std::vector<uint32_t> indices;
};
// GEMModelLoader::load (GEMLoader.h:344-365); returns false with err on a missing/bad file
// (the reference calls exit(0) there).
bool load_gem(const std::string& path, std::vector<GemMesh>& meshes, std::string& err);
bool write_gem(const std::string& path, const std::vector<GemVertex>& verts,
               const std::vector<uint32_t>& indices, std::string& err);

}  // namespace rth

// gem_json.cpp — see gem_json.h. The JSON dialect is the course loader's: numbers are parsed as
// float by strtof on their literal text, strings carry no escapes, a top-level array is a list of
// instances, every other top-level value becomes a scene property in its string form
// (numbers via std::to_string, i.e. "%f"), and object keys are visited in sorted order.
#include "gem_json.h"

#include <cctype>
#include <cerrno>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

namespace rth {

float Property::as_float(float dflt) const {
    const char* s = value.c_str();
    char* end = nullptr;
    errno = 0;
    float v = std::strtof(s, &end);
    if (end == s || errno == ERANGE) return dflt;
    return v;
}

int Property::as_int(int dflt) const {
    const char* s = value.c_str();
    char* end = nullptr;
    errno = 0;
    long v = std::strtol(s, &end, 10);
    if (end == s || errno == ERANGE || v < INT_MIN || v > INT_MAX) return dflt;
    return (int)v;
}

void Property::as_vec3(float& x, float& y, float& z, float dflt) const {
    // std::getline(ss, word, ' ') semantics: empty tokens between separators are kept, a
    // trailing separator produces no extra token.
    std::vector<float> vals;
    size_t i = 0;
    const std::string& s = value;
    while (i < s.size()) {
        size_t j = s.find(' ', i);
        std::string tok = s.substr(i, j == std::string::npos ? std::string::npos : j - i);
        Property p;
        p.value = tok;
        vals.push_back(p.as_float(dflt));
        if (j == std::string::npos) break;
        i = j + 1;
    }
    while (vals.size() < 3) vals.push_back(dflt);
    x = vals[0];
    y = vals[1];
    z = vals[2];
}

Property PropertyList::find(const std::string& name) const {
    for (const auto& p : props)
        if (p.name == name) return p;
    Property miss;
    miss.name = name;
    return miss;
}

// ---------------------------------------------------------------- mini JSON
namespace {
struct JVal {
    enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
    bool b = false;
    float num = 0;
    std::string str;
    std::vector<JVal> arr;
    std::map<std::string, JVal> obj;
    std::string as_str() const {
        switch (kind) {
        case Bool: return std::to_string((int)b);
        case Num: return std::to_string(num);
        case Str: return str;
        default: return "";
        }
    }
};

struct JParser {
    const std::string& s;
    size_t pos = 0;
    int depth = 0;  // nesting of arrays / objects: deeper than kMaxDepth parses as null (no stack overflow)
    static constexpr int kMaxDepth = 256;
    explicit JParser(const std::string& src) : s(src) {}
    char peek() const { return pos < s.size() ? s[pos] : 0; }
    char take() { return pos < s.size() ? s[pos++] : (pos++, 0); }
    void ws() { while (pos < s.size() && std::isspace((unsigned char)s[pos])) ++pos; }
    JVal value() {
        ws();
        char c = peek();
        JVal v;
        if (c == 'n') { pos += 4; return v; }
        if (c == 't' || c == 'f') { v.kind = JVal::Bool; v.b = c == 't'; pos += c == 't' ? 4 : 5; return v; }
        if (c == '-' || std::isdigit((unsigned char)c)) return number();
        if (c == '"') return string();
        if ((c == '[' || c == '{') && depth >= kMaxDepth) { pos = s.size(); return v; }
        if (c == '[') { ++depth; JVal a = array(); --depth; return a; }
        if (c == '{') { ++depth; JVal o = object(); --depth; return o; }
        return v;
    }
    JVal number() {
        size_t start = pos;
        if (peek() == '-') ++pos;
        if (peek() == '0') ++pos;
        else while (std::isdigit((unsigned char)peek())) ++pos;
        if (peek() == '.') { ++pos; while (std::isdigit((unsigned char)peek())) ++pos; }
        if (peek() == 'e' || peek() == 'E') {
            ++pos;
            if (peek() == '+' || peek() == '-') ++pos;
            while (std::isdigit((unsigned char)peek())) ++pos;
        }
        JVal v;
        v.kind = JVal::Num;
        std::string lit = s.substr(start, pos - start);
        v.num = std::strtof(lit.c_str(), nullptr);
        return v;
    }
    JVal string() {
        ++pos;  // opening quote
        JVal v;
        v.kind = JVal::Str;
        while (pos < s.size()) {
            char c = s[pos++];
            if (c == '"') break;
            v.str.push_back(c);
        }
        return v;
    }
    JVal array() {
        ++pos;
        ws();
        JVal v;
        v.kind = JVal::Arr;
        if (peek() == ']') { ++pos; return v; }
        while (pos < s.size()) {
            v.arr.push_back(value());
            ws();
            char c = take();
            if (c == ']') break;
            ws();
        }
        return v;
    }
    JVal object() {
        ++pos;
        ws();
        JVal v;
        v.kind = JVal::Obj;
        if (peek() == '}') { ++pos; return v; }
        while (pos < s.size()) {
            ws();
            std::string key = string().str;
            ws();
            ++pos;  // ':'
            ws();
            v.obj[key] = value();
            ws();
            char c = take();
            if (c == '}') break;
            ws();
        }
        return v;
    }
};
}  // namespace

bool parse_scene_json(const std::string& path, SceneFile& out, std::string& err) {
    std::ifstream f(path);
    if (!f) { err = "cannot open " + path; return false; }
    std::stringstream ss;
    ss << f.rdbuf();
    std::string text = ss.str();
    JParser p(text);
    p.ws();
    JVal root = p.value();
    if (root.kind != JVal::Obj) { err = "scene.json root is not an object: " + path; return false; }
    for (const auto& kv : root.obj) {
        if (kv.second.kind != JVal::Arr) {
            Property prop;
            prop.name = kv.first;
            prop.value = kv.second.as_str();
            prop.present = true;
            out.properties.props.push_back(prop);
            continue;
        }
        for (const JVal& inst : kv.second.arr) {
            Instance in;
            for (const auto& item : inst.obj) {
                if (item.first == "filename") {
                    in.mesh = item.second.as_str();
                } else if (item.first == "world") {
                    if (item.second.arr.size() < 16) { err = "instance world matrix needs 16 numbers"; return false; }
                    for (int i = 0; i < 16; ++i) in.world[i] = item.second.arr[i].num;
                } else {
                    Property prop;
                    prop.name = item.first;
                    prop.value = item.second.as_str();
                    prop.present = true;
                    in.material.props.push_back(prop);
                }
            }
            out.instances.push_back(in);
        }
    }
    return true;
}

// ---------------------------------------------------------------- .gem
static const uint32_t kGemMagic = 4058972161u;

bool load_gem(const std::string& path, std::vector<GemMesh>& meshes, std::string& err) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) { err = path + " is not a GE Model File (missing)"; return false; }
    auto rd = [&](void* p, size_t n) { return std::fread(p, 1, n, f) == n; };
    // the bytes left in the file bound every count read from it: a corrupted count fails as a
    // truncated file instead of asking for gigabytes (found by tests/test_sanitize.py)
    std::fseek(f, 0, SEEK_END);
    const long fsize = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    auto left = [&]() -> size_t { const long at = std::ftell(f); return (at < 0 || fsize < at) ? 0 : (size_t)(fsize - at); };
    uint32_t magic = 0, animated = 0, n_meshes = 0;
    if (!rd(&magic, 4) || magic != kGemMagic) { std::fclose(f); err = path + " is not a GE Model File"; return false; }
    if (!rd(&animated, 4) || !rd(&n_meshes, 4)) { std::fclose(f); err = "truncated " + path; return false; }
    if (animated) { std::fclose(f); err = "animated .gem not supported on the render path: " + path; return false; }
    for (uint32_t m = 0; m < n_meshes; ++m) {
        GemMesh mesh;
        uint32_t n_props = 0;
        if (!rd(&n_props, 4)) break;
        for (uint32_t i = 0; i < 2 * n_props; ++i) {  // name, value strings
            int32_t len = 0;
            if (!rd(&len, 4) || len < 0 || (size_t)len > left()) { std::fclose(f); err = "bad string in " + path; return false; }
            std::fseek(f, len, SEEK_CUR);
        }
        uint32_t nv = 0, ni = 0;
        if (!rd(&nv, 4) || (size_t)nv * sizeof(GemVertex) > left()) { std::fclose(f); err = "truncated " + path; return false; }
        mesh.vertices.resize(nv);
        if (nv && !rd(mesh.vertices.data(), (size_t)nv * sizeof(GemVertex))) { std::fclose(f); err = "truncated " + path; return false; }
        if (!rd(&ni, 4) || (size_t)ni * 4 > left()) { std::fclose(f); err = "truncated " + path; return false; }
        mesh.indices.resize(ni);
        if (ni && !rd(mesh.indices.data(), (size_t)ni * 4)) { std::fclose(f); err = "truncated " + path; return false; }
        meshes.push_back(std::move(mesh));
    }
    std::fclose(f);
    return true;
}

bool write_gem(const std::string& path, const std::vector<GemVertex>& verts,
               const std::vector<uint32_t>& indices, std::string& err) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) { err = "cannot write " + path; return false; }
    uint32_t hdr[4] = {kGemMagic, 0u, 1u, 0u};  // magic, static, 1 mesh, 0 material props
    bool ok = std::fwrite(hdr, 4, 4, f) == 4;
    uint32_t nv = (uint32_t)verts.size(), ni = (uint32_t)indices.size();
    ok = ok && std::fwrite(&nv, 4, 1, f) == 1;
    ok = ok && (nv == 0 || std::fwrite(verts.data(), sizeof(GemVertex), nv, f) == nv);
    ok = ok && std::fwrite(&ni, 4, 1, f) == 1;
    ok = ok && (ni == 0 || std::fwrite(indices.data(), 4, ni, f) == ni);
    std::fclose(f);
    if (!ok) err = "short write " + path;
    return ok;
}

}  // namespace rth

// rt_core.h — host-side value types with RTBase's exact float semantics.
//
// Every operator reproduces the reference's operation order so that results are bit-identical
// (compile with -ffp-contract=off): Colour RTBase/Core.h:16-93, Vec3 :95-174, Dot/Cross/Max/Min
// :176-195, Matrix :205-505, Frame :507-542. Only what the host front-end needs is here; the
// device restatement lives in csrc/device/rtg_device_math.h.
#pragma once
#include <cmath>
#include <cstring>
#include <cstdint>

namespace rth {

struct V3 {
    float x = 0, y = 0, z = 0;
    V3() = default;
    V3(float a, float b, float c) : x(a), y(b), z(c) {}
    V3 operator+(const V3& o) const { return {x + o.x, y + o.y, z + o.z}; }
    V3 operator-(const V3& o) const { return {x - o.x, y - o.y, z - o.z}; }
    V3 operator*(float s) const { return {x * s, y * s, z * s}; }
    V3 operator/(float s) const { return {x / s, y / s, z / s}; }
    V3 operator-() const { return {-x, -y, -z}; }
    float lengthSq() const { return (x * x) + (y * y) + (z * z); }
    float length() const { return std::sqrt(lengthSq()); }
    V3 normalize() const {
        float l = 1.0f / std::sqrt((x * x) + (y * y) + (z * z));
        return {x * l, y * l, z * l};
    }
    float dot(const V3& v) const { return (x * v.x) + (y * v.y) + (z * v.z); }
    V3 cross(const V3& v) const {
        return {(y * v.z) - (z * v.y), (z * v.x) - (x * v.z), (x * v.y) - (y * v.x)};
    }
    float& operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};

// Core.h:187-195 — explicit ternaries (NaN and signed-zero behaviour matter for box bounds).
inline V3 vmax(const V3& a, const V3& b) {
    return {a.x > b.x ? a.x : b.x, a.y > b.y ? a.y : b.y, a.z > b.z ? a.z : b.z};
}
inline V3 vmin(const V3& a, const V3& b) {
    return {a.x < b.x ? a.x : b.x, a.y < b.y ? a.y : b.y, a.z < b.z ? a.z : b.z};
}

struct Box {  // AABB, Geometry.h:133-192
    V3 max{-3.40282347e+38f, -3.40282347e+38f, -3.40282347e+38f};
    V3 min{3.40282347e+38f, 3.40282347e+38f, 3.40282347e+38f};
    void grow(const V3& p) { max = vmax(max, p); min = vmin(min, p); }
    void grow(const Box& b) { grow(b.min); grow(b.max); }
    float area() const {
        V3 s = max - min;
        return ((s.x * s.y) + (s.y * s.z) + (s.x * s.z)) * 2.0f;
    }
};

// Row-major 4x4, Core.h:205-505.
struct M4 {
    float m[16];
    M4() { set_identity(); }
    void set_identity() {
        std::memset(m, 0, sizeof(m));
        m[0] = m[5] = m[10] = m[15] = 1.0f;
    }
    float& at(int r, int c) { return m[r * 4 + c]; }
    V3 mul_point(const V3& v) const {
        return {((v.x * m[0] + v.y * m[1]) + v.z * m[2]) + m[3],
                ((v.x * m[4] + v.y * m[5]) + v.z * m[6]) + m[7],
                ((v.x * m[8] + v.y * m[9]) + v.z * m[10]) + m[11]};
    }
    V3 mul_vec(const V3& v) const {
        return {(v.x * m[0] + v.y * m[1]) + v.z * m[2],
                (v.x * m[4] + v.y * m[5]) + v.z * m[6],
                (v.x * m[8] + v.y * m[9]) + v.z * m[10]};
    }
    M4 transposed() const {
        M4 t;
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) t.m[c * 4 + r] = m[r * 4 + c];
        return t;
    }
    // Matrix::invert (Core.h:326-438): the MESA cofactor expansion. Each inverse entry is a
    // left-to-right sum of six signed triple products; a singular matrix resets *this* to the
    // identity (the reference mutates itself there) and divides by 1.
    M4 inverted();
};

// Cofactor table: for output entry k, six terms (sign, i, j, l) meaning sign * m[i]*m[j]*m[l].
struct CofTerm { int8_t s, i, j, l; };
extern const CofTerm kCofactors[16][6];

inline M4 M4::inverted() {
    M4 inv;
    for (int k = 0; k < 16; ++k) {
        float acc = 0.0f;
        for (int t = 0; t < 6; ++t) {
            const CofTerm& c = kCofactors[k][t];
            float p = (m[c.i] * m[c.j]) * m[c.l];
            if (t == 0) acc = c.s > 0 ? p : -p;
            else acc = c.s > 0 ? acc + p : acc - p;
        }
        inv.m[k] = acc;
    }
    float det = ((m[0] * inv.m[0] + m[1] * inv.m[4]) + m[2] * inv.m[8]) + m[3] * inv.m[12];
    if (det == 0) {
        set_identity();
        det = 1.0f;
    }
    det = 1.0f / det;
    for (int i = 0; i < 16; ++i) inv.m[i] = inv.m[i] * det;
    return inv;
}

// Matrix::lookAt (Core.h:439-459).
inline M4 look_at(const V3& from, const V3& to, const V3& up) {
    M4 r;
    V3 dir = (from - to).normalize();
    V3 left = up.cross(dir).normalize();
    V3 nup = dir.cross(left);
    const V3* rows[3] = {&left, &nup, &dir};
    for (int i = 0; i < 3; ++i) {
        r.at(i, 0) = rows[i]->x;
        r.at(i, 1) = rows[i]->y;
        r.at(i, 2) = rows[i]->z;
        r.at(i, 3) = -from.dot(*rows[i]);
    }
    r.at(3, 3) = 1;
    return r;
}

// Matrix::perspective (Core.h:460-471); tanf from the host libm, as the reference.
inline M4 perspective(float n, float f, float aspect, float fov) {
    M4 p;
    std::memset(p.m, 0, sizeof(p.m));
    float t = 1.0f / tanf(fov * 0.5f * 3.141592654f / 180.0f);
    p.at(0, 0) = t / aspect;
    p.at(1, 1) = t;
    p.at(2, 2) = -f / (f - n);
    p.at(2, 3) = -(f * n) / (f - n);
    p.at(3, 2) = -1.0f;
    return p;
}

inline float lum(float r, float g, float b) { return ((0.2126f * r) + (0.7152f * g)) + (0.0722f * b); }

}  // namespace rth

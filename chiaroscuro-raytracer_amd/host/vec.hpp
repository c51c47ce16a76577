// vec.hpp -- the few glm 0.9.8.5 value types and operations the host side of
// the render loop needs, with glm's exact evaluation order (func_geometric.inl,
// type_vec3.inl).  Any type with .x/.y/.z members (glm::vec3 included) converts
// implicitly, so reference call sites `rayTrace(glm::vec3, ...)` compile as is.
#pragma once
#include <cmath>

namespace chiaro {

struct vec2 {
    float x = 0.f, y = 0.f;
    vec2() = default;
    vec2(float a, float b) : x(a), y(b) {}
};

struct vec3 {
    float x = 0.f, y = 0.f, z = 0.f;
    vec3() = default; // glm zero-initialises (detail/type_vec3.inl:36-39)
    explicit vec3(float s) : x(s), y(s), z(s) {}
    vec3(float a, float b, float c) : x(a), y(b), z(c) {}
    template <class V, class = decltype(V{}.z)> vec3(const V &v) : x(v.x), y(v.y), z(v.z) {}
    float &operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};

inline vec3 operator+(vec3 a, vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline vec3 operator-(vec3 a, vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline vec3 operator*(vec3 a, vec3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline vec3 operator*(vec3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline vec3 operator*(float s, vec3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline vec3 operator/(vec3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline vec3 operator-(vec3 a) { return {-a.x, -a.y, -a.z}; }
inline bool operator==(vec3 a, vec3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
inline float dot(vec3 a, vec3 b) {
    vec3 t = a * b;
    return t.x + t.y + t.z;
}
inline vec3 cross(vec3 x, vec3 y) {
    return {x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y};
}
inline vec3 normalize(vec3 v) { return v * (1.0f / std::sqrt(dot(v, v))); }
inline float length(vec3 v) { return std::sqrt(dot(v, v)); }

// libstdc++ std::min/std::max on floats (argument order matters for -0/NaN)
inline float std_min(float a, float b) { return (b < a) ? b : a; }
inline float std_max(float a, float b) { return (a < b) ? b : a; }

} // namespace chiaro

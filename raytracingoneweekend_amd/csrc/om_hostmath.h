// om_hostmath.h — host-side f32 math for building frozen worlds.
//
// The device kernels consume matrices/bases computed HERE, so every value must
// carry the same bits the reference would compute: same operation order as
// math/{vec3,vec4,mat3x3,mat4x4}.rs, IEEE f32, no contraction (this file is
// compiled with -ffp-contract=off).  f32::max/min -> fmaxf/fminf.
#pragma once
#include <cmath>
#include <cstdint>

namespace om {

struct Vec3 {
    float e[3];
    float x() const { return e[0]; }
    float y() const { return e[1]; }
    float z() const { return e[2]; }
    static Vec3 make(float x, float y, float z) { Vec3 v; v.e[0] = x; v.e[1] = y; v.e[2] = z; return v; }
    static Vec3 load(const float* p) { return make(p[0], p[1], p[2]); }
    void store(float* p) const { p[0] = e[0]; p[1] = e[1]; p[2] = e[2]; }
    Vec3 neg() const { return make(-e[0], -e[1], -e[2]); }                               // vec3.rs:118-121
    Vec3 add(const Vec3& o) const { return make(e[0] + o.e[0], e[1] + o.e[1], e[2] + o.e[2]); }  // vec3.rs:184-193
    Vec3 sub(const Vec3& o) const { return add(o.neg()); }                               // vec3.rs:194-199
    Vec3 mul(const Vec3& o) const { return make(e[0] * o.e[0], e[1] * o.e[1], e[2] * o.e[2]); }  // vec3.rs:200-209
    Vec3 scale(float s) const { return make(e[0] * s, e[1] * s, e[2] * s); }             // vec3.rs:220-235
    Vec3 div(float s) const { return scale(1.0f / s); }                                  // vec3.rs:236-240
    float dot(const Vec3& o) const { return e[0] * o.e[0] + e[1] * o.e[1] + e[2] * o.e[2]; }  // vec3.rs:29-31
    float length_squared() const { return dot(*this); }
    float length() const { return std::sqrt(length_squared()); }
    Vec3 unit() const { return div(length()); }                                          // vec3.rs:38-40
    Vec3 cross(const Vec3& o) const {                                                    // vec3.rs:62-68
        return make(e[1] * o.e[2] - e[2] * o.e[1], e[2] * o.e[0] - e[0] * o.e[2], e[0] * o.e[1] - e[1] * o.e[0]);
    }
};

struct Vec4 {
    float e[4];
    static Vec4 make(float x, float y, float z, float w) { Vec4 v; v.e[0] = x; v.e[1] = y; v.e[2] = z; v.e[3] = w; return v; }
    static Vec4 vec(const Vec3& a) { return make(a.e[0], a.e[1], a.e[2], 0.0f); }       // vec4.rs:18
    static Vec4 point(const Vec3& a) { return make(a.e[0], a.e[1], a.e[2], 1.0f); }     // vec4.rs:19
    Vec3 xyz() const { return Vec3::make(e[0], e[1], e[2]); }
    float dot(const Vec4& o) const { return e[0] * o.e[0] + e[1] * o.e[1] + e[2] * o.e[2] + e[3] * o.e[3]; }  // vec4.rs:27-29
};

struct Mat3 {
    Vec3 r[3];
    float at(int i, int j) const { return r[i].e[j]; }
    static Mat3 rows(const Vec3& a, const Vec3& b, const Vec3& c) { Mat3 m; m.r[0] = a; m.r[1] = b; m.r[2] = c; return m; }
    static Mat3 cols(const Vec3& a, const Vec3& b, const Vec3& c) {                     // mat3x3.rs:22-26
        return rows(Vec3::make(a.x(), b.x(), c.x()), Vec3::make(a.y(), b.y(), c.y()), Vec3::make(a.z(), b.z(), c.z()));
    }
    Vec3 apply(const Vec3& v) const { return Vec3::make(r[0].dot(v), r[1].dot(v), r[2].dot(v)); }  // mat3x3.rs:27-29
    Mat3 transpose() const {                                                             // mat3x3.rs:49-51
        return rows(Vec3::make(at(0, 0), at(1, 0), at(2, 0)), Vec3::make(at(0, 1), at(1, 1), at(2, 1)), Vec3::make(at(0, 2), at(1, 2), at(2, 2)));
    }
    float determinant() const {                                                          // mat3x3.rs:52-68 (Kahan)
        const float terms[6] = {at(0, 0) * at(1, 1) * at(2, 2), at(0, 1) * at(1, 2) * at(2, 0), at(0, 2) * at(1, 0) * at(2, 1),
                                -at(0, 0) * at(1, 2) * at(2, 1), -at(0, 1) * at(1, 0) * at(2, 2), -at(0, 2) * at(1, 1) * at(2, 0)};
        float sum = 0.0f, comp = 0.0f;
        for (float term : terms) {
            const float y = term - comp;
            const float t = sum + y;
            comp = (t - sum) - y;
            sum = t;
        }
        return sum;
    }
    Mat3 inverse() const {                                                               // mat3x3.rs:69-81, 92-96
        const float det = determinant();
        const float s = 1.0f / det;
        const Vec3 a = Vec3::make(at(1, 1) * at(2, 2) - at(1, 2) * at(2, 1), at(0, 2) * at(2, 1) - at(0, 1) * at(2, 2),
                                  at(0, 1) * at(1, 2) - at(0, 2) * at(1, 1));
        const Vec3 b = Vec3::make(at(1, 2) * at(2, 0) - at(1, 0) * at(2, 2), at(0, 0) * at(2, 2) - at(0, 2) * at(2, 0),
                                  at(0, 2) * at(1, 0) - at(0, 0) * at(1, 2));
        const Vec3 c = Vec3::make(at(1, 0) * at(2, 1) - at(1, 1) * at(2, 0), at(0, 1) * at(2, 0) - at(0, 0) * at(2, 1),
                                  at(0, 0) * at(1, 1) - at(0, 1) * at(1, 0));
        return rows(a.scale(s), b.scale(s), c.scale(s));
    }
};

struct Mat4 {
    Vec4 r[4];
    static Mat4 rows(const Vec4& a, const Vec4& b, const Vec4& c, const Vec4& d) { Mat4 m; m.r[0] = a; m.r[1] = b; m.r[2] = c; m.r[3] = d; return m; }
    static Mat4 cols(const Vec4& a, const Vec4& b, const Vec4& c, const Vec4& d) {      // mat4x4.rs:32-37
        Mat4 m;
        for (int i = 0; i < 4; ++i) m.r[i] = Vec4::make(a.e[i], b.e[i], c.e[i], d.e[i]);
        return m;
    }
    static Mat4 load(const float* f) {
        return rows(Vec4::make(f[0], f[1], f[2], f[3]), Vec4::make(f[4], f[5], f[6], f[7]), Vec4::make(f[8], f[9], f[10], f[11]),
                    Vec4::make(f[12], f[13], f[14], f[15]));
    }
    void store(float* f) const { for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) f[4 * i + j] = r[i].e[j]; }
    static Mat4 identity() { return translate(Vec3::make(0.0f, 0.0f, 0.0f)); }
    static Mat4 translate(const Vec3& v) {                                               // mat4x4.rs:88-93
        return rows(Vec4::make(1, 0, 0, v.x()), Vec4::make(0, 1, 0, v.y()), Vec4::make(0, 0, 1, v.z()), Vec4::make(0, 0, 0, 1));
    }
    static Mat4 scale(const Vec3& v) {                                                   // mat4x4.rs:94-99
        return rows(Vec4::make(v.x(), 0, 0, 0), Vec4::make(0, v.y(), 0, 0), Vec4::make(0, 0, v.z(), 0), Vec4::make(0, 0, 0, 1));
    }
    static Mat4 rotate_x(float f) { const float c = std::cos(f), s = std::sin(f);       // mat4x4.rs:100-107
        return rows(Vec4::make(1, 0, 0, 0), Vec4::make(0, c, s, 0), Vec4::make(0, -s, c, 0), Vec4::make(0, 0, 0, 1)); }
    static Mat4 rotate_y(float f) { const float c = std::cos(f), s = std::sin(f);       // mat4x4.rs:108-115
        return rows(Vec4::make(c, 0, -s, 0), Vec4::make(0, 1, 0, 0), Vec4::make(s, 0, c, 0), Vec4::make(0, 0, 0, 1)); }
    static Mat4 rotate_z(float f) { const float c = std::cos(f), s = std::sin(f);       // mat4x4.rs:116-123
        return rows(Vec4::make(c, -s, 0, 0), Vec4::make(s, c, 0, 0), Vec4::make(0, 0, 1, 0), Vec4::make(0, 0, 0, 1)); }
    Vec4 col(int j) const { return Vec4::make(r[0].e[j], r[1].e[j], r[2].e[j], r[3].e[j]); }  // mat4x4.rs:81-83
    Mat4 transpose() const { return rows(col(0), col(1), col(2), col(3)); }
    Mat4 mul(const Mat4& m) const {                                                      // mat4x4.rs:66-72 (dot_mat, `^`)
        const Mat4 t = m.transpose();
        Mat4 o;
        for (int i = 0; i < 4; ++i) o.r[i] = Vec4::make(r[i].dot(t.r[0]), r[i].dot(t.r[1]), r[i].dot(t.r[2]), r[i].dot(t.r[3]));
        return o;
    }
    Vec4 apply(const Vec4& v) const { return Vec4::make(r[0].dot(v), r[1].dot(v), r[2].dot(v), r[3].dot(v)); }  // mat4x4.rs:45-47
    Vec3 apply_point(const Vec3& p) const { const Vec4 q = Vec4::point(p); return Vec3::make(r[0].dot(q), r[1].dot(q), r[2].dot(q)); }
    Vec3 apply_vec(const Vec3& p) const { const Vec4 q = Vec4::vec(p); return Vec3::make(r[0].dot(q), r[1].dot(q), r[2].dot(q)); }
    Mat4 fast_homogenous_inverse() const {                                               // mat4x4.rs:59-64
        const Mat3 lin = Mat3::rows(r[0].xyz(), r[1].xyz(), r[2].xyz()).inverse();
        const Mat4 s_inv = rows(Vec4::vec(lin.r[0]), Vec4::vec(lin.r[1]), Vec4::vec(lin.r[2]), Vec4::make(0.0f, 0.0f, 0.0f, 1.0f));
        const Mat4 t_inv = translate(col(3).xyz().neg());
        return s_inv.mul(t_inv);
    }
};

static const float kPi = 3.1415926535897932385f;  // utils.rs:29

}  // namespace om

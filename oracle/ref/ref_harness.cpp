// ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (oracle/_ref).
//
// Links the reference's own, unmodified sources (src/mesh.cpp for
// Texture::getColorAt, src/shader.cpp + src/glad.c which mesh.cpp needs to link)
// and uses its vendored glm 0.9.8.5, to produce golden vectors that pin the
// oracle's restatement of:
//   - Texture::getColorAt                          src/mesh.cpp:21-35   (called directly)
//   - the camera basis of RayTracer::rayTrace      src/rayTracer.cpp:41-49 (same 6 lines over glm)
//   - glm normalize / cross / dot / distance / length, mat3 inverse
//   - the kd-tree's per-triangle material normal   src/kdtree.cpp:58-60
//     and light surface                            src/kdtree.cpp:72-77
//   - the preview camera (src/camera.cpp, linked)  as OpenGLPreview drives it
//     (src/openglPreview.cpp:12-15, 39, 178-195)
// Nothing here is a stand-in for a missing header: every header it includes
// ships in /root/reference/include.
#include "camera.hpp"
#include "mesh.hpp"

#include <glm/glm.hpp>
#include <glm/gtc/matrix_transform.hpp>

#include <cstdint>
#include <cstring>

extern "C" {

void ref_tex_lookup(int w, int h, int nc, const unsigned char *data, float u, float v, float out[3]) {
    Texture t;
    t.id = 0;
    t.image = const_cast<unsigned char *>(data);
    t.width = w;
    t.height = h;
    t.nrComponents = nc;
    glm::vec3 c = t.getColorAt(glm::vec2(u, v));
    out[0] = c.x; out[1] = c.y; out[2] = c.z;
}

// rayTracer.cpp:41-49, verbatim semantics over the reference's glm.
void ref_camera(const float *e, const float *c, const float *u, float yview, unsigned xres, unsigned yres,
                float out[12]) {
    glm::vec3 eye(e[0], e[1], e[2]), center(c[0], c[1], c[2]), up(u[0], u[1], u[2]);
    float z = 1.f;
    float y = z * 0.5f * yview;
    float x = y * ((float)xres / (float)yres);
    auto rotate = glm::inverse(glm::mat3(glm::lookAt(eye, center, up)));
    const glm::vec3 dy = (1.f / yres) * rotate * glm::vec3(0.f, -2.f * y, 0.f);
    const glm::vec3 dx = (1.f / xres) * rotate * glm::vec3(2.f * x, 0.f, 0.f);
    const glm::vec3 leftUpper = rotate * glm::vec3(-x, y, -z);
    const glm::vec3 r[4] = {eye, leftUpper, dx, dy};
    for (int i = 0; i < 4; i++) { out[3 * i] = r[i].x; out[3 * i + 1] = r[i].y; out[3 * i + 2] = r[i].z; }
}

void ref_normalize(const float *v, float out[3]) {
    glm::vec3 r = glm::normalize(glm::vec3(v[0], v[1], v[2]));
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
void ref_cross(const float *a, const float *b, float out[3]) {
    glm::vec3 r = glm::cross(glm::vec3(a[0], a[1], a[2]), glm::vec3(b[0], b[1], b[2]));
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
float ref_dot(const float *a, const float *b) {
    return glm::dot(glm::vec3(a[0], a[1], a[2]), glm::vec3(b[0], b[1], b[2]));
}
float ref_distance(const float *a, const float *b) {
    return glm::distance(glm::vec3(a[0], a[1], a[2]), glm::vec3(b[0], b[1], b[2]));
}
// kdtree.cpp:58-60
void ref_material_normal(const float *n, float out[3]) {
    glm::vec3 r = (glm::vec3(n[0], n[1], n[2]) + glm::vec3(n[3], n[4], n[5]) + glm::vec3(n[6], n[7], n[8])) / 3.f;
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
// kdtree.cpp:72-77
float ref_light_surface(const float *p) {
    glm::vec3 A(p[0], p[1], p[2]), B(p[3], p[4], p[5]), C(p[6], p[7], p[8]);
    return 0.5f * glm::length(glm::cross(B - A, C - A));
}
}

extern "C" {
// OpenGLPreview's camera: Camera(VP, LA, UP), Zoom from yview, then nops operations
// (op 0..5 ProcessKeyboard(op, a0), 6 ProcessMouseMovement(a0, a1), 7
// ProcessMouseScroll(a0), 8 MovementSpeed = a0); after each: Position, Front, Up,
// Right, Yaw, Pitch, Zoom (15 floats).
void ref_preview_camera(const float *vp, const float *la, const float *up, float yview, const int *ops,
                        const float *args, int nops, float *out) {
    Camera cam(glm::vec3(vp[0], vp[1], vp[2]), glm::vec3(la[0], la[1], la[2]), glm::vec3(up[0], up[1], up[2]));
    cam.Zoom = glm::degrees(2.f * atanf(0.5f * yview));
    for (int i = 0; i < nops; i++) {
        const float a0 = args[2 * i], a1 = args[2 * i + 1];
        if (ops[i] >= 0 && ops[i] <= 5) cam.ProcessKeyboard((Camera_Movement)ops[i], a0);
        else if (ops[i] == 6) cam.ProcessMouseMovement(a0, a1);
        else if (ops[i] == 7) cam.ProcessMouseScroll(a0);
        else if (ops[i] == 8) cam.MovementSpeed = a0;
        const glm::vec3 v[4] = {cam.Position, cam.Front, cam.Up, cam.Right};
        float *o = out + 15 * i;
        for (int k = 0; k < 4; k++) { o[3 * k] = v[k].x; o[3 * k + 1] = v[k].y; o[3 * k + 2] = v[k].z; }
        o[12] = cam.Yaw; o[13] = cam.Pitch; o[14] = cam.Zoom;
    }
}
}

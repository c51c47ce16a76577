// raytracer.cpp -- host side of RayTracer (src/rayTracer.cpp), GPU render loop.
#include "raytracer.hpp"

#include "checkpoint.hpp"
#include "exr.hpp"

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>

#include <zlib.h>

namespace chiaro {

cr_camera make_camera(vec3 eye, vec3 center, vec3 up, float yview, unsigned xres, unsigned yres) {
    // rayTracer.cpp:41-43
    float z = 1.f;
    float y = z * 0.5f * yview;
    float x = y * ((float)xres / (float)yres);
    // gtc/matrix_transform.inl:521-546 lookAtRH, upper 3x3 as m[col][row]
    const vec3 f = normalize(center - eye);
    const vec3 s = normalize(cross(f, up));
    const vec3 u = cross(s, f);
    const float m[3][3] = {{s.x, u.x, -f.x}, {s.y, u.y, -f.y}, {s.z, u.z, -f.z}};
    // func_matrix.inl:272-294
    const float ood = 1.f / (+m[0][0] * (m[1][1] * m[2][2] - m[2][1] * m[1][2])
                             - m[1][0] * (m[0][1] * m[2][2] - m[2][1] * m[0][2])
                             + m[2][0] * (m[0][1] * m[1][2] - m[1][1] * m[0][2]));
    float r[3][3];
    r[0][0] = +(m[1][1] * m[2][2] - m[2][1] * m[1][2]) * ood;
    r[1][0] = -(m[1][0] * m[2][2] - m[2][0] * m[1][2]) * ood;
    r[2][0] = +(m[1][0] * m[2][1] - m[2][0] * m[1][1]) * ood;
    r[0][1] = -(m[0][1] * m[2][2] - m[2][1] * m[0][2]) * ood;
    r[1][1] = +(m[0][0] * m[2][2] - m[2][0] * m[0][2]) * ood;
    r[2][1] = -(m[0][0] * m[2][1] - m[2][0] * m[0][1]) * ood;
    r[0][2] = +(m[0][1] * m[1][2] - m[1][1] * m[0][2]) * ood;
    r[1][2] = -(m[0][0] * m[1][2] - m[1][0] * m[0][2]) * ood;
    r[2][2] = +(m[0][0] * m[1][1] - m[1][0] * m[0][1]) * ood;
    // rayTracer.cpp:47-49: (scalar * mat3) * vec3 (type_mat3x3.inl:419-433)
    auto mulv = [](const float a[3][3], vec3 v) {
        return vec3(a[0][0] * v.x + a[1][0] * v.y + a[2][0] * v.z, a[0][1] * v.x + a[1][1] * v.y + a[2][1] * v.z,
                    a[0][2] * v.x + a[1][2] * v.y + a[2][2] * v.z);
    };
    const float sy = 1.f / (float)yres, sx = 1.f / (float)xres;
    float a[3][3], b[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            a[i][j] = r[i][j] * sy;
            b[i][j] = r[i][j] * sx;
        }
    const vec3 dy = mulv(a, vec3(0.f, -2.f * y, 0.f));
    const vec3 dx = mulv(b, vec3(2.f * x, 0.f, 0.f));
    const vec3 lu = mulv(r, vec3(-x, y, -z));
    cr_camera c;
    c.eye[0] = eye.x; c.eye[1] = eye.y; c.eye[2] = eye.z;
    c.left_upper[0] = lu.x; c.left_upper[1] = lu.y; c.left_upper[2] = lu.z;
    c.dx[0] = dx.x; c.dx[1] = dx.y; c.dx[2] = dx.z;
    c.dy[0] = dy.x; c.dy[1] = dy.y; c.dy[2] = dy.z;
    return c;
}

RayTracer::RayTracer(Model &_model, Scene &_scene, int device)
    : scene(_scene), pixels((size_t)_scene.yres * _scene.xres * 3, 0.f), data((size_t)_scene.yres * _scene.xres * 3),
      kdtree(_model, _scene) {
    cr_scene_desc d;
    kdtree.describe(scene, d);
    if (scene.gpus > 1) {
        // GPUs device, device + 1, ...; with fewer GPUs than asked for the ranks wrap
        // around (a device then serves several ranks: same image, no speed-up)
        const int ndev = cr_device_count();
        if (ndev > 0 && (int)scene.gpus > ndev)
            std::cerr << "chiaro: gpus " << scene.gpus << " but " << ndev << " GPU(s) visible; ranks share GPUs\n";
        std::vector<int> devs;
        for (unsigned r = 0; r < scene.gpus; r++) devs.push_back(ndev > 0 ? (device + (int)r) % ndev : device);
        group_ = cr_group_create((int)scene.gpus, devs.data());
        if (cr_group_upload_scene(group_, &d) != CR_OK) {
            std::string msg = std::string("chiaro: scene upload failed: ") + cr_group_last_error(group_);
            cr_group_destroy(group_);
            group_ = nullptr;
            throw std::runtime_error(msg);
        }
        ctx_ = cr_group_ctx(group_, 0);
    } else {
        ctx_ = cr_create(device);
        if (cr_upload_scene(ctx_, &d) != CR_OK) {
            std::string msg = std::string("chiaro: scene upload failed: ") + cr_last_error(ctx_);
            cr_destroy(ctx_);
            ctx_ = nullptr;
            throw std::runtime_error(msg);
        }
    }
    kdtree.attach(ctx_);
}

RayTracer::~RayTracer() {
    if (group_) cr_group_destroy(group_); // owns ctx_
    else cr_destroy(ctx_);
}

void RayTracer::rayTrace(vec3 eye, vec3 center, vec3 up, float yview) { rayTraceLayers(1, eye, center, up, yview); }

void RayTracer::rayTraceLayers(unsigned n, vec3 eye, vec3 center, vec3 up, float yview) {
    if (n < 1) return;
    // rayTracer.cpp:24 -- including the reference's `(lastUp == lastUp)`: a
    // change of `up` alone does not reset the accumulation.
    const bool newLayer = (eye == lastEye) && (center == lastCenter) && (lastUp == lastUp) && (yview == lastYview);
    if (newLayer)
        layers_++;
    else {
        layers_ = 1;
        lastEye = eye;
        lastCenter = center;
        lastUp = up;
        lastYview = yview;
    }
    if (!std::getenv("CHIARO_QUIET"))
        std::cerr << "Camera at (" << eye.x << ", " << eye.y << ", " << eye.z << ") facing: (" << center.x << ", "
                  << center.y << ", " << center.z << ")\nRendering image of size " << scene.xres << "x" << scene.yres
                  << " with " << layers_ * scene.samples << " samples on the GPU...\t";
    const auto t0 = std::chrono::high_resolution_clock::now();
    const cr_camera cam = make_camera(eye, center, up, yview, scene.xres, scene.yres);
    cr_render_params p{};
    p.xres = scene.xres;
    p.yres = scene.yres;
    p.spp = scene.samples;
    p.k = scene.k;
    p.background[0] = scene.background.x;
    p.background[1] = scene.background.y;
    p.background[2] = scene.background.z;
    p.seed = scene.seed;
    p.layer = layers_;
    p.rank = 0;
    p.nranks = 1;
    p.tile = 32;
    // A failed render of several layers may leave the device accumulator holding an unknown number of this
    // call's layers (cr_render_layers blends group after group), and so may a failure past the blend: the
    // next rayTrace then starts over at layer 1, whose blend weight (L - 1 = 0) discards whatever the
    // accumulator holds.  A one-layer call that fails with CR_E_INVALID (parameter checks) or CR_E_OOM (buffer
    // growth) stopped before its only blend -- the pass's last kernel -- so the accumulator still holds
    // layers 1 .. layers_ - 1 intact, and a retry continues at the same layer instead of discarding them.
    auto rollback = [&](int rc) {
        if (n == 1 && (rc == CR_E_INVALID || rc == CR_E_OOM)) layers_--;
        else layers_ = 0;
    };
    if (group_) {
        if (const int rc = n == 1 ? cr_group_render(group_, &cam, &p, pixels.data())
                                  : cr_group_render_layers(group_, &cam, &p, n, pixels.data())) {
            rollback(rc);
            throw std::runtime_error(std::string("chiaro: render failed: ") + cr_group_last_error(group_));
        }
        layers_ += n - 1; // layers p.layer .. p.layer + n - 1 are in the frame
        cr_group_get_counters(group_, &counters_);
    } else {
        if (const int rc = n == 1 ? cr_render(ctx_, &cam, &p, pixels.data())
                                  : cr_render_layers(ctx_, &cam, &p, n, pixels.data())) {
            rollback(rc);
            throw std::runtime_error(std::string("chiaro: render failed: ") + cr_last_error(ctx_));
        }
        layers_ += n - 1; // layers p.layer .. p.layer + n - 1 are in the frame
        cr_get_counters(ctx_, &counters_);
    }
    // rayTracer.cpp:51,66-68 (computed after the render instead of racily inside it)
    maxVal = 0.f;
    for (float v : pixels) maxVal = maxVal > v ? maxVal : v;
    const auto t1 = std::chrono::high_resolution_clock::now();
    lastSeconds_ = std::chrono::duration<double>(t1 - t0).count();
    if (!std::getenv("CHIARO_QUIET")) std::cerr << "took " << lastSeconds_ << " seconds.\n";
}

uint8_t *RayTracer::getData() { return data.data(); }

void RayTracer::saveCheckpoint(const char *path) const {
    if (!layers_) throw std::runtime_error("checkpoint: nothing rendered yet");
    chiaro_checkpoint h{};
    h.xres = scene.xres;
    h.yres = scene.yres;
    h.samples = scene.samples;
    h.k = (uint32_t)scene.k;
    h.seed = scene.seed;
    h.layers = layers_;
    const vec3 *v[3] = {&lastEye, &lastCenter, &lastUp};
    float *dst[3] = {h.eye, h.center, h.up};
    for (int i = 0; i < 3; i++) {
        dst[i][0] = v[i]->x;
        dst[i][1] = v[i]->y;
        dst[i][2] = v[i]->z;
    }
    h.yview = lastYview;
    h.background[0] = scene.background.x;
    h.background[1] = scene.background.y;
    h.background[2] = scene.background.z;
    h.scene = scene_fingerprint(kdtree);
    checkpoint_write(path, h, pixels.data());
}

void RayTracer::resume(const char *path) {
    chiaro_checkpoint h{};
    checkpoint_read(path, h, nullptr);
    if (h.xres != scene.xres || h.yres != scene.yres || h.samples != scene.samples || h.k != (uint32_t)scene.k ||
        h.seed != scene.seed || h.background[0] != scene.background.x || h.background[1] != scene.background.y ||
        h.background[2] != scene.background.z)
        throw std::runtime_error("resume: the checkpoint is of another frame size / spp / depth / seed / background");
    if (h.scene != scene_fingerprint(kdtree)) throw std::runtime_error("resume: the checkpoint is of another scene");
    if (!h.layers) throw std::runtime_error("resume: empty checkpoint");
    checkpoint_read(path, h, pixels.data());
    const int rc = group_ ? cr_group_set_accumulator(group_, scene.xres, scene.yres, pixels.data())
                          : cr_set_accumulator(ctx_, scene.xres, scene.yres, pixels.data());
    if (rc != CR_OK)
        throw std::runtime_error(std::string("resume: ") + (group_ ? cr_group_last_error(group_) : cr_last_error(ctx_)));
    layers_ = h.layers;
    lastEye = vec3(h.eye[0], h.eye[1], h.eye[2]);
    lastCenter = vec3(h.center[0], h.center[1], h.center[2]);
    lastUp = vec3(h.up[0], h.up[1], h.up[2]);
    lastYview = h.yview;
    maxVal = 0.f;
    for (float x : pixels) maxVal = maxVal > x ? maxVal : x;
}

// rayTracer.cpp:196-222 (exrdisplay-style): the scalar setup on the host, the
// per-pixel transform on the GPU over the device accumulator of the last layer
// (cr_tonemap; bytes differ from the reference's glibc powf / logf only where a
// value lies within their error of a rounding boundary).
void RayTracer::normalizeImage(float exposure, float defog, float kneeLow, float kneeHigh, float gamma) {
    if (exposure == FLT_MAX) exposure = scene.exposure;
    cr_tonemap_params t;
    cr_tonemap_setup(exposure, defog, kneeLow, kneeHigh, gamma, &t);
    if (group_) {
        if (cr_group_tonemap(group_, &t, scene.xres, scene.yres, data.data()) != CR_OK)
            throw std::runtime_error(std::string("chiaro: tonemap failed: ") + cr_group_last_error(group_));
    } else if (cr_tonemap(ctx_, &t, scene.xres, scene.yres, data.data()) != CR_OK) {
        throw std::runtime_error(std::string("chiaro: tonemap failed: ") + cr_last_error(ctx_));
    }
}

namespace {
bool ends_with(const std::string &s, const char *suf) {
    const size_t n = std::strlen(suf);
    if (s.size() < n) return false;
    for (size_t i = 0; i < n; i++)
        if (std::tolower((unsigned char)s[s.size() - n + i]) != suf[i]) return false;
    return true;
}
void put_be32(std::vector<unsigned char> &v, uint32_t x) {
    for (int i = 3; i >= 0; i--) v.push_back((unsigned char)(x >> (8 * i)));
}
void png_chunk(std::ofstream &o, const char *type, const std::vector<unsigned char> &data) {
    std::vector<unsigned char> buf;
    put_be32(buf, (uint32_t)data.size());
    buf.insert(buf.end(), type, type + 4);
    buf.insert(buf.end(), data.begin(), data.end());
    uLong crc = crc32(0L, Z_NULL, 0);
    crc = crc32(crc, buf.data() + 4, (uInt)(buf.size() - 4));
    put_be32(buf, (uint32_t)crc);
    o.write((const char *)buf.data(), (std::streamsize)buf.size());
}
} // namespace

// rayTracer.cpp:225-279 with this build's own writers (FreeImage is not available):
// float formats keep pixels[0] as the top row, 8-bit formats go through normalizeImage.
void RayTracer::exportImage(const char *filename) {
    const std::string fn(filename);
    const unsigned W = scene.xres, H = scene.yres;
    std::ofstream o(fn, std::ios::binary);
    if (!o) {
        std::cerr << "Couldn't save the image.\nExport failed.\n";
        return;
    }
    if (ends_with(fn, ".pfm")) {
        o << "PF\n" << W << " " << H << "\n-1.0\n";
        for (unsigned y = H; y-- > 0;) o.write((const char *)&pixels[3 * (size_t)y * W], (std::streamsize)(12 * W));
    } else if (ends_with(fn, ".hdr")) { // Radiance RGBE, flat scanlines
        o << "#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y " << H << " +X " << W << "\n";
        std::vector<unsigned char> row(4 * (size_t)W);
        for (unsigned y = 0; y < H; y++) {
            for (unsigned x = 0; x < W; x++) {
                const float *p = &pixels[3 * ((size_t)y * W + x)];
                float v = std::max(p[0], std::max(p[1], p[2]));
                unsigned char *e = &row[4 * (size_t)x];
                if (v < 1e-32f) {
                    e[0] = e[1] = e[2] = e[3] = 0;
                } else {
                    int ex;
                    const float sc = std::frexp(v, &ex) * 256.0f / v;
                    e[0] = (unsigned char)(p[0] * sc); e[1] = (unsigned char)(p[1] * sc);
                    e[2] = (unsigned char)(p[2] * sc); e[3] = (unsigned char)(ex + 128);
                }
            }
            o.write((const char *)row.data(), (std::streamsize)row.size());
        }
    } else if (ends_with(fn, ".exr")) { // HALF B, G, R, PIZ: what FreeImage_Save(FIF_EXR, ..., 0) writes
        const std::vector<unsigned char> f = chiaro::exr_encode(pixels.data(), (int)W, (int)H);
        o.write((const char *)f.data(), (std::streamsize)f.size());
    } else { // 8-bit: rows of `data` are bottom-up (rayTracer.cpp:217), write top-down
        normalizeImage();
        if (ends_with(fn, ".png")) {
            static const unsigned char sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
            o.write((const char *)sig, 8);
            std::vector<unsigned char> ihdr;
            put_be32(ihdr, W);
            put_be32(ihdr, H);
            ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});
            png_chunk(o, "IHDR", ihdr);
            std::vector<unsigned char> raw;
            raw.reserve((3 * (size_t)W + 1) * H);
            for (unsigned y = 0; y < H; y++) {
                raw.push_back(0);
                const unsigned char *r = &data[3 * (size_t)(H - 1 - y) * W];
                raw.insert(raw.end(), r, r + 3 * (size_t)W);
            }
            uLongf cl = compressBound((uLong)raw.size());
            std::vector<unsigned char> comp(cl);
            compress2(comp.data(), &cl, raw.data(), (uLong)raw.size(), 6);
            comp.resize(cl);
            png_chunk(o, "IDAT", comp);
            png_chunk(o, "IEND", {});
        } else { // PPM
            o << "P6\n" << W << " " << H << "\n255\n";
            for (unsigned y = 0; y < H; y++) o.write((const char *)&data[3 * (size_t)(H - 1 - y) * W], 3 * (std::streamsize)W);
        }
    }
    if (o) std::cerr << "Render succesfully saved to file " << filename << "\n";
    else std::cerr << "Couldn't save the image.\nExport failed.\n";
}

} // namespace chiaro

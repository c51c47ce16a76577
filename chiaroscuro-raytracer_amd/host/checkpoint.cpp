// checkpoint.cpp -- see checkpoint.hpp.
#include "checkpoint.hpp"

#include "kdtree.hpp"

#include <cerrno>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <vector>

#include <zlib.h>

#include <fcntl.h>
#include <unistd.h>

namespace chiaro {

namespace {
const char kMagic[8] = {'C', 'H', 'I', 'A', 'R', 'O', 'C', 'K'};
const uint32_t kVersion = 1;

template <class T> void put(std::vector<unsigned char> &b, const T &v) {
    const unsigned char *p = (const unsigned char *)&v; // little-endian hosts (x86-64)
    b.insert(b.end(), p, p + sizeof(T));
}
template <class T> T get(const unsigned char *&p) {
    T v;
    std::memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
}
uint32_t crc_of(const float *px, size_t n) {
    uLong c = crc32(0L, Z_NULL, 0);
    const size_t bytes = n * sizeof(float);
    for (size_t off = 0; off < bytes; off += 1u << 30) {
        const size_t len = std::min<size_t>(bytes - off, 1u << 30);
        c = crc32(c, (const Bytef *)px + off, (uInt)len);
    }
    return (uint32_t)c;
}
size_t header_bytes() { return 8 + 4 + 6 * 4 + 13 * 4 + 8 + 4; }
} // namespace

uint64_t scene_fingerprint(const KDTree &kd) {
    uLong c = crc32(0L, Z_NULL, 0);
    if (!kd.triangles.empty())
        c = crc32(c, (const Bytef *)kd.triangles.data(), (uInt)(kd.triangles.size() * sizeof(Triangle)));
    uLong a = adler32(0L, Z_NULL, 0);
    const uint32_t counts[2] = {(uint32_t)kd.nodes.size(), (uint32_t)kd.refs.size()};
    a = adler32(a, (const Bytef *)counts, sizeof(counts));
    for (const auto &n : kd.nodes)
        if (!n.isLeaf) a = adler32(a, (const Bytef *)&n.split.position, sizeof(float));
    return ((uint64_t)(uint32_t)c << 32) | (uint32_t)a;
}

void checkpoint_write(const std::string &path, const chiaro_checkpoint &h, const float *pixels) {
    if (!pixels || !h.xres || !h.yres) throw std::runtime_error("checkpoint: empty frame");
    const size_t n = (size_t)h.xres * h.yres * 3;
    std::vector<unsigned char> b;
    b.insert(b.end(), kMagic, kMagic + 8);
    put(b, kVersion);
    for (uint32_t v : {h.xres, h.yres, h.samples, h.k, h.seed, h.layers}) put(b, v);
    for (int i = 0; i < 3; i++) put(b, h.eye[i]);
    for (int i = 0; i < 3; i++) put(b, h.center[i]);
    for (int i = 0; i < 3; i++) put(b, h.up[i]);
    put(b, h.yview);
    for (int i = 0; i < 3; i++) put(b, h.background[i]);
    put(b, h.scene);
    put(b, crc_of(pixels, n));
    // written next to the target and renamed over it: a crash leaves the old checkpoint whole
    // (closed and flushed to the disk before the rename; a failed write removes the partial file)
    const std::string tmp = path + ".tmp";
    const int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd < 0) throw std::runtime_error("checkpoint: cannot write " + tmp);
    auto write_all = [&](const void *data, size_t bytes) {
        const char *q = (const char *)data;
        while (bytes) {
            const ssize_t w = ::write(fd, q, bytes);
            if (w < 0 && errno == EINTR) continue;
            if (w <= 0) return false;
            q += w;
            bytes -= (size_t)w;
        }
        return true;
    };
    const bool ok = write_all(b.data(), b.size()) && write_all(pixels, n * sizeof(float)) && ::fsync(fd) == 0;
    if (::close(fd) != 0 || !ok) {
        ::unlink(tmp.c_str());
        throw std::runtime_error("checkpoint: write failed: " + tmp);
    }
    if (std::rename(tmp.c_str(), path.c_str()) != 0) {
        ::unlink(tmp.c_str());
        throw std::runtime_error("checkpoint: cannot rename to " + path);
    }
    // the rename itself made durable: fsync the directory that holds the checkpoint
    const size_t slash = path.find_last_of('/');
    const std::string dir = slash == std::string::npos ? "." : (slash == 0 ? "/" : path.substr(0, slash));
    const int dfd = ::open(dir.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
    if (dfd >= 0) {
        ::fsync(dfd);
        ::close(dfd);
    }
}

void checkpoint_read(const std::string &path, chiaro_checkpoint &h, float *pixels) {
    std::ifstream in(path, std::ios::binary);
    if (!in) throw std::runtime_error("checkpoint: cannot read " + path);
    std::vector<unsigned char> b(header_bytes());
    in.read((char *)b.data(), (std::streamsize)b.size());
    if (!in || std::memcmp(b.data(), kMagic, 8) != 0) throw std::runtime_error("checkpoint: not a checkpoint: " + path);
    const unsigned char *p = b.data() + 8;
    if (get<uint32_t>(p) != kVersion) throw std::runtime_error("checkpoint: unknown version: " + path);
    h.xres = get<uint32_t>(p);
    h.yres = get<uint32_t>(p);
    h.samples = get<uint32_t>(p);
    h.k = get<uint32_t>(p);
    h.seed = get<uint32_t>(p);
    h.layers = get<uint32_t>(p);
    for (int i = 0; i < 3; i++) h.eye[i] = get<float>(p);
    for (int i = 0; i < 3; i++) h.center[i] = get<float>(p);
    for (int i = 0; i < 3; i++) h.up[i] = get<float>(p);
    h.yview = get<float>(p);
    for (int i = 0; i < 3; i++) h.background[i] = get<float>(p);
    h.scene = get<uint64_t>(p);
    const uint32_t crc = get<uint32_t>(p);
    if (!pixels) return;
    const size_t n = (size_t)h.xres * h.yres * 3;
    in.read((char *)pixels, (std::streamsize)(n * sizeof(float)));
    if (!in) throw std::runtime_error("checkpoint: truncated: " + path);
    if (crc_of(pixels, n) != crc) throw std::runtime_error("checkpoint: pixel checksum mismatch: " + path);
}

} // namespace chiaro

// checkpoint.hpp -- checkpoint / resume of a progressive render: the
// persisted counterpart of the reference's in-process accumulation
// (src/rayTracer.cpp:18-33, 64 -- static layer count, last camera, running average),
// so a long schedule (C5: 30 layers x 100 spp at 4K) survives a restart.
//
// File (little-endian): "CHIAROCK", version 1, the chiaro_checkpoint header fields in
// order (uint32 xres yres samples k seed layers; float eye[3] center[3] up[3] yview
// background[3]; uint64 scene), uint32 crc32 of the pixels, then the running average
// as float32 [yres][xres][3], row 0 = top.  A resume is refused for another frame
// size, spp, depth, seed, background or scene (the fingerprint of the triangles and
// the kd tree): the layers would not belong to the same sum.
#pragma once
#include "chiaroscuro.h"

#include <string>

namespace chiaro {

class KDTree;
// crc32 of the triangle positions (KDTree order) << 32 | adler32 of the node and
// reference counts and the split planes -- which triangles, in which tree
uint64_t scene_fingerprint(const KDTree &kd);
// throw std::runtime_error on I/O errors, a bad file or a pixel checksum mismatch
void checkpoint_write(const std::string &path, const chiaro_checkpoint &h, const float *pixels);
// pixels may be null (header only); it must hold xres * yres * 3 floats otherwise
void checkpoint_read(const std::string &path, chiaro_checkpoint &h, float *pixels);

} // namespace chiaro

// exr.hpp -- OpenEXR scanline files as the reference's exportImage writes them:
// FreeImage_Save(FIF_EXR, FIT_RGBF bitmap, name, 0) (src/rayTracer.cpp:229-272), i.e. channels
// B, G, R of type HALF, PIZ compression (wavelet + Huffman), increasing-Y line order, the
// default header attributes.  The codec follows the OpenEXR file format's PIZ definition
// (bitmap / LUT of the used 16-bit values, the 14/16-bit Haar wavelet per channel plane, the
// canonical Huffman code with a run-length pseudo-symbol); the decoder reads any such file
// (tests decode the reference's own renders/*.exr with it).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace chiaro {

// float -> half, round to nearest even, overflow to infinity (OpenEXR's half(float))
uint16_t float_to_half(float f);
float half_to_float(uint16_t h);

// The file for a W x H image of halves, rgb[(y * W + x) * 3 + c] (c: R, G, B; row 0 = top).
std::vector<unsigned char> exr_encode_half(const uint16_t *rgb, int W, int H);
// The same from floats (each converted by float_to_half).
std::vector<unsigned char> exr_encode(const float *rgb, int W, int H);

// Decodes a scanline EXR with HALF channels R, G, B (any order in the file) and NO / PIZ
// compression into rgb halves as above; false (and err) for anything else.
bool exr_decode_half(const unsigned char *file, size_t n, int &W, int &H, std::vector<uint16_t> &rgb,
                     std::string &err);

} // namespace chiaro

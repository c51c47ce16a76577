// exr.cpp -- half-float PIZ OpenEXR writer (what the reference's FreeImage_Save(FIF_EXR, ..., 0)
// produces, src/rayTracer.cpp:229-272) and a reader for such files.  See exr.hpp.
#include "exr.hpp"

#include <algorithm>
#include <cstring>
#include <unordered_map>

namespace chiaro {

// ------------------------------------------------------------------ half --
uint16_t float_to_half(float f) {
    uint32_t i;
    std::memcpy(&i, &f, 4);
    const int s = (int)((i >> 16) & 0x8000u);
    int e = (int)((i >> 23) & 0xffu) - (127 - 15);
    int m = (int)(i & 0x7fffffu);
    if (e <= 0) {
        if (e < -10) return (uint16_t)s; // below half the smallest subnormal: signed zero
        m |= 0x800000;
        const int t = 14 - e;
        const int a = (1 << (t - 1)) - 1, b = (m >> t) & 1;
        m = (m + a + b) >> t; // round to nearest even (may carry into the exponent: fine)
        return (uint16_t)(s | m);
    }
    if (e == 0xff - (127 - 15)) {
        if (m == 0) return (uint16_t)(s | 0x7c00); // infinity
        m >>= 13;                                    // NaN: keep the top bits, never zero
        return (uint16_t)(s | 0x7c00 | m | (m == 0));
    }
    m = m + 0xfff + ((m >> 13) & 1);
    if (m & 0x800000) {
        m = 0;
        e += 1;
    }
    if (e > 30) return (uint16_t)(s | 0x7c00); // overflow: infinity
    return (uint16_t)(s | (e << 10) | (m >> 13));
}

float half_to_float(uint16_t h) {
    const uint32_t s = (uint32_t)(h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu, r;
    if (e == 0) {
        if (m == 0) {
            r = s;
        } else { // subnormal: normalise
            while (!(m & 0x400u)) {
                m <<= 1;
                e -= 1;
            }
            e += 1;
            m &= ~0x400u;
            r = s | ((e + (127 - 15)) << 23) | (m << 13);
        }
    } else if (e == 31) {
        r = s | 0x7f800000u | (m << 13);
    } else {
        r = s | ((e + (127 - 15)) << 23) | (m << 13);
    }
    float f;
    std::memcpy(&f, &r, 4);
    return f;
}

namespace {

// --------------------------------------------------------------- wavelet --
// 2-D Haar wavelet of a plane of 16-bit values (PIZ); 14-bit form when every value < 2^14.
const int A_OFFSET = 1 << 15, M_OFFSET = 1 << 15, MOD_MASK = (1 << 16) - 1;
inline void wenc14(uint16_t a, uint16_t b, uint16_t &l, uint16_t &h) {
    const int16_t as = (int16_t)a, bs = (int16_t)b;
    l = (uint16_t)(int16_t)((as + bs) >> 1);
    h = (uint16_t)(int16_t)(as - bs);
}
inline void wdec14(uint16_t l, uint16_t h, uint16_t &a, uint16_t &b) {
    const int16_t ls = (int16_t)l, hs = (int16_t)h;
    const int hi = hs, ai = ls + (hi & 1) + (hi >> 1);
    a = (uint16_t)(int16_t)ai;
    b = (uint16_t)(int16_t)(ai - hi);
}
inline void wenc16(uint16_t a, uint16_t b, uint16_t &l, uint16_t &h) {
    const int ao = (a + A_OFFSET) & MOD_MASK;
    int m = (ao + b) >> 1, d = ao - b;
    if (d < 0) m = (m + M_OFFSET) & MOD_MASK;
    d &= MOD_MASK;
    l = (uint16_t)m;
    h = (uint16_t)d;
}
inline void wdec16(uint16_t l, uint16_t h, uint16_t &a, uint16_t &b) {
    const int m = l, d = h, bb = (m - (d >> 1)) & MOD_MASK, aa = (d + bb - A_OFFSET) & MOD_MASK;
    b = (uint16_t)bb;
    a = (uint16_t)aa;
}

void wav2_encode(uint16_t *in, int nx, int ox, int ny, int oy, uint16_t mx) {
    const bool w14 = mx < (1 << 14);
    const int n = std::min(nx, ny);
    int p = 1, p2 = 2;
    auto enc = [&](uint16_t a, uint16_t b, uint16_t &l, uint16_t &h) { w14 ? wenc14(a, b, l, h) : wenc16(a, b, l, h); };
    while (p2 <= n) {
        uint16_t *py = in, *ey = in + oy * (ny - p2);
        const int oy1 = oy * p, oy2 = oy * p2, ox1 = ox * p, ox2 = ox * p2;
        uint16_t i00, i01, i10, i11;
        for (; py <= ey; py += oy2) {
            uint16_t *px = py, *ex = py + ox * (nx - p2);
            for (; px <= ex; px += ox2) {
                uint16_t *p01 = px + ox1, *p10 = px + oy1, *p11 = p10 + ox1;
                enc(*px, *p01, i00, i01);
                enc(*p10, *p11, i10, i11);
                enc(i00, i10, *px, *p10);
                enc(i01, i11, *p01, *p11);
            }
            if (nx & p) { // odd column
                uint16_t *p10 = px + oy1;
                enc(*px, *p10, i00, *p10);
                *px = i00;
            }
        }
        if (ny & p) { // odd line
            uint16_t *px = py, *ex = py + ox * (nx - p2);
            for (; px <= ex; px += ox2) {
                uint16_t *p01 = px + ox1;
                enc(*px, *p01, i00, *p01);
                *px = i00;
            }
        }
        p = p2;
        p2 <<= 1;
    }
}

void wav2_decode(uint16_t *in, int nx, int ox, int ny, int oy, uint16_t mx) {
    const bool w14 = mx < (1 << 14);
    const int n = std::min(nx, ny);
    auto dec = [&](uint16_t l, uint16_t h, uint16_t &a, uint16_t &b) { w14 ? wdec14(l, h, a, b) : wdec16(l, h, a, b); };
    int p = 1, p2;
    while (p <= n) p <<= 1;
    p >>= 1;
    p2 = p;
    p >>= 1;
    while (p >= 1) {
        uint16_t *py = in, *ey = in + oy * (ny - p2);
        const int oy1 = oy * p, oy2 = oy * p2, ox1 = ox * p, ox2 = ox * p2;
        uint16_t i00, i01, i10, i11;
        for (; py <= ey; py += oy2) {
            uint16_t *px = py, *ex = py + ox * (nx - p2);
            for (; px <= ex; px += ox2) {
                uint16_t *p01 = px + ox1, *p10 = px + oy1, *p11 = p10 + ox1;
                dec(*px, *p10, i00, i10);
                dec(*p01, *p11, i01, i11);
                dec(i00, i01, *px, *p01);
                dec(i10, i11, *p10, *p11);
            }
            if (nx & p) {
                uint16_t *p10 = px + oy1;
                dec(*px, *p10, i00, *p10);
                *px = i00;
            }
        }
        if (ny & p) {
            uint16_t *px = py, *ex = py + ox * (nx - p2);
            for (; px <= ex; px += ox2) {
                uint16_t *p01 = px + ox1;
                dec(*px, *p01, i00, *p01);
                *px = i00;
            }
        }
        p2 = p;
        p >>= 1;
    }
}

// --------------------------------------------------------------- Huffman --
const int HUF_ENCSIZE = (1 << 16) + 1;
const int SHORT_ZEROCODE_RUN = 59, LONG_ZEROCODE_RUN = 63;
const int SHORTEST_LONG_RUN = 2 + LONG_ZEROCODE_RUN - SHORT_ZEROCODE_RUN, LONGEST_LONG_RUN = 255 + SHORTEST_LONG_RUN;
typedef long long i64;

inline int huf_length(i64 code) { return (int)(code & 63); }
inline i64 huf_code(i64 code) { return code >> 6; }

struct BitOut {
    std::vector<unsigned char> &out;
    uint64_t c = 0; // only the low lc bits are live (older bits shift out)
    int lc = 0;
    void bits(int n, i64 b) {
        c = (c << n) | (uint64_t)b;
        lc += n;
        while (lc >= 8) out.push_back((unsigned char)(c >> (lc -= 8)));
    }
    void code(i64 hc) { bits(huf_length(hc), huf_code(hc)); }
};

// Code lengths -> canonical (code << 6 | length), numerically lowest codes for the longest lengths.
void huf_canonical(i64 *hcode) {
    i64 n[59] = {};
    for (int i = 0; i < HUF_ENCSIZE; i++) n[hcode[i]] += 1;
    i64 c = 0;
    for (int i = 58; i > 0; --i) {
        const i64 nc = (c + n[i]) >> 1;
        n[i] = c;
        c = nc;
    }
    for (int i = 0; i < HUF_ENCSIZE; i++) {
        const int l = (int)hcode[i];
        if (l > 0) hcode[i] = l | (n[l]++ << 6);
    }
}

// frq (counts) -> code table; im / iM: first / last symbol, iM the run-length pseudo-symbol.
// The merge order follows a binary min-heap of frequency pointers (std::make_heap / pop_heap /
// push_heap with "greater" as the ordering).
void huf_build_table(i64 *frq, int &im, int &iM) {
    std::vector<int> hlink(HUF_ENCSIZE);
    std::vector<i64 *> heap;
    im = 0;
    while (!frq[im]) im++;
    for (int i = im; i < HUF_ENCSIZE; i++) {
        hlink[i] = i;
        if (frq[i]) {
            heap.push_back(&frq[i]);
            iM = i;
        }
    }
    iM++;
    frq[iM] = 1;
    heap.push_back(&frq[iM]);
    auto cmp = [](i64 *a, i64 *b) { return *a > *b; };
    std::make_heap(heap.begin(), heap.end(), cmp);
    std::vector<i64> scode(HUF_ENCSIZE, 0);
    size_t nf = heap.size();
    while (nf > 1) {
        const int mm = (int)(heap[0] - frq);
        std::pop_heap(heap.begin(), heap.begin() + nf, cmp);
        --nf;
        const int m = (int)(heap[0] - frq);
        std::pop_heap(heap.begin(), heap.begin() + nf, cmp);
        frq[m] += frq[mm];
        std::push_heap(heap.begin(), heap.begin() + nf, cmp);
        for (int j = m;; j = hlink[j]) {
            scode[j]++;
            if (hlink[j] == j) {
                hlink[j] = mm;
                break;
            }
        }
        for (int j = mm;; j = hlink[j]) {
            scode[j]++;
            if (hlink[j] == j) break;
        }
    }
    huf_canonical(scode.data());
    std::memcpy(frq, scode.data(), sizeof(i64) * HUF_ENCSIZE);
}

void huf_pack_table(const i64 *hcode, int im, int iM, std::vector<unsigned char> &out) {
    BitOut bo{out};
    for (; im <= iM; im++) {
        const int l = huf_length(hcode[im]);
        if (l == 0) {
            int zerun = 1;
            while (im < iM && zerun < LONGEST_LONG_RUN) {
                if (huf_length(hcode[im + 1]) > 0) break;
                im++;
                zerun++;
            }
            if (zerun >= 2) {
                if (zerun >= SHORTEST_LONG_RUN) {
                    bo.bits(6, LONG_ZEROCODE_RUN);
                    bo.bits(8, zerun - SHORTEST_LONG_RUN);
                } else {
                    bo.bits(6, SHORT_ZEROCODE_RUN + zerun - 2);
                }
                continue;
            }
        }
        bo.bits(6, l);
    }
    if (bo.lc > 0) out.push_back((unsigned char)(bo.c << (8 - bo.lc)));
}

// A run of run_count + 1 copies of a symbol: explicitly, or the symbol, the run code and an 8-bit count.
void send_code(BitOut &bo, i64 scode, int run_count, i64 run_code) {
    if (huf_length(scode) + huf_length(run_code) + 8 < huf_length(scode) * run_count) {
        bo.code(scode);
        bo.code(run_code);
        bo.bits(8, run_count);
    } else {
        while (run_count-- >= 0) bo.code(scode);
    }
}

void huf_compress(const uint16_t *raw, size_t n, std::vector<unsigned char> &out) {
    if (n == 0) return;
    std::vector<i64> frq(HUF_ENCSIZE, 0);
    for (size_t i = 0; i < n; i++) frq[raw[i]]++;
    int im = 0, iM = 0;
    huf_build_table(frq.data(), im, iM);
    const size_t start = out.size();
    out.resize(start + 20, 0);
    huf_pack_table(frq.data(), im, iM, out);
    const size_t table_len = out.size() - start - 20, data_start = out.size();
    BitOut bo{out};
    uint16_t s = raw[0];
    int cs = 0;
    for (size_t i = 1; i < n; i++) {
        if (s == raw[i] && cs < 255) {
            cs++;
        } else {
            send_code(bo, frq[s], cs, frq[iM]);
            cs = 0;
        }
        s = raw[i];
    }
    send_code(bo, frq[s], cs, frq[iM]);
    if (bo.lc) out.push_back((unsigned char)((bo.c << (8 - bo.lc)) & 0xff));
    const uint64_t nbits = (uint64_t)(out.size() - data_start - (bo.lc ? 1 : 0)) * 8 + (uint64_t)bo.lc;
    auto put = [&](size_t at, uint32_t v) {
        for (int k = 0; k < 4; k++) out[start + at + k] = (unsigned char)(v >> (8 * k));
    };
    put(0, (uint32_t)im);
    put(4, (uint32_t)iM);
    put(8, (uint32_t)table_len);
    put(12, (uint32_t)nbits);
    put(16, 0u);
}

struct BitIn {
    const unsigned char *p, *end;
    uint64_t c = 0;
    int lc = 0;
    bool ok = true;
    i64 bits(int n) {
        while (lc < n) {
            if (p >= end) {
                ok = false;
                return 0;
            }
            c = (c << 8) | *p++;
            lc += 8;
        }
        lc -= n;
        return (i64)((c >> lc) & ((1ull << n) - 1));
    }
};

bool huf_uncompress(const unsigned char *in, size_t nin, uint16_t *raw, size_t nraw) {
    if (nraw == 0) return nin == 0;
    if (nin < 20) return false;
    auto rd = [&](int at) {
        return (uint32_t)in[at] | (uint32_t)in[at + 1] << 8 | (uint32_t)in[at + 2] << 16 | (uint32_t)in[at + 3] << 24;
    };
    const uint32_t im0 = rd(0), iM = rd(4), nbits = rd(12);
    if (im0 >= (uint32_t)HUF_ENCSIZE || iM >= (uint32_t)HUF_ENCSIZE || im0 > iM) return false;
    std::vector<i64> hcode(HUF_ENCSIZE, 0);
    BitIn bi{in + 20, in + nin};
    for (int im = (int)im0; im <= (int)iM; im++) {
        const i64 l = hcode[im] = bi.bits(6);
        if (!bi.ok) return false;
        int zerun = -1;
        if (l == LONG_ZEROCODE_RUN) zerun = (int)bi.bits(8) + SHORTEST_LONG_RUN;
        else if (l >= SHORT_ZEROCODE_RUN) zerun = (int)(l - SHORT_ZEROCODE_RUN + 2);
        if (zerun >= 0) {
            if (im + zerun > (int)iM + 1) return false;
            while (zerun--) hcode[im++] = 0;
            im--;
        }
    }
    huf_canonical(hcode.data());
    // (length, code) -> symbol
    std::unordered_map<i64, int> dec;
    for (int i = (int)im0; i <= (int)iM; i++)
        if (huf_length(hcode[i])) dec[(huf_code(hcode[i]) << 6) | huf_length(hcode[i])] = i;
    const unsigned char *data = bi.p;
    const size_t nbytes = (size_t)(in + nin - data);
    if ((nbits + 7) / 8 > nbytes) return false;
    size_t pos = 0, o = 0;
    i64 code = 0;
    int len = 0;
    while (pos < nbits) {
        code = (code << 1) | ((data[pos >> 3] >> (7 - (pos & 7))) & 1);
        pos++;
        if (++len > 58) return false;
        auto it = dec.find((code << 6) | len);
        if (it == dec.end()) continue;
        code = 0;
        len = 0;
        if (it->second == (int)iM) { // run: the previous symbol repeated an 8-bit count more times
            if (pos + 8 > nbits || o == 0) return false;
            int cs = 0;
            for (int k = 0; k < 8; k++, pos++) cs = (cs << 1) | ((data[pos >> 3] >> (7 - (pos & 7))) & 1);
            if (o + (size_t)cs > nraw) return false;
            const uint16_t s = raw[o - 1];
            while (cs-- > 0) raw[o++] = s;
        } else {
            if (o >= nraw) return false;
            raw[o++] = (uint16_t)it->second;
        }
    }
    return o == nraw && len == 0;
}

// ------------------------------------------------------------------- PIZ --
const int BITMAP_SIZE = 8192, USHORT_RANGE = 1 << 16;

// planes: nc channel planes of nx * ny halves, in file channel order; out: the compressed block
void piz_compress(std::vector<uint16_t> planes, int nx, int ny, int nc, std::vector<unsigned char> &out) {
    std::vector<unsigned char> bitmap(BITMAP_SIZE, 0);
    for (uint16_t v : planes) bitmap[v >> 3] |= (unsigned char)(1 << (v & 7));
    bitmap[0] &= (unsigned char)~1; // zero is always in the table, not stored
    int mn = BITMAP_SIZE - 1, mx = 0;
    for (int i = 0; i < BITMAP_SIZE; i++)
        if (bitmap[i]) {
            mn = std::min(mn, i);
            mx = std::max(mx, i);
        }
    std::vector<uint16_t> lut(USHORT_RANGE);
    int k = 0;
    for (int i = 0; i < USHORT_RANGE; i++) lut[i] = (i == 0 || (bitmap[i >> 3] & (1 << (i & 7)))) ? (uint16_t)k++ : 0;
    const uint16_t max_value = (uint16_t)(k - 1);
    for (uint16_t &v : planes) v = lut[v];
    auto u16 = [&](int v) {
        out.push_back((unsigned char)(v & 0xff));
        out.push_back((unsigned char)(v >> 8));
    };
    u16(mn);
    u16(mx);
    if (mn <= mx) out.insert(out.end(), bitmap.begin() + mn, bitmap.begin() + mx + 1);
    for (int c = 0; c < nc; c++) wav2_encode(planes.data() + (size_t)c * nx * ny, nx, 1, ny, nx, max_value);
    const size_t len_at = out.size();
    out.resize(len_at + 4, 0);
    huf_compress(planes.data(), planes.size(), out);
    const uint32_t length = (uint32_t)(out.size() - len_at - 4);
    for (int b = 0; b < 4; b++) out[len_at + b] = (unsigned char)(length >> (8 * b));
}

bool piz_uncompress(const unsigned char *in, size_t n, int nx, int ny, int nc, std::vector<uint16_t> &planes) {
    if (n < 4) return false;
    const int mn = in[0] | in[1] << 8, mx = in[2] | in[3] << 8;
    size_t at = 4;
    if (mx >= BITMAP_SIZE) return false;
    std::vector<unsigned char> bitmap(BITMAP_SIZE, 0);
    if (mn <= mx) {
        if (at + (size_t)(mx - mn + 1) > n) return false;
        std::memcpy(&bitmap[mn], in + at, (size_t)(mx - mn + 1));
        at += (size_t)(mx - mn + 1);
    }
    std::vector<uint16_t> lut(USHORT_RANGE, 0);
    int k = 0;
    for (int i = 0; i < USHORT_RANGE; i++)
        if (i == 0 || (bitmap[i >> 3] & (1 << (i & 7)))) lut[k++] = (uint16_t)i;
    const uint16_t max_value = (uint16_t)(k - 1);
    if (at + 4 > n) return false;
    const uint32_t length = (uint32_t)in[at] | (uint32_t)in[at + 1] << 8 | (uint32_t)in[at + 2] << 16 |
                            (uint32_t)in[at + 3] << 24;
    at += 4;
    if (at + length > n) return false;
    planes.assign((size_t)nx * ny * nc, 0);
    if (!huf_uncompress(in + at, length, planes.data(), planes.size())) return false;
    for (int c = 0; c < nc; c++) wav2_decode(planes.data() + (size_t)c * nx * ny, nx, 1, ny, nx, max_value);
    for (uint16_t &v : planes) v = lut[v];
    return true;
}

void put32(std::vector<unsigned char> &h, uint32_t v) {
    for (int i = 0; i < 4; i++) h.push_back((unsigned char)(v >> (8 * i)));
}
void put_str(std::vector<unsigned char> &h, const char *s) { h.insert(h.end(), s, s + std::strlen(s) + 1); }

} // namespace

std::vector<unsigned char> exr_encode_half(const uint16_t *rgb, int W, int H) {
    std::vector<unsigned char> h;
    put32(h, 20000630u); // magic
    put32(h, 2u);        // version 2, scanline file
    // the attributes FreeImage's EXR save sets, in OpenEXR's (alphabetical) order
    put_str(h, "channels");
    put_str(h, "chlist");
    put32(h, 3 * 18 + 1);
    for (const char *ch : {"B", "G", "R"}) {
        put_str(h, ch);
        put32(h, 1u); // HALF
        put32(h, 0u); // pLinear, reserved
        put32(h, 1u); // x sampling
        put32(h, 1u); // y sampling
    }
    h.push_back(0);
    put_str(h, "compression");
    put_str(h, "compression");
    put32(h, 1);
    h.push_back(4); // PIZ
    put_str(h, "dataWindow");
    put_str(h, "box2i");
    put32(h, 16);
    put32(h, 0);
    put32(h, 0);
    put32(h, (uint32_t)(W - 1));
    put32(h, (uint32_t)(H - 1));
    put_str(h, "displayWindow");
    put_str(h, "box2i");
    put32(h, 16);
    put32(h, 0);
    put32(h, 0);
    put32(h, (uint32_t)(W - 1));
    put32(h, (uint32_t)(H - 1));
    put_str(h, "lineOrder");
    put_str(h, "lineOrder");
    put32(h, 1);
    h.push_back(0); // increasing y
    put_str(h, "pixelAspectRatio");
    put_str(h, "float");
    put32(h, 4);
    put32(h, 0x3f800000u);
    put_str(h, "screenWindowCenter");
    put_str(h, "v2f");
    put32(h, 8);
    put32(h, 0);
    put32(h, 0);
    put_str(h, "screenWindowWidth");
    put_str(h, "float");
    put32(h, 4);
    put32(h, 0x3f800000u);
    h.push_back(0);
    const int nchunks = (H + 31) / 32;
    const size_t table_at = h.size();
    h.resize(table_at + 8 * (size_t)nchunks, 0);
    const int file_ch[3] = {2, 1, 0}; // B, G, R from the R, G, B input
    for (int cb = 0; cb < nchunks; cb++) {
        const int y0 = cb * 32, ny = std::min(32, H - y0);
        std::vector<uint16_t> planes((size_t)3 * W * ny);
        for (int c = 0; c < 3; c++)
            for (int ly = 0; ly < ny; ly++)
                for (int x = 0; x < W; x++)
                    planes[((size_t)c * ny + ly) * W + x] = rgb[(((size_t)(y0 + ly)) * W + x) * 3 + file_ch[c]];
        std::vector<unsigned char> comp;
        piz_compress(planes, W, ny, 3, comp);
        const size_t raw_bytes = (size_t)6 * W * ny;
        const uint64_t off = h.size();
        for (int b = 0; b < 8; b++) h[table_at + 8 * (size_t)cb + b] = (unsigned char)(off >> (8 * b));
        put32(h, (uint32_t)y0);
        if (comp.size() < raw_bytes) {
            put32(h, (uint32_t)comp.size());
            h.insert(h.end(), comp.begin(), comp.end());
        } else { // incompressible: the block as stored scanlines (per line, per channel)
            put32(h, (uint32_t)raw_bytes);
            for (int ly = 0; ly < ny; ly++)
                for (int c = 0; c < 3; c++)
                    for (int x = 0; x < W; x++) {
                        const uint16_t v = planes[((size_t)c * ny + ly) * W + x];
                        h.push_back((unsigned char)(v & 0xff));
                        h.push_back((unsigned char)(v >> 8));
                    }
        }
    }
    return h;
}

std::vector<unsigned char> exr_encode(const float *rgb, int W, int H) {
    std::vector<uint16_t> hv((size_t)3 * W * H);
    for (size_t i = 0; i < hv.size(); i++) hv[i] = float_to_half(rgb[i]);
    return exr_encode_half(hv.data(), W, H);
}

bool exr_decode_half(const unsigned char *f, size_t n, int &W, int &H, std::vector<uint16_t> &rgb, std::string &err) {
    auto rd32 = [&](size_t at) -> uint32_t {
        return (uint32_t)f[at] | (uint32_t)f[at + 1] << 8 | (uint32_t)f[at + 2] << 16 | (uint32_t)f[at + 3] << 24;
    };
    if (n < 8 || rd32(0) != 20000630u) return err = "not an OpenEXR file", false;
    if ((rd32(4) & 0xffu) != 2 || (rd32(4) & 0x200u)) return err = "not a single-part scanline file", false;
    size_t at = 8;
    std::vector<std::string> chans;
    int comp = -1, line_order = 0;
    int dw[4] = {0, 0, -1, -1};
    for (;;) {
        if (at >= n) return err = "truncated header", false;
        const size_t e = std::find(f + at, f + n, 0) - f;
        if (e >= n) return err = "truncated header", false;
        const std::string name((const char *)f + at, e - at);
        at = e + 1;
        if (name.empty()) break;
        const size_t e2 = std::find(f + at, f + n, 0) - f;
        if (e2 + 5 > n) return err = "truncated header", false;
        const std::string type((const char *)f + at, e2 - at);
        at = e2 + 1;
        const uint32_t size = rd32(at);
        at += 4;
        if (at + size > n) return err = "truncated attribute", false;
        if (name == "channels") {
            size_t k = at;
            while (k < at + size && f[k]) {
                const size_t ce = std::find(f + k, f + at + size, 0) - f;
                const std::string cn((const char *)f + k, ce - k);
                k = ce + 1;
                if (k + 16 > at + size) return err = "bad channel list", false;
                if (rd32(k) != 1u || rd32(k + 8) != 1u || rd32(k + 12) != 1u)
                    return err = "channel " + cn + " is not full-resolution HALF", false;
                chans.push_back(cn);
                k += 16;
            }
        } else if (name == "compression") {
            if (size < 1) return err = "bad compression attribute", false;
            comp = f[at];
        } else if (name == "dataWindow") {
            if (size < 16) return err = "bad dataWindow attribute", false;
            for (int i = 0; i < 4; i++) dw[i] = (int)rd32(at + 4 * i);
        } else if (name == "lineOrder") {
            if (size < 1) return err = "bad lineOrder attribute", false;
            line_order = f[at];
        }
        at += size;
    }
    // (64-bit arithmetic: the window's corners are untrusted int32s)
    const int64_t W64 = (int64_t)dw[2] - dw[0] + 1, H64 = (int64_t)dw[3] - dw[1] + 1;
    if (W64 <= 0 || H64 <= 0) return err = "empty data window", false;
    if (W64 > (1 << 16) || H64 > (1 << 16) || W64 * H64 > (int64_t)1 << 28) return err = "data window too large", false;
    W = (int)W64;
    H = (int)H64;
    if (comp != 0 && comp != 4) return err = "compression " + std::to_string(comp) + " not supported", false;
    (void)line_order; // chunks carry their own y
    int idx[3] = {-1, -1, -1};
    for (size_t i = 0; i < chans.size(); i++) {
        if (chans[i] == "R") idx[0] = (int)i;
        if (chans[i] == "G") idx[1] = (int)i;
        if (chans[i] == "B") idx[2] = (int)i;
    }
    if (idx[0] < 0 || idx[1] < 0 || idx[2] < 0) return err = "no R, G, B channels", false;
    const int nc = (int)chans.size(), lines = comp == 4 ? 32 : 1, nchunks = (H + lines - 1) / lines;
    if (at + 8 * (size_t)nchunks > n) return err = "truncated offset table", false;
    rgb.assign((size_t)3 * W * H, 0);
    for (int cb = 0; cb < nchunks; cb++) {
        uint64_t off = 0;
        for (int b = 0; b < 8; b++) off |= (uint64_t)f[at + 8 * (size_t)cb + b] << (8 * b);
        if (off + 8 > n) return err = "bad chunk offset", false;
        const int y0 = (int)rd32(off) - dw[1];
        const uint32_t size = rd32(off + 4);
        if (y0 < 0 || y0 >= H || off + 8 + size > n) return err = "bad chunk", false;
        const int ny = std::min(lines, H - y0);
        const size_t raw_bytes = (size_t)2 * nc * W * ny;
        std::vector<uint16_t> planes((size_t)nc * W * ny);
        if (size == raw_bytes) { // stored: per line, per channel
            size_t k = off + 8;
            for (int ly = 0; ly < ny; ly++)
                for (int c = 0; c < nc; c++)
                    for (int x = 0; x < W; x++, k += 2)
                        planes[((size_t)c * ny + ly) * W + x] = (uint16_t)(f[k] | f[k + 1] << 8);
        } else if (comp != 4 || !piz_uncompress(f + off + 8, size, W, ny, nc, planes)) {
            return err = "bad PIZ block at line " + std::to_string(y0), false;
        }
        for (int c = 0; c < 3; c++)
            for (int ly = 0; ly < ny; ly++)
                for (int x = 0; x < W; x++)
                    rgb[(((size_t)(y0 + ly)) * W + x) * 3 + c] = planes[((size_t)idx[c] * ny + ly) * W + x];
    }
    return true;
}

} // namespace chiaro

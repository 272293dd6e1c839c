// pt_image.cpp — host-side image output and the parity metric.
//
// Replaces Renderer/Images/WriteImage.cpp:8-99 of Damo12320/OptixPathtracer (tinyexr and
// stb_image_write are not used; the formats are written directly):
//   * EXR: float32 B,G,R channels (alphabetical, as tinyexr is told to write them), scanline,
//     uncompressed (InitEXRHeader leaves compression NONE), rows written top-down, so the
//     colorBuffer (row 0 = bottom, GL convention) is flipped as in WriteEXR (:46-60).  A pixel
//     with any NaN channel is written as 0 (:50-53).
//   * BMP: clamp(v, 0, 1) * 255 truncated to uint8, 24 bit (WriteBMP :8-32).
//   * PFM: little-endian float RGB, bottom row first (no flip needed).
// pt_image_read reads what these writers produce (and uncompressed half/float scanline EXR
// in general), and pt_image_mse is the per-image parity metric of SURVEY.md §8(c).
#include <cctype>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <string>
#include <utility>
#include <vector>

#include "../../include/ptamd.h"

namespace {

thread_local std::string g_img_error;

int img_fail(const std::string& msg) {
    g_img_error = msg;
    return PT_ERR_INVALID;
}

struct File {
    FILE* f = nullptr;
    explicit File(const char* path, const char* mode) : f(std::fopen(path, mode)) {}
    ~File() {
        if (f) std::fclose(f);
    }
};

void put_u8(std::vector<uint8_t>& b, uint8_t v) { b.push_back(v); }
void put_i32(std::vector<uint8_t>& b, int32_t v) {
    for (int k = 0; k < 4; ++k) b.push_back((uint8_t)((uint32_t)v >> (8 * k)));
}
void put_u64(std::vector<uint8_t>& b, uint64_t v) {
    for (int k = 0; k < 8; ++k) b.push_back((uint8_t)(v >> (8 * k)));
}
void put_f32(std::vector<uint8_t>& b, float v) {
    uint32_t u;
    std::memcpy(&u, &v, 4);
    put_i32(b, (int32_t)u);
}
void put_str(std::vector<uint8_t>& b, const char* s) {
    while (*s) b.push_back((uint8_t)*s++);
    b.push_back(0);
}
void attr(std::vector<uint8_t>& b, const char* name, const char* type, int32_t size) {
    put_str(b, name);
    put_str(b, type);
    put_i32(b, size);
}

bool nan_px(const float* p) { return std::isnan(p[0]) || std::isnan(p[1]) || std::isnan(p[2]); }

float half_to_float(uint16_t h) {
    const uint32_t s = (uint32_t)(h >> 15) << 31;
    int e = (h >> 10) & 0x1f;
    uint32_t m = h & 0x3ff;
    uint32_t u;
    if (e == 0) {
        if (m == 0) {
            u = s;
        } else {  // subnormal
            e = 1;
            while (!(m & 0x400)) {
                m <<= 1;
                --e;
            }
            m &= 0x3ff;
            u = s | ((uint32_t)(e + 112) << 23) | (m << 13);
        }
    } else if (e == 31) {
        u = s | 0x7f800000u | (m << 13);
    } else {
        u = s | ((uint32_t)(e + 112) << 23) | (m << 13);
    }
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

struct Reader {
    const std::vector<uint8_t>& b;
    size_t p = 0;
    bool ok = true;
    explicit Reader(const std::vector<uint8_t>& buf) : b(buf) {}
    bool need(size_t n) {
        if (p + n > b.size()) ok = false;
        return ok;
    }
    int32_t i32() {
        if (!need(4)) return 0;
        uint32_t v = (uint32_t)b[p] | ((uint32_t)b[p + 1] << 8) | ((uint32_t)b[p + 2] << 16) | ((uint32_t)b[p + 3] << 24);
        p += 4;
        return (int32_t)v;
    }
    uint64_t u64() {
        uint64_t lo = (uint32_t)i32(), hi = (uint32_t)i32();
        return lo | (hi << 32);
    }
    std::string str() {
        std::string s;
        while (ok && need(1) && b[p] != 0) s.push_back((char)b[p++]);
        if (ok && need(1)) ++p;
        return s;
    }
};

int read_exr(const std::vector<uint8_t>& buf, float* rgb, int32_t* w, int32_t* h) {
    Reader r(buf);
    if (r.i32() != 20000630) return img_fail("pt_image_read: not an OpenEXR file");
    const int32_t ver = r.i32();
    if ((ver & 0xff) != 2 || (ver & 0x1a00)) return img_fail("pt_image_read: only single-part scanline EXR");
    struct Ch {
        std::string name;
        int type;
    };
    std::vector<Ch> chans;
    int comp = -1, x0 = 0, y0 = 0, x1 = -1, y1 = -1, order = 0;
    while (r.ok) {
        std::string name = r.str();
        if (name.empty()) break;
        std::string type = r.str();
        const int32_t size = r.i32();
        if (!r.need((size_t)size)) break;
        const size_t end = r.p + (size_t)size;
        if (name == "channels") {
            while (r.p < end) {
                std::string cn = r.str();
                if (cn.empty()) break;
                const int t = r.i32();
                r.p += 4;  // pLinear + reserved
                const int xs = r.i32(), ys = r.i32();
                if (xs != 1 || ys != 1) return img_fail("pt_image_read: subsampled channels");
                chans.push_back({cn, t});
            }
        } else if (name == "compression") {
            comp = r.b[r.p];
        } else if (name == "dataWindow") {
            x0 = r.i32();
            y0 = r.i32();
            x1 = r.i32();
            y1 = r.i32();
        } else if (name == "lineOrder") {
            order = r.b[r.p];
        }
        r.p = end;
    }
    if (!r.ok) return img_fail("pt_image_read: truncated EXR header");
    if (comp != 0) return img_fail("pt_image_read: only uncompressed EXR is supported");
    const int W = x1 - x0 + 1, H = y1 - y0 + 1;
    if (W <= 0 || H <= 0) return img_fail("pt_image_read: empty data window");
    *w = W;
    *h = H;
    if (!rgb) return PT_OK;
    (void)order;
    int idx[3] = {-1, -1, -1};
    size_t row_bytes = 0;
    std::vector<size_t> ch_off(chans.size());
    for (size_t c = 0; c < chans.size(); ++c) {
        if (chans[c].type != 1 && chans[c].type != 2) return img_fail("pt_image_read: uint channels unsupported");
        ch_off[c] = row_bytes;
        row_bytes += (size_t)W * (chans[c].type == 1 ? 2 : 4);
        if (chans[c].name == "R") idx[0] = (int)c;
        if (chans[c].name == "G") idx[1] = (int)c;
        if (chans[c].name == "B") idx[2] = (int)c;
    }
    std::vector<uint64_t> offs((size_t)H);
    for (int y = 0; y < H; ++y) offs[(size_t)y] = r.u64();
    for (int k = 0; k < H && r.ok; ++k) {
        r.p = (size_t)offs[(size_t)k];
        const int y = r.i32() - y0;
        const int32_t size = r.i32();
        if (y < 0 || y >= H || (size_t)size != row_bytes || !r.need(row_bytes))
            return img_fail("pt_image_read: bad EXR scanline block");
        float* dst = rgb + (size_t)(H - 1 - y) * (size_t)W * 3;  // file rows are top-down
        for (int c = 0; c < 3; ++c) {
            if (idx[c] < 0) {
                for (int x = 0; x < W; ++x) dst[3 * x + c] = 0.0f;
                continue;
            }
            const uint8_t* src = &r.b[r.p + ch_off[(size_t)idx[c]]];
            for (int x = 0; x < W; ++x) {
                if (chans[(size_t)idx[c]].type == 2) {
                    float v;
                    std::memcpy(&v, src + 4 * x, 4);
                    dst[3 * x + c] = v;
                } else {
                    uint16_t hv = (uint16_t)(src[2 * x] | (src[2 * x + 1] << 8));
                    dst[3 * x + c] = half_to_float(hv);
                }
            }
        }
    }
    return r.ok ? PT_OK : img_fail("pt_image_read: truncated EXR data");
}

int read_pfm(const std::vector<uint8_t>& buf, float* rgb, int32_t* w, int32_t* h) {
    size_t p = 0;
    auto token = [&]() {
        while (p < buf.size() && std::isspace(buf[p])) ++p;
        std::string t;
        while (p < buf.size() && !std::isspace(buf[p])) t.push_back((char)buf[p++]);
        return t;
    };
    const std::string magic = token();
    if (magic != "PF") return img_fail("pt_image_read: only colour PFM (PF) is supported");
    const int W = std::atoi(token().c_str()), H = std::atoi(token().c_str());
    const double scale = std::atof(token().c_str());
    ++p;  // single whitespace after the scale
    if (W <= 0 || H <= 0) return img_fail("pt_image_read: bad PFM size");
    *w = W;
    *h = H;
    if (!rgb) return PT_OK;
    const size_t n = (size_t)W * (size_t)H * 3;
    if (p + 4 * n > buf.size()) return img_fail("pt_image_read: truncated PFM");
    const bool little = scale < 0.0;
    for (size_t i = 0; i < n; ++i) {
        uint8_t q[4];
        std::memcpy(q, &buf[p + 4 * i], 4);
        if (!little) std::swap(q[0], q[3]), std::swap(q[1], q[2]);
        std::memcpy(&rgb[i], q, 4);
    }
    return PT_OK;
}

}  // namespace

extern "C" {

const char* pt_image_last_error(void) { return g_img_error.c_str(); }

int pt_image_write_exr(const char* path, const float* rgb, int32_t width, int32_t height) {
    if (!path || !rgb || width <= 0 || height <= 0) return img_fail("pt_image_write_exr: invalid argument");
    std::vector<uint8_t> b;
    put_i32(b, 20000630);
    put_i32(b, 2);
    attr(b, "channels", "chlist", 3 * (2 + 16) + 1);
    for (const char* c : {"B", "G", "R"}) {
        put_str(b, c);
        put_i32(b, 2);  // FLOAT
        put_u8(b, 0);   // pLinear
        put_u8(b, 0);
        put_u8(b, 0);
        put_u8(b, 0);
        put_i32(b, 1);
        put_i32(b, 1);
    }
    put_u8(b, 0);
    attr(b, "compression", "compression", 1);
    put_u8(b, 0);
    attr(b, "dataWindow", "box2i", 16);
    put_i32(b, 0);
    put_i32(b, 0);
    put_i32(b, width - 1);
    put_i32(b, height - 1);
    attr(b, "displayWindow", "box2i", 16);
    put_i32(b, 0);
    put_i32(b, 0);
    put_i32(b, width - 1);
    put_i32(b, height - 1);
    attr(b, "lineOrder", "lineOrder", 1);
    put_u8(b, 0);
    attr(b, "pixelAspectRatio", "float", 4);
    put_f32(b, 1.0f);
    attr(b, "screenWindowCenter", "v2f", 8);
    put_f32(b, 0.0f);
    put_f32(b, 0.0f);
    attr(b, "screenWindowWidth", "float", 4);
    put_f32(b, 1.0f);
    put_u8(b, 0);
    const size_t row_bytes = (size_t)width * 4 * 3;
    const size_t table = b.size();
    const size_t first = table + 8 * (size_t)height;
    for (int y = 0; y < height; ++y) put_u64(b, first + (size_t)y * (8 + row_bytes));
    for (int y = 0; y < height; ++y) {
        put_i32(b, y);
        put_i32(b, (int32_t)row_bytes);
        const float* row = rgb + (size_t)(height - 1 - y) * (size_t)width * 3;  // flip (WriteEXR :46)
        for (int c : {2, 1, 0}) {                                            // B, G, R
            for (int x = 0; x < width; ++x) {
                const float* px = row + 3 * x;
                put_f32(b, nan_px(px) ? 0.0f : px[c]);
            }
        }
    }
    File f(path, "wb");
    if (!f.f) return img_fail(std::string("pt_image_write_exr: cannot open ") + path);
    if (std::fwrite(b.data(), 1, b.size(), f.f) != b.size()) return img_fail("pt_image_write_exr: write failed");
    return PT_OK;
}

int pt_image_write_pfm(const char* path, const float* rgb, int32_t width, int32_t height) {
    if (!path || !rgb || width <= 0 || height <= 0) return img_fail("pt_image_write_pfm: invalid argument");
    File f(path, "wb");
    if (!f.f) return img_fail(std::string("pt_image_write_pfm: cannot open ") + path);
    std::fprintf(f.f, "PF\n%d %d\n-1.0\n", width, height);
    const size_t n = (size_t)width * (size_t)height * 3;
    if (std::fwrite(rgb, sizeof(float), n, f.f) != n) return img_fail("pt_image_write_pfm: write failed");
    return PT_OK;
}

int pt_image_write_bmp(const char* path, const float* rgb, int32_t width, int32_t height) {
    if (!path || !rgb || width <= 0 || height <= 0) return img_fail("pt_image_write_bmp: invalid argument");
    const int pad = (4 - (width * 3) % 4) % 4;
    const uint32_t data = (uint32_t)((width * 3 + pad) * height);
    std::vector<uint8_t> b;
    b.push_back('B');
    b.push_back('M');
    put_i32(b, (int32_t)(54 + data));
    put_i32(b, 0);
    put_i32(b, 54);
    put_i32(b, 40);
    put_i32(b, width);
    put_i32(b, height);  // positive: rows bottom-up, i.e. colorBuffer order
    b.push_back(1);
    b.push_back(0);
    b.push_back(24);
    b.push_back(0);
    put_i32(b, 0);
    put_i32(b, (int32_t)data);
    put_i32(b, 2835);
    put_i32(b, 2835);
    put_i32(b, 0);
    put_i32(b, 0);
    auto q = [](float v) { return (uint8_t)((v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v)) * 255.0f); };
    for (int y = 0; y < height; ++y) {
        const float* row = rgb + (size_t)y * (size_t)width * 3;
        for (int x = 0; x < width; ++x) {
            b.push_back(q(row[3 * x + 2]));
            b.push_back(q(row[3 * x + 1]));
            b.push_back(q(row[3 * x]));
        }
        for (int k = 0; k < pad; ++k) b.push_back(0);
    }
    File f(path, "wb");
    if (!f.f) return img_fail(std::string("pt_image_write_bmp: cannot open ") + path);
    if (std::fwrite(b.data(), 1, b.size(), f.f) != b.size()) return img_fail("pt_image_write_bmp: write failed");
    return PT_OK;
}

int pt_image_read(const char* path, float* rgb, int32_t* width, int32_t* height) {
    if (!path || !width || !height) return img_fail("pt_image_read: invalid argument");
    File f(path, "rb");
    if (!f.f) return img_fail(std::string("pt_image_read: cannot open ") + path);
    std::vector<uint8_t> buf;
    uint8_t chunk[1 << 16];
    size_t n;
    while ((n = std::fread(chunk, 1, sizeof chunk, f.f)) > 0) buf.insert(buf.end(), chunk, chunk + n);
    if (buf.size() >= 4 && buf[0] == 0x76 && buf[1] == 0x2f && buf[2] == 0x31 && buf[3] == 0x01)
        return read_exr(buf, rgb, width, height);
    if (buf.size() >= 2 && buf[0] == 'P' && buf[1] == 'F') return read_pfm(buf, rgb, width, height);
    return img_fail("pt_image_read: unknown format (EXR and PFM are supported)");
}

double pt_image_mse(const float* a, const float* b, int64_t n_pixels) {
    if (!a || !b || n_pixels <= 0) return 0.0;
    double s = 0.0;
    for (int64_t i = 0; i < n_pixels; ++i) {
        const float* pa = a + 3 * i;
        const float* pb = b + 3 * i;
        const bool na = nan_px(pa), nb = nan_px(pb);
        for (int c = 0; c < 3; ++c) {
            const double d = (double)(na ? 0.0f : pa[c]) - (double)(nb ? 0.0f : pb[c]);
            s += d * d;
        }
    }
    return s / (3.0 * (double)n_pixels);
}

}  // extern "C"

// ---- FLIP (LDR) ------------------------------------------------------------------------------
// The README's second image metric ("FLIP vs PBRT-v4", README.md:42-46) is NVIDIA's FLIP
// (Andersson et al. 2020, "FLIP: A Difference Evaluator for Alternating Images"), computed
// there with external tools.  This is the published LDR-FLIP algorithm: linear radiance is
// clamped to [0,1] and sRGB-encoded (the display image), then
//   colour: sRGB -> linear -> XYZ -> YCxCz, CSF-shaped Gaussian filtering per opponent channel
//           (constants of the paper), back to linear RGB clamped to [0,1], CIELab with Hunt
//           adjustment (a, b scaled by L/100), HyAB distance, ^0.7, redistributed with
//           pc = 0.4 / pt = 0.95 against the green-blue maximum;
//   feature: edge / point detectors (first / second Gaussian derivatives, sigma = 0.5 * 0.082 *
//           ppd, positive and negative lobes normalised to 1) on (Y + 16) / 116;
//   per pixel E = Ec ^ (1 - Ef), Ef = (max(|d edge|, |d point|) / sqrt(2)) ^ 0.5; FLIP = mean E.
// All filters are separable and evaluated with edge-clamped borders.
namespace {

struct Img3 {
    int w, h;
    std::vector<float> c[3];
};

void conv_sep(const std::vector<float>& in, std::vector<float>& out, int w, int h, const std::vector<float>& kx,
              const std::vector<float>& ky) {
    const int rx = (int)kx.size() / 2, ry = (int)ky.size() / 2;
    std::vector<float> tmp((size_t)w * h);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            double s = 0.0;
            for (int k = -rx; k <= rx; ++k) {
                const int xx = x + k < 0 ? 0 : (x + k >= w ? w - 1 : x + k);
                s += (double)kx[(size_t)(k + rx)] * in[(size_t)y * w + xx];
            }
            tmp[(size_t)y * w + x] = (float)s;
        }
    out.assign((size_t)w * h, 0.0f);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            double s = 0.0;
            for (int k = -ry; k <= ry; ++k) {
                const int yy = y + k < 0 ? 0 : (y + k >= h ? h - 1 : y + k);
                s += (double)ky[(size_t)(k + ry)] * tmp[(size_t)yy * w + x];
            }
            out[(size_t)y * w + x] = (float)s;
        }
}

const double kPi = 3.14159265358979323846;
// linear RGB <-> XYZ (sRGB primaries, D65), as in the FLIP reference implementation
const double kRgb2Xyz[3][3] = {{10135552.0 / 24577794.0, 8788810.0 / 24577794.0, 4435075.0 / 24577794.0},
                               {2613072.0 / 12288897.0, 8788810.0 / 12288897.0, 887015.0 / 12288897.0},
                               {1425312.0 / 73733382.0, 8788810.0 / 73733382.0, 70074185.0 / 73733382.0}};
const double kXyz2Rgb[3][3] = {{3.241003275, -1.537398934, -0.498615861},
                               {-0.969224334, 1.875930071, 0.041554224},
                               {0.055639423, -0.204011202, 1.057148933}};

void mat3(const double m[3][3], const double in[3], double out[3]) {
    for (int r = 0; r < 3; ++r) out[r] = m[r][0] * in[0] + m[r][1] * in[1] + m[r][2] * in[2];
}
double srgb2lin(double x) { return x > 0.04045 ? std::pow((x + 0.055) / 1.055, 2.4) : x / 12.92; }
double lin2srgb(double x) { return x > 0.0031308 ? 1.055 * std::pow(x, 1.0 / 2.4) - 0.055 : 12.92 * x; }

void white(double wp[3]) {
    const double one[3] = {1, 1, 1};
    mat3(kRgb2Xyz, one, wp);
}
void xyz2ycxcz(const double xyz[3], double o[3]) {
    double wp[3];
    white(wp);
    const double x = xyz[0] / wp[0], y = xyz[1] / wp[1], z = xyz[2] / wp[2];
    o[0] = 116.0 * y - 16.0;
    o[1] = 500.0 * (x - y);
    o[2] = 200.0 * (y - z);
}
void ycxcz2xyz(const double c[3], double o[3]) {
    double wp[3];
    white(wp);
    const double y = (c[0] + 16.0) / 116.0, x = c[1] / 500.0 + y, z = y - c[2] / 200.0;
    o[0] = x * wp[0];
    o[1] = y * wp[1];
    o[2] = z * wp[2];
}
void xyz2lab(const double xyz[3], double o[3]) {
    double wp[3];
    white(wp);
    const double d = 6.0 / 29.0;
    auto f = [&](double t) { return t > d * d * d ? std::cbrt(t) : t / (3.0 * d * d) + 4.0 / 29.0; };
    const double fx = f(xyz[0] / wp[0]), fy = f(xyz[1] / wp[1]), fz = f(xyz[2] / wp[2]);
    o[0] = 116.0 * fy - 16.0;
    o[1] = 500.0 * (fx - fy);
    o[2] = 200.0 * (fy - fz);
}
// linear RGB -> Hunt-adjusted L*a*b*
void rgb2hunt(const double rgb[3], double o[3]) {
    double xyz[3];
    mat3(kRgb2Xyz, rgb, xyz);
    xyz2lab(xyz, o);
    o[1] *= 0.01 * o[0];
    o[2] *= 0.01 * o[0];
}
double hyab(const double a[3], const double b[3]) {
    return std::fabs(a[0] - b[0]) + std::sqrt((a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]));
}

// The CSF filter of one opponent channel: a1*sqrt(pi/b1)*exp(-pi^2 d^2/b1) + a2*..., d in degrees,
// normalised to unit sum.  Each term is a separable Gaussian with sigma^2 = b / (2 pi^2) deg^2.
void csf_filter(const std::vector<float>& in, std::vector<float>& out, int w, int h, double ppd, double a1,
                double b1, double a2, double b2, int r) {
    auto term = [&](double a, double b, std::vector<float>& res, double& mass) {
        std::vector<float> k((size_t)(2 * r + 1));
        double s = 0.0;
        for (int i = -r; i <= r; ++i) {
            const double dd = (double)i / ppd;
            const double v = std::exp(-kPi * kPi * dd * dd / b);
            k[(size_t)(i + r)] = (float)v;
            s += v;
        }
        // 2D term = a*sqrt(pi/b) * g(x) g(y); its total mass = a*sqrt(pi/b) * s^2
        mass = a * std::sqrt(kPi / b) * s * s;
        conv_sep(in, res, w, h, k, k);
        for (float& v : res) v = (float)(v * a * std::sqrt(kPi / b));
    };
    std::vector<float> t1, t2;
    double m1 = 0.0, m2 = 0.0;
    term(a1, b1, t1, m1);
    if (a2 != 0.0) term(a2, b2, t2, m2);
    out.assign(in.size(), 0.0f);
    const double tot = m1 + m2;
    for (size_t i = 0; i < in.size(); ++i) out[i] = (float)((t1[i] + (a2 != 0.0 ? t2[i] : 0.0f)) / tot);
}

void feature_kernels(double ppd, std::vector<float>& g, std::vector<float>& d1, std::vector<float>& d2) {
    const double sd = 0.5 * 0.082 * ppd;
    const int r = (int)std::ceil(3.0 * sd);
    g.assign((size_t)(2 * r + 1), 0.0f);
    d1 = g;
    d2 = g;
    double sg = 0.0, p1 = 0.0, p2 = 0.0, n2 = 0.0;
    for (int i = -r; i <= r; ++i) {
        const double gv = std::exp(-(double)i * i / (2.0 * sd * sd));
        sg += gv;
        const double a = -(double)i * gv, b = ((double)i * i / (sd * sd) - 1.0) * gv;
        if (a > 0) p1 += a;
        if (b > 0) p2 += b;
        else n2 -= b;
        g[(size_t)(i + r)] = (float)gv;
        d1[(size_t)(i + r)] = (float)a;
        d2[(size_t)(i + r)] = (float)b;
    }
    for (size_t i = 0; i < g.size(); ++i) {
        g[i] = (float)(g[i] / sg);
        d1[i] = (float)(d1[i] / p1);
        d2[i] = (float)(d2[i] > 0 ? d2[i] / p2 : d2[i] / n2);
    }
}

}  // namespace

extern "C" double pt_image_flip(const float* ref, const float* test, int32_t width, int32_t height,
                                float pixels_per_degree, float* error_map) {
    if (!ref || !test || width <= 0 || height <= 0) return -1.0;
    const int w = width, h = height;
    const size_t n = (size_t)w * h;
    const double ppd = pixels_per_degree > 0.0f ? pixels_per_degree : 67.0;
    // display images: clamp linear radiance to [0,1], sRGB-encode, then the FLIP input transform
    std::vector<float> ycx[2][3];
    for (int im = 0; im < 2; ++im) {
        const float* src = im ? test : ref;
        for (int c = 0; c < 3; ++c) ycx[im][c].resize(n);
        for (size_t i = 0; i < n; ++i) {
            double rgb[3], xyz[3], o[3];
            for (int c = 0; c < 3; ++c) {
                double v = src[3 * i + c];
                v = std::isnan(v) ? 0.0 : (v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v));
                rgb[c] = srgb2lin(lin2srgb(v));
            }
            mat3(kRgb2Xyz, rgb, xyz);
            xyz2ycxcz(xyz, o);
            for (int c = 0; c < 3; ++c) ycx[im][c][i] = (float)o[c];
        }
    }
    // colour pipeline
    const double bmax = 0.04;  // max scale parameter of the three CSFs
    const int r = (int)std::ceil(3.0 * std::sqrt(bmax / (2.0 * kPi * kPi)) * ppd);
    const double csf[3][4] = {{1.0, 0.0047, 0.0, 1e-5}, {1.0, 0.0053, 0.0, 1e-5}, {34.1, 0.04, 13.5, 0.025}};
    std::vector<float> filt[2][3];
    for (int im = 0; im < 2; ++im)
        for (int c = 0; c < 3; ++c)
            csf_filter(ycx[im][c], filt[im][c], w, h, ppd, csf[c][0], csf[c][1], csf[c][2], csf[c][3], r);
    double green[3] = {0, 1, 0}, blue[3] = {0, 0, 1}, hg[3], hb[3];
    rgb2hunt(green, hg);
    rgb2hunt(blue, hb);
    const double qc = 0.7, pc = 0.4, pt = 0.95;
    const double cmax = std::pow(hyab(hg, hb), qc);
    // feature pipeline on the achromatic channel (Y + 16) / 116
    std::vector<float> gk, d1, d2;
    feature_kernels(ppd, gk, d1, d2);
    std::vector<float> feat[2][4];
    for (int im = 0; im < 2; ++im) {
        std::vector<float> yn(n);
        for (size_t i = 0; i < n; ++i) yn[i] = (float)((ycx[im][0][i] + 16.0) / 116.0);
        conv_sep(yn, feat[im][0], w, h, d1, gk);  // edge x
        conv_sep(yn, feat[im][1], w, h, gk, d1);  // edge y
        conv_sep(yn, feat[im][2], w, h, d2, gk);  // point x
        conv_sep(yn, feat[im][3], w, h, gk, d2);  // point y
    }
    double sum = 0.0;
    for (size_t i = 0; i < n; ++i) {
        double lab[2][3];
        for (int im = 0; im < 2; ++im) {
            double yc[3] = {filt[im][0][i], filt[im][1][i], filt[im][2][i]}, xyz[3], rgb[3];
            ycxcz2xyz(yc, xyz);
            mat3(kXyz2Rgb, xyz, rgb);
            for (double& v : rgb) v = v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v);
            rgb2hunt(rgb, lab[im]);
        }
        const double dc = std::pow(hyab(lab[0], lab[1]), qc);
        const double ec = dc < pc * cmax ? pt / (pc * cmax) * dc : pt + (dc - pc * cmax) / (cmax - pc * cmax) * (1.0 - pt);
        const double er = std::hypot((double)feat[0][0][i], (double)feat[0][1][i]);
        const double et = std::hypot((double)feat[1][0][i], (double)feat[1][1][i]);
        const double pr = std::hypot((double)feat[0][2][i], (double)feat[0][3][i]);
        const double ptt = std::hypot((double)feat[1][2][i], (double)feat[1][3][i]);
        const double df = std::max(std::fabs(er - et), std::fabs(pr - ptt));
        const double ef = std::pow(df / std::sqrt(2.0), 0.5);
        const double e = std::pow(ec, 1.0 - ef);
        if (error_map) error_map[i] = (float)e;
        sum += e;
    }
    return sum / (double)n;
}

// pt_gltf.cpp — glTF 2.0 scene loader.
//
// Replaces ModelLoader::LoadModel / ParseScene / ParseNodes / ParseMaterial /
// ParseTransformation / LoadTextures (ModelLoading/ModelLoader.cpp:10-244) and
// Mesh::GetModelMatrix (ModelLoading/Mesh.cpp:6-22) of Damo12320/OptixPathtracer, which use
// tiny_gltf + stb_image.  Output is a pt_scene (the Model of ModelLoading/Model.h) that
// pt_create consumes directly.
//
// Kept from the reference: one mesh per primitive with that primitive's material
// (ModelLoader.cpp:97-98); POSITION / NORMAL / TEXCOORD_0; albedo = baseColorFactor.rgb,
// metallic / roughness factors, baseColor / metallicRoughness / normal texture indices
// (:160-186); model matrix = T * R * S with the glm quaternion (w = rotation[3], :229-236)
// and glm's mat4 product order; textures decoded to RGBA8, rows as stored (the reference
// leaves the y-mirror commented out, :61-70).
//
// Deliberate deviations (the reference's loader bugs):
//   * index accessors of any component type (the reference reads uint16 only, :143);
//   * byteStride honoured (ignored by the reference);
//   * the whole node hierarchy with composed transforms (the reference takes root nodes
//     only and would index meshes[-1] for a node without a mesh);
//   * a missing NORMAL stays missing (the reference's operator[] inserts accessor 0, :117);
//   * no bufferView/buffer clobbering (the reference assigns through references, :106-143);
//   * a missing material gets the glTF default material (albedo 1, metallic 1, roughness 1)
//     where the reference leaves metallic/roughness/texture ids uninitialised (:158-161);
//   * texture ids stay aligned with glTF texture indices; a texture that cannot be decoded
//     is an error (the reference skips it and shifts every later id, :55-77).
// Images: PNG is decoded here (zlib inflate + unfiltering); other formats (JPEG, ...) go
// through the caller's decode callback, as stb_image would have decoded them.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/ptamd.h"

namespace {

thread_local std::string g_gltf_error;

// ---- minimal JSON ---------------------------------------------------------------------
struct Json {
    enum Type { Null, Bool, Num, Str, Arr, Obj } type = Null;
    bool b = false;
    double num = 0.0;
    std::string str;
    std::vector<Json> arr;
    std::vector<std::pair<std::string, Json>> obj;

    const Json* get(const char* key) const {
        if (type != Obj) return nullptr;
        for (const auto& kv : obj)
            if (kv.first == key) return &kv.second;
        return nullptr;
    }
    double num_or(const char* key, double d) const {
        const Json* v = get(key);
        return v && v->type == Num ? v->num : d;
    }
    int int_or(const char* key, int d) const {  // d also for a non-finite or out-of-int-range number
        const double x = num_or(key, (double)d);
        return (std::isfinite(x) && x >= -2147483648.0 && x <= 2147483647.0) ? (int)x : d;
    }
    std::string str_or(const char* key, const std::string& d) const {
        const Json* v = get(key);
        return v && v->type == Str ? v->str : d;
    }
    size_t size() const { return type == Arr ? arr.size() : 0; }
    // bounds-checked: an index past the end (or into a non-array) reads as JSON null
    const Json& at(size_t i) const {
        static const Json null_value;
        return (type == Arr && i < arr.size()) ? arr[i] : null_value;
    }
};

// A JSON number used as an index or a size: finite, integral, in [0, limit).  Untrusted files
// may hold negative, fractional, huge or non-numeric values; every conversion goes through here
// (casting such a double to an integer is undefined behaviour).
bool as_index(const Json* v, size_t limit, size_t& out) {
    if (!v || v->type != Json::Num || !std::isfinite(v->num) || v->num < 0.0 || v->num != std::floor(v->num) ||
        v->num >= (double)limit)
        return false;
    out = (size_t)v->num;
    return true;
}
// An optional non-negative integer field (byteOffset, byteStride, count, ...); `d` when absent.
bool size_field(const Json& o, const char* key, size_t d, size_t limit, size_t& out) {
    const Json* v = o.get(key);
    if (!v) {
        out = d;
        return true;
    }
    return as_index(v, limit, out);
}
constexpr size_t kMaxElements = (size_t)1 << 28;  // accessor counts, texels: refuse absurd sizes

struct JsonParser {
    const char* p;
    const char* end;
    std::string err;

    void ws() {
        while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
    }
    bool fail(const char* m) {
        if (err.empty()) err = m;
        return false;
    }
    static void utf8(std::string& s, uint32_t c) {
        if (c < 0x80) {
            s.push_back((char)c);
        } else if (c < 0x800) {
            s.push_back((char)(0xC0 | (c >> 6)));
            s.push_back((char)(0x80 | (c & 0x3F)));
        } else if (c < 0x10000) {
            s.push_back((char)(0xE0 | (c >> 12)));
            s.push_back((char)(0x80 | ((c >> 6) & 0x3F)));
            s.push_back((char)(0x80 | (c & 0x3F)));
        } else {
            s.push_back((char)(0xF0 | (c >> 18)));
            s.push_back((char)(0x80 | ((c >> 12) & 0x3F)));
            s.push_back((char)(0x80 | ((c >> 6) & 0x3F)));
            s.push_back((char)(0x80 | (c & 0x3F)));
        }
    }
    bool hex4(uint32_t& v) {
        if (end - p < 4) return fail("json: bad \\u escape");
        v = 0;
        for (int k = 0; k < 4; ++k) {
            char c = *p++;
            v <<= 4;
            if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
            else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
            else return fail("json: bad \\u escape");
        }
        return true;
    }
    bool string(std::string& s) {
        if (p >= end || *p != '"') return fail("json: expected string");
        ++p;
        while (p < end && *p != '"') {
            char c = *p++;
            if (c != '\\') {
                s.push_back(c);
                continue;
            }
            if (p >= end) return fail("json: bad escape");
            char e = *p++;
            switch (e) {
                case '"': s.push_back('"'); break;
                case '\\': s.push_back('\\'); break;
                case '/': s.push_back('/'); break;
                case 'b': s.push_back('\b'); break;
                case 'f': s.push_back('\f'); break;
                case 'n': s.push_back('\n'); break;
                case 'r': s.push_back('\r'); break;
                case 't': s.push_back('\t'); break;
                case 'u': {
                    uint32_t v;
                    if (!hex4(v)) return false;
                    if (v >= 0xD800 && v < 0xDC00 && end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
                        p += 2;
                        uint32_t lo;
                        if (!hex4(lo)) return false;
                        v = 0x10000 + ((v - 0xD800) << 10) + (lo - 0xDC00);
                    }
                    utf8(s, v);
                    break;
                }
                default: return fail("json: bad escape");
            }
        }
        if (p >= end) return fail("json: unterminated string");
        ++p;
        return true;
    }
    bool value(Json& v, int depth) {
        if (depth > 256) return fail("json: nesting too deep");
        ws();
        if (p >= end) return fail("json: unexpected end");
        char c = *p;
        if (c == '{') {
            ++p;
            v.type = Json::Obj;
            ws();
            if (p < end && *p == '}') {
                ++p;
                return true;
            }
            while (true) {
                ws();
                std::string key;
                if (!string(key)) return false;
                ws();
                if (p >= end || *p != ':') return fail("json: expected ':'");
                ++p;
                v.obj.emplace_back(key, Json());
                if (!value(v.obj.back().second, depth + 1)) return false;
                ws();
                if (p < end && *p == ',') {
                    ++p;
                    continue;
                }
                if (p < end && *p == '}') {
                    ++p;
                    return true;
                }
                return fail("json: expected ',' or '}'");
            }
        }
        if (c == '[') {
            ++p;
            v.type = Json::Arr;
            ws();
            if (p < end && *p == ']') {
                ++p;
                return true;
            }
            while (true) {
                v.arr.emplace_back();
                if (!value(v.arr.back(), depth + 1)) return false;
                ws();
                if (p < end && *p == ',') {
                    ++p;
                    continue;
                }
                if (p < end && *p == ']') {
                    ++p;
                    return true;
                }
                return fail("json: expected ',' or ']'");
            }
        }
        if (c == '"') {
            v.type = Json::Str;
            return string(v.str);
        }
        if (end - p >= 4 && !std::strncmp(p, "true", 4)) {
            p += 4;
            v.type = Json::Bool;
            v.b = true;
            return true;
        }
        if (end - p >= 5 && !std::strncmp(p, "false", 5)) {
            p += 5;
            v.type = Json::Bool;
            return true;
        }
        if (end - p >= 4 && !std::strncmp(p, "null", 4)) {
            p += 4;
            return true;
        }
        std::string num;
        while (p < end && *p && std::strchr("+-0123456789.eE", *p)) num.push_back(*p++);
        if (num.empty()) return fail("json: unexpected character");
        char* e = nullptr;
        v.type = Json::Num;
        v.num = std::strtod(num.c_str(), &e);
        if (!e || *e) return fail("json: bad number");
        return true;
    }
};

// ---- zlib inflate (RFC 1950/1951) + PNG -------------------------------------------------
struct BitIn {
    const uint8_t* d;
    size_t n, pos = 0;
    uint32_t bitbuf = 0;
    int bitcnt = 0;
    bool bad = false;
    int bits(int k) {
        while (bitcnt < k) {
            if (pos >= n) {
                bad = true;
                return 0;
            }
            bitbuf |= (uint32_t)d[pos++] << bitcnt;
            bitcnt += 8;
        }
        int v = (int)(bitbuf & ((1u << k) - 1));
        bitbuf >>= k;
        bitcnt -= k;
        return v;
    }
};

struct Huff {
    uint16_t count[16] = {0};
    uint16_t sym[320] = {0};
    bool build(const uint8_t* len, int n) {
        std::memset(count, 0, sizeof count);
        for (int i = 0; i < n; ++i) count[len[i]]++;
        count[0] = 0;
        int left = 1;
        for (int l = 1; l < 16; ++l) {
            left <<= 1;
            left -= count[l];
            if (left < 0) return false;
        }
        uint16_t offs[16];
        offs[1] = 0;
        for (int l = 1; l < 15; ++l) offs[l + 1] = (uint16_t)(offs[l] + count[l]);
        for (int i = 0; i < n; ++i)
            if (len[i]) sym[offs[len[i]]++] = (uint16_t)i;
        return true;
    }
    int decode(BitIn& in) const {
        int code = 0, first = 0, index = 0;
        for (int l = 1; l < 16; ++l) {
            code |= in.bits(1);
            int c = count[l];
            if (code - c < first) return sym[index + (code - first)];
            index += c;
            first += c;
            first <<= 1;
            code <<= 1;
            if (in.bad) return -1;
        }
        return -1;
    }
};

bool inflate(const uint8_t* src, size_t n, std::vector<uint8_t>& out) {
    if (n < 2 || (src[0] & 0x0f) != 8 || ((src[0] << 8) | src[1]) % 31) return false;  // zlib header
    BitIn in{src + 2, n - 2};
    static const uint16_t lbase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                       35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
    static const uint8_t lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
    static const uint16_t dbase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129,
                                       193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
    static const uint8_t dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
    int final = 0;
    while (!final) {
        final = in.bits(1);
        const int type = in.bits(2);
        if (in.bad) return false;
        if (type == 0) {  // stored
            in.bitbuf = 0;
            in.bitcnt = 0;
            if (in.pos + 4 > in.n) return false;
            const uint16_t len = (uint16_t)(in.d[in.pos] | (in.d[in.pos + 1] << 8));
            in.pos += 4;
            if (in.pos + len > in.n) return false;
            out.insert(out.end(), in.d + in.pos, in.d + in.pos + len);
            in.pos += len;
            continue;
        }
        Huff lit, dist;
        if (type == 1) {
            uint8_t l[288];
            for (int i = 0; i < 144; ++i) l[i] = 8;
            for (int i = 144; i < 256; ++i) l[i] = 9;
            for (int i = 256; i < 280; ++i) l[i] = 7;
            for (int i = 280; i < 288; ++i) l[i] = 8;
            lit.build(l, 288);
            uint8_t d[30];
            for (int i = 0; i < 30; ++i) d[i] = 5;
            dist.build(d, 30);
        } else if (type == 2) {
            const int hlit = in.bits(5) + 257, hdist = in.bits(5) + 1, hclen = in.bits(4) + 4;
            static const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
            uint8_t cl[19] = {0};
            for (int i = 0; i < hclen; ++i) cl[order[i]] = (uint8_t)in.bits(3);
            Huff clh;
            if (!clh.build(cl, 19)) return false;
            uint8_t lens[320] = {0};
            int i = 0;
            while (i < hlit + hdist) {
                int s = clh.decode(in);
                if (s < 0 || in.bad) return false;
                if (s < 16) {
                    lens[i++] = (uint8_t)s;
                } else {
                    int rep = 0;
                    uint8_t v = 0;
                    if (s == 16) {
                        if (i == 0) return false;
                        v = lens[i - 1];
                        rep = 3 + in.bits(2);
                    } else if (s == 17) {
                        rep = 3 + in.bits(3);
                    } else {
                        rep = 11 + in.bits(7);
                    }
                    if (i + rep > hlit + hdist) return false;
                    while (rep--) lens[i++] = v;
                }
            }
            if (!lit.build(lens, hlit) || !dist.build(lens + hlit, hdist)) return false;
        } else {
            return false;
        }
        while (true) {
            int s = lit.decode(in);
            if (s < 0 || in.bad) return false;
            if (s < 256) {
                out.push_back((uint8_t)s);
            } else if (s == 256) {
                break;
            } else {
                s -= 257;
                if (s >= 29) return false;
                const int len = lbase[s] + in.bits(lext[s]);
                const int ds = dist.decode(in);
                if (ds < 0 || ds >= 30) return false;
                const size_t d = (size_t)(dbase[ds] + in.bits(dext[ds]));
                if (in.bad || d > out.size()) return false;
                const size_t from = out.size() - d;
                for (int k = 0; k < len; ++k) out.push_back(out[from + (size_t)k]);
            }
        }
    }
    return true;
}

uint32_t be32(const uint8_t* p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }

// PNG -> RGBA8 (non-interlaced; bit depths 1/2/4/8/16; all colour types).
bool decode_png(const uint8_t* d, size_t n, std::vector<uint32_t>& rgba, int& W, int& H, std::string& err) {
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (n < 8 || std::memcmp(d, sig, 8)) return (err = "png: bad signature", false);
    size_t p = 8;
    int depth = 0, ctype = 0, interlace = 0;
    std::vector<uint8_t> idat, plte, trns;
    W = H = 0;
    while (p + 8 <= n) {
        const uint32_t len = be32(d + p);
        const uint8_t* t = d + p + 4;
        const uint8_t* c = d + p + 8;
        if (p + 12 + len > n) return (err = "png: truncated chunk", false);
        if (!std::memcmp(t, "IHDR", 4)) {
            W = (int)be32(c);
            H = (int)be32(c + 4);
            depth = c[8];
            ctype = c[9];
            interlace = c[12];
        } else if (!std::memcmp(t, "PLTE", 4)) {
            plte.assign(c, c + len);
        } else if (!std::memcmp(t, "tRNS", 4)) {
            trns.assign(c, c + len);
        } else if (!std::memcmp(t, "IDAT", 4)) {
            idat.insert(idat.end(), c, c + len);
        } else if (!std::memcmp(t, "IEND", 4)) {
            break;
        }
        p += 12 + len;
    }
    if (W <= 0 || H <= 0) return (err = "png: missing IHDR", false);
    if (interlace) return (err = "png: interlaced images are not supported", false);
    const int chans = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 3 ? 1 : ctype == 4 ? 2 : ctype == 6 ? 4 : 0;
    if (!chans) return (err = "png: bad colour type", false);
    std::vector<uint8_t> raw;
    if (!inflate(idat.data(), idat.size(), raw)) return (err = "png: corrupt zlib stream", false);
    const size_t bpp_bits = (size_t)chans * (size_t)depth;
    const size_t stride = ((size_t)W * bpp_bits + 7) / 8;
    const size_t bpp = (bpp_bits + 7) / 8;
    if (raw.size() < (stride + 1) * (size_t)H) return (err = "png: short image data", false);
    std::vector<uint8_t> img(stride * (size_t)H);
    for (int y = 0; y < H; ++y) {
        const uint8_t f = raw[(size_t)y * (stride + 1)];
        const uint8_t* s = &raw[(size_t)y * (stride + 1) + 1];
        uint8_t* o = &img[(size_t)y * stride];
        const uint8_t* up = y ? &img[(size_t)(y - 1) * stride] : nullptr;
        for (size_t x = 0; x < stride; ++x) {
            const int a = x >= bpp ? o[x - bpp] : 0, b = up ? up[x] : 0, cc = (up && x >= bpp) ? up[x - bpp] : 0;
            int v = s[x];
            switch (f) {
                case 0: break;
                case 1: v += a; break;
                case 2: v += b; break;
                case 3: v += (a + b) / 2; break;
                case 4: {
                    const int pp = a + b - cc, pa = std::abs(pp - a), pb = std::abs(pp - b), pc = std::abs(pp - cc);
                    v += (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : cc);
                    break;
                }
                default: return (err = "png: bad filter", false);
            }
            o[x] = (uint8_t)v;
        }
    }
    rgba.assign((size_t)W * (size_t)H, 0);
    auto sample = [&](const uint8_t* row, int x, int ch) -> int {  // channel value scaled to 8 bits
        if (depth == 8) return row[(size_t)x * chans + ch];
        if (depth == 16) return row[2 * ((size_t)x * chans + ch)];
        const size_t bit = ((size_t)x * chans + ch) * depth;
        const int v = (row[bit / 8] >> (8 - depth - (int)(bit % 8))) & ((1 << depth) - 1);
        return ctype == 3 ? v : v * 255 / ((1 << depth) - 1);
    };
    auto raw16 = [&](const uint8_t* row, int x, int ch) -> int {
        return depth == 16 ? (row[2 * ((size_t)x * chans + ch)] << 8) | row[2 * ((size_t)x * chans + ch) + 1]
                           : (depth == 8 ? row[(size_t)x * chans + ch] : -1);
    };
    for (int y = 0; y < H; ++y) {
        const uint8_t* row = &img[(size_t)y * stride];
        for (int x = 0; x < W; ++x) {
            int r, g, b, a = 255;
            if (ctype == 3) {
                const int i = sample(row, x, 0);
                if ((size_t)(3 * i + 2) >= plte.size()) return (err = "png: palette index out of range", false);
                r = plte[3 * i];
                g = plte[3 * i + 1];
                b = plte[3 * i + 2];
                if ((size_t)i < trns.size()) a = trns[(size_t)i];
            } else if (ctype == 0 || ctype == 4) {
                r = g = b = sample(row, x, 0);
                if (ctype == 4) a = sample(row, x, 1);
                else if (trns.size() >= 2 && depth >= 8 && raw16(row, x, 0) == ((trns[0] << 8) | trns[1])) a = 0;
            } else {
                r = sample(row, x, 0);
                g = sample(row, x, 1);
                b = sample(row, x, 2);
                if (ctype == 6) a = sample(row, x, 3);
                else if (trns.size() >= 6 && depth >= 8 && raw16(row, x, 0) == ((trns[0] << 8) | trns[1]) &&
                         raw16(row, x, 1) == ((trns[2] << 8) | trns[3]) && raw16(row, x, 2) == ((trns[4] << 8) | trns[5]))
                    a = 0;
            }
            rgba[(size_t)y * (size_t)W + (size_t)x] =
                (uint32_t)r | ((uint32_t)g << 8) | ((uint32_t)b << 16) | ((uint32_t)a << 24);
        }
    }
    return true;
}

// ---- glTF ---------------------------------------------------------------------------------
std::string dir_of(const std::string& path) {
    const size_t k = path.find_last_of("/\\");
    return k == std::string::npos ? std::string() : path.substr(0, k + 1);
}

bool read_file(const std::string& path, std::vector<uint8_t>& out) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) out.insert(out.end(), buf, buf + n);
    std::fclose(f);
    return true;
}

std::string uri_decode(const std::string& s) {
    std::string o;
    for (size_t i = 0; i < s.size(); ++i) {
        if (s[i] == '%' && i + 2 < s.size()) {
            o.push_back((char)std::strtol(s.substr(i + 1, 2).c_str(), nullptr, 16));
            i += 2;
        } else {
            o.push_back(s[i]);
        }
    }
    return o;
}

bool base64(const std::string& s, std::vector<uint8_t>& out) {
    int val = 0, bits = -8;
    for (char c : s) {
        int d;
        if (c >= 'A' && c <= 'Z') d = c - 'A';
        else if (c >= 'a' && c <= 'z') d = c - 'a' + 26;
        else if (c >= '0' && c <= '9') d = c - '0' + 52;
        else if (c == '+') d = 62;
        else if (c == '/') d = 63;
        else if (c == '=') break;
        else return false;
        val = (val << 6) | d;
        bits += 6;
        if (bits >= 0) {
            out.push_back((uint8_t)((val >> bits) & 0xFF));
            bits -= 8;
        }
    }
    return true;
}

struct Mat4 {
    float m[16];  // column-major (glm)
    static Mat4 identity() {
        Mat4 r{};
        r.m[0] = r.m[5] = r.m[10] = r.m[15] = 1.0f;
        return r;
    }
};
// glm operator*(mat4, mat4): Result[c] = ((A0*B[c][0] + A1*B[c][1]) + A2*B[c][2]) + A3*B[c][3]
Mat4 mul(const Mat4& a, const Mat4& b) {
    Mat4 r{};
    for (int c = 0; c < 4; ++c)
        for (int row = 0; row < 4; ++row) {
            float v = a.m[0 * 4 + row] * b.m[c * 4 + 0];
            v = v + a.m[1 * 4 + row] * b.m[c * 4 + 1];
            v = v + a.m[2 * 4 + row] * b.m[c * 4 + 2];
            v = v + a.m[3 * 4 + row] * b.m[c * 4 + 3];
            r.m[c * 4 + row] = v;
        }
    return r;
}

// Mesh::GetModelMatrix (Mesh.cpp:6-22): translate(I, t) * toMat4(quat(w, x, y, z)) * scale(I, s)
Mat4 trs(const Json& node) {
    float t[3] = {0, 0, 0}, s[3] = {1, 1, 1}, q[4] = {0, 0, 0, 1};  // q = x, y, z, w
    if (const Json* v = node.get("translation"))
        for (size_t k = 0; k < 3 && k < v->size(); ++k) t[k] = (float)v->at(k).num;
    if (const Json* v = node.get("scale"))
        for (size_t k = 0; k < 3 && k < v->size(); ++k) s[k] = (float)v->at(k).num;
    if (const Json* v = node.get("rotation"))
        for (size_t k = 0; k < 4 && k < v->size(); ++k) q[k] = (float)v->at(k).num;
    if (const Json* v = node.get("matrix")) {
        Mat4 r{};
        for (size_t k = 0; k < 16 && k < v->size(); ++k) r.m[k] = (float)v->at(k).num;
        return r;
    }
    const float x = q[0], y = q[1], z = q[2], w = q[3];
    // glm mat3_cast
    const float qxx = x * x, qyy = y * y, qzz = z * z, qxz = x * z, qxy = x * y, qyz = y * z, qwx = w * x,
                qwy = w * y, qwz = w * z;
    Mat4 R = Mat4::identity();
    R.m[0] = 1.0f - 2.0f * (qyy + qzz);
    R.m[1] = 2.0f * (qxy + qwz);
    R.m[2] = 2.0f * (qxz - qwy);
    R.m[4] = 2.0f * (qxy - qwz);
    R.m[5] = 1.0f - 2.0f * (qxx + qzz);
    R.m[6] = 2.0f * (qyz + qwx);
    R.m[8] = 2.0f * (qxz + qwy);
    R.m[9] = 2.0f * (qyz - qwx);
    R.m[10] = 1.0f - 2.0f * (qxx + qyy);
    Mat4 T = Mat4::identity();
    T.m[12] = t[0];
    T.m[13] = t[1];
    T.m[14] = t[2];
    Mat4 S = Mat4::identity();
    S.m[0] = s[0];
    S.m[5] = s[1];
    S.m[10] = s[2];
    return mul(mul(T, R), S);
}

}  // namespace

struct pt_model {
    struct MeshData {
        std::vector<float> v, n, uv;
        std::vector<int32_t> idx;
        std::string name;
    };
    std::vector<MeshData> data;
    std::vector<pt_mesh> meshes;
    std::vector<std::vector<uint32_t>> tex_pixels;
    std::vector<pt_texture> textures;
    pt_scene scene{};
};

namespace {

struct Loader {
    const Json& root;
    std::vector<std::vector<uint8_t>> buffers;
    std::string base;
    std::string err;
    pt_model& out;
    pt_image_decode_fn decode;
    void* user;

    bool fail(const std::string& m) {
        if (err.empty()) err = m;
        return false;
    }

    bool load_buffers(const std::vector<uint8_t>* glb_bin) {
        const Json* bufs = root.get("buffers");
        for (size_t i = 0; bufs && i < bufs->size(); ++i) {
            const Json& b = bufs->at(i);
            std::vector<uint8_t> data;
            const std::string uri = b.str_or("uri", "");
            if (uri.empty()) {
                if (!glb_bin || i != 0) return fail("gltf: buffer without uri");
                data = *glb_bin;
            } else if (uri.compare(0, 5, "data:") == 0) {
                const size_t k = uri.find(";base64,");
                if (k == std::string::npos || !base64(uri.substr(k + 8), data)) return fail("gltf: bad data uri");
            } else if (!read_file(base + uri_decode(uri), data)) {
                return fail("gltf: cannot read buffer " + base + uri);
            }
            size_t blen = 0;
            if (!size_field(b, "byteLength", 0, (size_t)1 << 40, blen)) return fail("gltf: bad buffer byteLength");
            if (data.size() < blen) return fail("gltf: buffer shorter than byteLength");
            buffers.push_back(std::move(data));
        }
        return true;
    }

    // Accessor -> floats (count * ncomp), with normalisation of integer types when asked.
    bool read_accessor(const Json* index, int want_comp, std::vector<double>& vals, size_t& count) {
        const Json* accs = root.get("accessors");
        size_t ai = 0;
        if (!accs || !as_index(index, accs->size(), ai)) return fail("gltf: bad accessor index");
        const Json& a = accs->at(ai);
        if (a.get("sparse")) return fail("gltf: sparse accessors are not supported");
        const std::string type = a.str_or("type", "");
        const int nc = type == "SCALAR" ? 1 : type == "VEC2" ? 2 : type == "VEC3" ? 3 : type == "VEC4" ? 4 : 0;
        if (!nc || (want_comp && nc != want_comp)) return fail("gltf: unexpected accessor type " + type);
        const int ct = a.int_or("componentType", 0);
        const int csize = (ct == 5120 || ct == 5121) ? 1 : (ct == 5122 || ct == 5123) ? 2 : (ct == 5125 || ct == 5126) ? 4 : 0;
        if (!csize) return fail("gltf: bad componentType");
        const bool norm = a.get("normalized") && a.get("normalized")->b;
        if (!size_field(a, "count", 0, kMaxElements, count)) return fail("gltf: bad accessor count");
        const Json* bvi = a.get("bufferView");
        if (!bvi) {  // all zeros (glTF 2.0 §3.6.2.1)
            vals.assign(count * (size_t)nc, 0.0);
            return true;
        }
        const Json* views = root.get("bufferViews");
        size_t vi = 0, bi = 0, voff = 0, aoff = 0, stride = 0;
        if (!views || !as_index(bvi, views->size(), vi)) return fail("gltf: bad bufferView index");
        const Json& v = views->at(vi);
        if (!as_index(v.get("buffer"), buffers.size(), bi)) return fail("gltf: bad buffer index");
        const std::vector<uint8_t>& buf = buffers[bi];
        const size_t elem = (size_t)nc * (size_t)csize;
        if (!size_field(v, "byteOffset", 0, buf.size() + 1, voff) || !size_field(a, "byteOffset", 0, buf.size() + 1, aoff) ||
            !size_field(v, "byteStride", elem, 256, stride) || stride < elem)
            return fail("gltf: bad accessor offset or stride");
        const size_t off = voff + aoff;
        // overflow-free form of off + stride * (count - 1) + elem <= buf.size()
        if (count && (off > buf.size() || elem > buf.size() - off || count - 1 > (buf.size() - off - elem) / stride))
            return fail("gltf: accessor out of range");
        vals.assign(count * (size_t)nc, 0.0);
        for (size_t i = 0; i < count; ++i) {
            const uint8_t* e = &buf[off + stride * i];
            for (int k = 0; k < nc; ++k) {
                const uint8_t* c = e + (size_t)k * (size_t)csize;
                double x = 0;
                switch (ct) {
                    case 5120: { int8_t t; std::memcpy(&t, c, 1); x = norm ? std::fmax(t / 127.0, -1.0) : t; break; }
                    case 5121: x = norm ? c[0] / 255.0 : c[0]; break;
                    case 5122: { int16_t t; std::memcpy(&t, c, 2); x = norm ? std::fmax(t / 32767.0, -1.0) : t; break; }
                    case 5123: { uint16_t t; std::memcpy(&t, c, 2); x = norm ? t / 65535.0 : t; break; }
                    case 5125: { uint32_t t; std::memcpy(&t, c, 4); x = t; break; }
                    case 5126: { float t; std::memcpy(&t, c, 4); x = t; break; }
                }
                vals[i * (size_t)nc + (size_t)k] = x;
            }
        }
        return true;
    }

    bool add_primitive(const Json& prim, const Mat4& world, const std::string& name) {
        const int mode = prim.int_or("mode", 4);
        if (mode != 4) return true;  // only triangle lists are renderable (OptiX GAS of triangles)
        const Json* attrs = prim.get("attributes");
        if (!attrs || !attrs->get("POSITION")) return fail("gltf: primitive without POSITION");
        pt_model::MeshData md;
        md.name = name;
        std::vector<double> vals;
        size_t nv = 0, cnt = 0;
        if (!read_accessor(attrs->get("POSITION"), 3, vals, nv)) return false;
        if (nv > (size_t)0x7fffffff) return fail("gltf: too many vertices");
        md.v.assign(vals.begin(), vals.end());
        if (const Json* a = attrs->get("NORMAL")) {
            if (!read_accessor(a, 3, vals, cnt)) return false;
            if (cnt != nv) return fail("gltf: NORMAL count differs from POSITION");
            md.n.assign(vals.begin(), vals.end());
        }
        if (const Json* a = attrs->get("TEXCOORD_0")) {
            if (!read_accessor(a, 2, vals, cnt)) return false;
            if (cnt != nv) return fail("gltf: TEXCOORD_0 count differs from POSITION");
            md.uv.assign(vals.begin(), vals.end());
        }
        if (const Json* ii = prim.get("indices")) {
            if (!read_accessor(ii, 1, vals, cnt)) return false;
            for (double x : vals) {
                if (x < 0 || x >= (double)nv) return fail("gltf: index out of range");
                md.idx.push_back((int32_t)x);
            }
        } else {
            for (size_t i = 0; i < nv; ++i) md.idx.push_back((int32_t)i);
        }
        md.idx.resize(md.idx.size() / 3 * 3);
        pt_mesh m{};
        std::memcpy(m.model_matrix, world.m, sizeof world.m);
        // glTF default material (albedo 1, metallic 1, roughness 1) when none is given
        m.albedo[0] = m.albedo[1] = m.albedo[2] = 1.0f;
        m.metallic = 1.0f;
        m.roughness = 1.0f;
        m.albedo_tex = m.normal_tex = m.metal_rough_tex = -1;
        const int mi = prim.int_or("material", -1);
        const Json* mats = root.get("materials");
        if (mats && mi >= 0 && (size_t)mi < mats->size()) {  // ModelLoader.cpp:158-186
            const Json& mat = mats->at((size_t)mi);
            if (const Json* pbr = mat.get("pbrMetallicRoughness")) {
                if (const Json* bc = pbr->get("baseColorFactor"))
                    for (size_t k = 0; k < 3 && k < bc->size(); ++k) m.albedo[k] = (float)bc->at(k).num;
                m.metallic = (float)pbr->num_or("metallicFactor", 1.0);
                m.roughness = (float)pbr->num_or("roughnessFactor", 1.0);
                if (const Json* t = pbr->get("baseColorTexture")) m.albedo_tex = t->int_or("index", -1);
                if (const Json* t = pbr->get("metallicRoughnessTexture")) m.metal_rough_tex = t->int_or("index", -1);
            }
            if (const Json* t = mat.get("normalTexture")) m.normal_tex = t->int_or("index", -1);
        }
        out.data.push_back(std::move(md));
        out.meshes.push_back(m);
        return true;
    }

    bool walk(const Json* index, const Mat4& parent, int depth) {
        const Json* nodes = root.get("nodes");
        size_t ni = 0;
        if (!nodes || !as_index(index, nodes->size(), ni)) return fail("gltf: bad node index");
        if (depth > 512) return fail("gltf: node hierarchy too deep (cycle?)");
        const Json& node = nodes->at(ni);
        const Mat4 world = mul(parent, trs(node));
        if (const Json* mj = node.get("mesh")) {
            const Json* meshes = root.get("meshes");
            size_t mi = 0;
            if (!meshes || !as_index(mj, meshes->size(), mi)) return fail("gltf: bad mesh index");
            const Json* prims = meshes->at(mi).get("primitives");
            for (size_t p = 0; prims && p < prims->size(); ++p)
                if (!add_primitive(prims->at(p), world, node.str_or("name", ""))) return false;
        }
        if (const Json* ch = node.get("children"))
            for (size_t k = 0; k < ch->size(); ++k)
                if (!walk(&ch->at(k), world, depth + 1)) return false;
        return true;
    }

    bool load_textures() {
        const Json* texs = root.get("textures");
        const Json* imgs = root.get("images");
        for (size_t i = 0; texs && i < texs->size(); ++i) {
            size_t src = 0;
            if (!imgs || !as_index(texs->at(i).get("source"), imgs->size(), src)) return fail("gltf: texture without image");
            const Json& im = imgs->at(src);
            std::vector<uint8_t> bytes;
            const std::string uri = im.str_or("uri", "");
            if (!uri.empty()) {
                if (uri.compare(0, 5, "data:") == 0) {
                    const size_t k = uri.find(";base64,");
                    if (k == std::string::npos || !base64(uri.substr(k + 8), bytes)) return fail("gltf: bad image data uri");
                } else if (!read_file(base + uri_decode(uri), bytes)) {
                    return fail("gltf: cannot read image " + base + uri);
                }
            } else if (const Json* bv = im.get("bufferView")) {
                const Json* views = root.get("bufferViews");
                size_t vi = 0, bi = 0, off = 0, len = 0;
                if (!views || !as_index(bv, views->size(), vi)) return fail("gltf: bad image bufferView index");
                const Json& v = views->at(vi);
                if (!as_index(v.get("buffer"), buffers.size(), bi)) return fail("gltf: bad image buffer index");
                const std::vector<uint8_t>& b = buffers[bi];
                if (!size_field(v, "byteOffset", 0, b.size() + 1, off) || !size_field(v, "byteLength", 0, b.size() + 1, len) ||
                    len > b.size() - off)
                    return fail("gltf: image bufferView out of range");
                bytes.assign(b.begin() + (long)off, b.begin() + (long)(off + len));
            }
            std::vector<uint32_t> px;
            int w = 0, h = 0;
            std::string perr;
            if (bytes.size() >= 8 && bytes[0] == 137 && bytes[1] == 'P' && bytes[2] == 'N' && bytes[3] == 'G') {
                if (!decode_png(bytes.data(), bytes.size(), px, w, h, perr)) return fail("gltf: " + perr);
            } else {
                if (!decode) return fail("gltf: image " + std::to_string(src) + " is not PNG and no decoder was given");
                int32_t dw = 0, dh = 0;
                if (decode(bytes.data(), bytes.size(), &dw, &dh, nullptr, user) != 0 || dw <= 0 || dh <= 0 ||
                    (size_t)dw * (size_t)dh > kMaxElements)
                    return fail("gltf: decoder failed on image " + std::to_string(src));
                px.assign((size_t)dw * (size_t)dh, 0);
                if (decode(bytes.data(), bytes.size(), &dw, &dh, reinterpret_cast<uint8_t*>(px.data()), user) != 0)
                    return fail("gltf: decoder failed on image " + std::to_string(src));
                w = dw;
                h = dh;
            }
            out.tex_pixels.push_back(std::move(px));
            out.textures.push_back(pt_texture{nullptr, w, h});
        }
        return true;
    }
};

}  // namespace

extern "C" {

const char* pt_model_last_error(void) { return g_gltf_error.c_str(); }

static int load_gltf_impl(const char* path, pt_image_decode_fn decode, void* user, pt_model** out);

int pt_model_load_gltf(const char* path, pt_image_decode_fn decode, void* user, pt_model** out) {
    // nothing may unwind through the C ABI: an allocation failure (or any other exception)
    // on a malformed file becomes an error status
    try {
        return load_gltf_impl(path, decode, user, out);
    } catch (const std::exception& e) {
        g_gltf_error = std::string("pt_model_load_gltf: ") + e.what();
    } catch (...) {
        g_gltf_error = "pt_model_load_gltf: unexpected exception";
    }
    if (out) *out = nullptr;
    return PT_ERR_INVALID;
}

static int load_gltf_impl(const char* path, pt_image_decode_fn decode, void* user, pt_model** out) {
    if (!path || !out) {
        g_gltf_error = "pt_model_load_gltf: NULL argument";
        return PT_ERR_INVALID;
    }
    *out = nullptr;
    std::vector<uint8_t> file;
    if (!read_file(path, file)) {
        g_gltf_error = std::string("pt_model_load_gltf: cannot read ") + path;
        return PT_ERR_INVALID;
    }
    std::string json_text;
    std::vector<uint8_t> bin;
    bool glb = false;
    if (file.size() >= 12 && !std::memcmp(file.data(), "glTF", 4)) {  // binary container
        glb = true;
        size_t p = 12;
        while (p + 8 <= file.size()) {
            uint32_t len, type;
            std::memcpy(&len, &file[p], 4);
            std::memcpy(&type, &file[p + 4], 4);
            if (p + 8 + len > file.size()) break;
            if (type == 0x4E4F534Au) json_text.assign((const char*)&file[p + 8], len);
            if (type == 0x004E4942u) bin.assign(file.begin() + (long)(p + 8), file.begin() + (long)(p + 8 + len));
            p += 8 + ((len + 3) & ~3u);
        }
    } else {
        json_text.assign(file.begin(), file.end());
    }
    Json root;
    JsonParser jp{json_text.data(), json_text.data() + json_text.size(), {}};
    if (!jp.value(root, 0) || root.type != Json::Obj) {
        g_gltf_error = "pt_model_load_gltf: " + (jp.err.empty() ? std::string("not a JSON object") : jp.err);
        return PT_ERR_INVALID;
    }
    std::unique_ptr<pt_model> m(new pt_model());
    Loader L{root, {}, dir_of(path), {}, *m, decode, user};
    bool ok = L.load_buffers(glb ? &bin : nullptr);
    if (ok) {
        const Json* scenes = root.get("scenes");
        const int si = root.int_or("scene", 0);  // the reference loads scenes[0] (ModelLoader.cpp:35)
        if (scenes && si >= 0 && (size_t)si < scenes->size()) {
            const Json* nodes = scenes->at((size_t)si).get("nodes");
            for (size_t k = 0; ok && nodes && k < nodes->size(); ++k)
                ok = L.walk(&nodes->at(k), Mat4::identity(), 0);
        }
    }
    if (ok) ok = L.load_textures();
    if (!ok) {
        g_gltf_error = "pt_model_load_gltf: " + L.err;
        return PT_ERR_INVALID;
    }
    for (size_t i = 0; i < m->meshes.size(); ++i) {
        pt_model::MeshData& d = m->data[i];
        pt_mesh& pm = m->meshes[i];
        pm.vertices = d.v.data();
        pm.normals = d.n.empty() ? nullptr : d.n.data();
        pm.texcoords = d.uv.empty() ? nullptr : d.uv.data();
        pm.indices = d.idx.data();
        pm.n_vertices = (int32_t)(d.v.size() / 3);
        pm.n_triangles = (int32_t)(d.idx.size() / 3);
    }
    for (size_t i = 0; i < m->textures.size(); ++i) m->textures[i].rgba8 = m->tex_pixels[i].data();
    m->scene.meshes = m->meshes.data();
    m->scene.n_meshes = (int32_t)m->meshes.size();
    m->scene.textures = m->textures.data();
    m->scene.n_textures = (int32_t)m->textures.size();
    *out = m.release();
    return PT_OK;
}

const pt_scene* pt_model_scene(const pt_model* m) { return m ? &m->scene : nullptr; }

const char* pt_model_mesh_name(const pt_model* m, int32_t i) {
    return (m && i >= 0 && (size_t)i < m->data.size()) ? m->data[(size_t)i].name.c_str() : nullptr;
}

int pt_model_destroy(pt_model* m) {
    delete m;
    return PT_OK;
}

int pt_image_decode_png(const uint8_t* data, size_t size, int32_t* width, int32_t* height, uint8_t* rgba_out) {
    if (!data || !width || !height) return PT_ERR_INVALID;
    std::vector<uint32_t> px;
    int w = 0, h = 0;
    std::string err;
    if (!decode_png(data, size, px, w, h, err)) {
        g_gltf_error = err;
        return PT_ERR_INVALID;
    }
    *width = w;
    *height = h;
    if (rgba_out) std::memcpy(rgba_out, px.data(), px.size() * 4);
    return PT_OK;
}

}  // extern "C"

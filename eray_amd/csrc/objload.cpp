// objload.cpp — Object::load_obj + Object::build (src/lib/object.rs:101-230, 396-421) for hosts
// that feed the C-ABI from an .obj file: the faces' vertex copies as three flat float arrays
// (eray_object's layout).  The same dialect and the same failures as the reference: every input
// that panics there returns ERAY_E_PARSE, build()'s Err ERAY_E_BUILD (eray_amd/objfile.py is the
// Python statement of the same rules; tests/test_objfile.py holds both to the oracle's cases).
//
// One pass over the file in memory, no per-line allocation: the reference's loader is input
// handling, not part of the per-frame path, but a 1M-face mesh should load in a fraction of a
// second (the Python statement takes seconds).
#include <cerrno>
#include <charconv>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/eray_hip.h"

int eray_internal_error(eray_ctx* ctx, int code, const char* msg);  // capi.cpp

namespace {

struct Fail {
    int code;
    std::string msg;
};

[[noreturn]] void parse_fail(size_t line, const std::string& what) {
    throw Fail{ERAY_E_PARSE, "line " + std::to_string(line) + ": " + what};
}

// str::split_whitespace's separators within a line: char::is_whitespace, Unicode White_Space —
// ASCII \t \v \f \r and space ('\n' ends the line), U+0085, U+00A0, U+1680, U+2000-U+200A,
// U+2028, U+2029, U+202F, U+205F, U+3000 (as UTF-8).  Returns the separator's length in bytes,
// or 0.  (The file is valid UTF-8 by then: read_to_string, utf8_valid.)
inline size_t ws_len(const char* q, const char* e) {
    const unsigned char c = (unsigned char)*q;
    if (c == ' ' || c == '\t' || c == '\v' || c == '\f' || c == '\r') return 1;
    if (c < 0xC2) return 0;
    const unsigned char c1 = e - q > 1 ? (unsigned char)q[1] : 0, c2 = e - q > 2 ? (unsigned char)q[2] : 0;
    if (c == 0xC2) return (c1 == 0x85 || c1 == 0xA0) ? 2 : 0;
    if (c == 0xE1) return (c1 == 0x9A && c2 == 0x80) ? 3 : 0;
    if (c == 0xE2) {
        if (c1 == 0x80) return (c2 <= 0x8A || c2 == 0xA8 || c2 == 0xA9 || c2 == 0xAF) ? 3 : 0;
        return (c1 == 0x81 && c2 == 0x9F) ? 3 : 0;
    }
    if (c == 0xE3) return (c1 == 0x80 && c2 == 0x80) ? 3 : 0;
    return 0;
}

// std::fs::read_to_string fails (io::ErrorKind::InvalidData) unless the file is UTF-8 as
// str::from_utf8 defines it: no stray or missing continuation bytes, no overlong forms, no
// surrogates (U+D800-U+DFFF), nothing above U+10FFFF.
bool utf8_valid(const unsigned char* p, size_t n) {
    size_t i = 0;
    while (i < n) {
        const unsigned char c = p[i];
        if (c < 0x80) {
            ++i;
            continue;
        }
        size_t len;
        unsigned char lo = 0x80, hi = 0xBF;  // the allowed range of the second byte
        if (c >= 0xC2 && c <= 0xDF) {
            len = 2;
        } else if (c >= 0xE0 && c <= 0xEF) {
            len = 3;
            if (c == 0xE0) lo = 0xA0;
            if (c == 0xED) hi = 0x9F;
        } else if (c >= 0xF0 && c <= 0xF4) {
            len = 4;
            if (c == 0xF0) lo = 0x90;
            if (c == 0xF4) hi = 0x8F;
        } else {
            return false;
        }
        if (i + len > n || p[i + 1] < lo || p[i + 1] > hi) return false;
        for (size_t k = 2; k < len; ++k)
            if (p[i + k] < 0x80 || p[i + k] > 0xBF) return false;
        i += len;
    }
    return true;
}

struct Tok {
    const char* b;
    const char* e;
    bool operator==(const char* s) const { return (size_t)(e - b) == std::strlen(s) && std::memcmp(b, s, e - b) == 0; }
    std::string str() const { return std::string(b, e); }
};

// Rust's str::parse::<f32> grammar: [+-] then digits [. digits] | . digits, optional exponent,
// or inf / infinity / nan in any case; correctly rounded (glibc strtof).
float parse_f32(const Tok& t, size_t line) {
    const char* p = t.b;
    const char* e = t.e;
    if (p < e && (*p == '+' || *p == '-')) ++p;
    auto word = [&](const char* w) {
        const size_t n = std::strlen(w);
        if ((size_t)(e - p) != n) return false;
        for (size_t i = 0; i < n; ++i)
            if ((p[i] | 0x20) != w[i]) return false;
        return true;
    };
    bool ok;
    if (word("inf") || word("infinity") || word("nan")) {
        ok = true;
    } else {
        const char* q = p;
        size_t digits = 0;
        while (q < e && *q >= '0' && *q <= '9') ++q, ++digits;
        if (q < e && *q == '.') {
            ++q;
            while (q < e && *q >= '0' && *q <= '9') ++q, ++digits;
        }
        ok = digits > 0;
        if (ok && q < e && (*q == 'e' || *q == 'E')) {
            ++q;
            if (q < e && (*q == '+' || *q == '-')) ++q;
            size_t ed = 0;
            while (q < e && *q >= '0' && *q <= '9') ++q, ++ed;
            ok = ed > 0;
        }
        ok = ok && q == e;
    }
    if (!ok) parse_fail(line, "Failed to parse coords, should be an f32: " + t.str());
    // std::from_chars is correctly rounded like strtof (and several times faster); a leading '+'
    // is Rust's, not from_chars', and out-of-range values (inf / 0 in Rust) go to strtof
    {
        const char* b = t.b + (*t.b == '+' ? 1 : 0);
        float v;
        const auto res = std::from_chars(b, t.e, v);
        if (res.ec == std::errc() && res.ptr == t.e) return v;
    }
    char buf[128];
    std::string big;
    const size_t n = (size_t)(t.e - t.b);
    const char* s;
    if (n < sizeof buf) {
        std::memcpy(buf, t.b, n);
        buf[n] = 0;
        s = buf;
    } else {
        big = t.str();
        s = big.c_str();
    }
    return std::strtof(s, nullptr);  // (also "nan" / "inf" with their sign, as Rust's parse)
}

// a usize index: [+] digits (Rust's usize::from_str); out of range -> no value
bool parse_index(const char* b, const char* e, uint64_t* out) {
    if (b < e && *b == '+') ++b;
    if (b == e) return false;
    uint64_t v = 0;
    for (const char* q = b; q < e; ++q) {
        if (*q < '0' || *q > '9') return false;
        if (v > (UINT64_MAX - 9) / 10) v = UINT64_MAX;  // beyond every array: out of range below
        else v = v * 10 + (uint64_t)(*q - '0');
    }
    *out = v;
    return true;
}

struct Mesh {
    std::vector<float> v, n, t;      // 3, 3, 2 floats per element
    std::vector<uint32_t> faces;     // 9 per face: (v, vt, vn) x 3, zero-based
};

void load(const char* data, size_t size, Mesh& m) {
    const char* p = data;
    const char* end = data + size;
    size_t line = 0;
    Tok tok[64];
    while (p < end) {
        const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(end - p)));
        const char* le = nl ? nl : end;
        const char* next = nl ? nl + 1 : end;
        if (le > p && le[-1] == '\r') --le;  // str::lines strips "\r\n"
        const size_t ln = line++;
        const char* lp = p;
        p = next;
        if (lp == le || *lp == '#') continue;
        size_t nt = 0;
        bool more = false;
        for (const char* q = lp; q < le;) {
            for (size_t w; q < le && (w = ws_len(q, le)) != 0;) q += w;
            if (q == le) break;
            const char* b = q;
            while (q < le && !ws_len(q, le)) ++q;
            if (nt < 64) tok[nt++] = Tok{b, q};
            else more = true;
        }
        if (!nt) parse_fail(ln, "whitespace-only line (tokens.next().unwrap())");
        const Tok& mk = tok[0];
        if (mk == "o" || mk == "g") {
            if (nt < 2) parse_fail(ln, "`" + mk.str() + "` without a name");
        } else if (mk == "s") {
            if (nt < 2 || !(tok[1] == "1" || tok[1] == "on" || tok[1] == "0" || tok[1] == "off"))
                parse_fail(ln, "Unhandled smooth shading setting");
        } else if (mk == "v" || mk == "vn" || mk == "vt") {
            float c[64];
            for (size_t i = 1; i < nt; ++i) c[i - 1] = parse_f32(tok[i], ln);
            const size_t count = nt - 1 + (more ? 1 : 0);
            if (more) {  // (the count check fails anyway; the extra tokens must still parse first)
                parse_fail(ln, "Invalid coordinate count");
            }
            if (count < 2 || count >= 4) parse_fail(ln, "Invalid coordinate count: " + std::to_string(count));
            if (mk == "vt") {
                m.t.push_back(c[0]);
                m.t.push_back(c[1]);
            } else {
                if (count < 3) parse_fail(ln, "coords[0..=2] out of range");
                auto& dst = mk == "v" ? m.v : m.n;
                dst.insert(dst.end(), c, c + 3);
            }
        } else if (mk == "f") {
            uint32_t idx[9];
            size_t nv = 0;
            const size_t sizes[3] = {m.v.size() / 3, m.t.size() / 2, m.n.size() / 3};
            static const char* what[3] = {"vertex", "uv", "normal"};
            for (size_t i = 1; i < nt; ++i) {
                const char* b = tok[i].b;
                const char* e = tok[i].e;
                bool parts_left = true;  // str::split('/') has a k-th part
                uint32_t trip[3];
                for (int k = 0; k < 3; ++k) {
                    const char* s = b;
                    while (s < e && *s != '/') ++s;
                    uint64_t v = 0;
                    if (!parts_left || !parse_index(b, s, &v))
                        parse_fail(ln, std::string("missing ") + what[k] + " index in `" + tok[i].str() + "`");
                    if (v == 0 || v > sizes[k])
                        parse_fail(ln, std::string(what[k]) + " index " + std::to_string(v) + " out of range");
                    trip[k] = (uint32_t)(v - 1);
                    parts_left = s < e;  // a '/' follows: the next part exists (possibly empty)
                    b = parts_left ? s + 1 : e;
                }
                if (nv < 3) std::memcpy(idx + 3 * nv, trip, sizeof trip);
                ++nv;
            }
            if (more) ++nv;
            if (nv != 3) parse_fail(ln, "Invalid vertex count for face (should be 3, is " + std::to_string(nv) + ")");
            m.faces.insert(m.faces.end(), idx, idx + 9);
        } else {
            parse_fail(ln, "Unhandled marker " + mk.str());
        }
    }
    if (m.v.empty()) throw Fail{ERAY_E_BUILD, "Missing vertices"};
    if (m.n.empty()) throw Fail{ERAY_E_BUILD, "Missing normals"};
}

}  // namespace

extern "C" int eray_obj_load(const char* path, eray_obj_mesh* out) {
    if (!path || !out) return eray_internal_error(nullptr, ERAY_E_INVALID_ARGUMENT, "null argument");
    std::memset(out, 0, sizeof *out);
    FILE* f = std::fopen(path, "rb");
    if (!f) return eray_internal_error(nullptr, ERAY_E_IO, (std::string("cannot read ") + path).c_str());
    std::vector<char> data;
    bool err = std::fseek(f, 0, SEEK_END) != 0;
    const long size = err ? -1L : std::ftell(f);
    err = err || size < 0 || std::fseek(f, 0, SEEK_SET) != 0;
    if (!err) {  // the whole file in one read
        data.resize((size_t)size);
        err = std::fread(data.data(), 1, data.size(), f) != data.size();
    }
    err = err || std::ferror(f) != 0;
    std::fclose(f);
    if (err) return eray_internal_error(nullptr, ERAY_E_IO, (std::string("cannot read ") + path).c_str());
    if (!utf8_valid(reinterpret_cast<const unsigned char*>(data.data()), data.size()))
        return eray_internal_error(nullptr, ERAY_E_IO,
                                   (std::string(path) + ": stream did not contain valid UTF-8 (read_to_string)").c_str());
    Mesh m;
    try {
        load(data.data(), data.size(), m);
    } catch (const Fail& e) {
        return eray_internal_error(nullptr, e.code, e.msg.c_str());
    } catch (const std::bad_alloc&) {
        return eray_internal_error(nullptr, ERAY_E_OUT_OF_MEMORY, "obj: out of host memory");
    }
    const size_t T = m.faces.size() / 9;
    if (T > UINT32_MAX) return eray_internal_error(nullptr, ERAY_E_UNSUPPORTED, "obj: more than 2^32 faces");
    float* pos = static_cast<float*>(std::malloc(sizeof(float) * 9 * (T ? T : 1)));
    float* nrm = static_cast<float*>(std::malloc(sizeof(float) * 9 * (T ? T : 1)));
    float* uv = static_cast<float*>(std::malloc(sizeof(float) * 6 * (T ? T : 1)));
    if (!pos || !nrm || !uv) {
        std::free(pos);
        std::free(nrm);
        std::free(uv);
        return eray_internal_error(nullptr, ERAY_E_OUT_OF_MEMORY, "obj: out of host memory");
    }
    for (size_t i = 0; i < T; ++i) {  // faces copy their vertices by value (object.rs:160-186)
        const uint32_t* x = &m.faces[9 * i];
        for (int k = 0; k < 3; ++k) {
            std::memcpy(pos + 9 * i + 3 * k, &m.v[3 * (size_t)x[3 * k]], 12);
            std::memcpy(uv + 6 * i + 2 * k, &m.t[2 * (size_t)x[3 * k + 1]], 8);
            std::memcpy(nrm + 9 * i + 3 * k, &m.n[3 * (size_t)x[3 * k + 2]], 12);
        }
    }
    out->positions = pos;
    out->normals = nrm;
    out->uvs = uv;
    out->triangles = (uint32_t)T;
    return ERAY_OK;
}

extern "C" void eray_obj_free(eray_obj_mesh* mesh) {
    if (!mesh) return;
    std::free(mesh->positions);
    std::free(mesh->normals);
    std::free(mesh->uvs);
    std::memset(mesh, 0, sizeof *mesh);
}

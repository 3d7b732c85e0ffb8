// rt_host.cpp -- host front end of the MI355X renderer (librt_host.so).
//
// Drop-in for the parts of the reference that surround the hot path:
//   scene parser      main.cpp:88-602, keyword table src/config.h:17-50
//   P3 texture reader src/utility.h:59-139
//   camera            main.cpp:677-710
//   quantisation      main.cpp:760-762
//   PPM writer        main.cpp:613-650, remove_extension src/utility.h:34-41
//
// The parser keeps the reference's observable quirks (see DESIGN.md §Front
// end): tokens are split on single spaces and an empty token is fatal; a
// command with no arguments or an unknown keyword (including '#') is ignored;
// std::stof prefix parsing ("1git" -> 1); mtlcolor resets texture mode;
// 'f' vertex formats are tried as v/t/n, v//n, v/t, v with sscanf and the
// last vertex decides smooth shading; unknown v/vn/vt indices resolve to zero.
// Where the reference reads past a std::vector (too few arguments) it has
// undefined behaviour; here that is reported like a stof failure.
#include "rt_host.h"

#include <fcntl.h>
#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <charconv>
#include <climits>
#include <cstdint>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace {

// ---------------------------------------------------------------------------
// float semantics of src/definitions.h Vector3 (no FMA: built -ffp-contract=off)
// ---------------------------------------------------------------------------
struct F3 {
    float x, y, z;
};
inline F3 add(F3 a, F3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline F3 sub(F3 a, F3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline F3 scale(F3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline F3 divs(F3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline float hsum(F3 a) { return a.x + a.y + a.z; }
inline float dot(F3 a, F3 b) { return hsum({a.x * b.x, a.y * b.y, a.z * b.z}); }
inline F3 unit(F3 a) { return divs(a, std::sqrt(dot(a, a))); }
inline F3 cross(F3 a, F3 b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

// A parse failure: the std::cerr lines the reference prints before the
// exception escapes main(), and the escaping exception's what().
struct ParseFailure {
    std::vector<std::string> cerr_lines;
    std::string what;
    bool out_of_range;
};

struct Fatal : std::exception {
    ParseFailure f;
};

[[noreturn]] void fail(std::vector<std::string> lines, std::string what, bool oor = false) {
    Fatal e;
    e.f = {std::move(lines), std::move(what), oor};
    throw e;
}

}  // namespace

struct rth_scene {
    std::vector<rt_sphere_desc> spheres;
    std::vector<rt_face_desc> faces;
    std::vector<rt_light_desc> lights;
    std::vector<std::vector<unsigned char>> texels;
    std::vector<rt_texture_desc> textures;
    rt_scene_desc desc{};
    F3 eye{}, viewdir{}, updir{};
    float fov = 0;
    int width = 0, height = 0;

    void finalize() {
        desc.n_spheres = (int)spheres.size();
        desc.spheres = spheres.data();
        desc.n_faces = (int)faces.size();
        desc.faces = faces.data();
        desc.n_lights = (int)lights.size();
        desc.lights = lights.data();
        for (size_t i = 0; i < textures.size(); i++) textures[i].rgb = texels[i].data();
        desc.n_textures = (int)textures.size();
        desc.textures = textures.data();
    }
};

namespace {

// ---------------------------------------------------------------------------
// read_texture (src/utility.h:59-139): P3 only, maxval token must be "255",
// '#' lines skipped, an empty line throws (line.at(0)), tokens split on ' '.
// ---------------------------------------------------------------------------
void load_p3(const std::string &path, int &w, int &h, std::vector<unsigned char> &rgb) {
    std::ifstream in(path, std::ios::binary);
    std::string data;
    if (in) {
        in.seekg(0, std::ios::end);
        const std::streamoff size = in.tellg();
        in.seekg(0, std::ios::beg);
        if (size > 0) {
            data.resize((size_t)size);
            in.read(&data[0], size);
            data.resize((size_t)in.gcount());
        }
    } else {
        throw std::runtime_error("cannot open texture '" + path + "'");
    }
    size_t ntok = 0, need = 0, got = 0;
    w = h = 0;
    const char *p = data.data(), *end = p + data.size();
    while (p < end) {
        const char *nl = static_cast<const char *>(memchr(p, '\n', (size_t)(end - p)));
        const char *le = nl ? nl : end;
        if (le == p) throw std::out_of_range("basic_string::at: __n (which is 0) >= this->size() (which is 0)");
        if (*p != '#') {
            const char *q = p;
            while (q < le) {
                const char *t = q;
                while (t < le && *t != ' ') t++;
                if (t > q && ntok >= 4) {
                    // a texel value: std::stoi, or a plain token of 1-9 digits
                    // without it; values past the image are never converted
                    // (the reference converts only w * h * 3 tokens,
                    // src/utility.h:118-127)
                    ntok++;
                    if (got < need) {
                        int v = 0;
                        bool plain = t - q <= 9;
                        for (const char *c = q; plain && c < t; c++) plain = *c >= '0' && *c <= '9';
                        if (plain)
                            for (const char *c = q; c < t; c++) v = v * 10 + (*c - '0');
                        else
                            v = std::stoi(std::string(q, t));
                        rgb[got] = (unsigned char)std::clamp(v, 0, 255);
                    }
                    got++;
                } else if (t > q) {
                    std::string tok(q, t);
                    ntok++;
                    if (ntok == 1) {
                        if (tok != "P3") throw std::invalid_argument("Only supports PPM 'P3' file format.");
                    } else if (ntok == 2) {
                        w = std::stoi(tok);
                    } else if (ntok == 3) {
                        h = std::stoi(tok);
                        if (w > 0 && h > 0) {
                            need = (size_t)w * (size_t)h * 3;
                            rgb.assign(need, 0);
                        }
                    } else {
                        if (tok != "255") throw std::invalid_argument("PPM pixel value must be between 0 - 255 .");
                    }
                }
                q = t + 1;
            }
        }
        p = le + 1;
    }
    if (w <= 0 || h <= 0 || got < need) throw std::out_of_range("vector::_M_range_check");
}

// std::stof of a plain decimal token ([-]digits[.digits], at most 15
// significant digits -- what scene files hold) without strtof: M / 10^k with
// M < 2^53 and k <= 22 is one correctly rounded double operation on exact
// operands (Clinger's fast path), and rounding that double to float gives the
// correctly rounded float -- strtof's result -- unless the double sits
// exactly halfway between two floats (the true quotient may then lie on
// either side): those, and every other token form (exponents, '+', hex,
// inf / nan, prefixes like "1git", leading blanks), go to std::stof itself.
float fast_stof(const std::string &s) {
    static const double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                      1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
    const char *p = s.data();
    const size_t n = s.size();
    size_t i = 0;
    const bool neg = n > 0 && p[0] == '-';
    if (neg) i = 1;
    uint64_t m = 0;
    int digits = 0, frac = 0;
    bool dot = false, any = false;
    for (; i < n; i++) {
        const char c = p[i];
        if (c >= '0' && c <= '9') {
            any = true;
            if (m == 0 && c == '0') {                     // leading zeros: no significant digit
                if (dot) frac++;
                continue;
            }
            if (++digits > 15) break;               // m < 10^15 < 2^53: exact in a double
            m = m * 10 + (uint64_t)(c - '0');
            if (dot) frac++;
        } else if (c == '.' && !dot) {
            dot = true;
        } else {
            break;
        }
    }
    if (i == n && any && frac <= 22) {
        double q = (double)m / kPow10[frac];              // exact operands: one rounding
        uint64_t b;
        std::memcpy(&b, &q, sizeof b);
        const int e = (int)((b >> 52) & 0x7ff) - 1023;
        // halfway between two normal floats: the 29 bits below float precision are 100...0
        const bool tie = m != 0 && (b & ((uint64_t(1) << 29) - 1)) == (uint64_t(1) << 28);
        if (!tie && (m == 0 || (e >= -126 && e <= 127))) {
            const float f = (float)q;
            return neg ? -f : f;
        }
    }
    return std::stof(s);
}

float stof_or(const std::vector<std::string> &a, size_t i) {
    if (i >= a.size()) throw std::invalid_argument("stof");
    return fast_stof(a[i]);
}

enum Cmd { EYE, VIEWDIR, UPDIR, HFOV, IMSIZE, BKGCOLOR, MTLCOLOR, TEXTURE, SPHERE, LIGHT, V, VN, VT, FACE };

const std::pair<const char *, Cmd> kKeywords[] = {
    {"eye", EYE},     {"viewdir", VIEWDIR}, {"updir", UPDIR},     {"hfov", HFOV},       {"imsize", IMSIZE},
    {"bkgcolor", BKGCOLOR}, {"mtlcolor", MTLCOLOR}, {"texture", TEXTURE}, {"sphere", SPHERE},
    {"light", LIGHT}, {"v", V},             {"vn", VN},           {"vt", VT},           {"f", FACE},
};

bool lookup(const std::string &s, Cmd &c) {
    for (auto &kv : kKeywords)
        if (s == kv.first) {
            c = kv.second;
            return true;
        }
    return false;
}

struct Parser {
    rth_scene &S;
    std::vector<F3> verts, norms;
    std::vector<std::pair<float, float>> uvs;
    rt_material cur{};
    bool have_mtl = false, textured = false;
    int cur_tex = -1;
    bool seen[6] = {};

    explicit Parser(rth_scene &s) : S(s) {}

    static F3 lookup3(const std::vector<F3> &v, unsigned idx) {
        return (idx >= 1 && idx <= v.size()) ? v[idx - 1] : F3{0, 0, 0};
    }

    // each case mirrors a 'case ArgValues::...' of main.cpp:141-556; `inner`
    // is the message the case's own catch prints before rethrowing.
    void vec3_cmd(const std::vector<std::string> &a, F3 &dst, const char *name) {
        try {
            dst = {stof_or(a, 0), stof_or(a, 1), stof_or(a, 2)};
        } catch (const std::exception &e) {
            fail({e.what(), std::string("ERROR: Invalid args for '") + name + "' command. Please verify."}, "");
        }
    }

    void material_cmd(const std::vector<std::string> &a) {
        textured = false;
        rt_material m{};
        try {
            for (int i = 0; i < 3; i++) m.diffuse[i] = stof_or(a, i);
            for (int i = 0; i < 3; i++) m.specular[i] = stof_or(a, 3 + i);
            m.ka = stof_or(a, 6);
            m.kd = stof_or(a, 7);
            m.ks = stof_or(a, 8);
            m.n = stof_or(a, 9);
            if (a.size() == 12) {
                m.opacity = std::clamp<float>(stof_or(a, 10), 0.0f, 1.0f);
                m.eta = stof_or(a, 11);
            } else {
                m.opacity = 1.0f;
                m.eta = 1.0f;
            }
        } catch (const std::exception &e) {
            fail({e.what(), "ERROR: Issue parsing 'material' from arguments. Please verify."}, "");
        }
        cur = m;
        have_mtl = true;
    }

    void attach_material(rt_material &m, int &tex, std::vector<std::string> &why) {
        m = cur;
        tex = -1;
        if (textured) {
            if (!have_mtl || cur_tex < 0) {
                why = {"ERROR: Must define a 'mtlcolor' and 'texture'. Please verify."};
                return;
            }
            tex = cur_tex;
        } else if (!have_mtl) {
            why = {"ERROR: Must define a 'mtlcolor'. Please verify."};
        }
    }

    void sphere_cmd(const std::vector<std::string> &a) {
        rt_sphere_desc s{};
        try {
            s.radius = stof_or(a, 3);
            s.center[0] = stof_or(a, 0);
            s.center[1] = stof_or(a, 1);
            s.center[2] = stof_or(a, 2);
        } catch (const std::exception &e) {
            fail({e.what(), "ERROR: Invalid args for 'sphere' object. Please verify."}, "");
        }
        std::vector<std::string> why;
        attach_material(s.mat, s.texture, why);
        if (!why.empty()) {
            why.push_back("ERROR: Invalid args for 'mtlcolor' command. Please verify.");
            fail(why, "");
        }
        S.spheres.push_back(s);
    }

    void face_cmd(const std::vector<std::string> &a) {
        rt_face_desc f{};
        std::vector<std::string> why;
        for (int i = 0; i < 3; i++) {
            // main.cpp:487-517: formats tried in this order; the last vertex
            // token decides smooth shading
            unsigned v = 0, t = 0, n = 0;
            int fmt = 0;  // 1 v/t/n, 2 v//n, 3 v/t, 4 v
            if ((size_t)i < a.size()) {
                const char *s = a[i].c_str();
                if (sscanf(s, "%d/%d/%d", (int *)&v, (int *)&t, (int *)&n) == 3) fmt = 1;
                else if (sscanf(s, "%d//%d", (int *)&v, (int *)&n) == 2) fmt = 2;
                else if (sscanf(s, "%d/%d", (int *)&v, (int *)&t) == 2) fmt = 3;
                else if (sscanf(s, "%d", (int *)&v) == 1) fmt = 4;
            }
            if (fmt == 0) {
                why = {"ERROR: Invalid args for 'f' object. Please verify."};
                break;
            }
            F3 pv = lookup3(verts, v);
            f.v[i][0] = pv.x, f.v[i][1] = pv.y, f.v[i][2] = pv.z;
            f.smooth = (fmt == 1 || fmt == 2) ? 1 : 0;
            if (fmt == 1 || fmt == 2) {
                F3 pn = lookup3(norms, n);
                f.vn[i][0] = pn.x, f.vn[i][1] = pn.y, f.vn[i][2] = pn.z;
            }
            if (fmt == 1 || fmt == 3) {
                bool ok = t >= 1 && t <= uvs.size();
                f.vt[i][0] = ok ? uvs[t - 1].first : 0.0f;
                f.vt[i][1] = ok ? uvs[t - 1].second : 0.0f;
            }
        }
        if (why.empty()) attach_material(f.mat, f.texture, why);
        if (!why.empty()) {
            why.push_back("ERROR: Invalid args for 'f' (face) object. Please verify.");
            fail(why, "");
        }
        S.faces.push_back(f);
    }

    std::string name_;                       // this line's keyword token
    std::vector<std::string> args_;          // and its arguments (storage reused line to line)

    void line(const std::string &text) {
        // tokenise exactly like main.cpp:107-117
        size_t pos = 0, ntok = 0;
        while (pos < text.size()) {
            size_t sp = text.find(' ', pos);
            if (sp == std::string::npos) sp = text.size();
            if (sp == pos) fail({}, "basic_string::at: __n (which is 0) >= this->size() (which is 0)", true);
            if (ntok == 0) {
                name_.assign(text, pos, sp - pos);
            } else {
                if (args_.size() < ntok) args_.resize(ntok);
                args_[ntok - 1].assign(text, pos, sp - pos);
            }
            ntok++;
            pos = sp + 1;
        }
        if (ntok == 0) return;
        args_.resize(ntok - 1);
        const std::string &name = name_;
        const std::vector<std::string> &a = args_;
        Cmd c;
        if (a.empty() || !lookup(name, c)) return;
        try {
            dispatch(c, a);
        } catch (Fatal &e) {
            // main.cpp:558-561: every failure is reported as an unknown command
            e.f.what = "ERROR: Command '" + name + "' is undefined. Please verify input.";
            throw;
        }
    }

    void dispatch(Cmd c, const std::vector<std::string> &a) {
        switch (c) {
            case EYE: seen[1] = true; vec3_cmd(a, S.eye, "eye"); break;
            case VIEWDIR: seen[2] = true; vec3_cmd(a, S.viewdir, "viewdir"); break;
            case UPDIR: seen[3] = true; vec3_cmd(a, S.updir, "updir"); break;
            case HFOV:
                seen[4] = true;
                try {
                    S.fov = stof_or(a, 0);
                } catch (const std::exception &e) {
                    fail({e.what(), "ERROR: Invalid args for 'hfov' command. Please verify."}, "");
                }
                break;
            case IMSIZE: {
                seen[0] = true;
                const char *msg = "ERROR: Invalid image dimensions. Please verify.";
                int w = 0, h = 0;
                try {
                    if (a.size() < 2) throw std::invalid_argument("stoi");
                    h = std::stoi(a[1]);
                    w = std::stoi(a[0]);
                } catch (const std::exception &e) {
                    fail({e.what(), msg}, "");
                }
                if (h <= 1 || w <= 1) fail({msg}, "");
                S.width = w;
                S.height = h;
                break;
            }
            case BKGCOLOR:
                seen[5] = true;
                try {
                    for (int i = 0; i < 3; i++) S.desc.bkg[i] = stof_or(a, i);
                    if (a.size() > 3) S.desc.eta_bkg = std::stof(a[3]);
                } catch (const std::exception &e) {
                    fail({e.what(), "ERROR: Invalid args for 'bkgcolor' command. Please verify."}, "");
                }
                break;
            case MTLCOLOR: material_cmd(a); break;
            case TEXTURE: {
                textured = true;
                int w = 0, h = 0;
                std::vector<unsigned char> rgb;
                try {
                    load_p3(a[0], w, h, rgb);
                } catch (const std::exception &e) {
                    fail({e.what(), "ERROR: Issue reading 'texture' from ppm. Please verify."}, "");
                }
                S.texels.push_back(std::move(rgb));
                S.textures.push_back({w, h, nullptr});
                cur_tex = (int)S.textures.size() - 1;
                break;
            }
            case SPHERE: sphere_cmd(a); break;
            case LIGHT: {
                rt_light_desc l{};
                try {
                    l.w = stof_or(a, 3);
                    for (int i = 0; i < 3; i++) l.xyz[i] = stof_or(a, i);
                    for (int i = 0; i < 3; i++) l.color[i] = stof_or(a, 4 + i);
                } catch (const std::exception &e) {
                    fail({e.what(), "ERROR: Invalid args for 'light' command. Please verify."}, "");
                }
                S.lights.push_back(l);
                break;
            }
            case V:
            case VN: {
                F3 p{};
                try {
                    p = {stof_or(a, 0), stof_or(a, 1), stof_or(a, 2)};
                } catch (const std::exception &e) {
                    fail({e.what(), c == V ? "ERROR: Invalid args for vertex. Please verify."
                                           : "ERROR: Invalid args for vertex normal. Please verify."},
                         "");
                }
                (c == V ? verts : norms).push_back(p);
                break;
            }
            case VT: {
                std::pair<float, float> t;
                try {
                    t = {stof_or(a, 0), stof_or(a, 1)};
                } catch (const std::exception &e) {
                    fail({e.what(), "ERROR: Invalid args for texture coordinate. Please verify."}, "");
                }
                uvs.push_back(t);
                break;
            }
            case FACE: face_cmd(a); break;
        }
    }
};

void copy_msg(char *msg, int msglen, const std::string &s) {
    if (!msg || msglen <= 0) return;
    size_t n = std::min((size_t)msglen - 1, s.size());
    memcpy(msg, s.data(), n);
    msg[n] = 0;
}

// Host threads for the writer: the process's CPU affinity, at most
// OMP_NUM_THREADS when set (a GPU box's lease share) and 64.
int host_threads() {
    int n = 1;
    cpu_set_t cs;
    if (sched_getaffinity(0, sizeof cs, &cs) == 0) n = CPU_COUNT(&cs);
    if (const char *e = std::getenv("OMP_NUM_THREADS")) {
        const int k = std::atoi(e);
        if (k > 0) n = std::min(n, k);
    }
    return std::max(1, std::min(n, 64));
}

// main.cpp:760 on x86-64 (cvttss2si): NaN and out-of-range -> INT_MIN
inline long long quantize1(float c) {
    float x = (c - 0.0f) * (255.0f - 0.0f) / (1.0f - 0.0f) + 0.0f;
    if (x >= -2147483648.0f && x < 2147483648.0f) return (long long)(int)x;
    return (long long)INT_MIN;
}

}  // namespace

// An open P3 file being written row block by row block (rth_ppm_open)
struct rth_ppm_stream {
    int fd;
    int W, H, rows;                    // rows written so far
    size_t off;                        // file offset of the next row
    int threads;
    bool good;
};

extern "C" {

int rth_parse_file(const char *path, rth_scene **out, char *msg, int msglen) {
    *out = nullptr;
    std::ifstream in(path);
    if (!in.is_open()) {
        copy_msg(msg, msglen,
                 std::string("ERROR: Issue reading input file '") + path + "'. Please verify path.");
        return 1;
    }
    auto *S = new rth_scene();
    S->desc.epsilon = 1.0e-3f;  // main.cpp:101
    S->desc.depth = 4;          // main.cpp:100
    S->desc.eta_bkg = 0.0f;     // main.cpp:751 default-insert
    Parser P(*S);
    std::string text;
    try {
        while (std::getline(in, text)) P.line(text);
    } catch (Fatal &e) {
        std::string s;
        for (auto &l : e.f.cerr_lines) s += l + "\n";
        s += e.f.what;
        copy_msg(msg, msglen, s);
        delete S;
        return e.f.out_of_range ? -2 : -1;
    }
    static const char *need[] = {"imsize", "eye", "viewdir", "updir", "hfov", "bkgcolor"};
    for (int i = 0; i < 6; i++) {
        if (!P.seen[i]) {
            copy_msg(msg, msglen, std::string("Error: Requires command '") + need[i] + "'");
            delete S;
            return 1;
        }
    }
    S->finalize();
    *out = S;
    return 0;
}

void rth_free(rth_scene *s) { delete s; }
const rt_scene_desc *rth_desc(const rth_scene *s) { return &s->desc; }
void rth_set_depth(rth_scene *s, int depth) { s->desc.depth = depth; }
void rth_set_imsize(rth_scene *s, int w, int h) {
    s->width = w;
    s->height = h;
}
int rth_width(const rth_scene *s) { return s->width; }
int rth_height(const rth_scene *s) { return s->height; }

// main.cpp:607 (normalised view vectors) + :677-710
int rth_camera(const rth_scene *s, int W, int H, rt_camera *cam) {
    if (!s || !cam || W < 1 || H < 1) return RT_E_INVALID;
    const double kPi = 3.14159265358979323846;  // src/config.h:11
    const double kD = 5.0;                      // src/config.h:8
    F3 n = unit(s->viewdir), up = unit(s->updir);
    float res_w = (float)W, res_h = (float)H;
    F3 u = unit(cross(n, up));
    F3 v = cross(u, n);
    float aspect = res_w / res_h;
    float w = (float)(2.0f * kD * std::tan((0.5 * (double)s->fov) * kPi / 180.0f));
    float h = w / aspect;
    F3 c = add(s->eye, scale(n, (float)kD));
    F3 half_u = scale(u, w / 2.0f), half_v = scale(v, h / 2.0f);
    F3 ul = add(sub(c, half_u), half_v);
    F3 ur = add(add(c, half_u), half_v);
    F3 ll = sub(sub(c, half_u), half_v);
    F3 dh = divs(sub(ur, ul), res_w - 1.0f);
    F3 dv = divs(sub(ll, ul), res_h - 1.0f);
    F3 *dst[4] = {(F3 *)cam->eye, (F3 *)cam->ul, (F3 *)cam->dh, (F3 *)cam->dv};
    F3 src[4] = {s->eye, ul, dh, dv};
    for (int i = 0; i < 4; i++) memcpy(dst[i], &src[i], sizeof(F3));
    return RT_OK;
}

void rth_quantize(const float *rgb, long long n, long long *out) {
    for (long long i = 0; i < n; i++) out[i] = quantize1(rgb[i]);
}

// main.cpp:628-648: "r g b \n" per pixel, each value the std::to_string of
// the quantised size_t.  Host threads take chunks of pixels in order, format
// each into a buffer of their own and write it with pwrite at its place in
// the file: a chunk's offset is known once every earlier chunk has its length
// (published in order, under a lock), so formatting and writing run on every
// thread at once.  Values 0..255 (nearly all) come from a table; the rest
// (background > 1, NaN's INT_MIN, negative values as size_t) through
// std::to_chars.
int rth_write_ppm(const char *path, const float *rgb, int W, int H, int threads) {
    rth_ppm_stream *st = nullptr;
    if (rth_ppm_open(path, W, H, threads, &st) != 0) return -1;
    const int rc = rth_ppm_write_rows(st, rgb, H);
    return (rth_ppm_close(st) == 0 && rc == 0) ? 0 : -1;
}

int rth_ppm_open(const char *path, int W, int H, int threads, rth_ppm_stream **out) {
    if (!path || !out || W < 0 || H < 0) return -1;
    *out = nullptr;
    const int fd = ::open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) return -1;
    char head[64];
    const int hn = std::snprintf(head, sizeof head, "P3 \n%d %d \n255 \n", W, H);
    auto *st = new rth_ppm_stream;
    st->fd = fd;
    st->W = W;
    st->H = H;
    st->rows = 0;
    st->off = (size_t)hn;
    st->threads = threads <= 0 ? host_threads() : threads;
    st->good = ::pwrite(fd, head, (size_t)hn, 0) == (ssize_t)hn;
    *out = st;
    return st->good ? 0 : -1;
}

}  // extern "C"

namespace {

// The next nrows image rows: every host thread takes chunks of 32 768
// pixels in order, formats them (a table for 0..255, std::to_chars for the
// rest) and pwrites them at their offset, known once every earlier chunk has
// its length; no thread waits for a single writer.  value(i) is the i-th
// value's size_t (rth_quantize of a float, or a byte the device quantised).
template <class Value>
int ppm_write_rows(rth_ppm_stream *st, int nrows, Value value) {
    static const struct Lut {
        char s[256][4];
        unsigned char n[256];
        Lut() {
            for (int v = 0; v < 256; v++) {
                char *o = std::to_chars(s[v], s[v] + 3, v).ptr;
                n[v] = (unsigned char)(o - s[v] + 1);
                *o = ' ';
            }
        }
    } lut;
    const size_t npx = (size_t)st->W * (size_t)nrows;
    const size_t chunk = 1 << 15;
    const size_t nchunks = (npx + chunk - 1) / chunk;
    std::vector<size_t> len(nchunks, SIZE_MAX);       // formatted length of each chunk
    std::mutex mu;
    std::condition_variable cv;
    size_t next = 0;                                  // next chunk to take
    size_t known = 0;                                 // chunks [0, known) have their offsets
    size_t end_off = st->off;                         // file offset after chunk known - 1
    std::vector<size_t> off(nchunks, 0);
    auto format = [&](size_t c, std::string &o) {
        const size_t p0 = c * chunk, p1 = std::min(npx, p0 + chunk);
        o.resize((p1 - p0) * (3 * 21 + 1));
        char *q = o.data();
        for (size_t p = p0; p < p1; p++) {
            for (int k = 0; k < 3; k++) {
                const unsigned long long v = value(p * 3 + k);
                if (v < 256) {
                    std::memcpy(q, lut.s[v], 4);
                    q += lut.n[v];
                } else {
                    q = std::to_chars(q, q + 20, v).ptr;
                    *q++ = ' ';
                }
            }
            *q++ = '\n';
        }
        o.resize((size_t)(q - o.data()));
    };
    std::atomic<bool> good{true};
    const int fd = st->fd;
    auto worker = [&] {
        std::string buf;
        for (;;) {
            size_t c;
            {
                std::lock_guard<std::mutex> lk(mu);
                if (next >= nchunks) return;
                c = next++;
            }
            format(c, buf);
            size_t at;
            {
                std::unique_lock<std::mutex> lk(mu);
                len[c] = buf.size();
                while (known < nchunks && len[known] != SIZE_MAX) {
                    off[known] = end_off;
                    end_off += len[known];
                    known++;
                }
                cv.notify_all();
                cv.wait(lk, [&] { return known > c; });
                at = off[c];
            }
            size_t done = 0;
            while (done < buf.size()) {
                const ssize_t w = ::pwrite(fd, buf.data() + done, buf.size() - done, (off_t)(at + done));
                if (w <= 0) {
                    good = false;
                    break;
                }
                done += (size_t)w;
            }
        }
    };
    std::vector<std::thread> pool;
    const int nt = (int)std::min<size_t>((size_t)st->threads, std::max<size_t>(1, nchunks));
    for (int t = 1; t < nt; t++) pool.emplace_back(worker);
    worker();
    for (auto &th : pool) th.join();
    st->off = end_off;
    st->rows += nrows;
    if (!good) st->good = false;
    return good ? 0 : -1;
}

}  // namespace

extern "C" {

int rth_ppm_write_rows(rth_ppm_stream *st, const float *rgb, int nrows) {
    if (!st || (!rgb && nrows > 0) || nrows < 0 || st->rows + nrows > st->H) return -1;
    return ppm_write_rows(st, nrows, [rgb](size_t i) { return (unsigned long long)quantize1(rgb[i]); });
}

int rth_ppm_write_rows_u8(rth_ppm_stream *st, const unsigned char *v, int nrows) {
    if (!st || (!v && nrows > 0) || nrows < 0 || st->rows + nrows > st->H) return -1;
    return ppm_write_rows(st, nrows, [v](size_t i) { return (unsigned long long)v[i]; });
}

int rth_write_ppm_u8(const char *path, const unsigned char *v, int W, int H, int threads) {
    rth_ppm_stream *st = nullptr;
    if (rth_ppm_open(path, W, H, threads, &st) != 0) return -1;
    const int rc = rth_ppm_write_rows_u8(st, v, H);
    return (rth_ppm_close(st) == 0 && rc == 0) ? 0 : -1;
}

int rth_ppm_close(rth_ppm_stream *st) {
    if (!st) return -1;
    bool good = st->good && st->rows == st->H;
    if (::close(st->fd) != 0) good = false;
    delete st;
    return good ? 0 : -1;
}

int rth_output_path(const char *scene_path, char *out, int outlen) {
    std::string s(scene_path);
    size_t dot = s.rfind('.');
    if (dot != std::string::npos) s.resize(dot);
    s += ".ppm";
    if ((int)s.size() + 1 > outlen) return -1;
    memcpy(out, s.c_str(), s.size() + 1);
    return 0;
}

}  // extern "C"

extern "C" int rth_row_set(int H, int world, int rank, int block, int *y0, int *step, int *nrows, int *rows_per) {
    if (H < 1 || world < 1 || rank < 0 || rank >= world || block < 1 || !y0 || !step || !nrows || !rows_per)
        return -1;
    const int nblocks = (H + block - 1) / block;
    auto rows_of = [&](int r) {
        int n = 0;
        for (int b = r; b < nblocks; b += world) n += std::min(block, H - b * block);
        return n;
    };
    *y0 = rank * block;
    *step = block * world;
    *nrows = rows_of(rank);
    int mx = 1;
    for (int r = 0; r < world; r++) mx = std::max(mx, rows_of(r));
    *rows_per = mx;
    return 0;
}

// rt_kernels.hip -- MI355X (gfx950) ray-trace kernel + the C ABI of rt_hip.h.
//
// Replaces the reference's hot path: the pixel loop main.cpp:718-764, TraceRay
// main.cpp:1215-1407 and ShadeRay main.cpp:783-1207 (called recursively).
//
// Execution model:
//  * persistent workgroups; every lane owns one pixel at a time and walks
//    that pixel's ShadeRay tree as an explicit state machine (frames in
//    scratch), one TraceRay-equivalent scan per loop iteration;
//  * all active lanes of a wave scan the primitive list together (uniform
//    loop, primitive data broadcast from LDS or scalar-loaded), whatever kind
//    of ray each lane carries (primary / shadow / refraction / reflection);
//  * a lane that finishes its pixel is refilled in the same iteration: the
//    wave ballots its idle lanes, one lane takes a block of pixel indices with
//    a single atomicAdd and each idle lane picks its own by a prefix count of
//    the ballot (mbcnt) -- wave-level ballot/prefix compaction of the work;
//  * scene arrays are staged once per workgroup into LDS when they fit,
//    otherwise read through the scalar cache;
//  * framebuffer: 12 B/pixel fp32 RGB stores (pre-quantisation colour).
//
// Numerics follow the reference operation by operation (built with
// -ffp-contract=off, correctly rounded div/sqrt, std::clamp-style compares,
// the reference's double-precision intermediates where they change the
// result).  Two documented relaxations: the sphere C and discriminant use one
// fmaf each instead of the reference's double expression (identical except for
// a double-rounding tie, ~2^-29 per test), and libm (glibc) vs ocml
// powf/acosf/asinf/acos/atan2 differences.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rt_bvh.h"
#include "rt_hip.h"

namespace rt {

// ---------------------------------------------------------------------------
// Device-side geometry/colour semantics of src/definitions.h
// ---------------------------------------------------------------------------
struct V3 {
    float x, y, z;
};
struct C3 {
    float r, g, b;
};

__host__ __device__ __forceinline__ V3 vadd(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__host__ __device__ __forceinline__ V3 vsub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__host__ __device__ __forceinline__ V3 vmul(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__host__ __device__ __forceinline__ V3 vdiv(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
__host__ __device__ __forceinline__ float vdot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__host__ __device__ __forceinline__ V3 vnorm(V3 a) { return vdiv(a, sqrtf(vdot(a, a))); }
__host__ __device__ __forceinline__ V3 vcross(V3 a, V3 b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
// std::clamp(v, 0, 1): NaN passes through (not fminf/fmaxf)
__device__ __forceinline__ float clamp01(float v) { return (v < 0.0f) ? 0.0f : ((1.0f < v) ? 1.0f : v); }
__device__ __forceinline__ float clampr(float v, float lo, float hi) { return (v < lo) ? lo : ((hi < v) ? hi : v); }
__device__ __forceinline__ C3 cmulc(C3 a, C3 b) { return {clamp01(b.r * a.r), clamp01(b.g * a.g), clamp01(b.b * a.b)}; }
__device__ __forceinline__ C3 cmulf(C3 a, float f) { return {clamp01(f * a.r), clamp01(f * a.g), clamp01(f * a.b)}; }
__device__ __forceinline__ C3 cadd(C3 a, C3 b) { return {clamp01(b.r + a.r), clamp01(b.g + a.g), clamp01(b.b + a.b)}; }
__device__ __forceinline__ float max0(float x) { return (0.0f < x) ? x : 0.0f; }

constexpr double kPi = 3.14159265358979323846;        // src/config.h:11
constexpr double kRightAngle = 90.0 * kPi / 180.0;    // main.cpp:964
constexpr float kFltMax = 3.40282347e+38f;            // std::numeric_limits<float>::max()

enum { ENTERING = 0, EXITING = 1 };

// Read-only scene data seen through the constant address space: the loads
// are wave-uniform and invariant, so they become scalar (s_load) reads into
// SGPRs through the scalar cache instead of 64 identical per-lane loads.
#define RT_CONST __attribute__((address_space(4)))
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 f4(f4v v) { return make_float4(v.x, v.y, v.z, v.w); }
template <typename T>
__device__ __forceinline__ const RT_CONST T *cst(const T *p) {
    return (const RT_CONST T *)p;
}
// uniform float4 read via the scalar unit
__device__ __forceinline__ float4 sld4(const float4 *p, int i) {
    f4v v = cst((const f4v *)p)[i];
    return make_float4(v.x, v.y, v.z, v.w);
}


// ---------------------------------------------------------------------------
// Device scene layout (built by rt_scene_create)
// ---------------------------------------------------------------------------
// Faces (object index 0..nf-1), 5 x float4 each, per-face invariants hoisted
// exactly as TraceRay computes them (main.cpp:1280-1301, :1361-1366):
//   [0] v0.xyz, D = -n.v0     [1] n.xyz, det = d11*d22 - d12*d12
//   [2] e1.xyz, d11           [3] e2.xyz, d22        [4] d12, -, -, -
// Spheres (object index nf..nf+ns-1): float4 center.xyz, radius.
struct ObjK {                 // per object, shading data
    float dif[3], ka;
    float spc[3], kd;
    float ks, n, opacity, eta;
    int tex;                  // texture index or -1
    int is_sphere;
    int pad[2];
};
struct FaceShadeK {           // per face, shading-only data
    float vn[3][3];           // vertex_normal[k].norm() (main.cpp:1382-1384)
    float vt[3][2];           // clamp<float>(texture_coords, 0, 1) (main.cpp:835-841)
    int smooth;
    int pad[2];
};
struct LightK {
    float xyz[3], w;          // position or direction, w
    float col[3], pad0;
    float L[3], pad1;         // directional: light.direction.norm() * -1 (main.cpp:887)
    float sdir[3], pad2;      // directional: light.direction * -1 (main.cpp:895, unnormalised)
};
static_assert(sizeof(LightK) % sizeof(float4) == 0, "lights are staged in LDS as float4s");
struct TexK {
    int w, h;
    long long off;                       // first byte in Params::texels
};
// directional light: its shadow-region tree over the spheres (rt host:
// dir_trees) -- root node in Params::bvh (-1: no sphere can shadow) and the
// rotation R (rows) into the frame the tree's boxes were built in
struct DirK {
    float R[9];
    int root;
    float cone_k;                        // max(0, |d|^2 - 1), rounded up
    float cone_h;                        // |d| < 1: height bound of the shadow region, else +inf
};

struct Params {
    const float4 *__restrict__ fscan;
    const float4 *__restrict__ sscan;
    const float *__restrict__ ofac;      // (float)(1.0 - opacity) per object (main.cpp:909)
    const ObjK *__restrict__ objs;
    const FaceShadeK *__restrict__ fsh;
    const LightK *__restrict__ lights;
    const unsigned char *__restrict__ texels;   // all textures: RGB bytes, row-major
    const TexK *__restrict__ texs;
    float *__restrict__ out;
    unsigned int *__restrict__ work;     // pixel work counter
    unsigned long long *__restrict__ stats;
    int nf, ns, nl;
    float bkg[3];
    float eta_bkg, eps;
    int depth;
    float eye[3], ul[3], dh[3], dv[3];
    int W, y0, rows;                     // render `rows` rows of a W-wide image: local row r is
    int rblock, rstep;                   // image row y0 + (r / rblock) * rstep + r % rblock
    unsigned int total;                  // W * rows
    // BVH (MODE_BVH): 8 float4 per 4-wide node (rt_bvh.h Node4), leaf-ordered object keys
    const float4 *__restrict__ bvh;
    const float4 *__restrict__ leafrec;  // leaf-ordered primitive records (rt_bvh.h leaf_records)
    int dir_bf;                          // directional lights in a scene with spheres: 0 none,
                                         // 1 brute-force scan, 2 faces by the BVH + shadow-region trees
    const DirK *__restrict__ dirk;       // per light (dir_bf == 2)
    int shadow_early_out;                // no NaN shadow factor: an opaque hit ends a shadow ray
    int ovf_stride;                      // BVH: stack spill entries per lane (deepest tree, kSpill multiple)
    int lights_lds;                      // the lights' copy in LDS: float4 offset in rt_lds
    int stack_cap;                       // BVH: stack entries kept in LDS (<= kLdsStack)
    unsigned chunk;                      // work items a wave takes from the counter at a time (0: its idle lanes' count)
    unsigned refill_min;                 // refill only when at least this many lanes are idle (or all are)
    unsigned gate_x;                     // hold reflection/refraction searches until this many lanes have one
    void *__restrict__ frames;           // grid x kBlock x MAXF cold ShadeRay frames
    int *__restrict__ ovf;               // grid x kBlock x ovf_stride spilled BVH stack entries
};

enum Mode { MODE_SCAN = 0, MODE_SCAN_LDS = 1, MODE_BVH = 2 };
#ifndef RT_PROF
#define RT_PROF 0                        // 1: per-wave cycle/occupancy counters in stats[9..15]
#endif
#ifndef RT_MIN_WAVES
#define RT_MIN_WAVES 5                   // waves per SIMD the register budget must allow (A/B: 5 best)
#endif
// Largest worst-case BVH stack a tree may need (entries per lane; the spill
// area is sized per tree, Params::ovf_stride).  Refill tags kRefill + b stay
// far below the leaf links (> INT_MIN + 256) for b <= kStackMax / kSpill.
constexpr int kStackMax = 1024;
// BVH traversal stack entries per lane in LDS (entry 0: the sentinel); a
// deeper stack spills its oldest kSpill entries to device memory (rare)
constexpr int kLdsStack = 16;            // most entries the LDS share may hold (option lds_stack)
constexpr int kLdsStackDefault = 14;     // 16 (32 KB per block with the shading state): 5 blocks per CU
                                         // on paper, -8.6 % measured; 14: 270 spills per C3 frame
constexpr int kSpill = 8;
static_assert(kStackMax % kSpill == 0 && kStackMax / kSpill < 200 && kLdsStack - 3 > kSpill, "stack spill blocks");
constexpr int kBlock = 256;
constexpr unsigned kGateX = 32;          // option gate_x (A/B: 24..48 within 0.2 % on C3 and C5)

// ---------------------------------------------------------------------------
// One lane's ray query (a TraceRay call + the consumer loop that follows it)
// ---------------------------------------------------------------------------
//  closest : smallest t with tmin < t < running min, ties -> first in order
//            (main.cpp:732-742, :992-1011, :1113-1124); skipchk applies the
//            SKIP_TRANS rule (main.cpp:1000-1002) against object `back`
//  shadow  : every intersection of every object != self with tmin < t (and
//            t < tmax unless unbounded) multiplies mask by (1 - opacity)
//            (main.cpp:898-912, :930-949)
struct Query {
    V3 o, d;
    float tmin, tmax;
    int self, back, win;
    bool closest, unb, skipchk, skipped;
    bool bf;                              // BVH mode: this query needs the brute-force scan
    C3 mask;
};

constexpr float kInf = __builtin_huge_valf();

__device__ __forceinline__ void offer(Query &q, float t, int obj, const float *__restrict__ ofac) {
    bool in = (t > q.tmin) & ((t < q.tmax) | q.unb) & (obj != q.self);
    if (in) {
        if (q.closest) {
            if (q.skipchk & (obj != q.back)) {
                q.skipped = true;
                q.tmin = kInf;               // 'goto SKIP_TRANS': the scan is over
            } else {
                q.tmax = t;
                q.win = obj;
            }
        } else {
            float f = cst(ofac)[obj];
            q.mask = cmulf(q.mask, f);
            // an opaque occluder zeroes the mask for good: any-hit termination
            if ((q.mask.r == 0.0f) & (q.mask.g == 0.0f) & (q.mask.b == 0.0f)) q.tmin = kInf;
        }
    }
}

// TraceRay's face test (main.cpp:1296-1378); returns t if the ray hits the
// triangle's open interior.
__device__ __forceinline__ bool face_test(float4 f0, float4 f1, float4 f2, float4 f3, float4 f4, V3 o, V3 d,
                                          float &t, float &a, float &b, float &g) {
    V3 n = {f1.x, f1.y, f1.z};
    float dem = vdot(n, d);
    // branch-free: dem == 0 (ray parallel to the plane) still means no hit,
    // but every load of the face is needed up front (one batch per test)
    V3 v0 = {f0.x, f0.y, f0.z};
    t = -(vdot(n, o) + f0.w) / dem;
    V3 ep = vsub(vadd(o, vmul(d, t)), v0);
    V3 e1 = {f2.x, f2.y, f2.z}, e2 = {f3.x, f3.y, f3.z};
    float d1p = vdot(e1, ep), d2p = vdot(e2, ep);
    float d11 = f2.w, d22 = f3.w, d12 = f4.x, det = f1.w;
    b = (d22 * d1p - d12 * d2p) / det;
    g = (d11 * d2p - d12 * d1p) / det;
    a = 1.0f - (b + g);
    return (dem != 0.0f) & (0.0f < a) & (a < 1.0f) & (0.0f < b) & (b < 1.0f) & (0.0f < g) & (g < 1.0f);
}

// TraceRay's sphere test (main.cpp:1225-1258): both roots, A = 1 assumed.
__device__ __forceinline__ bool sphere_test(float4 s, V3 o, V3 d, float &t1, float &t2) {
    V3 dir = {o.x - s.x, o.y - s.y, o.z - s.z};
    float B = 2.0f * vdot(d, dir);
    float C = fmaf(-s.w, s.w, vdot(dir, dir));      // (float)((double)|dir|^2 - (double)r*r)
    float det = fmaf(B, B, -4.0f * C);              // (float)((double)B*B - 4.0*C)
    if (__builtin_signbitf(det)) return false;
    float sq = sqrtf(det);
    t1 = (-B + sq) * 0.5f;
    t2 = (-B - sq) * 0.5f;
    return true;
}

// The scan every active lane of the wave runs together.  SRC_LDS: primitive
// arrays were staged into LDS (lds_f, lds_s); otherwise scalar loads.
template <bool SRC_LDS>
__device__ __forceinline__ void scan(Query &q, const Params &p, const float4 *lds_f, const float4 *lds_s,
                                     bool part, unsigned &ft, unsigned &st) {
    if (!part) return;
    ft += (unsigned)p.nf;
    st += (unsigned)p.ns;
    for (int i = 0; i < p.nf; i++) {
        float4 f0, f1, f2, f3, f4;
        if (SRC_LDS) {
            f0 = lds_f[5 * i + 0], f1 = lds_f[5 * i + 1], f2 = lds_f[5 * i + 2], f3 = lds_f[5 * i + 3];
            f4 = lds_f[5 * i + 4];
        } else {
            f0 = sld4(p.fscan, 5 * i + 0), f1 = sld4(p.fscan, 5 * i + 1), f2 = sld4(p.fscan, 5 * i + 2);
            f3 = sld4(p.fscan, 5 * i + 3), f4 = sld4(p.fscan, 5 * i + 4);
        }
        if (f1.w == 0.0f) continue;                 // det == 0: never intersects (main.cpp:1367)
        if (q.tmin < kInf) {
            float t, a, b, g;
            if (face_test(f0, f1, f2, f3, f4, q.o, q.d, t, a, b, g)) offer(q, t, i, p.ofac);
        }
    }
    for (int i = 0; i < p.ns; i++) {
        float4 s = SRC_LDS ? lds_s[i] : sld4(p.sscan, i);
        if (q.tmin < kInf) {
            float t1, t2;
            if (sphere_test(s, q.o, q.d, t1, t2)) {
                offer(q, t1, p.nf + i, p.ofac);
                offer(q, t2, p.nf + i, p.ofac);
            }
        }
    }
}


// ---------------------------------------------------------------------------
// BVH traversal (MODE_BVH).  Candidates come from the BVH in any order; the
// reference's sequential semantics are restored:
//   closest : keep the smallest t, ties -> smallest object index (= the
//             reference's first-in-order winner under its strict '<');
//   shadow  : every valid hit multiplies the mask.  All factors and the mask
//             lie in [0,1] (the clamps never fire), so the product in
//             traversal order differs from the reference's object order by
//             rounding only (<= 1 ulp per factor); an opaque
//             hit zeroes the mask whatever the order (early exit when no
//             factor is NaN).
// Queries the BVH cannot reproduce (SKIP_TRANS checks, directional shadow
// rays against spheres) set q.bf and are re-run by the brute-force scan.
// ---------------------------------------------------------------------------
// Per-lane counters kept small (VGPR pressure): ray kinds are counted per
// wave with ballots in the main loop (scalar registers); only the rare events
// and the executed-test counts stay per lane.
struct Counters {
    unsigned skip, ub;
    unsigned boxes, ftests, stests;             // ray-box, ray-face, ray-sphere tests executed
#if RT_PROF
    unsigned trips;                             // traversal loop iterations of this lane
    unsigned trips_kind[3];                     // ... of primary / shadow / refraction + reflection queries
#endif
#if RT_PROF >= 2
    unsigned long long t_fetch, t_trip;         // inner-node trips: cycles to node data, whole trip
#endif
};
enum RayKind { RK_NONE = 0, RK_SHADOW = 1, RK_REFR = 2, RK_REFL = 3, RK_PRIMARY = 4 };

// Nearest root of object `obj` alone along q with tmin < t < FLT_MAX
// (kFltMax: none) -- the minimum the reference's in-order scan holds once it
// has passed that object (main.cpp:997, :1004).
__device__ __forceinline__ float own_nearest(const Query &q, const Params &p, int obj, Counters &cnt) {
    float tb = kFltMax;
    if (obj < p.nf) {
        const float4 *F = p.fscan + 5 * obj;
        float t, a, b, g;
        cnt.ftests++;
        if (face_test(F[0], F[1], F[2], F[3], F[4], q.o, q.d, t, a, b, g) & (F[1].w != 0.0f) & (t > q.tmin) &
            (t < kFltMax))
            tb = t;
    } else {
        float t1, t2;
        cnt.stests++;
        if (sphere_test(p.sscan[obj - p.nf], q.o, q.d, t1, t2)) {
            if ((t1 > q.tmin) & (t1 < tb)) tb = t1;
            if ((t2 > q.tmin) & (t2 < tb)) tb = t2;
        }
    }
    return tb;
}


constexpr int kNodeF4 = 5;                       // float4 per 4-wide node (rt_bvh.h Node4H)
static_assert(kNodeF4 * 16 == sizeof(rtbvh::Node4H), "node layout");
typedef _Float16 h2v __attribute__((ext_vector_type(2)));   // two binary16 plane offsets
// while-while traversal: stop descending when at most this many lanes still
// look for a leaf (A/B, C3 Mrays/s: 0 -> 5912, 1 -> 5960, 2 -> 5957, 3 -> 5954,
// 6 -> 5924, 12 -> 5849; with one leaf per round: 0 -> 5885, 2 -> 6021,
// 5 -> 6031; profiles/r02/ab_leaf_*.txt)
constexpr unsigned kLeafWait = 2;
// The depth > 4 instantiation (MAXF 9/17: C5, depth 8, whose 100 000-sphere
// tree is 12 levels deep) keeps descending until 12 lanes lack a leaf: C5
// +2.2 % (2: C3 best, 8 there -1.2 %; a run-time threshold cost C3 1 %,
// profiles/r02/ab_leafwait_r2final.txt)
constexpr unsigned leaf_wait_for(int maxf) { return maxf > 5 ? 12u : kLeafWait; }
constexpr int kRefill = rtbvh::kEmpty + 1;       // LDS stack sentinel with blocks spilled (+ count - 1)
constexpr int kNStats = 40;                      // device counter slots (rt_scene_debug_counters)

__device__ __forceinline__ float safe_rcp(float x) {
    return x == 0.0f ? __builtin_copysignf(1e30f, x) : 1.0f / x;
}

// One leaf's primitives against q: faces (5 words each) then spheres (2 words),
// rt_bvh.h leaf_records.  Closest: running (best, win); shadow: every valid
// hit multiplies the mask (an opaque one ends the ray).
__device__ __forceinline__ void leaf_visit(Query &q, const Params &p, int link, Counters &cnt, float &best, int &win,
                                           bool &opaque, bool faces_only) {
    int v = -link - 1;
    const float4 *R = p.leafrec + (v >> 8);
    int nfc = (v >> 4) & 15, count = v & 15;
    if (faces_only) count = nfc;             // the leaf's faces come first
    for (int k = 0; k < count; k++) {
        float t[2];
        int nt = 0;
        int key;
        float fac;
        // one batch of loads for either kind; the face words 2..4 only when
        // some lane of the wave is at a face (a sphere then reads 3 words past
        // its record; the stream is padded for the last one) -- the vector
        // memory path (TA), not the ALU, is the busier one here
        const f4v *RV = reinterpret_cast<const f4v *>(R);
        f4v w0 = RV[0], w1 = RV[1], w2 = {0.0f, 0.0f, 0.0f, 0.0f}, w3 = w2, w4 = w2;
        if (__ballot(k < nfc)) w2 = RV[2], w3 = RV[3], w4 = RV[4];
        asm volatile("" ::"v"(w0), "v"(w1), "v"(w2), "v"(w3), "v"(w4));
        float4 f0 = make_float4(w0.x, w0.y, w0.z, w0.w), f1 = make_float4(w1.x, w1.y, w1.z, w1.w);
        float4 f2 = make_float4(w2.x, w2.y, w2.z, w2.w), f3 = make_float4(w3.x, w3.y, w3.z, w3.w);
        float4 f4 = make_float4(w4.x, w4.y, w4.z, w4.w);
        if (k < nfc) {
            R += 5;
            key = __float_as_int(f4.y);
            fac = f4.z;
            float a, bb, g;
            cnt.ftests++;
            if (face_test(f0, f1, f2, f3, f4, q.o, q.d, t[0], a, bb, g) & (f1.w != 0.0f)) nt = 1;
        } else {
            R += 2;
            key = __float_as_int(f1.x);
            fac = f1.y;
            cnt.stests++;
            if (sphere_test(f0, q.o, q.d, t[0], t[1])) nt = 2;
        }
        for (int r = 0; r < nt; r++) {
            float tt = t[r];
            if (q.closest) {
                bool valid = (tt > q.tmin) & (tt < kFltMax);
                bool better = (tt < best) | ((tt == best) & (key < win));
                if (valid & better) {
                    best = tt;
                    win = key;
                }
            } else if (q.skipchk) {
                // SKIP_TRANS (main.cpp:997-1002): a candidate of another
                // object that the reference's in-order scan would see as a
                // new minimum -- any one before the stack top's object in
                // order, or nearer than the stack top's own nearest root
                // (q.tmax) -- aborts the refraction
                if ((key != q.back) & (tt > q.tmin) & (tt < kFltMax) & ((key < q.back) | (tt < q.tmax))) opaque = true;
            } else if ((key != q.self) & (tt > q.tmin) & ((tt < q.tmax) | q.unb)) {
                if (fac == 0.0f && p.shadow_early_out) {
                    opaque = true;
                } else {
                    q.mask = cmulf(q.mask, fac);
                }
            }
        }
    }
}

// The six plane distances of a 4-wide node's children (rt_bvh.h Node4H):
// plane a of child i at origin_a + h * 2^e_a (h binary16), i.e.
// t = h * (2^e_a / d_a) + (origin_a - o_a) / d_a = fma(h, A_a, B_a) -- one
// v_fma_mix_f32 per plane (h converted inside the fma, exactly); the rounding
// (~ulp(D) in distance) is far inside the primitive padding.  (i, o) =
// (1 / d, o / d) per axis, or (1, o) for a point query: then the planes are
// the children's offsets from o.  Near / far plane per axis by the ray's
// octant: t(h) is monotonic in h with the sign of A (= the sign of 1/d), so
// min(t(lo), t(hi)) is t(near) exactly -- 4 min/max per child, not 10.
struct ChildPlanes {
    float tn[3][4], tf[3][4];                   // [axis][child]: near / far plane
};
__device__ __forceinline__ ChildPlanes child_planes(float4 w0, float4 w1, float4 w2, float4 w3, float ix, float iy,
                                                    float iz, float ox, float oy, float oz, bool neg_x, bool neg_y,
                                                    bool neg_z) {
    // 2^e * (1/d): exact power-of-two scaling (one v_bfe_i32 + v_ldexp per
    // axis; signed exponents in bytes 0..2 of w0.w), finite by the caps
    const int ex = __float_as_int(w0.w);
    const float A[3] = {__builtin_amdgcn_ldexpf(ix, __builtin_amdgcn_sbfe(ex, 0, 8)),
                        __builtin_amdgcn_ldexpf(iy, __builtin_amdgcn_sbfe(ex, 8, 8)),
                        __builtin_amdgcn_ldexpf(iz, __builtin_amdgcn_sbfe(ex, 16, 8))};
    const float B[3] = {fmaf(w0.x, ix, -ox), fmaf(w0.y, iy, -oy), fmaf(w0.z, iz, -oz)};
    // lower / upper bounds per axis, two children per word
    const unsigned lo[3][2] = {{__float_as_uint(w1.x), __float_as_uint(w1.y)},
                               {__float_as_uint(w1.z), __float_as_uint(w1.w)},
                               {__float_as_uint(w2.x), __float_as_uint(w2.y)}};
    const unsigned hi[3][2] = {{__float_as_uint(w2.z), __float_as_uint(w2.w)},
                               {__float_as_uint(w3.x), __float_as_uint(w3.y)},
                               {__float_as_uint(w3.z), __float_as_uint(w3.w)}};
    const bool neg[3] = {neg_x, neg_y, neg_z};
    ChildPlanes cp;
#pragma unroll
    for (int a = 0; a < 3; a++) {
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const h2v n = __builtin_bit_cast(h2v, neg[a] ? hi[a][j] : lo[a][j]);
            const h2v f = __builtin_bit_cast(h2v, neg[a] ? lo[a][j] : hi[a][j]);
#pragma unroll
            for (int e = 0; e < 2; e++) {
                cp.tn[a][2 * j + e] = fmaf((float)n[e], A[a], B[a]);
                cp.tf[a][2 * j + e] = fmaf((float)f[e], A[a], B[a]);
            }
        }
    }
    return cp;
}

// Entry distance of a ray into child i within [tlo, thi]: +inf for a miss or
// an empty slot (unused slots link to the empty leaf, kEmptyLeaf: entering one
// is harmless, so no link test; their inverted boxes miss anyway).
__device__ __forceinline__ float child_entry(const ChildPlanes &cp, int i, float tlo, float thi) {
    const float tn = fmaxf(fmaxf(cp.tn[0][i], cp.tn[1][i]), fmaxf(cp.tn[2][i], tlo));
    const float tf = fminf(fminf(cp.tf[0][i], cp.tf[1][i]), fminf(cp.tf[2][i], thi));
    return (tn <= tf) ? tn : kInf;
}

// stk: this lane's traversal stack in LDS (entries kBlock apart).
//
// While-while traversal with speculative leaf postponement (Aila & Laine
// 2009): a lane that reaches a leaf parks it and keeps descending inner nodes
// until all but kLeafWait active lanes of the wave hold a leaf; the leaves are
// then visited together.  Node visits stay one dependent fetch each, and the leaf
// code runs with most lanes active instead of in almost every wave trip (+6 %
// over an if-if loop).  The result does not depend on the visiting order.
//
// point: a CONE query instead of a ray (directional shadow rays against
// spheres; dir_tree on the host) -- which boxes of the tree at `root` may
// hold a sphere whose shadow region contains the point po (the origin in
// the light's frame): the same traversal with direction (1, 1, 1), so that
// the plane distances are the child boxes' offsets from po, and a cone test
// per child instead of the slab test; its leaves are still tested with the
// query's own ray (q.o, q.d).
template <bool point, unsigned LEAF_WAIT = kLeafWait>
__device__ void bvh_trace(Query &q, const Params &p, int *stk, Counters &cnt, int root = 0,
                          V3 po = V3{0.0f, 0.0f, 0.0f}, float cone_k = 0.0f, float cone_h = 0.0f) {
    // |1/d| capped at 2^100 (1/0 -> 1e30 as before): the quantised planes'
    // 2^e * (1/d) then never overflows (the builder keeps e <= kQExpMax = 27),
    // and the cap is conservative: an axis with |d| < 2^-100 moves the ray by
    // less than 2^-100 D along it, far inside the 2^-16 D primitive padding
    const float ix = point ? 1.0f : clampr(safe_rcp(q.d.x), -0x1p100f, 0x1p100f);
    const float iy = point ? 1.0f : clampr(safe_rcp(q.d.y), -0x1p100f, 0x1p100f);
    const float iz = point ? 1.0f : clampr(safe_rcp(q.d.z), -0x1p100f, 0x1p100f);
    const bool neg_x = ix < 0.0f, neg_y = iy < 0.0f, neg_z = iz < 0.0f;
    const float ox = point ? po.x : q.o.x * ix, oy = point ? po.y : q.o.y * iy, oz = point ? po.z : q.o.z * iz;
    const float tlo = point ? 0.0f : q.tmin - fabsf(q.tmin) * 0x1p-16f;
    // directional shadow ray in a scene with spheres: this pass tests the
    // faces only, the spheres come in the point pass
    const bool faces_only = !point && !q.closest && !q.skipchk && q.unb && p.dir_bf == 2;
    // A ray with a NaN in its origin or direction meets nothing in the
    // reference (every distance and barycentric comparison is false): "no
    // hit", mask unchanged, no SKIP.  The slab test would enter every box
    // (fmaxf/fminf drop NaN) -- a whole-tree traversal.  (The cone pass
    // rejects such a ray at its root: its cone tests are comparisons.)
    if (!point && (__builtin_isnan(q.o.x) | __builtin_isnan(q.o.y) | __builtin_isnan(q.o.z) |
                   __builtin_isnan(q.d.x) | __builtin_isnan(q.d.y) | __builtin_isnan(q.d.z))) {
        atomicAdd(&p.stats[35], 1ull);
        return;
    }
    float best = q.tmax;                       // closest: running min (kFltMax at start)
    int win = -1;
    bool opaque = false;
    // stack entry 0 holds kEmpty for good (written once per kernel): popping
    // the empty stack yields kEmpty with no bounds test
    int sp = 1;
    int node = rtbvh::kEmpty;                  // >= 0 inner node, < 0 leaf, kEmpty: done
    int leaf = rtbvh::kEmpty;                  // postponed leaf
    auto thi_now = [&] {
        return point ? 0.0f : q.closest ? best + best * 0x1p-16f : (q.unb ? kInf : q.tmax + q.tmax * 0x1p-16f);
    };
    // LDS holds stack entries [0, kLdsStack); entry 0 is kEmpty, or kRefill + b
    // when b blocks of kSpill older entries wait in device memory (ovf).
    auto ovf_lane = [&]() -> int * {
        return p.ovf + ((size_t)blockIdx.x * kBlock + threadIdx.x) * p.ovf_stride;
    };
    auto spill = [&]() {                       // move the oldest kSpill entries out
        const int tag = stk[0];
        const int nb = tag == rtbvh::kEmpty ? 0 : tag - kRefill;
        int *o = ovf_lane() + nb * kSpill;
        for (int i = 0; i < kSpill; i++) o[i] = stk[(1 + i) * kBlock];
        for (int i = kSpill + 1; i < sp; i++) stk[(i - kSpill) * kBlock] = stk[i * kBlock];
        sp -= kSpill;
        stk[0] = kRefill + nb + 1;
        atomicAdd(&p.stats[34], 1ull);
    };
    auto pop = [&]() -> int {
        int n = stk[(--sp) * kBlock];
        if ((unsigned)n - (unsigned)kRefill - 1u < (unsigned)(kStackMax / kSpill)) {   // rare: bring a block back
            const int nb = n - kRefill;
            const int *o = ovf_lane() + (nb - 1) * kSpill;
            for (int i = 0; i < kSpill; i++) stk[(1 + i) * kBlock] = o[i];
            stk[0] = nb > 1 ? n - 1 : rtbvh::kEmpty;
            sp = kSpill;
            n = o[kSpill - 1];                 // the block's newest entry is the top
        }
        return n;
    };
    // One 4-wide node (rt_bvh.h Node4H, child_planes): slab-test the
    // children, push the far hits, continue with the nearest, park the first
    // leaf reached.
    auto visit_q = [&](float4 w0, float4 w1, float4 w2, float4 w3, float4 w4) {
#if RT_PROF
        cnt.trips++;
#endif
        cnt.boxes += 4;
        float thi = thi_now();
        int c0 = __float_as_int(w4.x), c1 = __float_as_int(w4.y), c2 = __float_as_int(w4.z), c3 = __float_as_int(w4.w);
        const ChildPlanes cp = child_planes(w0, w1, w2, w3, ix, iy, iz, ox, oy, oz, neg_x, neg_y, neg_z);
        float k[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            if (!point) {
                k[i] = child_entry(cp, i, tlo, thi);
            } else {
                // shadow cone (see dir_tree): the child's box lies at offsets
                // [tn, tf] from the origin po, z along the light; it may hold
                // a shadowing sphere iff its top is not below po and its
                // lateral distance d satisfies d^2 <= cone_k * top^2 (and,
                // for a bounded region, its bottom is within cone_h)
                const float tnx = cp.tn[0][i], tny = cp.tn[1][i], tnz = cp.tn[2][i];
                const float tfx = cp.tf[0][i], tfy = cp.tf[1][i], tfz = cp.tf[2][i];
                float dx = fmaxf(fmaxf(tnx, -tfx), 0.0f), dy = fmaxf(fmaxf(tny, -tfy), 0.0f);
                float d2 = fmaf(dx, dx, dy * dy);
                bool in = (tfz >= 0.0f) & (d2 <= cone_k * (tfz * tfz)) & (tnz <= cone_h);
                k[i] = in ? d2 : kInf;           // nearest the cone's axis first
            }
        }
        // up to 3 pushes below write stk[sp .. sp + 2]: make room (rare)
        if (sp > p.stack_cap - 3) spill();
        float k0 = k[0], k1 = k[1], k2 = k[2], k3 = k[3];
        // nearest child by a 3-comparator tournament, registers only
#define RT_CSWAP(ka, ca, kb, cb)                 \
    {                                            \
        bool sw = kb < ka;                       \
        float tk = sw ? kb : ka;                 \
        kb = sw ? ka : kb;                       \
        ka = tk;                                 \
        int tc = sw ? cb : ca;                   \
        cb = sw ? ca : cb;                       \
        ca = tc;                                 \
    }
        RT_CSWAP(k0, c0, k1, c1);
        RT_CSWAP(k2, c2, k3, c3);
        RT_CSWAP(k0, c0, k2, c2);
#undef RT_CSWAP
        // branch-free pushes: a missed child is written above the top and not
        // counted (the LDS stack has one spare entry for it).  c0 is the
        // nearest, c2 (the final's loser) goes on top, the first round's
        // losers c1, c3 below it -- the visiting order only affects speed,
        // every hit child is visited
        stk[sp * kBlock] = c3;
        sp += k3 < kInf ? 1 : 0;
        stk[sp * kBlock] = c1;
        sp += k1 < kInf ? 1 : 0;
        stk[sp * kBlock] = c2;
        sp += k2 < kInf ? 1 : 0;
        if (k0 < kInf) {
            node = c0;
        } else {
            node = pop();
        }
        if (node < 0 && node != rtbvh::kEmpty && leaf == rtbvh::kEmpty) {
            leaf = node;                       // park it, keep descending
            node = pop();
        }
    };
    // The root (every trace starts there; wave-uniform) comes through scalar
    // loads: the first step then has no vector-memory wait, which on gfx950
    // would also wait for every frame store the shading step just issued
    // (loads and stores share vmcnt, in order).
    if (point)
        node = root;
    else
        visit_q(sld4(p.bvh, 0), sld4(p.bvh, 1), sld4(p.bvh, 2), sld4(p.bvh, 3), sld4(p.bvh, 4));
    for (;;) {
        while (node >= 0) {
#if RT_PROF >= 2
            const unsigned long long t_a = __builtin_amdgcn_s_memtime();
#endif
            const float4 *N = p.bvh + kNodeF4 * node;
            float4 w0 = N[0], w1 = N[1], w2 = N[2], w3 = N[3], w4 = N[4];
#if RT_PROF >= 2
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::"v"(w0.x), "v"(w3.x) : "memory");
            cnt.t_fetch += __builtin_amdgcn_s_memtime() - t_a;
#endif
            visit_q(w0, w1, w2, w3, w4);
#if RT_PROF >= 2
            cnt.t_trip += __builtin_amdgcn_s_memtime() - t_a;
#endif
            // all but kLeafWait lanes hold a leaf: visit the leaves now (the
            // few still descending wait one leaf round)
            if ((unsigned)__popcll(__ballot(leaf == rtbvh::kEmpty)) <= LEAF_WAIT) break;
        }
        // visit the parked leaf; a leaf the lane stopped on is parked for the
        // next round (one leaf per lane per round: +0.8 % over visiting them
        // back to back, profiles/r02/ab_leaf_one_per_round.txt)
        if (leaf != rtbvh::kEmpty) {
#if RT_PROF
            cnt.trips++;
#endif
            leaf_visit(q, p, leaf, cnt, best, win, opaque, faces_only);
            leaf = rtbvh::kEmpty;
            if (opaque) {
                node = rtbvh::kEmpty;
                stk[0] = rtbvh::kEmpty;        // drop any spilled entries with the rest
                break;
            }
            if (node < 0 && node != rtbvh::kEmpty) {
                leaf = node;
                node = pop();
            }
        }
        if (node == rtbvh::kEmpty && leaf == rtbvh::kEmpty) break;
    }
    if (q.closest) {
        if (win >= 0) {
            q.tmax = best;
            q.win = win;
        }
    } else if (q.skipchk) {
        q.skipped = opaque;
    } else if (opaque) {
        q.mask = {0.0f, 0.0f, 0.0f};
    }
}

// ---------------------------------------------------------------------------
// ShadeRay as a per-lane state machine
// ---------------------------------------------------------------------------
enum Phase { PH_LIGHT = 0, PH_REFR = 1, PH_REFL = 2, PH_REFR_CHILD = 3, PH_REFL_CHILD = 4 };

// ShadeRay state of a lane.  The reference recurses (ShadeRay calls itself,
// main.cpp:1072-1083, :1184-1194); here every lane walks its pixel's shade
// tree as a state machine with one frame per recursion level.
//
//  * LDS, per lane (16 words, kBlock apart: conflict-free): the state of the
//    node being shaded -- shading normal N (flipped for spheres), I = -ray,
//    diffuse colour (after the light loop: F_t, the transmission Fresnel,
//    in its first word), running colour, object, packed phase / light /
//    medium state / stack size, eta_i, eta_t.  Shading a node, and every
//    shadow step of it (63 % of the rays), touches no device memory.
//  * Cold frame per level, in a device buffer (per lane contiguous; not
//    compiler scratch, which interleaves lanes per dword): the node's medium
//    stack (written by the transition that opens the node) and -- only when
//    the node opens a child -- its LDS state and hit point, saved for the
//    child's return.
//
// cos(theta_i) is not stored: it is N.I with the node's final N (main.cpp:
// 864-872 recompute it after the flip).  The shadow mask is not stored
// either: it starts at {1,1,1} before the light loop (main.cpp:788) and lives
// in the shadow query from one light to the next; the hit point of the top
// node lives in the query's origin.
enum { PH_DONE = PH_REFL_CHILD + 1 };
struct HotR {                        // register form of the top node's state
    V3 N, I;
    C3 dif;                          // dif.r holds F_t after the light loop
    C3 acc;
    int obj;
    unsigned meta;                   // phase:3 | state:1 | stack size:5 | light:23
    float ei, et;
};
__device__ __forceinline__ int h_phase(const HotR &h) { return (int)(h.meta & 7u); }
__device__ __forceinline__ int h_state(const HotR &h) { return (int)((h.meta >> 3) & 1u); }
__device__ __forceinline__ int h_sn(const HotR &h) { return (int)((h.meta >> 4) & 31u); }
__device__ __forceinline__ int h_light(const HotR &h) { return (int)(h.meta >> 9); }
__device__ __forceinline__ unsigned mk_meta(int phase, int state, int sn, int light) {
    return (unsigned)phase | ((unsigned)state << 3) | ((unsigned)sn << 4) | ((unsigned)light << 9);
}
__device__ __forceinline__ void set_phase(HotR &h, int phase) { h.meta = (h.meta & ~7u) | (unsigned)phase; }
__device__ __forceinline__ float cos_i(const HotR &h) { return vdot(h.N, h.I); }

// LDS words of the state (word w of lane l at [w * kBlock + l])
enum {
    LW_N = 0, LW_I = 3, LW_DIF = 6, LW_ACC = 9, LW_OBJ = 12, LW_META = 13, LW_EI = 14, LW_ET = 15,
    kLdsHot = 16
};
extern __shared__ float4 rt_lds[];   // dynamic LDS of render_kernel: state, then stack / primitives, lights

// The lights, staged in LDS at kernel start: a shading step's light reads are
// then LDS latency, not a dependent trip to L2 (one dependent load per
// shading step costs ~1 % of C3, profiles/r02/ab_shading_probe.txt)
__device__ __forceinline__ const LightK *lds_lights(const Params &p) {
    return reinterpret_cast<const LightK *>(rt_lds + p.lights_lds);
}

__device__ __forceinline__ float *lane_lds() { return reinterpret_cast<float *>(rt_lds) + threadIdx.x; }
__device__ __forceinline__ int h_light_lds() { return (int)(__float_as_uint(lane_lds()[LW_META * kBlock]) >> 9); }
__device__ __forceinline__ void lds_load(HotR &h) {
    const float *l = lane_lds();
    h.N = {l[(LW_N + 0) * kBlock], l[(LW_N + 1) * kBlock], l[(LW_N + 2) * kBlock]};
    h.I = {l[(LW_I + 0) * kBlock], l[(LW_I + 1) * kBlock], l[(LW_I + 2) * kBlock]};
    h.dif = {l[(LW_DIF + 0) * kBlock], l[(LW_DIF + 1) * kBlock], l[(LW_DIF + 2) * kBlock]};
    h.acc = {l[(LW_ACC + 0) * kBlock], l[(LW_ACC + 1) * kBlock], l[(LW_ACC + 2) * kBlock]};
    h.obj = __float_as_int(l[LW_OBJ * kBlock]);
    h.meta = __float_as_uint(l[LW_META * kBlock]);
    h.ei = l[LW_EI * kBlock];
    h.et = l[LW_ET * kBlock];
}
__device__ __forceinline__ void lds_store(const HotR &h) {
    float *l = lane_lds();
    l[(LW_N + 0) * kBlock] = h.N.x, l[(LW_N + 1) * kBlock] = h.N.y, l[(LW_N + 2) * kBlock] = h.N.z;
    l[(LW_I + 0) * kBlock] = h.I.x, l[(LW_I + 1) * kBlock] = h.I.y, l[(LW_I + 2) * kBlock] = h.I.z;
    l[(LW_DIF + 0) * kBlock] = h.dif.r, l[(LW_DIF + 1) * kBlock] = h.dif.g, l[(LW_DIF + 2) * kBlock] = h.dif.b;
    l[(LW_ACC + 0) * kBlock] = h.acc.r, l[(LW_ACC + 1) * kBlock] = h.acc.g, l[(LW_ACC + 2) * kBlock] = h.acc.b;
    l[LW_OBJ * kBlock] = __int_as_float(h.obj);
    l[LW_META * kBlock] = __uint_as_float(h.meta);
    l[LW_EI * kBlock] = h.ei;
    l[LW_ET * kBlock] = h.et;
}
// what a shadow step changes: the running colour and the light index
__device__ __forceinline__ void lds_store_light(const HotR &h) {
    float *l = lane_lds();
    l[(LW_ACC + 0) * kBlock] = h.acc.r, l[(LW_ACC + 1) * kBlock] = h.acc.g, l[(LW_ACC + 2) * kBlock] = h.acc.b;
    l[LW_META * kBlock] = __uint_as_float(h.meta);
}
// what the light loop's end / a traced refraction or reflection changes
__device__ __forceinline__ void lds_store_phase(const HotR &h) {
    float *l = lane_lds();
    l[LW_DIF * kBlock] = h.dif.r;
    l[(LW_ACC + 0) * kBlock] = h.acc.r, l[(LW_ACC + 1) * kBlock] = h.acc.g, l[(LW_ACC + 2) * kBlock] = h.acc.b;
    l[LW_META * kBlock] = __uint_as_float(h.meta);
}

template <int MAXF>
struct Cold {
    float4 saved[4];                 // the node's LDS state while a child runs
    float P[3];                      // its hit point (incidence_object_intersection.point)
    int stack[MAXF];                 // the CHILD's medium stack (incident_object_stack), object indices:
                                     // written with the node's own state when it opens the child, so
                                     // one frame line is dirtied per child open, not two
    int pad_[(MAXF + 3 + 15) / 16 * 16 - (MAXF + 3)];
};
static_assert(sizeof(Cold<5>) == 128 && sizeof(Cold<9>) == 128 && sizeof(Cold<17>) == 192, "cold frame sizes");

template <int MAXF>
__device__ __forceinline__ void cold_save(Cold<MAXF> &c, V3 P, const HotR &h) {
    f4v *v = reinterpret_cast<f4v *>(c.saved);
    v[0] = f4v{h.N.x, h.N.y, h.N.z, h.I.x};
    v[1] = f4v{h.I.y, h.I.z, h.dif.r, h.dif.g};
    v[2] = f4v{h.dif.b, h.acc.r, h.acc.g, h.acc.b};
    v[3] = f4v{__int_as_float(h.obj), __uint_as_float(h.meta), h.ei, h.et};
    c.P[0] = P.x, c.P[1] = P.y, c.P[2] = P.z;
}
template <int MAXF>
__device__ __forceinline__ V3 cold_restore(const Cold<MAXF> &c, HotR &h) {
    const f4v *v = reinterpret_cast<const f4v *>(c.saved);
    f4v a = v[0], b = v[1], d = v[2], e = v[3];
    h.N = {a.x, a.y, a.z};
    h.I = {a.w, b.x, b.y};
    h.dif = {b.z, b.w, d.x};
    h.acc = {d.y, d.z, d.w};
    h.obj = __float_as_int(e.x);
    h.meta = __float_as_uint(e.y);
    h.ei = e.z;
    h.et = e.w;
    return V3{c.P[0], c.P[1], c.P[2]};
}

// Hit record of the winning intersection, recomputed exactly as TraceRay did.
__device__ void hit_geometry(const Params &p, int obj, V3 o, V3 d, float t, V3 &P, V3 &N, V3 &bary) {
    P = vadd(o, vmul(d, t));
    if (obj < p.nf) {
        const float4 *F = p.fscan + 5 * obj;
        float4 f0 = F[0], f1 = F[1], f2 = F[2], f3 = F[3], f4 = F[4];
        V3 ep = vsub(P, V3{f0.x, f0.y, f0.z});
        V3 e1 = {f2.x, f2.y, f2.z}, e2 = {f3.x, f3.y, f3.z};
        float d1p = vdot(e1, ep), d2p = vdot(e2, ep);
        float b = (f3.w * d1p - f4.x * d2p) / f1.w;
        float g = (f2.w * d2p - f4.x * d1p) / f1.w;
        float a = 1.0f - (b + g);
        bary = {a, b, g};
        const FaceShadeK &fs = p.fsh[obj];
        if (fs.smooth) {
            V3 n0 = {fs.vn[0][0], fs.vn[0][1], fs.vn[0][2]};
            V3 n1 = {fs.vn[1][0], fs.vn[1][1], fs.vn[1][2]};
            V3 n2 = {fs.vn[2][0], fs.vn[2][1], fs.vn[2][2]};
            N = vnorm(vadd(vadd(vmul(n0, a), vmul(n1, b)), vmul(n2, g)));
        } else {
            N = {f1.x, f1.y, f1.z};
        }
    } else {
        float4 s = p.sscan[obj - p.nf];
        N = vnorm(vdiv(vsub(P, V3{s.x, s.y, s.z}), s.w));
        bary = {0, 0, 0};
    }
}

// Texel (x, y) of a texture, channel c -- the reference's nearest texel
// (main.cpp:816-818, :850-852) through map(v, 0, 255, 0, 1) in float.
// Textures are RGB bytes, row-major, in HBM (gfx950 exposes
// no image arrays through HIP, and 32-bit texels in 8x8 tiles measured no
// faster on C4).
__device__ __forceinline__ float texel(const Params &p, const TexK &t, int x, int y, int c) {
    float v = (float)p.texels[t.off + ((long long)y * t.w + x) * 3 + c];
    return (v - 0.0f) * (1.0f - 0.0f) / (255.0f - 0.0f) + 0.0f;   // map(v, 0, 255, 0, 1)
}

// ShadeRay prologue (main.cpp:785-872): hit record, diffuse / texture and the
// sphere normal flip, for the node opened on object `obj` by the closest hit
// at t along (o, d) with medium state m.  Writes the node's LDS state, ready
// for the light loop; returns the hit point.
struct Medium;
__device__ V3 node_open(const Params &p, int obj, V3 o, V3 d, float t, Medium m);

// Direction of light l's shadow ray and the L vector (main.cpp:885-928).
__device__ __forceinline__ void light_vectors(const LightK &lt, V3 P, V3 &L, V3 &sdir, float &distL, bool &unb) {
    if (lt.w == 0.0f) {
        L = {lt.L[0], lt.L[1], lt.L[2]};
        sdir = {lt.sdir[0], lt.sdir[1], lt.sdir[2]};
        distL = 0.0f;
        unb = true;
    } else {
        V3 pos = {lt.xyz[0], lt.xyz[1], lt.xyz[2]};
        L = vnorm(vsub(pos, P));
        V3 dl = vsub(P, pos);
        distL = sqrtf(vdot(dl, dl));
        sdir = L;
        unb = false;
    }
}

// Specular power powf(max(0, N.H), n) (main.cpp:954): exp2(n * log2 x) on the
// transcendental unit (v_log_f32 / v_exp_f32) instead of ocml's ~170-
// instruction powf.  The base is in [0, 1]; relative error ~1e-6 * max(1, |n
// log2 x|), far inside the 1e-4 parity bar on a colour term.  powf's special
// cases that exp2/log2 would get wrong are kept: x^0 = 1 (also for NaN, 0),
// 1^n = 1 (also for n = inf, NaN).
__device__ __forceinline__ float spec_pow(float x, float n) {
    if ((n == 0.0f) | (x == 1.0f)) return 1.0f;
    return __builtin_amdgcn_exp2f(n * __builtin_amdgcn_logf(x));
}

// (float)(F_0 + (1.0 - F_0) * powf(1.0 - cos, 5.0)), main.cpp:966 / :1104
__device__ __forceinline__ float schlick(float F0, float cosI) {
    // powf(x, 5) as x^2^2 * x: within 2 ulp of glibc's powf, and 0 exactly
    // when x is (the `Fr != 0` test of main.cpp:1104 keeps its outcome)
    float x = (float)(1.0 - (double)cosI);
    float x2 = x * x;
    float p5 = (x2 * x2) * x;
    return (float)((double)F0 + (1.0 - (double)F0) * (double)p5);
}
// reflection Fresnel of object ob at cos(theta_i) (main.cpp:1103-1104)
__device__ __forceinline__ float refl_fresnel(const ObjK &ob, float cosI) {
    float F0 = (ob.eta - 1) / (ob.eta + 1);
    return schlick(F0 * F0, cosI);
}

template <int MAXF>
__device__ __forceinline__ bool in_stack(const Cold<MAXF> &f, int sn, int obj) {
    bool in = false;
    for (int q = 0; q < sn; q++) in |= (f.stack[q] == obj);
    return in;
}

// The parent's medium stack into the child's (frame fc holds the parent's,
// c the child's: the frames one level up).  The root node's (level 0, a
// primary hit) is always {its own object} (main.cpp:751-757) and lives in no
// frame.
template <int MAXF>
__device__ __forceinline__ void copy_stack(const HotR &f, const Cold<MAXF> &fc, Cold<MAXF> &c, bool root) {
    if (root) {
        c.stack[0] = f.obj;
    } else {
        const int fsn = h_sn(f);
        for (int q = 0; q < fsn; q++) c.stack[q] = fc.stack[q];
    }
}

// The child's medium state after a transition: state, stack size, eta_i, eta_t
// (its stack is written into the child's cold frame).
struct Medium {
    int state, sn;
    float ei, et;
};

__device__ V3 node_open(const Params &p, int obj, V3 o, V3 d, float t, Medium m) {
    V3 P, N, bary;
    hit_geometry(p, obj, o, d, t, P, N, bary);
    const ObjK &ob = p.objs[obj];
    V3 I = vmul(d, -1.0f);
    float cosI = vdot(N, I);
    C3 dif = {ob.dif[0], ob.dif[1], ob.dif[2]};
    if (ob.tex >= 0) {
        TexK tx = p.texs[ob.tex];
        float width = (float)tx.w, height = (float)tx.h;
        if (ob.is_sphere) {                                          // main.cpp:805-826
            float v = (float)(acos((double)N.z) / kPi);
            float phi = (float)atan2((double)N.y, (double)N.x);
            float u = (phi - (float)-kPi) * (1.0f - 0.0f) / ((float)kPi - (float)-kPi) + 0.0f;
            v = clampr(v, 0.0f, 1.0f);
            u = clampr(u, 0.0f, 1.0f);
            int i = (int)clampr((float)round(((double)height - 1.0) * (double)v), 0.0f,
                                (float)((double)height - 1.0));
            int j = (int)clampr((float)round(((double)width - 1.0) * (double)u), 0.0f,
                                (float)((double)width - 1.0));
            dif = {texel(p, tx, j, i, 0), texel(p, tx, j, i, 1), texel(p, tx, j, i, 2)};
        } else {                                                     // main.cpp:834-861
            const FaceShadeK &fs = p.fsh[obj];
            float u = (bary.x * fs.vt[0][0]) + (bary.y * fs.vt[1][0]) + (bary.z * fs.vt[2][0]);
            float v = (bary.x * fs.vt[0][1]) + (bary.y * fs.vt[1][1]) + (bary.z * fs.vt[2][1]);
            v = clampr(v, 0.0f, 1.0f);
            u = clampr(u, 0.0f, 1.0f);
            int i = (int)clampr(roundf((width - 1.0f) * u), 0.0f, (float)((double)width - 1.0));
            int j = (int)clampr(roundf((height - 1.0f) * v), 0.0f, (float)((double)height - 1.0));
            dif = {texel(p, tx, i, j, 0), texel(p, tx, i, j, 1), texel(p, tx, i, j, 2)};
        }
    }
    if ((double)cosI < 0.0 && ob.is_sphere) {                      // main.cpp:869-872
        N = vmul(N, -1.0f);
    }
    HotR h;
    h.N = N;
    h.I = I;
    h.dif = dif;
    h.acc = C3{0.0f, 0.0f, 0.0f};    // tmp_specular while lights run
    h.obj = obj;
    h.meta = mk_meta(PH_LIGHT, m.state, m.sn, 0);
    h.ei = m.ei;
    h.et = m.et;
    lds_store(h);
    return P;
}

// Medium-stack transition for the refraction child (main.cpp:1021-1070).
template <int MAXF>
__device__ Medium refr_transition(const Params &p, const HotR &f, const Cold<MAXF> &fc, Cold<MAXF> &c, int hit,
                                  bool root, Counters &cnt) {
    const int fsn = h_sn(f);
    copy_stack(f, fc, c, root);
    int n = fsn;
    Medium m;
    float hit_eta = p.objs[hit].eta;
    if (h_state(f) == ENTERING) {
        if (hit == f.obj) {
            m.state = EXITING;
            if (n > 0) {
                m.ei = p.objs[c.stack[n - 1]].eta;
                n--;
            } else {
                m.ei = p.eta_bkg;            // back() on an empty vector: UB in the reference
                cnt.ub++;
            }
            m.et = n > 0 ? p.objs[c.stack[n - 1]].eta : p.eta_bkg;
            if (n > 0) n--;
        } else {
            m.state = ENTERING;
            m.ei = f.et;
            m.et = hit_eta;
            c.stack[n++] = hit;
        }
    } else if (n > 0) {
        if (!(root ? hit == f.obj : in_stack(fc, fsn, hit))) {
            m.state = ENTERING;
            m.ei = f.et;
            m.et = hit_eta;
            c.stack[n++] = hit;
        } else {
            m.state = EXITING;
            m.ei = f.et;
            m.et = p.objs[c.stack[n - 1]].eta;
            n--;
        }
    } else {
        m.state = ENTERING;
        m.ei = p.eta_bkg;
        m.et = hit_eta;
        c.stack[0] = hit;
        n = 1;
    }
    m.sn = n;
    return m;
}

// Medium-stack transition for the reflection child (main.cpp:1134-1182).
template <int MAXF>
__device__ Medium refl_transition(const Params &p, const HotR &f, const Cold<MAXF> &fc, Cold<MAXF> &c, int hit,
                                  bool root) {
    const int fsn = h_sn(f);
    copy_stack(f, fc, c, root);
    int n = fsn;
    Medium m;
    float hit_eta = p.objs[hit].eta;
    if (h_state(f) == ENTERING) {
        m.state = ENTERING;
        m.ei = f.ei;
        if (n > 0) {
            if (!(root ? hit == f.obj : in_stack(fc, fsn, hit))) {
                m.et = hit_eta;
                c.stack[n++] = f.obj;        // pushes the incidence object, as the reference does
            } else {
                m.et = p.objs[c.stack[n - 1]].eta;
                n--;
            }
        } else {
            m.et = hit_eta;
            c.stack[0] = hit;
            n = 1;
        }
    } else {
        m.ei = f.ei;
        if (hit == f.obj) {
            m.state = EXITING;
            m.et = f.et;
        } else {
            m.state = ENTERING;
            m.et = hit_eta;
            c.stack[n++] = hit;
        }
    }
    m.sn = n;
    return m;
}

// Lane state between scans: the recursion level of its top node; its cold
// frames (Params::frames, MAXF per lane, contiguous) are addressed from the
// workgroup / lane ids where they are used rather than kept in 2 VGPRs across
// the traversal.
template <int MAXF>
struct LaneState {
    void *frames;
    int top;                         // -1: primary ray pending
    __device__ __forceinline__ Cold<MAXF> *cold() const {
        // opaque: LLVM would otherwise hoist the address out of the
        // persistent loop and keep it in a (spilled) VGPR pair
        unsigned t;
        asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"((unsigned)threadIdx.x));
        return reinterpret_cast<Cold<MAXF> *>(frames) + ((size_t)blockIdx.x * kBlock + t) * MAXF;
    }
};

__device__ __forceinline__ void shadow_query(Query &q, const Params &p, int light, int self) {
    V3 L, sd;
    float dl;
    bool unb;
    light_vectors(lds_lights(p)[light], q.o, L, sd, dl, unb);
    q.d = sd;
    q.tmin = p.eps;
    q.tmax = dl;
    q.unb = unb;
    q.self = self;
    q.closest = false;
    q.skipchk = false;
    q.skipped = false;
    q.win = -1;
}

__device__ __forceinline__ void closest_query(Query &q, const Params &p, V3 d) {
    q.d = d;
    q.tmin = p.eps;
    q.tmax = kFltMax;
    q.unb = false;
    q.self = -1;
    q.closest = true;
    q.skipchk = false;
    q.skipped = false;
    q.win = -1;
}

// Advance one lane after its scan: consume the result, run ShadeRay logic
// until the next TraceRay (returns its kind, RK_SHADOW/RK_REFR/RK_REFL, with q
// set up) or until the pixel is done (returns RK_NONE with `color` set).
// Invariant: while a node is on top, q.o is its hit point.
template <int MAXF>
__device__ int advance(const Params &p, LaneState<MAXF> &ls, Query &q, Counters &cnt, C3 &color) {
    const C3 bkg = {p.bkg[0], p.bkg[1], p.bkg[2]};
    int top = ls.top;
    HotR h;
    // a closest hit opens node `top` (primary hit, refraction or reflection
    // child); its ShadeRay prologue runs at ONE call site below, so a wave
    // whose lanes open nodes for different reasons runs it once
    bool open = false;
    Medium m;
    // ---- consume the scan result ----
    if (top < 0) {                                   // primary (main.cpp:729-758)
        if (q.win < 0) {
            color = bkg;
            return RK_NONE;
        }
        m = Medium{ENTERING, 1, p.eta_bkg, p.objs[q.win].eta};   // stack {q.win}: implicit (copy_stack)
        open = true;
        top = 0;
    } else {
        lds_load(h);
        const int phase = h_phase(h);
        if (phase == PH_LIGHT) {                     // main.cpp:952-958
            const int light = h_light(h);
            // the light's words in one batch (LightK: xyz w | col | L)
            const f4v *lw = reinterpret_cast<const f4v *>(lds_lights(p) + light);
            const f4v lw0 = lw[0], lw1 = lw[1], lw2 = lw[2];
            // L as light_vectors computed it for the shadow ray just traced:
            // that ray's direction for a point light, the constant -L for a
            // directional one (q.d is not modified by a trace)
            V3 L = lw0.w == 0.0f ? V3{lw2.x, lw2.y, lw2.z} : q.d;
            const ObjK &ob = p.objs[h.obj];
            // H only feeds the specular power: rsqrt instead of 3 IEEE
            // divisions (<= 2 ulp; vnorm(0) = NaN either way)
            V3 hv = vadd(L, h.I);
            V3 H = vmul(hv, __builtin_amdgcn_rsqf(vdot(hv, hv)));
            C3 dc = cmulf(cmulf(h.dif, ob.kd), max0(vdot(h.N, L)));
            C3 sc = cmulf(cmulf(C3{ob.spc[0], ob.spc[1], ob.spc[2]}, ob.ks), spec_pow(max0(vdot(h.N, H)), ob.n));
            C3 lc = {lw1.x, lw1.y, lw1.z};
            h.acc = cadd(h.acc, cmulc(cmulc(lc, q.mask), cadd(dc, sc)));
            h.meta += 1u << 9;                       // next light
            if (light + 1 < p.nl) {
                // next light's shadow ray from the same point: origin, self
                // and cumulative mask are already in q (main.cpp:885-928)
                lds_store_light(h);
                // (opaque index: reusing this light's address for the next
                // one kept a 64-bit pointer live -- and spilled -- across the
                // shading code)
                int next = light + 1;
                asm volatile("" : "+v"(next));
                shadow_query(q, p, next, h.obj);
                ls.top = top;
                return RK_SHADOW;
            }
        } else if (phase == PH_REFR) {
            if (q.skipped) {
                cnt.skip++;                          // tmp_transparency stays 0
                set_phase(h, PH_REFL);
            } else if (q.win >= 0) {
                m = refr_transition(p, h, ls.cold()[top > 0 ? top - 1 : 0], ls.cold()[top], q.win, top == 0, cnt);
                set_phase(h, PH_REFR_CHILD);
                open = true;
            } else {
                const ObjK &ob = p.objs[h.obj];
                C3 tr = cmulf(cmulf(bkg, (float)(1.0 - (double)h.dif.r)), (float)(1.0 - (double)ob.opacity));
                h.acc = cadd(h.acc, tr);
                set_phase(h, PH_REFL);
            }
        } else {                                     // PH_REFL
            if (q.win >= 0) {
                m = refl_transition(p, h, ls.cold()[top > 0 ? top - 1 : 0], ls.cold()[top], q.win, top == 0);
                set_phase(h, PH_REFL_CHILD);
                open = true;
            } else {
                // miss: refl = bkg * F_r; finish this node below
                h.acc = cadd(h.acc, cmulf(bkg, refl_fresnel(p.objs[h.obj], cos_i(h))));
                set_phase(h, PH_DONE);
            }
        }
        if (open) {                                  // the recursion: save the parent
            cold_save(ls.cold()[top], q.o, h);
            top++;
        }
    }
    if (open) {
        q.o = node_open(p, q.win, q.o, q.d, q.tmax, m);
        ls.top = top;
        if (p.nl > 0) {                              // shadow ray for light 0 (main.cpp:885-928)
            shadow_query(q, p, 0, q.win);
            q.mask = C3{1.0f, 1.0f, 1.0f};           // the node's first light (main.cpp:788)
            return RK_SHADOW;
        }
        lds_load(h);                                 // no lights: straight to the light loop's end
    }
    // ---- run the top node forward (phase PH_LIGHT here: its last light is done) ----
    for (;;) {
        const ObjK &ob = p.objs[h.obj];
        if (h_phase(h) == PH_LIGHT) {
            // ambient + specular sum, then Fresnel / transmission (main.cpp:961-992)
            h.acc = cadd(cmulf(h.dif, ob.ka), h.acc);
            const float cosI = cos_i(h);
            float snell = h.ei / h.et;
            float crit = asinf(h.et / h.ei);
            float inc = acosf(cosI);
            bool tir = (crit < inc) && ((double)inc < kRightAngle);
            float F0 = (h.et - h.ei) / (h.et + h.ei);
            h.dif.r = schlick(F0 * F0, cosI);        // F_t (the diffuse colour is no longer needed)
            if (p.depth - top > 0 && !tir && (double)ob.opacity < 1.0 && ob.eta > 0) {
                float k = sqrtf((float)(1.0 - (double)(snell * snell) * (1.0 - (double)(cosI * cosI))));
                V3 T = vadd(vmul(vmul(h.N, -1.0f), k), vmul(vsub(vmul(h.N, cosI), h.I), snell));
                closest_query(q, p, T);
                const int sn = h_sn(h);
                q.skipchk = (sn > 0) && !ob.is_sphere;
                q.back = sn > 0 ? (top == 0 ? h.obj : ls.cold()[top - 1].stack[sn - 1]) : -1;
                set_phase(h, PH_REFR);
                lds_store_phase(h);
                ls.top = top;
                return RK_REFR;
            }
            set_phase(h, PH_REFL);
        }
        if (h_phase(h) == PH_REFL) {                 // main.cpp:1103-1124
            const float cosI = cos_i(h);
            float Fr = refl_fresnel(ob, cosI);
            if (p.depth - top > 0 && (double)Fr != 0.0 && (double)ob.ks > 0.0) {
                V3 R = vsub(vmul(h.N, (float)(2.0 * (double)cosI)), h.I);
                closest_query(q, p, R);
                lds_store_phase(h);
                ls.top = top;
                return RK_REFL;
            }
            set_phase(h, PH_DONE);
        }
        // node complete: ((dka + spec) + trans) + refl already folded into acc
        const C3 c = h.acc;
        if (top == 0) {
            color = c;
            ls.top = -1;
            return RK_NONE;
        }
        top--;
        q.o = cold_restore(ls.cold()[top], h);
        const ObjK &pob = p.objs[h.obj];
        if (h_phase(h) == PH_REFR_CHILD) {           // main.cpp:1072-1083
            C3 tr = cmulf(cmulf(c, (float)(1.0 - (double)h.dif.r)), (float)(1.0 - (double)pob.opacity));
            h.acc = cadd(h.acc, tr);
            set_phase(h, PH_REFL);
        } else {                                     // PH_REFL_CHILD, main.cpp:1184-1194
            h.acc = cadd(h.acc, cmulf(c, refl_fresnel(pob, cos_i(h))));
            set_phase(h, PH_DONE);
        }
        lds_store(h);                                // the parent is the top node again
    }
}

// image row of local row r (block-interleaved row sets for multi-GPU balance)
__device__ __forceinline__ int image_row(const Params &p, int r) {
    return p.y0 + (r / p.rblock) * p.rstep + r % p.rblock;
}

// Pixel index -> (x, y): strips of kStrip rows, column by column along the
// strip, so a refill batch of consecutive indices is a compact block of
// pixels (32 lanes: 4 columns x 8 rows).  Z order inside 8x8 tiles was +0.6 %
// while every idle lane was refilled at once; with the batched refill column
// order is C3 +1.9 %, C5 +2.5 % (profiles/r02/ab_pixel_order.txt).  A
// bijection, so the image does not change.
constexpr int kStrip = 8;   // 4 / 16-row strips: C3 -1.6 / -4 %, C5 -3.7 / -3.9 %
__device__ __forceinline__ void pixel_xy(const Params &p, unsigned idx, int &x, int &y) {
    unsigned strip_px = (unsigned)p.W * (unsigned)kStrip;
    unsigned s = idx / strip_px;
    unsigned r = idx - s * strip_px;
    int sh = min(kStrip, p.rows - (int)s * kStrip);
    x = (int)(r / (unsigned)sh);
    y = (int)s * kStrip + (int)(r % (unsigned)sh);
}

// Primary ray of local pixel (x, y): p = ul + dh * x + dv * row, direction
// (p - eye).norm() (main.cpp:720-728, that association order)
__device__ __forceinline__ V3 primary_dir(const Params &p, int x, int y) {
    V3 pt = vadd(vadd(V3{p.ul[0], p.ul[1], p.ul[2]}, vmul(V3{p.dh[0], p.dh[1], p.dh[2]}, (float)x)),
                 vmul(V3{p.dv[0], p.dv[1], p.dv[2]}, (float)image_row(p, y)));
    return vnorm(vsub(pt, V3{p.eye[0], p.eye[1], p.eye[2]}));
}

template <int MAXF, int MODE>
__global__ void __launch_bounds__(kBlock, RT_MIN_WAVES) render_kernel(Params p) {
    constexpr bool SRC_LDS = MODE == MODE_SCAN_LDS;
    // LDS: every lane's shading state (kLdsHot words, kBlock apart), then the
    // staged primitives (MODE_SCAN_LDS) or the BVH traversal stacks (MODE_BVH)
    float4 *lds = rt_lds + kLdsHot * kBlock / 4;
    const float4 *lds_f = lds;
    const float4 *lds_s = lds + 5 * p.nf;
    if (SRC_LDS) {
        int nf4 = 5 * p.nf, ns4 = p.ns;
        for (int i = threadIdx.x; i < nf4; i += blockDim.x) lds[i] = p.fscan[i];
        for (int i = threadIdx.x; i < ns4; i += blockDim.x) lds[nf4 + i] = p.sscan[i];
    }
    {
        const int nl4 = p.nl * (int)(sizeof(LightK) / sizeof(float4));
        const float4 *src = reinterpret_cast<const float4 *>(p.lights);
        for (int i = threadIdx.x; i < nl4; i += blockDim.x) rt_lds[p.lights_lds + i] = src[i];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    LaneState<MAXF> ls;
    ls.top = -1;
    ls.frames = p.frames;
    Counters cnt = {0, 0, 0, 0, 0};
    unsigned long long w_prim = 0, w_shadow = 0, w_refr = 0, w_refl = 0;   // per wave (uniform)
    unsigned w_known = 0, w_bf = 0;
    int *stk = reinterpret_cast<int *>(lds) + threadIdx.x;  // MODE_BVH: stack[k * kBlock]
    if (MODE == MODE_BVH) stk[0] = rtbvh::kEmpty;           // bvh_trace's stack bottom (never overwritten)
    Query q;
    bool busy = false;         // lane owns a pixel
    bool pending = false;      // q holds a finished scan to consume
    bool held = false;         // q is set up but its search is held back (p.gate_x)
    int held_kind = RK_NONE;
    bool drained = false;      // wave saw the work counter run out
    unsigned chunk_pos = 0, chunk_end = 0;   // the wave's tile: its unused work items [pos, end)
    int px = 0, py = 0;
#if RT_PROF >= 2
    cnt.t_fetch = cnt.t_trip = 0;
#endif
    // launch timeline on the constant 100 MHz clock (comparable across CUs /
    // XCDs): first wave start .. last wave end = the launch's device time even
    // when launches of several frames overlap (rt_scene_last_stats)
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
#if RT_PROF
    cnt.trips = 0;
    cnt.trips_kind[0] = cnt.trips_kind[1] = cnt.trips_kind[2] = 0;
    unsigned long long pc_shade = 0, pc_trace = 0, pc_bf = 0, pc_iter = 0, pc_lanes = 0, pc_wtrips = 0;
    unsigned long long pc_mixed = 0;     // trace steps with primary and secondary/shadow searches together
    unsigned long long t_drain = 0;
#endif
    for (;;) {
#if RT_PROF
        unsigned long long c0 = __builtin_amdgcn_s_memtime();
#endif
        int kind = RK_NONE;
        if (pending && !held) {
            C3 color;
            kind = advance<MAXF>(p, ls, q, cnt, color);
            pending = kind != RK_NONE;
            if (!pending) {
                float *o = p.out + ((size_t)py * p.W + px) * 3;
                o[0] = color.r;
                o[1] = color.g;
                o[2] = color.b;
                busy = false;
            }
        }
        // refill idle lanes: ballot + one atomic per wave + mbcnt prefix.
        // Only once at least p.refill_min lanes are idle (or all are): the
        // lanes a wave refills together start their pixels in the same phase
        // and stay in step, so a trace step seldom mixes primary searches
        // with the shorter shadow searches of other lanes, and the step,
        // which lasts as long as its longest search, is not stretched by a
        // few new primaries.  Idle lanes sit out the steps until then
        // (C3 +10 %, C4 +30 %, C5 +50 % against refilling every idle lane at
        // once; see refill_for).
        if (!drained) {
            unsigned long long idle = __ballot(!busy);
            if (idle && ((unsigned)__popcll(idle) >= p.refill_min || idle == ~0ull)) {
                unsigned n = (unsigned)__popcll(idle);
                int leader = __ffsll((long long)idle) - 1;
                // The wave takes max(p.chunk, n) work items at a time and
                // refills its lanes from them (p.chunk = 0, the default: just
                // its idle lanes' count; option chunk = 64 keeps a wave on one
                // 8x8 tile, chunk_for).  Ranks < split take the rest of the
                // current chunk, the others the start of the next one.
                const unsigned left = chunk_end - chunk_pos;
                const unsigned base = chunk_pos, split = min(n, left);
                unsigned nbase = 0;
                if (n > left) {
                    unsigned g = 0;
                    const unsigned take = max(p.chunk, n - split);
                    if (lane == leader) g = atomicAdd(p.work, take);
                    nbase = (unsigned)__builtin_amdgcn_readlane((int)g, leader);   // uniform: an SGPR
                    chunk_pos = nbase + (n - split);
                    chunk_end = nbase + take;
                    if (nbase >= p.total) drained = true;
                } else {
                    chunk_pos += n;
                }
#if RT_PROF
                if (drained) t_drain = __builtin_amdgcn_s_memrealtime();
#endif
                if (!busy) {
                    unsigned rank = (unsigned)__popcll(idle & ((1ull << lane) - 1ull));
                    unsigned idx = rank < split ? base + rank : nbase + (rank - split);
                    if (idx < p.total) {
                        pixel_xy(p, idx, px, py);
                        q.o = V3{p.eye[0], p.eye[1], p.eye[2]};
                        q.d = primary_dir(p, px, py);
                        q.tmin = 0.0f;               // primary rays accept any t > 0 (main.cpp:736)
                        q.tmax = kFltMax;
                        q.unb = false;
                        q.self = -1;
                        q.closest = true;
                        q.skipchk = false;
                        q.skipped = false;
                        q.win = -1;
                        ls.top = -1;
                        kind = RK_PRIMARY;
                        busy = true;
                        pending = true;
                    }
                }
            }
        }
        if (!pending) q.tmin = kInf;                 // lane sits this scan out
        if (__ballot(pending) == 0ull) break;
        // A shadow ray whose cumulative mask (main.cpp:788, carried across the
        // lights) is already exactly 0 keeps it 0 whatever it hits: every
        // factor is in [0, 1] when none is NaN (shadow_early_out), and
        // clamp01(0 * f) = 0.  It is still a TraceRay call of the reference
        // (counted above); its result is known without searching.
        const bool known = pending && !q.closest && p.shadow_early_out && (q.mask.r == 0.0f) &
                           (q.mask.g == 0.0f) & (q.mask.b == 0.0f);
        // Reflection / refraction searches (closest hit, the longest after
        // the primaries) are held back until at least p.gate_x lanes of the
        // wave have one, unless nothing else would search in this step: like
        // the deferred refill, this batches them into fewer trace steps
        // instead of stretching almost every step with a few of them (C3
        // +8.7 %, C5 +4.6 %; holding shadow searches too: -0.7 %,
        // profiles/r02/ab_gate.txt).  A held lane keeps its query and skips
        // the shading step.
        {
            const int k = held ? held_kind : kind;
            const bool sec = pending && (k == RK_REFR || k == RK_REFL);
            const unsigned nsec = (unsigned)__popcll(__ballot(sec));
            const bool others = __ballot(pending && !sec) != 0ull;
            held = sec && others && nsec < p.gate_x;
            held_kind = k;
        }
        const bool search = pending && !known && !held;

        w_prim += (unsigned long long)__popcll(__ballot(kind == RK_PRIMARY));
        w_shadow += (unsigned long long)__popcll(__ballot(kind == RK_SHADOW));
        w_refr += (unsigned long long)__popcll(__ballot(kind == RK_REFR));
        w_refl += (unsigned long long)__popcll(__ballot(kind == RK_REFL));
        w_known += (unsigned)__popcll(__ballot(known));
        if (MODE == MODE_BVH) {
            // dir_bf == 1: directional shadow rays go to the scan (a light's
            // shadow-region tree could not be built)
            q.bf = search && !q.closest && q.unb && p.dir_bf == 1;
            // SKIP_TRANS check (main.cpp:997-1002): the stack top's own
            // nearest root first, then an any-hit search for a candidate the
            // reference's in-order scan would have taken before it
            const bool skip = search && q.skipchk;
            if (skip) {
                q.tmax = own_nearest(q, p, q.back, cnt);
                q.closest = false;
                q.unb = true;
            }
#if RT_PROF
            unsigned long long c1 = __builtin_amdgcn_s_memtime();
            pc_shade += c1 - c0;
            pc_iter++;
            pc_lanes += (unsigned long long)__popcll(__ballot(search && !q.bf));
            unsigned tr0 = cnt.trips;
#endif
            if (search && !q.bf) bvh_trace<false, leaf_wait_for(MAXF)>(q, p, stk, cnt);
            if (skip) {
                q.closest = true;
                q.unb = false;
                if (!q.skipped) q.win = q.tmax < kFltMax ? q.back : -1;
            }
            // directional shadow rays against spheres: a point query in the
            // light's shadow-region tree (the pass above tested the faces),
            // unless the faces already made the mask 0 for good
            if (p.dir_bf == 2) {
                const bool pt = search && !q.closest && q.unb && !q.bf &&
                                !(p.shadow_early_out && (q.mask.r == 0.0f) & (q.mask.g == 0.0f) & (q.mask.b == 0.0f));
                if (__ballot(pt) && pt) {
                    const DirK &dk = p.dirk[h_light_lds()];
                    const int root = dk.root;
                    if (root >= 0) {
                        V3 po = {fmaf(dk.R[0], q.o.x, fmaf(dk.R[1], q.o.y, dk.R[2] * q.o.z)),
                                 fmaf(dk.R[3], q.o.x, fmaf(dk.R[4], q.o.y, dk.R[5] * q.o.z)),
                                 fmaf(dk.R[6], q.o.x, fmaf(dk.R[7], q.o.y, dk.R[8] * q.o.z))};
                        bvh_trace<true>(q, p, stk, cnt, root, po, dk.cone_k, dk.cone_h);
                    }
                }
            }
#if RT_PROF
            int d = (int)(cnt.trips - tr0);
            cnt.trips_kind[kind == RK_PRIMARY ? 0 : kind == RK_SHADOW ? 1 : 2] += (unsigned)d;
            for (int o = 32; o > 0; o >>= 1) d = max(d, __shfl_xor(d, o));
            pc_wtrips += (unsigned long long)d;
            pc_mixed += (__ballot(search && kind == RK_PRIMARY) != 0ull) && (__ballot(search && kind != RK_PRIMARY) != 0ull);
            unsigned long long c2 = __builtin_amdgcn_s_memtime();
            pc_trace += c2 - c1;
#endif
            bool need = search && q.bf;
            const unsigned long long nb = __ballot(need);
            w_bf += (unsigned)__popcll(nb);
            if (nb) scan<false>(q, p, lds_f, lds_s, need, cnt.ftests, cnt.stests);
#if RT_PROF
            pc_bf += __builtin_amdgcn_s_memtime() - c2;
#endif
        } else {
            scan<SRC_LDS>(q, p, lds_f, lds_s, search, cnt.ftests, cnt.stests);
        }
    }
    unsigned long long *st = p.stats;
    if (lane == 0) {
        atomicAdd(&st[0], w_prim);
        atomicAdd(&st[1], w_shadow);
        atomicAdd(&st[2], w_refr);
        atomicAdd(&st[3], w_refl);
        atomicAdd(&st[32], (unsigned long long)w_known);
        atomicAdd(&st[33], (unsigned long long)w_bf);
    }
    atomicAdd(&st[4], (unsigned long long)cnt.skip);
    atomicAdd(&st[5], (unsigned long long)cnt.ub);
    atomicAdd(&st[6], (unsigned long long)cnt.boxes);
    atomicAdd(&st[7], (unsigned long long)cnt.ftests);
    atomicAdd(&st[8], (unsigned long long)cnt.stests);
    const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        atomicMin(&st[24], t_start);                 // kernel start (first wave)
        atomicMax(&st[26], t_end);                   // last wave done
    }
#if RT_PROF
    if (lane == 0) {
        atomicAdd(&st[9], pc_shade);
        atomicAdd(&st[10], pc_trace);
        atomicAdd(&st[11], pc_bf);
        atomicAdd(&st[12], pc_iter);
        atomicAdd(&st[13], pc_lanes);
        atomicAdd(&st[14], pc_wtrips);
        atomicAdd(&st[39], pc_mixed);
    }
    atomicAdd(&st[15], (unsigned long long)cnt.trips);
    atomicAdd(&st[36], (unsigned long long)cnt.trips_kind[0]);
    atomicAdd(&st[37], (unsigned long long)cnt.trips_kind[1]);
    atomicAdd(&st[38], (unsigned long long)cnt.trips_kind[2]);
    if (lane == 0) {
        if (!t_drain) t_drain = t_end;
        atomicMin(&st[25], t_drain);                 // work counter ran out
        atomicAdd(&st[27], t_end - t_drain);         // sum of per-wave tails
        atomicAdd(&st[28], t_end - t_start);         // sum of wave lifetimes
        atomicAdd(&st[29], 1ull);                    // waves
    }
#if RT_PROF >= 2
    atomicAdd(&st[30], cnt.t_fetch);
    atomicAdd(&st[31], cnt.t_trip);
#endif
#endif
}

// Gathered row sets -> image order (rt_deinterleave_rows): one thread per
// float4 of an image row; image row y belongs to rank (y / block) % world as
// its local row (y / (block * world)) * block + y % block.
__global__ void deinterleave_kernel(const float *__restrict__ gathered, int world, int rows_per, int W, int H,
                                    int block, float *__restrict__ image) {
    const int y = blockIdx.y;
    const int rank = (y / block) % world;
    const int k = (y / (block * world)) * block + y % block;
    const size_t n = (size_t)W * 3;
    const float *src = gathered + ((size_t)rank * rows_per + k) * n;
    float *dst = image + (size_t)y * n;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

}  // namespace rt

// ===========================================================================
// Host side: scene upload and the C ABI
// ===========================================================================
using namespace rt;

// One render in flight: its work counter, counters, ShadeRay frame buffer and
// events.  A scene has `inflight` of them (rt_scene_set_option "inflight"):
// with one, a render runs on the caller's stream; with more, render k runs on
// slot k mod n's own stream, ordered against the caller's stream by events, so
// that renders issued on different caller streams (independent frames) overlap:
// the next frame's workgroups fill the CUs that the current frame's tail leaves
// idle.
struct RenderSlot {
    hipStream_t stream = nullptr;      // slots > 1 only (high priority: its own HW queue pool)
    hipEvent_t ev_in = nullptr;        // caller stream -> slot stream
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    unsigned int *work = nullptr;
    unsigned long long *stats = nullptr;
    void *d_frames = nullptr;          // ShadeRay frames of the launch
    size_t frames_cap = 0;
    bool used = false;                 // ev1 marks a render issued through this slot
};

struct rt_scene {
    int device = 0;
    hipStream_t stream = nullptr;
    Params base{};
    std::vector<void *> allocs;
    float *dev_out = nullptr;          // staging buffer when the caller passes host memory
    size_t dev_out_bytes = 0;
    std::vector<RenderSlot> slots;     // slots[0] always exists
    int next_slot = 0;                 // slot of the next render
    int last_slot = 0;                 // slot of the last render
    int num_cu = 0;
    size_t lds_bytes = 0;
    long long opt_lds = -1;            // -1 auto, 0 off, 1 on
    long long opt_grid = 0;            // blocks (0 = occupancy-derived)
    long long opt_chunk = -1;          // refill chunk (-1: default, chunk_for)
    long long opt_refill_min = -1;     // idle lanes before a refill (-1: by the scene, refill_for)
    bool secondary = false;            // some material reflects (ks > 0) or refracts (opacity < 1, eta > 0)
    long long opt_reserve = 0;         // occupancy-derived grid: block slots left free for other kernels
    long long opt_accel = -1;          // -1 auto, 0 brute-force scan, 1 BVH
    long long opt_bvh_leaf = 8;        // SAH max leaf size
    long long opt_bvh_trav = 500;      // SAH traversal cost, x1000 of a sphere test (A/B: 0.5 best)
    long long opt_bvh_collapse = 1;    // binary -> 4-wide: 0 greedy (largest area first), 1 SAH-optimal DP
    long long opt_bvh_node = 500;      // DP collapse: cost of a 4-wide node visit, x1000 of a sphere test
                                       // (A/B, C3: 0.25 / 0.5 / 0.75 / 1 / 2 -> +0.6 / +0.5 / +0.5 / +0.2 / -1.7 %)
    long long opt_fail_bvh_upload = 0; // test hook: the next BVH uploads fail (RT_E_NOMEM)
    // BVH inputs kept on the host (the boxes' padding depends on the eye)
    struct PrimSrc {
        int key;
        bool sphere;
        float lo[3], hi[3];            // face: vertex bounds; sphere: centre +- r
        float c[3], r;                 // sphere centre / radius
        double cond;                   // face: |e1|^2 |e2|^2 / det
    };
    std::vector<PrimSrc> prims;
    float scene_lo[3] = {0, 0, 0}, scene_hi[3] = {0, 0, 0};
    double bvh_D = -1.0;               // distance bound the current BVH was padded for
    float4 *d_bvh = nullptr;
    float4 *d_leafrec = nullptr;
    DirK *d_dirk = nullptr;            // per light: shadow-region tree (directional lights)
    std::vector<float4> h_fscan, h_sscan;   // host copies for the leaf records
    std::vector<float> h_ofac;
    std::vector<LightK> h_lights;

    int bvh_depth = 0;
    int bvh_stack = 0;
    int ovf_stride = kSpill;           // spilled BVH stack entries per lane (Params::ovf_stride)
    bool bvh_ok = false;
    double bvh_build_ms = 0.0;         // host time of the last BVH (re)build
    long long last_blocks_per_cu = 0, last_grid = 0, last_lds = 0, last_mode = -1;
    long long bvh_nodes = 0;
    bool last_valid = false;
};

namespace {

const char *kErr[] = {"ok", "invalid argument", "no such HIP device", "HIP runtime error", "out of device memory",
                      "unsupported"};

template <typename T, typename P>
int upload(rt_scene *s, const std::vector<T> &v, P &dst) {
    size_t bytes = std::max<size_t>(1, v.size()) * sizeof(T);
    void *d = nullptr;
    if (hipMalloc(&d, bytes) != hipSuccess) return RT_E_NOMEM;
    s->allocs.push_back(d);
    if (!v.empty() && hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice) != hipSuccess)
        return RT_E_HIP;
    dst = static_cast<P>(d);
    return RT_OK;
}

V3 f3(const float *p) { return {p[0], p[1], p[2]}; }

// Dynamic LDS of render_kernel: the per-lane shading state, the mode's region
// (BVH stacks or the staged primitives), then the lights.
size_t mode_region_end(const rt_scene *s, int mode) {
    size_t shade = (size_t)kLdsHot * kBlock * sizeof(float);         // per-lane shading state
    if (mode == MODE_SCAN_LDS) return shade + s->lds_bytes;
    if (mode == MODE_BVH) return shade + (size_t)s->base.stack_cap * kBlock * sizeof(int);
    return shade;
}
size_t mode_lds_bytes(const rt_scene *s, int mode) {
    return mode_region_end(s, mode) + (size_t)s->base.nl * sizeof(LightK);
}

// Work items a wave takes from the pixel counter at a time: by default
// exactly its idle lanes' count.  A whole 8x8 tile per wave (64) was +5 % on
// C3 while every idle lane was refilled at once; with the deferred refill
// (refill_for) it is -3 % on C3 and -10 % on C4, and it never changes the
// image (profiles/r02/ab_chunk_auto.txt, ab_refill_min.txt).
static unsigned chunk_for(const rt_scene *s) {
    return s->opt_chunk >= 0 ? (unsigned)s->opt_chunk : 0u;
}

// How many lanes of a wave must be idle before it refills them.  With only
// primary and shadow rays, a pixel lasts a few trace steps: the whole wave
// starts 64 pixels together and finishes them before the next batch (C4
// 10.9 G rays/s against 10.7 at 48 and 8.3 at 1).  With reflection /
// refraction, 32 up to depth 4 (C3 +0.8 % over 40 in 4 rounds, C3G +0.9 %,
// C3D -0.2 %) and 48 for deeper shade trees, whose pixels live longer (C5
// +0.8 % over 40, -1.6 % at 32; profiles/r02/ab_refill_min.txt, ab_gate.txt).
static unsigned refill_for(const rt_scene *s, const Params &p) {
    if (s->opt_refill_min > 0) return (unsigned)s->opt_refill_min;
    if (!s->secondary || p.depth <= 0) return 64u;
    return p.depth > 4 ? 48u : 32u;
}

template <int MAXF, int MODE>
hipError_t launch_one(rt_scene *s, RenderSlot &slot, const Params &p, hipStream_t st, bool dry) {
    size_t shm = mode_lds_bytes(s, MODE);
    int nb = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, render_kernel<MAXF, MODE>, kBlock, shm);
    if (nb < 1) nb = 1;
    long long grid = s->opt_grid > 0 ? s->opt_grid : (long long)nb * s->num_cu - s->opt_reserve;
    long long need = ((long long)p.total + kBlock - 1) / kBlock;
    if (grid > need) grid = need;
    if (grid < 1) grid = 1;
    Params pl = p;
    pl.chunk = chunk_for(s);
    pl.refill_min = refill_for(s, pl);
    pl.lights_lds = (int)(mode_region_end(s, MODE) / sizeof(float4));
    const size_t cold_bytes = (size_t)grid * kBlock * MAXF * sizeof(Cold<MAXF>);
    size_t fbytes = cold_bytes + (size_t)grid * kBlock * s->ovf_stride * sizeof(int);
    if (slot.frames_cap < fbytes) {
        // (re)size every slot's buffer now, not each at its first use: a
        // frame pipeline then allocates once, in its first (warm-up) frame
        for (RenderSlot &r : s->slots) {
            if (r.frames_cap >= fbytes) continue;
            if (r.d_frames) (void)hipFree(r.d_frames);
            r.d_frames = nullptr;
            r.frames_cap = 0;
            if (hipMalloc(&r.d_frames, fbytes) != hipSuccess) return hipErrorOutOfMemory;
            r.frames_cap = fbytes;
        }
    }
    pl.frames = slot.d_frames;
    pl.ovf = reinterpret_cast<int *>(static_cast<char *>(slot.d_frames) + cold_bytes);
    s->last_blocks_per_cu = nb;
    s->last_grid = grid;
    s->last_lds = (long long)shm;
    s->last_mode = MODE;
    if (dry) return hipSuccess;                  // rt_scene_prepare: buffers only
    hipLaunchKernelGGL((render_kernel<MAXF, MODE>), dim3((unsigned)grid), dim3(kBlock), shm, st, pl);
    return hipGetLastError();
}

template <int MAXF>
hipError_t launch_mode(rt_scene *s, RenderSlot &slot, const Params &p, int mode, hipStream_t st, bool dry) {
    if (mode == MODE_BVH) return launch_one<MAXF, MODE_BVH>(s, slot, p, st, dry);
    if (mode == MODE_SCAN_LDS) return launch_one<MAXF, MODE_SCAN_LDS>(s, slot, p, st, dry);
    return launch_one<MAXF, MODE_SCAN>(s, slot, p, st, dry);
}

// Distance bound for the BVH padding: from any ray origin (the eye, or a point
// inside the scene's bounds) to any primitive.
double distance_bound(const rt_scene *s, const float eye[3]) {
    double diag2 = 0, far2 = 0, mag = 0;
    for (int k = 0; k < 3; k++) {
        double e = s->scene_hi[k] - s->scene_lo[k];
        diag2 += e * e;
        double a = std::fabs(eye[k] - s->scene_lo[k]), b = std::fabs(eye[k] - s->scene_hi[k]);
        far2 += std::max(a, b) * std::max(a, b);
        mag = std::max(mag, std::max(std::fabs((double)s->scene_lo[k]), std::fabs((double)s->scene_hi[k])));
        mag = std::max(mag, std::fabs((double)eye[k]));
    }
    return std::max(std::sqrt(diag2), std::sqrt(far2)) + mag + 1.0;
}

// Binary SAH tree over P, collapsed into 4-wide nodes (opt_bvh_collapse: 0
// greedy, largest child area first; 1 SAH-optimal) and renumbered breadth-first
// (the top levels first: cache locality of the hot nodes).
bool build_wide(rt_scene *s, std::vector<rtbvh::Prim> &P, rtbvh::Result &R, rtbvh::Result4 &Q) {
    rtbvh::Builder B(P);
    B.max_leaf = s->opt_bvh_collapse ? 1 : (int)s->opt_bvh_leaf;
    B.trav_cost = (float)s->opt_bvh_trav / 1000.0f;
    if (!B.build(R) || R.nodes.empty()) return false;
    if (s->opt_bvh_collapse)
        rtbvh::collapse_sah<4>(R, Q, (int)s->opt_bvh_leaf, (float)s->opt_bvh_node / 1000.0f);
    else
        rtbvh::collapse<4>(R, Q);
    rtbvh::bfs_order(Q);
    return true;
}

// Shadow-cone tree of a directional light (Params::dirk, dir_bf == 2).
//
// The reference's directional shadow ray runs TraceRay with the light's
// UNNORMALISED direction d = -dir (main.cpp:895), and the sphere test
// assumes |d| = 1 (main.cpp:1225-1258).  With s = |d|, n = d / s, k = s^2 - 1,
// h = n.(c - o) (how far the centre is ahead of the origin along the ray) and
// l = the lateral distance of c from the ray's line, the discriminant is
//     det / 4 = (d.w)^2 - |w|^2 + r^2 = k h^2 - l^2 + r^2,
// and the sphere shadows o iff det >= 0 and its far root (-B + sqrt det) / 2
// exceeds epsilon: for h < 0 that needs o inside the sphere; for h >= 0 it is
// l^2 <= r^2 + k h^2 -- a cylinder (s = 1), a cone widening away from the
// light (s > 1) or a bounded cap (s < 1).  It is NOT a ray-geometry
// question, so the ray BVH cannot cull it.  Here the spheres get a tree of
// their own, built in the frame whose z axis is n (rows of R: u1, u2, n) over
// boxes c' +- r_e, and a shadow ray becomes a cone query from R o (device:
// bvh_trace<true>): a child is entered iff its top is not below the origin
// (tz >= 0), its lateral distance d from the origin satisfies
// d^2 <= max(0, k) tz^2, and for s < 1 its bottom is within
// r_e / sqrt(1 - s^2).  Every candidate is then tested with the exact
// reference arithmetic; the tree only decides which spheres are tested.
// Conservative margins: the computed discriminant's error, up to ~2^-21
// (1 + s^2) D^2, grows r^2 by 2^-18 (1 + s^2) D^2 (r_e), boxes grow by 2^-16 D,
// k is rounded up.  Returns false if the direction or the geometry is not
// finite, or the scene is so large that one ulp of B reaches epsilon (then
// the h < 0 side is no longer safe): the caller falls back to the scan.
bool dir_tree(rt_scene *s, const LightK &lt, double D, std::vector<rtbvh::Node4H> &nodes, std::vector<float4> &rec,
              DirK &out, int &max_stack) {
    for (int k = 0; k < 9; k++) out.R[k] = (k % 4 == 0) ? 1.0f : 0.0f;
    out.root = -1;
    out.cone_k = 0.0f;
    out.cone_h = INFINITY;
    const double dx = lt.sdir[0], dy = lt.sdir[1], dz = lt.sdir[2];
    const double sl = std::sqrt(dx * dx + dy * dy + dz * dz);
    if (!std::isfinite(sl) || !(sl > 0.0)) return false;
    if (std::ldexp(2.0 * sl * D, -23) >= 0.5 * (double)s->base.eps) return false;
    const double n[3] = {dx / sl, dy / sl, dz / sl};
    // u1 perpendicular to n (cross with the axis least aligned with n), u2 = n x u1
    int ax = 0;
    for (int k = 1; k < 3; k++)
        if (std::fabs(n[k]) < std::fabs(n[ax])) ax = k;
    double e[3] = {0, 0, 0};
    e[ax] = 1.0;
    double u1[3] = {n[1] * e[2] - n[2] * e[1], n[2] * e[0] - n[0] * e[2], n[0] * e[1] - n[1] * e[0]};
    const double l1 = std::sqrt(u1[0] * u1[0] + u1[1] * u1[1] + u1[2] * u1[2]);
    for (double &v : u1) v /= l1;
    const double u2[3] = {n[1] * u1[2] - n[2] * u1[1], n[2] * u1[0] - n[0] * u1[2], n[0] * u1[1] - n[1] * u1[0]};
    for (int k = 0; k < 3; k++) {
        out.R[k] = (float)u1[k];
        out.R[3 + k] = (float)u2[k];
        out.R[6 + k] = (float)n[k];
    }
    // the device rotates with the float R: boxes are computed with it too
    // (its rounding of R o, ~2^-22 D, is far inside the 2^-16 D margins)
    double R[9];
    for (int k = 0; k < 9; k++) R[k] = out.R[k];
    const double pad = std::ldexp(D, -16);
    const double s2 = sl * sl;
    std::vector<rtbvh::Prim> P;
    double re_max = 0.0;
    for (const auto &src : s->prims) {
        if (!src.sphere) continue;
        const double c[3] = {src.c[0], src.c[1], src.c[2]};
        const double r = std::fabs((double)src.r);
        if (!std::isfinite(c[0]) || !std::isfinite(c[1]) || !std::isfinite(c[2]) || !std::isfinite(r)) return false;
        const double re = std::sqrt(r * r + std::ldexp((1.0 + s2) * D * D, -18)) + 2.0 * pad;
        re_max = std::max(re_max, re);
        rtbvh::Prim q;
        q.key = src.key;
        q.cost = 1.0f;
        for (int k = 0; k < 3; k++) {
            const double cr = R[3 * k] * c[0] + R[3 * k + 1] * c[1] + R[3 * k + 2] * c[2];
            q.box.lo[k] = std::nextafter((float)(cr - re), -INFINITY);
            q.box.hi[k] = std::nextafter((float)(cr + re), INFINITY);
            q.c[k] = (float)cr;
        }
        P.push_back(q);
    }
    if (P.empty()) return true;                          // root -1: no sphere can shadow
    out.cone_k = std::nextafter((float)(std::max(0.0, s2 - 1.0) * (1.0 + std::ldexp(1.0, -16))), INFINITY);
    if (s2 < 1.0) out.cone_h = std::nextafter((float)(re_max / std::sqrt(1.0 - s2) + pad), INFINITY);
    rtbvh::Result Rb;
    rtbvh::Result4 Q;
    if (!build_wide(s, P, Rb, Q) || Q.max_stack > kStackMax) return false;
    max_stack = Q.max_stack;
    const int nf = s->base.nf;
    bool ok = rtbvh::leaf_records(
        Q, Rb.keys, [](int32_t) { return false; },
        [&](int32_t k) {
            float kb;
            memcpy(&kb, &k, sizeof kb);
            rec.push_back(s->h_sscan[k - nf]);
            rec.push_back(make_float4(kb, s->h_ofac[k], 0.0f, 0.0f));
            return 2;
        },
        rec.size());
    std::vector<rtbvh::Node4H> QQ;
    if (!ok || !rtbvh::quantize(Q, QQ)) return false;
    const int base = (int)nodes.size();
    for (auto &z : QQ) {
        for (auto &l : z.link) {
            if (l == rtbvh::kEmpty) l = rtbvh::kEmptyLeaf;
            else if (l >= 0) l += base;
        }
        nodes.push_back(z);
    }
    out.root = base;
    return true;
}

// (Re)build the BVH with boxes padded for distance bound D (see rt_bvh.h):
//   face   pad = 2^-16 * D * max(1, cond)                 (32x the rounding bound)
//   sphere radius' = sqrt(r^2 + 2^-18 D^2) + 2^-16 D     (discriminant error)
int build_bvh(rt_scene *s, double D) {
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<rtbvh::Prim> P(s->prims.size());
    for (size_t i = 0; i < P.size(); i++) {
        const auto &src = s->prims[i];
        rtbvh::Prim &q = P[i];
        q.key = src.key;
        if (!src.sphere) {
            double pad = std::ldexp(D, -16) * std::max(1.0, src.cond);
            for (int k = 0; k < 3; k++) {
                q.box.lo[k] = (float)(src.lo[k] - pad);
                q.box.hi[k] = (float)(src.hi[k] + pad);
                q.c[k] = 0.5f * (src.lo[k] + src.hi[k]);
            }
            q.cost = 3.0f;
        } else {
            double r = std::fabs((double)src.r);
            double rr = std::sqrt(r * r + std::ldexp(D * D, -18)) + std::ldexp(D, -16);
            for (int k = 0; k < 3; k++) {
                q.box.lo[k] = (float)(src.c[k] - rr);
                q.box.hi[k] = (float)(src.c[k] + rr);
                q.c[k] = src.c[k];
            }
            q.cost = 1.0f;
        }
        // float rounding of the padded box must not shrink it
        for (int k = 0; k < 3; k++) {
            q.box.lo[k] = std::nextafter(q.box.lo[k], -INFINITY);
            q.box.hi[k] = std::nextafter(q.box.hi[k], INFINITY);
            if (!std::isfinite(q.box.lo[k]) || !std::isfinite(q.box.hi[k])) {
                q.box.lo[k] = -INFINITY;   // NaN/inf geometry: a box every ray enters
                q.box.hi[k] = INFINITY;
            }
        }
    }
    rtbvh::Result R;
    rtbvh::Result4 Q;
    bool ok = P.empty() || build_wide(s, P, R, Q);
    // leaf records: face = its 5 scan words with (key, shadow factor) in the
    // last one's y, z; sphere = (centre, r), (key, shadow factor, 0, 0)
    std::vector<float4> rec;
    const int nf = s->base.nf;
    if (ok && !Q.nodes.empty())
        ok = rtbvh::leaf_records(Q, R.keys, [nf](int32_t k) { return k < nf; }, [&](int32_t k) {
            float kb;
            memcpy(&kb, &k, sizeof kb);
            float fac = s->h_ofac[k];
            if (k < nf) {
                for (int j = 0; j < 5; j++) rec.push_back(s->h_fscan[5 * (size_t)k + j]);
                rec.back().y = kb;
                rec.back().z = fac;
                return 5;
            }
            rec.push_back(s->h_sscan[k - nf]);
            rec.push_back(make_float4(kb, fac, 0.0f, 0.0f));
            return 2;
        });
    rec.resize(rec.size() + 3, make_float4(0.0f, 0.0f, 0.0f, 0.0f));   // 5-word reads of a last sphere
    std::vector<rtbvh::Node4H> QQ;
    if (ok && !Q.nodes.empty() && !rtbvh::quantize(Q, QQ)) ok = false;     // non-finite geometry: scan
    for (auto &z : QQ)                                  // device form: unused slot -> the empty leaf
        for (auto &l : z.link)
            if (l == rtbvh::kEmpty) l = rtbvh::kEmptyLeaf;
    // the spill area is sized for the deepest tree (kStackMax: far beyond any
    // tree the builder's depth cap allows)
    ok = ok && !Q.nodes.empty() && Q.max_stack <= kStackMax;
    // directional lights in a scene with spheres: shadow-region trees, after
    // the main tree in the same node and record arrays
    std::vector<DirK> dirk(s->h_lights.size());
    int dir_mode = 0;
    int stack_all = Q.max_stack;                 // deepest stack over the main and the cone trees
    if (ok && s->base.ns > 0) {
        rec.resize(rec.size() - 3);                  // the 3 padding words go after the last tree
        for (size_t l = 0; l < s->h_lights.size(); l++) {
            if (s->h_lights[l].w != 0.0f) continue;
            if (dir_mode == 0) dir_mode = 2;
            int st = 0;
            if (!dir_tree(s, s->h_lights[l], D, QQ, rec, dirk[l], st)) dir_mode = 1;
            stack_all = std::max(stack_all, st);
        }
        rec.resize(rec.size() + 3, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
        if ((rec.size() >> 8) >= (1u << 23) - 2) ok = false;
    }
    // The old tree stays valid until the new one is on the device: upload into
    // new buffers first, then swap (a failed rebuild leaves no dangling
    // pointers and no tree marked valid that is not there).
    float4 *nb = nullptr, *nr = nullptr;
    DirK *nd = nullptr;
    int rc = RT_OK;
    if (ok && s->opt_fail_bvh_upload) {        // test hook: as if the device allocation failed
        rc = RT_E_NOMEM;
        ok = false;
    }
    if (ok) {
        const size_t node_bytes = QQ.size() * sizeof(QQ[0]);
        const size_t dir_bytes = std::max<size_t>(1, dirk.size()) * sizeof(DirK);
        if (hipMalloc(&nb, node_bytes) != hipSuccess ||
            hipMalloc(&nr, std::max<size_t>(1, rec.size()) * sizeof(float4)) != hipSuccess ||
            hipMalloc(&nd, dir_bytes) != hipSuccess)
            rc = RT_E_NOMEM;
        else if (hipMemcpy(nb, QQ.data(), node_bytes, hipMemcpyHostToDevice) != hipSuccess ||
                 hipMemcpy(nr, rec.data(), rec.size() * sizeof(float4), hipMemcpyHostToDevice) != hipSuccess ||
                 (!dirk.empty() && hipMemcpy(nd, dirk.data(), dirk.size() * sizeof(DirK), hipMemcpyHostToDevice) !=
                                       hipSuccess))
            rc = RT_E_HIP;
        if (rc) {
            if (nb) (void)hipFree(nb);
            if (nr) (void)hipFree(nr);
            if (nd) (void)hipFree(nd);
            nb = nr = nullptr;
            nd = nullptr;
        }
    }
    // renders still queued may read the old tree: free it after they finish
    if (s->d_bvh || s->d_leafrec || s->d_dirk) {
        (void)hipDeviceSynchronize();
        if (s->d_bvh) (void)hipFree(s->d_bvh);
        if (s->d_leafrec) (void)hipFree(s->d_leafrec);
        if (s->d_dirk) (void)hipFree(s->d_dirk);
    }
    s->d_bvh = nb;
    s->d_leafrec = nr;
    s->d_dirk = nd;
    s->base.bvh = nb;
    s->base.leafrec = nr;
    s->base.dirk = nd;
    s->base.dir_bf = dir_mode;
    s->bvh_ok = ok && rc == RT_OK;
    s->bvh_D = rc == RT_OK ? D : -1.0;   // a failed upload is retried; an unusable tree (scan) is not
    s->bvh_depth = s->bvh_ok ? Q.depth : 0;
    s->bvh_stack = s->bvh_ok ? Q.max_stack : 0;
    // spill area per lane: every block of kSpill entries a stack can push out
    s->ovf_stride = s->bvh_ok ? (stack_all / kSpill + 1) * kSpill : kSpill;
    s->bvh_nodes = s->bvh_ok ? (long long)Q.nodes.size() : 0;
    s->bvh_build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

int launch(rt_scene *s, RenderSlot &slot, Params &p, hipStream_t st, bool dry = false) {
    int depth = p.depth < 0 ? 0 : p.depth;
    if (depth > 16) return RT_E_UNSUPPORTED;
    int nobj = p.nf + p.ns;
    bool bvh = s->opt_accel == 1 || (s->opt_accel == -1 && nobj > 32);
    int mode = MODE_SCAN;
    if (bvh) {
        double D = distance_bound(s, p.eye);
        if (D > s->bvh_D) {
            int rc = build_bvh(s, std::max(D, 1.5 * s->bvh_D));
            if (rc) return rc;
        }
        if (s->bvh_ok) {
            mode = MODE_BVH;
            p.bvh = s->base.bvh;
            p.leafrec = s->base.leafrec;
            p.dirk = s->base.dirk;
            p.dir_bf = s->base.dir_bf;
            p.ovf_stride = s->ovf_stride;
        }
    }
    if (mode == MODE_SCAN) {
        bool lds = s->opt_lds == 1 || (s->opt_lds == -1 && s->lds_bytes <= 64 * 1024);
        if (s->lds_bytes > 64 * 1024) lds = false;
        if (lds) mode = MODE_SCAN_LDS;
    }
    hipError_t e;
    if (depth <= 4) e = launch_mode<5>(s, slot, p, mode, st, dry);
    else if (depth <= 8) e = launch_mode<9>(s, slot, p, mode, st, dry);
    else e = launch_mode<17>(s, slot, p, mode, st, dry);
    return e == hipSuccess ? RT_OK : RT_E_HIP;
}

void free_slot(RenderSlot &r) {
    if (r.stream) (void)hipStreamSynchronize(r.stream);
    if (r.work) (void)hipFree(r.work);
    if (r.stats) (void)hipFree(r.stats);
    if (r.d_frames) (void)hipFree(r.d_frames);
    if (r.ev_in) (void)hipEventDestroy(r.ev_in);
    if (r.ev0) (void)hipEventDestroy(r.ev0);
    if (r.ev1) (void)hipEventDestroy(r.ev1);
    if (r.stream) (void)hipStreamDestroy(r.stream);
    r = RenderSlot{};
}

// own_stream: slots of a scene with more than one render in flight get a
// stream of their own, at the highest priority: HIP keeps a separate hardware
// queue pool per priority, so the slot's dispatches never queue behind barrier
// packets of caller (or collective) streams that share a hardware queue.
int init_slot(RenderSlot &r, bool own_stream) {
    if (hipMalloc(&r.work, sizeof(unsigned)) != hipSuccess) return RT_E_NOMEM;
    if (hipMalloc(&r.stats, kNStats * sizeof(unsigned long long)) != hipSuccess) return RT_E_NOMEM;
    if (hipEventCreate(&r.ev0) != hipSuccess || hipEventCreate(&r.ev1) != hipSuccess ||
        hipEventCreateWithFlags(&r.ev_in, hipEventDisableTiming) != hipSuccess)
        return RT_E_HIP;
    if (own_stream) {
        int lo = 0, hi = 0;
        if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) return RT_E_HIP;
        if (hipStreamCreateWithPriority(&r.stream, hipStreamNonBlocking, hi) != hipSuccess) return RT_E_HIP;
    }
    return RT_OK;
}

int set_inflight(rt_scene *s, long long n) {
    if (n < 1 || n > 4) return RT_E_INVALID;
    if ((size_t)n == s->slots.size()) return RT_OK;
    if (hipSetDevice(s->device) != hipSuccess) return RT_E_HIP;
    for (auto &r : s->slots) free_slot(r);
    s->slots.assign((size_t)n, RenderSlot{});
    s->next_slot = s->last_slot = 0;
    s->last_valid = false;
    for (auto &r : s->slots) {
        int rc = init_slot(r, n > 1);
        if (rc) return rc;
        // HIP binds a stream to a hardware queue at its first command: do it
        // here, not in the first frame that uses the slot
        if (r.stream && (hipMemsetAsync(r.work, 0, sizeof(unsigned), r.stream) != hipSuccess ||
                         hipStreamSynchronize(r.stream) != hipSuccess))
            return RT_E_HIP;
    }
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char *rt_strerror(int code) {
    int i = -code;
    if (i < 0 || i > 5) return "unknown error";
    return kErr[i];
}

int rt_scene_create(int device, const rt_scene_desc *desc, rt_scene **out) {
    if (!desc || !out) return RT_E_INVALID;
    *out = nullptr;
    if (desc->n_spheres < 0 || desc->n_faces < 0 || desc->n_lights < 0 || desc->n_textures < 0) return RT_E_INVALID;
    if ((desc->n_spheres && !desc->spheres) || (desc->n_faces && !desc->faces) ||
        (desc->n_lights && !desc->lights) || (desc->n_textures && !desc->textures))
        return RT_E_INVALID;
    for (int i = 0; i < desc->n_spheres; i++)
        if (desc->spheres[i].texture >= desc->n_textures) return RT_E_INVALID;
    for (int i = 0; i < desc->n_faces; i++)
        if (desc->faces[i].texture >= desc->n_textures) return RT_E_INVALID;
    for (int i = 0; i < desc->n_textures; i++)
        if (desc->textures[i].width <= 0 || desc->textures[i].height <= 0 || !desc->textures[i].rgb)
            return RT_E_INVALID;
    int ndev = rt_device_count();
    if (device < 0 || device >= ndev) return RT_E_NODEVICE;
    if (hipSetDevice(device) != hipSuccess) return RT_E_HIP;

    auto *s = new rt_scene();
    s->device = device;
    const int nf = desc->n_faces, ns = desc->n_spheres, nobj = nf + ns;

    // --- faces: exact per-face invariants (TraceRay recomputes these per call)
    std::vector<float4> fscan((size_t)nf * 5);
    std::vector<FaceShadeK> fsh((size_t)nf);
    std::vector<ObjK> objs((size_t)nobj);
    std::vector<float> ofac((size_t)nobj);
    auto fill_obj = [&](int k, const rt_material &m, int tex, int is_sphere) {
        ObjK &o = objs[k];
        for (int c = 0; c < 3; c++) o.dif[c] = m.diffuse[c], o.spc[c] = m.specular[c];
        o.ka = m.ka, o.kd = m.kd, o.ks = m.ks, o.n = m.n, o.opacity = m.opacity, o.eta = m.eta;
        o.tex = tex;
        o.is_sphere = is_sphere;
        ofac[k] = (float)(1.0 - (double)m.opacity);
        if (m.ks > 0.0f || (m.opacity < 1.0f && m.eta > 0.0f)) s->secondary = true;
    };
    for (int i = 0; i < nf; i++) {
        const rt_face_desc &F = desc->faces[i];
        V3 v0 = f3(F.v[0]), v1 = f3(F.v[1]), v2 = f3(F.v[2]);
        V3 e1 = vsub(v1, v0), e2 = vsub(v2, v0);
        V3 n = vnorm(vcross(e1, e2));                         // main.cpp:537-539
        float D = -vdot(n, v0);
        float d11 = vdot(e1, e1), d12 = vdot(e1, e2), d22 = vdot(e2, e2);
        float det = (d11 * d22 - d12 * d12);
        fscan[5 * i + 0] = make_float4(v0.x, v0.y, v0.z, D);
        fscan[5 * i + 1] = make_float4(n.x, n.y, n.z, det);
        fscan[5 * i + 2] = make_float4(e1.x, e1.y, e1.z, d11);
        fscan[5 * i + 3] = make_float4(e2.x, e2.y, e2.z, d22);
        fscan[5 * i + 4] = make_float4(d12, 0.0f, 0.0f, 0.0f);
        FaceShadeK &fs = fsh[i];
        for (int k = 0; k < 3; k++) {
            V3 vn = vnorm(f3(F.vn[k]));
            fs.vn[k][0] = vn.x, fs.vn[k][1] = vn.y, fs.vn[k][2] = vn.z;
            for (int c = 0; c < 2; c++) {
                float t = F.vt[k][c];
                fs.vt[k][c] = (t < 0.0f) ? 0.0f : ((1.0f < t) ? 1.0f : t);
            }
        }
        fs.smooth = F.smooth;
        fill_obj(i, F.mat, F.texture, 0);
    }
    // BVH sources (padding is applied per build, it depends on the eye)
    s->prims.reserve((size_t)nobj);
    for (int i = 0; i < nf; i++) {
        rt_scene::PrimSrc ps{};
        ps.key = i;
        ps.sphere = false;
        const rt_face_desc &F = desc->faces[i];
        for (int k = 0; k < 3; k++) {
            ps.lo[k] = std::min(F.v[0][k], std::min(F.v[1][k], F.v[2][k]));
            ps.hi[k] = std::max(F.v[0][k], std::max(F.v[1][k], F.v[2][k]));
        }
        float4 a = fscan[5 * i + 1], b2 = fscan[5 * i + 2], c2 = fscan[5 * i + 3];
        double det = a.w, d11 = b2.w, d22 = c2.w;
        ps.cond = det > 0 ? d11 * d22 / det : 1e30;
        s->prims.push_back(ps);
    }
    std::vector<float4> sscan((size_t)ns);
    for (int i = 0; i < ns; i++) {
        const rt_sphere_desc &S = desc->spheres[i];
        sscan[i] = make_float4(S.center[0], S.center[1], S.center[2], S.radius);
        fill_obj(nf + i, S.mat, S.texture, 1);
        rt_scene::PrimSrc ps{};
        ps.key = nf + i;
        ps.sphere = true;
        for (int k = 0; k < 3; k++) {
            ps.c[k] = S.center[k];
            ps.lo[k] = S.center[k] - std::fabs(S.radius);
            ps.hi[k] = S.center[k] + std::fabs(S.radius);
        }
        ps.r = S.radius;
        s->prims.push_back(ps);
    }
    for (int k = 0; k < 3; k++) s->scene_lo[k] = INFINITY, s->scene_hi[k] = -INFINITY;
    for (const auto &ps : s->prims)
        for (int k = 0; k < 3; k++) {
            if (std::isfinite(ps.lo[k])) s->scene_lo[k] = std::min(s->scene_lo[k], ps.lo[k]);
            if (std::isfinite(ps.hi[k])) s->scene_hi[k] = std::max(s->scene_hi[k], ps.hi[k]);
        }
    for (int k = 0; k < 3; k++)
        if (!(s->scene_lo[k] <= s->scene_hi[k])) s->scene_lo[k] = s->scene_hi[k] = 0.0f;
    bool nan_fac = false;
    for (float f : ofac) nan_fac |= std::isnan(f);
    s->h_fscan = fscan;
    s->h_sscan = sscan;
    s->h_ofac = ofac;
    s->h_lights.clear();
    std::vector<LightK> lights((size_t)desc->n_lights);
    for (int i = 0; i < desc->n_lights; i++) {
        const rt_light_desc &L = desc->lights[i];
        LightK &k = lights[i];
        memset(&k, 0, sizeof k);
        for (int c = 0; c < 3; c++) k.xyz[c] = L.xyz[c], k.col[c] = L.color[c];
        k.w = L.w;
        V3 dir = f3(L.xyz);
        V3 Ld = vmul(vnorm(dir), -1.0f);
        V3 sd = vmul(dir, -1.0f);
        k.L[0] = Ld.x, k.L[1] = Ld.y, k.L[2] = Ld.z;
        k.sdir[0] = sd.x, k.sdir[1] = sd.y, k.sdir[2] = sd.z;
    }
    s->h_lights = lights;
    std::vector<TexK> texs((size_t)desc->n_textures);

    int rc = RT_OK;
    Params &p = s->base;
    if (!rc) rc = upload(s, fscan, p.fscan);
    if (!rc) rc = upload(s, sscan, p.sscan);
    if (!rc) rc = upload(s, ofac, p.ofac);
    if (!rc) rc = upload(s, objs, p.objs);
    if (!rc) rc = upload(s, fsh, p.fsh);
    if (!rc) rc = upload(s, lights, p.lights);
    std::vector<unsigned char> texels;
    for (int i = 0; i < desc->n_textures; i++) {
        const rt_texture_desc &T = desc->textures[i];
        texs[i].w = T.width, texs[i].h = T.height, texs[i].off = (long long)texels.size();
        texels.insert(texels.end(), T.rgb, T.rgb + (size_t)T.width * T.height * 3);
    }
    if (!rc) rc = upload(s, texels, p.texels);
    if (!rc) rc = upload(s, texs, p.texs);
    if (!rc && hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) rc = RT_E_HIP;
    if (!rc) {
        s->slots.assign(1, RenderSlot{});
        rc = init_slot(s->slots[0], false);
    }
    if (!rc) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) != hipSuccess) rc = RT_E_HIP;
        else s->num_cu = prop.multiProcessorCount;
    }
    if (rc) {
        rt_scene_destroy(s);
        return rc;
    }
    p.nf = nf;
    p.ns = ns;
    p.nl = desc->n_lights;
    for (int c = 0; c < 3; c++) p.bkg[c] = desc->bkg[c];
    p.eta_bkg = desc->eta_bkg;
    p.eps = desc->epsilon;
    p.depth = desc->depth;
    p.dir_bf = 0;                      // set with the BVH (build_bvh); the scan needs none
    p.shadow_early_out = nan_fac ? 0 : 1;
    p.stack_cap = kLdsStackDefault;
    p.chunk = 0;                       // launch_one: chunk_for, refill_for
    p.refill_min = 1;
    p.gate_x = kGateX;
    s->lds_bytes = (size_t)(5 * nf + ns) * sizeof(float4);
    *out = s;
    return RT_OK;
}

int rt_scene_destroy(rt_scene *s) {
    if (!s) return RT_OK;
    (void)hipSetDevice(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    for (auto &r : s->slots)           // renders still running on caller or slot streams
        if (r.ev1) (void)hipEventSynchronize(r.ev1);
    for (void *d : s->allocs) (void)hipFree(d);

    if (s->d_bvh) (void)hipFree(s->d_bvh);
    if (s->d_leafrec) (void)hipFree(s->d_leafrec);
    if (s->d_dirk) (void)hipFree(s->d_dirk);
    if (s->dev_out) (void)hipFree(s->dev_out);
    for (auto &r : s->slots) free_slot(r);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
    return RT_OK;
}

int rt_scene_set_option(rt_scene *s, const char *key, long long value) {
    if (!s || !key) return RT_E_INVALID;
    std::string k(key);
    if (k == "lds") s->opt_lds = value;
    else if (k == "grid") s->opt_grid = value;
    else if (k == "reserve") s->opt_reserve = std::max(0LL, value);
    else if (k == "depth") s->base.depth = (int)value;
    else if (k == "accel") s->opt_accel = value;
    else if (k == "inflight") return set_inflight(s, value);
    else if (k == "fail_bvh_upload") s->opt_fail_bvh_upload = value;
    else if (k == "gate_x") {
        if (value < 0 || value > 64) return RT_E_INVALID;
        s->base.gate_x = (unsigned)value;
    }
    else if (k == "refill_min") {
        if (value < 1 || value > 64) return RT_E_INVALID;
        s->opt_refill_min = value;
    }
    else if (k == "chunk") {
        if (value < 0 || value > 4096) return RT_E_INVALID;
        s->opt_chunk = value;
    }
    else if (k == "lds_stack") {
        if (value < 12 || value > kLdsStack) return RT_E_INVALID;
        s->base.stack_cap = (int)value;
    }
    else if (k == "bvh_leaf" || k == "bvh_trav" || k == "bvh_collapse" || k == "bvh_node") {
        if (k == "bvh_leaf") s->opt_bvh_leaf = std::max(1LL, std::min(15LL, value));
        else if (k == "bvh_trav") s->opt_bvh_trav = std::max(0LL, value);
        else if (k == "bvh_collapse") s->opt_bvh_collapse = value != 0;
        else s->opt_bvh_node = std::max(0LL, value);
        s->bvh_D = -1.0;               // rebuild on the next render
    }
    else return RT_E_INVALID;
    return RT_OK;
}

int rt_render_row_blocks_async(rt_scene *s, const rt_camera *cam, int W, int H, int y0, int block, int step,
                               int nrows, float *out_rgb, void *hip_stream) {
    if (!s || !cam || !out_rgb || W < 2 || H < 2 || y0 < 0 || block < 1 || step < block || nrows < 1)
        return RT_E_INVALID;
    long long last = (long long)y0 + (long long)((nrows - 1) / block) * step + (nrows - 1) % block;
    if (last >= H) return RT_E_INVALID;
    if ((long long)W * nrows >= (1ll << 31)) return RT_E_UNSUPPORTED;
    if (hipSetDevice(s->device) != hipSuccess) return RT_E_HIP;
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : s->stream;
    Params p = s->base;
    for (int c = 0; c < 3; c++) {
        p.eye[c] = cam->eye[c];
        p.ul[c] = cam->ul[c];
        p.dh[c] = cam->dh[c];
        p.dv[c] = cam->dv[c];
    }
    p.W = W;
    p.y0 = y0;
    p.rows = nrows;
    p.rblock = block;
    p.rstep = step;
    p.total = (unsigned)((long long)W * nrows);
    p.out = out_rgb;
    RenderSlot &slot = s->slots[(size_t)s->next_slot];
    s->last_slot = s->next_slot;
    s->next_slot = (s->next_slot + 1) % (int)s->slots.size();
    hipStream_t caller = st;
    if (slot.stream) {                 // several in flight: run on the slot's stream
        if (hipEventRecord(slot.ev_in, caller) != hipSuccess) return RT_E_HIP;
        if (hipStreamWaitEvent(slot.stream, slot.ev_in, 0) != hipSuccess) return RT_E_HIP;
        st = slot.stream;
    } else if (slot.used && hipStreamWaitEvent(st, slot.ev1, 0) != hipSuccess) {
        // one slot, any caller stream: this render reuses the slot's work
        // counter, counters and frames, so it waits for the slot's previous
        // render (issued on whatever stream) before touching them
        return RT_E_HIP;
    }
    p.work = slot.work;
    p.stats = slot.stats;
    if (hipMemsetAsync(slot.work, 0, sizeof(unsigned), st) != hipSuccess) return RT_E_HIP;
    if (hipMemsetAsync(slot.stats, 0, kNStats * sizeof(unsigned long long), st) != hipSuccess) return RT_E_HIP;
    // timeline minima start at all-ones
    if (hipMemsetAsync(slot.stats + 24, 0xff, 2 * sizeof(unsigned long long), st) != hipSuccess) return RT_E_HIP;
    (void)hipEventRecord(slot.ev0, st);
    int rc = launch(s, slot, p, st);
    (void)hipEventRecord(slot.ev1, st);
    slot.used = true;
    if (slot.stream && hipStreamWaitEvent(caller, slot.ev1, 0) != hipSuccess) return RT_E_HIP;
    s->last_valid = rc == RT_OK;
    return rc;
}

int rt_deinterleave_rows(const float *gathered, int world, int rows_per, int W, int H, int block, float *image,
                         void *hip_stream) {
    if (!gathered || !image || world < 1 || rows_per < 1 || W < 1 || H < 1 || block < 1) return RT_E_INVALID;
    if (H > 65535) return RT_E_UNSUPPORTED;
    // every image row's source row must exist: each rank's row count <= rows_per
    const int nblocks = (H + block - 1) / block;
    for (int r = 0; r < world; r++) {
        int rows = 0;
        for (int b = r; b < nblocks; b += world) rows += std::min(block, H - b * block);
        if (rows > rows_per) return RT_E_INVALID;
    }
    const unsigned gx = (unsigned)std::min<size_t>(64, ((size_t)W * 3 + 255) / 256);
    hipLaunchKernelGGL(deinterleave_kernel, dim3(gx, (unsigned)H), dim3(256), 0, (hipStream_t)hip_stream, gathered,
                       world, rows_per, W, H, block, image);
    return hipGetLastError() == hipSuccess ? RT_OK : RT_E_HIP;
}

int rt_scene_prepare(rt_scene *s, const rt_camera *cam, int W, int H) {
    if (!s || !cam || W < 2 || H < 2) return RT_E_INVALID;
    if ((long long)W * H >= (1ll << 31)) return RT_E_UNSUPPORTED;
    if (hipSetDevice(s->device) != hipSuccess) return RT_E_HIP;
    Params p = s->base;
    for (int c = 0; c < 3; c++) {
        p.eye[c] = cam->eye[c];
        p.ul[c] = cam->ul[c];
        p.dh[c] = cam->dh[c];
        p.dv[c] = cam->dv[c];
    }
    p.W = W;
    p.rows = H;
    p.total = (unsigned)((long long)W * H);
    int rc = launch(s, s->slots[0], p, s->stream, true);
    if (rc == RT_OK && hipDeviceSynchronize() != hipSuccess) rc = RT_E_HIP;
    return rc;
}

int rt_render_rows_async(rt_scene *s, const rt_camera *cam, int W, int H, int y0, int y1, float *out_rgb,
                         void *hip_stream) {
    if (y1 <= y0) return RT_E_INVALID;
    return rt_render_row_blocks_async(s, cam, W, H, y0, y1 - y0, y1 - y0, y1 - y0, out_rgb, hip_stream);
}

int rt_scene_last_stats(rt_scene *s, rt_stats *stats) {
    if (!s || !stats) return RT_E_INVALID;
    if (!s->last_valid) return RT_E_INVALID;
    if (hipSetDevice(s->device) != hipSuccess) return RT_E_HIP;
    const RenderSlot &slot = s->slots[(size_t)s->last_slot];
    if (hipEventSynchronize(slot.ev1) != hipSuccess) return RT_E_HIP;
    unsigned long long h[kNStats];
    if (hipMemcpy(h, slot.stats, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return RT_E_HIP;
    stats->primary = h[0];
    stats->shadow = h[1];
    stats->refraction = h[2];
    stats->reflection = h[3];
    stats->skip_trans = h[4];
    stats->ub_back = h[5];
    stats->box_tests = h[6];
    stats->face_tests = h[7];
    stats->sphere_tests = h[8];
    stats->shadow_known = h[32];
    stats->bf_queries = h[33];
    stats->stack_spills = h[34];
    stats->bvh_build_ms = s->bvh_build_ms;
    // device time of the launch: first wave start .. last wave end (100 MHz
    // clock); the events' interval also holds any wait for a previous frame
    // still on the CUs
    if (h[26] > h[24]) {
        stats->kernel_ms = (double)(h[26] - h[24]) * 1e-5;
    } else {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, slot.ev0, slot.ev1);
        stats->kernel_ms = ms;
    }
    return RT_OK;
}

int rt_scene_debug_counters(rt_scene *s, unsigned long long *out, int n) {
    if (!s || !out || n < 0 || n > kNStats || !s->last_valid) return RT_E_INVALID;
    if (hipSetDevice(s->device) != hipSuccess) return RT_E_HIP;
    const RenderSlot &slot = s->slots[(size_t)s->last_slot];
    if (hipEventSynchronize(slot.ev1) != hipSuccess) return RT_E_HIP;
    unsigned long long h[kNStats];
    if (hipMemcpy(h, slot.stats, kNStats * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess)
        return RT_E_HIP;
    h[16] = (unsigned long long)s->last_mode;
    h[17] = (unsigned long long)s->last_blocks_per_cu;
    h[18] = (unsigned long long)s->last_grid;
    h[19] = (unsigned long long)s->last_lds;
    h[20] = (unsigned long long)s->bvh_nodes;
    h[21] = (unsigned long long)s->bvh_depth;
    h[22] = (unsigned long long)s->bvh_stack;
    h[23] = (unsigned long long)s->num_cu;
    for (int i = 0; i < n; i++) out[i] = h[i];
    return RT_OK;
}

int rt_render_rows(rt_scene *s, const rt_camera *cam, int W, int H, int y0, int y1, float *out_rgb, rt_stats *stats) {
    if (!s || !cam || !out_rgb || W < 2 || H < 2 || y0 < 0 || y1 > H || y0 >= y1) return RT_E_INVALID;
    return rt_render_row_blocks(s, cam, W, H, y0, y1 - y0, y1 - y0, y1 - y0, out_rgb, stats);
}

int rt_render_row_blocks(rt_scene *s, const rt_camera *cam, int W, int H, int y0, int block, int step, int nrows,
                         float *out_rgb, rt_stats *stats) {
    if (!s || !cam || !out_rgb || nrows < 1) return RT_E_INVALID;
    if (hipSetDevice(s->device) != hipSuccess) return RT_E_HIP;
    hipPointerAttribute_t attr;
    bool on_device = false;
    if (hipPointerGetAttributes(&attr, out_rgb) == hipSuccess)
        on_device = attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
    else
        (void)hipGetLastError();
    size_t bytes = (size_t)W * (size_t)nrows * 3 * sizeof(float);
    float *dst = out_rgb;
    if (!on_device) {
        if (s->dev_out_bytes < bytes) {
            if (s->dev_out) (void)hipFree(s->dev_out);
            s->dev_out = nullptr;
            s->dev_out_bytes = 0;
            if (hipMalloc(&s->dev_out, bytes) != hipSuccess) return RT_E_NOMEM;
            s->dev_out_bytes = bytes;
        }
        dst = s->dev_out;
    }
    int rc = rt_render_row_blocks_async(s, cam, W, H, y0, block, step, nrows, dst, nullptr);
    if (rc) return rc;
    if (!on_device && hipMemcpyAsync(out_rgb, dst, bytes, hipMemcpyDeviceToHost, s->stream) != hipSuccess)
        return RT_E_HIP;
    if (hipStreamSynchronize(s->stream) != hipSuccess) return RT_E_HIP;
    if (stats) return rt_scene_last_stats(s, stats);
    return RT_OK;
}

}  // extern "C"

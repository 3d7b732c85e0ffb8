// rt_kernels.hip -- MI355X (gfx950) ray-trace kernel.
//
// Replaces the reference's hot path: the pixel loop main.cpp:718-764, TraceRay
// main.cpp:1215-1407 and ShadeRay main.cpp:783-1207 (called recursively).
// The host side (scene upload, render slots, the rt_hip.h C ABI) is
// rt_scene.cpp; the two share rt_device.h.
//
// Execution model:
//  * persistent workgroups; every lane owns one pixel at a time and walks
//    that pixel's ShadeRay tree as an explicit state machine: the node being
//    shaded lives in LDS, the parents' state in per-lane cold frames in HBM;
//    one TraceRay-equivalent search per loop iteration (BVH traversal, or a
//    brute-force scan for scenes of <= 32 objects);
//  * a lane that finishes its pixel waits until enough lanes of its wave are
//    idle; the wave ballots its idle lanes, one lane takes a block of pixel
//    indices with a single atomicAdd and each idle lane picks its own by a
//    prefix count of the ballot (mbcnt) -- wave-level ballot/prefix compaction
//    of the work; reflection / refraction searches are batched the same way;
//  * framebuffer: 12 B/pixel fp32 RGB stores (pre-quantisation colour).
//
// Numerics follow the reference operation by operation (built with
// -ffp-contract=off, correctly rounded div/sqrt, std::clamp-style compares,
// the reference's double-precision intermediates where they change the
// result); the documented relaxations are in DESIGN.md §5.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <type_traits>

#include "rt_bvh.h"
#include "rt_device.h"

namespace rt {

// Counters (rt_stats: rays by kind, known-zero shadow rays, brute-force
// queries, SKIP_TRANS and ub_back events, executed ray-box / face / sphere
// tests): only in the counting instantiation of the kernel
// (render_kernel<.., COUNT = true>, option counters, the default); in the
// other one they are compiled out -- their registers, live across the whole
// loop, cost the traversal ~4 %.  RT_COUNT(x) runs x where a
// counter object `cnt` of a counting type is in scope; RT_COUNT_IF(on, x)
// where the switch is a template parameter.
#define RT_COUNT_IF(on, x) \
    do {                   \
        if constexpr (on) { x; } \
    } while (0)
#define RT_COUNT(x) RT_COUNT_IF(std::remove_reference_t<decltype(cnt)>::kCount, x)

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


// Row i of a per-object array, addressed where it is read: the opaque index
// keeps LLVM from computing the 64-bit address once and holding it in a VGPR
// pair across the shading code (where it was spilled to scratch and reloaded
// every step); recomputing it is two VALU instructions.
template <typename T>
__device__ __forceinline__ const T &row(const T *base, int i) {
    asm volatile("" : "+v"(i));
    return base[i];
}

// ---------------------------------------------------------------------------
// One lane's ray query (a TraceRay call + the consumer loop that follows it)
// ---------------------------------------------------------------------------
//  closest : smallest t with tmin < t < running min, ties -> first in order
//            (main.cpp:732-742, :992-1011, :1113-1124); skipchk applies the
//            SKIP_TRANS rule (main.cpp:1000-1002) against object `back`
//  shadow  : every intersection of every object != self with tmin < t (and
//            t < tmax unless unbounded) multiplies mask by (1 - opacity)
//            (main.cpp:898-912, :930-949)
// The shadow mask (main.cpp:788) is grey: it starts at {1,1,1} and every
// occluder multiplies all three channels by the same factor (1 - opacity),
// so it is kept as one float.  A shadow query multiplies its own light's
// factors from 1 (q.mask); the cumulative mask of the node's earlier lights
// rides in q.back (as float bits: back is a SKIP_TRANS field, unused by shadow
// queries) and the light step multiplies the two (advance, PH_LIGHT): the
// same product as the reference's running one, reassociated (all factors in
// [0, 1]: relaxation 3 of DESIGN.md §5).  (Round 4 measured idle lanes
// tracing a node's next light in the same step on this representation: C3
// -3 %)
struct Query {
    V3 o, d;
    float tmin, tmax;
    int self, back, win;
    bool closest, unb, skipchk, skipped;
    bool bf;                              // BVH mode: this query needs the brute-force scan
    float mask;                           // shadow: product of this light's factors so far
};
__device__ __forceinline__ float prior_mask(const Query &q) { return __int_as_float(q.back); }

constexpr float kInf = __builtin_huge_valf();

__device__ __forceinline__ void offer(Query &q, float t, int obj, const float *__restrict__ ofac) {
    // (closest queries carry their origin object in q.self for the BVH's
    // origin-leaf pass, bvh_trace; they never exclude it)
    bool in = (t > q.tmin) & ((t < q.tmax) | q.unb) & (q.closest | (obj != q.self));
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
            q.mask = clamp01(f * q.mask);
            // an opaque occluder zeroes the mask for good: any-hit termination
            if (q.mask == 0.0f) q.tmin = kInf;
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
    // 0 < a, b, g < 1 as two compares of the NaN-propagating minimum / maximum
    // (gfx950 v_minimum3_f32 / v_maximum3_f32): a NaN fails both, as it fails
    // every one of the six compares; six compares joined by & were lowered to
    // ~20 bit operations on bytes
    const float mn = __builtin_elementwise_minimum(__builtin_elementwise_minimum(a, b), g);
    const float mx = __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), g);
    return (dem != 0.0f) && (mn > 0.0f) && (mx < 1.0f);
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
template <bool SRC_LDS, bool COUNT>
__device__ __forceinline__ void scan(Query &q, const Params &p, const float4 *lds_f, const float4 *lds_s,
                                     bool part, unsigned &ft, unsigned &st) {
    if (!part) return;
    RT_COUNT_IF(COUNT, ft += (unsigned)p.nf);
    RT_COUNT_IF(COUNT, st += (unsigned)p.ns);
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
// The reference's two order-dependent cases are answered on the BVH too
// (DESIGN.md §3.3): a SKIP_TRANS check is the stack top's own nearest root
// (own_nearest) plus an any-hit search (q.skipchk); a directional shadow ray
// tests the faces here and the spheres by a cone query in the light's
// shadow-region tree (bvh_trace<true>).  Only when such a tree could not be
// built (Params::dir_bf == 1) do directional shadow rays set q.bf and go to
// the brute-force scan.
// ---------------------------------------------------------------------------
// Per-lane counters kept small (VGPR pressure): ray kinds are counted per
// wave with ballots in the main loop (scalar registers); only the rare events
// and the executed-test counts stay per lane.
template <bool COUNT>
struct CountersT {
    static constexpr bool kCount = COUNT;
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
template <class CNT>
__device__ __forceinline__ float own_nearest(const Query &q, const Params &p, int obj, CNT &cnt) {
    float tb = kFltMax;
    if (obj < p.nf) {
        const float4 *F = p.fscan + 5 * obj;
        float t, a, b, g;
        RT_COUNT(cnt.ftests++);
        if (face_test(F[0], F[1], F[2], F[3], F[4], q.o, q.d, t, a, b, g) & (F[1].w != 0.0f) & (t > q.tmin) &
            (t < kFltMax))
            tb = t;
    } else {
        float t1, t2;
        RT_COUNT(cnt.stests++);
        if (sphere_test(p.sscan[obj - p.nf], q.o, q.d, t1, t2)) {
            if ((t1 > q.tmin) & (t1 < tb)) tb = t1;
            if ((t2 > q.tmin) & (t2 < tb)) tb = t2;
        }
    }
    return tb;
}


// Raw buffer resource over a device array (gfx9 dword3: 32-bit data format;
// the range is not used for bounds: every offset the kernel forms is in range)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buffer_rsrc(const void *base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, 0x7fffffff, 0x00020000);
}
// 16 bytes at byte offset off + imm (imm a constant: the instruction's offset field)
__device__ __forceinline__ f4v bldv(__amdgpu_buffer_rsrc_t r, int off, int imm) {
    return __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(r, off + imm, 0, 0));
}
__device__ __forceinline__ float4 bld4(__amdgpu_buffer_rsrc_t r, int off, int imm) { return f4(bldv(r, off, imm)); }

static_assert(sizeof(rtbvh::Node4H) == 104 && rtbvh::kNodeAxisOff == 16 && rtbvh::kNodeLinkOff == 88, "node layout");
// uniform float4 at a byte offset (4-byte aligned), via the scalar unit
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ float4 sld4b(const void *p, int off) {
    f4u v = *(const RT_CONST f4u *)((const RT_CONST char *)p + off);
    return make_float4(v.x, v.y, v.z, v.w);
}
typedef _Float16 h2v __attribute__((ext_vector_type(2)));   // two binary16 plane offsets
// while-while traversal: stop descending when at most this many lanes still
// look for a leaf (A/B, C3 Mrays/s: 0 -> 5912, 1 -> 5960, 2 -> 5957, 3 -> 5954,
// 6 -> 5924, 12 -> 5849; with one leaf per round: 0 -> 5885, 2 -> 6021,
// 5 -> 6031; profiles/r02/ab_leaf_*.txt).  Re-swept on round 6's final kernel
// (profiles/r06/leafwait/): the recursive depth <= 4 instantiation (C3) at 1
// instead of 2, C3 +0.3 / +0.4 % (0: -1.7 %); the one without recursion (C2,
// C4) at 0, C4 +0.8 %, C2 +0.8 % (1: +0.6 / +-0 %)
#ifndef RT_LEAF_WAIT
#define RT_LEAF_WAIT 1
#endif
#ifndef RT_LEAF_WAIT_FLAT
#define RT_LEAF_WAIT_FLAT 0
#endif
constexpr unsigned kLeafWait = RT_LEAF_WAIT;
#ifndef RT_LEAF_WAIT_CONE
#define RT_LEAF_WAIT_CONE 2                      // the directional cone pass
#endif
constexpr unsigned kLeafWaitCone = RT_LEAF_WAIT_CONE;
// The depth > 4 instantiation (MAXF 9/17: C5, depth 8, whose 100 000-sphere
// tree is 12 levels deep) keeps descending until 12 lanes lack a leaf: C5
// +2.2 % (2: C3 best, 8 there -1.2 %; a run-time threshold cost C3 1 %,
// profiles/r02/ab_leafwait_r2final.txt; round 6: 8 -0.35 %, 16 / 20 / 24 within
// +0.1 %)
#ifndef RT_LEAF_WAIT_DEEP
#define RT_LEAF_WAIT_DEEP 12
#endif
constexpr unsigned leaf_wait_for(int maxf) {
    return maxf > 5 ? (unsigned)RT_LEAF_WAIT_DEEP : maxf == 1 ? (unsigned)RT_LEAF_WAIT_FLAT : kLeafWait;
}
constexpr int kRefill = rtbvh::kEmpty + 1;       // LDS stack sentinel with blocks spilled (+ count - 1)

// 1/x for the slab planes: v_rcp_f32 (1 ulp; 1/+-0 = +-inf, capped by the
// caller).  The planes need no correctly rounded reciprocal: a relative error
// of 2^-23 in 1/d moves a plane distance by far less than the 2^-16 D
// padding of every primitive's box (one v_rcp instead of a ~10-instruction
// IEEE division per axis and trace)
__device__ __forceinline__ float safe_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

// One leaf's primitives against q: faces (5 words each) then spheres (2 words),
// rt_bvh.h leaf_records.  Closest: running (best, win); shadow: every valid
// hit multiplies the mask (an opaque one ends the ray).
//
// PRE: the origin-leaf pass (bvh_trace): a shadow query only looks for an
// opaque occluder there (its other factors are multiplied by the full search
// that follows, which visits this leaf again); closest and SKIP queries are
// idempotent under a repeated candidate and run as usual.
template <bool PRE = false, class CNT>
__device__ __forceinline__ void leaf_visit(Query &q, const Params &p, int link, CNT &cnt, float &best, int &win,
                                           bool &opaque, bool faces_only) {
    int v = -link - 1;
    const __amdgpu_buffer_rsrc_t rs = buffer_rsrc(p.leafrec);
    int off = (v >> 8) * 16;                 // byte offset of the leaf's first record (< 2^27)
    int nfc = (v >> 4) & 15, count = v & 15;
    if (faces_only) count = nfc;             // the leaf's faces come first
    for (int k = 0; k < count; k++) {
        float t0, t1;                        // candidate roots: a face has one (h0), a sphere two (h0, h1);
                                             // a root is read only under its flag
        bool h0, h1;
        int key;
        float fac;
        // one batch of loads for either kind; the face words 2..4 only when
        // some lane of the wave is at a face (a sphere then reads 3 words past
        // its record; the stream is padded for the last one) -- the vector
        // memory path (TA), not the ALU, is the busier one here
        // (w2..w4 are not zeroed when no lane is at a face: only the face
        // branch reads them, and no lane takes it then -- 12 v_mov per leaf
        // primitive saved)
        f4v w0 = bldv(rs, off, 0), w1 = bldv(rs, off, 16), w2, w3, w4;
        if (__ballot(k < nfc))
            w2 = bldv(rs, off, 32), w3 = bldv(rs, off, 48), w4 = bldv(rs, off, 64);
        else                                 // whatever the registers hold: no instruction
            asm("" : "=v"(w2), "=v"(w3), "=v"(w4));
        asm volatile("" ::"v"(w0), "v"(w1), "v"(w2), "v"(w3), "v"(w4));
        float4 f0 = make_float4(w0.x, w0.y, w0.z, w0.w), f1 = make_float4(w1.x, w1.y, w1.z, w1.w);
        float4 f2 = make_float4(w2.x, w2.y, w2.z, w2.w), f3 = make_float4(w3.x, w3.y, w3.z, w3.w);
        float4 f4 = make_float4(w4.x, w4.y, w4.z, w4.w);
        if (k < nfc) {
            off += 80;
            key = __float_as_int(f4.y);
            fac = f4.z;
            float a, bb, g;
            RT_COUNT(cnt.ftests++);
            h0 = face_test(f0, f1, f2, f3, f4, q.o, q.d, t0, a, bb, g) && (f1.w != 0.0f);
            h1 = false;
        } else {
            off += 32;
            key = __float_as_int(f1.x);
            fac = f1.y;
            RT_COUNT(cnt.stests++);
            h0 = h1 = sphere_test(f0, q.o, q.d, t0, t1);
        }
        // the roots in order, straight-line (a loop over them cost a select,
        // a counter and a branch per root)
        if (q.closest) {
            auto take = [&](float tt, bool h) {
                const bool valid = h & (tt > q.tmin) & (tt < kFltMax);
                const bool better = (tt < best) | ((tt == best) & (key < win));
                if (valid & better) {
                    best = tt;
                    win = key;
                }
            };
            take(t0, h0);
            take(t1, h1);
        } else if (q.skipchk) {
            // SKIP_TRANS (main.cpp:997-1002): a candidate of another object
            // that the reference's in-order scan would see as a new minimum --
            // any one before the stack top's object in order, or nearer than
            // the stack top's own nearest root (q.tmax) -- aborts the refraction
            auto aborts = [&](float tt, bool h) {
                return h & (tt > q.tmin) & (tt < kFltMax) & ((key < q.back) | (tt < q.tmax));
            };
            if ((key != q.back) & (aborts(t0, h0) | aborts(t1, h1))) opaque = true;
        } else if (key != q.self) {
            auto shadows = [&](float tt, bool h) { return h & (tt > q.tmin) & ((tt < q.tmax) | q.unb); };
            const bool s0 = shadows(t0, h0), s1 = shadows(t1, h1);
            if (s0 || s1) {
                if (fac == 0.0f && p.shadow_early_out) {
                    opaque = true;
                } else if (!PRE) {
                    if (s0) q.mask = clamp01(fac * q.mask);
                    if (s1) q.mask = clamp01(fac * q.mask);
                }
            }
        }
    }
}

// The six plane distances of a 4-wide node's children (rt_bvh.h Node4H):
// plane a of child i at origin_a + h * 2^e (h binary16, one scale 2^e per
// node), i.e. t = h * (2^e / d_a) + (origin_a - o_a) / d_a = fma(h, A_a, B_a)
// -- one v_fma_mix_f32 per plane (h converted inside the fma, exactly); the
// rounding (~ulp(D) in distance) is far inside the primitive padding.  (i, o)
// = (1 / d, o / d) per axis, or (1, o) for a point query: then the planes are
// the children's offsets from o.  Near / far plane per axis by the ray's
// octant: t(h) is monotonic in h with the sign of A (= the sign of 1/d), so
// min(t(lo), t(hi)) is t(near) exactly -- 4 min/max per child, not 10.
//
// wa[a]: axis a's window as the ray reads it -- (near 0,1  near 2,3  far 0,1
// far 2,3) as binary16 pairs: the node stores each axis as lo lo hi hi lo lo,
// and a ray with a negative direction along the axis loads the 16 bytes from
// word 2 on (near_window; the root, read through scalar loads, swaps instead).
struct ChildPlanes {
    float tn[3][4], tf[3][4];                   // [axis][child]: near / far plane
};
__device__ __forceinline__ ChildPlanes child_planes(float4 w0, const float4 wa[3], float ix, float iy, float iz,
                                                    float ox, float oy, float oz) {
    // 2^e * (1/d): an exact power-of-two scaling (w0.w = 2^e), finite by the
    // caps (|1/d| <= 2^100, e <= kQExpMax)
    const float A[3] = {ix * w0.w, iy * w0.w, iz * w0.w};
    const float B[3] = {fmaf(w0.x, ix, -ox), fmaf(w0.y, iy, -oy), fmaf(w0.z, iz, -oz)};
    ChildPlanes cp;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const unsigned nw[2] = {__float_as_uint(wa[a].x), __float_as_uint(wa[a].y)};
        const unsigned fw[2] = {__float_as_uint(wa[a].z), __float_as_uint(wa[a].w)};
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const h2v n = __builtin_bit_cast(h2v, nw[j]);
            const h2v f = __builtin_bit_cast(h2v, fw[j]);
#pragma unroll
            for (int e = 0; e < 2; e++) {
                cp.tn[a][2 * j + e] = fmaf((float)n[e], A[a], B[a]);
                cp.tf[a][2 * j + e] = fmaf((float)f[e], A[a], B[a]);
            }
        }
    }
    return cp;
}
// (lo, hi) window -> the ray's (near, far) window
__device__ __forceinline__ float4 near_first(float4 w, bool neg) {
    return neg ? make_float4(w.z, w.w, w.x, w.y) : w;
}

// Sort key of a child: the bits of its entry distance, kMissKey for a miss or
// an empty slot (unused slots link to the empty leaf, kEmptyLeaf: entering one
// is harmless, so no link test; their inverted boxes miss anyway).  The entry
// distance is >= tlo >= 0 whenever tmin >= 0, and for non-negative floats the
// unsigned order is the float order; otherwise only the visiting order (speed)
// changes.  kMissKey (-1) is an inline constant, +inf as a float is not (one
// v_mov per node visit); as a float it is a NaN, which tn <= tf excludes.
constexpr unsigned kMissKey = ~0u;
//
// tlo / thi join through the NaN-propagating maximum / minimum (gfx950
// v_maximum3_f32 / v_minimum3_f32), which need no canonicalised operands:
// with fmaxf / fminf the compiler canonicalises the two loop-carried bounds in
// every node visit.  A plane is NaN only if fma(h, A, B) meets inf - inf
// (coordinates beyond ~2^26 with a capped 1/d); the outer fmaxf / fminf then
// drop the bound together with it -- a wider interval, still conservative.
__device__ __forceinline__ unsigned child_entry(const ChildPlanes &cp, int i, float tlo, float thi) {
    const float tn = fmaxf(fmaxf(cp.tn[0][i], cp.tn[1][i]), __builtin_elementwise_maximum(cp.tn[2][i], tlo));
    const float tf = fminf(fminf(cp.tf[0][i], cp.tf[1][i]), __builtin_elementwise_minimum(cp.tf[2][i], thi));
    return (tn <= tf) ? __float_as_uint(tn) : kMissKey;
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
//
// org_pass: run the origin-leaf pass first (option org_first, by ray kind).
template <bool point, unsigned LEAF_WAIT = kLeafWait, class CNT>
__device__ void bvh_trace(Query &q, const Params &p, int *stk, CNT &cnt, bool org_pass = false, int root = 0,
                          V3 po = V3{0.0f, 0.0f, 0.0f}, float cone_k = 0.0f, float cone_h = 0.0f) {
    // |1/d| capped at 2^100 (1/0 -> the cap): the quantised planes' scale *
    // (1/d) then never overflows (the builder keeps e <= kQExpMax = 27), and
    // the cap is conservative: an axis with |d| below 1/cap moves the ray by
    // less than D / cap along it, far inside the 2^-16 D primitive padding
    constexpr float kCap = 0x1p100f;
    const float ix = point ? 1.0f : clampr(safe_rcp(q.d.x), -kCap, kCap);
    const float iy = point ? 1.0f : clampr(safe_rcp(q.d.y), -kCap, kCap);
    const float iz = point ? 1.0f : clampr(safe_rcp(q.d.z), -kCap, kCap);
    const bool neg_x = ix < 0.0f, neg_y = iy < 0.0f, neg_z = iz < 0.0f;
    // per axis: the byte offset of the window with the near planes first
    // (rt_bvh.h Node4H: lo lo hi hi lo lo -- word 2 on for a negative direction)
    const int wo_x = neg_x ? 8 : 0, wo_y = neg_y ? 8 : 0, wo_z = neg_z ? 8 : 0;
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
        RT_COUNT(atomicAdd(&p.stats[35], 1ull));   // counting instantiation only
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
    // the culling bound, widened by 2^-16: one multiply of the selected bound
    // (x * (1 + 2^-16) rounds the real x + x 2^-16 once, as x + x * 2^-16
    // does: the same bound, one instruction fewer)
    auto thi_now = [&] {
        return point ? 0.0f : (q.closest ? best : (q.unb ? kInf : q.tmax)) * (1.0f + 0x1p-16f);
    };
    // LDS holds stack entries [0, kLdsStack); entry 0 is kEmpty, or kRefill + b
    // when b blocks of kSpill older entries wait in device memory (ovf).
    // spilled block b of this lane: [workgroup][block][lane] -- a wave's
    // lanes' block b in adjacent bytes, like the dense frame heads (C5 +0.7 %,
    // reads 166 -> 154 GB against per-lane blocks; profiles/r05/ab/dense_spill_*)
    auto ovf_block = [&](int b) -> int * {
        return p.ovf + (((size_t)blockIdx.x * (p.ovf_stride / kSpill) + b) * kBlock + threadIdx.x) * kSpill;
    };
    // RT_CHECK builds (lib_check/, not the benched library): the stack-bottom
    // invariant -- entry 0 is kEmpty, or kRefill + b with 1 <= b blocks in
    // the lane's spill area (b * kSpill <= ovf_stride) -- at every traversal
    // entry and exit, spill and refill; a violation is counted
    // (stats[kCheckSlot], rt_scene_debug_counters [49]) and the access it
    // would make is skipped
    auto check = [&](bool ok) -> bool {
        if (RT_CHECK && !ok) atomicAdd(&p.stats[kCheckSlot], 1ull);
        return !RT_CHECK || ok;
    };
    auto bottom_ok = [&](int tag) {
        return tag == rtbvh::kEmpty || (tag > kRefill && (tag - kRefill) * kSpill <= p.ovf_stride);
    };
    if (RT_CHECK) (void)check(stk[0] == rtbvh::kEmpty);
    auto spill = [&]() {                       // move the oldest kSpill entries out
        const int tag = stk[0];
        const int nb = tag == rtbvh::kEmpty ? 0 : tag - kRefill;
        if (!check(bottom_ok(tag) && (nb + 1) * kSpill <= p.ovf_stride && sp <= p.stack_cap)) return;
        int *o = ovf_block(nb);
        for (int i = 0; i < kSpill; i++) o[i] = stk[(1 + i) * kBlock];
        for (int i = kSpill + 1; i < sp; i++) stk[(i - kSpill) * kBlock] = stk[i * kBlock];
        sp -= kSpill;
        stk[0] = kRefill + nb + 1;
        // counted in the workgroup's copy of the exit counters: a per-lane
        // counter held in a register costs more (C3 -0.5 %, ab_stat_copies.txt)
        atomicAdd(&p.stats[stat_copy_off((int)(blockIdx.x & (kStatCopies - 1))) + 34], 1ull);
    };
    // pop the top entry, whose value n the caller has already read (stk[sp - 1])
    auto pop_value = [&](int n) -> int {
        --sp;
        if ((unsigned)n - (unsigned)kRefill - 1u < (unsigned)(kStackMax / kSpill)) {   // rare: bring a block back
            const int nb = n - kRefill;
            if (!check(sp == 0 && n == stk[0] && bottom_ok(n))) return rtbvh::kEmpty;
            const int *o = ovf_block(nb - 1);
            for (int i = 0; i < kSpill; i++) stk[(1 + i) * kBlock] = o[i];
            stk[0] = nb > 1 ? n - 1 : rtbvh::kEmpty;
            sp = kSpill;
            n = o[kSpill - 1];                 // the block's newest entry is the top
        }
        return n;
    };
    auto pop = [&]() -> int { return pop_value(stk[(sp - 1) * kBlock]); };
    // One 4-wide node (rt_bvh.h Node4H, child_planes): slab-test the
    // children, push the far hits, continue with the nearest, park the first
    // leaf reached.
    auto visit_q = [&](float4 w0, float4 wx, float4 wy, float4 wz, float4 w4) {
#if RT_PROF
        cnt.trips++;
#endif
        RT_COUNT(cnt.boxes += 4);
        // the stack top, read while the node's planes are computed: a pop at
        // the end of the visit then waits for no LDS read before the next
        // node fetch (spill() below moves entries, not the top's value)
        const int top0 = stk[(sp - 1) * kBlock];
        float thi = thi_now();
        int c0 = __float_as_int(w4.x), c1 = __float_as_int(w4.y), c2 = __float_as_int(w4.z), c3 = __float_as_int(w4.w);
        const float4 wa[3] = {wx, wy, wz};
        const ChildPlanes cp = child_planes(w0, wa, ix, iy, iz, ox, oy, oz);
        unsigned k[4];
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
                k[i] = in ? __float_as_uint(d2) : kMissKey;   // nearest the cone's axis first (d2 >= 0)
            }
        }
        // up to 3 pushes below write stk[sp .. sp + 2]: make room (rare)
        if (sp > p.stack_cap - 3) spill();
        unsigned k0 = k[0], k1 = k[1], k2 = k[2], k3 = k[3];
        // nearest child by a 3-comparator tournament, registers only
#define RT_CSWAP(ka, ca, kb, cb)                 \
    {                                            \
        bool sw = kb < ka;                       \
        unsigned tk = sw ? kb : ka;              \
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
        sp += k3 != kMissKey ? 1 : 0;
        stk[sp * kBlock] = c1;
        sp += k1 != kMissKey ? 1 : 0;
        stk[sp * kBlock] = c2;
        sp += k2 != kMissKey ? 1 : 0;
        // the top after the pushes, from registers
        const int top1 = k2 != kMissKey ? c2 : k1 != kMissKey ? c1 : k3 != kMissKey ? c3 : top0;
        if (k0 != kMissKey) {
            node = c0;
        } else {
            node = pop_value(top0);            // no child hit: nothing was pushed
        }
        if (node < 0 && node != rtbvh::kEmpty && leaf == rtbvh::kEmpty) {
            leaf = node;                       // park it, keep descending
            node = k0 != kMissKey ? pop_value(top1) : pop();
        }
    };
    // The root (every trace starts there; wave-uniform) comes through scalar
    // loads: the first step then has no vector-memory wait, which on gfx950
    // would also wait for every frame store the shading step just issued
    // (loads and stores share vmcnt, in order).
    // Origin-leaf pass (org_pass; option org_first): a secondary ray starts on an
    // object, and in a dense scene what it meets first is often in that
    // object's own leaf -- a refraction ray entering a sphere meets the
    // sphere's far side, a reflection or shadow ray a neighbour.  The leaf is
    // tested before the search from the root: a closest hit found there bounds
    // the search (thi), an opaque occluder ends a shadow ray.  The search
    // visits the leaf again; that changes no result (PRE, leaf_visit).
    const __amdgpu_buffer_rsrc_t bvh_rs = buffer_rsrc(p.bvh);
    bool ended = false;
    if (!point && org_pass && !faces_only && !q.skipchk && q.self >= 0 && (q.closest || p.shadow_early_out)) {
        leaf_visit<true>(q, p, p.objleaf[q.self], cnt, best, win, opaque, false);
        ended = opaque;
    }
    if (point)
        node = root;
    else if (!ended) {
        visit_q(sld4b(p.bvh, 0), near_first(sld4b(p.bvh, rtbvh::kNodeAxisOff), neg_x),
                near_first(sld4b(p.bvh, rtbvh::kNodeAxisOff + 24), neg_y),
                near_first(sld4b(p.bvh, rtbvh::kNodeAxisOff + 48), neg_z), sld4b(p.bvh, rtbvh::kNodeLinkOff));
    }
    for (;;) {
        while (node >= 0) {
#if RT_PROF >= 2
            const unsigned long long t_a = __builtin_amdgcn_s_memtime();
#endif
            // node = the node's byte offset (rt_scene.cpp): five buffer loads
            // at immediate offsets from it; each axis window at the ray's
            // near-first offset (wo_*: 0 or 8 bytes, per lane)
            const float4 w0 = bld4(bvh_rs, node, 0), w4 = bld4(bvh_rs, node, rtbvh::kNodeLinkOff);
            const float4 wx = bld4(bvh_rs, node + wo_x, rtbvh::kNodeAxisOff);
            const float4 wy = bld4(bvh_rs, node + wo_y, rtbvh::kNodeAxisOff + 24);
            const float4 wz = bld4(bvh_rs, node + wo_z, rtbvh::kNodeAxisOff + 48);
#if RT_PROF >= 2
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::"v"(w0.x), "v"(w4.x) : "memory");
            cnt.t_fetch += __builtin_amdgcn_s_memtime() - t_a;
#endif
            visit_q(w0, wx, wy, wz, w4);
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
            // the stack top, read while the leaf's primitives are tested (the
            // leaf visit does not touch the stack)
            const int top = stk[(sp - 1) * kBlock];
            leaf_visit(q, p, leaf, cnt, best, win, opaque, faces_only);
            leaf = rtbvh::kEmpty;
            if (opaque) {
                node = rtbvh::kEmpty;
                stk[0] = rtbvh::kEmpty;        // drop any spilled entries with the rest
                break;
            }
            if (node < 0 && node != rtbvh::kEmpty) {
                leaf = node;
                node = pop_value(top);
            }
        }
        if (node == rtbvh::kEmpty && leaf == rtbvh::kEmpty) break;
    }
    if (RT_CHECK) (void)check(stk[0] == rtbvh::kEmpty);
    if (q.closest) {
        if (win >= 0) {
            q.tmax = best;
            q.win = win;
        }
    } else if (q.skipchk) {
        q.skipped = opaque;
    } else if (opaque) {
        q.mask = 0.0f;
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
// The split head slots (head_split) keep no meta: their instantiations keep in
// the top byte of a node's meta a bit per level above it -- bit kKindsShift + k:
// the node at level k + 1 on its path is a refraction child -- and the light
// index in the 15 bits below (scenes of more lights take MAXF 17, rt_scene.cpp)
constexpr int kKindsShift = 24;
constexpr unsigned kKindsMask = 0xFF000000u;
static_assert(kKindsShift - 9 == kSplitLightBits, "meta: light bits below the kinds");
template <int MAXF>
__device__ __forceinline__ int h_light(const HotR &h) {
    return head_split(MAXF) ? (int)((h.meta >> 9) & ((1u << kSplitLightBits) - 1)) : (int)(h.meta >> 9);
}
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
static_assert(kLdsHot == kLdsHotWords, "LDS state words (rt_device.h)");
extern __shared__ float4 rt_lds[];   // dynamic LDS of render_kernel: state, then stack / primitives, lights

// The lights, staged in LDS at kernel start: a shading step's light reads are
// then LDS latency, not a dependent trip to L2 (one dependent load per
// shading step costs ~1 % of C3, profiles/r02/ab_shading_probe.txt)
//
// Light i's words (LightK: xyz w | col | L | sdir): from the LDS copy, or --
// when the scene's lights do not all fit under the workgroup's LDS limit
// (thousands of lights) -- from device memory.  The condition is a kernel
// argument, so the branch is a scalar one (a per-lane test cost C3 1 %,
// profiles/r03/ab_light_fallback.txt).
struct LightW {
    f4v w0, w1, w2, w3;
};
__device__ __forceinline__ LightW light_words(const Params &p, int i) {
    static_assert(sizeof(LightK) == 4 * sizeof(f4v), "LightK = 4 float4");
    // (the device-memory copy through buffer loads: with two plain loads the
    // compiler merged the branches into one flat load of a selected address,
    // which waits on every outstanding vector-memory access as well)
    LightW r;
    if (p.lights_in_lds) {
        const f4v *l = reinterpret_cast<const f4v *>(rt_lds + p.lights_lds) + 4 * i;
        r.w0 = l[0], r.w1 = l[1], r.w2 = l[2], r.w3 = l[3];
    } else {
        const __amdgpu_buffer_rsrc_t rs = buffer_rsrc(p.lights);
        r.w0 = bldv(rs, 64 * i, 0), r.w1 = bldv(rs, 64 * i, 16), r.w2 = bldv(rs, 64 * i, 32);
        r.w3 = bldv(rs, 64 * i, 48);
    }
    return r;
}

__device__ __forceinline__ float *lane_lds() { return reinterpret_cast<float *>(rt_lds) + threadIdx.x; }
template <int MAXF>
__device__ __forceinline__ int h_light_lds() {
    const unsigned meta = __float_as_uint(lane_lds()[LW_META * kBlock]);
    return head_split(MAXF) ? (int)((meta >> 9) & ((1u << kSplitLightBits) - 1)) : (int)(meta >> 9);
}
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

// Cold frame of a node that opened a child (one per recursion level, per
// lane, in device memory): what the node needs when the child returns.
//  * head (bytes 0..19): acc, f -- F_t for a refraction child, F_r for a
//    reflection child -- and the node's meta; then the CHILD's medium stack
//    (written by the transition in the same line);
//  * ext (from byte kColdExt on), refraction children only: N, I, obj, eta_i,
//    eta_t and the hit point -- after a refraction child the node goes on to
//    its reflection; after a reflection child it is complete and needs only
//    acc and F_r.
// A reflection child (~80 % of the child opens) thus dirties only the first
// 64 bytes of the frame's line for MAXF <= 9, and its return reads only those.
constexpr int cold_ext(int maxf) { return 20 + 4 * maxf <= 64 ? 64 : (20 + 4 * maxf + 15) / 16 * 16; }
constexpr int cold_size(int maxf) { return (cold_ext(maxf) + 48 + 63) / 64 * 64; }
template <int MAXF>
struct Cold {
    float4 head;                     // acc.rgb, f
    unsigned meta;                   // phase:3 | state:1 | stack size:5 | light:23
    int stack[MAXF];                 // the CHILD's medium stack (incident_object_stack), object indices
    int pad0_[(cold_ext(MAXF) - 20 - 4 * MAXF) / 4];
    float4 ext[3];                   // (N, I.x), (I.y, I.z, obj, eta_i), (eta_t, P)
    unsigned xmeta;                  // head_split: the node's meta (its head slot keeps none)
    int pad1_[(cold_size(MAXF) - cold_ext(MAXF) - 52) / 4];
};
static_assert(sizeof(Cold<5>) == 128 && sizeof(Cold<9>) == 128 && sizeof(Cold<17>) == 192, "cold frame sizes");
static_assert(cold_ext(5) == 64 && cold_ext(9) == 64, "a reflection child's frame is one 64-B half line");

// One level's frame as the shading code sees it: the lane's Cold record and,
// in the recursive instantiations (dense_heads(MAXF)), the level's slots in
// dense arrays ([block][level][lane], from Params::heads): the slots of one
// level for consecutive lanes of a workgroup are consecutive, so a wave's
// slots share lines.  Stack entries past the dense ones, and a refraction
// child's extension, stay in the Cold record.
//  * head_split(MAXF) (MAXF 5 and 9): a 16-B head slot -- acc, f -- and, in a
//    second array after the heads, a 16-B stack slot -- the child's first 4
//    medium-stack entries.  The node's meta is not saved with the head: a
//    reflection child's return needs only acc and f (the parent is then
//    complete), a refraction child's return reads the extension anyway, and
//    the meta travels there (Cold::xmeta); which of the two the parent
//    opened is a bit of the child's own meta (kKindsShift).
//  * MAXF 17: one 32-B slot -- acc, f, meta and the
//    first 3 stack entries.
//
// Why: a child's return reads its parent's head back after the child's
// whole subtree, and with each head alone in a 128-B line of a 377-MB frame
// area (C5) that read missed L2 nearly every time -- the head stream was
// ~140 of C5's 266 GB read (the head-copy probe).  Dense 32-B
// slots: C5 266 -> 166 GB read, +2.1 %; C3 3.5 -> 2.0 GB read, +0.4 %
// (profiles/r05/ab/dense_heads_*).  The returns' line misses follow the slot
// density (64-B slots: C5 215 GB read, -1.7 %, profiles/r06/heads); the split
// 16-B heads: C5 154 -> 104 GB read, +0.7 %; C3 +0.2 % (profiles/r06/heads/
// ab_split_*).  (Addressed [level][lane] over the whole grid instead, the
// slot arithmetic cost C3 0.2 ... 0.7 %.)
template <int MAXF, bool D = dense_heads(MAXF)>
struct Fr {                          // plain frames (and MAXF = 1, which opens no child)
    static constexpr bool kDense = false;
    Cold<MAXF> *c;
    __device__ __forceinline__ int stk(int i) const { return c->stack[i]; }
    __device__ __forceinline__ void set_stk(int i, int v) const { c->stack[i] = v; }
};
template <int MAXF>
struct Fr<MAXF, true> {              // dense heads (dense_heads(MAXF))
    static constexpr bool kDense = true;
    Cold<MAXF> *c;
    int *hs;
    int *ss;                         // the stack slot (head_split: its own array; else hs + 5)
    __device__ __forceinline__ int stk(int i) const { return i < head_stack(MAXF) ? ss[i] : c->stack[i]; }
    __device__ __forceinline__ void set_stk(int i, int v) const {
        if (i < head_stack(MAXF))
            ss[i] = v;
        else
            c->stack[i] = v;
    }
};
template <int MAXF>
__device__ __forceinline__ void cold_save_head(const Fr<MAXF> &fr, const HotR &h, float f) {
    if constexpr (Fr<MAXF>::kDense) {
        reinterpret_cast<f4v *>(fr.hs)[0] = f4v{h.acc.r, h.acc.g, h.acc.b, f};
        if constexpr (!head_split(MAXF)) fr.hs[4] = (int)h.meta;
    } else {
        Cold<MAXF> &c = *fr.c;
        reinterpret_cast<f4v &>(c.head) = f4v{h.acc.r, h.acc.g, h.acc.b, f};
        c.meta = h.meta;
    }
}
template <int MAXF>
__device__ __forceinline__ void cold_save_ext(const Fr<MAXF> &fr, V3 P, const HotR &h) {
    f4v *v = reinterpret_cast<f4v *>(fr.c->ext);
    v[0] = f4v{h.N.x, h.N.y, h.N.z, h.I.x};
    v[1] = f4v{h.I.y, h.I.z, __int_as_float(h.obj), h.ei};
    v[2] = f4v{h.et, P.x, P.y, P.z};
    if constexpr (head_split(MAXF)) fr.c->xmeta = h.meta;
}
// the head: h.acc, h.meta; returns f
template <int MAXF>
__device__ __forceinline__ float cold_restore_head(const Fr<MAXF> &fr, HotR &h) {
    f4v a;
    if constexpr (Fr<MAXF>::kDense) {
        a = reinterpret_cast<const f4v *>(fr.hs)[0];
        if constexpr (!head_split(MAXF)) h.meta = (unsigned)fr.hs[4];
    } else {
        a = reinterpret_cast<const f4v &>(fr.c->head);
        h.meta = fr.c->meta;
    }
    h.acc = {a.x, a.y, a.z};
    return a.w;
}
// the rest of a refraction child's parent; returns its hit point
template <int MAXF>
__device__ __forceinline__ V3 cold_restore_ext(const Fr<MAXF> &fr, HotR &h) {
    const f4v *v = reinterpret_cast<const f4v *>(fr.c->ext);
    const f4v a = v[0], b = v[1], d = v[2];
    h.N = {a.x, a.y, a.z};
    h.I = {a.w, b.x, b.y};
    h.obj = __float_as_int(b.z);
    h.ei = b.w;
    h.et = d.x;
    if constexpr (head_split(MAXF)) h.meta = fr.c->xmeta;
    return V3{d.y, d.z, d.w};
}

// Hit record of the winning intersection, recomputed exactly as TraceRay did:
// the point, the normal and (faces) the barycentric coordinates.  Plain
// scalars, not out-parameters: a V3 written in two branches through a
// reference was kept in scratch (a store and a reload per node open).
struct HitRec {
    V3 P, N;
    float ba, bb, bg;
};
__device__ __forceinline__ HitRec hit_geometry(const Params &p, int obj, V3 o, V3 d, float t) {
    HitRec h;
    h.P = vadd(o, vmul(d, t));
    h.ba = h.bb = h.bg = 0.0f;
    if (obj < p.nf) {
        const float4 *F = &row(p.fscan, 5 * obj);
        float4 f0 = F[0], f1 = F[1], f2 = F[2], f3 = F[3], f4 = F[4];
        V3 ep = vsub(h.P, V3{f0.x, f0.y, f0.z});
        V3 e1 = {f2.x, f2.y, f2.z}, e2 = {f3.x, f3.y, f3.z};
        float d1p = vdot(e1, ep), d2p = vdot(e2, ep);
        float b = (f3.w * d1p - f4.x * d2p) / f1.w;
        float g = (f2.w * d2p - f4.x * d1p) / f1.w;
        float a = 1.0f - (b + g);
        h.ba = a, h.bb = b, h.bg = g;
        const FaceShadeK &fs = row(p.fsh, obj);
        if (fs.smooth) {
            V3 n0 = {fs.vn[0][0], fs.vn[0][1], fs.vn[0][2]};
            V3 n1 = {fs.vn[1][0], fs.vn[1][1], fs.vn[1][2]};
            V3 n2 = {fs.vn[2][0], fs.vn[2][1], fs.vn[2][2]};
            h.N = vnorm(vadd(vadd(vmul(n0, a), vmul(n1, b)), vmul(n2, g)));
        } else {
            h.N = {f1.x, f1.y, f1.z};
        }
    } else {
        float4 s = row(p.sscan, obj - p.nf);
        h.N = vnorm(vdiv(vsub(h.P, V3{s.x, s.y, s.z}), s.w));
    }
    return h;
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
__device__ __forceinline__ void light_vectors(const LightW &lt, V3 P, V3 &L, V3 &sdir, float &distL, bool &unb) {
    if (lt.w0.w == 0.0f) {
        L = {lt.w2.x, lt.w2.y, lt.w2.z};
        sdir = {lt.w3.x, lt.w3.y, lt.w3.z};
        distL = 0.0f;
        unb = true;
    } else {
        V3 pos = {lt.w0.x, lt.w0.y, lt.w0.z};
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
__device__ __forceinline__ bool in_stack(const Fr<MAXF> &f, int sn, int obj) {
    bool in = false;
    for (int q = 0; q < sn; q++) in |= (f.stk(q) == obj);
    return in;
}

// The parent's medium stack into the child's (frame fc holds the parent's,
// c the child's: the frames one level up).  The root node's (level 0, a
// primary hit) is always {its own object} (main.cpp:751-757) and lives in no
// frame.
template <int MAXF>
__device__ __forceinline__ void copy_stack(const HotR &f, const Fr<MAXF> &fc, const Fr<MAXF> &c, bool root) {
    if (root) {
        c.set_stk(0, f.obj);
    } else {
        const int fsn = h_sn(f);
        for (int q = 0; q < fsn; q++) c.set_stk(q, fc.stk(q));
    }
}

// The child's medium state after a transition: state, stack size, eta_i, eta_t
// (its stack is written into the child's cold frame).
struct Medium {
    int state, sn;
    float ei, et;
    unsigned kinds;                  // head_split: the child's meta kinds (kKindsShift)
};

__device__ V3 node_open(const Params &p, int obj, V3 o, V3 d, float t, Medium m) {
    const HitRec hr = hit_geometry(p, obj, o, d, t);
    V3 N = hr.N;
    const ObjK &ob = row(p.objs, obj);
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
            const FaceShadeK &fs = row(p.fsh, obj);
            float u = (hr.ba * fs.vt[0][0]) + (hr.bb * fs.vt[1][0]) + (hr.bg * fs.vt[2][0]);
            float v = (hr.ba * fs.vt[0][1]) + (hr.bb * fs.vt[1][1]) + (hr.bg * fs.vt[2][1]);
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
    h.meta = mk_meta(PH_LIGHT, m.state, m.sn, 0) | m.kinds;
    h.ei = m.ei;
    h.et = m.et;
    lds_store(h);
    // the hit point again, as hit_geometry computed it (the same operations on
    // the same inputs: the same value): held across the texture and shading
    // code above it was spilled to scratch
    float tt = t;
    asm volatile("" : "+v"(tt));
    return vadd(o, vmul(d, tt));
}

// Image coordinates of work item `pix` (defined with pixel_xy below).
__device__ __forceinline__ void image_xy(const Params &p, unsigned pix, int &x, int &y);

// back() of an empty medium stack (main.cpp:1028, undefined in the
// reference): count it and log the pixel (stats[44] events, their pixels
// after the counters, rt_scene_debug_ub_pixels) -- a rare branch
__device__ __forceinline__ void ub_note(const Params &p, unsigned pix) {
    const unsigned long long k = atomicAdd(&p.stats[44], 1ull);
    if (k < (unsigned long long)kUbLogMax) {
        int x, y;
        image_xy(p, pix, x, y);
        p.stats[kUbLogOff + k] = ((unsigned long long)(unsigned)x << 32) | (unsigned)y;
    }
}

// Medium-stack transition for the refraction child (main.cpp:1021-1070).
template <int MAXF, class CNT>
__device__ Medium refr_transition(const Params &p, const HotR &f, const Fr<MAXF> &fc, const Fr<MAXF> &c, int hit,
                                  bool root, CNT &cnt, unsigned pix) {
    const int fsn = h_sn(f);
    copy_stack(f, fc, c, root);
    int n = fsn;
    Medium m;
    float hit_eta = row(p.objs, hit).eta;
    if (h_state(f) == ENTERING) {
        if (hit == f.obj) {
            m.state = EXITING;
            if (n > 0) {
                m.ei = row(p.objs, c.stk(n - 1)).eta;
                n--;
            } else {
                m.ei = p.eta_bkg;            // back() on an empty vector: UB in the reference
                RT_COUNT(cnt.ub++);
                ub_note(p, pix);
            }
            m.et = n > 0 ? row(p.objs, c.stk(n - 1)).eta : p.eta_bkg;
            if (n > 0) n--;
        } else {
            m.state = ENTERING;
            m.ei = f.et;
            m.et = hit_eta;
            c.set_stk(n++, hit);
        }
    } else if (n > 0) {
        if (!(root ? hit == f.obj : in_stack(fc, fsn, hit))) {
            m.state = ENTERING;
            m.ei = f.et;
            m.et = hit_eta;
            c.set_stk(n++, hit);
        } else {
            m.state = EXITING;
            m.ei = f.et;
            m.et = row(p.objs, c.stk(n - 1)).eta;
            n--;
        }
    } else {
        m.state = ENTERING;
        m.ei = p.eta_bkg;
        m.et = hit_eta;
        c.set_stk(0, hit);
        n = 1;
    }
    m.sn = n;
    return m;
}

// Medium-stack transition for the reflection child (main.cpp:1134-1182).
template <int MAXF>
__device__ Medium refl_transition(const Params &p, const HotR &f, const Fr<MAXF> &fc, const Fr<MAXF> &c, int hit,
                                  bool root) {
    const int fsn = h_sn(f);
    copy_stack(f, fc, c, root);
    int n = fsn;
    Medium m;
    float hit_eta = row(p.objs, hit).eta;
    if (h_state(f) == ENTERING) {
        m.state = ENTERING;
        m.ei = f.ei;
        if (n > 0) {
            if (!(root ? hit == f.obj : in_stack(fc, fsn, hit))) {
                m.et = hit_eta;
                c.set_stk(n++, f.obj);        // pushes the incidence object, as the reference does
            } else {
                m.et = row(p.objs, c.stk(n - 1)).eta;
                n--;
            }
        } else {
            m.et = hit_eta;
            c.set_stk(0, hit);
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
            c.set_stk(n++, hit);
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
    // level k's frame; the dense slots (dense_heads: Params::heads, after the
    // frames and the spill area, rt_scene.cpp launch_one) are [block][level]
    // [lane] -- 16-B heads then 16-B stack slots (head_split), or 32-B slots --
    // addressed where used, like the frames, rather than held in registers
    // across the traversal
    __device__ __forceinline__ Fr<MAXF> fr(const Params &p, int k) const {
        Fr<MAXF> f;
        f.c = cold() + k;
        if constexpr (Fr<MAXF>::kDense) {
        unsigned t;
        asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"((unsigned)threadIdx.x));
        // (slot index < 2^25: levels <= 17, lanes of the grid < 2^20)
        if constexpr (head_split(MAXF)) {
            const size_t slot = (size_t)((blockIdx.x * MAXF + (unsigned)k) * kBlock + t);
            f.hs = static_cast<int *>(p.heads) + slot * 4;
            f.ss = static_cast<int *>(p.heads) + ((size_t)gridDim.x * MAXF * kBlock + slot) * 4;
        } else {
            f.hs = static_cast<int *>(p.heads) + (size_t)((blockIdx.x * MAXF + (unsigned)k) * kBlock + t) * kHeadInts;
            f.ss = f.hs + 5;
        }
        }
        return f;
    }
};

__device__ __forceinline__ void shadow_query(Query &q, const Params &p, int light, int self) {
    V3 L, sd;
    float dl;
    bool unb;
    light_vectors(light_words(p, light), q.o, L, sd, dl, unb);
    q.d = sd;
    q.tmin = p.eps;
    q.tmax = dl;
    q.unb = unb;
    q.self = self;
    q.closest = false;
    q.skipchk = false;
    q.skipped = false;
    q.win = -1;
    q.mask = 1.0f;                   // this light's factors, from 1 (the prior mask is the caller's, q.back)
}

__device__ __forceinline__ void closest_query(Query &q, const Params &p, V3 d, int org) {
    q.d = d;
    q.tmin = p.eps;
    q.tmax = kFltMax;
    q.unb = false;
    q.self = org;                    // origin object (not excluded: offer)
    q.closest = true;
    q.skipchk = false;
    q.skipped = false;
    q.win = -1;
}

// MAXF = 1: the instantiation for scenes where no material reflects or
// refracts (or depth 0): the recursion's code is compiled out -- its
// conditions are false at run time there anyway (launch: maxf_for) -- and
// the registers it frees carry the last light's zero-Phong skip, which costs
// the recursive instantiations more than it saves them (C3 -2.1 %, C5 -1.8 %;
// C4 +2.6 %, profiles/r04/ab/llskip_*.txt).
template <int MAXF>
constexpr bool kRecurse = MAXF > 1;

// A light's diffuse + specular sum for light direction L (main.cpp:930-950)
__device__ __forceinline__ C3 phong_sum(const HotR &h, const ObjK &ob, V3 L) {
    // H only feeds the specular power: rsqrt instead of 3 IEEE divisions
    // (<= 2 ulp; vnorm(0) = NaN either way)
    V3 hv = vadd(L, h.I);
    V3 H = vmul(hv, __builtin_amdgcn_rsqf(vdot(hv, hv)));
    C3 dc = cmulf(cmulf(h.dif, ob.kd), max0(vdot(h.N, L)));
    C3 sc = cmulf(cmulf(C3{ob.spc[0], ob.spc[1], ob.spc[2]}, ob.ks), spec_pow(max0(vdot(h.N, H)), ob.n));
    return cadd(dc, sc);
}

// Advance one lane after its scan: consume the result, run ShadeRay logic
// until the next TraceRay (returns its kind, RK_SHADOW/RK_REFR/RK_REFL, with q
// set up) or until the pixel is done (returns RK_NONE with `color` set).
// Invariant: while a node is on top, q.o is its hit point.
template <int MAXF, class CNT>
__device__ int advance(const Params &p, LaneState<MAXF> &ls, Query &q, CNT &cnt, C3 &color, unsigned pix) {
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
        m = Medium{ENTERING, 1, p.eta_bkg, row(p.objs, q.win).eta, 0u};   // stack {q.win}: implicit (copy_stack)
        open = true;
        top = 0;
    } else {
        lds_load(h);
        const int phase = h_phase(h);
        if (phase == PH_LIGHT) {                     // main.cpp:952-958
            // one light step per iteration (the loop continues only past known
            // shadow rays, below)
            for (;;) {
                const int light = h_light<MAXF>(h);
                const ObjK &ob = row(p.objs, h.obj);
                // the light's words in one batch (LightK: xyz w | col | L)
                const LightW lw = light_words(p, light);
                const f4v lw0 = lw.w0, lw1 = lw.w1, lw2 = lw.w2;
                // L as light_vectors computed it for the shadow ray just traced:
                // that ray's direction for a point light, the constant -L for a
                // directional one (q.d is not modified by a trace)
                V3 L = lw0.w == 0.0f ? V3{lw2.x, lw2.y, lw2.z} : q.d;
                C3 lc = {lw1.x, lw1.y, lw1.z};
                // the cumulative mask after this light: the earlier lights'
                // times this light's factors (one product, reassociated)
                const float mcum = clamp01(q.mask * prior_mask(q));
                h.acc = cadd(h.acc, cmulc(cmulf(lc, mcum), phong_sum(h, ob, L)));
                q.back = __float_as_int(mcum);
                h.meta += 1u << 9;                       // next light
                // stored at once, in the block that computed it: kept in registers
                // across the other phases' code of the shading step, the colour
                // was spilled to scratch and reloaded -- a reload whose vmcnt wait
                // also waited for the frame stores of lanes that opened a child
                lds_store_light(h);
                if (light + 1 >= p.nl) break;        // the light loop is done
                {
                    // next light's shadow ray from the same point: origin, self
                    // and cumulative mask are already in q (main.cpp:885-928)
                    // (opaque index: reusing this light's address for the next
                    // one kept a 64-bit pointer live -- and spilled -- across the
                    // shading code)
                    int next = light + 1;
                    asm volatile("" : "+v"(next));
                    // The node's last light, with a Phong sum of exactly 0: its
                    // term lc * mask * 0 is 0 whatever the ray meets, and its mask
                    // is not used after the light loop (main.cpp:788 starts the
                    // next node's at 1).  A prior mask of 0 makes the query a known
                    // one (counted, not searched) and its term 0 (Params::
                    // last_light_skip: finite light colours, no NaN factor).
                    // Tested before the query is set up, while the node's N, I
                    // and colour are still in registers.
                    bool zero = false;
#ifndef RT_LLSKIP
#define RT_LLSKIP 1
#endif
                    if (RT_LLSKIP && !kRecurse<MAXF> && p.last_light_skip && next == p.nl - 1) {
                        const LightW nw = light_words(p, next);
                        V3 Ln, sd;
                        float dl;
                        bool unb;
                        light_vectors(nw, q.o, Ln, sd, dl, unb);   // Ln: the light step's L for either kind
                        const C3 t = phong_sum(h, ob, Ln);
                        zero = (t.r == 0.0f) & (t.g == 0.0f) & (t.b == 0.0f);
                    }
                    shadow_query(q, p, next, h.obj);
                    if (zero) q.back = __float_as_int(0.0f);
                    // A known shadow ray (its prior mask is already 0, so its
                    // cumulative mask stays 0 whatever it meets: render_kernel
                    // counts it and does not search it): in the instantiation
                    // without counters and without recursion (MAXF = 1) its
                    // light step is taken at once, in this shading step,
                    // instead of after a trace step the lane would sit out --
                    // the same operations on the same values (mask 1 from
                    // shadow_query times the prior 0; L from the query just
                    // set up), so the same colour; the pixel then ends a step
                    // sooner (C4 +1.5 %).  In the recursive instantiations the
                    // lane would issue its reflection / refraction search a
                    // step ahead of the wave's other lanes, which are still
                    // tracing that light's shadow ray: C3 -2.4 %, C5 -2.1 %
                    // (profiles/r06/ab/known_all_*.txt).  The counting
                    // instantiation returns it, to count it.
                    if constexpr (!std::remove_reference_t<decltype(cnt)>::kCount && !kRecurse<MAXF>) {
                        if (p.shadow_early_out && prior_mask(q) == 0.0f) continue;
                    }
                    ls.top = top;
                    return RK_SHADOW;
                }
            }
        } else if (phase == PH_REFR) {
            if (q.skipped) {
                RT_COUNT(cnt.skip++);                // tmp_transparency stays 0
                set_phase(h, PH_REFL);
            } else if (q.win >= 0) {
                m = refr_transition(p, h, ls.fr(p, top > 0 ? top - 1 : 0), ls.fr(p, top), q.win, top == 0, cnt, pix);
                set_phase(h, PH_REFR_CHILD);
                open = true;
            } else {
                C3 tr = cmulf(cmulf(bkg, (float)(1.0 - (double)h.dif.r)),
                              (float)(1.0 - (double)row(p.objs, h.obj).opacity));
                h.acc = cadd(h.acc, tr);
                set_phase(h, PH_REFL);
            }
        } else {                                     // PH_REFL
            if (q.win >= 0) {
                m = refl_transition(p, h, ls.fr(p, top > 0 ? top - 1 : 0), ls.fr(p, top), q.win, top == 0);
                set_phase(h, PH_REFL_CHILD);
                open = true;
            } else {
                // miss: refl = bkg * F_r (F_r in dif.r since the query was
                // issued); finish this node below
                h.acc = cadd(h.acc, cmulf(bkg, h.dif.r));
                set_phase(h, PH_DONE);
            }
        }
        if (open) {                                  // the recursion: save the parent
            const Fr<MAXF> c = ls.fr(p, top);
            // dif.r: F_t (refraction child) or F_r (reflection child)
            if (h_phase(h) == PH_REFR_CHILD) cold_save_ext(c, q.o, h);
            cold_save_head(c, h, h.dif.r);
            if constexpr (head_split(MAXF))          // the child's kinds: ours and its own
                m.kinds = (h.meta & kKindsMask) | ((unsigned)(h_phase(h) == PH_REFR_CHILD) << (kKindsShift + top));
            top++;
        }
    }
    if (open) {
        q.o = node_open(p, q.win, q.o, q.d, q.tmax, m);
        ls.top = top;
        if (p.nl > 0) {                              // shadow ray for light 0 (main.cpp:885-928)
            shadow_query(q, p, 0, q.win);
            q.back = __float_as_int(1.0f);           // the node's first light: mask {1,1,1} (main.cpp:788)
            return RK_SHADOW;
        }
        lds_load(h);                                 // no lights: straight to the light loop's end
    }
    // ---- run the top node forward (phase PH_LIGHT here: its last light is done) ----
    for (;;) {
        if (h_phase(h) == PH_LIGHT) {
            const ObjK &ob = row(p.objs, h.obj);
            // ambient + specular sum, then Fresnel / transmission (main.cpp:961-992)
            h.acc = cadd(cmulf(h.dif, ob.ka), h.acc);
            // TIR, F_t and the refraction direction only for a node that can
            // refract: the reference computes them for every node
            // (main.cpp:961-992), but they feed nothing else, and a wave with
            // no such lane then skips the asinf / acosf / double Schlick code
            bool refr = kRecurse<MAXF> && p.depth - top > 0 && (double)ob.opacity < 1.0 && ob.eta > 0;
            float cosI = 0.0f, snell = 0.0f;
            if (refr) {
                cosI = cos_i(h);
                snell = h.ei / h.et;
                float crit = asinf(h.et / h.ei);
                float inc = acosf(cosI);
                bool tir = (crit < inc) && ((double)inc < kRightAngle);
                float F0 = (h.et - h.ei) / (h.et + h.ei);
                h.dif.r = schlick(F0 * F0, cosI);    // F_t (the diffuse colour is no longer needed)
                refr = !tir;
            }
            if (refr) {
                float k = sqrtf((float)(1.0 - (double)(snell * snell) * (1.0 - (double)(cosI * cosI))));
                V3 T = vadd(vmul(vmul(h.N, -1.0f), k), vmul(vsub(vmul(h.N, cosI), h.I), snell));
                closest_query(q, p, T, h.obj);
                const int sn = h_sn(h);
                q.skipchk = (sn > 0) && !ob.is_sphere;
                q.back = sn > 0 ? (top == 0 ? h.obj : ls.fr(p, top - 1).stk(sn - 1)) : -1;
                set_phase(h, PH_REFR);
                lds_store_phase(h);
                ls.top = top;
                return RK_REFR;
            }
            set_phase(h, PH_REFL);
        }
        if (h_phase(h) == PH_REFL) {                 // main.cpp:1103-1124
            const ObjK &ob = row(p.objs, h.obj);
            const float cosI = cos_i(h);
            float Fr = refl_fresnel(ob, cosI);
            if (kRecurse<MAXF> && p.depth - top > 0 && (double)Fr != 0.0 && (double)ob.ks > 0.0) {
                V3 R = vsub(vmul(h.N, (float)(2.0 * (double)cosI)), h.I);
                closest_query(q, p, R, h.obj);
                h.dif.r = Fr;                        // for the child's return or the miss (F_t is done with)
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
        const Fr<MAXF> pc = ls.fr(p, top);
        const float f = cold_restore_head(pc, h);
        if (head_split(MAXF) ? ((h.meta >> (kKindsShift + top)) & 1u) != 0 : h_phase(h) == PH_REFR_CHILD) {   // main.cpp:1072-1083
            q.o = cold_restore_ext(pc, h);
            h.dif.r = f;                             // F_t
            const ObjK &pob = row(p.objs, h.obj);
            C3 tr = cmulf(cmulf(c, (float)(1.0 - (double)f)), (float)(1.0 - (double)pob.opacity));
            h.acc = cadd(h.acc, tr);
            set_phase(h, PH_REFL);
            lds_store(h);                            // the parent is the top node again
        } else {                                     // PH_REFL_CHILD, main.cpp:1184-1194
            h.acc = cadd(h.acc, cmulf(c, f));        // f = F_r
            set_phase(h, PH_DONE);                   // complete: nothing else of it is needed
        }
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
    if (p.pix) {       // a pixel list (rt_render_pixels): image coordinates
        x = p.pix[2 * idx];
        y = p.pix[2 * idx + 1];
        return;
    }
    unsigned strip_px = (unsigned)p.W * (unsigned)kStrip;
    unsigned s = idx / strip_px;
    unsigned r = idx - s * strip_px;
    int sh = min(kStrip, p.rows - (int)s * kStrip);
    x = (int)(r / (unsigned)sh);
    y = (int)s * kStrip + (int)(r % (unsigned)sh);
}

__device__ __forceinline__ void image_xy(const Params &p, unsigned pix, int &x, int &y) {
    pixel_xy(p, pix, x, y);
    if (!p.pix) y = image_row(p, y);
}

// Primary ray of local pixel (x, y): p = ul + dh * x + dv * row, direction
// (p - eye).norm() (main.cpp:720-728, that association order)
__device__ __forceinline__ V3 primary_dir(const Params &p, int x, int y) {
    V3 pt = vadd(vadd(V3{p.ul[0], p.ul[1], p.ul[2]}, vmul(V3{p.dh[0], p.dh[1], p.dh[2]}, (float)x)),
                 vmul(V3{p.dv[0], p.dv[1], p.dv[2]}, (float)image_row(p, y)));
    return vnorm(vsub(pt, V3{p.eye[0], p.eye[1], p.eye[2]}));
}

template <int MAXF, int MODE, bool COUNT>
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
        const int nl4 = p.lights_in_lds ? p.nl * (int)(sizeof(LightK) / sizeof(float4)) : 0;
        const float4 *src = reinterpret_cast<const float4 *>(p.lights);
        for (int i = threadIdx.x; i < nl4; i += blockDim.x) rt_lds[p.lights_lds + i] = src[i];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    LaneState<MAXF> ls;
    ls.top = -1;
    ls.frames = p.frames;
    CountersT<COUNT> cnt = {0, 0, 0, 0, 0};
    unsigned long long w_prim = 0, w_shadow = 0, w_refr = 0, w_refl = 0;   // per wave (uniform)
    unsigned w_known = 0, w_bf = 0;
    int *stk = reinterpret_cast<int *>(lds) + threadIdx.x;  // MODE_BVH: stack[k * kBlock]
    // bvh_trace's stack bottom: kEmpty, or a refill tag (kRefill + blocks) while
    // spilled entries wait in device memory (spill / pop); every traversal
    // leaves it kEmpty
    if (MODE == MODE_BVH) stk[0] = rtbvh::kEmpty;
    Query q;
    bool busy = false;         // lane owns a pixel
    bool pending = false;      // q holds a finished scan to consume
    bool held = false;         // q is set up but its search is held back (p.gate_x)
    int held_kind = RK_NONE;
    bool drained = false;      // wave saw the work counter run out
    unsigned chunk_pos = 0, chunk_end = 0;   // the wave's tile: its unused work items [pos, end)
    // the wave's band of the work items (uniform, one register): bits 0-3 the
    // band (its XCD's first, then the next ones), 4-7 the bands not yet
    // exhausted, bit 8: no batch taken yet (the static first batch)
#ifndef RT_STATIC_FIRST
#define RT_STATIC_FIRST 1                // 0: the first batch from the counter too (A/B)
#endif
    unsigned wband = (blockIdx.x & ((1u << p.work_shift) - 1u)) | (1u << (p.work_shift + 4)) |
                     (p.chunk == 0 && RT_STATIC_FIRST ? 256u : 0u);
    unsigned pix_idx = 0;      // the lane's work item (its pixel's (x, y) is recomputed for the store)
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
    // lanes that sit a trace step out, by reason: no pixel (waiting for a
    // refill batch, or the work has run out), a held reflection / refraction
    // search, a known shadow result
    unsigned long long pc_nopix = 0, pc_held = 0, pc_known = 0;
    unsigned long long pc_mixed = 0;     // trace steps with primary and secondary/shadow searches together
    unsigned long long t_drain = 0;
    unsigned long long n_refill = 0, pc_refill = 0;
    const unsigned long long t_loop = __builtin_amdgcn_s_memrealtime();
    unsigned long long t_first = 0;      // end of the first trace step (its code fetched cold)
#endif
    for (;;) {
#if RT_PROF
        unsigned long long c0 = __builtin_amdgcn_s_memtime();
#endif
        int kind = RK_NONE;
        // The shading step and the refill run at a raised wave priority: a
        // shading step is a chain of dependent loads (§3.6 of DESIGN.md), and
        // issuing each of its instructions ahead of the other waves' traversal
        // gets its next load out sooner (C3 +0.5 %, one frame -1.3 %, C5
        // +0.7 %; raising the traversal instead: -1 %, profiles/r03/ab_prio.txt)
#if RT_PRIO
        __builtin_amdgcn_s_setprio(2);
#endif
        if (pending && !held) {
            C3 color;
            kind = advance<MAXF>(p, ls, q, cnt, color, pix_idx);
            pending = kind != RK_NONE;
            if (!pending) {
                // the pixel's 12 bytes in one store (global_store_dwordx3),
                // non-temporal: the framebuffer is not read again by the kernel,
                // and its lines no longer take L2 from the frame heads and the
                // tree (C3 +0.45 %, C5 +0.2 %, C4 +0.4 %, one frame -1.5 % on C3;
                // the same hint on the heads' loads: C3 -2.5 %, C5 -1.8 %; on the
                // refraction extensions' stores / loads: -0.8 % / +-0,
                // profiles/r06/nt/)
                typedef float f3v __attribute__((ext_vector_type(3), aligned(4)));
                // (x, y) from the work item again: two registers fewer live
                // across the whole pixel; a pixel list's k-th colour goes to out[3k..]
                int px = (int)pix_idx, py = 0;
                if (!p.pix) pixel_xy(p, pix_idx, px, py);
                __builtin_nontemporal_store(f3v{color.r, color.g, color.b},
                                            reinterpret_cast<f3v *>(p.out + ((size_t)py * p.W + px) * 3));
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
        //
        // Work items come in p.work_parts bands (8: one per XCD, workgroup b
        // runs on XCD b mod 8) with a counter each; a wave starts on its
        // XCD's band and moves to the next band when its own runs out.  Its
        // first batch is assigned statically (wave k of the band: items
        // [64 k, 64 k + 64) of it; the band's counter counts from there):
        // 5120 waves asking one counter at once, and again whenever their
        // batches end together, is what held short frames back (C2: 160 us
        // per trace step, profiles/r04/timeline_C2.json).
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
                const unsigned sh = p.work_shift, P = 1u << sh;
                // the current chunk's items are of the current band: [.., old_end)
                const unsigned old_end = (unsigned)(((unsigned long long)((wband & 15u) + 1) * p.total) >> sh);
                unsigned nbase = 0, new_end = 0;
                if (n > left) {
                    const unsigned take = max(p.chunk, n - split);
                    // a band that has run out: the next one, at once (a wave
                    // leaves only when every band has run out)
                    for (;;) {
                        const unsigned band = wband & 15u;
                        const unsigned band_lo = (unsigned)(((unsigned long long)band * p.total) >> sh);
                        new_end = (unsigned)(((unsigned long long)(band + 1) * p.total) >> sh);
                        // work items the band's waves take statically, before its counter
                        // (none when they take chunks: option chunk)
                        const unsigned nstatic =
                            p.chunk || !RT_STATIC_FIRST ? 0u : ((gridDim.x - band + P - 1) >> sh) * (unsigned)kBlock;
                        unsigned g;
                        if (wband & 256u) {
                            // (the wave's index, uniform: readfirstlane keeps g in an SGPR)
                            g = ((blockIdx.x >> sh) * (unsigned)(kBlock / 64) +
                                 (unsigned)__builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64))) * 64u;
                        } else {
                            g = 0;
#if RT_PROF
                            const unsigned long long ta = __builtin_amdgcn_s_memtime();
#endif
                            if (lane == leader)
                                g = nstatic + atomicAdd(reinterpret_cast<unsigned *>(p.stats + kWorkSlots +
                                                                                     kWorkStride * band),
                                                        take);
                            g = (unsigned)__builtin_amdgcn_readlane((int)g, leader);   // uniform: an SGPR
#if RT_PROF
                            n_refill++;
                            pc_refill += __builtin_amdgcn_s_memtime() - ta;   // the counter's round trip
#endif
                        }
                        wband &= ~256u;
                        nbase = band_lo + g;
                        if (nbase < new_end) {
                            chunk_pos = nbase + (n - split);
                            chunk_end = nbase + take;
                            break;
                        }
                        chunk_pos = chunk_end = 0;      // this band is done
                        wband -= 16u;
                        if ((wband >> 4) == 0) {
                            drained = true;
                            new_end = 0;
                            break;
                        }
                        wband = (wband & ~15u) | (band + 1 == P ? 0u : band + 1);
                    }
                } else {
                    chunk_pos += n;
                }
#if RT_PROF
                if (drained) t_drain = __builtin_amdgcn_s_memrealtime();
#endif
                if (!busy) {
                    // idle lanes below this one (v_mbcnt: no per-lane mask kept in registers)
                    unsigned rank = __builtin_amdgcn_mbcnt_hi((unsigned)(idle >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)idle, 0u));
                    unsigned idx = rank < split ? base + rank : nbase + (rank - split);
                    if (idx < (rank < split ? old_end : new_end)) {
                        int px, py;
                        pixel_xy(p, idx, px, py);
                        q.o = V3{p.eye[0], p.eye[1], p.eye[2]};
                        q.d = primary_dir(p, px, py);
                        pix_idx = idx;
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
#if RT_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
        if (!pending) q.tmin = kInf;                 // lane sits this scan out
        if (__ballot(pending) == 0ull) break;
        // A shadow ray whose cumulative mask (main.cpp:788, carried across the
        // lights) is already exactly 0 keeps it 0 whatever it hits: every
        // factor is in [0, 1] when none is NaN (shadow_early_out), and
        // clamp01(0 * f) = 0.  It is still a TraceRay call of the reference
        // (counted above); its result is known without searching.
        const bool known = pending && !q.closest && p.shadow_early_out && prior_mask(q) == 0.0f;
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

        if constexpr (COUNT) {
            w_prim += (unsigned long long)__popcll(__ballot(kind == RK_PRIMARY));
            w_shadow += (unsigned long long)__popcll(__ballot(kind == RK_SHADOW));
            w_refr += (unsigned long long)__popcll(__ballot(kind == RK_REFR));
            w_refl += (unsigned long long)__popcll(__ballot(kind == RK_REFL));
            w_known += (unsigned)__popcll(__ballot(known));
        }
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
            pc_nopix += (unsigned long long)__popcll(__ballot(!pending));
            pc_held += (unsigned long long)__popcll(__ballot(pending && held));
            pc_known += (unsigned long long)__popcll(__ballot(pending && known));
            unsigned tr0 = cnt.trips;
#endif
            // origin-leaf pass by the query's kind (held_kind: this step's):
            // bit 0 shadow, 1 refraction, 2 reflection rays
            const bool org_pass = held_kind >= RK_SHADOW && held_kind <= RK_REFL &&
                                  ((p.org_first >> (held_kind - RK_SHADOW)) & 1);
            if (search && !q.bf) bvh_trace<false, leaf_wait_for(MAXF)>(q, p, stk, cnt, org_pass);
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
                                !(p.shadow_early_out && q.mask == 0.0f);
                if (__ballot(pt) && pt) {
                    const DirK &dk = p.dirk[h_light_lds<MAXF>()];
                    const int root = dk.root;
                    if (root >= 0) {
                        V3 po = {fmaf(dk.R[0], q.o.x, fmaf(dk.R[1], q.o.y, dk.R[2] * q.o.z)),
                                 fmaf(dk.R[3], q.o.x, fmaf(dk.R[4], q.o.y, dk.R[5] * q.o.z)),
                                 fmaf(dk.R[6], q.o.x, fmaf(dk.R[7], q.o.y, dk.R[8] * q.o.z))};
                        bvh_trace<true, kLeafWaitCone>(q, p, stk, cnt, false, root, po, dk.cone_k, dk.cone_h);
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
            if (!t_first) t_first = __builtin_amdgcn_s_memrealtime();
#endif
            bool need = search && q.bf;
            const unsigned long long nb = __ballot(need);
            if constexpr (COUNT) w_bf += (unsigned)__popcll(nb);
            if (nb) scan<false, COUNT>(q, p, lds_f, lds_s, need, cnt.ftests, cnt.stests);
#if RT_PROF
            pc_bf += __builtin_amdgcn_s_memtime() - c2;
#endif
        } else {
            scan<SRC_LDS, COUNT>(q, p, lds_f, lds_s, search, cnt.ftests, cnt.stests);
        }
    }
    unsigned long long *st = p.stats;
    // this workgroup's copy of the exit counters (rt_device.h kStatCopies)
    unsigned long long *sc = st + stat_copy_off((int)(blockIdx.x & (kStatCopies - 1)));
    if constexpr (COUNT) {
        if (lane == 0) {
            atomicAdd(&sc[0], w_prim);
            atomicAdd(&sc[1], w_shadow);
            atomicAdd(&sc[2], w_refr);
            atomicAdd(&sc[3], w_refl);
            atomicAdd(&sc[32], (unsigned long long)w_known);
            atomicAdd(&sc[33], (unsigned long long)w_bf);
        }
        atomicAdd(&sc[4], (unsigned long long)cnt.skip);
        atomicAdd(&sc[5], (unsigned long long)cnt.ub);
        atomicAdd(&sc[6], (unsigned long long)cnt.boxes);
        atomicAdd(&sc[7], (unsigned long long)cnt.ftests);
        atomicAdd(&sc[8], (unsigned long long)cnt.stests);
    }
    const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        atomicMax(&sc[24], ~t_start);                // kernel start (first wave): the counters start
                                                     // at 0 (one memset per frame), so minima are kept
                                                     // as maxima of the complement
        atomicMax(&sc[26], t_end);                   // last wave done
    }
#if RT_PROF
    if (lane == 0) {
        atomicAdd(&st[9], pc_shade);
        atomicAdd(&st[10], pc_trace);
        atomicAdd(&st[11], pc_bf);
        atomicAdd(&st[12], pc_iter);
        atomicAdd(&st[13], pc_lanes);
        atomicAdd(&st[50], pc_nopix);
        atomicAdd(&st[51], pc_held);
        atomicAdd(&st[52], pc_known);
        atomicAdd(&st[14], pc_wtrips);
        atomicAdd(&st[39], pc_mixed);
        atomicAdd(&st[46], pc_refill);               // cycles waiting for the work counter
        atomicAdd(&st[47], n_refill);
    }
    atomicAdd(&st[15], (unsigned long long)cnt.trips);
    atomicAdd(&st[36], (unsigned long long)cnt.trips_kind[0]);
    atomicAdd(&st[37], (unsigned long long)cnt.trips_kind[1]);
    atomicAdd(&st[38], (unsigned long long)cnt.trips_kind[2]);
    {
        const unsigned w = blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
        if (lane == 0 && w < (unsigned)kWaveLogMax) {
            unsigned long long *wl = st + kWaveLogOff + (size_t)w * kWaveLogWords;
            wl[0] = t_start;
            wl[1] = t_loop;
            wl[2] = t_drain;
            wl[3] = t_end;
            wl[4] = t_first;
            wl[5] = ((unsigned long long)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4) << 32) |   // HW_REG_HW_ID
                    (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);                              // HW_REG_XCC_ID
            wl[6] = pc_iter;
            wl[7] = n_refill;
        }
    }
    if (lane == 0) {
        if (!t_drain) t_drain = t_end;
        atomicMax(&st[25], ~t_drain);                // work counter ran out (complement, as [24])
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

// Gathered row sets -> image order (rt_deinterleave_rows, _u8): image row y
// belongs to rank (y / block) % world as its local row (y / (block * world)) *
// block + y % block; a row is n elements of T (16-B vectors when the row's
// bytes allow, else the row's own element type).
template <typename T>
__global__ void deinterleave_kernel(const T *__restrict__ gathered, int world, int rows_per, size_t n, int block,
                                    int H, T *__restrict__ image) {
    // rows grid-strided in y: the grid's y extent is capped at 65535
    for (int y = blockIdx.y; y < H; y += gridDim.y) {
        const int rank = (y / block) % world;
        const int k = (y / (block * world)) * block + y % block;
        const T *src = gathered + ((size_t)rank * rows_per + k) * n;
        T *dst = image + (size_t)y * n;
        for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
            dst[i] = src[i];
    }
}

// The P3 writer's values (main.cpp:760: (size_t)(int)(c * 255), rth_quantize)
// as bytes, for a gather of 3 B instead of 12 per pixel: a value is stored as
// its byte when the writer's value is 0..255 -- c * 255 in (-1, 256), where
// the truncation gives 0..255 -- and otherwise (NaN, a background above 1,
// a negative colour) *flag gets bit 0 and the byte is 0: the caller must then
// use the floats.  Four values per thread (float4 in, 4 bytes out).
__global__ void quantize_u8_kernel(const float4 *__restrict__ rgb, size_t n4, const float *__restrict__ tail,
                                   size_t ntail, unsigned *__restrict__ out, unsigned char *__restrict__ out_tail,
                                   unsigned *__restrict__ flag) {
    auto q1 = [](float c, bool &bad) -> unsigned {
        const float x = c * 255.0f;                  // (c - 0) * (255 - 0) / (1 - 0) + 0, exactly
        const bool ok = (x > -1.0f) & (x < 256.0f);  // false for NaN
        bad |= !ok;
        return ok ? (unsigned)(int)x : 0u;
    };
    bool bad = false;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n4) {
        const float4 v = rgb[i];
        out[i] = q1(v.x, bad) | (q1(v.y, bad) << 8) | (q1(v.z, bad) << 16) | (q1(v.w, bad) << 24);
    }
    if (i < ntail) out_tail[i] = (unsigned char)q1(tail[i], bad);
    if (__ballot(bad) && (threadIdx.x & 63) == (unsigned)(__ffsll((long long)__ballot(bad)) - 1))
        atomicOr(flag, 1u);
}

hipError_t quantize_u8_launch(const float *rgb, size_t n, unsigned char *out, unsigned *flag, hipStream_t st) {
    const size_t n4 = n / 4, ntail = n % 4;
    const size_t threads = std::max<size_t>(n4, ntail);
    if (threads == 0) return hipSuccess;
    const unsigned blocks = (unsigned)((threads + 255) / 256);
    hipLaunchKernelGGL(quantize_u8_kernel, dim3(blocks), dim3(256), 0, st, reinterpret_cast<const float4 *>(rgb), n4,
                       rgb + 4 * n4, ntail, reinterpret_cast<unsigned *>(out), out + 4 * n4, flag);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Launch interface (rt_device.h)
// ---------------------------------------------------------------------------
int maxf_for_depth(int depth) {
    if (depth < 0) depth = 0;
    return depth <= 4 ? 5 : depth <= 8 ? 9 : depth <= 16 ? 17 : -1;
}

int maxf_for(int depth, bool secondary) { return !secondary || depth <= 0 ? 1 : maxf_for_depth(depth); }

size_t cold_frame_bytes(int maxf) {
    return maxf == 1 ? sizeof(Cold<1>) : maxf == 5 ? sizeof(Cold<5>) : maxf == 9 ? sizeof(Cold<9>) : sizeof(Cold<17>);
}

// occupancy of the instantiation that will be launched (the counting one may
// use more registers than the benched one)
template <int MAXF, int MODE>
static int blocks_one(bool count, size_t lds_bytes) {
    int nb = 0;
    const hipError_t e =
        count ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, render_kernel<MAXF, MODE, true>, kBlock, lds_bytes)
              : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, render_kernel<MAXF, MODE, false>, kBlock, lds_bytes);
    return e == hipSuccess ? nb : 0;
}

template <int MAXF>
static int blocks_mode(int mode, bool count, size_t lds_bytes) {
    if (mode == MODE_BVH) return blocks_one<MAXF, MODE_BVH>(count, lds_bytes);
    if (mode == MODE_SCAN_LDS) return blocks_one<MAXF, MODE_SCAN_LDS>(count, lds_bytes);
    return blocks_one<MAXF, MODE_SCAN>(count, lds_bytes);
}

int render_blocks_per_cu(int maxf, int mode, bool count, size_t lds_bytes) {
    if (maxf == 1) return blocks_mode<1>(mode, count, lds_bytes);
    if (maxf == 5) return blocks_mode<5>(mode, count, lds_bytes);
    if (maxf == 9) return blocks_mode<9>(mode, count, lds_bytes);
    return blocks_mode<17>(mode, count, lds_bytes);
}

template <int MAXF, bool COUNT>
static hipError_t launch_mode(int mode, const Params &p, unsigned grid, size_t lds_bytes, hipStream_t st) {
    if (mode == MODE_BVH)
        hipLaunchKernelGGL((render_kernel<MAXF, MODE_BVH, COUNT>), dim3(grid), dim3(kBlock), lds_bytes, st, p);
    else if (mode == MODE_SCAN_LDS)
        hipLaunchKernelGGL((render_kernel<MAXF, MODE_SCAN_LDS, COUNT>), dim3(grid), dim3(kBlock), lds_bytes, st, p);
    else
        hipLaunchKernelGGL((render_kernel<MAXF, MODE_SCAN, COUNT>), dim3(grid), dim3(kBlock), lds_bytes, st, p);
    return hipGetLastError();
}

template <bool COUNT>
static hipError_t launch_maxf(int maxf, int mode, const Params &p, unsigned grid, size_t lds_bytes, hipStream_t st) {
    if (maxf == 1) return launch_mode<1, COUNT>(mode, p, grid, lds_bytes, st);
    if (maxf == 5) return launch_mode<5, COUNT>(mode, p, grid, lds_bytes, st);
    if (maxf == 9) return launch_mode<9, COUNT>(mode, p, grid, lds_bytes, st);
    if (maxf == 17) return launch_mode<17, COUNT>(mode, p, grid, lds_bytes, st);
    return hipErrorInvalidValue;
}

hipError_t render_launch(int maxf, int mode, bool count, const Params &p, unsigned grid, size_t lds_bytes,
                         hipStream_t st) {
    return count ? launch_maxf<true>(maxf, mode, p, grid, lds_bytes, st)
                 : launch_maxf<false>(maxf, mode, p, grid, lds_bytes, st);
}

hipError_t deinterleave_launch(const void *gathered, size_t row_bytes, size_t elem_bytes, int world, int rows_per,
                               int H, int block, void *image, hipStream_t st) {
    const bool vec = row_bytes % 16 == 0 && reinterpret_cast<uintptr_t>(gathered) % 16 == 0 &&
                     reinterpret_cast<uintptr_t>(image) % 16 == 0;
    const size_t eb = vec ? 16 : elem_bytes, n = row_bytes / eb;
    const unsigned gx = (unsigned)std::min<size_t>(64, (n + 255) / 256);
    const dim3 grid(gx, (unsigned)std::min(H, 65535));
    if (vec)
        hipLaunchKernelGGL(deinterleave_kernel<uint4>, grid, dim3(256), 0, st, static_cast<const uint4 *>(gathered),
                           world, rows_per, n, block, H, static_cast<uint4 *>(image));
    else if (eb == 4)
        hipLaunchKernelGGL(deinterleave_kernel<unsigned>, grid, dim3(256), 0, st,
                           static_cast<const unsigned *>(gathered), world, rows_per, n, block, H,
                           static_cast<unsigned *>(image));
    else
        hipLaunchKernelGGL(deinterleave_kernel<unsigned char>, grid, dim3(256), 0, st,
                           static_cast<const unsigned char *>(gathered), world, rows_per, n, block, H,
                           static_cast<unsigned char *>(image));
    return hipGetLastError();
}

}  // namespace rt

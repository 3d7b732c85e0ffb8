// rt_scene.cpp -- host side of librt_hip.so: scene upload (the device layout
// of rt_device.h), BVH build and upload (rt_bvh.h), render slots, and the C ABI
// of include/rt_hip.h.  The kernels are in rt_kernels.hip.
//
// The seam this replaces: create_view_window_and_ray_trace (main.cpp:607,
// :670-767) and its implicit inputs from the global `environment`
// (main.cpp:58, src/definitions.h:304-311).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rt_bvh.h"
#include "rt_device.h"
#include "rt_hip.h"

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
    int *dev_pix = nullptr;            // rt_render_pixels: the pixel list on the device
    size_t dev_pix_bytes = 0;
    std::vector<RenderSlot> slots;     // slots[0] always exists
    int next_slot = 0;                 // slot of the next render
    int last_slot = 0;                 // slot of the last render
    int num_cu = 0;
    size_t max_lds = 64 * 1024;        // the device's LDS limit per workgroup
    size_t lds_bytes = 0;
    long long opt_lds = -1;            // -1 auto, 0 off, 1 on
    long long opt_lds_stack = -1;      // BVH stack entries in LDS (-1: by depth, launch)
    double crossings = 0.0;            // objects a line across the scene meets on average (org_first)
    int org_first_auto = 0;            // org_first by that density
    long long opt_grid = 0;            // blocks (0 = occupancy-derived)
    long long opt_chunk = -1;          // refill chunk (-1: default, chunk_for)
    long long opt_refill_min = -1;     // idle lanes before a refill (-1: by the scene, refill_for)
    bool secondary = false;            // some material reflects (ks > 0) or refracts (opacity < 1, eta > 0)
    long long opt_reserve = 0;         // occupancy-derived grid: block slots left free for other kernels
    long long opt_accel = -1;          // -1 auto, 0 brute-force scan, 1 BVH
    long long opt_bvh_leaf = 8;        // SAH max leaf size
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
    int *d_objleaf = nullptr;          // per object: its leaf's link in the main tree
    std::vector<float4> h_fscan, h_sscan;   // host copies for the leaf records
    std::vector<float> h_ofac;
    std::vector<LightK> h_lights;

    int bvh_depth = 0;
    int bvh_stack = 0;
    int ovf_stride = kSpill;           // spilled BVH stack entries per lane (Params::ovf_stride)
    bool bvh_ok = false;
    double bvh_build_ms = 0.0;         // host time of the last BVH (re)build
    long long last_blocks_per_cu = 0, last_grid = 0, last_lds = 0, last_mode = -1;
    long long last_org_first = 0, last_stack_cap = 0, last_lights_in_lds = 0;
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
// (BVH stacks or the staged primitives), then the lights when they all fit
// under the device's per-workgroup LDS limit (else the kernel reads them from
// device memory, Params::lights_in_lds: a scene with thousands of lights
// still renders).
size_t mode_region_end(const rt_scene *s, int mode, const Params &p) {
    size_t shade = (size_t)kLdsHotWords * kBlock * sizeof(float);    // per-lane shading state
    if (mode == MODE_SCAN_LDS) return shade + s->lds_bytes;
    if (mode == MODE_BVH) return shade + (size_t)p.stack_cap * kBlock * sizeof(int);
    return shade;
}
// The launch's dynamic LDS; decides Params::lights_in_lds: the lights are
// staged when they fit under the limit and do not cost a resident workgroup
// per CU (by the occupancy calculator), else they come from device memory.
size_t mode_lds_bytes(const rt_scene *s, int maxf, int mode, Params &p) {
    const size_t end = mode_region_end(s, mode, p);
    const size_t with = end + (size_t)p.nl * sizeof(LightK);
    p.lights_lds = (int)(end / sizeof(float4));
    p.lights_in_lds = with <= s->max_lds && render_blocks_per_cu(maxf, mode, with) >= render_blocks_per_cu(maxf, mode, end);
    return p.lights_in_lds ? with : end;
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

hipError_t launch_one(rt_scene *s, RenderSlot &slot, const Params &p, int maxf, int mode, hipStream_t st, bool dry) {
    Params pl = p;
    size_t shm = mode_lds_bytes(s, maxf, mode, pl);
    int nb = render_blocks_per_cu(maxf, mode, shm);
    if (nb < 1) nb = 1;
    long long grid = s->opt_grid > 0 ? s->opt_grid : (long long)nb * s->num_cu - s->opt_reserve;
    long long need = ((long long)p.total + kBlock - 1) / kBlock;
    if (grid > need) grid = need;
    if (grid < 1) grid = 1;
    pl.chunk = chunk_for(s);
    pl.refill_min = refill_for(s, pl);
    const size_t cold_bytes = (size_t)grid * kBlock * maxf * cold_frame_bytes(maxf);
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
    s->last_mode = mode;
    s->last_org_first = pl.org_first;
    s->last_stack_cap = pl.stack_cap;
    s->last_lights_in_lds = pl.lights_in_lds;
    if (dry) return hipSuccess;                  // rt_scene_prepare: buffers only
    return render_launch(maxf, mode, pl, (unsigned)grid, shm, st);
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
    B.trav_cost = 0.5f;                // SAH node cost, in sphere tests (A/B over 0.25-2: 0.5 best, round 1)
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
    // every object's leaf in the main tree (the origin-leaf pass, bvh_trace)
    std::vector<int32_t> objleaf((size_t)std::max(1, nf + s->base.ns), rtbvh::kEmptyLeaf);
    if (ok)
        for (const auto &n : Q.nodes)
            for (int32_t l : n.link) {
                if (l >= 0 || l == rtbvh::kEmpty) continue;
                const int v = -l - 1, nfc = (v >> 4) & 15, count = v & 15;
                size_t off = (size_t)(v >> 8);
                for (int k = 0; k < count; k++) {
                    int32_t key;
                    if (k < nfc) {
                        memcpy(&key, &rec[off + 4].y, sizeof key);
                        off += 5;
                    } else {
                        memcpy(&key, &rec[off + 1].x, sizeof key);
                        off += 2;
                    }
                    objleaf[(size_t)key] = l;
                }
            }
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
    }
    // device links: an inner node's link is its byte offset in the node array
    // (the kernel fetches a node with buffer loads at that offset: no address
    // arithmetic per visit), leaf links stay as they are
    if (ok && QQ.size() * sizeof(rtbvh::Node4H) > (size_t)INT32_MAX) ok = false;
    if (ok) {
        for (auto &z : QQ)
            for (auto &l : z.link)
                if (l >= 0) l *= (int32_t)sizeof(rtbvh::Node4H);
        for (auto &d : dirk)
            if (d.root >= 0) d.root *= (int)sizeof(rtbvh::Node4H);
    }
    // The old tree stays valid until the new one is on the device: upload into
    // new buffers first, then swap (a failed rebuild leaves no dangling
    // pointers and no tree marked valid that is not there).
    float4 *nb = nullptr, *nr = nullptr;
    DirK *nd = nullptr;
    int *nl = nullptr;
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
            hipMalloc(&nd, dir_bytes) != hipSuccess || hipMalloc(&nl, objleaf.size() * sizeof(int32_t)) != hipSuccess)
            rc = RT_E_NOMEM;
        else if (hipMemcpy(nb, QQ.data(), node_bytes, hipMemcpyHostToDevice) != hipSuccess ||
                 hipMemcpy(nr, rec.data(), rec.size() * sizeof(float4), hipMemcpyHostToDevice) != hipSuccess ||
                 (!dirk.empty() && hipMemcpy(nd, dirk.data(), dirk.size() * sizeof(DirK), hipMemcpyHostToDevice) !=
                                       hipSuccess) ||
                 hipMemcpy(nl, objleaf.data(), objleaf.size() * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess)
            rc = RT_E_HIP;
        if (rc) {
            if (nb) (void)hipFree(nb);
            if (nr) (void)hipFree(nr);
            if (nd) (void)hipFree(nd);
            if (nl) (void)hipFree(nl);
            nb = nr = nullptr;
            nd = nullptr;
            nl = nullptr;
        }
    }
    // renders still queued may read the old tree: free it after they finish
    if (s->d_bvh || s->d_leafrec || s->d_dirk || s->d_objleaf) {
        (void)hipDeviceSynchronize();
        if (s->d_bvh) (void)hipFree(s->d_bvh);
        if (s->d_leafrec) (void)hipFree(s->d_leafrec);
        if (s->d_dirk) (void)hipFree(s->d_dirk);
        if (s->d_objleaf) (void)hipFree(s->d_objleaf);
    }
    s->d_bvh = nb;
    s->d_leafrec = nr;
    s->d_dirk = nd;
    s->d_objleaf = nl;
    s->base.objleaf = nl;
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
    if (maxf_for_depth(depth) < 0) return RT_E_UNSUPPORTED;
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
            p.objleaf = s->base.objleaf;
            p.dir_bf = s->base.dir_bf;
            p.ovf_stride = s->ovf_stride;
        }
    }
    if (mode == MODE_SCAN) {
        bool lds = s->opt_lds == 1 || (s->opt_lds == -1 && s->lds_bytes <= 64 * 1024);
        if (s->lds_bytes > 64 * 1024) lds = false;
        if (lds) mode = MODE_SCAN_LDS;
    }
    if (mode == MODE_SCAN_LDS && mode_region_end(s, MODE_SCAN_LDS, p) > s->max_lds) mode = MODE_SCAN;
    // BVH stack entries in LDS (option lds_stack, else per instantiation): 16
    // cost C3 8.6 % with the lights staged and 10 % without, C5 8.5 %: a
    // workgroup above ~31 KB of LDS loses a resident workgroup per CU in
    // practice (profiles/r02/ab_lds_stack.txt, profiles/r03/ab_deep_stack.txt)
    p.stack_cap = s->opt_lds_stack > 0 ? (int)s->opt_lds_stack : depth > 4 ? kLdsStackDeep : kLdsStackDefault;
    hipError_t e = launch_one(s, slot, p, maxf_for_depth(depth), mode, st, dry);
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
    if (n < 1 || n > 8) return RT_E_INVALID;
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

// Params of one render: the scene's, with this camera and image width.
Params frame_params(const rt_scene *s, const rt_camera *cam, int W) {
    Params p = s->base;
    for (int c = 0; c < 3; c++) {
        p.eye[c] = cam->eye[c];
        p.ul[c] = cam->ul[c];
        p.dh[c] = cam->dh[c];
        p.dv[c] = cam->dv[c];
    }
    p.W = W;
    p.pix = nullptr;
    return p;
}

// Queue one render (work counter and counters reset, the launch, events) on
// the next render slot, ordered against the caller's stream `st`.
int submit(rt_scene *s, Params &p, hipStream_t st) {
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
        else {
            s->num_cu = prop.multiProcessorCount;
            s->max_lds = prop.sharedMemPerBlock;
        }
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
    p.chunk = 0;                       // launch_one: chunk_for, refill_for
    p.refill_min = 1;
    p.gate_x = kGateX;
    // The origin-leaf pass for reflection and refraction rays pays in dense
    // scenes (C5: +2.3 %) and costs sparse ones (C3: -1.1 %;
    // profiles/r03/ab_origin_leaf.txt).  Density here: the objects a straight
    // line across the scene's box meets on average -- total cross-section
    // (spheres pi r^2, triangles area / 2, averaged over directions) per
    // volume, times the box diagonal (C3: ~3, C5: ~200).
    {
        double xs = 0.0, vol = 1.0, diag2 = 0.0;
        for (int i = 0; i < nf; i++) {
            V3 c = vcross(f3(&fscan[5 * i + 2].x), f3(&fscan[5 * i + 3].x));
            xs += 0.25 * std::sqrt((double)c.x * c.x + (double)c.y * c.y + (double)c.z * c.z);
        }
        for (int i = 0; i < ns; i++) xs += kPi * (double)sscan[i].w * (double)sscan[i].w;
        for (int k = 0; k < 3; k++) {
            const double e = (double)s->scene_hi[k] - (double)s->scene_lo[k];
            vol *= e;
            diag2 += e * e;
        }
        s->crossings = vol > 0.0 && std::isfinite(xs) ? xs / vol * std::sqrt(diag2) : 0.0;
        s->org_first_auto = s->crossings > kOrgDensity ? kOrgFirst : 0;
        p.org_first = s->org_first_auto;
    }
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
    if (s->d_objleaf) (void)hipFree(s->d_objleaf);
    if (s->dev_out) (void)hipFree(s->dev_out);
    if (s->dev_pix) (void)hipFree(s->dev_pix);
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
    else if (k == "org_first") {
        if (value < -1 || value > 7) return RT_E_INVALID;
        s->base.org_first = value < 0 ? s->org_first_auto : (int)value;
    }
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
        if (value < kSpill + 4 || value > kLdsStack) return RT_E_INVALID;
        s->opt_lds_stack = value;
    }
    else if (k == "bvh_leaf" || k == "bvh_collapse" || k == "bvh_node") {
        if (k == "bvh_leaf") s->opt_bvh_leaf = std::max(1LL, std::min(15LL, value));
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
    Params p = frame_params(s, cam, W);
    p.y0 = y0;
    p.rows = nrows;
    p.rblock = block;
    p.rstep = step;
    p.total = (unsigned)((long long)W * nrows);
    p.out = out_rgb;
    return submit(s, p, hip_stream ? (hipStream_t)hip_stream : s->stream);
}

int rt_render_pixels(rt_scene *s, const rt_camera *cam, int W, int H, const int *xy, int n, float *out_rgb,
                     rt_stats *stats) {
    if (!s || !cam || !xy || !out_rgb || W < 2 || H < 2 || n < 1) return RT_E_INVALID;
    for (int k = 0; k < n; k++)
        if (xy[2 * k] < 0 || xy[2 * k] >= W || xy[2 * k + 1] < 0 || xy[2 * k + 1] >= H) return RT_E_INVALID;
    if (hipSetDevice(s->device) != hipSuccess) return RT_E_HIP;
    const size_t pix_bytes = (size_t)n * 2 * sizeof(int), out_bytes = (size_t)n * 3 * sizeof(float);
    // the list and the colours pass through device buffers of the scene
    if (s->dev_pix_bytes < pix_bytes) {
        if (s->dev_pix) (void)hipFree(s->dev_pix);
        s->dev_pix = nullptr;
        s->dev_pix_bytes = 0;
        if (hipMalloc(&s->dev_pix, pix_bytes) != hipSuccess) return RT_E_NOMEM;
        s->dev_pix_bytes = pix_bytes;
    }
    if (s->dev_out_bytes < out_bytes) {
        if (s->dev_out) (void)hipFree(s->dev_out);
        s->dev_out = nullptr;
        s->dev_out_bytes = 0;
        if (hipMalloc(&s->dev_out, out_bytes) != hipSuccess) return RT_E_NOMEM;
        s->dev_out_bytes = out_bytes;
    }
    // the scene's stream runs after every render issued through its slots
    for (auto &r : s->slots)
        if (r.used && hipStreamWaitEvent(s->stream, r.ev1, 0) != hipSuccess) return RT_E_HIP;
    if (hipMemcpyAsync(s->dev_pix, xy, pix_bytes, hipMemcpyHostToDevice, s->stream) != hipSuccess) return RT_E_HIP;
    Params p = frame_params(s, cam, W);
    p.y0 = 0;                          // image_row(r) = r: the list holds image rows
    p.rows = H;
    p.rblock = p.rstep = 1;
    p.total = (unsigned)n;
    p.pix = s->dev_pix;
    p.out = s->dev_out;
    int rc = submit(s, p, s->stream);
    if (rc) return rc;
    if (hipMemcpyAsync(out_rgb, s->dev_out, out_bytes, hipMemcpyDeviceToHost, s->stream) != hipSuccess ||
        hipStreamSynchronize(s->stream) != hipSuccess)
        return RT_E_HIP;
    if (stats) return rt_scene_last_stats(s, stats);
    return RT_OK;
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
    return deinterleave_launch(gathered, world, rows_per, W, H, block, image, (hipStream_t)hip_stream) == hipSuccess
               ? RT_OK
               : RT_E_HIP;
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
    h[40] = (unsigned long long)s->last_org_first;
    h[41] = (unsigned long long)(s->crossings * 1000.0);
    h[42] = (unsigned long long)s->last_stack_cap;
    h[43] = (unsigned long long)s->last_lights_in_lds;
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